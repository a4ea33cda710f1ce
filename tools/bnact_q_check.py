"""Diagnostic of the split-output BatchNorm passes inside the avse1 bench model (B = 4): at every bnact call that
writes its output (forward) or input gradient (backward) as the split layout, the same call is repeated with fp32
output and the decoded split is compared with it: bound / max ratio and max error relative to max |.|."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from avse_challenge_amd import kernels as K  # noqa: E402


def decode(t):
    q = K.q_view(t).view(torch.float16).reshape(-1, t.shape[1] // 16, 2, 16).double()
    bits = int(getattr(t, K.ABSMAX_ATTR).item())
    e = max(-100, min(100, 14 - (((bits >> 23) & 0xFF) - 127))) if bits else 0
    n, c, h, w = t.shape
    return ((q[:, :, 0, :] + q[:, :, 1, :]) * 2.0 ** -e).reshape(n, h, w, c).permute(0, 3, 1, 2)


def report(kind, q, ref):
    m = float(ref.abs().max())
    bound = float(getattr(q, K.ABSMAX_ATTR).view(torch.float32).item())
    err = float((decode(q) - ref.double()).abs().max())
    print(json.dumps({"site": kind, "shape": list(q.shape), "max": m, "bound_over_max": bound / max(m, 1e-30),
                      "err_over_max": err / max(m, 1e-30), "nonfinite": int((~torch.isfinite(decode(q))).sum())}),
          flush=True)


def main():
    dev = torch.device("cuda")
    fwd0, bwd0 = K.bnact_fwd, K.bnact_bwd

    def fwd(*a, q_out=False, **kw):
        y, st = fwd0(*a, q_out=q_out, **kw)
        x = a[0]
        print(json.dumps({"call": "fwd", "shape": list(x.shape), "q_out": bool(q_out), "split": K.is_split_q(y),
                          "q_ok": K._q_ok(x, kw.get("res", a[10] if len(a) > 10 else None)),
                          "training": bool(a[5]), "strides": list(x.stride())}), flush=True)
        if K.is_split_q(y):
            args = list(a)
            rm, rv = args[3], args[4]
            keep = (rm.clone(), rv.clone()) if rm is not None else None
            yr, _ = fwd0(*a, **kw)
            if keep is not None:
                rm.copy_(keep[0]), rv.copy_(keep[1])
            report("fwd", y, yr)
        return y, st

    def bwd(*a, q_out=False, **kw):
        out = bwd0(*a, q_out=q_out, **kw)
        if K.is_split_q(out[0]):
            report("bwd", out[0], bwd0(*a, **kw)[0])
        return out

    K.bnact_fwd, K.bnact_bwd = fwd, bwd
    st = bench.Avse1Step(4, dev, 0, 1, 96)
    loss = st.loss()
    loss.backward()
    torch.cuda.synchronize()
    print("loss", float(loss))


if __name__ == "__main__":
    main()
