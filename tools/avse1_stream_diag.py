"""Diagnose the avse1 two-stream eager gradient gap (GPUTEST_r03: test_avse1_branch_streams_equal_serial[False]).

Runs the B=2 eager step of the test (bench.Avse1Step, dropout 0) in a sequence of modes and reports, against the
first serial run, the bitwise / relative differences of the lip-branch forward activations (front-end output, trunk
layers, TCN output = vis), of the gradients arriving at those points, and of each parameter group's gradient.

  serial        AVSE_AVSE1_STREAMS=0
  stream        lip branch on the side stream (product default: the join hands its gradient over with record_stream)
  stream_nohold as stream, without avse1._JoinFromSide (round 3's join)
  stream_sync   as stream, with torch.cuda.synchronize() after the lip forward and around the backward
  det           serial / stream with torch.backends.cudnn.deterministic = True

usage: python tools/avse1_stream_diag.py [mode ...]   (default: serial serial stream stream stream_sync serial)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from avse_challenge_amd import avse1  # noqa: E402

DEV = torch.device("cuda:0")


def run(mode):
    os.environ["AVSE_AVSE1_STREAMS"] = "0" if mode.startswith("serial") else "1"
    os.environ["AVSE_AVSE1_JOIN_HOLD"] = "0" if "nohold" in mode else "1"
    torch.backends.cudnn.deterministic = mode.endswith("_det")
    torch.manual_seed(5)
    st = bench.Avse1Step(2, DEV, 0, 1, 96)
    m = st.model
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    vf = m.net_visualfeat
    acts, grads = {}, {}

    def tap(name):
        def hook(_mod, _inp, out):
            acts[name] = out.detach().clone()
            if out.requires_grad:
                out.register_hook(lambda g: grads.__setitem__(name, g.detach().clone()))
        return hook

    def pre_tap(name):
        def hook(_mod, inp):
            x = inp[0]
            acts[name] = x.detach().clone()
            if x.requires_grad:
                x.register_hook(lambda g: grads.__setitem__(name, g.detach().clone()))
        return hook

    hs = [vf.trunk.register_forward_pre_hook(pre_tap("frontend_out"))]
    for i in range(1, 5):
        hs.append(getattr(vf.trunk, f"layer{i}").register_forward_hook(tap(f"trunk.layer{i}")))
    hs.append(vf.tcn.register_forward_hook(tap("tcn_out")))
    hs.append(vf.register_forward_hook(tap("vis")))
    hs.append(m.net_audiofeat.register_forward_hook(tap("audio")))
    if mode.startswith("stream_sync"):
        hs.append(vf.register_forward_hook(lambda *a: torch.cuda.synchronize()))
        torch.cuda.synchronize()
    loss = st.loss()
    if mode.startswith("stream_sync"):
        torch.cuda.synchronize()
    loss.backward()
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    pg = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    out = {"loss": float(loss), "acts": acts, "grads": grads, "pgrads": pg}
    del st, m
    torch.cuda.empty_cache()
    return out


def rel(a, b):
    d = float((a.double() - b.double()).norm())
    return d / max(1e-30, float(b.double().norm())), int((a != b).sum())


def group(k):
    if k.startswith("net_visualfeat.trunk."):
        return ".".join(k.split(".")[:3])
    if k.startswith("net_visualfeat."):
        return ".".join(k.split(".")[:2])
    return k.split(".")[0]


def main():
    modes = sys.argv[1:] or ["serial", "serial", "stream_nohold", "stream_nohold", "stream", "stream", "stream_sync",
                             "serial"]
    base = None
    for i, mode in enumerate(modes):
        r = run(mode)
        if base is None:
            base = r
            print(f"[{i}] {mode}: loss {r['loss']:.9g} (reference run)", flush=True)
            continue
        print(f"[{i}] {mode}: loss {r['loss']:.9g}  dloss {r['loss'] - base['loss']:+.3e}", flush=True)
        for k in base["acts"]:
            e, n = rel(r["acts"][k], base["acts"][k])
            print(f"    fwd  {k:16s} rel {e:.3e}  differing {n}/{r['acts'][k].numel()}")
        for k in ["vis", "tcn_out", "trunk.layer4", "trunk.layer3", "trunk.layer2", "trunk.layer1", "frontend_out",
                  "audio"]:
            if k in base["grads"] and k in r["grads"]:
                e, n = rel(r["grads"][k], base["grads"][k])
                print(f"    grad {k:16s} rel {e:.3e}  differing {n}/{r['grads'][k].numel()}")
        groups = {}
        for k, g in base["pgrads"].items():
            groups.setdefault(group(k), []).append(k)
        for gname, keys in groups.items():
            a = torch.cat([r["pgrads"][k].reshape(-1) for k in keys])
            b = torch.cat([base["pgrads"][k].reshape(-1) for k in keys])
            e, n = rel(a, b)
            print(f"    pgrad {gname:28s} rel {e:.3e}  differing {n}/{a.numel()}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
