"""Micro-benchmark of the avse4 TCN PReLU -> gLN kernels at C4 (16 x 512 x 3999; HIP events, best of 3 x 20):
the fused dwconv -> PReLU -> gLN pair (fwd: x read, y1 + y written = 12 B/elem; bwd: x, y1, dy read, dx written =
16 B/elem) and the plain PReLU -> gLN pair (fwd: x read, y written = 8 B/elem; bwd: x, dy read, dx written =
12 B/elem); frac = algorithmic bytes / time / 8 TB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402


def ev_ms(fn, n=20):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        best = ms if best is None else min(best, ms)
    return best


B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
xd = torch.randn(B, 512, 3999, device="cuda")
wd = 0.3 * torch.randn(512, 1, 3, device="cuda")
al = torch.tensor([0.25], device="cuda")
gm = torch.rand(1, 512, 1, device="cuda") + 0.5
bt = torch.randn(1, 512, 1, device="cuda")
gy = torch.randn_like(xd)
n = xd.numel()
out = {"shape": [B, 512, 3999]}
_, y1, st = K.dwconv_gln_fwd(xd, wd, 128, al, gm, bt)
for name, fn, bpe in (("dwconv_gln_fwd", lambda: K.dwconv_gln_fwd(xd, wd, 128, al, gm, bt), 12),
                      ("dwconv_gln_bwd", lambda: K.dwconv_gln_bwd(xd, wd, 128, y1, al, gm, st, gy), 16)):
    ms = ev_ms(fn)
    out[name] = {"ms": round(ms, 4), "frac": round(bpe * n / (ms * 1e-3) / 8e12, 4)}
_, st2 = K.prelu_gln_fwd(xd, al, gm, bt)
for name, fn, bpe in (("prelu_gln_fwd", lambda: K.prelu_gln_fwd(xd, al, gm, bt), 8),
                      ("prelu_gln_bwd", lambda: K.prelu_gln_bwd(xd, al, gm, st2, gy), 12)):
    ms = ev_ms(fn)
    out[name] = {"ms": round(ms, 4), "frac": round(bpe * n / (ms * 1e-3) / 8e12, 4)}
print(json.dumps(out), flush=True)
