"""Micro-benchmark of the fused avse4 dwconv -> PReLU -> gLN kernels at C4 (16 x 512 x 3999, dil 128); HIP events.
frac: algorithmic bytes (fwd 12, bwd 16 per element) / time / 8 TB/s."""
import sys, os, json, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from avse_challenge_amd import kernels as K
from dconv_bench import timeit
xd = torch.randn(16, 512, 3999, device="cuda"); wd = 0.3 * torch.randn(512, 1, 3, device="cuda")
al = torch.tensor([0.25], device="cuda"); gm = torch.rand(512, device="cuda") + 0.5; bt = torch.randn(512, device="cuda")
gy = torch.randn_like(xd)
_, y1, st = K.dwconv_gln_fwd(xd, wd, 128, al, gm, bt)
f = timeit(lambda: K.dwconv_gln_fwd(xd, wd, 128, al, gm, bt), 20)
b = timeit(lambda: K.dwconv_gln_bwd(xd, wd, 128, y1, al, gm, st, gy), 20)
n = xd.numel()
print(json.dumps({"fwd_ms": round(f, 4), "fwd_frac": round(12 * n / (f * 1e-3) / 1e9 / 8000, 3), "bwd_ms": round(b, 4), "bwd_frac": round(16 * n / (b * 1e-3) / 1e9 / 8000, 3)}))
