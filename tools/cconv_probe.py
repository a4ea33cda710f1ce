"""Causal conv1d fwd/bwd time and HBM rate at the Mamba shapes, fp32 and bf16 (x = the x half of xz, as in the model)."""
import sys
import torch
sys.path.insert(0, ".")
from avse_challenge_amd import kernels as K


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for b, l in ((32, 5999), (64, 3999)):
    for dt in (torch.float32, torch.bfloat16):
        d = 1024
        xz = torch.randn(b, 2 * d, l, device="cuda").to(dt)
        x = xz[:, :d]
        w, bias = torch.randn(d, 4, device="cuda"), torch.randn(d, device="cuda")
        dout = torch.randn(b, d, l, device="cuda").to(dt)
        dx = torch.empty_like(xz)[:, :d]
        tf = timeit(lambda: K.causal_conv1d_fwd(x, w, bias, True))
        tb = timeit(lambda: K.causal_conv1d_bwd(x, w, bias, dout, dx=dx, silu=True))
        s = x.element_size() * b * d * l
        print(f"b={b} l={l} {str(dt):15s} fwd {tf * 1e3:7.1f} us {2 * s / tf / 1e6:6.0f} GB/s   "
              f"bwd {tb * 1e3:7.1f} us {3 * s / tb / 1e6:6.0f} GB/s", flush=True)
