"""Scan fwd/bwd time by dtype and shape (HIP events): separates the bf16 path from the shape (occupancy) effect."""
import sys
import torch
sys.path.insert(0, ".")
from avse_challenge_amd import kernels as K


def run(b, d, l, dt):
    dev = "cuda"
    u, z = torch.randn(b, d, l, device=dev).to(dt), torch.randn(b, d, l, device=dev).to(dt)
    dl = (0.1 * torch.randn(b, d, l, device=dev)).to(dt)
    A = -torch.rand(d, 16, device=dev) - 0.5
    Bm, Cm = torch.randn(b, 16, l, device=dev).to(dt), torch.randn(b, 16, l, device=dev).to(dt)
    D, bias = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    f = lambda: K.selective_scan_fwd(u, dl, A, Bm, Cm, D, z, bias, True, return_out=False)
    _, x, _ = f()
    dout = torch.randn(b, d, l, device=dev).to(dt)
    g = lambda: K.selective_scan_bwd(u, dl, A, Bm, Cm, D, z, bias, dout, x, None, None, True, False)
    res = []
    for fn in (f, g):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / 5)
    print(f"b={b:3d} d={d} l={l} {str(dt):15s} fwd {res[0]:.3f} ms  bwd {res[1]:.3f} ms  "
          f"fwd {res[0] * 1e6 / (b * l):.2f} ns/(row-step of 1024 ch)", flush=True)


for b, l in ((64, 3999), (32, 5999), (64, 5999), (48, 3999)):
    for dt in (torch.float32, torch.bfloat16):
        run(b, 1024, l, dt)
