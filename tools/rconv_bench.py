"""Micro-benchmark of the avse1 lip-trunk 3x3 convolution weight gradients at the C2 shape (B*T = 2400 frames of
96x96 lips: 24 .. 3 pixels): HIP MFMA kernel (K.rconv_wgrad) vs MIOpen (torch.nn.grad.conv2d_weight), NCHW fp32.
FLOPs per launch 2*N*COUT*CIN*9*HO*WO; HIP events.  python tools/rconv_bench.py [--frames 2400] [--iters 5]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avse_challenge_amd  # noqa: E402,F401
from avse_challenge_amd import kernels as K  # noqa: E402

SHAPES = [(64, 64, 24, 1), (64, 128, 24, 2), (128, 128, 12, 1), (128, 256, 12, 2), (256, 256, 6, 1), (256, 512, 6, 2),
          (512, 512, 3, 1)]


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=2400)
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--nhwc", action="store_true", help="channels-last activations (the NHWC kernel / MIOpen NHWC)")
    a = p.parse_args()
    N = a.frames
    for cin, cout, hw, s in SHAPES:
        ho = (hw - 1) // s + 1
        fmt = torch.channels_last if a.nhwc else torch.contiguous_format
        x = torch.randn(N, cin, hw, hw, device="cuda").contiguous(memory_format=fmt)
        dy = torch.randn(N, cout, ho, ho, device="cuda").contiguous(memory_format=fmt)
        flops = 2.0 * N * cout * cin * 9 * ho * ho
        rec = {"cin": cin, "cout": cout, "hw": hw, "stride": s, "nhwc": a.nhwc, "gflop": round(flops / 1e9, 1)}
        for name, fn in (("hip", lambda: K.rconv_wgrad(x, dy, s)),
                         ("miopen", lambda: torch.nn.grad.conv2d_weight(x, (cout, cin, 3, 3), dy, s, 1))):
            ms = timeit(fn, a.iters)
            rec[name] = {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1), "frac": round(flops / ms / 1e9 / 157.3, 3)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
