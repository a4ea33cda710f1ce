"""Micro-benchmark of the avse1 AudioFeatNet dilated 64->64 5x5 convolutions at the C2 shape (B=32, 376 x 257,
channels-last): weight gradient on the HIP MFMA kernel (K.dconv_wgrad) vs MIOpen (torch.nn.grad.conv2d_weight), plus
MIOpen forward / input-gradient for reference.  FLOPs per launch 2*B*64*64*25*H*W (633.3 GF at C2); HIP events.
python tools/dconv_bench.py [--batch 32] [--iters 5]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avse_challenge_amd  # noqa: E402,F401
from avse_challenge_amd import kernels as K  # noqa: E402

os.environ.setdefault("PYTORCH_MIOPEN_SUGGEST_NHWC", "1")


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
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--no-miopen", action="store_true")
    a = p.parse_args()
    B, H, W = a.batch, 376, 257
    cl = torch.channels_last
    x = torch.randn(B, 64, H, W, device="cuda").contiguous(memory_format=cl)
    dy = torch.randn(B, 64, H, W, device="cuda").contiguous(memory_format=cl)
    w = (0.05 * torch.randn(64, 64, 5, 5, device="cuda")).contiguous(memory_format=cl)
    flops = 2.0 * B * 64 * 64 * 25 * H * W
    for d in (2, 4, 8, 16):
        rec = {"dilation": d, "batch": B, "gflop": round(flops / 1e9, 1)}
        ms = timeit(lambda: K.dconv_wgrad(x, dy, d), a.iters)
        rec["hip_wgrad"] = {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1), "frac": round(flops / ms / 1e9 / 157.3, 3)}
        if not a.no_miopen:
            for name, fn in (("miopen_wgrad", lambda: torch.nn.grad.conv2d_weight(x, w.shape, dy, 1, 2 * d, d)),
                             ("miopen_fwd", lambda: torch.nn.functional.conv2d(x, w, None, 1, 2 * d, d)),
                             ("miopen_dgrad", lambda: torch.nn.grad.conv2d_input(x.shape, w, dy, 1, 2 * d, d))):
                ms = timeit(fn, a.iters)
                rec[name] = {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1), "frac": round(flops / ms / 1e9 / 157.3, 3)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
