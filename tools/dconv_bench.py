"""Micro-benchmark of the avse1 AudioFeatNet dilated 64->64 5x5 convolutions at the C2 shape (B=32, 376 x 257,
channels-last): weight gradient on the HIP MFMA kernel (K.dconv_wgrad) vs MIOpen (torch.nn.grad.conv2d_weight); forward
and input gradient on the split-fp16 MFMA kernel (K.dconv_fwd: split + weight prep + conv, and the conv launch alone)
vs MIOpen.  FLOPs per launch 2*B*64*64*25*H*W (633.3 GF at C2, fp32-equivalent); HIP events.
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
    p.add_argument("--dils", default="2,4,8,16")
    a = p.parse_args()
    B, H, W = a.batch, 376, 257
    cl = torch.channels_last
    x = torch.randn(B, 64, H, W, device="cuda").contiguous(memory_format=cl)
    dy = torch.randn(B, 64, H, W, device="cuda").contiguous(memory_format=cl)
    w = (0.05 * torch.randn(64, 64, 5, 5, device="cuda")).contiguous(memory_format=cl)
    flops = 2.0 * B * 64 * 64 * 25 * H * W
    for d in [int(v) for v in a.dils.split(",")]:
        rec = {"dilation": d, "batch": B, "gflop": round(flops / 1e9, 1)}
        ms = timeit(lambda: K.dconv_wgrad(x, dy, d), a.iters)
        rec["hip_wgrad"] = {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1), "frac": round(flops / ms / 1e9 / 157.3, 3)}
        L = K._lib.lib()
        mb = torch.empty(2, device="cuda", dtype=torch.int32)
        xq = K.split16(x, mb)
        wq = K.dconv_wprep(w, False, mb)
        y = torch.empty_like(x)
        conv = lambda: K.check(L.avse_dconv_fwd(B, H, W, d, K.ptr(xq), K.ptr(wq), K.ptr(mb), None, K.ptr(y),  # noqa: E731
                                                K.stream_ptr()), "dconv_fwd")
        for name, fn in (("split_fwd_total", lambda: K.dconv_fwd(x, w, d)),
                         ("split_dgrad_total", lambda: K.dconv_fwd(dy, w, d, transposed=True)),
                         ("split_conv_only", conv), ("split16_only", lambda: K.split16(x, mb)),
                         ("split_wgrad16", lambda: K.dconv_wgrad16((xq, mb[:1]), (xq, mb[:1]), tuple(x.shape), d,
                                                                   bias_grad=True))):
            ms = timeit(fn, a.iters)
            rec[name] = {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1), "frac_fp32": round(flops / ms / 1e9 / 157.3, 3),
                         "frac_f16x3": round(3 * flops / ms / 1e9 / 2500.0, 3)}
        if not a.no_miopen:
            for name, fn in (("miopen_wgrad", lambda: torch.nn.grad.conv2d_weight(x, w.shape, dy, 1, 2 * d, d)),
                             ("miopen_fwd", lambda: torch.nn.functional.conv2d(x, w, None, 1, 2 * d, d)),
                             ("miopen_dgrad", lambda: torch.nn.grad.conv2d_input(x.shape, w, dy, 1, 2 * d, d))):
                ms = timeit(fn, a.iters)
                rec[name] = {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1), "frac": round(flops / ms / 1e9 / 157.3, 3)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
