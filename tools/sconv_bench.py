"""Micro-benchmark of csrc/sconv.hip (split-fp16 MFMA 3x3 trunk convs) vs MIOpen fp32 at the avse1 C2 lip-trunk shapes
(2400 frames, channels-last): forward, input gradient (stride 1 and the stride-2 phases), weight gradient; split passes timed apart.
One JSON line per layer shape; frac_fp32 = fp32 algorithmic TFLOP/s / 157.3, frac_f16x3 = / (2500 / 3)."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402

CL = torch.channels_last


def ev_ms(fn, n=5):
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=2400)
    p.add_argument("--no-miopen", action="store_true")
    args = p.parse_args()
    dev = "cuda"
    torch.backends.cudnn.benchmark = False
    shapes = [(64, 24, 64, 1), (64, 24, 128, 2), (128, 12, 128, 1), (128, 12, 256, 2), (256, 6, 256, 1),
              (256, 6, 512, 2), (512, 3, 512, 1)]
    N = args.frames
    for ci, H, co, s in shapes:
        g = torch.Generator(device=dev).manual_seed(ci + co)
        x = torch.randn((N, ci, H, H), device=dev, generator=g).contiguous(memory_format=CL)
        w = 0.05 * torch.randn((co, ci, 3, 3), device=dev, generator=g)
        ho = (H - 1) // s + 1
        dy = torch.randn((N, co, ho, ho), device=dev, generator=g).contiguous(memory_format=CL)
        flops = 2.0 * N * ho * ho * co * ci * 9
        xm = torch.empty(1, device=dev, dtype=torch.int32)
        dm = torch.empty(1, device=dev, dtype=torch.int32)
        xq = K.split_nhwc(x, xm)
        dq = K.split_nhwc(dy, dm)
        r = {"shape": [N, ci, H, H, co, s], "gflop": round(flops / 1e9, 1)}

        def rec(name, ms):
            tf = flops / (ms * 1e-3) / 1e12
            r[name] = {"ms": round(ms, 3), "tflops": round(tf, 1), "frac_fp32": round(tf / 157.3, 3),
                       "frac_f16x3": round(tf / (2500 / 3), 3)}

        rec("split_fwd", ev_ms(lambda: K.sconv_fwd((xq, xm), tuple(x.shape), w, s)))
        r["split_x_ms"] = round(ev_ms(lambda: K.split_nhwc(x, xm)), 3)
        if s == 1:
            rec("split_dgrad", ev_ms(lambda: K.sconv_fwd((dq, dm), tuple(dy.shape), w, 1, transposed=True)))
        else:
            rec("split_dgrad", ev_ms(lambda: K.sconv_dgrad2((dq, dm), tuple(x.shape), w)))
        rec("split_wgrad", ev_ms(lambda: K.sconv_wgrad((xq, xm), (dq, dm), tuple(x.shape), co, s)))
        if not args.no_miopen:
            rec("miopen_fwd", ev_ms(lambda: F.conv2d(x, w, None, s, 1)))
            rec("miopen_dgrad", ev_ms(lambda: torch.ops.aten.convolution_backward(
                dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])))
            rec("miopen_wgrad", ev_ms(lambda: torch.ops.aten.convolution_backward(
                dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])))
        print(json.dumps(r), flush=True)
        del x, dy, xq, dq
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
