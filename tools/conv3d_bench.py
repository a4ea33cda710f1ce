"""Micro-benchmark of the avse1 lip front-end Conv3d(3, 64, (5,7,7), (1,2,2), (2,3,3)) at the C2 shape (B=32, T=75,
96 x 96 uint8 frames): forward on the HIP MFMA kernel (K.conv3d_fwd, uint8 and fp32 input) vs MIOpen (the folded
Conv2d over frames the model ran before, copies included, and F.conv3d); weight gradient on K.conv3d_wgrad (uint8 and
fp32 input).  FLOPs per launch 2*B*T*48*48*64*3*245 (520 GF at C2); HIP events.
--avse4: the avse4 front-end Conv3d(1, 64, ...) at C4 (B=16, T=125, 112 x 112 normalised fp32 frames): forward, and
the weight gradient split (round 6) vs exact-fp32 (kernels.C3W_F16 = False), dy's max attached as the BatchNorm
backward attaches it in the model.
python tools/conv3d_bench.py [--batch 32] [--iters 5] [--no-miopen] [--avse4]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avse_challenge_amd  # noqa: E402,F401
from avse_challenge_amd import kernels as K, layers  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dconv_bench import timeit  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--frames", type=int, default=75)
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--no-miopen", action="store_true")
    p.add_argument("--avse4", action="store_true")
    a = p.parse_args()
    if a.avse4:
        return avse4(a)
    B, T = a.batch, a.frames
    xu = torch.randint(0, 256, (B, 3, T, 96, 96), dtype=torch.uint8, device="cuda")
    xf = xu.float()
    w = 0.01 * torch.randn(64, 3, 5, 7, 7, device="cuda")
    dy = torch.randn(B, 64, T, 48, 48, device="cuda")
    flops = 2.0 * B * T * 48 * 48 * 64 * 3 * 245

    def rec(ms):
        return {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1), "frac": round(flops / ms / 1e9 / 157.3, 3)}

    out = {"batch": B, "frames": T, "gflop": round(flops / 1e9, 1)}
    out["hip_fwd_u8"] = rec(timeit(lambda: K.conv3d_fwd(xu, w), a.iters))
    out["hip_fwd_f32"] = rec(timeit(lambda: K.conv3d_fwd(xf, w), a.iters))
    out["hip_wgrad_u8"] = rec(timeit(lambda: K.conv3d_wgrad(xu, dy, (5, 7, 7), (2, 3, 3)), a.iters))
    out["hip_wgrad_f32"] = rec(timeit(lambda: K.conv3d_wgrad(xf, dy, (5, 7, 7), (2, 3, 3)), a.iters))
    if not a.no_miopen:
        out["miopen_fwd_folded"] = rec(timeit(lambda: layers._conv3d_fwd_folded(xf, w, (2, 3, 3)), a.iters))
        out["miopen_fwd_folded_with_cast"] = rec(timeit(lambda: layers._conv3d_fwd_folded(xu.float(), w, (2, 3, 3)),
                                                        a.iters))
        ref = layers._conv3d_fwd_folded(xf, w, (2, 3, 3))
        got = K.conv3d_fwd(xu, w)
        out["max_rel_diff_vs_miopen"] = float((got - ref).abs().max() / ref.abs().max())
    print(json.dumps(out), flush=True)


def avse4(a):
    B, T = 16, 125
    x = (torch.rand(B, 1, T, 112, 112, device="cuda") - 0.421) / 0.165
    w = 0.01 * torch.randn(64, 1, 5, 7, 7, device="cuda")
    dy = torch.randn(B, 64, T, 56, 56, device="cuda")
    setattr(dy, K.ABSMAX_ATTR, dy.abs().amax().reshape(1).view(torch.int32))
    _, xmax = K.conv3d_fwd(x, w, return_xmax=True)
    flops = 2.0 * B * T * 56 * 56 * 64 * 245
    mb = (x.numel() + dy.numel()) * 4 / 1e6

    def rec(ms):
        return {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1), "frac_split": round(flops / ms / 1e9 / 833.3, 3),
                "GB/s": round(mb / ms, 1)}

    out = {"shape": [B, 1, T, 112, 112], "gflop": round(flops / 1e9, 1)}
    out["hip_fwd_f32"] = rec(timeit(lambda: K.conv3d_fwd(x, w), a.iters))
    out["hip_wgrad_f32_split"] = rec(timeit(lambda: K.conv3d_wgrad(x, dy, (5, 7, 7), (2, 3, 3), xmax=xmax), a.iters))
    old = K.C3W_F16
    try:
        K.C3W_F16 = False
        out["hip_wgrad_f32_exact"] = rec(timeit(lambda: K.conv3d_wgrad(x, dy, (5, 7, 7), (2, 3, 3)), a.iters))
        ex = K.conv3d_wgrad(x, dy, (5, 7, 7), (2, 3, 3))
    finally:
        K.C3W_F16 = old
    sp = K.conv3d_wgrad(x, dy, (5, 7, 7), (2, 3, 3), xmax=xmax)
    out["wgrad_split_vs_exact_max_rel"] = float((sp - ex).abs().max() / ex.abs().max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
