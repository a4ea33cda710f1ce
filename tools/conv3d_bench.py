"""Micro-benchmark of the avse1 lip front-end Conv3d(3, 64, (5,7,7), (1,2,2), (2,3,3)) at the C2 shape (B=32, T=75,
96 x 96 uint8 frames): forward on the HIP MFMA kernel (K.conv3d_fwd, uint8 and fp32 input) vs MIOpen (the folded
Conv2d over frames the model ran before, copies included, and F.conv3d); weight gradient on K.conv3d_wgrad (uint8 and
fp32 input).  FLOPs per launch 2*B*T*48*48*64*3*245 (520 GF at C2); HIP events.
python tools/conv3d_bench.py [--batch 32] [--iters 5] [--no-miopen]"""
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
    a = p.parse_args()
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


if __name__ == "__main__":
    main()
