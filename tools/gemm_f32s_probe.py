"""A/B of the fp32 projection GEMM on split fp16 planes (csrc/projgemm.hip avse_gemm_f32s, kernels.gemm_f32s) against
hipBLASLt fp32 (torch.bmm / matmul) at the Mamba-TasNet-L C3 shapes (B = 64, L = 3999, d_model 512, d_inner 1024), in
the model's layouts.  Prints one JSON line per GEMM: time of the whole call (both splits + GEMM), of the GEMM launch
alone, the library's time, and the fp32-equivalent rate.  usage: python tools/gemm_f32s_probe.py [--batch B] [--reps N]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402

FP32_PEAK, F16_PEAK = 157.3, 2500.0


def timed(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seqlen", type=int, default=3999)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    b, L, dm, di = args.batch, args.seqlen, 512, 1024
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(b, L, dm, device=dev, generator=g)
    w_in, w_out = 0.05 * torch.randn(2 * di, dm, device=dev, generator=g), 0.05 * torch.randn(dm, di, device=dev, generator=g)
    dxz = K.bdl_empty(b, 2 * di, L, torch.float32, dev).copy_(torch.randn(b, 2 * di, L, device=dev, generator=g))
    y = K.bdl_empty(b, di, L, torch.float32, dev).copy_(torch.randn(b, di, L, device=dev, generator=g))
    xz = K.bdl_empty(b, 2 * di, L, torch.float32, dev)
    dh = torch.empty(b, L, dm, device=dev)
    o = torch.empty(b, L, dm, device=dev)
    dwin = torch.empty(b // 8, 2 * di, dm, device=dev)
    cases = [
        ("in_proj fwd", 2.0 * b * L * dm * 2 * di, (h, w_in[None], xz, 1.0, 1),
         lambda: torch.bmm(w_in.expand(b, -1, -1), h.transpose(1, 2))),
        ("in_proj dgrad", 2.0 * b * L * dm * 2 * di, (w_in.t()[None], dxz.transpose(1, 2), dh, 1.0, 1),
         lambda: torch.bmm(dxz.transpose(1, 2), w_in.expand(b, -1, -1))),
        ("in_proj wgrad", 2.0 * b * L * dm * 2 * di, (h.transpose(1, 2), dxz, dwin, 1.0, 8),
         lambda: dxz.transpose(0, 1).reshape(2 * di, -1) @ h.reshape(-1, dm) if dxz.is_contiguous() else
         torch.bmm(dxz, h).sum(0)),
        ("out_proj fwd", 2.0 * b * L * dm * di, (w_out[None], y.transpose(1, 2), o, 0.5, 1),
         lambda: torch.bmm(y.transpose(1, 2), (0.5 * w_out.t()).expand(b, -1, -1))),
    ]
    for name, flops, (P, Q, out, alpha, fold), lib in cases:
        ms = timed(lambda: K.gemm_f32s(P, Q, out, alpha, fold), args.reps)
        sp, sq = K.split_planes(P), K.split_planes(Q)
        ph, pl, pm, qh, ql, qm = sp.hi, sp.lo, sp.mb, sq.hi, sq.lo, sq.mb
        ms_s = timed(lambda: K.split_planes(Q), args.reps)
        a = K._lib.GemmF32sArgs()
        a.batch, a.mp, a.mq, a.k, a.fold = out.shape[0] * fold, P.shape[1], Q.shape[1], P.shape[2], fold
        a.p_hi, a.p_lo, (a.p_bs, a.p_sx, a.p_sk), a.p_extent, a.p_max = ph.data_ptr(), pl.data_ptr(), \
            K._gemm_operand(ph), K._extent(ph), pm.data_ptr()
        a.q_hi, a.q_lo, (a.q_bs, a.q_sx, a.q_sk), a.q_extent, a.q_max = qh.data_ptr(), ql.data_ptr(), \
            K._gemm_operand(qh), K._extent(qh), qm.data_ptr()
        a.c, a.c_bs, a.c_sq, a.alpha = out.data_ptr(), out.stride(0), out.stride(1), float(alpha)
        ms_g = timed(lambda: K.check(K._lib.lib().avse_gemm_f32s(a, K.stream_ptr(dev)), "gemm"), args.reps)
        ms_l = timed(lib, args.reps)
        rec = {"gemm": name, "shape": [b, L, dm, di], "gflop": round(flops / 1e9, 1),
               "f32s_total_ms": round(ms, 3), "f32s_gemm_ms": round(ms_g, 3), "split_q_ms": round(ms_s, 3),
               "q_elems": Q.numel(), "lib_ms": round(ms_l, 3),
               "f32s_gemm_frac_f16x3": round(3 * flops / ms_g / 1e9 / F16_PEAK, 3),
               "f32s_total_tflops_fp32eq": round(flops / ms / 1e9, 1), "lib_frac_fp32": round(flops / ms_l / 1e9 / FP32_PEAK, 3)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
