"""A/B of the bf16 projection GEMM (csrc/projgemm.hip) against the library GEMM the model used before (torch.bmm ->
hipBLASLt) at the C5 AV Mamba-TasNet-L shapes (B = 32, L = 5999, d_model 512, d_inner 1024), in the model's layouts.
Checks each result against an fp32 matmul of the same bf16 operands and prints one JSON line per GEMM.

usage: python tools/gemm_probe.py [--reps N] [--batch B] [--seqlen L]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402

BF16_PEAK = 2500.0     # TFLOP/s dense (MI355X_MICROARCH.md)


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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seqlen", type=int, default=5999)
    ap.add_argument("--case", default="", help="run only the GEMMs whose name contains this")
    ap.add_argument("--no-lib", action="store_true", help="skip the library leg")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    b, L, dm, di = args.batch, args.seqlen, 512, 1024
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: torch.randn(*s, device=dev, generator=g).to(bf)  # noqa: E731

    def bdl(d):
        return K.bdl_empty(b, d, L, bf, dev).copy_(torch.randn(b, d, L, device=dev, generator=g))

    w_in, w_out = rnd(2 * di, dm) * 0.05, rnd(dm, di) * 0.05
    h = rnd(b, L, dm)                       # block input (b, l, d_model)
    y = bdl(di)                             # direction sum (b, d_inner, l), padded time stride
    dxz = bdl(2 * di)                       # in_proj output gradient
    dout = rnd(b, L, dm)                    # out_proj output gradient
    cases = []
    # in_proj: xz[b, n, l] = sum_k W_in[n, k] h[b, l, k]
    xz = K.bdl_empty(b, 2 * di, L, bf, dev)
    cases.append(("in_proj fwd", h, w_in[None], xz, 1.0,
                  lambda: torch.bmm(w_in.expand(b, *w_in.shape), h.transpose(1, 2), out=xz),
                  lambda: torch.matmul(w_in.float(), h.float().transpose(1, 2))))
    # out_proj: out[b, l, m] = 0.5 sum_d y[b, d, l] W_out[m, d]
    o = torch.empty(b, L, dm, device=dev, dtype=bf)
    wt = 0.5 * w_out.t()
    cases.append(("out_proj fwd", w_out[None], y.transpose(1, 2), o, 0.5,
                  lambda: torch.bmm(y.transpose(1, 2), wt.expand(b, *wt.shape), out=o),
                  lambda: torch.matmul(y.float().transpose(1, 2), 0.5 * w_out.float().t())))
    # in_proj input gradient: dh[b, l, c] = sum_n dxz[b, n, l] W_in[n, c]
    dh = torch.empty(b, L, dm, device=dev, dtype=bf)
    cases.append(("in_proj dgrad", w_in.t()[None], dxz.transpose(1, 2), dh, 1.0,
                  lambda: torch.bmm(dxz.transpose(1, 2), w_in.expand(b, *w_in.shape), out=dh),
                  lambda: torch.matmul(dxz.float().transpose(1, 2), w_in.float())))
    # out_proj input gradient: dy[b, d, l] = 0.5 sum_m W_out[m, d] dout[b, l, m]
    dy = K.bdl_empty(b, di, L, bf, dev)
    wt2 = 0.5 * w_out.t()
    cases.append(("out_proj dgrad", dout, w_out.t()[None], dy, 0.5,
                  lambda: torch.bmm(wt2.expand(b, *wt2.shape), dout.transpose(1, 2), out=dy),
                  lambda: torch.matmul(0.5 * w_out.float().t(), dout.float().transpose(1, 2))))
    # weight gradients (fp32 out, batches folded: ONE output group per `fold` batches, summed after):
    # dW_in[n, c] = sum_{b,l} dxz[b, n, l] h[b, l, c];  dW_out[m, d] = 0.5 sum_{b,l} dout[b, l, m] y[b, d, l]
    wcases = [("in_proj wgrad", h.transpose(1, 2), dxz, 1.0, 2 * di, dm,
               lambda: torch.bmm(dxz, h).float().sum(0),
               lambda: torch.einsum("bnl,blc->nc", dxz.float(), h.float())),
              ("out_proj wgrad", y, dout.transpose(1, 2), 0.5, dm, di,
               lambda: 0.5 * torch.bmm(dout.transpose(1, 2), y.transpose(1, 2)).float().sum(0),
               lambda: 0.5 * torch.einsum("blm,bdl->md", dout.float(), y.float()))]
    for name, P, Q, alpha, m, n, lib_fn, ref_fn in wcases:
        if args.case not in name:
            continue
        flops = 2.0 * b * L * m * n
        ref = ref_fn()
        rec = {"gemm": name, "m": m, "n": n, "k": b * L, "gflop": round(flops / 1e9, 2)}
        if not args.no_lib:
            lib_ms = timed(lib_fn, args.reps)
            rec.update(lib_ms=round(lib_ms, 4), lib_frac=round(flops / lib_ms / 1e9 / BF16_PEAK, 4),
                       lib_rel_err=float((lib_fn() - ref).norm() / ref.norm()))
        tiles = -(-m // 256) * -(-n // 256)
        fold = max(1, b * tiles // 256)
        while b % fold:
            fold -= 1
        out = torch.empty(b // fold, m, n, device=dev, dtype=torch.float32)
        hip_fn = lambda: K.gemm_bf16(P, Q, out, alpha, fold).sum(0)  # noqa: E731
        hip_ms = timed(hip_fn, args.reps)
        rec.update(fold=fold, hip_ms=round(hip_ms, 4), hip_frac=round(flops / hip_ms / 1e9 / BF16_PEAK, 4),
                   hip_rel_err=float((hip_fn() - ref).norm() / ref.norm()))
        print(json.dumps(rec), flush=True)
    for name, P, Q, out, alpha, lib_fn, ref_fn in cases:
        if args.case not in name:
            continue
        kmax = P.shape[2]
        flops = 2.0 * b * P.shape[1] * Q.shape[1] * kmax
        rec = {"gemm": name, "p": list(P.shape), "q": list(Q.shape), "k": kmax, "gflop": round(flops / 1e9, 2)}
        ref = ref_fn()
        lib_ms = 0.0 if args.no_lib else timed(lib_fn, args.reps)
        lib_err = float((out.float() - ref).norm() / ref.norm())
        out.zero_()
        ok = K.gemm_bf16_supported(P, Q, out)
        rec["hip_supported"] = ok
        if ok:
            hip_ms = timed(lambda: K.gemm_bf16(P, Q, out, alpha), args.reps)
            err = float((out.float() - ref).norm() / ref.norm())
            rec.update(hip_ms=round(hip_ms, 4), hip_frac=round(flops / hip_ms / 1e9 / BF16_PEAK, 4),
                       hip_rel_err=err)
        if not args.no_lib:
            rec.update(lib_ms=round(lib_ms, 4), lib_frac=round(flops / lib_ms / 1e9 / BF16_PEAK, 4), lib_rel_err=lib_err)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
