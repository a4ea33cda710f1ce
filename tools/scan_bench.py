"""Micro-benchmark of the HIP selective-scan / causal-conv kernels at BASELINE shapes (HIP events).

python tools/scan_bench.py [--cfg B,D,L ...] [--iters N]
Algorithmic bytes (per row of B): training fwd (u, delta, z, B, C read; out_z written)
s*L*(4*D + 2*16); bwd as the model calls it (u, delta, z, dout, B, C read; du, ddelta, dz, fp32 dB, dC written)
L*(7*s*D + 2*s*16 + 2*4*16); causal conv fwd 2*s*D*L, bwd 3*s*D*L.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402


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
    p.add_argument("--cfg", nargs="*", default=["16,1024,3999", "64,1024,3999", "64,256,3999", "32,1024,5999"])
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--dtype", default="fp32")
    p.add_argument("--pad", action="store_true", help="inputs with a 128-B aligned time stride (set "
                   "AVSE_TIME_ALIGN_BYTES=128 for the outputs too)")
    p.add_argument("--rev", action="store_true", help="also time the reverse-direction launches")
    p.add_argument("--no-conv", action="store_true")
    args = p.parse_args()
    dt = torch.float32 if args.dtype == "fp32" else torch.bfloat16
    es = 4 if dt == torch.float32 else 2
    dev = "cuda"
    for cfg in args.cfg:
        b, d, l = map(int, cfg.replace("x", ",").split(","))   # BxDxL also accepted
        g = torch.Generator(device=dev).manual_seed(0)
        per = 128 // es
        lp = -(-l // per) * per if args.pad else l

        def mk(rows, scale=1.0):
            t = torch.empty(b, rows, lp, device=dev, dtype=dt)
            t[..., :l] = (scale * torch.randn(b, rows, l, device=dev, generator=g)).to(dt)
            return t[..., :l]
        u, dl, z = mk(d), mk(d, 0.1), mk(d)
        A = -torch.rand(d, 16, device=dev, generator=g) - 0.5
        Bm, Cm = mk(16), mk(16)
        D, bias = torch.ones(d, device=dev), torch.zeros(d, device=dev)
        res = {}
        for rev in ((False, True) if args.rev else (False,)):
            sfx = "_rev" if rev else ""
            _, x, _ = K.selective_scan_fwd(u, dl, A, Bm, Cm, D, z, bias, True, reverse=rev, return_out=False)
            # training forward (what MambaInnerNoOutProj runs): out_z + checkpoints only, 4*D + 32 per step
            ms = timeit(lambda: K.selective_scan_fwd(u, dl, A, Bm, Cm, D, z, bias, True, reverse=rev,
                                                     return_out=False), args.iters)
            res["scan_fwd_train" + sfx] = (ms, es * b * l * (4 * d + 2 * 16) / ms / 1e6)
            gout = mk(d)
            # backward as the model calls it (out=None, no out_z recompute): 7 (b, d, l) tensors + B, C, fp32 dB, dC
            ms = timeit(lambda: K.selective_scan_bwd(u, dl, A, Bm, Cm, D, z, bias, gout, x, None, None, True, False,
                                                     reverse=rev), max(2, args.iters // 2))
            res["scan_bwd" + sfx] = (ms, b * l * (7 * es * d + 2 * es * 16 + 2 * 4 * 16) / ms / 1e6)
        if dt == torch.float32 and not args.no_conv:
            w, cb = torch.randn(d, 4, device=dev), torch.randn(d, device=dev)
            ms = timeit(lambda: K.causal_conv1d_fwd(u, w, cb, True), args.iters)
            res["cconv_fwd"] = (ms, 2 * 4 * b * d * l / ms / 1e6)
            ms = timeit(lambda: K.causal_conv1d_bwd(u, w, cb, gout, silu=True), args.iters)
            res["cconv_bwd"] = (ms, 3 * 4 * b * d * l / ms / 1e6)
        print(json.dumps({"cfg": cfg, "dtype": args.dtype,
                          **{k: {"ms": round(v[0], 4), "GBps": round(v[1], 1), "frac_8TBs": round(v[1] / 8000, 4)}
                             for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
