"""Micro-benchmark of the HIP selective-scan / causal-conv kernels at BASELINE shapes (HIP events).

python tools/scan_bench.py [--cfg B,D,L ...] [--iters N]
Algorithmic bytes: scan fwd 4*L*(5*D + 2*16) per row of B (u, delta, z read; out,
out_z written; B, C read), training fwd (no out) 4*L*(4*D + 2*16); scan bwd 4*L*(9*D + 4*16); causal conv fwd 2*4*D*L, bwd 3*4*D*L.
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
    args = p.parse_args()
    dt = torch.float32 if args.dtype == "fp32" else torch.bfloat16
    es = 4 if dt == torch.float32 else 2
    dev = "cuda"
    for cfg in args.cfg:
        b, d, l = map(int, cfg.split(","))
        g = torch.Generator(device=dev).manual_seed(0)
        u = torch.randn(b, d, l, device=dev, generator=g).to(dt)
        dl = (0.1 * torch.randn(b, d, l, device=dev, generator=g)).to(dt)
        z = torch.randn(b, d, l, device=dev, generator=g).to(dt)
        A = -torch.rand(d, 16, device=dev, generator=g) - 0.5
        Bm = torch.randn(b, 16, l, device=dev, generator=g).to(dt)
        Cm = torch.randn(b, 16, l, device=dev, generator=g).to(dt)
        D, bias = torch.ones(d, device=dev), torch.zeros(d, device=dev)
        res = {}
        for rev in (False, True):
            out, x, oz = K.selective_scan_fwd(u, dl, A, Bm, Cm, D, z, bias, True, reverse=rev)
            ms = timeit(lambda: K.selective_scan_fwd(u, dl, A, Bm, Cm, D, z, bias, True, reverse=rev), args.iters)
            byts = es * b * l * (5 * d + 2 * 16)
            res[f"scan_fwd{'_rev' if rev else ''}"] = (ms, byts / ms / 1e6)
            # training forward (what MambaInnerNoOutProj runs): out_z + checkpoints only, 4*D + 32 per step
            ms = timeit(lambda: K.selective_scan_fwd(u, dl, A, Bm, Cm, D, z, bias, True, reverse=rev,
                                                     return_out=False), args.iters)
            res[f"scan_fwd_train{'_rev' if rev else ''}"] = (ms, es * b * l * (4 * d + 2 * 16) / ms / 1e6)
            gout = torch.randn_like(u)
            ms = timeit(lambda: K.selective_scan_bwd(u, dl, A, Bm, Cm, D, z, bias, gout, x, out, None, True, False,
                                                     reverse=rev), max(2, args.iters // 2))
            byts = es * b * l * (9 * d + 4 * 16)
            res[f"scan_bwd{'_rev' if rev else ''}"] = (ms, byts / ms / 1e6)
        if dt == torch.float32:
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
