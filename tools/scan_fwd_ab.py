"""A/B of the two selective-scan forward kernels (avse_scan_fwd_variant 1 vs 2) at the BASELINE shapes: bitwise
equality of out_z and the checkpoints, and the HIP-event time of each (interleaved repeats).
python tools/scan_fwd_ab.py [--reps 5]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402


def ev_ms(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    for (b, d, l, dt) in [(64, 1024, 3999, torch.float32), (32, 1024, 5999, torch.bfloat16)]:
        def rnd(*s, scale=1.0):
            if len(s) == 3:
                t = K.bdl_empty(*s, dt, dev)
                t.copy_(scale * torch.randn(s, device=dev, generator=g))
                return t
            return (scale * torch.randn(s, device=dev, generator=g)).to(dt)
        u, delta, z = rnd(b, d, l), rnd(b, d, l, scale=0.5), rnd(b, d, l)
        A = -torch.exp(0.5 * torch.randn(d, 16, device=dev, generator=g))
        Bm, Cm = rnd(b, 1, 16, l), rnd(b, 1, 16, l)
        D = torch.randn(d, device=dev, generator=g)
        bias = 0.1 * torch.randn(d, device=dev, generator=g)
        s = 2 if dt == torch.bfloat16 else 4
        byts = s * l * (4 * d + 2 * 16) * b
        outs, times = {}, {1: [], 2: []}
        for v in (1, 2):
            K.SCAN_FWD_VARIANT = v
            outs[v] = K.selective_scan_fwd(u, delta, A, Bm, Cm, D, z, bias, True)
        torch.cuda.synchronize()
        same = bool(torch.equal(outs[1][2], outs[2][2])) and bool(torch.equal(outs[1][1], outs[2][1]))
        for _ in range(args.reps):
            for v in (1, 2):
                K.SCAN_FWD_VARIANT = v
                times[v].append(ev_ms(lambda: K.selective_scan_fwd(u, delta, A, Bm, Cm, D, z, bias, True)))
        K.SCAN_FWD_VARIANT = 1
        res = {"shape": [b, d, l], "dtype": str(dt), "bitwise_equal": same}
        for v in (1, 2):
            ms = min(times[v])
            res[f"v{v}_ms"] = round(ms, 4)
            res[f"v{v}_frac"] = round(byts / (ms * 1e-3) / 8e12, 4)
        print(json.dumps(res), flush=True)
        del u, delta, z, Bm, Cm, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
