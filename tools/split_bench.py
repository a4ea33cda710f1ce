"""Micro-benchmark of the split-fp16 operand passes of the C3 (Mamba-TasNet-L, B = 64, L = 3999) projections:
avse_add_max (the BiMamba direction sum over padded (b, 1024, 4000) rows with max |y|) and avse_split16_planes on the
(b, 4000, 512) in_proj input and the (b, 1024, 3999) padded out_proj input.  HIP events, best of 3 x 10; GB/s counts
the bytes each pass must move."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402


def ev_ms(fn, n=10):
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
    b, d, l, lp, dm = 64, 1024, 3999, 4000, 512
    f = torch.randn(b, d, lp, device="cuda")
    g = torch.randn(b, d, lp, device="cuda")
    h = torch.randn(b, l, dm, device="cuda")
    recs = []
    ms = ev_ms(lambda: K.add_max(f, g, l))
    recs.append({"pass": "avse_add_max (b, 1024, 4000 padded)", "ms": round(ms, 4), "GB/s": round(3 * f.numel() * 4 / ms / 1e6, 1)})
    ms = ev_ms(lambda: K.split_planes(h))
    recs.append({"pass": "avse_split16_planes (b, 3999, 512) contiguous", "ms": round(ms, 4),
                 "GB/s": round((2 * h.numel() * 4 + h.numel() * 4) / ms / 1e6, 1), "note": "absmax + split: read 2x, write 1x"})
    setattr(h, K.ABSMAX_ATTR, h.abs().amax().reshape(1).view(torch.int32))       # a producer's max: the split pass only
    ms = ev_ms(lambda: K.split_planes(h))
    recs.append({"pass": "avse_split16_planes_known (b, 3999, 512) contiguous", "ms": round(ms, 4),
                 "GB/s": round(2 * h.numel() * 4 / ms / 1e6, 1)})
    y = K.add_max(f, g, l)
    ms = ev_ms(lambda: K.split_planes(y))
    recs.append({"pass": "avse_split16_planes_known (b, 1024, 3999 of 4000) after add_max", "ms": round(ms, 4),
                 "GB/s": round(2 * y.numel() * 4 / ms / 1e6, 1)})
    for r in recs:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
