"""Micro-benchmark of csrc/dtproj.hip (dt_proj + bias + softplus) at the Mamba-TasNet-L C3 (fp32, 64 x 1024 x 3999)
and AV Mamba C5 (bf16, 32 x 1024 x 5999) shapes, with x as the model passes it (the first 32 rows of x_proj's padded
(b, 64, l) output).  HIP events, best of 3 x 20; frac = (x rows read + delta written) / time / 8 TB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402


def ev_ms(fn, n=20):
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
    dev = torch.device("cuda")
    for tag, (b, d, l), dt in (("C3", (64, 1024, 3999), torch.float32), ("C5", (32, 1024, 5999), torch.bfloat16)):
        g = torch.Generator(device=dev).manual_seed(b + l)
        xdbl = K.bdl_empty(b, 64, l, dt, dev)
        xdbl.copy_(torch.randn(b, 64, l, device=dev, generator=g))
        w = (0.2 * torch.randn(d, 32, device=dev, generator=g)).to(dt)
        bias = torch.randn(d, device=dev, generator=g) - 4.0
        ms = ev_ms(lambda: K.dtproj(w, xdbl[:, :32], bias))
        s = xdbl.element_size()
        byts = s * b * l * (d + 32)
        print(json.dumps({"shape": [b, d, l], "tag": tag, "dtype": str(dt).replace("torch.", ""), "ms": round(ms, 4),
                          "gbps": round(byts / ms / 1e6, 1), "frac": round(byts / ms / 1e6 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
