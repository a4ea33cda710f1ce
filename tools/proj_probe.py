"""Library choices for the C5 (bf16) / C3 (fp32) BiMambaV2 projection GEMMs, default solution selection only (no
exhaustive tuning: TunableOp's candidate sweep faulted the GPU on the stride-0 batched weight, round 3).

python tools/proj_probe.py
Variants of in_proj (W (2di, dm) @ h_b^T -> (b, 2di, l), padded ldc) and out_proj (y_b^T @ W^T -> (b, l, dm)):
  lt:      hipBLASLt (torch default), weight expanded with batch stride 0 (what mamba_tasnet does)
  rocblas: torch.backends.cuda.preferred_blas_library("cublas") -> rocBLAS
  mat:     the weight materialised per batch (no stride-0 operand)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402


def ev_ms(fn, iters=10):
    for _ in range(3):
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
    for tag, b, l, dt, peak in (("C5", 32, 5999, torch.bfloat16, 2500.0), ("C3", 64, 3999, torch.float32, 157.3)):
        dm, di = 512, 1024
        h = torch.randn(b, l, dm, device="cuda").to(dt)
        y = torch.randn(b, di, l, device="cuda").to(dt)
        w_in = (0.05 * torch.randn(2 * di, dm, device="cuda")).to(dt)
        w_out = (0.05 * torch.randn(dm, di, device="cuda")).to(dt)
        xz = K.bdl_empty(b, 2 * di, l, dt, h.device)
        o = torch.empty(b, l, dm, device="cuda", dtype=dt)
        w_in_m = w_in.expand(b, *w_in.shape).contiguous()
        w_out_t = w_out.t()
        w_out_m = w_out_t.expand(b, *w_out_t.shape).contiguous()
        fl_in, fl_out = 2.0 * b * l * dm * 2 * di, 2.0 * b * l * di * dm
        res = {"cfg": tag}
        for lib in ("lt", "rocblas", "mat"):
            torch.backends.cuda.preferred_blas_library("cublas" if lib == "rocblas" else "cublaslt")
            if lib == "mat":
                fin = lambda: torch.bmm(w_in_m, h.transpose(1, 2), out=xz)              # noqa: E731
                fout = lambda: torch.bmm(y.transpose(1, 2), w_out_m, out=o)             # noqa: E731
            else:
                fin = lambda: torch.bmm(w_in.expand(b, *w_in.shape), h.transpose(1, 2), out=xz)   # noqa: E731
                fout = lambda: torch.bmm(y.transpose(1, 2), w_out_t.expand(b, *w_out_t.shape), out=o)  # noqa: E731
            for name, fn, fl in (("in_proj", fin, fl_in), ("out_proj", fout, fl_out)):
                ms = ev_ms(fn)
                res[f"{name}_{lib}"] = {"ms": round(ms, 4), "frac": round(fl / (ms * 1e-3) / 1e12 / peak, 4)}
        torch.backends.cuda.preferred_blas_library("cublaslt")
        # flat: the (channel, batch, time) layout makes every projection ONE GEMM over N = b*l (no batch, no stride 0)
        hf = h.reshape(b * l, dm)
        xzf = torch.empty(2 * di, b * l, device="cuda", dtype=dt)
        yf = torch.randn(di, b * l, device="cuda").to(dt)
        of = torch.empty(b * l, dm, device="cuda", dtype=dt)
        dxzf = torch.randn(2 * di, b * l, device="cuda").to(dt)
        for name, fn, fl in (("in_proj_flat", lambda: torch.mm(w_in, hf.t(), out=xzf), fl_in),
                             ("out_proj_flat", lambda: torch.mm(yf.t(), w_out_t, out=of), fl_out),
                             ("in_proj_dW_flat", lambda: torch.mm(dxzf, hf), fl_in),
                             ("in_proj_dh_flat", lambda: torch.mm(dxzf.t(), w_in), fl_in)):
            ms = ev_ms(fn)
            res[name] = {"ms": round(ms, 4), "frac": round(fl / (ms * 1e-3) / 1e12 / peak, 4)}
        del hf, xzf, yf, of, dxzf
        print(json.dumps(res), flush=True)
        del h, y, xz, o, w_in_m, w_out_m
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
