"""C5 (bf16) BiMamba in_proj / out_proj forward GEMM: the product's strided-batched call vs alternative operand
layouts, one line per measurement (HIP events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402
from avse_challenge_amd import mamba_tasnet as M  # noqa: E402


def t(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


b, l, dm, di, dt = 32, 5999, 512, 1024, torch.bfloat16
fl_in = 2.0 * b * l * dm * 2 * di
h = torch.randn(b, l, dm, device="cuda", dtype=dt)
w = torch.randn(2 * di, dm, device="cuda", dtype=dt) * 0.05


def report(name, ms, fl):
    print(f"{name:55s} {ms:.3f} ms  {fl / ms / 1e9:.0f} TF/s  ({fl / ms / 1e9 / 2500:.3f} of bf16 peak)", flush=True)


with torch.no_grad():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        report("product _InProj (bmm, padded (b, 2di, l) out)", t(lambda: M._InProj.apply(h, w)), fl_in)
    report("bmm contiguous out (b, 2di, l)", t(lambda: torch.bmm(w.expand(b, *w.shape), h.transpose(1, 2))), fl_in)
    out = K.bdl_empty(b, 2 * di, l, dt, h.device)
    report("bmm out= padded (b, 2di, l)", t(lambda: torch.bmm(w.expand(b, *w.shape), h.transpose(1, 2), out=out)), fl_in)
    h2 = h.reshape(b * l, dm)
    report("linear (b*l, 2di) row-major out", t(lambda: torch.nn.functional.linear(h2, w)), fl_in)
    report("mm W @ H^T (2di, b*l)", t(lambda: torch.mm(w, h2.t())), fl_in)
    hT = h.transpose(1, 2).contiguous()           # (b, dm, l): the operand already channels-first
    report("bmm W @ hT (b, dm, l) contiguous operand", t(lambda: torch.bmm(w.expand(b, *w.shape), hT)), fl_in)
    report("matmul broadcast W @ hT", t(lambda: torch.matmul(w, hT)), fl_in)
    f = torch.randn(b, di, l, device="cuda", dtype=dt)
    wo = torch.randn(dm, di, device="cuda", dtype=dt) * 0.05
    fl_out = 2.0 * b * l * di * dm
    with torch.autocast("cuda", dtype=torch.bfloat16):
        report("product _BiOutProj (add + bmm -> (b, l, dm))", t(lambda: M._BiOutProj.apply(f, f, wo)), fl_out)
    report("bmm f^T W^T (b, l, dm)", t(lambda: torch.bmm(f.transpose(1, 2), wo.t().expand(b, di, dm))), fl_out)
    fr = f.transpose(1, 2).contiguous()
    report("linear on (b*l, di) row-major operand", t(lambda: torch.nn.functional.linear(fr.reshape(b * l, di), wo)), fl_out)
