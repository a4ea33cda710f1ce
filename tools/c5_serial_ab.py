"""A/B of the serial bf16 BiMamba direction sums (round 6): `--old` runs bench.py with mamba_tasnet.BiMambaSerial
replaced by the round-5 composition (two MambaInnerNoOutProj nodes behind _Fork, the outputs and the xz gradients
summed by torch bf16 adds -- fp32: avse_add_max, as round 5's C3), so both variants run in one tree on one box.
python tools/c5_serial_ab.py [--old] -- <bench.py args>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from avse_challenge_amd import mamba_tasnet as mt  # noqa: E402


class _SumFn(torch.autograd.Function):
    """round 5's direction sum: inside the graph, fp32 via avse_add_max (with its max), bf16 a torch add; the gradient
    goes to both directions unchanged (as _BiOutProj's backward handed it)."""

    @staticmethod
    def forward(ctx, f, bk):
        if f.dtype == bk.dtype == torch.float32 and f.stride() == bk.stride():
            fa, fb = mt._padded_full(f), mt._padded_full(bk)
            if fa is not None and fb is not None and fa.is_contiguous() and fb.is_contiguous():
                return mt.K.add_max(fa, fb, f.size(2))
        return mt._padded_add(f, bk)

    @staticmethod
    def backward(ctx, g):
        return g, g


class _OldSerial:
    @staticmethod
    def apply(xz, cw, cb, xw, dw, A, D, db, cw_b, cb_b, xw_b, dw_b, A_b, D_b, db_b):
        x1, x2 = mt._Fork.apply(xz)
        f = mt.MambaInnerNoOutProj.apply(x1, cw, cb, xw, dw, A, D, db)
        bk = mt.MambaInnerNoOutProj.apply(x2, cw_b, cb_b, xw_b, dw_b, A_b, D_b, db_b, True)
        return _SumFn.apply(f, bk)


if __name__ == "__main__":
    args = sys.argv[1:]
    if "--old" in args:
        args.remove("--old")
        mt.BiMambaSerial = _OldSerial
    if args and args[0] == "--":
        args = args[1:]
    sys.argv = [bench.__file__] + args
    bench.main()
