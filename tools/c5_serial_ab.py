"""A/B of the serial bf16 BiMamba direction sums (round 6): `--old` runs bench.py with mamba_tasnet.BiMambaSerial
replaced by the round-5 composition (two MambaInnerNoOutProj nodes behind _Fork, the outputs and the xz gradients
summed by torch bf16 adds), so both variants run in one tree on one box.
python tools/c5_serial_ab.py [--old] -- <bench.py args>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from avse_challenge_amd import mamba_tasnet as mt  # noqa: E402


class _OldSerial:
    @staticmethod
    def apply(xz, cw, cb, xw, dw, A, D, db, cw_b, cb_b, xw_b, dw_b, A_b, D_b, db_b):
        x1, x2 = mt._Fork.apply(xz)
        f = mt.MambaInnerNoOutProj.apply(x1, cw, cb, xw, dw, A, D, db)
        bk = mt.MambaInnerNoOutProj.apply(x2, cw_b, cb_b, xw_b, dw_b, A_b, D_b, db_b, True)
        return mt._padded_add(f, bk)


if __name__ == "__main__":
    args = sys.argv[1:]
    if "--old" in args:
        args.remove("--old")
        mt.BiMambaSerial = _OldSerial
    if args and args[0] == "--":
        args = args[1:]
    sys.argv = [bench.__file__] + args
    bench.main()
