"""Micro-benchmark of the LSTM recurrence kernels at the avse1 C2 FusionNet shape (B=32, T=376, H=257): the grouped
kernels (csrc/lstm_group.hip, W_hh in LDS over G workgroups per sequence) vs one workgroup per sequence (csrc/lstm.hip).
python tools/lstm_bench.py [--batch 32] [--iters 10]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avse_challenge_amd  # noqa: E402,F401
from avse_challenge_amd import kernels as K  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dconv_bench import timeit  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--frames", type=int, default=376)
    p.add_argument("--hidden", type=int, default=257)
    p.add_argument("--iters", type=int, default=10)
    a = p.parse_args()
    B, T, H = a.batch, a.frames, a.hidden
    gx = torch.randn(B, T, 4 * H, device="cuda")
    w = 0.06 * torch.randn(4 * H, H, device="cuda")
    dh = torch.randn(B, T, H, device="cuda")
    out = {"batch": B, "frames": T, "hidden": H, "groups": int(K._lib.lib().avse_lstm_group_size(B, H))}
    for mode in ("1", "0"):
        os.environ["AVSE_LSTM_GROUP"] = mode
        h, c, g = K.lstm_fwd(gx, w)
        f = timeit(lambda: K.lstm_fwd(gx, w), a.iters)
        b = timeit(lambda: K.lstm_bwd(dh, g, c, w), a.iters)
        key = "grouped" if mode == "1" else "one_wg_per_sequence"
        out[key] = {"fwd_ms": round(f, 3), "bwd_ms": round(b, 3), "fwd_us_per_step": round(1e3 * f / T, 2),
                    "bwd_us_per_step": round(1e3 * b / T, 2)}
    out["status"] = K.lstm_group_status()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
