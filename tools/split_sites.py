"""Diagnostic: every split_planes / split_rows8 call of one eager train step of a bench workload, with the operand's
shape and whether its producer supplied the max (no absmax pass).  usage: python tools/split_sites.py mamba|avse4"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from avse_challenge_amd import kernels as K  # noqa: E402


def main():
    wl = sys.argv[1]
    dev = torch.device("cuda")
    calls = collections.Counter()
    for name in ("split_planes", "split_rows8"):
        orig = getattr(K, name)

        def spy(t, orig=orig, name=name):
            calls[(name, tuple(t.shape), K._known_absmax(t) is not None, t.stride(2) == 1)] += 1
            return orig(t)
        setattr(K, name, spy)
    st = bench.MambaStep(64, dev, 0, 1, "L") if wl == "mamba" else bench.Avse4Step(16, dev, 0, 1)
    loss = st.loss()
    loss.backward()
    torch.cuda.synchronize()
    for k, v in sorted(calls.items(), key=lambda kv: -kv[1]):
        print(v, k, flush=True)


if __name__ == "__main__":
    main()
