import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
import avse_challenge_amd  # noqa: E402,F401  (MIOpen find-db path, before any convolution)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture
def golden():
    return load_golden


def pytest_collection_modifyitems(config, items):
    # Multi-process tests (several ranks sharing one card) run after the single-process suite, so under -x a
    # failure there cannot hide the kernel / model parity results (stable: file order kept otherwise).
    items.sort(key=lambda it: os.path.basename(str(it.fspath)) in ("test_gpu_dist.py", "test_dist_cpu.py"))
    # GPU tests need the card; skip them cleanly (not fail) when torch sees no GPU and
    # the user did not explicitly select them.
    try:
        import torch
        have_gpu = torch.cuda.is_available()
    except Exception:
        have_gpu = False
    if have_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
