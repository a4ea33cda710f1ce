"""Probe: can a grouped LSTM launch (csrc/lstm_group.hip, B = 32 x 8 workgroups) be made non-co-resident by a
bounded kernel holding all CUs but 4 (tests/hip/occupy.hip, 160 KB LDS per workgroup)?  Runs the occupier in a child
process (or this one: --same), launches the LSTM once the occupier is resident, and reports whether the kernel's
hand-off waits timed out (the sticky error flag) and how long the launch took.  Round 4 on MI355X: the LSTM never
ran beside the occupier (same process, high-priority stream, or another process): it completed only after the
occupier ended, so no timeout could be forced this way.
python tools/lstm_hog_probe.py [seconds]"""
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from avse_challenge_amd import kernels as K  # noqa: E402

CHILD = r"""
import ctypes, os, sys, time, torch
occ = ctypes.CDLL(os.path.join(sys.argv[1], "tests", "hip", "libocc.so"))
ncu = torch.cuda.get_device_properties(0).multi_processor_count
arrived = torch.zeros(1, dtype=torch.int32, device="cuda")
hog = torch.cuda.Stream()
assert occ.occupy_cus(ncu - 4, ctypes.c_void_p(arrived.data_ptr()), ctypes.c_double(float(sys.argv[2])),
                      ctypes.c_void_p(hog.cuda_stream)) == 0
t = time.time()
with torch.cuda.stream(torch.cuda.Stream()):
    while int(arrived.item()) < ncu - 4 and time.time() - t < 3.0:
        time.sleep(0.005)
    print("HELD", int(arrived.item()), ncu, flush=True)
hog.synchronize()
print("DONE", flush=True)
"""

sec = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
hog = subprocess.Popen([sys.executable, "-c", CHILD, ROOT, str(sec)], stdout=subprocess.PIPE, text=True)
print(hog.stdout.readline().strip(), flush=True)
B, T, H = 32, 4, 257
gx = torch.randn(B, T, 4 * H, device="cuda")
w = 0.06 * torch.randn(4 * H, H, device="cuda")
t = time.time()
K.lstm_fwd(gx, w)
torch.cuda.synchronize()
print(f"lstm launch took {time.time() - t:.3f} s; error flag {K.lstm_group_status():#x}", flush=True)
print(hog.stdout.readline().strip(), flush=True)
hog.wait(timeout=60)
