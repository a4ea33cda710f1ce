"""Lip Conv3d(Cin, 64, (5,7,7), (1,2,2), (2,3,3)) forward (default: the avse1 C2 shape; argv[1] = "B,Cin,T,H,W"): the library's 3-D path vs the time-folded Conv2d
(layers._conv3d_fwd_folded), immediate mode and after a MIOpen find (records go to MIOPEN_USER_DB_PATH). HIP events."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avse_challenge_amd  # noqa: E402,F401
from avse_challenge_amd.layers import _conv3d_fwd_folded  # noqa: E402


def ms(fn, n=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


shape = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "32,3,75,96,96").split(","))   # B,Cin,T,H,W
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.floor(256 * torch.rand(*shape, device="cuda", generator=g))
w = 0.01 * torch.randn(64, shape[1], 5, 7, 7, device="cuda", generator=g)
ref = lambda: F.conv3d(x, w, None, (1, 2, 2), (2, 3, 3))  # noqa: E731
fold = lambda: _conv3d_fwd_folded(x, w, (2, 3, 3))  # noqa: E731
a, b = ref(), fold()
print("max rel diff", float((a - b).abs().max() / a.abs().max()), flush=True)
print("conv3d", round(ms(ref), 3), "ms; fold (immediate)", round(ms(fold), 3), "ms", flush=True)
torch.backends.cudnn.benchmark = True
fold()
torch.cuda.synchronize()
print("fold (after find)", round(ms(fold), 3), "ms", flush=True)
