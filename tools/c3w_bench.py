"""Time the lip front-end Conv3d weight-gradient kernel at the avse1 (C2) and avse4 (C4) shapes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402

for name, (B, cin, T, H, W) in {"avse1": (32, 3, 75, 96, 96), "avse4": (16, 1, 125, 112, 112)}.items():
    x = torch.randn(B, cin, T, H, W, device="cuda")
    HO, WO = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    dy = torch.randn(B, 64, T, HO, WO, device="cuda")
    for _ in range(2):
        K.conv3d_wgrad(x, dy, (5, 7, 7), (2, 3, 3))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        K.conv3d_wgrad(x, dy, (5, 7, 7), (2, 3, 3))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    flops = 2.0 * B * T * HO * WO * 64 * cin * 245
    print(json.dumps({"shape": name, "ms": round(ms, 3), "TFLOPs": round(flops / ms / 1e9, 1),
                      "frac_fp32_peak": round(flops / ms / 1e9 / 157.3, 3)}), flush=True)
