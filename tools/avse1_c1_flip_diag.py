"""C1 (audio-only avse1, batch 1) train-mode forward vs the fp64 oracle with the fused BN kernels on / off:
prediction error and the number of sign flips of (pred - mask) that the L1 gradient sees (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import avse1  # noqa: E402
from oracle import avse1_ref  # noqa: E402
from oracle.det_init import det_init_, det_input  # noqa: E402

spec, mask = det_input((1, 1, 376, 257), 508).abs(), det_input((1, 1, 376, 257), 509).abs()
ref64 = det_init_(avse1_ref.AVNet(a_only=True), 55).double().train()
with torch.no_grad():
    p64 = ref64({"noisy_audio_spec": spec.double()})
d64 = p64 - mask.double()
for b in ("1", "0", "1"):
    os.environ["AVSE_BNACT"] = b
    net = det_init_(avse1.AVNet(a_only=True), 55).cuda().train()
    with torch.no_grad():
        p = net({"noisy_audio_spec": spec.cuda()}).double().cpu()
    d = p - mask.double()
    flips = int(((d > 0) != (d64 > 0)).sum())
    print(f"bnact={b}: max|pred - fp64| {float((p - p64).abs().max()):.3e}  rms {float((p - p64).pow(2).mean().sqrt()):.3e}"
          f"  sign flips {flips} of {d.numel()}", flush=True)

# gradient accuracy per parameter (train mode, L1 loss) vs fp64, fused BN on / off
ref64.zero_grad()
ref64.cal_loss({"noisy_audio_spec": spec.double(), "mask": mask.double()}).backward()
truth = {k: q.grad for k, q in ref64.named_parameters() if q.grad is not None}
res = {}
for b in ("1", "0"):
    os.environ["AVSE_BNACT"] = b
    net = det_init_(avse1.AVNet(a_only=True), 55).cuda().train()
    net.training_step({"noisy_audio_spec": spec.cuda(), "mask": mask.cuda()}).backward()
    for k, q in net.named_parameters():
        if k in truth and q.grad is not None:
            t = truth[k].reshape(-1)
            g = q.grad.double().cpu().reshape(-1)
            cos = float((g * t).sum() / (g.norm() * t.norm() + 1e-300))
            res.setdefault(k, {})[b] = (float((g - t).abs().max() / (t.abs().max() + 1e-300)), 1 - cos)
for k, v in res.items():
    print(f"{k:40s} on e={v['1'][0]:.2e} 1-cos={v['1'][1]:.2e} | off e={v['0'][0]:.2e} 1-cos={v['0'][1]:.2e}")
