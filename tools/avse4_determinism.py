"""Run-to-run check of the avse4 train step: repeat the same step on fresh identical models and
report the max gradient difference between repeats (HIP path), then the same for each HIP op alone."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import avse4, kernels as K  # noqa: E402
from oracle.det_init import det_init_, det_input  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
kw = dict(N=64, L=40, B=64, H=128, P=3, X=3, R=2, C=2)
batch = {"noisy_audio": 0.1 * det_input((2, 2, 8000), 611), "vis_feat": det_input((2, 1, 13, 112, 112), 612, "uniform"),
         "clean": 0.1 * det_input((2, 2, 8000), 613)}
bg = {k: v.cuda() for k, v in batch.items()}


def grads(only_sep=False):
    m = det_init_(avse4.AVSE4BaselineModule(num_channels=2, **kw), 61).cuda().train()
    if only_sep:
        vis = torch.randn(2, 13, 512, generator=torch.Generator().manual_seed(5)).cuda()
        est = m.model(bg["noisy_audio"], vis)
        from avse_challenge_amd.losses import avse4_loss
        avse4_loss(bg["clean"], est).backward()
    else:
        m.training_step(bg).backward()
    return {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}


for only_sep in (False, True):
    ref = grads(only_sep)
    worst = {}
    for rep in range(4):
        g = grads(only_sep)
        for k in ref:
            d = float((g[k] - ref[k]).abs().max()) / max(1e-12, float(ref[k].abs().max()))
            worst[k] = max(worst.get(k, 0.0), d)
    top = sorted(worst.items(), key=lambda kv: -kv[1])[:8]
    print("separator only" if only_sep else "full step", "max rel diff between repeats:", flush=True)
    for k, v in top:
        print(f"   {k:56s} {v:.3e}")

x = torch.randn(2, 128, 399, device="cuda")
w = torch.randn(128, 1, 3, device="cuda")
a = torch.full((1,), 0.25, device="cuda")
gm, bt = torch.rand(128, device="cuda") + 0.5, torch.randn(128, device="cuda")
dy = torch.randn_like(x)
r0 = [K.dwconv_fwd(x, w, 4), *K.dwconv_bwd(x, w, dy, 4)]
y0, st0 = K.prelu_gln_fwd(x, a, gm, bt)
q0 = K.prelu_gln_bwd(x, a, gm, st0, dy)
bad = 0
for _ in range(200):
    r = [K.dwconv_fwd(x, w, 4), *K.dwconv_bwd(x, w, dy, 4)]
    y, st = K.prelu_gln_fwd(x, a, gm, bt)
    q = K.prelu_gln_bwd(x, a, gm, st, dy)
    bad += sum(int(not torch.equal(u, v)) for u, v in zip(r + [y, st, *q], r0 + [y0, st0, *q0]))
print("kernel repeats with any bit difference:", bad, flush=True)
