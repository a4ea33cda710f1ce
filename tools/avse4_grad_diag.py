"""Gradient-error diagnosis for the reduced avse4 train step: ours (HIP) vs the oracle in fp32 on the
GPU (torch/MIOpen) and on the CPU, all against the fp64 oracle; then ours with one HIP op at a time
swapped for its torch equivalent, to see which op carries the error."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import avse4  # noqa: E402
from oracle import avse4_ref  # noqa: E402
from oracle.det_init import det_init_, det_input  # noqa: E402
from oracle.losses_ref import avse4_loss  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
kw = dict(N=64, L=40, B=64, H=128, P=3, X=3, R=2, C=2)
batch = {"noisy_audio": 0.1 * det_input((2, 2, 8000), 611), "vis_feat": det_input((2, 1, 13, 112, 112), 612, "uniform"),
         "clean": 0.1 * det_input((2, 2, 8000), 613)}
bg = {k: v.cuda() for k, v in batch.items()}
b64 = {k: v.double() for k, v in batch.items()}
r64 = det_init_(avse4_ref.AVSE4BaselineModule(num_channels=2, **kw), 61).double().train()
avse4_loss(b64["clean"], r64.model(b64["noisy_audio"], r64.visual_frontend(b64["vis_feat"]))).backward()
truth = dict(r64.named_parameters())


def errs(model):
    out = {}
    for k, p in model.named_parameters():
        q = truth[k]
        if q.grad is None or p.grad is None:
            continue
        s = max(1e-3, float(q.grad.abs().max()))
        out[k] = float((p.grad.double().cpu() - q.grad).abs().max()) / s
    return out


def run_ours():
    m = det_init_(avse4.AVSE4BaselineModule(num_channels=2, **kw), 61).cuda().train()
    m.training_step(bg).backward()
    return errs(m)


def gln_torch(x, a, g, b, eps=1e-8):
    y = F.prelu(x, a)
    mean = y.mean(dim=(1, 2), keepdim=True)
    var = ((y - mean) ** 2).mean(dim=(1, 2), keepdim=True)
    return g * (y - mean) / torch.pow(var + eps, 0.5) + b


cols = {}
cols["ours"] = run_ours()
g32 = det_init_(avse4_ref.AVSE4BaselineModule(num_channels=2, **kw), 61).cuda().train()
g32.cal_loss(bg).backward()
cols["torchgpu"] = errs(g32)
c32 = det_init_(avse4_ref.AVSE4BaselineModule(num_channels=2, **kw), 61).train()
c32.cal_loss(batch).backward()
cols["cpu32"] = errs(c32)
orig = (avse4.prelu_gln, avse4.dwconv1d, avse4._PReLUFn)
avse4.prelu_gln = gln_torch
cols["-gln"] = run_ours()
avse4.prelu_gln = orig[0]
avse4.dwconv1d = lambda x, w, d: F.conv1d(x, w, None, 1, (w.shape[-1] - 1) // 2 * d, d, x.shape[1])
cols["-dwconv"] = run_ours()
avse4.dwconv1d = orig[1]


class _P:
    apply = staticmethod(F.prelu)


avse4._PReLUFn = _P
cols["-prelu"] = run_ours()
avse4._PReLUFn = orig[2]
names = list(cols)
print(f"{'param':56s} " + " ".join(f"{n:>9s}" for n in names))
for k in cols["ours"]:
    print(f"{k:56s} " + " ".join(f"{cols[n].get(k, float('nan')):9.2e}" for n in names))
