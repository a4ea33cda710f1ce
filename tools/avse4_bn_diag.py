"""avse4 reduced train step: per-parameter gradient error vs fp64 for ours (fused bnact), ours with the library
BatchNorm + ReLU (AVSE_BNACT=0), ours again (run-to-run), and the oracle in fp32 on the GPU and the CPU —
to tell an activation-mask flip from a kernel error (diagnostic, not a test)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import avse4  # noqa: E402
from oracle import avse4_ref  # noqa: E402
from oracle.det_init import det_init_, det_input  # noqa: E402
from oracle.losses_ref import avse4_loss  # noqa: E402

kw = dict(N=64, L=40, B=64, H=128, P=3, X=3, R=2, C=2)
batch = {"noisy_audio": 0.1 * det_input((2, 2, 8000), 611), "vis_feat": det_input((2, 1, 13, 112, 112), 612, "uniform"),
         "clean": 0.1 * det_input((2, 2, 8000), 613)}
bg = {k: v.cuda() for k, v in batch.items()}
b64 = {k: v.double() for k, v in batch.items()}
r64 = det_init_(avse4_ref.AVSE4BaselineModule(num_channels=2, **kw), 61).double().train()
avse4_loss(b64["clean"], r64.model(b64["noisy_audio"], r64.visual_frontend(b64["vis_feat"]))).backward()
truth = dict(r64.named_parameters())


def grads(model):
    return {k: p.grad.double().cpu() for k, p in model.named_parameters() if p.grad is not None}


def ours(bnact):
    os.environ["AVSE_BNACT"] = bnact
    m = det_init_(avse4.AVSE4BaselineModule(num_channels=2, **kw), 61).cuda().train()
    m.training_step(bg).backward()
    return grads(m)


cols = {"ours": ours("1"), "ours2": ours("1"), "lib_bn": ours("0")}
g32 = det_init_(avse4_ref.AVSE4BaselineModule(num_channels=2, **kw), 61).cuda().train()
g32.cal_loss(bg).backward()
cols["torchgpu"] = grads(g32)
c32 = det_init_(avse4_ref.AVSE4BaselineModule(num_channels=2, **kw), 61).train()
c32.cal_loss(batch).backward()
cols["cpu32"] = grads(c32)
names = list(cols)
print(f"{'param':48s} " + " ".join(f"{n:>9s}" for n in names) + "   worst-channel err (ours) / #ch > 1e-3")
for k, q in truth.items():
    if q.grad is None or not k.startswith("visual_frontend"):
        continue
    s = max(1e-6, float(q.grad.abs().max()))
    e = {n: float((c[k] - q.grad).abs().max()) / s for n, c in cols.items()}
    if max(e.values()) < 2e-3:
        continue
    d = ((cols["ours"][k] - q.grad).abs() / s).reshape(q.grad.shape[0], -1).amax(1)
    print(f"{k[16:]:48s} " + " ".join(f"{e[n]:9.2e}" for n in names) + f"   {int(d.argmax())}:{float(d.max()):.2e} / {int((d > 1e-3).sum())}")
