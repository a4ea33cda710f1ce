"""Gradient-error diagnosis for the avse1 train step (test_avse1_wave_frontend... setting): ours vs the
oracle on the GPU in fp32 and on the CPU in fp32, all against fp64; then ours with PReLU / LipConv3d
swapped for the torch ops, and ours run twice (run-to-run spread)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avse_challenge_amd  # noqa: E402,F401
from avse_challenge_amd import avse1, layers  # noqa: E402
from oracle import avse1_ref, stft_ref  # noqa: E402
from oracle.det_init import det_init_, det_input  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
noisy = 0.1 * det_input((2, 48000), 603)
clean = 0.1 * det_input((2, 48000), 604)
lips = det_input((2, 3, 75, 64, 64), 605, "uint8")
rb = {"noisy_audio_spec": torch.from_numpy(stft_ref.stft_mag_T(noisy.numpy()))[:, None],
      "mask": torch.from_numpy(stft_ref.stft_mag_T(clean.numpy()))[:, None], "lip_images": lips}
rbg = {k: v.cuda() for k, v in rb.items()}


def nodrop(m):
    for x in m.modules():
        if isinstance(x, torch.nn.Dropout):
            x.p = 0.0
    return m


r64 = nodrop(det_init_(avse1_ref.AVNet(), 55).double().train())
r64.cal_loss({k: (v.double() if v.dtype == torch.float32 else v) for k, v in rb.items()}).backward()
truth = dict(r64.named_parameters())


def errs(model):
    out = {}
    for k, p in model.named_parameters():
        q = truth[k]
        if q.grad is None or p.grad is None:
            continue
        out[k] = float((p.grad.double().cpu() - q.grad).abs().max()) / max(1e-12, float(q.grad.abs().max()))
    return out


def ours():
    m = nodrop(det_init_(avse1.AVNet(), 55).cuda().train())
    m.training_step(dict(rbg)).backward()
    return errs(m)


cols = {"ours": ours(), "ours2": ours()}
tg = nodrop(det_init_(avse1_ref.AVNet(), 55).cuda().train())
tg.cal_loss(dict(rbg)).backward()
cols["torchgpu"] = errs(tg)
c32 = nodrop(det_init_(avse1_ref.AVNet(), 55).train())
c32.cal_loss(dict(rb)).backward()
cols["cpu32"] = errs(c32)
orig_fwd = layers.PReLU.forward
layers.PReLU.forward = lambda self, x: F.prelu(x, self.weight)
cols["-prelu"] = ours()
layers.PReLU.forward = orig_fwd
orig_c3 = layers.LipConv3d.forward
layers.LipConv3d.forward = lambda self, x: F.conv3d(x, self.weight, None, self.stride, self.padding)
cols["-c3w"] = ours()
layers.LipConv3d.forward = orig_c3
names = list(cols)
print(f"{'param':52s} " + " ".join(f"{n:>9s}" for n in names))
for k in sorted(cols["ours"], key=lambda k: -cols["ours"][k])[:45]:
    print(f"{k:52s} " + " ".join(f"{cols[n].get(k, float('nan')):9.2e}" for n in names))
