"""avse1 C1 train-mode forward, fused BN on / off: each BatchNorm site's output vs the fp64 oracle (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import avse1  # noqa: E402
from oracle import avse1_ref  # noqa: E402
from oracle.det_init import det_init_, det_input  # noqa: E402

spec = det_input((1, 1, 376, 257), 508).abs()
ref64 = det_init_(avse1_ref.AVNet(a_only=True), 55).double().train()
outs64 = {}
for name, m in ref64.named_modules():
    if isinstance(m, torch.nn.BatchNorm2d):
        m.register_forward_hook(lambda mod, i, o, n=name: outs64.__setitem__(n, o.detach()))
with torch.no_grad():
    ref64({"noisy_audio_spec": spec.double()})
for b in ("1", "0"):
    os.environ["AVSE_BNACT"] = b
    net = det_init_(avse1.AVNet(a_only=True), 55).cuda().train()
    got = {}
    orig = avse1.bn_act

    def spy(x, bn, act=None, res=None):
        name = [k for k, m in net.named_modules() if m is bn][0]
        os.environ["AVSE_BNACT"] = "0"
        pre = bn(x).detach() if b == "0" else None
        os.environ["AVSE_BNACT"] = b
        y = orig(x, bn, None, res) if b == "1" else pre
        if b == "0":
            bn.num_batches_tracked.sub_(1)
        got[name] = y.detach().double().cpu()
        return y if act is None else torch.relu(y)
    avse1.bn_act = spy
    with torch.no_grad():
        net({"noisy_audio_spec": spec.cuda()})
    avse1.bn_act = orig
    line = []
    for k in outs64:
        t = outs64[k]
        flips = int(((got[k] > 0) != (t > 0)).sum())
        line.append(f"{k.split('.')[-1]}:{float((got[k] - t).abs().max() / t.abs().max()):.1e}/{flips}")
    print(f"bnact={b}: " + " ".join(line), flush=True)
