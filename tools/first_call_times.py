"""Which layers pay MIOpen's first-call kernel compilation?  Times the first forward and backward of
every leaf module of a workload's model (synchronised hooks), prints the slowest.
usage: first_call_times.py avse1|avse4 [B]"""
import os
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
torch.backends.cudnn.benchmark = False
which = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dev = torch.device("cuda")
from avse_challenge_amd import data  # noqa: E402

if which == "avse1":
    from avse_challenge_amd import avse1
    model = avse1.AVNet().to(dev).train()
    noisy, clean, lips = data.avse1_batch(B, dev, 1, 96)

    def loss_fn():
        b = avse1.AVNet.features_from_waves(noisy, clean)
        b["lip_images"] = lips
        return model.loss(model(b), b["mask"])
else:
    from avse_challenge_amd import avse4
    model = avse4.AVSE4BaselineModule(num_channels=2).to(dev).train()
    batch = data.avse4_batch(B, dev, 1)

    def loss_fn():
        return model.training_step(batch)

times = defaultdict(float)
t_start = {}


def pre(name):
    def f(m, inp):
        torch.cuda.synchronize()
        t_start[("f", name)] = time.perf_counter()
    return f


def post(name):
    def f(m, inp, out):
        torch.cuda.synchronize()
        times[("fwd", name, type(m).__name__)] += time.perf_counter() - t_start[("f", name)]
    return f


def bpre(name):
    def f(m, gout):
        torch.cuda.synchronize()
        t_start[("b", name)] = time.perf_counter()
    return f


def bpost(name):
    def f(m, gin, gout):
        torch.cuda.synchronize()
        if ("b", name) in t_start:
            times[("bwd", name, type(m).__name__)] += time.perf_counter() - t_start[("b", name)]
    return f


for name, m in model.named_modules():
    if len(list(m.children())) == 0:
        m.register_forward_pre_hook(pre(name))
        m.register_forward_hook(post(name))
        m.register_full_backward_pre_hook(bpre(name))
        m.register_full_backward_hook(bpost(name))
t0 = time.perf_counter()
loss = loss_fn()
torch.cuda.synchronize()
t1 = time.perf_counter()
loss.backward()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"first step: fwd {t1 - t0:.1f}s bwd {t2 - t1:.1f}s", flush=True)
for (k, n, ty), v in sorted(times.items(), key=lambda kv: -kv[1])[:40]:
    if v > 0.5:
        print(f"{v:8.2f}s {k} {ty:20s} {n}", flush=True)
