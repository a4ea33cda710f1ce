"""A/B of the world-1 Trainer's gradient buffers (round 6): `--flat` runs bench.py with the round-5 form (every .grad a
view of one zeroed flat buffer that autograd adds into) in place of the round-6 one (.grad reset to None, the computed
gradient handed over without an add).  python tools/trainer_ab.py [--flat] -- <bench.py args>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from avse_challenge_amd import ddp  # noqa: E402

_init = ddp.Trainer.__init__


def _flat_init(self, step, world, dev, *a, **k):
    _init(self, step, world, dev, *a, **k)
    if self.flat is None:
        self.flat = torch.zeros(sum(p.numel() for p in self.params), device=dev)
        off = 0
        for p in self.params:
            seg = self.flat[off:off + p.numel()]
            p.grad = seg.as_strided(p.size(), p.stride()) if ddp._dense(p) else seg.view_as(p)
            off += p.numel()


def _flat_fwd_bwd(self, out=None):
    self.flat.zero_()
    loss = self.step.loss()
    if out is not None:
        out.copy_(loss.detach())
    loss.backward()
    return loss.detach() if out is None else out


if __name__ == "__main__":
    args = sys.argv[1:]
    if "--flat" in args:
        args.remove("--flat")
        ddp.Trainer.__init__ = _flat_init
        ddp.Trainer._fwd_bwd = _flat_fwd_bwd
    if args and args[0] == "--":
        args = args[1:]
    sys.argv = [bench.__file__] + args
    bench.main()
