"""bnact channels-last ReLU vs fp64 over sizes: where do the gradients go wrong? (diagnostic)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd.layers import bn_act  # noqa: E402

torch.manual_seed(0)
for C, H, W, cl in ((64, 8, 8, True), (64, 32, 32, True), (64, 64, 64, True), (64, 128, 128, True),
                    (64, 376, 257, True), (16, 376, 257, True), (64, 376, 257, False), (8, 8, 16, True)):
    shape = (1, C, H, W)
    x = (torch.randn(shape) * 2 + 0.5).double().requires_grad_(True)
    gy = (torch.randn(shape) * 1e-5).double()
    ref = torch.nn.BatchNorm2d(C).double()
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.uniform_(-0.1, 0.1)
    y = torch.relu(ref(x))
    y.backward(gy)
    bn = torch.nn.BatchNorm2d(C).cuda()
    bn.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    fmt = torch.channels_last if cl else torch.contiguous_format
    xg = x.detach().float().cuda().contiguous(memory_format=fmt).requires_grad_(True)
    yg = bn_act(xg, bn, "relu")
    yg.backward(gy.float().cuda())
    e = lambda a, b: float((a.double().cpu() - b).abs().max() / b.abs().max())  # noqa: E731
    bad = ((xg.grad.double().cpu() - x.grad).abs() > 1e-3 * x.grad.abs().max())
    idx = bad.nonzero()[:3].tolist()
    print(f"C={C} HxW={H}x{W} cl={cl}: y {e(yg.detach(), y.detach()):.2e} dx {e(xg.grad, x.grad):.2e} "
          f"dgamma {e(bn.weight.grad, ref.weight.grad):.2e} dbeta {e(bn.bias.grad, ref.bias.grad):.2e} "
          f"bad dx {int(bad.sum())} first {idx}", flush=True)
