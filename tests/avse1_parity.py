"""avse1 train-step gradient parity against the fp64 oracle with OUR run's activation masks imposed (test helper).

Why: a ReLU / PReLU whose input sits within fp32 rounding of 0 takes one branch in an fp32 run and possibly the other
in fp64.  One such flip moves one term of the activation's BatchNorm bias gradient, which is a sum of thousands of
terms cancelling to ~1e-2 of their size in the avse1 ResNet trunk: measured 1.1e-2 of the gradient's max at
net_visualfeat.trunk.layer3.0.bn1 from 2 flips with |z| < 8e-7, while the gradient reaching that site was within
3.5e-6 of fp64 (tools/avse1_site_diag.py @ 8f1eec2, profiles/r03_avse1_site_diag.txt).  No fp32 tolerance separates that from
a bug.  So the truth is the fp64 oracle evaluated with the activation patterns (and L1 signs) of the run under test:
every ReLU / PReLU of baseline/avse1/model.py:29-34, 199-215, utils/resnet.py:26-67 and utils/tcn.py:144-243 and the
L1 loss of model.py:164-168 are replaced by torch.where on our masks, and each disagreement with fp64's own sign must
be a rounding-level one (|z64| tiny against the site's scale), which the helper asserts.  What remains between the
two runs is then fp32 arithmetic error only, which the tests bound tightly.
"""
import contextlib

import torch

from avse_challenge_amd import avse1, layers

Z_TIE = 1e-4      # a flip is legitimate only where |z64| <= Z_TIE * max|z64| of its site (fp32 rounding: ~1e-6)


@contextlib.contextmanager
def capture_masks(model):
    """While active, every forward of the avse_challenge_amd AVNet ``model`` records (CPU bool tensors, keyed by the
    oracle's module names): the sign pattern of each bn_act ReLU / PReLU output (y > 0 <=> z > 0 for a positive
    slope), of each TCN PReLU module, and the prediction (key "pred")."""
    masks = {}
    names = {id(m): n for n, m in model.named_modules()}
    orig = avse1.bn_act

    def spy(x, bn, act=None, res=None, folded_bias=None, **kw):
        y = orig(x, bn, act, res, folded_bias=folded_bias, **kw)
        if act is not None:
            key = names[id(bn)] if act == "relu" else names[id(act)]
            if act != "relu":
                assert bool((act.weight > 0).all()), key
            masks[key] = layers.K.positive(y).detach().cpu()      # (split-output tensors: from their planes)
        return y

    handles = []
    for n, m in model.named_modules():
        if isinstance(m, layers.PReLU):
            def hook(mod, inp, out, n=n):
                if names.get(id(mod)) is not None:
                    assert bool((mod.weight > 0).all()), n
                masks[n] = (out > 0).detach().cpu()
            handles.append(m.register_forward_hook(hook))
    handles.append(model.register_forward_hook(lambda mod, inp, out: masks.__setitem__("pred", out.detach().cpu())))
    avse1.bn_act = spy
    try:
        yield masks
    finally:
        avse1.bn_act = orig
        for h in handles:
            h.remove()
        # the TCN runs time-major: its activations are (B, C, T, 1) channels-last views, and relu1 / relu2 are applied
        # (fused with the BatchNorm) BEFORE the symmetric chomp — bring those masks to the oracle's (B, C, T) sites
        for key in list(masks):
            m = masks[key]
            if ".tcn." in key and m.dim() == 4 and m.shape[3] == 1:
                m = m.squeeze(3)
                if key.endswith(".relu1") or key.endswith(".relu2"):
                    h = model.get_submodule(key.rsplit(".", 1)[0]).pad // 2
                    m = m[:, :, h:m.shape[2] - h]
                masks[key] = m.contiguous()


def impose_masks(ref, masks, flips):
    """Make the oracle AVNet ``ref`` (oracle/avse1_ref.py) use ``masks`` at every activation; ``flips[key]`` collects
    (number of sign disagreements with the oracle's own pre-activation, max |z| among them, max |z|).  Returns a
    callable that removes the hooks."""
    handles = []

    def where(key, z, neg):
        m = masks[key].to(z.device)
        assert m.shape == z.shape, (key, tuple(m.shape), tuple(z.shape))
        d = (z > 0) != m
        zmax = float(z.detach().abs().max())
        flips[key] = (int(d.sum()), float(z.detach().abs()[d].max()) if bool(d.any()) else 0.0, zmax)
        return torch.where(m, z, neg)

    for n, mod in ref.named_modules():
        if isinstance(mod, torch.nn.PReLU) and n in masks:
            def hook(m_, inp, out, n=n):
                z = inp[0]
                w = m_.weight.view([1, -1] + [1] * (z.dim() - 2)) if m_.weight.numel() > 1 else m_.weight
                return where(n, z, w * z)
            handles.append(mod.register_forward_hook(hook))
    af = ref.net_audiofeat
    orig_fwd = af.forward

    def af_forward(x):                           # oracle AudioFeatNet.forward with the ReLUs on our masks
        T = x.shape[2]
        x = af.bn0(x)
        for i in range(af.num_conv):
            z = getattr(af, f"bn{i + 1}")(getattr(af, f"conv{i + 1}")(x))
            x = where(f"net_audiofeat.bn{i + 1}", z, torch.zeros_like(z))
        z = af.bn_last(af.convf(x))
        x = where("net_audiofeat.bn_last", z, torch.zeros_like(z))
        return x.permute(0, 2, 1, 3).reshape(-1, T, af.embed_size * af.last_filter)

    af.forward = af_forward

    def remove():
        af.forward = orig_fwd
        for h in handles:
            h.remove()
    return remove


def masked_l1(pred, target, pred_ours):
    """F.l1_loss(pred, target) with the sign pattern of OUR prediction (equal in value where the signs agree)."""
    s = torch.sign(pred_ours.to(pred.device, pred.dtype) - target)
    return (s * (pred - target)).mean()


def check_flips(flips):
    """Every sign disagreement between our run and fp64 must sit at a rounding-level pre-activation."""
    n = 0
    for key, (cnt, zflip, zmax) in flips.items():
        assert zflip <= Z_TIE * zmax, (key, cnt, zflip, zmax)
        n += cnt
    return n
