"""avse4 train-step gradient parity against the fp64 oracle with OUR run's activation masks imposed (test helper).

The avse4 counterpart of tests/avse1_parity.py: a ReLU / PReLU whose input sits within fp32 rounding of 0 takes one
branch in an fp32 run and possibly the other in fp64, and the BatchNorm / gLN backward of that site turns the flip
into a gradient change far above fp32 rounding (the reason test_avse4_full_train_step_vs_oracle needs 1e-2 .. 1e-1
floors: profiles/r02c_avse4_grad_diag.txt).  Here every activation of baseline/avse4/model.py:52-118 (TCN PReLUs,
visual-conv ReLU / PReLU, encoder and mask ReLUs) and utils.py:40-118 (front-end and ResNet ReLUs) in the fp64
oracle follows the sign pattern our fp32 GPU step took, and each disagreement with fp64's own sign must sit at a
rounding-level pre-activation.  What remains between the two runs is fp32 arithmetic error only.

Sites (keys = module names shared by both trees):
  * bn_act(..., "relu") sites: the BatchNorm's name (visual_frontend.frontend3D.1, ...resnet.layerX.{bn1a,outbna,
    bn1b,outbnb}); in the oracle the frontend's nn.ReLU and the ResNetLayer's functional relus;
  * PReLU sites: the nn.PReLU module's name (TemporalBlock net.1 before gLN, DepthwiseSeparableConv net.1 after the
    depthwise conv, VisualConv1D net.3): ours inside the fused prelu_gln / dwconv_prelu_gln kernels or _PReLUFn;
  * VisualConv1D net.0 (ReLU of the block input), model.encoder (relu of the encoder conv), model.separator.mask
    (relu of mask_conv1x1).
"""
import contextlib

import torch
import torch.nn as nn
import torch.nn.functional as F

from avse_challenge_amd import avse4, layers

Z_TIE = 1e-4      # a flip is legitimate only where |z64| <= Z_TIE * max|z64| of its site (fp32 rounding: ~1e-6)


@contextlib.contextmanager
def capture_masks(model):
    """While active, every forward of the avse_challenge_amd AVSE4BaselineModule ``model`` records CPU bool masks
    (pre-activation > 0) keyed by the oracle's site names (module docstring)."""
    masks = {}
    names = {id(m): n for n, m in model.named_modules()}
    pnames = {id(p): n[:-len(".weight")] for n, p in model.named_parameters()}
    orig = (avse4.bn_act, avse4.prelu_gln, avse4.dwconv_prelu_gln, avse4._PReLUFn)

    def bn_spy(x, bn, act=None, res=None, folded_bias=None, **kw):
        y = orig[0](x, bn, act, res, folded_bias=folded_bias, **kw)
        if act == "relu":
            masks[names[id(bn)]] = layers.K.positive(y).detach().cpu()    # (split-output tensors: from their planes)
        return y

    def pg_spy(x, alpha, gamma, beta, eps=1e-8, **kw):
        masks[pnames[id(alpha)]] = (x > 0).detach().cpu()
        return orig[1](x, alpha, gamma, beta, eps, **kw)

    def dpg_spy(x, w, alpha, gamma, beta, dilation, eps=1e-8, **kw):
        y = orig[2](x, w, alpha, gamma, beta, dilation, eps, **kw)
        masks[pnames[id(alpha)]] = (y.grad_fn.saved_tensors[2] > 0).detach().cpu()     # y1 = dwconv(x)
        return y

    class PReLUSpy:
        @staticmethod
        def apply(y, a):
            masks[pnames[id(a)]] = (y > 0).detach().cpu()
            return orig[3].apply(y, a)

    handles = [model.model.encoder.register_forward_hook(
        lambda mod, inp, out: masks.__setitem__("model.encoder", (out > 0).detach().cpu()))]
    sep = model.model.separator
    handles.append(sep.register_forward_hook(lambda mod, inp, out: masks.__setitem__(
        "model.separator.mask", (out.reshape(out.shape[0], -1, out.shape[-1]) > 0).detach().cpu())))
    for n, m in model.named_modules():
        if isinstance(m, avse4.VisualConv1D):
            handles.append(m.register_forward_pre_hook(
                lambda mod, inp, n=n: masks.__setitem__(n + ".net.0", (inp[0] > 0).detach().cpu())))
    avse4.bn_act, avse4.prelu_gln, avse4.dwconv_prelu_gln, avse4._PReLUFn = bn_spy, pg_spy, dpg_spy, PReLUSpy
    try:
        yield masks
    finally:
        avse4.bn_act, avse4.prelu_gln, avse4.dwconv_prelu_gln, avse4._PReLUFn = orig
        for h in handles:
            h.remove()


def impose_masks(ref, masks, flips):
    """Make the oracle AVSE4BaselineModule ``ref`` (oracle/avse4_ref.py) use ``masks`` at every activation;
    ``flips[key]`` collects (sign disagreements with the oracle's own pre-activation, max |z| among them, max |z|).
    Returns a callable that removes the hooks and the patched forwards."""
    from oracle import avse4_ref
    handles, patched = [], []

    def where(key, z, neg):
        m = masks[key].to(z.device)
        assert m.shape == z.shape, (key, tuple(m.shape), tuple(z.shape))
        d = (z > 0) != m
        zmax = float(z.detach().abs().max())
        flips[key] = (int(d.sum()), float(z.detach().abs()[d].max()) if bool(d.any()) else 0.0, zmax)
        return torch.where(m, z, neg)

    def relu_at(key, z):
        return where(key, z, torch.zeros_like(z))

    for n, mod in ref.named_modules():
        if isinstance(mod, nn.PReLU) and n in masks:
            def hook(m_, inp, out, n=n):
                z = inp[0]
                w = m_.weight.view([1, -1] + [1] * (z.dim() - 2)) if m_.weight.numel() > 1 else m_.weight
                return where(n, z, w * z)
            handles.append(mod.register_forward_hook(hook))
        elif isinstance(mod, nn.ReLU):
            key = n if n in masks else n[:-2] + ".1"          # frontend3D.2 -> its BatchNorm frontend3D.1
            handles.append(mod.register_forward_hook(lambda m_, inp, out, key=key: relu_at(key, inp[0])))
        elif isinstance(mod, avse4_ref.ResNetLayer):
            def fwd(x, L=mod, n=n):
                y = L.conv2a(relu_at(n + ".bn1a", L.bn1a(L.conv1a(x))))
                y = y + (x if L.stride == 1 else L.downsample(x))
                mid = y
                y = relu_at(n + ".outbna", L.outbna(y))
                y = L.conv2b(relu_at(n + ".bn1b", L.bn1b(L.conv1b(y)))) + mid
                return relu_at(n + ".outbnb", L.outbnb(y))
            patched.append(mod)
            mod.forward = fwd
    enc = ref.model.encoder
    enc.forward = lambda m: relu_at("model.encoder", enc.conv1d_U(m))
    patched.append(enc)
    tcn = ref.model.separator

    def tcn_forward(x, visual):
        visual = tcn.visual_conv(visual.transpose(1, 2))
        x = tcn.bottleneck_conv1x1(tcn.layer_norm(x))
        bsz, Bc, K = x.shape
        for i in range(len(tcn.tcn)):
            v = tcn.ve_conv1x1[i](visual)
            v = F.interpolate(v, tcn.up * v.shape[-1], mode="linear")
            v = F.pad(v, (0, K - v.shape[-1]))
            x = tcn.tcn[i](torch.cat((x, v), 1))
        x = relu_at("model.separator.mask", tcn.mask_conv1x1(x))
        return x.reshape(bsz, tcn.num_channels, Bc, K)

    tcn.forward = tcn_forward
    patched.append(tcn)

    def remove():
        for m in patched:
            del m.forward                                     # back to the class's forward
        for h in handles:
            h.remove()
    return remove


def check_flips(flips):
    """Every sign disagreement between our run and fp64 must sit at a rounding-level pre-activation; returns the
    number of disagreements."""
    n = 0
    for key, (cnt, zflip, zmax) in flips.items():
        assert zflip <= Z_TIE * zmax, (key, cnt, zflip, zmax)
        n += cnt
    return n
