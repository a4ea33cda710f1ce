"""CPU tests of host-side logic of the product package (no GPU kernels called)."""
import pytest
import torch
import torch.nn.functional as F


@pytest.mark.parametrize("n_in,K", [(125, 3999), (13, 399), (25, 799), (3, 100), (4, 140), (5, 150)])
def test_avse4_upsample_matrix_matches_interpolate_and_pad(n_in, K):
    """avse4 visual upsampling (model.py:166-168: linear x32, align_corners=False, then pad/crop to K)
    is run as one GEMM with a fixed interpolation matrix."""
    from avse_challenge_amd.avse4 import _upsample_matrix
    v = torch.randn(2, 7, n_in, dtype=torch.float64)
    ref = F.pad(F.interpolate(v, 32 * n_in, mode="linear"), (0, K - 32 * n_in))
    got = v @ _upsample_matrix(n_in, 32, K, v.device).double()
    assert torch.allclose(got, ref, atol=1e-12, rtol=0)


@pytest.mark.parametrize("L,K", [(3999, 250), (499, 250), (250, 250), (7, 4)])
def test_dpmamba_segmentation_overlap_add(L, K):
    """Dual-path chunking (50 % overlap, zero padding) and its overlap-add: every frame lands in exactly two
    chunks, so over_add(segment(x)) == 2 x; the chunk tensor equals the oracle's speechbrain restatement."""
    from avse_challenge_amd.dpmamba import DualPathModel
    from oracle.dpmamba_ref import Dual_Path_Model
    x = torch.randn(2, 3, L, dtype=torch.float64)
    seg, gap = DualPathModel._segmentation(x, K)
    ref_mod = Dual_Path_Model.__new__(Dual_Path_Model)
    seg_r, gap_r = ref_mod._Segmentation(x, K)
    assert gap == gap_r and torch.equal(seg, seg_r)
    assert torch.allclose(DualPathModel._over_add(seg, gap), 2 * x, atol=0, rtol=0)


def test_dpmamba_state_dict_keys_match_oracle():
    from avse_challenge_amd.dpmamba import DPMAMBA_SIZES, DPMambaTasNet
    from oracle.dpmamba_ref import DPMambaTasNet as Ref
    for kw in ({"N": 64, "n_dp": 2}, {**DPMAMBA_SIZES["XS"], "n_dp": 1}):
        a = {k: tuple(v.shape) for k, v in DPMambaTasNet(**kw).state_dict().items()}
        b = {k: tuple(v.shape) for k, v in Ref(**kw).state_dict().items()}
        assert a == b


@pytest.mark.parametrize("tv,L", [(5, 499), (75, 5999), (7, 7), (3, 10)])
def test_avmamba_visual_upsampling_matrix_equals_interpolate(tv, L):
    """C5 visual upsampling: the fixed (T_v, L) GEMM matrix == F.interpolate(linear) by ceil(L/T_v) + crop/pad,
    the form the oracle assembly uses (oracle/avmamba_ref.py)."""
    import math
    import torch.nn.functional as F
    from avse_challenge_amd import avse4
    up = max(1, math.ceil(L / tv))
    v = torch.randn(2, 3, tv, dtype=torch.float64)
    ref = F.pad(F.interpolate(v, scale_factor=up, mode="linear", align_corners=False), (0, L - up * tv))
    m = avse4._upsample_matrix(tv, up, L, "cpu").double()
    torch.testing.assert_close(v @ m, ref, atol=1e-6, rtol=0)


def test_avmamba_oracle_assembly_shapes_and_keys():
    from oracle import avmamba_ref
    m = avmamba_ref.AVMambaTasNet(N=32, n_mamba=1)
    with torch.no_grad():
        y = m(0.1 * torch.randn(1, 800), torch.rand(1, 1, 2, 112, 112))
    assert y.shape == (1, 800)
    from avse_challenge_amd import avmamba
    assert list(dict(avmamba.AVMambaTasNet(N=32, n_mamba=1).named_parameters())) == \
        list(dict(m.named_parameters()))


@pytest.mark.parametrize("k,stride,hw,cl", [(3, 1, 3, False), (3, 2, 6, False), (3, 1, 6, False), (3, 2, 12, False),
                                           (1, 2, 12, False), (1, 2, 7, False), (3, 2, 7, False), (1, 2, 12, True),
                                           (1, 1, 6, True)])
def test_gemm_conv_matches_conv2d_fp64(k, stride, hw, cl):
    """layers._GemmConvFn (the lip-trunk small-frame convs and 1x1 shortcuts as one im2col GEMM, col2im backward) equals
    F.conv2d(padding (k-1)/2, stride, bias=False) in fp64: output and input / weight gradients (pure torch ops, so the
    host runs the same arithmetic the GPU path launches as hipBLASLt GEMMs)."""
    import torch.nn.functional as F
    from avse_challenge_amd.layers import _GemmConvFn
    g = torch.Generator().manual_seed(k * 100 + stride * 10 + hw)
    x = torch.randn(5, 8, hw, hw, generator=g, dtype=torch.float64)
    if cl:                                            # the channels-last lip trunk (bench layout)
        x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    w = torch.randn(6, 8, k, k, generator=g, dtype=torch.float64, requires_grad=True)
    y = _GemmConvFn.apply(x, w, stride)
    yr = F.conv2d(x, w, None, stride, (k - 1) // 2)
    assert y.shape == yr.shape and (not cl or y.is_contiguous(memory_format=torch.channels_last))
    torch.testing.assert_close(y, yr, rtol=1e-12, atol=1e-12)
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    dx, dw = torch.autograd.grad(y, (x, w), gy)
    dxr, dwr = torch.autograd.grad(yr, (x, w), gy)
    torch.testing.assert_close(dx, dxr, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(dw, dwr, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("add_bias", [True, False])
def test_conv1_gemm_matches_conv2d_fp64(add_bias):
    """layers._Conv1Fn (AudioFeatNet.conv1, Conv2d(1, 64, 5, padding=2), model.py:199-215, as im2col GEMMs with the bias
    as a ones column and a 25-plane col2im backward) equals F.conv2d in fp64: output (channels-last memory), input /
    weight / bias gradients.  add_bias=False leaves the bias out of the output (BatchNorm-folded) but returns db."""
    import torch.nn.functional as F
    from avse_challenge_amd.layers import _Conv1Fn
    g = torch.Generator().manual_seed(11 + add_bias)
    x = torch.randn(3, 1, 11, 17, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(8, 1, 5, 5, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(8, generator=g, dtype=torch.float64, requires_grad=True)
    y = _Conv1Fn.apply(x, w, b, add_bias)
    yr = F.conv2d(x, w, b if add_bias else None, padding=2)
    assert y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y, yr, rtol=1e-12, atol=1e-12)
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    got = torch.autograd.grad(y, (x, w, b), gy)
    xr, wr, br = (t.detach().requires_grad_(True) for t in (x, w, b))
    ref = torch.autograd.grad(F.conv2d(xr, wr, br, padding=2), (xr, wr, br), gy)
    for a_, r_ in zip(got, ref):
        torch.testing.assert_close(a_, r_, rtol=1e-12, atol=1e-12)


def test_time_conv1d_matches_conv1d_fp64():
    """layers._TimeConv1dFn (the avse1 TCN conv: im2col GEMM on time-major activations) == nn.Conv1d with padding
    (k-1)*dil (utils/tcn.py:163-166) in fp64: output and the input / weight / bias gradients, dilations 1..8."""
    import torch.nn as nn
    from avse_challenge_amd.layers import time_conv1d
    torch.manual_seed(0)
    for dil in (1, 2, 4, 8):
        conv = nn.Conv1d(12, 10, 3, padding=2 * dil, dilation=dil).double()
        x = torch.randn(2, 12, 19, dtype=torch.float64, requires_grad=True)
        y_ref = conv(x)                                           # (B, C', T + pad)
        g = torch.randn_like(y_ref)
        gx_ref, gw_ref, gb_ref = torch.autograd.grad((y_ref * g).sum(), (x, conv.weight, conv.bias))
        xt = x.detach().transpose(1, 2).contiguous().requires_grad_(True)     # (B, T, C) time-major
        y = time_conv1d(xt, conv)
        assert y.shape == (2, 19 + 2 * dil, 10)
        assert torch.allclose(y.transpose(1, 2), y_ref, atol=1e-12)
        gx, gw, gb = torch.autograd.grad((y * g.transpose(1, 2)).sum(), (xt, conv.weight, conv.bias))
        assert torch.allclose(gx.transpose(1, 2), gx_ref, atol=1e-12)
        assert torch.allclose(gw, gw_ref, atol=1e-12) and torch.allclose(gb, gb_ref, atol=1e-12)


def test_time_major_tcn_chomp_matches_reference_order():
    """The avse1 TCN's time-major half-block order — BatchNorm statistics over the whole (T + pad) conv output, the
    elementwise PReLU before the symmetric chomp — equals the reference's conv -> BN -> chomp -> PReLU (fp64, torch
    ops standing in for the bnact kernel)."""
    import torch.nn as nn
    import torch.nn.functional as F
    torch.manual_seed(1)
    dil, C, T = 2, 8, 15
    conv = nn.Conv1d(C, C, 3, padding=2 * dil, dilation=dil).double()
    bn = nn.BatchNorm1d(C).double().train()
    a = torch.full((C,), 0.25, dtype=torch.float64)
    x = torch.randn(2, C, T, dtype=torch.float64)
    ref = F.prelu(bn(conv(x))[:, :, dil:T + 2 * dil - dil], a)          # reference: chomp then PReLU
    from avse_challenge_amd.layers import time_conv1d
    y = time_conv1d(x.transpose(1, 2).contiguous(), conv)                # (B, T + pad, C)
    bn2 = nn.BatchNorm1d(C).double().train()
    z = F.prelu(bn2(y.transpose(1, 2)), a)[:, :, dil:y.shape[1] - dil]   # ours: BN + PReLU, then chomp
    assert torch.allclose(z, ref, atol=1e-12)
