"""bf16 projection GEMM (csrc/projgemm.hip, kernels.gemm_bf16) vs an fp64 matmul of the same bf16 operands.

The op is the bf16 F.linear of the Mamba projections under autocast (Mamba-TasNet/modules/mamba/bimamba.py:190-196,
250-253): fp32 accumulation, one round to bf16 at the end.  Bar per element: |out - ref| <= 2^-8 |ref| (half a bf16
ulp, the final rounding) + 1e-5 * sum_k |P Q| (fp32 accumulation in another order).  Outputs outside the logical
shape (the padded time columns of the model's layout) must stay untouched.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def K():
    from avse_challenge_amd import kernels
    return kernels


def _operand(b, rows, k, kc, g, shared=False):
    """A (b or 1, rows, k) bf16 view that is K-contiguous (kc) or contiguous along rows, with padded strides."""
    nb = 1 if shared else b
    if kc:
        base = torch.randn(nb, rows, k + 8, device=DEV, generator=g).to(torch.bfloat16)
        return base[:, :, :k]
    base = torch.randn(nb, k, -(-rows // 8) * 8 + 16, device=DEV, generator=g).to(torch.bfloat16)
    return base[:, :, :rows].transpose(1, 2)


def _check(out, P, Q, alpha, mp):
    ref = alpha * torch.matmul(Q.double(), P.double().transpose(1, 2))              # (b, mq, mp)
    mag = torch.matmul(Q.double().abs(), P.double().abs().transpose(1, 2)) * abs(alpha)
    got = out[..., :mp].double()
    bad = (got - ref).abs() > 2.0 ** -8 * ref.abs() + 1e-5 * mag
    assert not bool(bad.any()), (int(bad.sum()), float((got - ref).abs().max()))


@pytest.mark.parametrize("p_kc", [True, False])
@pytest.mark.parametrize("q_kc", [True, False])
@pytest.mark.parametrize("shared", ["p", "q", None])
def test_gemm_bf16_layouts_ragged(p_kc, q_kc, shared):
    g = torch.Generator(device=DEV).manual_seed(7 + 2 * p_kc + q_kc)
    b, mp, mq, k = 3, 300, 200, 192
    P = _operand(b, mp, k, p_kc, g, shared == "p")
    Q = _operand(b, mq, k, q_kc, g, shared == "q")
    out = torch.full((b, mq, mp + 20), float("nan"), device=DEV, dtype=torch.bfloat16)[..., :mp]
    assert K().gemm_bf16_supported(P, Q, out)
    K().gemm_bf16(P, Q, out, 0.5)
    _check(out, P, Q, 0.5, mp)
    pad = torch.as_strided(out, (b, mq, 20), out.stride(), out.storage_offset() + mp)
    assert bool(torch.isnan(pad.float()).all()), "the GEMM wrote outside the logical output"


@pytest.mark.parametrize("mp,mq,k", [(1, 1, 64), (129, 127, 64), (4, 640, 1024), (640, 4, 2048)])
def test_gemm_bf16_edge_shapes(mp, mq, k):
    g = torch.Generator(device=DEV).manual_seed(mp * 31 + mq)
    P = _operand(2, mp, k, True, g)
    Q = _operand(2, mq, k, False, g, shared=True)
    out = torch.empty((2, mq, mp + (-mp) % 4), device=DEV, dtype=torch.bfloat16)[..., :mp]
    K().gemm_bf16(P, Q, out)
    _check(out, P, Q, 1.0, mp)


def test_gemm_bf16_mamba_layouts_c5_rows():
    """The four C5 projections as mamba_tasnet lays them out (B = 2, L = 999 with the 128-B padded time stride)."""
    k = K()
    g = torch.Generator(device=DEV).manual_seed(3)
    b, L, dm, di, bf = 2, 999, 512, 1024, torch.bfloat16
    rnd = lambda *s: torch.randn(*s, device=DEV, generator=g).to(bf)  # noqa: E731
    w_in, w_out = rnd(2 * di, dm), rnd(dm, di)
    h, dout = rnd(b, L, dm), rnd(b, L, dm)
    y = k.bdl_empty(b, di, L, bf, DEV).copy_(torch.randn(b, di, L, device=DEV, generator=g))
    dxz = k.bdl_empty(b, 2 * di, L, bf, DEV).copy_(torch.randn(b, 2 * di, L, device=DEV, generator=g))
    xz = k.bdl_empty(b, 2 * di, L, bf, DEV)
    _check(k.gemm_bf16(h, w_in[None], xz), h, w_in[None], 1.0, L)                                # in_proj
    o = torch.empty(b, L, dm, device=DEV, dtype=bf)
    _check(k.gemm_bf16(w_out[None], y.transpose(1, 2), o, 0.5), w_out[None], y.transpose(1, 2), 0.5, dm)
    dh = torch.empty(b, L, dm, device=DEV, dtype=bf)
    _check(k.gemm_bf16(w_in.t()[None], dxz.transpose(1, 2), dh), w_in.t()[None], dxz.transpose(1, 2), 1.0, dm)
    dy = k.bdl_empty(b, di, L, bf, DEV)
    _check(k.gemm_bf16(dout, w_out.t()[None], dy, 0.5), dout, w_out.t()[None], 0.5, L)


def _nan_padded_bdl(b, d, L, g):
    """A (b, d, L) bf16 tensor in the model's padded layout whose pad columns hold NaN."""
    t = K().bdl_empty(b, d, L, torch.bfloat16, DEV)
    full = torch.as_strided(t, (b, d, t.stride(1)), t.stride(), t.storage_offset())
    full.fill_(float("nan"))
    return t.copy_(torch.randn(b, d, L, device=DEV, generator=g))


@pytest.mark.parametrize("L", [999, 64, 37])
def test_gemm_bf16_weight_grads_fold_fp32(L):
    """dW_in = sum_{b,l} dxz[b, :, l] h[b, l, :] and dW_out = 0.5 sum_{b,l} dout[b, l, :] y[b, :, l] (bimamba.py:190-196,
    250-253 backward): fp32 out, all batches folded into one output, k = L not a multiple of the stage (the pad
    columns past L hold NaN and must not reach the sums)."""
    k = K()
    g = torch.Generator(device=DEV).manual_seed(L)
    b, dm, di = 3, 512, 1024
    h = torch.randn(b, L, dm, device=DEV, generator=g).to(torch.bfloat16)
    dout = torch.randn(b, L, dm, device=DEV, generator=g).to(torch.bfloat16)
    dxz, y = _nan_padded_bdl(b, 2 * di, L, g), _nan_padded_bdl(b, di, L, g)
    dw_in = torch.empty(1, 2 * di, dm, device=DEV, dtype=torch.float32)
    k.gemm_bf16(h.transpose(1, 2), dxz, dw_in, 1.0, fold=b)
    ref = torch.einsum("bnl,blc->nc", dxz.double(), h.double())
    mag = torch.einsum("bnl,blc->nc", dxz.double().abs(), h.double().abs())
    assert bool(((dw_in[0].double() - ref).abs() <= 1e-5 * mag).all())
    dw_out = torch.empty(1, dm, di, device=DEV, dtype=torch.float32)
    k.gemm_bf16(y, dout.transpose(1, 2), dw_out, 0.5, fold=b)
    ref = 0.5 * torch.einsum("blm,bdl->md", dout.double(), y.double())
    mag = 0.5 * torch.einsum("blm,bdl->md", dout.double().abs(), y.double().abs())
    assert bool(((dw_out[0].double() - ref).abs() <= 1e-5 * mag).all())


def test_gemm_bf16_rejects_unsupported():
    k = K()
    a = torch.randn(2, 64, 128, device=DEV).to(torch.bfloat16)[:, :, ::2]      # neither the row nor the k stride is 1
    out = torch.empty(2, 64, 64, device=DEV, dtype=torch.bfloat16)
    assert not k.gemm_bf16_supported(a, a, out)
    with pytest.raises(RuntimeError):
        k.gemm_bf16(a, a, out)


# ------------------------------------------------------------------ fp32 GEMM on split fp16 planes (avse_gemm_f32s)

def _operand32(b, rows, k, kc, g, shared=False, spread=False):
    """A (b or 1, rows, k) fp32 view, K-contiguous (kc) or contiguous along rows, with padded strides (NaN in the pads:
    the split writes nothing there and the GEMM must not sum them); spread: magnitudes over ~7 decades."""
    nb = 1 if shared else b
    if kc:
        base = torch.full((nb, rows, k + 8), float("nan"), device=DEV)
        v = base[:, :, :k]
    else:
        base = torch.full((nb, k, -(-rows // 8) * 8 + 16), float("nan"), device=DEV)
        v = base[:, :, :rows].transpose(1, 2)
    x = torch.randn(v.shape, device=DEV, generator=g)
    if spread:
        x = x * torch.exp(4.0 * torch.randn(v.shape, device=DEV, generator=g))
    v.copy_(x)
    return v


def _check32(out, P, Q, alpha, mp, fold=1):
    prod = torch.matmul(Q.double(), P.double().transpose(1, 2))
    mag = torch.matmul(Q.double().abs(), P.double().abs().transpose(1, 2))
    if fold > 1:
        prod = prod.reshape(-1, fold, *prod.shape[1:]).sum(1)
        mag = mag.reshape(-1, fold, *mag.shape[1:]).sum(1)
    ref, mag = alpha * prod, abs(alpha) * mag
    err = ((out[..., :mp].double() - ref).abs() / (mag + 1e-300)).max()
    return float(err)


@pytest.mark.parametrize("p_kc", [True, False])
@pytest.mark.parametrize("q_kc", [True, False])
@pytest.mark.parametrize("shared", ["p", "q", None])
def test_gemm_f32s_layouts_ragged_vs_fp64(p_kc, q_kc, shared):
    """avse_gemm_f32s (fp32 GEMM as P_hi Q_hi + P_hi Q_lo + P_lo Q_hi on the f16 MFMA) vs fp64: every element within 1e-5
    of its sum_k |P Q| (22-bit operands; fp32 accumulation: the fp32 class), with operands spread over ~7 decades, ragged sizes, a K
    tail, NaN in every padding column, and nothing written outside the logical output; compared with hipBLASLt's fp32
    error on the same operands for the record."""
    g = torch.Generator(device=DEV).manual_seed(70 + 2 * p_kc + q_kc)
    b, mp, mq, k = 3, 300, 200, 200
    P = _operand32(b, mp, k, p_kc, g, shared == "p", spread=True)
    Q = _operand32(b, mq, k, q_kc, g, shared == "q")
    out = torch.full((b, mq, mp + 20), float("nan"), device=DEV)[..., :mp]
    assert K().gemm_f32s_supported(P, Q, out)
    K().gemm_f32s(P, Q, out, 0.5)
    err = _check32(out, P, Q, 0.5, mp)
    lib = 0.5 * torch.matmul(Q.expand(b, -1, -1), P.expand(b, -1, -1).transpose(1, 2))
    print(f"gemm_f32s err {err:.2e} of sum|PQ| (hipBLASLt fp32 {_check32(lib, P, Q, 1.0, mp):.2e})")
    assert err <= 1e-5, err
    pad = torch.as_strided(out, (b, mq, 20), out.stride(), out.storage_offset() + mp)
    assert bool(torch.isnan(pad).all()), "the GEMM wrote outside the logical output"


@pytest.mark.parametrize("mp,mq,k,fold", [(1, 1, 64, 1), (129, 127, 64, 1), (4, 640, 1024, 1), (640, 4, 2048, 1),
                                           (512, 300, 1000, 3), (1024, 512, 640, 2)])
def test_gemm_f32s_edge_shapes_and_fold(mp, mq, k, fold):
    """Single elements, tile remainders, long K, and the folded weight-gradient form (groups of batches summed)."""
    g = torch.Generator(device=DEV).manual_seed(mp * 37 + mq + fold)
    b = 2 * fold
    P = _operand32(b, mp, k, True, g)
    Q = _operand32(b, mq, k, False, g)
    out = torch.empty((b // fold, mq, mp + (-mp) % 4), device=DEV)[..., :mp]
    K().gemm_f32s(P, Q, out, fold=fold)
    assert _check32(out, P, Q, 1.0, mp, fold) <= 1e-5


def test_gemm_f32s_c3_layouts_vs_fp64():
    """The four Mamba-TasNet-L fp32 projection layouts at reduced batch (in_proj fwd and input gradient, out_proj fwd,
    weight gradient with fold), each within 1e-5 of sum |PQ| of the fp64 product."""
    g = torch.Generator(device=DEV).manual_seed(99)
    b, l, dm, di = 2, 600, 512, 1024
    h = torch.randn(b, l, dm, device=DEV, generator=g)                   # (b, l, d_model)
    w_in = 0.05 * torch.randn(2 * di, dm, device=DEV, generator=g)
    xz = torch.empty(b, 2 * di, l + 8, device=DEV)[..., :l]
    K().gemm_f32s(h, w_in[None], xz)                                     # xz = W_in h^T  (P = h, p = l)
    assert _check32(xz, h, w_in[None], 1.0, l) <= 1e-5
    dxz = torch.randn(b, 2 * di, l, device=DEV, generator=g)
    dh = torch.empty(b, l, dm, device=DEV)
    K().gemm_f32s(w_in.t()[None], dxz.transpose(1, 2), dh)               # dh = dxz^T W_in
    assert _check32(dh, w_in.t()[None], dxz.transpose(1, 2), 1.0, dm) <= 1e-5
    y = torch.randn(b, di, l, device=DEV, generator=g)
    w_out = 0.05 * torch.randn(dm, di, device=DEV, generator=g)
    o = torch.empty(b, l, dm, device=DEV)
    K().gemm_f32s(w_out[None], y.transpose(1, 2), o, 0.5)                 # out = 0.5 y^T W_out^T
    assert _check32(o, w_out[None], y.transpose(1, 2), 0.5, dm) <= 1e-5
    dw = torch.empty(1, 2 * di, dm, device=DEV)
    K().gemm_f32s(h.transpose(1, 2), dxz, dw, fold=b)                    # dW_in = sum_b dxz h
    assert _check32(dw, h.transpose(1, 2), dxz, 1.0, dm, b) <= 1e-5


@pytest.mark.parametrize("b,c,l", [(2, 64, 3999), (3, 40, 17), (1, 8, 4)])
def test_add_max_padded_rows(b, c, l):
    """avse_add_max (the C3 out_proj input, bimamba.py:253): the sum over the padded storage equals a + b on the logical
    columns, and its max is max |a + b| over them exactly, whatever the pad columns hold (NaN here); split_planes then
    takes that max (no absmax pass) and yields the same planes as from a copy."""
    from avse_challenge_amd import kernels as K
    g = torch.Generator(device="cuda").manual_seed(b * c + l)
    a = K.bdl_empty(b, c, l, torch.float32, torch.device("cuda"))
    bb = K.bdl_empty(b, c, l, torch.float32, torch.device("cuda"))
    lp = a.stride(1)
    fa = a.as_strided((b, c, lp), a.stride())
    fb = bb.as_strided((b, c, lp), bb.stride())
    fa.fill_(float("nan"))
    fb.fill_(float("nan"))
    a.copy_(torch.randn(b, c, l, device="cuda", generator=g))
    bb.copy_(3 * torch.randn(b, c, l, device="cuda", generator=g))
    y = K.add_max(fa, fb, l)
    assert y.shape == (b, c, l) and torch.equal(y, a + bb)
    mb = getattr(y, K.ABSMAX_ATTR)
    assert int(mb.item()) == int((a + bb).abs().max().view(torch.int32).item())
    s1, s2 = K.split_planes(y), K.split_planes(y.clone())
    assert torch.equal(s1.hi, s2.hi) and torch.equal(s1.lo, s2.lo) and torch.equal(s1.mb, s2.mb)


@pytest.mark.parametrize("b,c,k", [(2, 24, 3999), (3, 16, 17), (1, 8, 5)])
def test_split_rows8_planes(b, c, k):
    """avse_split16_planes_to: the padded-row planes of a (b, c, k) tensor (rows k not 16-B aligned) decode to x within
    2^-22 of max |x|, equal split_planes' planes of the same tensor element for element, and share its max."""
    from avse_challenge_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(b * 1000 + k)
    x = torch.randn(b, c, k, device=DEV, generator=g) * torch.exp(2.0 * torch.randn(b, c, k, device=DEV, generator=g))
    s = K.split_rows8(x)
    assert s.hi.shape == x.shape and s.hi.stride(1) % 8 == 0 and s.hi.stride(2) == 1
    ref = K.split_planes(x)
    assert torch.equal(s.mb, ref.mb)
    assert torch.equal(s.hi, ref.hi) and torch.equal(s.lo, ref.lo)
    bits = int(s.mb.item())
    e = max(-100, min(100, 14 - (((bits >> 23) & 0xFF) - 127)))
    dec = (s.hi.double() + s.lo.double()) * 2.0 ** -e
    assert float((dec - x.double()).abs().max()) <= 2.0 ** -22 * float(x.abs().max())
    cp = s.hi.stride(1)
    if cp != k:                               # the padding columns are written as 0 (the time-chunked weight gradient)
        for pl in (s.hi, s.lo):
            pad = torch.as_strided(pl, (b, c, cp - k), pl.stride(), pl.storage_offset() + k)
            assert bool((pad == 0).all())


@pytest.mark.parametrize("k", [3999, 125, 64])
@pytest.mark.parametrize("chan_contig", [False, True])
def test_avse4_pointwise_conv_split_vs_fp64(k, chan_contig):
    """The avse4 1x1 Conv1d (baseline/avse4/model.py:255-293) on avse_gemm_f32s: forward, input gradient and weight
    gradient vs fp64 within 1e-5 of sum |x w| (the fp32 class), K = 3999 (rows not 16-B aligned: padded planes, per-element
    output rows), the visual K = 125, and a channel-contiguous input (the ChannelWiseLayerNorm output's layout)."""
    from avse_challenge_amd import avse4
    g = torch.Generator(device=DEV).manual_seed(k + 7 * chan_contig)
    b, cin, cout = 3, 256, 512
    if chan_contig:
        x = torch.randn(b, k, cin, device=DEV, generator=g).transpose(1, 2)
    else:
        x = torch.randn(b, cin, k, device=DEV, generator=g)
    x.requires_grad_(True)
    w = (0.05 * torch.randn(cout, cin, device=DEV, generator=g)).requires_grad_(True)
    assert avse4._pw_split_ok(w, x)
    y = avse4._PointwiseFn.apply(w, x)
    dy = torch.randn(b, cout, k, device=DEV, generator=g)
    y.backward(dy)
    xd, wd, dyd = x.detach().double(), w.detach().double(), dy.double()
    ref = torch.matmul(wd, xd)
    mag = torch.matmul(wd.abs(), xd.abs())
    assert float(((y.double() - ref).abs() / mag).max()) <= 1e-5
    dx_ref = torch.matmul(wd.t(), dyd)
    dx_mag = torch.matmul(wd.t().abs(), dyd.abs())
    assert float(((x.grad.double() - dx_ref).abs() / dx_mag).max()) <= 1e-5
    dw_ref = torch.matmul(dyd, xd.transpose(1, 2)).sum(0)
    dw_mag = torch.matmul(dyd.abs(), xd.abs().transpose(1, 2)).sum(0)
    assert float(((w.grad.double() - dw_ref).abs() / dw_mag).max()) <= 1e-5


@pytest.mark.parametrize("k,dil", [(3999, 128), (37, 1)])
def test_dwconv_gln_planes_output(k, dil):
    """avse_dwconv_gln_fwd_q: the gLN output written only as the planes of its consumer GEMM decodes to the fp32 path's y
    within 2^-21 of max |y|; the bound it scaled by is >= max |y| and within 0.1 % of it; y1 and the statistics equal
    the fp32 path's bit for bit."""
    from avse_challenge_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(k + dil)
    b, c = 2, 64
    x = torch.randn(b, c, k, device=DEV, generator=g)
    w = torch.randn(c, 1, 3, device=DEV, generator=g)
    alpha = torch.full((1,), 0.25, device=DEV)
    gamma = 1.0 + 0.5 * torch.randn(c, device=DEV, generator=g)
    beta = 0.1 * torch.randn(c, device=DEV, generator=g)
    y, y1, st = K.dwconv_gln_fwd(x, w, dil, alpha, gamma, beta)
    yq, y1q, stq = K.dwconv_gln_fwd(x, w, dil, alpha, gamma, beta, planes=True)
    assert torch.equal(y1, y1q) and torch.equal(st, stq)
    sp = K.planes_of(yq)
    assert sp is not None and sp.hi.shape == y.shape and sp.hi.stride(1) % 8 == 0
    bound = float(sp.mb.view(torch.float32).item())
    m = float(y.abs().max())
    assert m <= bound <= 1.001 * m, (m, bound)
    bits = int(sp.mb.item())
    e = max(-100, min(100, 14 - (((bits >> 23) & 0xFF) - 127)))
    dec = (sp.hi.double() + sp.lo.double()) * 2.0 ** -e
    assert float((dec - y.double()).abs().max()) <= 2.0 ** -21 * m
    cp = sp.hi.stride(1)
    if cp != k:
        for pl in (sp.hi, sp.lo):
            pad = torch.as_strided(pl, (b, c, cp - k), pl.stride(), pl.storage_offset() + k)
            assert bool((pad == 0).all())


@pytest.mark.parametrize("k", [3999, 37])
def test_prelu_gln_bwd_planes_output(k):
    """avse_prelu_gln_bwd_q: the PReLU -> gLN input gradient written only as the planes of the GEMM that produced x decodes
    to the fp32 path's dx within 2^-21 of max |dx|; its bound is >= max |dx| (and within 16x of it); the parameter
    gradients equal the fp32 path's bit for bit; the padding columns are 0."""
    from avse_challenge_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(k)
    b, c = 2, 64
    x = torch.randn(b, c, k, device=DEV, generator=g)
    alpha = torch.full((1,), 0.25, device=DEV)
    gamma = 1.0 + 0.5 * torch.randn(c, device=DEV, generator=g)
    beta = 0.1 * torch.randn(c, device=DEV, generator=g)
    _, st = K.prelu_gln_fwd(x, alpha, gamma, beta)
    dy = torch.randn(b, c, k, device=DEV, generator=g)
    dx, da, dg, db = K.prelu_gln_bwd(x, alpha, gamma, st, dy)
    dq, daq, dgq, dbq = K.prelu_gln_bwd(x, alpha, gamma, st, dy, planes=True)
    assert torch.equal(da, daq) and torch.equal(dg, dgq) and torch.equal(db, dbq)
    sp = K.planes_of(dq)
    assert sp is not None and sp.hi.shape == dx.shape
    m = float(dx.abs().max())
    bound = float(sp.mb.view(torch.float32).item())
    assert m <= bound <= 16 * m, (m, bound)
    bits = int(sp.mb.item())
    e = max(-100, min(100, 14 - (((bits >> 23) & 0xFF) - 127)))
    dec = (sp.hi.double() + sp.lo.double()) * 2.0 ** -e
    assert float((dec - dx.double()).abs().max()) <= 2.0 ** -21 * m
    cp = sp.hi.stride(1)
    if cp != k:
        for pl in (sp.hi, sp.lo):
            pad = torch.as_strided(pl, (b, c, cp - k), pl.stride(), pl.storage_offset() + k)
            assert bool((pad == 0).all())


def test_split_rows8_zeroes_pads_of_padded_rows():
    """split_rows8 of a view whose rows are already padded to the planes' row length (K = 3999 in rows of 4000, pad
    columns holding NaN): the planes' pad columns are still written as 0 (the time-chunked weight gradient sums them)."""
    from avse_challenge_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(5)
    base = torch.full((2, 16, 4000), float("nan"), device=DEV)
    x = base[..., :3999]
    x.copy_(torch.randn(2, 16, 3999, device=DEV, generator=g))
    s = K.split_rows8(x)
    assert s.hi.stride(1) == 4000
    for pl in (s.hi, s.lo):
        pad = torch.as_strided(pl, (2, 16, 1), pl.stride(), pl.storage_offset() + 3999)
        assert bool((pad == 0).all())
    ref = K.split_planes(x.contiguous())
    assert torch.equal(s.hi, ref.hi) and torch.equal(s.lo, ref.lo) and torch.equal(s.mb, ref.mb)


def test_add_max_flat_residual():
    """kernels.add_max_flat (the avse4 TemporalBlock residual): equals a + b, carries max |a + b| exactly, and a
    split of it (known max: no absmax pass) equals the split of a copy."""
    from avse_challenge_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(3)
    a = torch.randn(3, 256, 3999, device=DEV, generator=g)
    b = 2 * torch.randn(3, 256, 3999, device=DEV, generator=g)
    assert K.add_max_flat_ok(a, b)
    y = K.add_max_flat(a, b)
    assert torch.equal(y, a + b)
    assert int(getattr(y, K.ABSMAX_ATTR).item()) == int((a + b).abs().max().view(torch.int32).item())
    s1, s2 = K.split_rows8(y), K.split_rows8(y.clone())
    assert torch.equal(s1.hi, s2.hi) and torch.equal(s1.lo, s2.lo) and torch.equal(s1.mb, s2.mb)


# ------------------------------------------------------------------ row-chunked weight gradients (TCN / shortcuts)

@pytest.mark.parametrize("rows,units,ca,cb", [(2464, 32, 1536, 512), (2912, 32, 1536, 512), (30 * 144, 30, 64, 128),
                                              (77 * 5, 5, 40, 24)])
def test_gemm_f32s_rows_tn_vs_fp64(rows, units, ca, cb):
    """kernels.gemm_f32s_rows_tn: b^T a over ``rows`` rows cut into whole units (utterances / frames) that run as
    folded batches, at the avse1 TCN weight-gradient shapes (B To = 32 x 77 / 91 rows, 1536 / 512 columns) and a
    lip-shortcut shape (frames x 144 pixels), within 1e-5 of sum |a b| of fp64."""
    g = torch.Generator(device=DEV).manual_seed(rows + ca)
    a = torch.randn(rows, ca, device=DEV, generator=g) * torch.exp(2.0 * torch.randn(rows, ca, device=DEV, generator=g))
    b = torch.randn(rows, cb, device=DEV, generator=g)
    got = K().gemm_f32s_rows_tn(K().split_planes(a[None]), K().split_planes(b[None]), units)
    ref = b.double().t() @ a.double()
    mag = b.double().abs().t() @ a.double().abs()
    assert got.shape == (cb, ca)
    err = float(((got.double() - ref).abs() / (mag + 1e-300)).max())
    print(f"rows_tn {rows, units, ca, cb}: {err:.2e} of sum|ab|")
    assert err <= 1e-5, err


def test_time_conv1d_split_gemm_backward_vs_fp64():
    """layers._TimeConv1dFn on the GPU (the avse1 TCN conv: hipBLASLt forward, split-GEMM weight and input gradients)
    vs nn.Conv1d in fp64 on the same weights: output, input, weight and bias gradients."""
    from avse_challenge_amd.layers import time_conv1d
    torch.manual_seed(5)
    B, T, C, k, dil = 4, 75, 512, 3, 4
    conv = torch.nn.Conv1d(C, C, k, padding=(k - 1) * dil, dilation=dil).double()
    x = torch.randn(B, T, C, dtype=torch.float64)
    gy = torch.randn(B, T + (k - 1) * dil, C, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    (conv(xr.transpose(1, 2)).transpose(1, 2) * gy).sum().backward()
    cg = torch.nn.Conv1d(C, C, k, padding=(k - 1) * dil, dilation=dil).to(DEV)
    cg.load_state_dict({n: v.float() for n, v in conv.state_dict().items()})
    xg = x.float().to(DEV).requires_grad_(True)
    y = time_conv1d(xg, cg)
    (y * gy.float().to(DEV)).sum().backward()
    for got, want, what in ((y, conv(x.transpose(1, 2)).transpose(1, 2), "y"), (xg.grad, xr.grad, "dx"),
                            (cg.weight.grad, conv.weight.grad, "dw"), (cg.bias.grad, conv.bias.grad, "db")):
        err = float((got.detach().double().cpu() - want.detach()).abs().max())
        sc = float(want.detach().abs().max())
        assert err <= 2e-5 * sc, (what, err, sc)


@pytest.mark.parametrize("cin,cout,s,H", [(64, 128, 2, 24), (256, 512, 2, 6), (64, 64, 1, 12)])
def test_pointwise_conv2d_split_wgrad_vs_fp64(cin, cout, s, H):
    """layers.PointwiseConv2d (the lip ResNet 1x1 shortcut: one GEMM forward, split-GEMM weight gradient over frame
    groups) on channels-last activations vs nn.Conv2d in fp64."""
    from avse_challenge_amd.layers import PointwiseConv2d
    torch.manual_seed(11)
    ref = torch.nn.Conv2d(cin, cout, 1, stride=s, bias=False).double()
    ours = PointwiseConv2d(cin, cout, s).to(DEV).to(memory_format=torch.channels_last)
    ours.load_state_dict({n: v.float() for n, v in ref.state_dict().items()})
    x = torch.randn(40, cin, H, H, dtype=torch.float64)
    ho = (H - 1) // s + 1
    gy = torch.randn(40, cout, ho, ho, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    (ref(xr) * gy).sum().backward()
    xg = x.float().to(DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    (ours(xg) * gy.float().to(DEV)).sum().backward()
    for got, want, what in ((xg.grad, xr.grad, "dx"), (ours.weight.grad, ref.weight.grad, "dw")):
        err = float((got.double().cpu() - want).abs().max())
        sc = float(want.abs().max())
        assert err <= 2e-5 * sc, (what, err, sc)
