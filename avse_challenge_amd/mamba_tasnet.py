"""Mamba-TasNet separator on the MI355X kernels (drop-in for the reference modules).

Mirrors, with identical parameter names / state_dict keys (checkpoints load unchanged):
  MambaInnerNoOutProj  Mamba-TasNet/modules/mamba/selective_scan_interface.py:160-294
  BiMambaV2            modules/mamba/bimamba.py:39-174 (params), :176-253 (v2 forward)
  Block                modules/mamba/bimamba.py:409-462 (Add -> RMSNorm -> mixer)
  MambaBlocksSequential modules/mamba_blocks.py:87-212
  MaskNet              modules/mamba_masknet.py:13-139
  Encoder / Decoder    speechbrain dual_path Encoder/Decoder (hparams mambatasnet_*.yaml)
  MambaTasNet.forward  train_wsj0mix.py:86-111 compute_forward
The scan, the causal conv and the add+RMSNorm run in libavse_hip.so; the dense projections
are GEMMs: bf16 (autocast) in_proj / out_proj / x_proj and their input gradients on the HIP MFMA GEMM
(csrc/projgemm.hip); the fp32 in_proj / out_proj, their input and weight gradients on the same kernel's split-fp16 mode
(avse_gemm_f32s, fp32-accurate); the rank-sized x_proj GEMMs and the bf16 weight gradients on hipBLASLt
(torch.matmul); dt_proj (K = dt_rank) is csrc/dtproj.hip with the scan's softplus in its epilogue.  No CPU fallback:
CPU tensors raise.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K

NSTATE = 16
# bf16 autocast (BASELINE configs[4]): the projections then run as bf16 GEMMs and the conv / scan on bf16
# activations with fp32 state, as mamba-ssm's custom_fwd / custom_bwd functions do
# (selective_scan_interface.py:170-176); the backward runs under the forward's autocast state.
_FWD = torch.amp.custom_fwd(device_type="cuda")
_BWD = torch.amp.custom_bwd(device_type="cuda")


# bf16 projections (BASELINE configs[4]) on the HIP MFMA GEMM (csrc/projgemm.hip) at the sites where it measured faster
# than hipBLASLt at C5 (profiles/r04g_projgemm_probe_vs_lib.jsonl: in_proj forward 0.26 vs 0.25 of the bf16 peak, in_proj
# input gradient 0.34 vs 0.32, out_proj input gradient 0.30 vs 0.25); out_proj forward (0.29 vs 0.35) and the bf16 weight
# gradients (0.29-0.32 vs 0.34-0.36) stay on the library.


def _autocast_dtype():
    return torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else None


def _hip_gemm(P, Q, out, alpha=1.0, fold=1):
    """out[g, q, p] = alpha sum_{b in group g} sum_k P[b, p, k] Q[b, q, k] on the HIP bf16 GEMM; None when it does not
    take them.  Reductions shorter than 64 stay on the library: their single-stage tiles are all epilogue."""
    if min(P.shape[1], Q.shape[1]) >= 128 and P.shape[2] >= 64 and K.gemm_bf16_supported(P, Q, out, fold):
        return K.gemm_bf16(P, Q, out, alpha, fold)
    return None


# fp32 projections (Mamba-TasNet C3) on the split-fp16 MFMA GEMM (avse_gemm_f32s: both operands split into hi / lo fp16
# planes, three MFMAs per product, fp32 accumulation; fp32-accurate) where the tiles fill.


def _f32_ok(P, Q, out, fold=1):
    return (min(P.shape[1], Q.shape[1]) >= 128 and P.shape[2] >= 64
            and K.gemm_f32s_supported(P, Q, out, fold))


def _f32_gemm(P, Q, out, alpha=1.0, fold=1):
    """out[g, q, p] = alpha sum_{b in group g} sum_k P[b, p, k] Q[b, q, k] in fp32 on avse_gemm_f32s; None when it does
    not take them (the x_proj / dt_proj rank-sized projections stay on the library).  The in / out projections call
    gemm_f32s themselves with shared Splits (an activation used by two GEMMs is split once)."""
    if _f32_ok(P, Q, out, fold):
        return K.gemm_f32s(P, Q, out, alpha, fold)
    return None


def _wbmm(w, x, alpha=1.0):
    """alpha (m, k) weight @ (b, k, n) -> (b, m, n) as one strided-batched GEMM (weight batch stride 0).
    Keeping every projection in the scan's (b, channels, l) layout means no layout copies.  The output rows get
    the kernels' cache-line-aligned time stride (kernels.TIME_ALIGN_BYTES; the GEMM writes with ldc = the padded
    stride), so every (b, d, l) operand of the conv / scan kernels starts its rows on a 128-B line."""
    dt = _autocast_dtype()
    if dt is not None:
        w, x = w.to(dt), x.to(dt)
    else:
        dt = torch.result_type(w, x)
    out = K.bdl_empty(x.shape[0], w.shape[0], x.shape[2], dt, x.device)
    if _hip_gemm(x.transpose(1, 2), w[None], out, alpha) is not None:
        return out
    if dt == torch.float32 and _f32_gemm(x.transpose(1, 2), w[None], out, alpha) is not None:
        return out
    if alpha != 1.0:
        w = alpha * w
    with torch.autocast("cuda", enabled=False):
        return torch.bmm(w.expand(x.shape[0], *w.shape), x, out=out)


def _padded_full(t):
    """t's (b, c, Lp) padded storage as a contiguous tensor (the 128-B time stride of kernels.bdl_empty), or None."""
    if t.dim() != 3 or t.stride(2) != 1 or t.stride(1) < t.size(2) or t.stride(0) != t.size(1) * t.stride(1):
        return None
    need = (t.storage_offset() + t.size(0) * t.stride(0)) * t.element_size()
    if t.untyped_storage().nbytes() < need:
        return None
    return t.as_strided((t.size(0), t.size(1), t.stride(1)), t.stride())


def _padded_add(a, b):
    """a + b for two (b, c, l) operands with the same padded time stride: one contiguous vectorised add over the
    padded storage (the pad columns hold don't-care values), returned as the (b, c, l) view.  torch's add on the
    strided views takes its generic non-vectorised kernel (~0.75 ms instead of ~0.45 ms per C3 Mamba-L tensor)."""
    if a is None:
        return b
    if b is None:
        return a
    if a.stride() == b.stride() and a.dtype == b.dtype:
        fa, fb = _padded_full(a), _padded_full(b)
        if fa is not None and fb is not None:
            return torch.add(fa, fb)[..., :a.size(2)]
    return a + b


class _Fork(torch.autograd.Function):
    """xz consumed by both BiMamba directions: the two incoming gradients are summed by _padded_add (autograd's own
    accumulation would take the strided generic kernel)."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x), x.view_as(x)

    @staticmethod
    def backward(ctx, g1, g2):
        if g1 is not None and g2 is not None and g1.dtype == g2.dtype == torch.float32 and g1.stride() == g2.stride():
            fa, fb = _padded_full(g1), _padded_full(g2)
            if fa is not None and fb is not None and fa.is_contiguous() and fb.is_contiguous():
                return K.add_max(fa, fb, g1.size(2))    # with its max: the fp32 in_proj backward's split skips its pass
        return _padded_add(g1, g2)


def _unit_stride(t):
    """t, or a contiguous copy when neither of its last two dims has unit stride (split_planes needs one)"""
    return t if t.stride(2) == 1 or t.stride(1) == 1 else t.contiguous()


def _fold_for(nb, m, n):
    """batches folded into groups so that a weight-gradient launch has about one 256 x 256 tile per CU"""
    fold = max(1, nb * (-(-m // 256)) * (-(-n // 256)) // 256)
    while nb % fold:
        fold -= 1
    return fold


def _bsum_split(a_split, bt_split, m, n, alpha=1.0):
    """alpha sum_b a[b] @ bt[b] (m, n) fp32 from the Splits of a (b, m, l) and bt (b, l, n) (avse_gemm_f32s, folded)."""
    nb = a_split.hi.shape[0]
    fold = _fold_for(nb, m, n)
    out = torch.empty(nb // fold, m, n, device=a_split.hi.device, dtype=torch.float32)
    K.gemm_f32s_split(bt_split.t(), a_split, out, alpha, fold)
    return out.sum(0)


def _bsum_mm(a, bt, alpha=1.0):
    """alpha sum_b a[b] @ bt[b] for a (b, m, l), bt (b, l, n): the weight gradient of a batched projection, fp32.
    fp32 operands: the split-fp16 GEMM (avse_gemm_f32s, batches folded into groups).  Under bf16 autocast (the library's
    bf16 weight gradients measured faster than avse_gemm_bf16) and where the split GEMM does not apply: one
    strided-batched GEMM + sum while the (b, m, n) partials are small (Mamba-TasNet: b = batch);
    as ONE (m, b*l) x (b*l, n) GEMM when they are not (DPMamba's inter pass has b = B*250 sequences of
    34 frames: the partials would take 33 GB, and each GEMM's depth would be 34)."""
    nb, m, l = a.shape
    n = bt.shape[2]
    dt = _autocast_dtype()
    if dt is None and a.dtype == bt.dtype == torch.float32:
        # batches folded into groups so that the launch has about one 256 x 256 tile per CU; groups summed after
        fold = _fold_for(nb, m, n)
        out = torch.empty(nb // fold, m, n, device=a.device, dtype=torch.float32)
        if _f32_gemm(bt.transpose(1, 2), a, out, alpha, fold=fold) is not None:
            return out.sum(0)
    if nb * m * n <= (1 << 27):
        r = torch.bmm(a, bt).float().sum(0)
    else:
        r = (a.transpose(0, 1).reshape(m, nb * l) @ bt.reshape(nb * l, n)).float()
    return r if alpha == 1.0 else alpha * r


# dt_proj with the softplus in its epilogue (csrc/dtproj.hip) feeding the scan in delta_softplus mode 2; a rank above 64
# (no reference config): the GEMM and the scan's own per-element softplus (mode 1), as the reference calls it.


def _delta(dt_proj_w, x_rows, dt_bias):
    """(delta, delta_bias, delta_softplus) for the scan: softplus(W x + b) from the fused kernel (bias None, mode 2), or
    the raw GEMM output with the bias and mode 1 (rank > 64)."""
    if dt_proj_w.shape[1] <= 64:
        dt = _autocast_dtype() or torch.result_type(dt_proj_w, x_rows)
        return K.dtproj(dt_proj_w.to(dt), x_rows.to(dt), dt_bias, True), None, 2
    return _wbmm(dt_proj_w, x_rows), dt_bias, True


def _dir_fwd(xz, conv_w, conv_b, x_proj_w, dt_proj_w, A, D, dt_bias, reverse, acc=None, out_max=None):
    """One BiMamba direction's forward (MambaInnerNoOutProj): -> (out_z, tensors to save).  acc: a tensor the gated
    output is added to in place (the scan's flush) and returned as out_z; out_max: a zeroed word for max |out_z|."""
    R = dt_proj_w.shape[1]
    x, z = xz.chunk(2, dim=1)
    conv_out = K.causal_conv1d_fwd(x, conv_w, conv_b, silu=True, reverse=reverse)     # (b, d, l)
    x_dblT = _wbmm(x_proj_w, conv_out)                                       # (b, R + 2n, l)
    delta, bias, mode = _delta(dt_proj_w, x_dblT[:, :R], dt_bias)             # (b, d, l)
    Bm, Cm = x_dblT[:, R:R + NSTATE], x_dblT[:, R + NSTATE:]                 # (b, n, l) views
    # the pre-gate `out` is neither written nor saved (the reference saves it, :212): the scan
    # backward recomputes y + D u per step anyway, so it only cost HBM traffic and memory
    _, xck, out_z = K.selective_scan_fwd(conv_out, delta, A, Bm, Cm, D, z, bias, mode, reverse=reverse,
                                         return_out=False, out_z_acc=acc, out_z_max=out_max)
    return out_z, (xz, conv_w, conv_b, x_dblT, x_proj_w, dt_proj_w, A, D, dt_bias, xck)


def _dir_bwd(saved, dout, reverse, dxz=None, accumulate=False, dmax=None):
    """One direction's backward -> (dxz, dconv_w, dconv_b, dx_proj_w, ddt_proj_w, dA, dD, ddt_bias).  dxz /
    accumulate: write the xz gradient into the given buffer, or add it there (the other direction's, round 6); dmax: a
    zeroed word for max |dxz| (both halves: the scan's dz and the conv's dx)."""
    xz, conv_w, conv_b, x_dblT, x_proj_w, dt_proj_w, A, D, dt_bias, xck = saved
    R = dt_proj_w.shape[1]
    x, z = xz.chunk(2, dim=1)
    conv_out = K.causal_conv1d_fwd(x, conv_w, conv_b, silu=True, reverse=reverse)
    delta, bias, mode = _delta(dt_proj_w, x_dblT[:, :R], dt_bias)             # the forward's values bit for bit
    Bm, Cm = x_dblT[:, R:R + NSTATE], x_dblT[:, R + NSTATE:]
    if dxz is None:
        dxz = K.bdl_empty(xz.shape[0], xz.shape[1], xz.shape[2], xz.dtype, xz.device)
    dx, dz = dxz.chunk(2, dim=1)
    dx_dblT = K.bdl_empty(*x_dblT.shape, torch.float32, x_dblT.device)         # scan writes fp32 dB/dC
    # ddelta / ddt_bias: gradients w.r.t. the pre-softplus dt_proj output and the bias in either mode
    dconv, ddelta, dA, _, _, dD, ddt_bias, dz, _ = K.selective_scan_bwd(
        conv_out, delta, A, Bm, Cm, D, z, bias, dout, xck, None, dz, mode, False, reverse=reverse,
        dB_out=dx_dblT[:, R:R + NSTATE], dC_out=dx_dblT[:, R + NSTATE:], dz_accumulate=accumulate, dz_max=dmax)
    dx_dblT[:, :R] = _wbmm(dt_proj_w.t(), ddelta)
    ddt_proj_w = _bsum_mm(ddelta, x_dblT[:, :R].transpose(1, 2))               # (d, R)
    dxd = dx_dblT.to(dconv.dtype)          # bf16 under autocast: one cast for both GEMMs (the bmm would cast its own)
    dx_proj_w = _bsum_mm(dxd if _autocast_dtype() is not None else dx_dblT, conv_out.transpose(1, 2))  # (R + 2n, d)
    wxt = x_proj_w.t().to(dconv.dtype)
    dconv.baddbmm_(wxt.expand(dconv.shape[0], *wxt.shape), dxd)
    _, dconv_w, dconv_b = K.causal_conv1d_bwd(x, conv_w, conv_b, dconv, dx=dx, silu=True, reverse=reverse,
                                              dx_accumulate=accumulate, dx_max=dmax)
    return dxz, dconv_w.view_as(conv_w), dconv_b, dx_proj_w, ddt_proj_w, dA, dD, ddt_bias


class MambaInnerNoOutProj(torch.autograd.Function):
    """Conv1d(k4)+SiLU -> x_proj -> dt_proj -> selective scan (z-gated); checkpoint_lvl 1.

    The x_proj output is kept transposed, x_dblT = W_x conv_out of shape (b, R + 2n, l): delta,
    B and C are then row slices in the scan's layout (the reference builds x_dbl as (b*l, R+2n)
    and rearranges, :180-197); every forward / backward GEMM is a strided-batched GEMM on the
    (b, channels, l) layout, so no (b, d, l) tensor is ever transposed in memory.

    ``reverse=True`` is the v2 backward direction WITHOUT the two flip copies of bimamba.py:236,253:
    the conv and the scan walk time backwards by index, so the result is already the reference's
    ``out_b.flip(-1)`` in natural time order."""

    @staticmethod
    @_FWD
    def forward(ctx, xz, conv_w, conv_b, x_proj_w, dt_proj_w, A, D, dt_bias, reverse=False):
        out_z, saved = _dir_fwd(xz, conv_w, conv_b, x_proj_w, dt_proj_w, A, D, dt_bias, reverse)
        ctx.save_for_backward(*saved)
        ctx.reverse = reverse
        return out_z

    @staticmethod
    @_BWD
    def backward(ctx, dout):
        return (*_dir_bwd(ctx.saved_tensors, dout, ctx.reverse), None)


class BiMambaSerial(torch.autograd.Function):
    """Both v2 directions as ONE autograd node, run one after the other on one stream (round 6):
    -> y = out_f + out_b (natural time order; the 0.5 of bimamba.py:253 is the out_proj's alpha).  The backward
    direction's scan adds its gated output to the forward one's in its flush, and in the backward the two
    directions sum their xz gradients in one buffer (the scan's dz and the conv's dx accumulate): no (b, d_inner, l)
    add in the forward and no (b, 2 d_inner, l) add in the backward (C5 bf16: torch adds, 18.5 ms per step; C3 fp32:
    avse_add_max, 0.62 ms per call).  fp32: the accumulating kernels also report max |y| and max |dxz| (atomic max per
    wave), attached as the producer-side max that the projections' operand splits would otherwise compute."""

    @staticmethod
    @_FWD
    def forward(ctx, xz, cw, cb, xw, dw, A, D, db, cw_b, cb_b, xw_b, dw_b, A_b, D_b, db_b):
        mx = torch.zeros(1, device=xz.device, dtype=torch.int32) if xz.dtype == torch.float32 else None
        f, sf = _dir_fwd(xz, cw, cb, xw, dw, A, D, db, False)
        y, sb = _dir_fwd(xz, cw_b, cb_b, xw_b, dw_b, A_b, D_b, db_b, True, acc=f, out_max=mx)
        ctx.save_for_backward(*sf, *sb)
        if mx is not None:
            K._set_absmax(y, mx)
        return y

    @staticmethod
    @_BWD
    def backward(ctx, dy):
        saved = ctx.saved_tensors
        n = len(saved) // 2
        xz = saved[0]
        mx = torch.zeros(1, device=xz.device, dtype=torch.int32) if xz.dtype == torch.float32 else None
        gb = _dir_bwd(saved[n:], dy, True)                        # writes the xz gradient
        gf = _dir_bwd(saved[:n], dy, False, gb[0], True, mx)     # adds its own to it
        if mx is not None:
            K._set_absmax(gf[0], mx)
        return (gf[0], *gf[1:], *gb[1:])


class _InProj(torch.autograd.Function):
    """xz = W_in h^T: (b, l, d_model) -> (b, 2 d_inner, l) (bimamba.py:192-196); grads in the
    layouts their consumers want: dh (b, l, d_model) contiguous, no transposed copies."""

    @staticmethod
    @_FWD
    def forward(ctx, h, w):
        if _autocast_dtype() is None and h.dtype == w.dtype == torch.float32:
            # fp32 (C3): h's split planes serve the forward GEMM and, saved in place of h, the weight gradient
            out = K.bdl_empty(h.shape[0], w.shape[0], h.shape[1], torch.float32, h.device)
            if _f32_ok(h, w[None], out):
                hs = K.split_planes(h)
                K.gemm_f32s(h, w[None], out, ps=hs)
                ctx.save_for_backward(hs.hi, hs.lo, hs.mb, w)
                ctx.split = True
                return out
        dt = _autocast_dtype()
        if dt is not None and h.dtype != dt:
            # under autocast: cast once and keep the copy for the weight gradient (its bmm would cast h again: one
            # (b, l, d_model) copy per layer and step, profiles/r06z_c5_library_ops.txt)
            h = h.to(dt)
        ctx.save_for_backward(h, w)
        ctx.split = False
        return _wbmm(w, h.transpose(1, 2))

    @staticmethod
    @_BWD
    def backward(ctx, dxz):
        if ctx.split:
            # fp32 split path: dxz split once for both GEMMs; h only as its planes
            hhi, hlo, hmb, w = ctx.saved_tensors
            dxz = _unit_stride(dxz)
            out = torch.empty(dxz.shape[0], dxz.shape[2], w.shape[1], device=dxz.device, dtype=torch.float32)
            ds = K.split_planes(dxz)
            if _f32_ok(w.t()[None], dxz.transpose(1, 2), out):
                dh = K.gemm_f32s(w.t()[None], dxz.transpose(1, 2), out, qs=ds.t())
            else:
                dh = torch.bmm(dxz.transpose(1, 2), w.expand(dxz.shape[0], *w.shape))
            return dh, _bsum_split(ds, K.Split(hhi, hlo, hmb), dxz.shape[1], hhi.shape[2])
        h, w = ctx.saved_tensors
        dt = _autocast_dtype()
        dh = None
        if dt is not None:
            wc, dxc = w.to(dt), dxz.to(dt)
            dh = _hip_gemm(wc.t()[None], dxc.transpose(1, 2),
                           torch.empty(dxz.shape[0], dxz.shape[2], w.shape[1], device=dxz.device, dtype=dt))
        elif dxz.dtype == torch.float32:
            out = torch.empty(dxz.shape[0], dxz.shape[2], w.shape[1], device=dxz.device, dtype=torch.float32)
            dh = _f32_gemm(w.t()[None], dxz.transpose(1, 2), out)
        if dh is None:
            dh = torch.bmm(dxz.transpose(1, 2), w.expand(dxz.shape[0], *w.shape))
        dw = _bsum_mm(dxz, h)
        return dh, dw


class _BiOutProj(torch.autograd.Function):
    """out = (0.5 f + 0.5 b)^T W_out^T for the two v2 directions (bimamba.py:253, flip-free):
    (b, d_inner, l) x 2 -> (b, l, d_model).  One add in the forward; the backward hands the same
    (b, d_inner, l) gradient to both directions (no 0.5-scaled copies)."""

    @staticmethod
    @_FWD
    def forward(ctx, f, bk, w):
        dt = _autocast_dtype()
        y = None
        ctx.two = bk is not None                   # bk None: f already holds the direction sum
        if (bk is not None and dt is None and f.dtype == bk.dtype == w.dtype == torch.float32
                and f.stride() == bk.stride()):
            fa, fb = _padded_full(f), _padded_full(bk)
            if fa is not None and fb is not None and fa.is_contiguous() and fb.is_contiguous():
                y = K.add_max(fa, fb, f.size(2))        # the sum with its max: the split below skips the absmax pass
        if y is None:
            y = _padded_add(f, bk)
        ctx.split = False
        if dt is None and y.dtype == w.dtype == torch.float32:
            # fp32 (C3): y's split planes serve the forward GEMM and, saved in place of y, the weight gradient
            out = torch.empty(y.shape[0], y.shape[2], w.shape[0], device=y.device, dtype=torch.float32)
            if _f32_ok(w[None], y.transpose(1, 2), out):
                ys = K.split_planes(y)
                K.gemm_f32s(w[None], y.transpose(1, 2), out, 0.5, qs=ys.t())
                ctx.save_for_backward(ys.hi, ys.lo, ys.mb, w)
                ctx.split = True
                return out
        ctx.save_for_backward(y, w)
        if dt is None and y.dtype == torch.float32:
            out = _f32_gemm(w[None], y.transpose(1, 2),
                            torch.empty(y.shape[0], y.shape[2], w.shape[0], device=y.device, dtype=torch.float32), 0.5)
            if out is not None:
                return out
        wt = 0.5 * w.t()
        return torch.bmm(y.transpose(1, 2), wt.expand(y.shape[0], *wt.shape))

    @staticmethod
    @_BWD
    def backward(ctx, dout):
        if ctx.split:
            yhi, ylo, ymb, w = ctx.saved_tensors
            ys = K.Split(yhi, ylo, ymb)
            dout = _unit_stride(dout)
            dy = K.bdl_empty(dout.shape[0], w.shape[1], dout.shape[1], torch.float32, dout.device)
            dsp = K.split_planes(dout)                 # (b, l, d_model): shared by the input and the weight gradient
            if _f32_ok(dout, w.t()[None], dy):
                K.gemm_f32s(dout, w.t()[None], dy, 0.5, ps=dsp)                      # dy = 0.5 W^T dout^T
            else:
                torch.bmm((0.5 * w.t()).expand(dout.shape[0], *w.t().shape), dout.transpose(1, 2), out=dy)
            dw = _bsum_split(dsp.t(), ys.t(), w.shape[0], w.shape[1], 0.5)         # 0.5 sum_b dout^T y^T
            return dy, (dy if ctx.two else None), dw
        y, w = ctx.saved_tensors
        dt = _autocast_dtype()
        if dt is not None and dout.dtype != dt:
            dout = dout.to(dt)                          # one cast for both GEMMs below (each would cast its own copy)
        dy = _wbmm(w.t(), dout.transpose(1, 2), 0.5)                             # (b, d_inner, l)
        dw = _bsum_mm(dout.transpose(1, 2), y.transpose(1, 2), 0.5)               # (d_model, d_inner)
        return dy, (dy if ctx.two else None), dw


class AddRMSNorm(torch.autograd.Function):
    """(RMSNorm(h + res) * w, h + res) — bimamba.py:447-451 with mamba-ssm RMSNorm (eps 1e-5)."""

    @staticmethod
    def forward(ctx, h, res, weight, eps, mixer_input=False):
        # mixer_input (Block): under bf16 autocast the norm output is written in bf16 — the mixer's in_proj casts it
        # there anyway, and mamba-ssm's fused add_norm returns its input's dtype (bf16 under autocast) — and h (the
        # previous mixer's bf16 output) is read as it is; h + res and the statistics stay fp32 (residual_in_fp32)
        dt = _autocast_dtype() if mixer_input else None
        y, res_out, rstd = K.add_rmsnorm_fwd(h, res, weight, eps, out_dtype=dt if dt == torch.bfloat16 else None)
        ctx.has_res = res is not None
        ctx.save_for_backward(res_out, weight, rstd)
        return y, res_out

    @staticmethod
    def backward(ctx, dy, dres):
        res_out, weight, rstd = ctx.saved_tensors
        dx, dw = K.rmsnorm_bwd(dy, dres, res_out, weight, rstd)
        return dx, (dx if ctx.has_res else None), dw, None, None


class RMSNorm(nn.Module):
    def __init__(self, hidden_size, eps=1e-5, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hidden_size, device=device))

    def forward(self, x, residual=None):
        return AddRMSNorm.apply(x, residual, self.weight, self.eps)[0]


_STREAMS = {}
# set_direction_streams(True): the v2 backward direction on a second HIP stream.  Off by default: the two directions'
# selective scans each fill the GPU (C5 B=32: 512 scan-backward workgroups = 2 per CU), so concurrent launches only
# share the CUs (5.85 vs 2.90 ms per launch) and the step was slower with the streams (571.7 vs 552.5 ms per C5 step,
# gpurun_out/r06e_c5_*.log; round 1, before the scan kernels filled the GPU, the streams gained 762 -> 727 ms)
DIRECTION_STREAMS = False


def set_direction_streams(on):
    """Run BiMamba v2's backward direction on a second HIP stream (True) or serially on the current stream (False,
    the default); returns the previous setting."""
    global DIRECTION_STREAMS
    old, DIRECTION_STREAMS = DIRECTION_STREAMS, bool(on)
    return old


def _direction_stream(device):
    """Second HIP stream for the v2 backward direction, one per device (DIRECTION_STREAMS)."""
    if device.type != "cuda" or not DIRECTION_STREAMS:
        return None
    if device not in _STREAMS:
        _STREAMS[device] = torch.cuda.Stream(device)
    return _STREAMS[device]


class BiMambaV2(nn.Module):
    """bimamba.Mamba(bimamba_type='v2', if_devide_out=True): same parameters and init."""

    def __init__(self, d_model, d_state=16, d_conv=4, expand=2, dt_min=0.001, dt_max=0.1, dt_init_floor=1e-4):
        super().__init__()
        assert d_state == NSTATE, "the HIP scan is built for d_state 16 (all reference configs)"
        self.d_model, self.d_state, self.d_conv = d_model, d_state, d_conv
        self.d_inner = expand * d_model
        self.dt_rank = math.ceil(d_model / 16)
        di, r, n = self.d_inner, self.dt_rank, d_state
        self.in_proj = nn.Linear(d_model, 2 * di, bias=False)
        self.conv1d = nn.Conv1d(di, di, d_conv, groups=di, padding=d_conv - 1, bias=True)
        self.x_proj = nn.Linear(di, r + 2 * n, bias=False)
        self.dt_proj = nn.Linear(r, di, bias=True)
        self.A_log = nn.Parameter(torch.log(torch.arange(1, n + 1, dtype=torch.float32)).repeat(di, 1))
        self.D = nn.Parameter(torch.ones(di))
        self.A_b_log = nn.Parameter(torch.log(torch.arange(1, n + 1, dtype=torch.float32)).repeat(di, 1))
        self.conv1d_b = nn.Conv1d(di, di, d_conv, groups=di, padding=d_conv - 1, bias=True)
        self.x_proj_b = nn.Linear(di, r + 2 * n, bias=False)
        self.dt_proj_b = nn.Linear(r, di, bias=True)
        self.D_b = nn.Parameter(torch.ones(di))
        self.out_proj = nn.Linear(di, d_model, bias=False)
        # dt init as bimamba.py:101-120
        std = self.dt_rank ** -0.5
        with torch.no_grad():
            for proj in (self.dt_proj, self.dt_proj_b):
                nn.init.uniform_(proj.weight, -std, std)
                dt = torch.exp(torch.rand(di) * (math.log(dt_max) - math.log(dt_min)) + math.log(dt_min))
                dt = dt.clamp(min=dt_init_floor)
                proj.bias.copy_(dt + torch.log(-torch.expm1(-dt)))

    def forward(self, h):                                        # (b, l, d_model)
        xz = _InProj.apply(h, self.in_proj.weight)                               # (b, 2di, l), no copy
        A = -torch.exp(self.A_log.float())
        A_b = -torch.exp(self.A_b_log.float())
        side = _direction_stream(xz.device)
        if side is None:
            # serial directions (C3, C5): one node that sums both the outputs and the xz gradients in place (fp32:
            # with the sums' maxima for the projections' splits)
            y = BiMambaSerial.apply(xz, self.conv1d.weight, self.conv1d.bias, self.x_proj.weight, self.dt_proj.weight,
                                    A, self.D.float(), self.dt_proj.bias.float(), self.conv1d_b.weight,
                                    self.conv1d_b.bias, self.x_proj_b.weight, self.dt_proj_b.weight, A_b,
                                    self.D_b.float(), self.dt_proj_b.bias.float())
            return _BiOutProj.apply(y, None, self.out_proj.weight)
        xz, xz_b = _Fork.apply(xz)                # one input per direction; their gradients meet in _padded_add
        if side is not None:
            # the two directions are independent: the backward one runs on a second HIP stream, so its conv /
            # projection / scan kernels fill the CUs the forward one leaves idle (the scan grid at B=32 is
            # 512 workgroups for 768 slots). Autograd runs each direction's backward on the same stream.
            main = torch.cuda.current_stream(xz.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                bk = MambaInnerNoOutProj.apply(xz_b, self.conv1d_b.weight, self.conv1d_b.bias, self.x_proj_b.weight,
                                               self.dt_proj_b.weight, A_b, self.D_b.float(),
                                               self.dt_proj_b.bias.float(), True)
            xz_b.record_stream(side)
            A_b.record_stream(side)
        f = MambaInnerNoOutProj.apply(xz, self.conv1d.weight, self.conv1d.bias, self.x_proj.weight,
                                      self.dt_proj.weight, A, self.D.float(), self.dt_proj.bias.float())
        if side is None:
            bk = MambaInnerNoOutProj.apply(xz_b, self.conv1d_b.weight, self.conv1d_b.bias, self.x_proj_b.weight,
                                           self.dt_proj_b.weight, A_b, self.D_b.float(), self.dt_proj_b.bias.float(),
                                           True)
        else:
            main.wait_stream(side)
            bk.record_stream(main)
        # == out_proj(0.5*out + 0.5*out_b.flip(-1)) of bimamba.py:253, flip-free, one batched GEMM
        return _BiOutProj.apply(f, bk, self.out_proj.weight)


class Block(nn.Module):
    def __init__(self, d_model, mixer, eps=1e-5):
        super().__init__()
        self.mixer = mixer
        self.norm = RMSNorm(d_model, eps)

    def forward(self, h, residual=None):
        y, residual = AddRMSNorm.apply(h, residual, self.norm.weight, self.norm.eps, True)
        return self.mixer(y), residual


class MambaBlocksSequential(nn.Module):
    def __init__(self, n_mamba, d_model, d_state=16, expand=2, d_conv=4, eps=1e-5):
        super().__init__()
        self.layers = nn.Sequential(*[Block(d_model, BiMambaV2(d_model, d_state, d_conv, expand), eps)
                                      for _ in range(n_mamba)])
        self.norm_f = RMSNorm(d_model, eps)

    def forward(self, x):
        h, res = x, None
        for layer in self.layers:
            h, res = layer(h, res)
        return AddRMSNorm.apply(h, res, self.norm_f.weight, self.norm_f.eps)[0]


class ChannelwiseLayerNorm(nn.Module):
    """speechbrain conv_tasnet.ChannelwiseLayerNorm (EPS 1e-8, biased var over channels)."""

    def __init__(self, channels, eps=1e-8):
        super().__init__()
        self.eps = eps
        self.gamma = nn.Parameter(torch.ones(1, 1, channels))
        self.beta = nn.Parameter(torch.zeros(1, 1, channels))

    def forward(self, y):
        var, mean = torch.var_mean(y, dim=2, keepdim=True, unbiased=False)
        return self.gamma * (y - mean) * torch.rsqrt(var + self.eps) + self.beta


class Conv1x1(nn.Module):
    """speechbrain nnet.CNN.Conv1d(kernel_size=1, bias=False) on (B, L, C); key conv.weight."""

    def __init__(self, cin, cout):
        super().__init__()
        self.conv = nn.Conv1d(cin, cout, 1, bias=False)

    def forward(self, x):
        return F.linear(x, self.conv.weight[:, :, 0])


class MaskNet(nn.Module):
    def __init__(self, enc_dim, bot_dim, n_spk=2, n_mamba=16, d_model=256, d_state=16, expand=2, d_conv=4):
        super().__init__()
        self.n_spk = n_spk
        self.layer_norm = ChannelwiseLayerNorm(enc_dim)
        self.bottleneck_conv1x1 = Conv1x1(enc_dim, bot_dim)
        self.mamba_net = MambaBlocksSequential(n_mamba, d_model, d_state, expand, d_conv)
        self.mask_conv1x1 = Conv1x1(bot_dim, n_spk * enc_dim)

    def forward(self, mixture_w):                      # (M, N, K) -> (n_spk, M, N, K)
        x = mixture_w.permute(0, 2, 1)
        Bn, L, D = x.shape
        y = self.mask_conv1x1(self.mamba_net(self.bottleneck_conv1x1(self.layer_norm(x))))
        return F.relu(y.reshape(Bn, L, self.n_spk, D).permute(2, 0, 3, 1))


class Encoder(nn.Module):
    """Conv1d(1, N, k, stride k/2) + ReLU as framing + GEMM (MIOpen's pick for this shape is a naive
    direct kernel: 270 ms per backward call at B=16, profiles/)."""

    def __init__(self, kernel_size=16, out_channels=512):
        super().__init__()
        self.conv1d = nn.Conv1d(1, out_channels, kernel_size, stride=kernel_size // 2, bias=False)

    def forward(self, x):                                      # (B, T) -> (B, N, L)
        k = self.conv1d.kernel_size[0]
        frames = x.unfold(-1, k, self.conv1d.stride[0])        # (B, L, k) view
        return F.relu(torch.matmul(self.conv1d.weight[:, 0, :], frames.transpose(1, 2)))


class Decoder(nn.ConvTranspose1d):
    """ConvTranspose1d(N, 1, k, stride k/2) as GEMM + overlap-add (F.fold)."""

    def forward(self, x):                                      # (B, N, L) -> (B, T')
        k, s = self.kernel_size[0], self.stride[0]
        L = x.shape[-1]
        frames = torch.matmul(self.weight[:, 0, :].t(), x)     # (B, k, L)
        T = (L - 1) * s + k
        return F.fold(frames, (1, T), (1, k), stride=(1, s))[:, 0, 0, :]


class MambaTasNet(nn.Module):
    """Encoder / MaskNet / Decoder with compute_forward semantics (train_wsj0mix.py:86-111)."""

    def __init__(self, N=512, kernel_size=16, n_mamba=32, n_spk=2, d_state=16, expand=2, d_conv=4):
        super().__init__()
        self.num_spks = n_spk
        self.encoder = Encoder(kernel_size, N)
        self.masknet = MaskNet(N, N, n_spk, n_mamba, N, d_state, expand, d_conv)
        self.decoder = Decoder(N, 1, kernel_size, stride=kernel_size // 2, bias=False)

    def forward(self, mix):                            # (B, T) -> (B, T, n_spk)
        mix_w = self.encoder(mix)
        est_mask = self.masknet(mix_w)
        sep_h = mix_w.unsqueeze(0) * est_mask
        est = torch.stack([self.decoder(sep_h[i]) for i in range(self.num_spks)], dim=-1)
        T = mix.shape[1]
        if T > est.shape[1]:
            return F.pad(est, (0, 0, 0, T - est.shape[1]))
        return est[:, :T, :]


MAMBA_TASNET_SIZES = {"XS": dict(N=128, n_mamba=16), "S": dict(N=256, n_mamba=16),
                      "M": dict(N=256, n_mamba=32), "L": dict(N=512, n_mamba=32)}
