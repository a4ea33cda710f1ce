"""nn.Module drop-ins whose hot halves run in libavse_hip.so (same parameter names as torch's).

prelu_gln    fused PReLU -> GlobalLayerNorm (avse4 TCN) autograd op
dwconv1d     depthwise dilated "same" conv1d autograd op (avse4 VisualConv1D)
dwconv_prelu_gln  the avse4 TCN's dwconv -> PReLU -> gLN as two fused passes each way

PReLU        nn.PReLU(num_parameters): fwd + fused dx / slope-gradient bwd kernels (NCS and channels-last)
bn_act       act(nn.BatchNorm{1,2,3}d(x) [+ res]) with act None / ReLU / PReLU, two passes each way
maxpool3d    nn.MaxPool3d((1, k, k), (1, s, s), (0, p, p)) of the lip front-ends (byte argmax, gather backward)
HipLSTM      nn.LSTM(..., num_layers=1, batch_first=True[, bidirectional]) whose recurrence is one HIP launch
             per direction (avse1 FusionNet, avse2 DPRNN)
DilatedConv2d  nn.Conv2d(64, 64, 5, padding=2d, dilation=d) of the avse1 AudioFeatNet: weight gradient on the
             MFMA implicit-GEMM kernel (channels-last activations)
TrunkConv2d  nn.Conv2d(cin, cout, 3, stride, padding=1, bias=False) of the lip ResNet trunks: channels-last activations
             on the split-fp16 MFMA kernels (csrc/sconv.hip)
PointwiseConv2d  the 1x1 shortcut convs as one GEMM
LipConv3d    nn.Conv3d(Cin, 64, k, stride (1,2,2), pad, bias=False) of the lip front-ends:
             forward on MIOpen, weight gradient on the MFMA implicit-GEMM kernel (the lips are
             data: no input gradient is needed on the reference path; if one is requested it is
             computed with the library transposed conv).
"""

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K


class _PReLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, a):
        ctx.save_for_backward(x, a)
        return K.prelu_fwd(x, a)

    @staticmethod
    def backward(ctx, dy):
        x, a = ctx.saved_tensors
        dx, da = K.prelu_bwd(x, a, dy)
        return dx, da


class PReLU(nn.Module):
    def __init__(self, num_parameters=1, init=0.25):
        super().__init__()
        self.num_parameters = num_parameters
        self.weight = nn.Parameter(torch.full((num_parameters,), init))

    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("PReLU runs on the GPU kernels only")
        return _PReLUFn.apply(x, self.weight)


class _BNActFn(torch.autograd.Function):
    """act(BatchNorm(x) [+ res]) in two HBM passes forward and two backward (csrc/bnact.hip)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, alpha, res, running_mean, running_var, training, momentum, eps, act, q_fwd, q_bwd):
        if K._bn_view(x) is None:                  # neither contiguous nor channels-last: the layout the kernels read
            x = x.contiguous()
        y, stats = K.bnact_fwd(x, gamma, beta, running_mean, running_var, training, momentum, eps, act, alpha, res,
                               q_out=q_fwd)
        ctx.save_for_backward(x, res, stats, gamma, beta, alpha)
        ctx.act, ctx.training, ctx.q_bwd = act, training, q_bwd
        return y

    @staticmethod
    def backward(ctx, dy):
        x, res, stats, gamma, beta, alpha = ctx.saved_tensors
        dx, dres, dgamma, dbeta, dalpha = K.bnact_bwd(x, res, dy, stats, gamma, beta, ctx.act, alpha, ctx.training,
                                                      q_out=ctx.q_bwd)
        return (dx, dgamma if ctx.needs_input_grad[1] else None, dbeta if ctx.needs_input_grad[2] else None,
                dalpha if ctx.needs_input_grad[3] else None, dres, None, None, None, None, None, None, None, None)


def bn_act(x, bn, act=None, res=None, folded_bias=None, q_fwd=False, q_bwd=False):
    """act(bn(x) [+ res]) for an nn.BatchNorm{1,2,3}d `bn` (its parameters, buffers, momentum and eps; running
    statistics and num_batches_tracked updated in train mode as torch does).  act: None, "relu" or a PReLU module.
    x: fp32 contiguous or channels-last; the output keeps x's memory format.
    q_fwd / q_bwd (round 5): the output / the input gradient as a split-output tensor (kernels.SPLITQ_ATTR) -- ONLY
    when its sole consumer is a split-fp16 convolution: the next conv's forward (q_fwd; DilatedConv2d.q_ok /
    TrunkConv2d.q_ok) or the producing conv's backward (q_bwd; q_ok(..., grad=True)).  Ignored where the kernels
    cannot produce it (eval forward, residual, NCHW).
    folded_bias (training mode only): x is a convolution output whose per-channel bias was left out; the result is
    act(bn(x + bias)) — equal to act(bn(x)), the batch statistics shift with the bias — and the running mean takes
    the bias in (momentum * bias)."""
    if folded_bias is not None:
        if not (bn.training and bn.track_running_stats) or res is not None or bn.momentum is None:
            raise RuntimeError("bn_act: folded_bias needs a training-mode BatchNorm with running stats and a momentum "
                               "(not the cumulative average), no residual")
        y = bn_act(x, bn, act, q_fwd=q_fwd, q_bwd=q_bwd)
        # through .data, as the kernel's own running-stat update: no version bump (under DDP the BatchNorm buffers are
        # views of one flat tensor, and a bump would invalidate every library BatchNorm's saved running stats)
        bn.running_mean.data.add_(folded_bias.detach(), alpha=bn.momentum)
        return y
    if not x.is_cuda:
        raise RuntimeError("bn_act runs on the GPU kernels only")
    training = bn.training or not bn.track_running_stats
    if bn.training and bn.track_running_stats:
        if bn.momentum is None:
            raise NotImplementedError("bn_act: cumulative-average BatchNorm (momentum=None)")
        bn.num_batches_tracked.add_(1)
    if act is None:
        code, alpha = K.ACT_NONE, None
    elif act == "relu":
        code, alpha = K.ACT_RELU, None
    else:
        code, alpha = K.ACT_PRELU, act.weight
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    return _BNActFn.apply(x.float(), bn.weight, bn.bias, alpha, res, rm, rv, training,
                          bn.momentum if bn.momentum is not None else 0.0, bn.eps, code, bool(q_fwd), bool(q_bwd))


class _MaxPoolPlanesFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = K.maxpool_planes_fwd(x, k, s, p)
        ctx.save_for_backward(idx)
        ctx.cfg, ctx.in_shape = (k, s, p), x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        k, s, p = ctx.cfg
        return K.maxpool_planes_bwd(dy, idx, ctx.in_shape, k, s, p), None, None, None


def maxpool3d(x, pool):
    """nn.MaxPool3d `pool` with a (1, KH, KW) window, stride (1, SH, SW), padding (0, PH, PW) (the lip front-ends)
    on the HIP plane kernels (csrc/maxpool.hip); any other configuration raises."""
    k, s, p = (tuple(v) if isinstance(v, (tuple, list)) else (v,) * 3 for v in (pool.kernel_size, pool.stride,
                                                                                 pool.padding))
    d = pool.dilation if isinstance(pool.dilation, (tuple, list)) else (pool.dilation,) * 3
    if k[0] != 1 or s[0] != 1 or p[0] != 0 or tuple(d) != (1, 1, 1) or pool.ceil_mode or pool.return_indices:
        raise NotImplementedError(f"maxpool3d: only (1, KH, KW) windows, got {pool}")
    if not x.is_cuda:
        raise RuntimeError("maxpool3d runs on the GPU kernels only")
    return _MaxPoolPlanesFn.apply(x, k[1:], s[1:], p[1:])


def _conv3d_fwd_folded(x, w, padding):
    """Conv3d with time stride 1 as one Conv2d over frames: the KT time taps fold into the input channels
    (x_unf[b*T + t, ci*KT + kt] = x_pad[b, ci, t + kt], plane copies), the weight (Cout, Cin, KT, KH, KW) is then
    (Cout, Cin*KT, KH, KW) as it lies, and the (B*T, Cout, Ho, Wo) result is permuted back to (B, Cout, T, Ho, Wo).
    MIOpen runs this 2-D shape (Winograd f3x2, find-db record) in 7.1 ms against 8.6 ms for its 3-D path at the avse1
    C2 shape, copies included (tools/conv3d_fold_probe.py @ 8f1eec2)."""
    B, Cin, T, H, W = x.shape
    Co, _, KT, KH, KW = w.shape
    PT, PH, PW = padding
    xp = F.pad(x, (0, 0, 0, 0, PT, PT))
    Tn = T + 2 * PT - KT + 1
    xu = xp.unfold(2, KT, 1)                                   # (B, Cin, Tn, H, W, KT)
    xu = xu.permute(0, 2, 1, 5, 3, 4).reshape(B * Tn, Cin * KT, H, W)
    y = F.conv2d(xu, w.reshape(Co, Cin * KT, KH, KW), None, (2, 2), (PH, PW))
    return y.view(B, Tn, Co, y.shape[-2], y.shape[-1]).transpose(1, 2).contiguous()


class _LipConv3dFn(torch.autograd.Function):
    """The lip front-end Conv3d (baseline/avse1/model.py:29-34). x may be the uint8 frames as stored (the
    reference's `lip_images.float()`, model.py:122, happens inside the kernels: no fp32 copy of the clip)."""

    @staticmethod
    def forward(ctx, x, w, stride, padding):
        hip = x.is_cuda and K.conv3d_fwd_supported(x, w, stride, padding)
        if not hip and x.dtype != torch.float32:
            x = x.float()
        ctx.stride, ctx.padding = stride, padding
        ctx.xmax = None
        if hip:                           # split-fp16 MFMA implicit GEMM (csrc/conv3d_fwd.hip)
            y, xmax = K.conv3d_fwd(x, w, return_xmax=True)
            ctx.save_for_backward(x, w, xmax if xmax is not None else x.new_zeros(0, dtype=torch.int32))
            ctx.xmax = xmax is not None   # fp32 frames: the forward's max |x| scales the weight gradient's x split
            return y
        ctx.save_for_backward(x, w, x.new_zeros(0, dtype=torch.int32))
        # other shapes: the avse1 front-end as a Conv2d over frames (Cin = 3); the Cin = 1 front-ends of avse2 /
        # avse4 fold to a 5-channel Conv2d without a find-db record (a find pass over the avse4 step did not finish
        # in 400 s): they keep conv3d
        if tuple(stride) == (1, 2, 2) and x.shape[1] == 3:
            return _conv3d_fwd_folded(x, w, padding)
        return F.conv3d(x, w, None, stride, padding)

    @staticmethod
    def backward(ctx, dy):
        x, w, xmax = ctx.saved_tensors
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.nn.grad.conv3d_input(x.shape, w, dy, ctx.stride, ctx.padding)
        dw = None
        if ctx.needs_input_grad[1]:
            if dy.shape[-1] <= K.CONV3D_WGRAD_MAX_WO:
                dw = K.conv3d_wgrad(x, dy, tuple(w.shape[2:]), ctx.padding, xmax=xmax if ctx.xmax else None)
            else:   # wider frames (avse2's 224x224 lips -> 112 output columns): the library's GPU kernel
                dw = torch.nn.grad.conv3d_weight(x.float(), w.shape, dy, ctx.stride, ctx.padding)
        return dx, dw, None, None


class LipConv3d(nn.Conv3d):
    def __init__(self, cin, cout, kernel_size, stride=(1, 2, 2), padding=(2, 3, 3), bias=False):
        super().__init__(cin, cout, kernel_size, stride=stride, padding=padding, bias=bias)
        assert tuple(self.stride) == (1, 2, 2) and cout == 64 and not bias

    def forward(self, x):
        return _LipConv3dFn.apply(x, self.weight, tuple(self.stride), tuple(self.padding))


def _conv2d_dgrad(x, w, dy, stride, padding, dilation):
    """Input gradient of conv2d(x, w) in x's memory format.  torch.nn.grad.conv2d_input builds an NCHW input from
    the shape alone, so for channels-last activations MIOpen returned NCHW and the consumer copied it back (6 copies
    of (32, 64, 376, 257) per avse1 step, tools/avse1_op_profile.py --kernels direct_copy)."""
    pair = lambda v: [v, v] if isinstance(v, int) else list(v)                       # noqa: E731
    return torch.ops.aten.convolution_backward(dy, x, w, None, pair(stride), pair(padding), pair(dilation), False,
                                               [0, 0], 1, [True, False, False])[0]


# forward and input gradient of the 64 -> 64 dilated convs on csrc/dconv.hip (fp16x3 split-operand MFMA, fp32-accurate)
# where K.dconv_split_ok takes the shape; other shapes: MIOpen's fp32 convolutions + the exact-fp32 weight gradient


class _DilatedConvFn(torch.autograd.Function):
    """Conv2d(64, 64, 5, padding=2d, dilation=d): forward and input gradient on the split-fp16 MFMA implicit GEMM
    (csrc/dconv.hip) where it applies (W >= 256: the avse1 spectrogram's 257 bins), else MIOpen; the weight (and bias)
    gradient on the fp32 MFMA implicit GEMM (csrc/dconv_wgrad.hip).  add_bias=False leaves the bias out of the output
    (for a training-mode BatchNorm consumer, which removes it: see DilatedConv2d) but still returns its gradient."""

    @staticmethod
    def forward(ctx, x, w, b, dilation, add_bias):
        ctx.dilation = dilation
        ctx.split = K.dconv_split_ok(x, dilation)
        if K.is_split_q(x) and not ctx.split:
            raise RuntimeError("_DilatedConvFn: a split-output input needs the split path (DilatedConv2d.q_ok)")
        if ctx.split:
            # the fp16 hi / lo split of x is made once and kept for the weight gradient in place of x (same bytes)
            mb = torch.empty(2, device=x.device, dtype=torch.int32)
            xq = K.split16(x, mb)
            y = K.dconv_fwd(x, w, dilation, b if add_bias else None, split=(xq, mb))
            ctx.save_for_backward(xq, mb, w)
            ctx.shape = tuple(x.shape)
            return y
        ctx.save_for_backward(x, w)
        pad = 2 * dilation
        return F.conv2d(x, w, b if add_bias else None, 1, pad, dilation)

    @staticmethod
    def backward(ctx, dy):
        d = ctx.dilation
        dx = dw = db = None
        if ctx.split:
            xq, mb, w = ctx.saved_tensors
            mbd = torch.empty(2, device=dy.device, dtype=torch.int32)
            dyq = K.split16(dy, mbd)                   # shared by the input and the weight gradient
            if ctx.needs_input_grad[0]:
                dx = K.dconv_fwd(dy, w, d, transposed=True, split=(dyq, mbd))
            if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
                dw, db = K.dconv_wgrad16((xq, mb[:1]), (dyq, mbd[:1]), ctx.shape, d, bias_grad=True)
                dw = dw if ctx.needs_input_grad[1] else None
                db = db if ctx.needs_input_grad[2] else None
            return dx, dw, db, None, None
        x, w = ctx.saved_tensors
        if ctx.needs_input_grad[0]:
            dx = _conv2d_dgrad(x, w, dy, 1, 2 * d, d)
        if ctx.needs_input_grad[1] and ctx.needs_input_grad[2]:
            dw, db = K.dconv_wgrad(x, dy, d, bias_grad=True)
        elif ctx.needs_input_grad[1]:
            dw = K.dconv_wgrad(x, dy, d)
        elif ctx.needs_input_grad[2]:
            db = dy.sum((0, 2, 3))
        return dx, dw, db, None, None


class _FramesNHWC(torch.autograd.Function):
    """(B, C, T, H, W) contiguous -> (B*T, C, H, W) in channels-last memory (the frames of the lip front-end as the
    batch of the channels-last ResNet trunk, baseline/avse1/model.py:46-50), and the gradient back, as one batched
    64 x 64-tile transpose each way (csrc/transpose.hip) instead of torch's strided copies (~0.35 TB/s)."""

    @staticmethod
    def forward(ctx, x):
        B, C, T, H, W = x.shape
        ctx.shape = x.shape
        y = K.transpose_cp(x.contiguous().view(B, C, T * H * W))                  # (B, T*H*W, C)
        return y.view(B * T, H, W, C).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        B, C, T, H, W = ctx.shape
        d = dy.permute(0, 2, 3, 1).contiguous().view(B, T * H * W, C)           # a view for channels-last dy
        return K.transpose_cp(d).view(B, C, T, H, W)


def frames_nhwc(x):
    """(B, C, T, H, W) -> (B*T, C, H, W) channels-last; HIP transpose for fp32 GPU tensors, torch elsewhere."""
    B, C, T, H, W = x.shape
    if x.is_cuda and x.dtype == torch.float32:
        return _FramesNHWC.apply(x)
    return x.permute(0, 2, 3, 4, 1).reshape(B * T, H, W, C).permute(0, 3, 1, 2)


# AudioFeatNet.conv1 on csrc/conv1.hip (direct HBM-streaming kernels) for frames of >= 128 bins; narrower ones: the
# im2col GEMM form below


class _Conv1Fn(torch.autograd.Function):
    """AudioFeatNet.conv1 = Conv2d(1, 64, 5, padding=2) (model.py:199-215) as GEMMs over all B·T·F pixels, writing its
    output straight into channels-last memory.  MIOpen ran this single-input-channel conv in NCHW (for C = 1 the
    input is both NCHW- and NHWC-contiguous, and the library picks NCHW): its output and its incoming gradient were
    each copied between layouts (2 x 791 MB per step), the bias was a separate pass, and the input gradient took
    ~3.6 ms behind transposes.  Here: A = the (B·T·F, 26) im2col rows with a ones column (the bias); y = A @ [W^T; b]
    (K = 26); dW and db in ONE GEMM dy^T @ A; dx = col2im of (W^T @ dy^T) as 25 shifted adds of contiguous tap
    planes.  add_bias=False leaves b out of y (a training-mode BatchNorm consumer: DilatedConv2d) but returns db."""

    @staticmethod
    def _rows(x):
        n, _, h, w = x.shape
        xp = F.pad(x.reshape(n, h, w), (2, 2, 2, 2))                               # (n, h + 4, w + 4)
        hp, wp = h + 4, w + 4
        a = x.new_empty((n, h, w, 26))
        a[..., :25].view(n, h, w, 5, 5).copy_(xp.as_strided((n, h, w, 5, 5), (hp * wp, wp, 1, wp, 1)))
        a[..., 25] = 1.0
        return a.view(n * h * w, 26)

    @staticmethod
    def forward(ctx, x, w, b, add_bias):
        n, _, h, ww = x.shape
        ctx.hip = ww >= 128
        if ctx.hip:                                 # csrc/conv1.hip: direct kernels, x (not the im2col rows) kept
            ctx.save_for_backward(x, w)
            return K.conv1_fwd(x, w, b if add_bias else None)
        a = _Conv1Fn._rows(x)
        wb = torch.cat([w.reshape(w.shape[0], 25), (b if add_bias else torch.zeros_like(b)).reshape(-1, 1)], 1)
        y = a @ wb.t()                                                                # (n h w, 64): NHWC memory
        ctx.save_for_backward(a, w)
        ctx.shape = (n, h, ww)
        return y.view(n, h, ww, -1).permute(0, 3, 1, 2)                               # channels-last view

    @staticmethod
    def backward(ctx, dy):
        if ctx.hip:
            x, w = ctx.saved_tensors
            dx, dw, db = K.conv1_bwd(x, w, dy, ctx.needs_input_grad[0],
                                     ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
            return (dx, dw if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None, None)
        a, w = ctx.saved_tensors
        n, h, ww = ctx.shape
        cout = w.shape[0]
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)                                # a view for channels-last dy
        dx = dw = db = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            g = dy2.t() @ a                                                           # (64, 26): dW | db
            dw = g[:, :25].reshape(w.shape) if ctx.needs_input_grad[1] else None
            db = g[:, 25].contiguous() if ctx.needs_input_grad[2] else None
        if ctx.needs_input_grad[0]:
            gt = w.reshape(cout, 25).t() @ dy2.t()                                    # (25, n h w): tap planes
            gt = gt.view(5, 5, n, h, ww)
            dxp = dy2.new_zeros((n, h + 4, ww + 4))
            for i in range(5):
                for j in range(5):
                    dxp[:, i:i + h, j:j + ww] += gt[i, j]
            dx = dxp[:, 2:-2, 2:-2].reshape(n, 1, h, ww).contiguous()
        return dx, dw, db, None


# the 64 -> 64 dilated convs on the HIP kernels (DilatedConv2d.hip_ok); False: the library convolution with the bias in
# it (tests/test_gpu_kernels.py builds its comparison with it)
HIP_DCONV = True


class DilatedConv2d(nn.Conv2d):
    """nn.Conv2d(cin, cout, 5, padding=2*dilation, dilation) — the avse1 AudioFeatNet convs (same parameters and
    state_dict keys).  The 64 -> 64 ones on GPU tensors in channels-last memory (the benchmarked layout) take their
    weight and bias gradients from csrc/dconv_wgrad.hip; other inputs (the 1 -> 64 conv1, NCHW activations) run the
    library convolution unchanged.

    forward(x, bias_to_bn=True) on the HIP path returns the convolution WITHOUT the bias: the caller feeds it to a
    training-mode BatchNorm through bn_act(..., folded_bias=self.bias), which normalises z + b and z alike (batch
    mean and variance shift with b) and adds momentum * b to the running mean.  That saves the library's separate
    bias-add pass over the (B, 64, 376, 257) output (5 per avse1 step); the bias gradient is exact either way."""

    def __init__(self, cin, cout, kernel_size=5, padding=0, dilation=1):
        super().__init__(cin, cout, kernel_size, padding=padding, dilation=dilation)
        assert self.padding == (2 * self.dilation[0],) * 2 and self.kernel_size == (5, 5)

    nhwc_out = False          # set by AudioFeatNet.use_channels_last: conv1 (1 -> 64) writes channels-last output

    def conv1_ok(self, x):
        return (self.nhwc_out and x.is_cuda and self.in_channels == 1
                and self.dilation[0] == 1 and self.bias is not None and x.dtype == torch.float32 and x.is_contiguous())

    def hip_ok(self, x):
        if self.conv1_ok(x):
            return True
        # x.numel() < 2^29: the kernel's 32-bit buffer offsets (csrc/dconv_wgrad.hip; B >= ~87 at 3 s clips exceeds
        # it, and those shapes take the library path instead of failing in the backward)
        return (HIP_DCONV and x.is_cuda and self.in_channels == 64
                and self.out_channels == 64 and self.dilation[0] <= K.DCONV_WGRAD_MAX_DIL
                and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
                and x.numel() < (1 << 29))

    def q_ok(self, x, grad=False):
        """True when this conv's forward (or, grad=True, its backward) takes a split-output tensor for an input of x's
        shape and layout (the split-fp16 path of _DilatedConvFn)."""
        return (not self.conv1_ok(x)) and self.hip_ok(x) and K.dconv_split_ok(x, self.dilation[0])

    def forward(self, x, bias_to_bn=False):
        if self.conv1_ok(x):
            return _Conv1Fn.apply(x, self.weight, self.bias, not (bias_to_bn and self.bias is not None))
        if self.hip_ok(x):
            add_bias = not (bias_to_bn and self.bias is not None)
            return _DilatedConvFn.apply(x, self.weight, self.bias, self.dilation[0], add_bias)
        if bias_to_bn:
            raise RuntimeError("DilatedConv2d: bias_to_bn needs the HIP path (check hip_ok first)")
        return super().forward(x)


class _GemmConvFn(torch.autograd.Function):
    """Conv2d(cin, cout, k in {1, 3}, stride, padding (k - 1) / 2, bias=False) as ONE hipBLASLt GEMM over all frames'
    pixels: (N * HO * WO, cin * k * k) im2col rows times the (cout, cin * k * k) weight; backward = two GEMMs + col2im.
    For the lip trunks' small-spatial layers (<= 36 output pixels per frame) and 1x1 shortcut convs, where MIOpen's
    NCHW backward ran NHWC kernels behind batched transposes at ~32 TF/s or less (tools/avse1_op_profile.py)."""

    @staticmethod
    def _rows(x, k, stride):
        """(N * HO * WO, cin * k * k) im2col rows as ONE gather copy of a strided view of the zero-padded input
        (F.unfold launches one kernel per frame on this build: 38400 per step); for a 1x1 conv on channels-last memory
        at stride 1 the rows ARE the input (a view)."""
        n, cin, h, w = x.shape
        ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1
        if k == 1:
            xs = x[:, :, ::stride, ::stride]
            return xs.permute(0, 2, 3, 1).reshape(-1, cin), ho, wo
        xp = F.pad(x, (1, 1, 1, 1))
        hp, wp = h + 2, w + 2
        v = xp.as_strided((n, ho, wo, cin, 3, 3), (cin * hp * wp, stride * wp, stride, hp * wp, wp, 1))
        return v.reshape(-1, cin * 9), ho, wo

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, w, stride):
        k = w.shape[-1]
        a, ho, wo = _GemmConvFn._rows(x, k, stride)
        y = a @ w.reshape(w.shape[0], -1).t()                                     # (N * P, cout)
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.hw = stride, (ho, wo)
        y = y.view(x.shape[0], ho, wo, -1).permute(0, 3, 1, 2)                    # channels-last memory (a view)
        return y if x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous() else y.contiguous()

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")             # the forward's autocast state (bf16 C5 lip encoder)
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        s, (ho, wo) = ctx.stride, ctx.hw
        n, cin, h, ww = x.shape
        cout, k = w.shape[0], w.shape[-1]
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)                            # (N * P, cout)
        dx = dw = None
        if ctx.needs_input_grad[1]:
            a, _, _ = _GemmConvFn._rows(x, k, s)
            if _f32s_rows_ok(a, dy2):
                # split-fp16 MFMA GEMM with the N * P pixel reduction cut per frame group (hipBLASLt: 10-20 TF/s on
                # these 128 x 64 .. 512 x 256 outputs)
                dw = K.gemm_f32s_rows_tn(K.split_planes(a[None]), K.split_planes(dy2[None]), n).view_as(w)
            else:
                dw = (dy2.t() @ a).view_as(w)
        if ctx.needs_input_grad[0]:
            da = (dy2 @ w.reshape(cout, -1)).view(n, ho, wo, cin, k, k)           # im2col-row gradients
            if k == 1:
                dx = torch.zeros_like(x)                                          # x's memory format
                dx[:, :, ::s, ::s] = da[..., 0, 0].permute(0, 3, 1, 2)
            else:                                     # col2im: the 9 taps' strided adds into the padded gradient
                dxp = x.new_zeros((n, cin, h + 2, ww + 2))
                for kh in range(3):
                    for kw in range(3):
                        dxp[:, :, kh:kh + s * (ho - 1) + 1:s, kw:kw + s * (wo - 1) + 1:s] += da[..., kh, kw].permute(0, 3, 1, 2)
                dx = dxp[:, :, 1:-1, 1:-1].contiguous()
        return dx, dw, None


def gemm_conv_ok(x, k, stride):
    """The 1x1 shortcut convs (NCHW or channels-last fp32 GPU activations) run as one GEMM (_GemmConvFn).  The 3x3 form
    of _GemmConvFn (small frames as one im2col GEMM) measured slower in the avse1 step than the library (179.6 vs 199
    utt/s, profiles/r03_trunk_gemm_op_profile.txt) and then than csrc/sconv.hip: the product routes no 3x3 conv to it."""
    if k != 1 or not x.is_cuda or x.dtype != torch.float32:
        return False
    return x.is_contiguous() or x.is_contiguous(memory_format=torch.channels_last)


class _TimeConv1dFn(torch.autograd.Function):
    """Conv1d(C, C', k, dilation, padding=(k - 1) * dilation) with bias on TIME-MAJOR activations (B, T, C) ->
    (B, T + pad, C') as ONE GEMM: im2col rows [x(t + j d)]_{j < k} (B * T', k * C) built from k shifted slices of the
    zero-padded input, times the (C', k * C) weight re-laid [co][j][ci]; backward = two GEMMs + col2im (k shifted slice
    adds).  hipBLASLt GEMMs and slice copies only: bit-reproducible run to run (MIOpen's conv1d forward is not; its
    rounding-level jitter flipped PReLU signs in the avse1 TCN and moved the lip-branch gradients by up to 7e-3 between
    identical steps, profiles/r04a_avse1_stream_diag.txt)."""

    @staticmethod
    def forward(ctx, x, w, b, dil):
        B, T, C = x.shape
        Co, _, k = w.shape
        pad = (k - 1) * dil
        To = T + pad
        xp = F.pad(x, (0, 0, pad, pad))                                   # (B, T + 2 pad, C)
        cols = torch.cat([xp[:, j * dil:j * dil + To] for j in range(k)], dim=2).reshape(B * To, k * C)
        wm = w.permute(0, 2, 1).reshape(Co, k * C)
        y = torch.addmm(b, cols, wm.t()) if b is not None else cols @ wm.t()
        ctx.save_for_backward(cols, wm)
        ctx.shape = (B, T, C, k, dil, b is not None)
        return y.view(B, To, Co)

    @staticmethod
    def backward(ctx, dy):
        cols, wm = ctx.saved_tensors
        B, T, C, k, dil, has_b = ctx.shape
        pad = (k - 1) * dil
        To = T + pad
        Co = wm.shape[0]
        dy2 = dy.reshape(B * To, Co)
        if _f32s_rows_ok(cols, dy2):
            # both GEMMs on the split-fp16 MFMA GEMM (csrc/projgemm.hip): the weight gradient's reduction over B To rows
            # cut per utterance (hipBLASLt ran these 512 x 1536 outputs at 3-26 TF/s, tools/avse1_op_profile.py)
            sd = K.split_planes(dy2[None])                                          # shared by both GEMMs
            dw = K.gemm_f32s_rows_tn(K.split_planes(cols[None]), sd, B).view(Co, k, C).permute(0, 2, 1)
            dcols = K.gemm_f32s_split(K.split_planes(wm[None]).t(), sd,
                                      torch.empty((1, B * To, k * C), device=dy.device, dtype=torch.float32))
            dcols = dcols.view(B, To, k, C)
        else:
            dw = (dy2.t() @ cols).view(Co, k, C).permute(0, 2, 1)
            dcols = (dy2 @ wm).view(B, To, k, C)
        db = dy2.sum(0) if has_b else None
        dxp = torch.zeros((B, T + 2 * pad, C), device=dy.device, dtype=dy.dtype)
        for j in range(k):
            dxp[:, j * dil:j * dil + To] += dcols[:, :, j]
        return dxp[:, pad:pad + T], dw, db, None


class _ConvFFn(torch.autograd.Function):
    """AudioFeatNet.convf = Conv2d(64, 4, 1) on channels-last activations (csrc/convf.hip: HBM-streaming forward, input
    gradient and weight / bias gradient)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return K.convf_fwd(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        need_w = ctx.needs_input_grad[1] or (ctx.has_b and ctx.needs_input_grad[2])
        dx, dw, db = K.convf_bwd(x, w, dy, need_dx=ctx.needs_input_grad[0], need_dw=need_w)
        return dx, dw if ctx.needs_input_grad[1] else None, db if ctx.has_b and ctx.needs_input_grad[2] else None


def conv1x1_to4(x, conv):
    """nn.Conv2d(64, 4, 1) ``conv`` (AudioFeatNet.convf, baseline/avse1/model.py:211-213) on x: csrc/convf.hip for
    channels-last fp32 GPU activations, the module itself otherwise."""
    if (x.is_cuda and x.dtype == torch.float32 and conv.weight.dtype == torch.float32 and x.dim() == 4
            and x.shape[1] == 64 and tuple(conv.weight.shape) == (4, 64, 1, 1) and conv.stride == (1, 1)
            and conv.padding == (0, 0) and conv.groups == 1 and x.is_contiguous(memory_format=torch.channels_last)
            and x.data_ptr() % 16 == 0):
        return _ConvFFn.apply(x, conv.weight, conv.bias)
    return conv(x)


def _f32s_rows_ok(a, b):
    """Two (rows, c) fp32 GPU operands the split GEMM reads row-major (unit column stride, 16-B rows)."""
    return (a.is_cuda and a.dtype == b.dtype == torch.float32 and a.dim() == b.dim() == 2 and a.shape[0] == b.shape[0]
            and a.stride(1) == 1 and b.stride(1) == 1 and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0)


def time_conv1d(x, conv):
    """nn.Conv1d ``conv`` (padding (k - 1) * dilation, stride 1, groups 1) applied to TIME-MAJOR x (B, T, C):
    returns (B, T + pad, C') time-major (_TimeConv1dFn)."""
    assert conv.stride == (1,) and conv.groups == 1 and conv.padding == ((conv.kernel_size[0] - 1) * conv.dilation[0],)
    return _TimeConv1dFn.apply(x, conv.weight, conv.bias, conv.dilation[0])


def time_major_4d(x):
    """(B, T, C) contiguous -> the same memory as a (B, C, T, 1) channels-last 4-D view (what bn_act and the NHWC
    PReLU kernels read as (B * T, C) rows)."""
    B, T, C = x.shape
    return x.as_strided((B, C, T, 1), (T * C, 1, C, C))


class PointwiseConv2d(nn.Conv2d):
    """nn.Conv2d(cin, cout, 1, stride, bias=False) — the ResNet shortcut (utils/resnet.py:86-95 downsample): one GEMM
    (same parameters and state_dict keys)."""

    def __init__(self, cin, cout, stride=1):
        super().__init__(cin, cout, 1, stride=stride, bias=False)

    def forward(self, x):
        if gemm_conv_ok(x, 1, self.stride[0]):
            return _GemmConvFn.apply(x, self.weight, self.stride[0])
        return super().forward(x)


# 3x3 trunk convs on csrc/sconv.hip (split-fp16 MFMA, fp32-accurate) for channels-last activations


class _SConvFn(torch.autograd.Function):
    """Conv2d(ci, co, 3, stride, padding=1, bias=False) on csrc/sconv.hip: forward, weight gradient and the input
    gradient (stride 1: the flipped-weight forward; stride 2: the 4 parity phases, avse_sconv_dgrad2) as split-fp16
    MFMA implicit GEMMs, no library convolution.  The input's split is made once and kept for the weight gradient in
    place of the input (same bytes); the output gradient is split once for both of its GEMMs."""

    @staticmethod
    def forward(ctx, x, w, stride):
        xq, xm = K.split_q(x)                      # the producing BatchNorm pass's max when it comes with x
        ctx.shape, ctx.stride = tuple(x.shape), stride
        ctx.save_for_backward(xq, xm, w)
        return K.sconv_fwd((xq, xm), ctx.shape, w, stride)

    @staticmethod
    def backward(ctx, dy):
        xq, xm, w = ctx.saved_tensors
        s, shape = ctx.stride, ctx.shape
        dyq, dym = K.split_q(dy)                   # (the incoming gradient keeps its producer's max, if any)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if s == 1:
                dx = K.sconv_fwd((dyq, dym), tuple(dy.shape), w, 1, transposed=True)
            else:
                dx = K.sconv_dgrad2((dyq, dym), shape, w)
        if ctx.needs_input_grad[1]:
            dw = K.sconv_wgrad((xq, xm), (dyq, dym), shape, w.shape[0], s)
        return dx, dw, None


class TrunkConv2d(nn.Conv2d):
    """nn.Conv2d(cin, cout, 3, stride, padding=1, bias=False) of the lip-encoder ResNet trunks (same parameters and
    state_dict keys).  Channels-last fp32 GPU activations with channel counts that are multiples of 64 run on
    csrc/sconv.hip (_SConvFn); other layouts and shapes (NCHW trunks, avse2's Swish trunk) run the library convolution."""

    def __init__(self, cin, cout, stride=1):
        super().__init__(cin, cout, 3, stride=stride, padding=1, bias=False)

    def _sconv(self, x):
        return (x.is_contiguous(memory_format=torch.channels_last) and x.dtype == self.weight.dtype
                and K.sconv_ok(x, self.out_channels, self.stride[0])
                and (self.stride[0] == 1 or K.sconv_dgrad2_ok(tuple(x.shape), self.out_channels)))

    def q_ok(self, x, grad=False):
        """True when this conv's forward (grad=True: its backward, given its input x) takes a split-output tensor:
        the sconv path (both input-gradient forms read the output gradient's split)."""
        return self._sconv(x)

    def forward(self, x):
        if self._sconv(x):
            return _SConvFn.apply(x, self.weight, self.stride[0])
        return super().forward(x)


class _PReluGLNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, alpha, gamma, beta, eps, planes_bwd=False):
        y, stats = K.prelu_gln_fwd(x, alpha, gamma.reshape(-1), beta.reshape(-1), eps)
        ctx.save_for_backward(x, alpha, gamma, stats)
        ctx.planes_bwd = planes_bwd
        return y

    @staticmethod
    def backward(ctx, dy):
        x, alpha, gamma, stats = ctx.saved_tensors
        dx, da, dg, db = K.prelu_gln_bwd(x, alpha, gamma.reshape(-1), stats, dy, planes=ctx.planes_bwd)
        return dx, da.view_as(alpha), dg.view_as(gamma), db.view_as(gamma), None, None


def prelu_gln(x, alpha, gamma, beta, eps=1e-8, planes_bwd=False):
    """GlobalLayerNorm(PReLU(x)) for (B, C, K) fp32 GPU tensors (one PReLU slope).  planes_bwd: the input gradient is
    written only as the split-fp16 planes of the 1x1 Conv1d GEMM that produced x (kernels.PLANES_ATTR), which must
    then be x's only consumer (avse4.TemporalBlock)."""
    if not x.is_cuda:
        raise RuntimeError("prelu_gln runs on the GPU kernels only")
    return _PReluGLNFn.apply(x, alpha, gamma, beta, eps, planes_bwd)


class _DWConvGLNFn(torch.autograd.Function):
    """gLN(PReLU(dwconv(x))) as the two fused passes of csrc/gln.hip (avse_dwconv_gln_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, x, w, alpha, gamma, beta, dilation, eps, planes=False):
        y, y1, stats = K.dwconv_gln_fwd(x, w, dilation, alpha, gamma.reshape(-1), beta.reshape(-1), eps, planes)
        ctx.save_for_backward(x, w, y1, alpha, gamma, stats)
        ctx.dilation = dilation
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y1, alpha, gamma, stats = ctx.saved_tensors
        dx, dw, da, dg, db = K.dwconv_gln_bwd(x, w, ctx.dilation, y1, alpha, gamma.reshape(-1), stats, dy)
        return dx, dw, da.view_as(alpha), dg.view_as(gamma), db.view_as(gamma), None, None, None


def dwconv_prelu_gln(x, w, alpha, gamma, beta, dilation, eps=1e-8, planes=False):
    """GlobalLayerNorm(PReLU(depthwise dilated 'same' conv1d(x))) for (B, C, K) fp32 GPU tensors (fused passes).
    planes: the output is only the split-fp16 planes of the 1x1 Conv1d GEMM that consumes it (kernels.PLANES_ATTR)."""
    if not x.is_cuda:
        raise RuntimeError("dwconv_prelu_gln runs on the GPU kernels only")
    return _DWConvGLNFn.apply(x, w, alpha, gamma, beta, dilation, eps, planes)


class _DWConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, dilation):
        ctx.save_for_backward(x, w)
        ctx.dilation = dilation
        return K.dwconv_fwd(x, w, dilation)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx, dw = K.dwconv_bwd(x, w, dy, ctx.dilation)
        return dx, dw, None


def dwconv1d(x, w, dilation):
    """Depthwise 'same' conv1d: w (C, 1, P), padding (P-1)/2*dilation, no bias."""
    if not x.is_cuda:
        raise RuntimeError("dwconv1d runs on the GPU kernels only")
    return _DWConvFn.apply(x, w, dilation)


class _LSTMDirFn(torch.autograd.Function):
    """One direction of a single-layer LSTM: input projection as one GEMM, the recurrence in libavse_hip.so
    (avse_lstm_fwd / _bwd), the weight / input gradients as GEMMs over all steps."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh, reverse):
        Bn, T, I = x.shape
        H = w_hh.shape[1]
        x2 = x.reshape(Bn * T, I)
        gx = torch.addmm(b_ih + b_hh, x2, w_ih.t()).view(Bn, T, 4 * H)
        h, c, gates = K.lstm_fwd(gx, w_hh, reverse=reverse)
        ctx.save_for_backward(x, w_ih, w_hh, h, c, gates)
        ctx.reverse = reverse
        c_n = (c[:, 0] if reverse else c[:, -1]).clone()        # final cell state in the direction's time order
        ctx.mark_non_differentiable(c_n)
        return h, c_n

    @staticmethod
    def backward(ctx, dh, _dc_n):
        x, w_ih, w_hh, h, c, gates = ctx.saved_tensors
        Bn, T, I = x.shape
        H = w_hh.shape[1]
        dg = K.lstm_bwd(dh, gates, c, w_hh, reverse=ctx.reverse).view(Bn * T, 4 * H)
        dx = (dg @ w_ih).view(Bn, T, I)
        dw_ih = dg.t() @ x.reshape(Bn * T, I)
        hprev = torch.zeros_like(h)                     # h_{t-1} in the direction's own time order (h_0 = 0)
        if ctx.reverse:
            hprev[:, :-1] = h[:, 1:]
        else:
            hprev[:, 1:] = h[:, :-1]
        dw_hh = dg.t() @ hprev.view(Bn * T, H)
        db = dg.sum(0)
        return dx, dw_ih, dw_hh, db, db, None


class HipLSTM(nn.LSTM):
    """nn.LSTM(input, hidden, num_layers=1, batch_first=True[, bidirectional]) with the same parameters and
    state_dict keys (weight_ih_l0, weight_hh_l0, bias_ih_l0, bias_hh_l0, ..._reverse) whose recurrence runs as ONE
    HIP launch per direction (csrc/lstm.hip) instead of a library kernel + GEMM per time step; capturable in a
    HIP graph.  Zero initial state (the reference never passes one)."""

    def __init__(self, input_size, hidden_size, num_layers=1, bias=True, batch_first=True, dropout=0.0,
                 bidirectional=False):
        if num_layers != 1 or not bias or not batch_first:
            raise NotImplementedError("HipLSTM: single layer, with bias, batch_first (the reference's LSTMs)")
        super().__init__(input_size, hidden_size, num_layers, bias, batch_first, dropout, bidirectional)

    def forward(self, x, hx=None):
        if hx is not None:
            raise NotImplementedError("HipLSTM starts from a zero state (as every reference call does)")
        if not x.is_cuda:
            raise RuntimeError("HipLSTM runs on the GPU kernels only")
        x = x.float()
        dirs = [_LSTMDirFn.apply(x, self.weight_ih_l0, self.weight_hh_l0, self.bias_ih_l0, self.bias_hh_l0, False)]
        if self.bidirectional:
            dirs.append(_LSTMDirFn.apply(x, self.weight_ih_l0_reverse, self.weight_hh_l0_reverse,
                                         self.bias_ih_l0_reverse, self.bias_hh_l0_reverse, True))
        outs = [h for h, _ in dirs]
        out = outs[0] if len(outs) == 1 else torch.cat(outs, dim=-1)
        # nn.LSTM's (h_n, c_n): (num_directions, B, H), forward direction's last step, reverse direction's first;
        # h_n carries gradients, c_n does not (no reference caller reads either: model.py:94, avse2 dnn.py)
        h_n = torch.stack([outs[0][:, -1]] + ([outs[1][:, 0]] if len(outs) > 1 else []))
        c_n = torch.stack([c for _, c in dirs])
        return out, (h_n, c_n)
