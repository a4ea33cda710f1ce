"""avse4 binaural AV enhancement baseline on MI355X (drop-in for baseline/avse4/model.py).

Same module tree / state_dict keys as the reference (AVSE4BaselineModule -> model
(avse4_separator) + visual_frontend), so its Lightning checkpoints load unchanged.  Citations are
relative to /root/reference/baseline/avse4:
  overlap_and_add :19-66 -> F.fold        Encoder :97-109 -> framing GEMM     Decoder :112-123
  TemporalConvNet :126-182                TemporalBlock :255-269              DepthwiseSeparableConv :272-293
  GlobalLayerNorm :225-252                VisualConv1D :184-205               VisualFrontend utils.py:97-118
  AVSE4BaselineModule :295-393 (forward :316-321, training_step :323, enhance :335-352, cal_loss :374-383)
MI355X specifics: every (PReLU -> gLN) pair runs as the fused HIP prelu_gln kernels, every
depthwise dilated conv1d as the HIP dwconv kernels, the lip Conv3d weight gradient on the HIP
MFMA implicit GEMM; every 1x1 Conv1d (forward, input and weight gradient) on the split-fp16 MFMA GEMM
(csrc/projgemm.hip avse_gemm_f32s, fp32-accurate); the encoder / decoder basis are hipBLASLt GEMMs.
"""
import copy

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K
from . import losses
from .layers import (LipConv3d, PointwiseConv2d, TrunkConv2d, _PReLUFn, bn_act, dwconv1d, dwconv_prelu_gln, frames_nhwc,
                     maxpool3d, prelu_gln)

NORM_MEAN, NORM_STD = 0.4161, 0.1688


def _pw_split_ok(w, x):
    return (x.is_cuda and x.dtype == w.dtype == torch.float32 and x.dim() == 3
            and (x.stride(2) == 1 or x.stride(1) == 1) and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0
            and w.stride(1) == 1)


def _padded_rows(sp):
    """The planes are in the zero-padded row layout (split_rows8, the gLN planes output): rows of a multiple of 8."""
    h = sp.hi
    return h.stride(2) == 1 and h.stride(1) % 8 == 0 and h.stride(0) == h.shape[1] * h.stride(1)


def _split_act(x):
    """The split planes of a (B, C, K) activation as a GEMM operand, in the zero-padded row layout (rows of a multiple
    of 8 elements): the planes its producer wrote (the gLN of DepthwiseSeparableConv, kernels.PLANES_ATTR), else
    split_rows8 (a channel-contiguous x — the ChannelWiseLayerNorm output — is made time-contiguous first)."""
    sp = K.planes_of(x)
    if sp is not None:
        return sp
    return K.split_rows8(x if x.stride(2) == 1 else x.contiguous())


class _PointwiseFn(torch.autograd.Function):
    """1x1 Conv1d without bias on the (B, C, K) layout, no layout copies (model.py:255-293, nn.Conv1d(cin, cout, 1)):
    y_b = W x_b;  dx_b = W^T dy_b;  dW = sum_b dy_b x_b^T.  fp32 operands: avse_gemm_f32s (split-fp16 planes, three
    f16 MFMAs per product, fp32 accumulation) with out[b, q, p] = sum_k P[b, p, k] Q[b, q, k]:
      y:  P = x^T (B, K, Cin) read along K, Q = W (1, Cout, Cin)
      dx: P = dy^T (B, K, Cout),            Q = W^T (1, Cin, Cout)
      dW: P = x (B, Cin, K), Q = dy (B, Cout, K), the B batches folded into one output
    x and dy are split once each (the planes' rows padded to a multiple of 8: K = 3999), x's planes are what the backward
    keeps.  Otherwise batched hipBLASLt GEMMs (torch.bmm)."""

    @staticmethod
    def forward(ctx, w, x, dy_planes=False):
        ctx.split = _pw_split_ok(w, x)
        ctx.dy_planes = dy_planes
        if dy_planes and not ctx.split:
            raise RuntimeError("_PointwiseFn: gradient planes requested without the split-fp16 GEMM path")
        if not ctx.split:
            ctx.save_for_backward(w, x)
            return torch.bmm(w.expand(x.shape[0], *w.shape), x)
        xs = _split_act(x)
        ws = K.split_planes(w[None])                        # kept for the input gradient (W^T: its transposed view)
        y = torch.empty(x.shape[0], w.shape[0], x.shape[2], device=x.device, dtype=torch.float32)
        K.gemm_f32s_split(xs.t(), ws, y)
        ctx.save_for_backward(w, xs.hi, xs.lo, xs.mb, ws.hi, ws.lo, ws.mb)
        return y

    @staticmethod
    def backward(ctx, dy):
        dw = dx = None
        if not ctx.split:
            w, x = ctx.saved_tensors
            if ctx.needs_input_grad[0]:
                dw = torch.bmm(dy, x.transpose(1, 2)).sum(0)
            if ctx.needs_input_grad[1]:
                dx = torch.bmm(w.t().expand(dy.shape[0], w.shape[1], w.shape[0]), dy)
            return dw, dx, None
        w, xh, xl, xm, wh, wl, wm = ctx.saved_tensors
        if ctx.dy_planes and K.planes_of(dy) is None:
            raise RuntimeError("_PointwiseFn: the output gradient arrived without its split planes (its consumer must "
                               "be the only one and write them: prelu_gln(planes_bwd=True))")
        dys = _split_act(dy)
        if ctx.needs_input_grad[0]:
            xs = K.Split(xh, xl, xm)
            if _padded_rows(xs) and _padded_rows(dys) and xh.stride(1) == dys.hi.stride(1):
                dw = K.gemm_f32s_time_chunks(xs, dys)       # the time axis shared out over the workgroups
            else:
                out = torch.empty(1, w.shape[0], w.shape[1], device=dy.device, dtype=torch.float32)
                dw = K.gemm_f32s_split(xs, dys, out, fold=dy.shape[0])[0]
        if ctx.needs_input_grad[1]:
            dx = torch.empty(dy.shape[0], w.shape[1], dy.shape[2], device=dy.device, dtype=torch.float32)
            K.gemm_f32s_split(dys.t(), K.Split(wh, wl, wm).t(), dx)
        return dw, dx, None


def _pw(conv, x, dy_planes=False):
    """1x1 Conv1d without bias: (Cout, Cin) @ (B, Cin, K).  dy_planes: the output's consumer hands back its gradient as
    split planes (prelu_gln(planes_bwd=True)); the backward raises if they are missing."""
    return _PointwiseFn.apply(conv.weight[:, :, 0], x, dy_planes)


_INTERP = {}


def _upsample_matrix(n_in, up, n_out, device):
    """(n_in, n_out) matrix M with v @ M == F.pad(F.interpolate(v, up * n_in, mode='linear'), (0, n_out - up*n_in)):
    align_corners=False source coordinate (j + 0.5) / up - 0.5 clamped at 0 (model.py:166-168).  Two non-zeros
    per column whose weights are multiples of 1/up, so the GEMM reproduces the interpolation exactly."""
    key = (n_in, up, n_out, device)
    if key not in _INTERP:
        m = torch.zeros(n_in, n_out, dtype=torch.float64)
        j = torch.arange(min(n_out, up * n_in), dtype=torch.float64)
        src = ((j + 0.5) / up - 0.5).clamp(min=0.0)
        i0 = src.floor().long()
        lam = src - i0
        i1 = (i0 + 1).clamp(max=n_in - 1)
        cols = j.long()
        m.index_put_((i0, cols), 1.0 - lam, accumulate=True)
        m.index_put_((i1, cols), lam, accumulate=True)
        _INTERP[key] = m.float().to(device)
    return _INTERP[key]


class GlobalLayerNorm(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(1, c, 1))
        self.beta = nn.Parameter(torch.zeros(1, c, 1))


class ChannelWiseLayerNorm(nn.LayerNorm):
    def forward(self, x):
        return super().forward(x.transpose(1, 2)).transpose(1, 2)


class DepthwiseSeparableConv(nn.Module):
    def __init__(self, cin, cout, k, stride, padding, dilation):
        super().__init__()
        assert stride == 1 and padding == (k - 1) * dilation // 2
        self.dilation = dilation
        self.net = nn.Sequential(nn.Conv1d(cin, cin, k, stride=stride, padding=padding, dilation=dilation,
                                           groups=cin, bias=False),
                                 nn.PReLU(), GlobalLayerNorm(cin), nn.Conv1d(cin, cout, 1, bias=False))

    def forward(self, x):
        dw, pr, nm, pw = self.net
        # fused passes (gln.hip); with the pointwise conv on the split-fp16 GEMM the gLN writes that GEMM's planes
        planes = _pw_split_ok(pw.weight[:, :, 0], x)
        y = dwconv_prelu_gln(x, dw.weight, pr.weight, nm.gamma, nm.beta, self.dilation, planes=planes)
        return _pw(pw, y)


class _ResidualAddFn(torch.autograd.Function):
    """y = a + b (TemporalBlock's residual, model.py:268) as one pass that also keeps max |y| (kernels.add_max_flat):
    the next block's first 1x1 conv splits y without an absmax pass."""

    @staticmethod
    def forward(ctx, a, b):
        return K.add_max_flat(a, b)

    @staticmethod
    def backward(ctx, g):
        return g, g


class TemporalBlock(nn.Module):
    def __init__(self, cin, cout, k, stride, padding, dilation):
        super().__init__()
        self.net = nn.Sequential(nn.Conv1d(cin, cout, 1, bias=False), nn.PReLU(), GlobalLayerNorm(cout),
                                 DepthwiseSeparableConv(cout, cin, k, stride, padding, dilation))

    def forward(self, x):
        c1, pr, nm, ds = self.net
        # with the 1x1 conv on the split-fp16 GEMM, the gLN backward writes that GEMM's dy planes (its only consumer)
        planes = _pw_split_ok(c1.weight[:, :, 0], x)
        y = prelu_gln(_pw(c1, x, dy_planes=planes), pr.weight, nm.gamma, nm.beta, planes_bwd=planes)
        out = ds(y)
        if planes and K.add_max_flat_ok(out, x):
            return _ResidualAddFn.apply(out, x)
        return out + x


class VisualConv1D(nn.Module):
    def __init__(self, c=512):
        super().__init__()
        self.net = nn.Sequential(nn.ReLU(), nn.BatchNorm1d(c),
                                 nn.Conv1d(c, c, 3, padding=1, groups=c, bias=False), nn.PReLU(),
                                 nn.BatchNorm1d(c), nn.Conv1d(c, c, 1, bias=False))

    def forward(self, x):
        _, bn1, dw, pr, bn2, pw = self.net
        y = dwconv1d(bn1(F.relu(x)), dw.weight, 1)
        y = bn2(_PReLUFn.apply(y, pr.weight))
        return _pw(pw, y) + x


class TemporalConvNet(nn.Module):
    def __init__(self, N, B, H, P, X, R, C, num_channels=2, vis_dim=512, up=32):
        super().__init__()
        self.num_channels, self.C, self.up = num_channels, C, up
        self.layer_norm = ChannelWiseLayerNorm(N)
        self.bottleneck_conv1x1 = nn.Conv1d(N, B, 1, bias=False)
        blocks = [nn.Conv1d(2 * B, B, 1, bias=False)]
        for x in range(X):
            d = 2 ** x
            blocks.append(TemporalBlock(B, H, P, 1, (P - 1) * d // 2, d))
        self.tcn = nn.ModuleList([copy.deepcopy(nn.Sequential(*blocks)) for _ in range(R)])
        self.visual_conv = nn.Sequential(*[VisualConv1D(vis_dim) for _ in range(5)])
        self.ve_conv1x1 = nn.ModuleList([copy.deepcopy(nn.Conv1d(vis_dim, B, 1, bias=False)) for _ in range(R)])
        self.mask_conv1x1 = nn.Conv1d(B, N * num_channels, 1, bias=False)

    def forward(self, x, visual):
        visual = self.visual_conv(visual.transpose(1, 2))
        x = _pw(self.bottleneck_conv1x1, self.layer_norm(x))
        bsz, Bc, K = x.shape
        for i in range(len(self.tcn)):
            v = _pw(self.ve_conv1x1[i], visual)
            v = torch.matmul(v, _upsample_matrix(v.shape[-1], self.up, K, v.device))   # interpolate x32 + pad
            seq = self.tcn[i]
            x = _pw(seq[0], torch.cat((x, v), 1))
            for blk in list(seq)[1:]:
                x = blk(x)
        x = F.relu(_pw(self.mask_conv1x1, x))
        return x.reshape(bsz, self.num_channels, Bc, K)


class Encoder(nn.Module):
    def __init__(self, L, N, num_channels=2):
        super().__init__()
        self.L = L
        self.conv1d_U = nn.Conv1d(num_channels, N, L, stride=L // 2, bias=False)

    def forward(self, m):                                   # (B, C, T) -> (B, N, K)
        frames = m.unfold(-1, self.L, self.L // 2)          # (B, C, K, L)
        Bn, C, K, L = frames.shape
        f = frames.permute(0, 2, 1, 3).reshape(Bn, K, C * L)
        return F.relu(torch.matmul(self.conv1d_U.weight.reshape(self.conv1d_U.weight.shape[0], -1), f.transpose(1, 2)))


class Decoder(nn.Module):
    def __init__(self, N, L):
        super().__init__()
        self.L = L
        self.basis_signals = nn.Linear(N, L, bias=False)

    def forward(self, mixture_w, est_mask):                  # -> (B, C, 20*(K-1)+40)
        est = mixture_w[:, None] * est_mask                  # (B, C, N, K)
        Bn, C, N, K = est.shape
        frames = torch.matmul(self.basis_signals.weight, est.reshape(Bn * C, N, K))     # (B*C, L, K)
        T = (K - 1) * (self.L // 2) + self.L
        out = F.fold(frames, (1, T), (1, self.L), stride=(1, self.L // 2))
        return out.reshape(Bn, C, T)


class Separator(nn.Module):
    """avse4_separator (model.py:73-94)."""

    def __init__(self, N=256, L=40, B=256, H=512, P=3, X=8, R=4, C=2, num_channels=2):
        super().__init__()
        self.encoder = Encoder(L, N, num_channels)
        self.separator = TemporalConvNet(N, B, H, P, X, R, C, num_channels)
        self.decoder = Decoder(N, L)
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_normal_(p)

    def forward(self, mixture, visual):
        w = self.encoder(mixture)
        est = self.decoder(w, self.separator(w, visual))
        return F.pad(est, (0, mixture.shape[-1] - est.shape[-1]))


class ResNetLayer(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        bn = dict(momentum=0.01, eps=0.001)
        # the reference's nn.Conv2d 3x3 / 1x1 (same parameters and keys): channels-last activations run the 3x3 convs
        # on csrc/sconv.hip and the strided 1x1 shortcut as one GEMM (layers.TrunkConv2d / PointwiseConv2d)
        self.conv1a = TrunkConv2d(cin, cout, stride)
        self.bn1a = nn.BatchNorm2d(cout, **bn)
        self.conv2a = TrunkConv2d(cout, cout, 1)
        self.stride = stride
        self.downsample = PointwiseConv2d(cin, cout, stride)
        self.outbna = nn.BatchNorm2d(cout, **bn)
        self.conv1b = TrunkConv2d(cout, cout, 1)
        self.bn1b = nn.BatchNorm2d(cout, **bn)
        self.conv2b = TrunkConv2d(cout, cout, 1)
        self.outbnb = nn.BatchNorm2d(cout, **bn)

    def forward(self, x):
        # BN -> ReLU pairs as fused passes (csrc/bnact.hip); the residual adds precede their BatchNorm here.  Where a
        # BatchNorm's output (input gradient) goes only to a split-fp16 trunk conv's forward (backward), it is written
        # in that conv's split layout (bn_act q_fwd / q_bwd)
        h = self.conv1a(x)
        y = self.conv2a(bn_act(h, self.bn1a, "relu", q_fwd=self.conv2a.q_ok(h), q_bwd=self.conv1a.q_ok(x, grad=True)))
        y = y + (x if self.stride == 1 else self.downsample(x))
        mid = y
        y = bn_act(y, self.outbna, "relu", q_fwd=self.conv1b.q_ok(y))
        h = self.conv1b(y)
        y = self.conv2b(bn_act(h, self.bn1b, "relu", q_fwd=self.conv2b.q_ok(h), q_bwd=self.conv1b.q_ok(y, grad=True)))
        return bn_act(y + mid, self.outbnb, "relu")


class ResNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.layer1 = ResNetLayer(64, 64, 1)
        self.layer2 = ResNetLayer(64, 128, 2)
        self.layer3 = ResNetLayer(128, 256, 2)
        self.layer4 = ResNetLayer(256, 512, 2)
        self.avgpool = nn.AvgPool2d(4, stride=1)

    def forward(self, x):
        return self.avgpool(self.layer4(self.layer3(self.layer2(self.layer1(x)))))


class VisualFrontend(nn.Module):
    def __init__(self):
        super().__init__()
        self.frontend3D = nn.Sequential(
            LipConv3d(1, 64, (5, 7, 7), (1, 2, 2), (2, 3, 3)), nn.BatchNorm3d(64, momentum=0.01, eps=0.001), nn.ReLU(),
            nn.MaxPool3d((1, 3, 3), stride=(1, 2, 2), padding=(0, 1, 1)))
        self.resnet = ResNet()
        self.channels_last = False

    def use_channels_last(self, on=True):
        """NHWC ResNet trunk: the frames enter as (B*T, H, W, C) memory (csrc/transpose.hip), the 3x3 convs run on
        csrc/sconv.hip, BatchNorm -> ReLU on bnact's channels-last view (the same kernels as the avse1 lip trunk)."""
        self.channels_last = on
        self.resnet.to(memory_format=torch.channels_last if on else torch.contiguous_format)
        return self

    def forward(self, x):                                   # (B, 1, T, 112, 112) -> (B, T, 512)
        bsz = x.shape[0]
        conv, bn, _, pool = self.frontend3D
        y = maxpool3d(bn_act(conv((x - NORM_MEAN) / NORM_STD), bn, "relu"), pool)
        if self.channels_last:
            y = frames_nhwc(y)
        else:
            y = y.transpose(1, 2)
            y = y.reshape(y.shape[0] * y.shape[1], y.shape[2], y.shape[3], y.shape[4])
        return self.resnet(y).reshape(bsz, -1, 512)


class AVSE4BaselineModule(nn.Module):
    """LightningModule surface of AVSE4BaselineModule (forward / training_step / enhance / cal_loss)."""

    def __init__(self, lr=0.0001, a_only=False, num_channels=2, **sep_kwargs):
        super().__init__()
        assert num_channels in [1, 2], "Only mono and binaural audio are supported"
        self.lr, self.a_only, self.num_channels = lr, a_only, num_channels
        self.model = Separator(num_channels=num_channels, **sep_kwargs)
        self.visual_frontend = VisualFrontend()

    def forward(self, data):
        return self.model(data["noisy_audio"].float(), self.visual_frontend(data["vis_feat"].float()))

    def cal_loss(self, batch):
        return losses.avse4_loss(batch["clean"], self(batch))

    def training_step(self, batch, batch_idx=0):
        return self.cal_loss(batch)

    def validation_step(self, batch, batch_idx=0):
        return self.cal_loss(batch)

    def configure_optimizers(self):
        return torch.optim.Adam(self.parameters(), lr=self.lr)

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location="cpu", strict=True, **kwargs):
        """test.py:32 `AVSE4BaselineModule.load_from_checkpoint(cfg.ckpt_path)` (Lightning .ckpt, ckpt_io)."""
        from .ckpt_io import load_lightning_checkpoint
        return load_lightning_checkpoint(cls, checkpoint_path, map_location, strict, **kwargs)

    @torch.no_grad()
    def enhance(self, data):
        """model.py:335-352: forward one utterance and peak-normalise (returns numpy arrays)."""
        dev = next(self.parameters()).device
        inputs = {"noisy_audio": torch.as_tensor(np.asarray(data["noisy_audio"]))[None].to(dev),
                  "vis_feat": torch.as_tensor(np.asarray(data["vis_feat"]))[None].to(dev)}
        est = self(inputs)[0].cpu().numpy()
        est /= np.max(np.abs(est))
        return np.asarray(data["clean"]), np.asarray(data["noisy_audio"]), est
