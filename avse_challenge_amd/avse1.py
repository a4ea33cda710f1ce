"""avse1 AV speech-enhancement baseline on MI355X (drop-in for baseline/avse1/model.py:AVNet).

Module tree and state_dict keys are identical to the reference (Lightning checkpoints load with
``load_lightning_state_dict``).  Surface mirrored from baseline/avse1/model.py:
  forward(dict{noisy_audio_spec, lip_images}) :114-128, training_step :130-133, cal_loss :164-168,
  configure_optimizers :170-178 (Adam; the plateau scheduler is the harness's business).
MI355X specifics:
  * the STFT front-end that the reference runs on CPU in its DataLoader
    (dataset.py:112-118, librosa) and the iSTFT of test.py:85-88 run as HIP kernels
    (libavse_hip.so: framing + radix-4 FFT-512 per wave) — ``features_from_waves`` / ``enhance``;
  * the lip front-end Conv3d weight gradient runs on the HIP MFMA implicit-GEMM kernel and every
    PReLU on the HIP fwd / fused-bwd kernels (layers.py);
  * the FusionNet LSTM recurrence runs as one HIP launch per direction and pass (layers.HipLSTM, csrc/lstm.hip)
    instead of a library kernel + GEMM per time step, so the whole step is capturable in a HIP graph;
  * the remaining convolutions / BatchNorm / GEMMs are MIOpen / hipBLASLt MFMA kernels (fp32,
    exact f32 MFMA on gfx950 — no TF32 shortcut exists), channels-first like the reference.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K
from .layers import (DilatedConv2d, HipLSTM, LipConv3d, PointwiseConv2d, PReLU, TrunkConv2d, bn_act, conv1x1_to4,
                     frames_nhwc, maxpool3d, time_conv1d, time_major_4d)

STFT_BINS, NUM_STFT_FRAMES, NUM_FRAMES, SAMPLES = 257, 376, 75, 48000


def _prelu(c):
    return PReLU(c)          # HIP fwd + fused dx / slope-gradient bwd (layers.py)


class _BasicBlock(nn.Module):            # utils/resnet.py:26-67 (relu_type='prelu')
    def __init__(self, cin, cout, stride=1, downsample=None):
        super().__init__()
        self.conv1 = TrunkConv2d(cin, cout, stride)      # csrc/sconv.hip on the channels-last trunk
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu1, self.relu2 = _prelu(cout), _prelu(cout)
        self.conv2 = TrunkConv2d(cout, cout, 1)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = downsample

    def forward(self, x):
        # BN -> PReLU and BN -> (+ shortcut) -> PReLU as fused passes (csrc/bnact.hip); bn1's output and input gradient
        # go straight to the split-fp16 trunk convs in their split layout where those take them (bn_act q_fwd / q_bwd)
        h = self.conv1(x)
        y = self.conv2(bn_act(h, self.bn1, self.relu1, q_fwd=self.conv2.q_ok(h), q_bwd=self.conv1.q_ok(x, grad=True)))
        if self.downsample is None:
            sc = x
        else:
            ds_conv, ds_bn = self.downsample
            sc = bn_act(ds_conv(x), ds_bn)
        return bn_act(y, self.bn2, self.relu2, res=sc)


class _ResNet18(nn.Module):              # utils/resnet.py:70-124
    def __init__(self):
        super().__init__()
        chans, cin = (64, 128, 256, 512), 64
        for i, c in enumerate(chans):
            s = 1 if i == 0 else 2
            ds = None if (s == 1 and cin == c) else nn.Sequential(PointwiseConv2d(cin, c, s), nn.BatchNorm2d(c))
            setattr(self, f"layer{i + 1}", nn.Sequential(_BasicBlock(cin, c, s, ds), _BasicBlock(c, c)))
            cin = c
        self.avgpool = nn.AdaptiveAvgPool2d(1)

    def forward(self, x):
        for i in range(1, 5):
            x = getattr(self, f"layer{i}")(x)
        return self.avgpool(x).flatten(1)


class _Chomp(nn.Module):
    def __init__(self, n):
        super().__init__()
        self.n = n

    def forward(self, x):
        return x[:, :, self.n // 2: x.shape[-1] - self.n // 2]


class _TemporalBlock(nn.Module):          # utils/tcn.py:144-243 (dwpw=False, symm_chomp=True)
    """net = conv1 -> batchnorm1 -> chomp1 -> relu1 (PReLU) -> dropout1 -> conv2 -> ... -> dropout2; out = relu(net(x) + x)
    (same modules and state_dict keys).  Runs TIME-MAJOR (B, T, C): each Conv1d as one GEMM over im2col rows
    (layers._TimeConv1dFn, bit-reproducible), BatchNorm1d -> PReLU as ONE bnact pass over the conv's whole (T + pad)
    output (BatchNorm statistics over the unchomped output, as the reference; the PReLU is elementwise, so applying it
    before the symmetric chomp is the same), the chomp a slice, the final add + PReLU on the NHWC kernels."""

    def __init__(self, c, k, dil, p_drop):
        super().__init__()
        pad = (k - 1) * dil
        self.conv1 = nn.Conv1d(c, c, k, padding=pad, dilation=dil)
        self.batchnorm1 = nn.BatchNorm1d(c)
        self.chomp1 = _Chomp(pad)
        self.relu1 = _prelu(c)
        self.dropout1 = nn.Dropout(p_drop)
        self.conv2 = nn.Conv1d(c, c, k, padding=pad, dilation=dil)
        self.batchnorm2 = nn.BatchNorm1d(c)
        self.chomp2 = _Chomp(pad)
        self.relu2 = _prelu(c)
        self.dropout2 = nn.Dropout(p_drop)
        self.net = nn.Sequential(self.conv1, self.batchnorm1, self.chomp1, self.relu1, self.dropout1,
                                 self.conv2, self.batchnorm2, self.chomp2, self.relu2, self.dropout2)
        self.downsample = None
        self.relu = _prelu(c)
        self.pad = pad

    def _half(self, x, conv, bn, act, drop):
        y = time_conv1d(x, conv)                                          # (B, T + pad, C)
        y = bn_act(time_major_4d(y), bn, act)                             # BatchNorm1d -> PReLU, same memory layout
        h = self.pad // 2
        y = y.squeeze(3).transpose(1, 2)[:, h:y.shape[2] - h]             # (B, T, C) view: symmetric chomp
        return drop(y)

    def forward(self, x):                 # x: (B, T, C) time-major
        y = self._half(x, self.conv1, self.batchnorm1, self.relu1, self.dropout1)
        y = self._half(y, self.conv2, self.batchnorm2, self.relu2, self.dropout2)
        z = (y + x).contiguous()
        return self.relu(time_major_4d(z)).squeeze(3).transpose(1, 2)


class _TCNTrunk(nn.Module):
    def __init__(self, c=512, levels=4, k=3, p_drop=0.2):
        super().__init__()
        self.network = nn.Sequential(*[_TemporalBlock(c, k, 2 ** i, p_drop) for i in range(levels)])

    def forward(self, x):
        return self.network(x)


class _TCN(nn.Module):                    # utils/nn.py:106-128 (extract_feats=True)
    def __init__(self):
        super().__init__()
        self.tcn_trunk = _TCNTrunk()
        self.tcn_output = nn.Linear(512, 500)   # present in checkpoints, unused on the feature path

    def forward(self, x):                 # (B, T, 512) -> (B, T, 512); the reference's (B, 512, T) transposes are not made
        return self.tcn_trunk(x.contiguous())


class VisualFeatNet(nn.Module):           # model.py:17-58
    def __init__(self):
        super().__init__()
        self.trunk = _ResNet18()
        self.frontend3D = nn.Sequential(
            LipConv3d(3, 64, (5, 7, 7), (1, 2, 2), (2, 3, 3)), nn.BatchNorm3d(64), _prelu(64),
            nn.MaxPool3d((1, 3, 3), (1, 2, 2), (0, 1, 1)))
        self.tcn = _TCN()
        self.channels_last = False

    def use_channels_last(self, on=True):
        """NHWC ResNet trunk: MIOpen's NHWC implicit-GEMM convolutions without the batched transposes
        around each NCHW call, NHWC BatchNorm, and the channels-last PReLU kernels (avse_prelu_nhwc_*)."""
        self.channels_last = on
        self.trunk.to(memory_format=torch.channels_last if on else torch.contiguous_format)
        return self

    def forward(self, lips):              # (B, 3, T, H, W) raw 0..255 (uint8 as stored, or float) -> (B, T, 512)
        Bn = lips.shape[0]
        conv, bn, act, pool = self.frontend3D
        x = maxpool3d(bn_act(conv(lips), bn, act), pool)
        Tn, C, H, W = x.shape[2], x.shape[1], x.shape[3], x.shape[4]
        if self.channels_last:            # (B, C, T, H, W) -> (B*T, H, W, C) in memory, viewed as NCHW
            x = frames_nhwc(x)
        else:
            x = x.transpose(1, 2).reshape(Bn * Tn, C, H, W)
        x = self.trunk(x).view(Bn, Tn, -1)
        return self.tcn(x)


class AudioFeatNet(nn.Module):            # model.py:181-267 (5 dilated 5x5 convs + 1x1 -> 4)
    def __init__(self, num_conv=5, k=5, filters=64, last_filter=4):
        super().__init__()
        self.num_conv, self.last_filter = num_conv, last_filter
        self.bn0 = nn.BatchNorm2d(1)
        for i in range(num_conv):
            dil = 2 ** i
            setattr(self, f"conv{i + 1}", DilatedConv2d(1 if i == 0 else filters, filters, k, padding=(k - 1) * dil // 2,
                                                        dilation=dil))
            setattr(self, f"bn{i + 1}", nn.BatchNorm2d(filters))
        self.convf = nn.Conv2d(filters, last_filter, 1)
        self.bn_last = nn.BatchNorm2d(last_filter)
        self.channels_last = False

    def use_channels_last(self, on=True):
        """NHWC activations/weights: MIOpen's implicit-GEMM convs are NHWC kernels, so NCHW tensors
        pay a transpose in and out of every conv (needs PYTORCH_MIOPEN_SUGGEST_NHWC=1)."""
        self.channels_last = on
        self.to(memory_format=torch.channels_last if on else torch.contiguous_format)
        self.conv1.nhwc_out = on          # the 1 -> 64 conv as GEMMs into channels-last memory (layers._Conv1Fn)
        return self

    def forward(self, spec):              # (B, 1, T, F) -> (B, T, 4F)
        T, Fb = spec.shape[2], spec.shape[3]
        x = bn_act(spec, self.bn0)
        if self.channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
        for i in range(1, self.num_conv + 1):
            conv, bn = getattr(self, f"conv{i}"), getattr(self, f"bn{i}")
            nxt = getattr(self, f"conv{i + 1}") if i < self.num_conv else None
            if bn.training and bn.track_running_stats and bn.momentum is not None and conv.bias is not None \
                    and conv.hip_ok(x):
                # the conv bias goes into the BatchNorm (no separate bias-add pass): DilatedConv2d docstring
                y = conv(x, bias_to_bn=True)
                # BN -> ReLU writes its output (input gradient) in the split layout when the next (this) conv is a
                # split-fp16 kernel: no separate split pass over the (B, 64, T, F) tensor (bn_act q_fwd / q_bwd)
                x = bn_act(y, bn, "relu", folded_bias=conv.bias, q_fwd=nxt is not None and nxt.q_ok(y),
                           q_bwd=conv.q_ok(x, grad=True))
            else:
                x = bn_act(conv(x), bn, "relu")
        x = bn_act(conv1x1_to4(x, self.convf), self.bn_last, "relu")     # csrc/convf.hip (HBM-streaming 1x1)
        return x.permute(0, 2, 1, 3).reshape(-1, T, Fb * self.last_filter)


class FusionNet(nn.Module):               # model.py:81-96
    def __init__(self, a_only=False):
        super().__init__()
        # HIP recurrence (csrc/lstm.hip), nn.LSTM parameters / keys
        self.lstm_conv = HipLSTM((0 if a_only else 512) + 4 * STFT_BINS, STFT_BINS, num_layers=1, batch_first=True)
        self.time_distributed_1 = nn.Linear(STFT_BINS, STFT_BINS)

    def forward(self, x):
        return torch.sigmoid(self.time_distributed_1(self.lstm_conv(x)[0]))


_STREAMS = {}
# the lip branch on a second HIP stream (default); set_branch_streams(False) runs both branches on the current stream
BRANCH_STREAMS = True


def set_branch_streams(on):
    """Run the lip branch on a second HIP stream, concurrent with the audio branch (True, the default), or both
    branches on the current stream; returns the previous setting."""
    global BRANCH_STREAMS
    old, BRANCH_STREAMS = BRANCH_STREAMS, bool(on)
    return old


def _branch_stream(device):
    """Second HIP stream for the lip branch, one per device (BRANCH_STREAMS)."""
    if device.type != "cuda" or not BRANCH_STREAMS:
        return None
    if device not in _STREAMS:
        _STREAMS[device] = torch.cuda.Stream(device)
    return _STREAMS[device]


class _JoinFromSide(torch.autograd.Function):
    """Identity at the point where the lip branch (side stream) joins the main stream (model.py:124-126's concat).
    Backward (on the main stream, where the join ran): the gradient it hands to the lip branch's backward was
    allocated on the main stream; the side stream reads it, so it is recorded on the side stream (the caching
    allocator then keeps its block until the side stream's reads have completed) and the side stream is ordered
    after the main stream's production of it."""

    @staticmethod
    def forward(ctx, x, side):
        ctx.side = side
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        side = ctx.side
        main = torch.cuda.current_stream(g.device)
        if side is not None and side != main:
            side.wait_stream(main)
            g.record_stream(side)
        return g, None


class AVNet(nn.Module):
    """LightningModule surface of baseline/avse1/model.py:AVNet (forward / training_step / cal_loss)."""

    def __init__(self, a_only=False, loss="l1", lr=0.00158):
        super().__init__()
        self.a_only = a_only
        self.net_visualfeat = None if a_only else VisualFeatNet()
        self.net_audiofeat = AudioFeatNet()
        self.net_fusion = FusionNet(a_only)
        if loss.lower() == "l1":
            self.loss = F.l1_loss
        elif loss.lower() == "l2":
            self.loss = F.mse_loss
        else:
            raise NotImplementedError(f"{loss} is currently unavailable as loss function. Select one of l1, l2")
        self.lr = lr

    def forward(self, inp):
        spec = inp["noisy_audio_spec"]
        T = spec.shape[2]
        side = None if self.a_only else _branch_stream(spec.device)
        if side is not None:
            # the lip and audio branches are independent until the concatenation: the lip ResNet/TCN runs on a
            # second HIP stream (its backward too, via autograd), so each branch's small kernels (BatchNorm,
            # PReLU, transposes) fill the CUs the other leaves idle; both forks are captured in the step's graphs
            main = torch.cuda.current_stream(spec.device)
            side.wait_stream(main)
            lips = inp["lip_images"]
            with torch.cuda.stream(side):
                vis = self.net_visualfeat(lips)          # (B, 75, 512); lips.float() of model.py:122 in the conv
            lips.record_stream(side)
        audio = self.net_audiofeat(spec)
        if side is not None:
            main.wait_stream(side)
            vis.record_stream(main)
            vis = _JoinFromSide.apply(vis, side)
        if self.a_only:
            comb = audio
        else:
            if side is None:
                vis = self.net_visualfeat(inp["lip_images"])                  # (B, 75, 512)
            # F.interpolate(nearest, size=(T, 512)) on (B, 1, 75, 512) == gather of rows floor(t*75/T)
            idx = torch.div(torch.arange(T, device=spec.device) * vis.shape[1], T, rounding_mode="floor")
            comb = torch.cat((vis.index_select(1, idx), audio), dim=-1)
        mask = self.net_fusion(comb)
        return spec * mask.unsqueeze(1)

    def cal_loss(self, batch):
        return self.loss(self(batch), batch["mask"])

    def training_step(self, batch, batch_idx=0):
        return self.cal_loss(batch)

    def validation_step(self, batch, batch_idx=0):
        return self.cal_loss(batch)

    def configure_optimizers(self):
        return torch.optim.Adam(self.parameters(), lr=self.lr)

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location="cpu", strict=True, **kwargs):
        """test.py:47 `AVNet.load_from_checkpoint(ckpt_path, nets=..., ...)` (Lightning .ckpt, ckpt_io); the
        reference's `nets=` argument is not a constructor argument here (the sub-nets are built in place)."""
        from .ckpt_io import load_lightning_checkpoint
        return load_lightning_checkpoint(cls, checkpoint_path, map_location, strict, **kwargs)

    # ---- HIP front-end / back-end (what the reference does on CPU with librosa)
    @staticmethod
    def features_from_waves(noisy, clean=None):
        """(B, 48000) waveforms -> batch dict of |STFT|.T features (dataset.py:112-118, 154-157)."""
        out = {"noisy_audio_spec": K.stft(noisy).unsqueeze(1)}
        if clean is not None:
            out["mask"] = K.stft(clean).unsqueeze(1)
        return out

    @torch.no_grad()
    def enhance(self, noisy_wave, lip_images=None, length=None):
        """test.py:79-89: predicted magnitude x noisy phase -> iSTFT (all on the GPU); lip_images is
        unused (None) for the audio-only net (test.py:81)."""
        mag, spec = K.stft(noisy_wave, return_complex=True)
        inp = {"noisy_audio_spec": mag.unsqueeze(1)}
        if not self.a_only:
            inp["lip_images"] = lip_images
        pred = self(inp)[:, 0]
        return K.istft(pred, spec, noisy_wave.shape[-1] if length is None else length)


def load_lightning_state_dict(model, ckpt_state_dict):
    """Load a Lightning ``.ckpt['state_dict']`` (keys already match: net_visualfeat.*, net_audiofeat.*, ...)."""
    return model.load_state_dict(ckpt_state_dict, strict=True)
