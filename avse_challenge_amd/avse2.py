"""avse2 time-domain AV separator on the MI355X path.

Mirrors, with the reference's module tree and state_dict keys (Lightning ``.ckpt`` of baseline/avse2 loads
unchanged):
  AVSEModule / AVSE      baseline/avse2/model.py:194-274 (forward, cal_loss with the SI-SNR clamp at -30)
  VisualFeatNet          model.py:39-85 + utils/dnn.py:61-184 (ResNet-18 with Swish, lip Conv3d front-end)
  Separator / block      model.py:88-191 (DPRNN: bidirectional LSTMs on 200-frame chunks, 50 % overlap)
  AudioEncoder/Decoder   model.py:14-36
HIP parts: the lip Conv3d weight gradient (MFMA implicit GEMM, layers.LipConv3d), the separator PReLU
(layers.PReLU), the encoder as framing + GEMM and the decoder as GEMM + overlap-add (the Mamba-TasNet
Encoder/Decoder).  The DPRNN state is kept channels-last (B, S, K, N) so the intra LSTM reads (B*S, K, N)
without a copy, and GroupNorm(1) statistics run as a flat reduction (dpmamba._gln_cl).  The LSTMs, the
ResNet convolutions and BatchNorms are library calls (MIOpen / hipBLASLt).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .dpmamba import DualPathModel, _gln_cl
from .layers import HipLSTM, LipConv3d, PReLU
from .losses import cal_si_snr
from .mamba_tasnet import Decoder, Encoder


class Swish(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(x)


class BasicBlock(nn.Module):                   # utils/dnn.py:86-130 (relu_type 'swish')
    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu1 = Swish()
        self.relu2 = Swish()
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        residual = x if self.downsample is None else self.downsample(x)
        return self.relu2(self.bn2(self.conv2(self.relu1(self.bn1(self.conv1(x))))) + residual)


class ResNet(nn.Module):                       # utils/dnn.py:133-184
    def __init__(self):
        super().__init__()
        self.inplanes = 64
        self.layer1, self.layer2 = self._make(64, 1), self._make(128, 2)
        self.layer3, self.layer4 = self._make(256, 2), self._make(512, 2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)

    def _make(self, planes, stride):
        ds = None
        if stride != 1 or self.inplanes != planes:
            ds = nn.Sequential(nn.Conv2d(self.inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
        blocks = [BasicBlock(self.inplanes, planes, stride, ds)]
        self.inplanes = planes
        blocks.append(BasicBlock(planes, planes))
        return nn.Sequential(*blocks)

    def forward(self, x):
        return self.avgpool(self.layer4(self.layer3(self.layer2(self.layer1(x))))).flatten(1)


class VisualFeatNet(nn.Module):                # model.py:39-85
    def __init__(self):
        super().__init__()
        self.trunk = ResNet()
        self.frontend3D = nn.Sequential(LipConv3d(1, 64, (5, 7, 7), (1, 2, 2), (2, 3, 3)), nn.BatchNorm3d(64), Swish(),
                                        nn.MaxPool3d((1, 3, 3), (1, 2, 2), (0, 1, 1)))
        self.nn_out = nn.Linear(512, 256, bias=False)

    def forward(self, x):                      # (B, 1, T, H, W) -> (B, T, 256)
        B = x.shape[0]
        x = self.frontend3D(x)
        T = x.shape[2]
        x = self.trunk(x.transpose(1, 2).reshape(B * T, x.shape[1], x.shape[3], x.shape[4]))
        return torch.relu(self.nn_out(x.view(B, T, -1)))


class SeparatorBlock(nn.Module):              # model.py:88-123, on the channels-last state (B, S, K, N)
    def __init__(self, out_channels, hidden_channels, bidirectional=True):
        super().__init__()
        self.intra_rnn = HipLSTM(out_channels, hidden_channels, 1, batch_first=True, bidirectional=bidirectional)
        self.inter_rnn = HipLSTM(out_channels, hidden_channels, 1, batch_first=True, bidirectional=bidirectional)
        self.intra_norm = nn.GroupNorm(1, out_channels, eps=1e-8)
        self.inter_norm = nn.GroupNorm(1, out_channels, eps=1e-8)
        h = hidden_channels * (2 if bidirectional else 1)
        self.intra_linear = nn.Linear(h, out_channels)
        self.inter_linear = nn.Linear(h, out_channels)

    def forward(self, x):
        B, S, K, N = x.shape
        intra, _ = self.intra_rnn(x.reshape(B * S, K, N))
        intra = self.intra_linear(intra).view(B, S, K, N)
        intra = _gln_cl(intra, self.intra_norm.weight, self.intra_norm.bias, self.intra_norm.eps) + x
        inter, _ = self.inter_rnn(intra.transpose(1, 2).reshape(B * K, S, N))
        inter = self.inter_linear(inter).view(B, K, S, N)
        inter = _gln_cl(inter, self.inter_norm.weight, self.inter_norm.bias, self.inter_norm.eps)
        return intra + inter.transpose(1, 2)


class Separator(nn.Module):                    # model.py:126-191
    def __init__(self, in_channels=512, out_channels=64, hidden_channels=128, bidirectional=True, num_layers=6, K=200):
        super().__init__()
        self.K = K
        self.input_conv = nn.Sequential(nn.GroupNorm(1, in_channels, eps=1e-8),
                                        nn.Conv1d(in_channels, out_channels, 1, bias=False))
        self.separator_blocks = nn.Sequential(*[SeparatorBlock(out_channels, hidden_channels, bidirectional)
                                                for _ in range(num_layers)])
        self.conv2d = nn.Conv2d(out_channels, out_channels, 1)
        self.end_conv1x1 = nn.Conv1d(out_channels, 256, 1, bias=False)
        self.prelu = PReLU()
        self.activation = nn.ReLU()
        self.output = nn.Sequential(nn.Conv1d(out_channels, out_channels, 1), nn.Tanh())
        self.output_gate = nn.Sequential(nn.Conv1d(out_channels, out_channels, 1), nn.Sigmoid())

    def forward(self, x):                      # (B, 512, L) -> (B, 256, L)
        x = self.input_conv(x)
        x, gap = DualPathModel._segmentation(x, self.K)                 # [B, N, K, S]
        x = self.separator_blocks(x.permute(0, 3, 2, 1).contiguous())    # channels-last (B, S, K, N)
        x = self.conv2d(self.prelu(x.permute(0, 3, 2, 1).contiguous()))
        x = DualPathModel._over_add(x, gap)
        x = self.end_conv1x1(self.output(x) * self.output_gate(x))
        return self.activation(x)


class AVSE(nn.Module):                         # model.py:194-216
    def __init__(self):
        super().__init__()
        self.audio_encoder = Encoder(16, 256)
        self.audio_decoder = Decoder(256, 1, 16, stride=8, bias=False)
        self.visual_encoder = VisualFeatNet()
        self.separator = Separator(512, 64, 128, bidirectional=True, num_layers=6)

    def forward(self, inp):
        enc = self.audio_encoder(inp["noisy_audio"])                      # (B, 256, L)
        vis = self.visual_encoder(inp["video_frames"].float())             # (B, T, 256)
        L = enc.shape[-1]
        up = F.interpolate(vis.unsqueeze(1), size=(L, vis.shape[-1]), mode="bilinear")[:, 0].transpose(1, 2)
        mask = self.separator(torch.cat((up, enc), dim=1))
        return self.audio_decoder(mask * enc)                              # (B, T')


class AVSEModule(nn.Module):                   # model.py:219-274 (the LightningModule surface)
    def __init__(self, lr=0.00015):
        super().__init__()
        self.lr = lr
        self.model = AVSE()

    def forward(self, data):
        return self.model(data)

    def cal_loss(self, batch):
        clean = batch["clean"].T
        pred = self(batch).T.reshape(clean.shape)
        loss = cal_si_snr(pred.unsqueeze(2), clean.unsqueeze(2))          # model.py:260 argument order
        return torch.where(loss < -30, torch.full_like(loss, -30.0), loss).mean()

    def training_step(self, batch, batch_idx=0):
        return self.cal_loss(batch)

    def validation_step(self, batch, batch_idx=0):
        return self.cal_loss(batch)

    def configure_optimizers(self):
        return torch.optim.Adam(self.parameters(), lr=self.lr)
