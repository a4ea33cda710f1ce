"""avse1 AV baseline, CPU restatement — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Citations relative to /root/reference/baseline/avse1:
  VisualFeatNet          model.py:17-58 (frontend3D :29-34, TCN feature path :48-58)
  ResNet-18 / BasicBlock utils/resnet.py:26-67, :70-124
  TCN / TemporalBlock    utils/nn.py:106-128, utils/tcn.py:144-243 (symmetric chomp, dwpw=False)
  AudioFeatNet           model.py:181-267
  FusionNet              model.py:81-96
  AVNet.forward          model.py:114-128; cal_loss :164-168 (l1, train.py:854 default)
Module trees (including the aliased ``net`` Sequential inside TemporalBlock) mirror the
reference so state_dict keys are identical.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

STFT_SIZE, WINDOW_SHIFT, NUM_STFT_FRAMES, NUM_FRAMES = 512, 128, 376, 75


# ---------------------------------------------------------------- visual stream

class BasicBlock(nn.Module):
    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu1 = nn.PReLU(planes)
        self.relu2 = nn.PReLU(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        out = self.bn2(self.conv2(self.relu1(self.bn1(self.conv1(x)))))
        res = x if self.downsample is None else self.downsample(x)
        return self.relu2(out + res)


class ResNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.inplanes = 64
        self.layer1 = self._make(64, 1)
        self.layer2 = self._make(128, 2)
        self.layer3 = self._make(256, 2)
        self.layer4 = self._make(512, 2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)

    def _make(self, planes, stride):
        ds = None
        if stride != 1 or self.inplanes != planes:
            ds = nn.Sequential(nn.Conv2d(self.inplanes, planes, 1, stride=stride, bias=False), nn.BatchNorm2d(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, ds), BasicBlock(planes, planes)]
        self.inplanes = planes
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.avgpool(x).flatten(1)


class Chomp1d(nn.Module):
    def __init__(self, size):
        super().__init__()
        self.size = size

    def forward(self, x):
        return x[:, :, self.size // 2:-(self.size // 2)].contiguous() if self.size else x


class TemporalBlock(nn.Module):
    def __init__(self, c, k, dilation, dropout=0.2):
        super().__init__()
        pad = (k - 1) * dilation
        self.conv1 = nn.Conv1d(c, c, k, padding=pad, dilation=dilation)
        self.batchnorm1 = nn.BatchNorm1d(c)
        self.chomp1 = Chomp1d(pad)
        self.relu1 = nn.PReLU(c)
        self.dropout1 = nn.Dropout(dropout)
        self.conv2 = nn.Conv1d(c, c, k, padding=pad, dilation=dilation)
        self.batchnorm2 = nn.BatchNorm1d(c)
        self.chomp2 = Chomp1d(pad)
        self.relu2 = nn.PReLU(c)
        self.dropout2 = nn.Dropout(dropout)
        self.net = nn.Sequential(self.conv1, self.batchnorm1, self.chomp1, self.relu1, self.dropout1,
                                 self.conv2, self.batchnorm2, self.chomp2, self.relu2, self.dropout2)
        self.downsample = None
        self.relu = nn.PReLU(c)

    def forward(self, x):
        return self.relu(self.net(x) + x)


class TemporalConvNet(nn.Module):
    def __init__(self, c=512, levels=4, k=3, dropout=0.2):
        super().__init__()
        self.network = nn.Sequential(*[TemporalBlock(c, k, 2 ** i, dropout) for i in range(levels)])

    def forward(self, x):
        return self.network(x)


class TCN(nn.Module):
    def __init__(self, c=512, levels=4, num_classes=500, dropout=0.2):
        super().__init__()
        self.tcn_trunk = TemporalConvNet(c, levels, 3, dropout)
        self.tcn_output = nn.Linear(c, num_classes)

    def forward(self, x):                      # (B, T, C) -> (B, C, T)
        return self.tcn_trunk(x.transpose(1, 2))


class VisualFeatNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.trunk = ResNet()
        self.frontend3D = nn.Sequential(
            nn.Conv3d(3, 64, (5, 7, 7), stride=(1, 2, 2), padding=(2, 3, 3), bias=False),
            nn.BatchNorm3d(64), nn.PReLU(64), nn.MaxPool3d((1, 3, 3), stride=(1, 2, 2), padding=(0, 1, 1)))
        self.tcn = TCN()

    def forward(self, x):                      # (B, 3, T, H, W) -> (B, T, 512)
        B = x.shape[0]
        x = self.frontend3D(x)
        T = x.shape[2]
        x = x.transpose(1, 2).reshape(B * T, x.shape[1], x.shape[3], x.shape[4])
        x = self.trunk(x).view(B, T, -1)
        return self.tcn(x).permute(0, 2, 1)


# ---------------------------------------------------------------- audio stream

class AudioFeatNet(nn.Module):
    def __init__(self, num_conv=5, k=5, filters=64, last_filter=4):
        super().__init__()
        self.num_conv, self.last_filter = num_conv, last_filter
        self.embed_size = STFT_SIZE // 2 + 1
        self.bn0 = nn.BatchNorm2d(1)
        for i in range(num_conv):
            cin = 1 if i == 0 else filters
            dil = 2 ** i
            setattr(self, f"conv{i + 1}", nn.Conv2d(cin, filters, (k, k), padding=(k - 1) * dil // 2, dilation=dil))
            setattr(self, f"bn{i + 1}", nn.BatchNorm2d(filters))
        self.convf = nn.Conv2d(filters, last_filter, 1)
        self.bn_last = nn.BatchNorm2d(last_filter)

    def forward(self, x):                      # (B, 1, T, F) -> (B, T, 4F)
        T = x.shape[2]
        x = self.bn0(x)
        for i in range(self.num_conv):
            x = F.relu(getattr(self, f"bn{i + 1}")(getattr(self, f"conv{i + 1}")(x)))
        x = F.relu(self.bn_last(self.convf(x)))
        return x.permute(0, 2, 1, 3).reshape(-1, T, self.embed_size * self.last_filter)


class FusionNet(nn.Module):
    def __init__(self, a_only=False):
        super().__init__()
        self.lstm_conv = nn.LSTM((0 if a_only else 512) + 1028, STFT_SIZE // 2 + 1, num_layers=1, batch_first=True)
        self.time_distributed_1 = nn.Linear(STFT_SIZE // 2 + 1, STFT_SIZE // 2 + 1)

    def forward(self, x):
        return torch.sigmoid(self.time_distributed_1(self.lstm_conv(x)[0]))


class AVNet(nn.Module):
    def __init__(self, a_only=False):
        super().__init__()
        self.a_only = a_only
        self.net_visualfeat = None if a_only else VisualFeatNet()
        self.net_audiofeat = AudioFeatNet()
        self.net_fusion = FusionNet(a_only)

    def forward(self, inp):
        spec = inp["noisy_audio_spec"]
        T = spec.shape[2]
        if self.a_only:
            comb = self.net_audiofeat(spec)
        else:
            # model.py:122 casts the uint8 lips with .float(); the fp64 oracle run casts to its own dtype
            lips = inp["lip_images"].to(self.net_audiofeat.conv1.weight.dtype)
            vis = self.net_visualfeat(lips).unsqueeze(1)
            vis = F.interpolate(vis, size=(T, 512)).reshape(-1, T, 512)
            comb = torch.cat((vis, self.net_audiofeat(spec)), dim=-1)
        mask = self.net_fusion(comb)
        return spec * mask.unsqueeze(1)

    def cal_loss(self, batch):
        return F.l1_loss(self(batch), batch["mask"])
