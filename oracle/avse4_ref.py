"""avse4 binaural AV baseline, CPU restatement — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Citations relative to /root/reference/baseline/avse4:
  overlap_and_add        model.py:19-66
  avse4_separator        model.py:73-94     Encoder model.py:97-109   Decoder model.py:112-123
  TemporalConvNet        model.py:126-182   VisualConv1D model.py:184-205
  ChannelWiseLayerNorm   model.py:208-222 (nn.LayerNorm, eps 1e-5)
  GlobalLayerNorm        model.py:225-252 (EPS 1e-8 inside pow(var+EPS, .5))
  TemporalBlock          model.py:255-269   DepthwiseSeparableConv model.py:272-293
  VisualFrontend/ResNet  utils.py:40-118
  AVSE4BaselineModule    model.py:295-393 (forward :316-321, cal_loss :374-383)
State-dict keys are identical to the reference (checked when goldens are made).
"""
import copy

import torch
import torch.nn as nn
import torch.nn.functional as F

from .losses_ref import avse4_loss

EPS = 1e-8
NORM_MEAN, NORM_STD = 0.4161, 0.1688


def overlap_and_add(frames, step):
    """frames (..., K, Lf) -> (..., step*(K-1)+Lf) by summing shifted frames."""
    *outer, K, Lf = frames.shape
    out = frames.new_zeros(*outer, step * (K - 1) + Lf)
    for k in range(K):
        out[..., k * step:k * step + Lf] += frames[..., k, :]
    return out


class GlobalLayerNorm(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(1, c, 1))
        self.beta = nn.Parameter(torch.zeros(1, c, 1))

    def forward(self, y):
        mean = y.mean(dim=1, keepdim=True).mean(dim=2, keepdim=True)
        var = ((y - mean) ** 2).mean(dim=1, keepdim=True).mean(dim=2, keepdim=True)
        return self.gamma * (y - mean) / torch.pow(var + EPS, 0.5) + self.beta


class ChannelWiseLayerNorm(nn.LayerNorm):
    def forward(self, x):
        return super().forward(x.transpose(1, 2)).transpose(1, 2)


class DepthwiseSeparableConv(nn.Module):
    def __init__(self, cin, cout, k, stride, padding, dilation):
        super().__init__()
        self.net = nn.Sequential(
            nn.Conv1d(cin, cin, k, stride=stride, padding=padding, dilation=dilation, groups=cin, bias=False),
            nn.PReLU(), GlobalLayerNorm(cin), nn.Conv1d(cin, cout, 1, bias=False))

    def forward(self, x):
        return self.net(x)


class TemporalBlock(nn.Module):
    def __init__(self, cin, cout, k, stride, padding, dilation):
        super().__init__()
        self.net = nn.Sequential(nn.Conv1d(cin, cout, 1, bias=False), nn.PReLU(), GlobalLayerNorm(cout),
                                 DepthwiseSeparableConv(cout, cin, k, stride, padding, dilation))

    def forward(self, x):
        return self.net(x) + x


class VisualConv1D(nn.Module):
    def __init__(self, c=512):
        super().__init__()
        self.net = nn.Sequential(nn.ReLU(), nn.BatchNorm1d(c),
                                 nn.Conv1d(c, c, 3, padding=1, groups=c, bias=False), nn.PReLU(),
                                 nn.BatchNorm1d(c), nn.Conv1d(c, c, 1, bias=False))

    def forward(self, x):
        return self.net(x) + x


class TemporalConvNet(nn.Module):
    def __init__(self, N, B, H, P, X, R, C, num_channels=2, vis_dim=512, up=32):
        super().__init__()
        self.num_channels, self.up = num_channels, up
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
        x = self.bottleneck_conv1x1(self.layer_norm(x))
        bsz, Bc, K = x.shape
        for i in range(len(self.tcn)):
            v = self.ve_conv1x1[i](visual)
            v = F.interpolate(v, self.up * v.shape[-1], mode="linear")
            v = F.pad(v, (0, K - v.shape[-1]))
            x = self.tcn[i](torch.cat((x, v), 1))
        x = F.relu(self.mask_conv1x1(x))
        return x.reshape(bsz, self.num_channels, Bc, K)


class Encoder(nn.Module):
    def __init__(self, L, N, num_channels=2):
        super().__init__()
        self.conv1d_U = nn.Conv1d(num_channels, N, L, stride=L // 2, bias=False)

    def forward(self, m):
        return F.relu(self.conv1d_U(m))


class Decoder(nn.Module):
    def __init__(self, N, L):
        super().__init__()
        self.L = L
        self.basis_signals = nn.Linear(N, L, bias=False)

    def forward(self, mixture_w, est_mask):
        est = (mixture_w[:, None] * est_mask).transpose(2, 3)
        return overlap_and_add(self.basis_signals(est), self.L // 2)


class Separator(nn.Module):
    def __init__(self, N=256, L=40, B=256, H=512, P=3, X=8, R=4, C=2, num_channels=2):
        super().__init__()
        self.encoder = Encoder(L, N, num_channels)
        self.separator = TemporalConvNet(N, B, H, P, X, R, C, num_channels)
        self.decoder = Decoder(N, L)

    def forward(self, mixture, visual):
        w = self.encoder(mixture)
        est = self.decoder(w, self.separator(w, visual))
        return F.pad(est, (0, mixture.shape[-1] - est.shape[-1]))


class ResNetLayer(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        bn = dict(momentum=0.01, eps=0.001)
        self.conv1a = nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)
        self.bn1a = nn.BatchNorm2d(cout, **bn)
        self.conv2a = nn.Conv2d(cout, cout, 3, padding=1, bias=False)
        self.stride = stride
        self.downsample = nn.Conv2d(cin, cout, 1, stride=stride, bias=False)
        self.outbna = nn.BatchNorm2d(cout, **bn)
        self.conv1b = nn.Conv2d(cout, cout, 3, padding=1, bias=False)
        self.bn1b = nn.BatchNorm2d(cout, **bn)
        self.conv2b = nn.Conv2d(cout, cout, 3, padding=1, bias=False)
        self.outbnb = nn.BatchNorm2d(cout, **bn)

    def forward(self, x):
        y = self.conv2a(F.relu(self.bn1a(self.conv1a(x))))
        y = y + (x if self.stride == 1 else self.downsample(x))
        mid = y
        y = F.relu(self.outbna(y))
        y = self.conv2b(F.relu(self.bn1b(self.conv1b(y)))) + mid
        return F.relu(self.outbnb(y))


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
            nn.Conv3d(1, 64, (5, 7, 7), stride=(1, 2, 2), padding=(2, 3, 3), bias=False),
            nn.BatchNorm3d(64, momentum=0.01, eps=0.001), nn.ReLU(),
            nn.MaxPool3d((1, 3, 3), stride=(1, 2, 2), padding=(0, 1, 1)))
        self.resnet = ResNet()

    def forward(self, x):                       # (B, 1, T, 112, 112) -> (B, T, 512)
        bsz = x.shape[0]
        y = self.frontend3D((x - NORM_MEAN) / NORM_STD).transpose(1, 2)
        y = y.reshape(y.shape[0] * y.shape[1], y.shape[2], y.shape[3], y.shape[4])
        return self.resnet(y).reshape(bsz, -1, 512)


class AVSE4BaselineModule(nn.Module):
    def __init__(self, num_channels=2, **sep_kwargs):
        super().__init__()
        self.num_channels = num_channels
        self.model = Separator(num_channels=num_channels, **sep_kwargs)
        self.visual_frontend = VisualFrontend()

    def forward(self, data):
        return self.model(data["noisy_audio"].float(), self.visual_frontend(data["vis_feat"].float()))

    def cal_loss(self, batch):
        return avse4_loss(batch["clean"], self(batch))
