"""Mamba-TasNet-L + lip-encoder AV fusion (BASELINE configs[4], SURVEY §8d "C5").

C5 has no reference model (SURVEY.md "Hard parts": "Config 5 (Mamba-L + lip fusion) has no reference
model: parity is per component only"). It is assembled from reference components, each of which
is pinned on its own:
  Encoder / Decoder          Conv1d(1, N, 16, s8) + ReLU / ConvTranspose1d(N, 1, 16, s8)
                             (train_wsj0mix.py:86-111, baseline/avse2/model.py:14-37)
  VisualFrontend             avse4 lip encoder (baseline/avse4/utils.py:97-118): Conv3d + ResNet-18
  visual upsampling          avse4 style (baseline/avse4/model.py:166-176): linear interpolation of the
                             T_v lip frames to the L encoder frames (align_corners=False), as one GEMM
                             with a fixed interpolation matrix
  MaskNet                    Mamba-TasNet MaskNet (mamba_masknet.py:101-139) whose bottleneck 1x1 takes the
                             concatenation [cLN(audio), visual] (2N -> N), one output (enhancement), ReLU mask
  loss                       avse4 cal_loss (-SI-SNR clamped at -30, baseline/avse4/model.py:374-383)
The step runs under bf16 autocast (torch.autocast("cuda", torch.bfloat16)): bf16 projections (MFMA),
bf16 conv / scan activations with fp32 scan state, fp32 residual stream / RMSNorm / loss; the lip
encoder runs in fp32 (``visual_bf16=False``, the default) or under the same autocast.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import avse4, losses
from .mamba_tasnet import ChannelwiseLayerNorm, Conv1x1, Decoder, Encoder, MambaBlocksSequential


class AVMaskNet(nn.Module):
    def __init__(self, N=512, v_dim=512, n_mamba=32, d_state=16, expand=2, d_conv=4):
        super().__init__()
        self.layer_norm = ChannelwiseLayerNorm(N)
        self.visual_conv1x1 = Conv1x1(v_dim, N)
        self.bottleneck_conv1x1 = Conv1x1(2 * N, N)
        self.mamba_net = MambaBlocksSequential(n_mamba, N, d_state, expand, d_conv)
        self.mask_conv1x1 = Conv1x1(N, N)

    def forward(self, mixture_w, v):                  # (M, N, L), (M, T_v, v_dim) -> mask (M, N, L)
        x = self.layer_norm(mixture_w.permute(0, 2, 1))                     # (M, L, N)
        L, Tv = x.shape[1], v.shape[1]
        up = max(1, math.ceil(L / Tv))
        interp = avse4._upsample_matrix(Tv, up, L, x.device)                # (T_v, L), crops / pads to L
        vl = torch.matmul(interp.t(), self.visual_conv1x1(v))               # (M, L, N)
        y = self.bottleneck_conv1x1(torch.cat([x, vl.to(x.dtype)], dim=-1))
        y = self.mask_conv1x1(self.mamba_net(y))
        return F.relu(y).permute(0, 2, 1)


class AVMambaTasNet(nn.Module):
    """mix (B, T) + lips (B, 1, T_v, 112, 112) in [0, 1) -> enhanced (B, T)."""

    def __init__(self, N=512, kernel_size=16, n_mamba=32, d_state=16, expand=2, d_conv=4, visual_bf16=False):
        super().__init__()
        self.visual_bf16 = visual_bf16
        self.encoder = Encoder(kernel_size, N)
        self.visual_frontend = avse4.VisualFrontend()
        self.masknet = AVMaskNet(N, 512, n_mamba, d_state, expand, d_conv)
        self.decoder = Decoder(N, 1, kernel_size, stride=kernel_size // 2, bias=False)

    def forward(self, mix, lips):
        on = torch.is_autocast_enabled("cuda")
        with torch.autocast("cuda", dtype=torch.get_autocast_dtype("cuda"), enabled=self.visual_bf16 and on):
            v = self.visual_frontend(lips)                                  # (B, T_v, 512)
        mix_w = self.encoder(mix)
        est = self.decoder(mix_w * self.masknet(mix_w, v))
        T = mix.shape[-1]
        if T > est.shape[-1]:
            return F.pad(est, (0, T - est.shape[-1]))
        return est[..., :T]

    def cal_loss(self, batch):
        est = self(batch["noisy_audio"], batch["vis_feat"])
        return losses.avse4_loss(batch["clean"][:, None].float(), est[:, None].float())


AV_MAMBA_SIZES = {"XS": dict(N=128, n_mamba=16), "S": dict(N=256, n_mamba=16),
                  "M": dict(N=256, n_mamba=32), "L": dict(N=512, n_mamba=32)}
