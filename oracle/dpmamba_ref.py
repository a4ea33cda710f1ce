"""DPMamba (dual-path Mamba) separator, CPU restatement — TEST INFRASTRUCTURE ONLY (oracle/__init__.py).

Restates (citations relative to /root/reference/Mamba-TasNet):
  Dual_Path_Model.forward     modules/dual_path.py:53-150 (the in-tree copy of speechbrain's forward;
                              skip_n_block = 0, use_global_pos_enc = False as in hparams/WSJ0Mix/dpmamba_*.yaml)
  Dual_Path_Model.__init__,   speechbrain 1.0.0 lobes/models/dual_path.py (un-vendored): norm 'ln' =
  _Segmentation, _over_add,   GroupNorm(1, C, eps 1e-8); conv1d 1x1 no bias; conv2d 1x1 with bias; PReLU;
  Dual_Computation_Block      gated output Conv1d+Tanh * Conv1d+Sigmoid; end 1x1 no bias; ReLU; chunking
                              with 50 % overlap and zero padding; intra/inter with GroupNorm after each
                              model, skip around intra, no linear layer (linear_layer_after_inter_intra False)
                              — parity unpinned (no speechbrain source or fixture in the reference)
  intra / inter models        modules/mamba_blocks.py:87-212 with n_mamba = n_mamba_dp // 2 = 1, BiMamba v2
                              (oracle.mamba_ref, pinned by tests/golden)
  sizes                       hparams/WSJ0Mix/dpmamba_{XS,S,M,L}.yaml:108-123
"""
import copy

import torch
import torch.nn as nn
import torch.nn.functional as F

from .mamba_ref import Decoder, Encoder, MambaBlocksSequential

DPMAMBA_SIZES = {"XS": dict(N=128, n_dp=8, skip_around_intra=False), "S": dict(N=256, n_dp=8, skip_around_intra=False),
                 "M": dict(N=256, n_dp=16, skip_around_intra=True), "L": dict(N=512, n_dp=16, skip_around_intra=True)}


class Dual_Computation_Block(nn.Module):
    def __init__(self, intra_mdl, inter_mdl, out_channels, skip_around_intra=True):
        super().__init__()
        self.intra_mdl = intra_mdl
        self.inter_mdl = inter_mdl
        self.skip_around_intra = skip_around_intra
        self.intra_norm = nn.GroupNorm(1, out_channels, eps=1e-8)
        self.inter_norm = nn.GroupNorm(1, out_channels, eps=1e-8)

    def forward(self, x):
        B, N, K, S = x.shape
        # intra: [BS, K, N]
        intra = x.permute(0, 3, 2, 1).contiguous().view(B * S, K, N)
        intra = self.intra_mdl(intra)
        intra = intra.view(B, S, K, N).permute(0, 3, 2, 1).contiguous()
        intra = self.intra_norm(intra)
        if self.skip_around_intra:
            intra = intra + x
        # inter: [BK, S, N]
        inter = intra.permute(0, 2, 3, 1).contiguous().view(B * K, S, N)
        inter = self.inter_mdl(inter)
        inter = inter.view(B, K, S, N).permute(0, 3, 1, 2).contiguous()
        inter = self.inter_norm(inter)
        return inter + intra


class Dual_Path_Model(nn.Module):
    def __init__(self, in_channels, out_channels, intra_model, inter_model, num_layers=1, K=200, num_spks=2,
                 skip_around_intra=True):
        super().__init__()
        self.K = K
        self.num_spks = num_spks
        self.num_layers = num_layers
        self.norm = nn.GroupNorm(1, in_channels, eps=1e-8)
        self.conv1d = nn.Conv1d(in_channels, out_channels, 1, bias=False)
        self.dual_mdl = nn.ModuleList([])
        for _ in range(num_layers):
            self.dual_mdl.append(copy.deepcopy(Dual_Computation_Block(intra_model, inter_model, out_channels,
                                                                      skip_around_intra)))
        self.conv2d = nn.Conv2d(out_channels, out_channels * num_spks, kernel_size=1)
        self.end_conv1x1 = nn.Conv1d(out_channels, in_channels, 1, bias=False)
        self.prelu = nn.PReLU()
        self.activation = nn.ReLU()
        self.output = nn.Sequential(nn.Conv1d(out_channels, out_channels, 1), nn.Tanh())
        self.output_gate = nn.Sequential(nn.Conv1d(out_channels, out_channels, 1), nn.Sigmoid())

    def _padding(self, input, K):
        B, N, L = input.shape
        P = K // 2
        gap = K - (P + L % K) % K
        if gap > 0:
            input = torch.cat([input, input.new_zeros(B, N, gap)], dim=2)
        _pad = input.new_zeros(B, N, P)
        return torch.cat([_pad, input, _pad], dim=2), gap

    def _Segmentation(self, input, K):
        B, N, L = input.shape
        P = K // 2
        input, gap = self._padding(input, K)
        input1 = input[:, :, :-P].contiguous().view(B, N, -1, K)
        input2 = input[:, :, P:].contiguous().view(B, N, -1, K)
        input = torch.cat([input1, input2], dim=3).view(B, N, -1, K).transpose(2, 3)
        return input.contiguous(), gap

    def _over_add(self, input, gap):
        B, N, K, S = input.shape
        P = K // 2
        input = input.transpose(2, 3).contiguous().view(B, N, -1, K * 2)
        input1 = input[:, :, :, :K].contiguous().view(B, N, -1)[:, :, P:]
        input2 = input[:, :, :, K:].contiguous().view(B, N, -1)[:, :, :-P]
        input = input1 + input2
        if gap > 0:
            input = input[:, :, :-gap]
        return input

    def forward(self, x):                        # modules/dual_path.py:76-150
        x = self.norm(x)
        x = self.conv1d(x)
        x, gap = self._Segmentation(x, self.K)
        for i in range(self.num_layers):
            x = self.dual_mdl[i](x)
        x = self.prelu(x)
        x = self.conv2d(x)
        B, _, K, S = x.shape
        x = x.view(B * self.num_spks, -1, K, S)
        x = self._over_add(x, gap)
        x = self.output(x) * self.output_gate(x)
        x = self.end_conv1x1(x)
        _, N, L = x.shape
        x = x.view(B, self.num_spks, N, L)
        x = self.activation(x)
        return x.transpose(0, 1)


class DPMambaTasNet(nn.Module):
    """Encoder / Dual_Path_Model / Decoder with train_wsj0mix.py:86-111 compute_forward semantics."""

    def __init__(self, N=512, n_dp=16, skip_around_intra=True, kernel_size=16, chunk_size=250, n_spk=2,
                 n_mamba_dp=2, d_state=16, expand=2, d_conv=4):
        super().__init__()
        self.num_spks = n_spk
        self.encoder = Encoder(kernel_size, N)
        intra = MambaBlocksSequential(n_mamba_dp // 2, N, d_state, expand, d_conv)
        inter = MambaBlocksSequential(n_mamba_dp // 2, N, d_state, expand, d_conv)
        self.masknet = Dual_Path_Model(N, N, intra, inter, n_dp, chunk_size, n_spk, skip_around_intra)
        self.decoder = Decoder(N, 1, kernel_size, stride=kernel_size // 2, bias=False)

    def forward(self, mix):
        mix_w = self.encoder(mix)
        est_mask = self.masknet(mix_w)
        sep_h = torch.stack([mix_w] * self.num_spks) * est_mask
        est = torch.stack([self.decoder(sep_h[i]) for i in range(self.num_spks)], dim=-1)
        T = mix.shape[1]
        if T > est.shape[1]:
            est = F.pad(est, (0, 0, 0, T - est.shape[1]))
        else:
            est = est[:, :T, :]
        return est
