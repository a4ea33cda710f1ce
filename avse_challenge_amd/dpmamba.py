"""DPMamba separator (dual-path Mamba) on the MI355X kernels.

Mirrors, with the reference's state_dict keys (``masknet.ckpt`` of hparams/WSJ0Mix/dpmamba_*.yaml):
  DualPathModel         speechbrain 1.0.0 lobes/models/dual_path.Dual_Path_Model (un-vendored; its forward is
                        restated in-tree at Mamba-TasNet/modules/dual_path.py:53-150, skip_n_block = 0;
                        __init__, _Segmentation, _over_add and Dual_Computation_Block are restated from the
                        published SpeechBrain source: parity of those parts unpinned)
  DualComputationBlock  speechbrain dual_path.Dual_Computation_Block (norm 'ln' = GroupNorm(1, N, eps 1e-8),
                        linear_layer_after_inter_intra False, skip_around_intra per size)
  intra / inter models  modules/mamba_blocks.MambaBlocksSequential(n_mamba_dp // 2 = 1, bidirectional)
                        -> mamba_tasnet.MambaBlocksSequential (HIP scan / causal conv / add+RMSNorm)
  Encoder / Decoder     as Mamba-TasNet (dpmamba_*.yaml:138,176)
  DPMambaTasNet.forward train_wsj0mix.py:86-111 compute_forward
The intra pass runs the BiMamba blocks on (B*S, K=250, N) chunks, the inter pass on (B*K, S, N): the same
selective-scan kernel at a short sequence length with a large batch of sequences.
"""
import copy

import torch
import torch.nn as nn
import torch.nn.functional as F

from .mamba_tasnet import Decoder, Encoder, MambaBlocksSequential

# hparams/WSJ0Mix/dpmamba_{XS,S,M,L}.yaml: N_encoder_out = out_channels, n_dp, skip_around_intra
DPMAMBA_SIZES = {"XS": dict(N=128, n_dp=8, skip_around_intra=False), "S": dict(N=256, n_dp=8, skip_around_intra=False),
                 "M": dict(N=256, n_dp=16, skip_around_intra=True), "L": dict(N=512, n_dp=16, skip_around_intra=True)}


def _gln_cl(x, weight, bias, eps):
    """GroupNorm(1, N) of a sample stored channels-last, (B, ..., N): statistics over all of the sample's
    elements (biased variance, eps inside the rsqrt), affine per channel.  torch's GroupNorm kernel gives
    each sample ONE workgroup (RowwiseMoments: 3.9 ms per call at B=16, K=250, S=34, N=512); the flat
    var_mean splits each sample over many workgroups."""
    B = x.shape[0]
    xs = x.reshape(B, -1)
    var, mean = torch.var_mean(xs, dim=1, keepdim=True, unbiased=False)
    return ((xs - mean) * torch.rsqrt(var + eps)).view_as(x) * weight + bias


class DualComputationBlock(nn.Module):
    def __init__(self, intra_mdl, inter_mdl, out_channels, skip_around_intra=True):
        super().__init__()
        self.intra_mdl, self.inter_mdl = intra_mdl, inter_mdl
        self.skip_around_intra = skip_around_intra
        self.intra_norm = nn.GroupNorm(1, out_channels, eps=1e-8)
        self.inter_norm = nn.GroupNorm(1, out_channels, eps=1e-8)

    def forward(self, x):
        """x: the dual-path state stored channels-last, (B, S, K, N) — the reference's [B, N, K, S] permuted
        so that the intra pass reads (B*S, K, N) without a copy; one S<->K transpose each way for inter."""
        B, S, K, N = x.shape
        intra = self.intra_mdl(x.reshape(B * S, K, N)).view(B, S, K, N)
        intra = _gln_cl(intra, self.intra_norm.weight, self.intra_norm.bias, self.intra_norm.eps)
        if self.skip_around_intra:
            intra = intra + x
        inter = self.inter_mdl(intra.transpose(1, 2).reshape(B * K, S, N)).view(B, K, S, N)
        inter = _gln_cl(inter, self.inter_norm.weight, self.inter_norm.bias, self.inter_norm.eps)
        return intra + inter.transpose(1, 2)             # output takes intra's (B, S, K, N) layout


class DualPathModel(nn.Module):
    def __init__(self, in_channels, out_channels, intra_model, inter_model, num_layers=1, K=200, num_spks=2,
                 skip_around_intra=True):
        super().__init__()
        self.K, self.num_spks, self.num_layers = K, num_spks, num_layers
        self.norm = nn.GroupNorm(1, in_channels, eps=1e-8)
        self.conv1d = nn.Conv1d(in_channels, out_channels, 1, bias=False)
        self.dual_mdl = nn.ModuleList([copy.deepcopy(DualComputationBlock(intra_model, inter_model, out_channels,
                                                                          skip_around_intra))
                                       for _ in range(num_layers)])
        self.conv2d = nn.Conv2d(out_channels, out_channels * num_spks, kernel_size=1)
        self.end_conv1x1 = nn.Conv1d(out_channels, in_channels, 1, bias=False)
        self.prelu = nn.PReLU()
        self.activation = nn.ReLU()
        self.output = nn.Sequential(nn.Conv1d(out_channels, out_channels, 1), nn.Tanh())
        self.output_gate = nn.Sequential(nn.Conv1d(out_channels, out_channels, 1), nn.Sigmoid())

    @staticmethod
    def _segmentation(x, K):
        """[B, N, L] -> [B, N, K, S] chunks of K with 50 % overlap, zero padded (returns the tail gap)."""
        B, N, L = x.shape
        P = K // 2
        gap = K - (P + L % K) % K
        x = F.pad(x, (P, gap + P))
        x1 = x[:, :, :-P].reshape(B, N, -1, K)
        x2 = x[:, :, P:].reshape(B, N, -1, K)
        return torch.cat([x1, x2], dim=3).view(B, N, -1, K).transpose(2, 3).contiguous(), gap

    @staticmethod
    def _over_add(x, gap):
        """[B, N, K, S] -> [B, N, L]: overlap-add of the 50 %-overlapping chunks."""
        B, N, K, S = x.shape
        P = K // 2
        x = x.transpose(2, 3).contiguous().view(B, N, -1, K * 2)
        x1 = x[:, :, :, :K].contiguous().view(B, N, -1)[:, :, P:]
        x2 = x[:, :, :, K:].contiguous().view(B, N, -1)[:, :, :-P]
        x = x1 + x2
        return x[:, :, :-gap] if gap > 0 else x

    def forward(self, x):                                   # [B, N, L] -> [spks, B, N, L]
        x = self.conv1d(self.norm(x))
        x, gap = self._segmentation(x, self.K)
        x = x.permute(0, 3, 2, 1).contiguous()              # [B, N, K, S] -> channels-last (B, S, K, N)
        for blk in self.dual_mdl:
            x = blk(x)
        x = self.conv2d(self.prelu(x.permute(0, 3, 2, 1)))  # [B, N*spks, K, S]
        B, _, K, S = x.shape
        x = self._over_add(x.view(B * self.num_spks, -1, K, S), gap)
        x = self.end_conv1x1(self.output(x) * self.output_gate(x))
        _, N, L = x.shape
        return self.activation(x.view(B, self.num_spks, N, L)).transpose(0, 1)


class DPMambaTasNet(nn.Module):
    """Encoder / DualPathModel(MambaBlocksSequential intra + inter) / Decoder (train_wsj0mix.py:86-111)."""

    def __init__(self, N=512, n_dp=16, skip_around_intra=True, kernel_size=16, chunk_size=250, n_spk=2,
                 n_mamba_dp=2, d_state=16, expand=2, d_conv=4):
        super().__init__()
        self.num_spks = n_spk
        self.encoder = Encoder(kernel_size, N)
        blocks = MambaBlocksSequential(n_mamba_dp // 2, N, d_state, expand, d_conv)
        self.masknet = DualPathModel(N, N, blocks, copy.deepcopy(blocks), n_dp, chunk_size, n_spk, skip_around_intra)
        self.decoder = Decoder(N, 1, kernel_size, stride=kernel_size // 2, bias=False)

    def forward(self, mix):                                 # (B, T) -> (B, T, n_spk)
        mix_w = self.encoder(mix)
        est_mask = self.masknet(mix_w)
        sep_h = mix_w.unsqueeze(0) * est_mask
        est = torch.stack([self.decoder(sep_h[i]) for i in range(self.num_spks)], dim=-1)
        T = mix.shape[1]
        if T > est.shape[1]:
            return F.pad(est, (0, 0, 0, T - est.shape[1]))
        return est[:, :T, :]
