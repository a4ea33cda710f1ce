"""Training objectives of the three families (vectorised, device-agnostic torch).

cal_si_snr      speechbrain cal_si_snr, in-tree copy baseline/avse2/utils/dnn.py:15-57
si_snr_pit      speechbrain get_si_snr_with_pitwrapper (Mamba-TasNet hparams :162):
                min over speaker permutations of the mean pairwise -SI-SNR, per utterance
avse4_loss      baseline/avse4/model.py:374-383 (-SI-SNR clamped at -30 from below, mean)
"""
import itertools

import torch

EPS = 1e-8


def cal_si_snr(source, estimate):
    """[T, B, C] -> [1, B, C] negative SI-SNR (dB)."""
    T = source.shape[0]
    s = source - source.sum(0, keepdim=True) / T
    e = estimate - estimate.sum(0, keepdim=True) / T
    dot = (e * s).sum(0, keepdim=True)
    proj = dot * s / ((s * s).sum(0, keepdim=True) + EPS)
    noise = e - proj
    ratio = (proj * proj).sum(0) / ((noise * noise).sum(0) + EPS)
    return -(10 * torch.log10(ratio + EPS)).unsqueeze(0)


def si_snr_pit(targets, preds):
    """targets, preds [B, T, C] -> per-utterance PIT loss [B]."""
    Bn, Tn, C = targets.shape
    # pairwise[b, i, j] = -SI-SNR(target j, pred i)
    t = targets.permute(1, 0, 2)[:, :, None, :].expand(Tn, Bn, C, C)
    p = preds.permute(1, 0, 2)[:, :, :, None].expand(Tn, Bn, C, C)
    pair = cal_si_snr(t.reshape(Tn, Bn, C * C), p.reshape(Tn, Bn, C * C)).reshape(Bn, C, C)
    best = None
    for perm in itertools.permutations(range(C)):
        v = sum(pair[:, perm[j], j] for j in range(C)) / C
        best = v if best is None else torch.minimum(best, v)
    return best


def avse4_loss(clean, pred):
    loss = cal_si_snr(clean.permute(2, 0, 1), pred.permute(2, 0, 1))
    return torch.clamp(loss, min=-30.0).mean()
