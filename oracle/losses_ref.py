"""SI-SNR losses, CPU restatement — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

cal_si_snr        speechbrain nnet.losses.cal_si_snr; in-tree copy baseline/avse2/utils/dnn.py:15-57
                  (pinned by golden vectors): [T, B, C] -> [1, B, C] negative SI-SNR, EPS 1e-8 x3.
si_snr_pit        speechbrain get_si_snr_with_pitwrapper (un-vendored; Mamba-TasNet
                  hparams mambatasnet_L.yaml:162): per utterance, min over speaker
                  permutations of the mean pairwise -SI-SNR — parity unpinned, restated.
avse4_loss        baseline/avse4/model.py:374-383 (clamp at -30, mean).
avse1_loss        baseline/avse1/model.py:164-168 with --loss l1 (train.py:854).
"""
import itertools

import torch
import torch.nn.functional as F

EPS = 1e-8


def cal_si_snr(source, estimate):
    """source, estimate: [T, B, C] -> [1, B, C] (= -SI-SNR dB)."""
    T = source.shape[0]
    mean_t = source.sum(0, keepdim=True) / T
    mean_e = estimate.sum(0, keepdim=True) / T
    s = source - mean_t
    e = estimate - mean_e
    dot = (e * s).sum(0, keepdim=True)
    energy = (s ** 2).sum(0, keepdim=True) + EPS
    proj = dot * s / energy
    noise = e - proj
    ratio = (proj ** 2).sum(0) / ((noise ** 2).sum(0) + EPS)
    return -(10 * torch.log10(ratio + EPS)).unsqueeze(0)


def si_snr_pit(targets, preds):
    """targets, preds: [B, T, C] -> [B] PIT loss."""
    B, T, C = targets.shape
    out = []
    for b in range(B):
        t = targets[b]          # [T, C]
        p = preds[b]
        # pairwise loss_mat[i, j] = -SI-SNR(target j, pred i)
        mat = torch.empty(C, C, dtype=preds.dtype)
        for i in range(C):
            for j in range(C):
                mat[i, j] = cal_si_snr(t[:, j:j + 1, None], p[:, i:i + 1, None]).reshape(())
        best = None
        for perm in itertools.permutations(range(C)):
            v = sum(mat[perm[j], j] for j in range(C)) / C
            best = v if best is None or v < best else best
        out.append(best)
    return torch.stack(out)


def avse4_loss(clean, pred):
    """clean, pred: [B, C, T] -> scalar."""
    loss = cal_si_snr(clean.permute(2, 0, 1), pred.permute(2, 0, 1))
    loss = torch.where(loss < -30, torch.full_like(loss, -30.0), loss)
    return loss.mean()


def avse1_loss(pred_mag, clean_mag):
    return F.l1_loss(pred_mag, clean_mag)


def si_sdr_db(reference, estimate):
    """Scale-invariant SDR in dB over the last axis (parity metric)."""
    reference = reference.double()
    estimate = estimate.double()
    reference = reference - reference.mean(-1, keepdim=True)
    estimate = estimate - estimate.mean(-1, keepdim=True)
    alpha = (estimate * reference).sum(-1, keepdim=True) / (reference.pow(2).sum(-1, keepdim=True) + 1e-12)
    target = alpha * reference
    noise = estimate - target
    return 10 * torch.log10(target.pow(2).sum(-1) / (noise.pow(2).sum(-1) + 1e-20))
