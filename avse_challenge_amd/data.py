"""Synthetic, GPU-resident inputs shaped like the reference datasets.

clean  = 0.1 * N(0,1) shaped by a 4 Hz syllabic envelope |sin(2*pi*4*t + phi)|
noise  = 0.1 * N(0,1) scaled to an SNR drawn from {0, 3, 6, 9} dB (baseline/avse1/config.py:4)
noisy  = clip(clean + noise, -1, 1)
lips   avse1: raw uint8 RGB (B, 3, 75, H, W) (baseline/avse1/dataset.py:150-153, model.py:122)
       avse4: float gray in [0, 1) (B, 1, T_v, 112, 112) (baseline/avse4/dataset.py:161-164)
Each rank draws from its own seeded generator (no data movement between ranks).
"""
import math

import torch

SNRS_DB = (0.0, 3.0, 6.0, 9.0)


def _gen(device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


def speech_like(B, T, sr, device, g, channels=None):
    t = torch.arange(T, device=device, dtype=torch.float32) / sr
    phi = 2 * math.pi * torch.rand((B, 1), device=device, generator=g)
    env = torch.sin(2 * math.pi * 4.0 * t[None, :] + phi).abs()
    shape = (B, T) if channels is None else (B, channels, T)
    x = 0.1 * torch.randn(shape, device=device, generator=g)
    return x * (env if channels is None else env[:, None, :])


def noisy_mixture(clean, g):
    B = clean.shape[0]
    noise = 0.1 * torch.randn(clean.shape, device=clean.device, generator=g)
    snr = torch.tensor(SNRS_DB, device=clean.device)[torch.randint(0, 4, (B,), device=clean.device, generator=g)]
    dims = tuple(range(1, clean.dim()))
    pc = clean.pow(2).mean(dims, keepdim=True)
    pn = noise.pow(2).mean(dims, keepdim=True)
    scale = torch.sqrt(pc / (pn * torch.pow(10.0, snr.view(-1, *([1] * (clean.dim() - 1))) / 10.0)))
    return torch.clamp(clean + noise * scale, -1.0, 1.0 - 2 ** -15)


def avse1_batch(B, device, seed, lip_hw=96, T=48000, frames=75):
    g = _gen(device, seed)
    clean = speech_like(B, T, 16000, device, g)
    noisy = noisy_mixture(clean, g)
    lips = torch.randint(0, 256, (B, 3, frames, lip_hw, lip_hw), device=device, generator=g, dtype=torch.uint8)
    return noisy, clean, lips


def avse4_batch(B, device, seed, T=80000, frames=125, channels=2):
    g = _gen(device, seed)
    clean = speech_like(B, T, 16000, device, g, channels)
    noisy = noisy_mixture(clean, g)
    vis = torch.rand((B, 1, frames, 112, 112), device=device, generator=g)
    return {"noisy_audio": noisy, "clean": clean, "vis_feat": vis}


def wsj0mix_batch(B, device, seed, T=32000):
    g = _gen(device, seed)
    s1 = speech_like(B, T, 8000, device, g)
    s2 = speech_like(B, T, 8000, device, g)
    return s1 + s2, torch.stack([s1, s2], dim=-1)
