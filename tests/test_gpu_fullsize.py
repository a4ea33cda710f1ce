"""North-star parity at the BASELINE utterance sizes (BASELINE.json north_star: "outputs match the
reference PyTorch-CPU path on identical inputs within 1e-4 RMS waveform error (SI-SDR within 0.01 dB)").

The HIP path and the CPU oracle (fp64, the reference semantics pinned by tests/golden) get identical
det_init weights and identical synthetic speech-like inputs (avse_challenge_amd/data.py) at the configs'
full utterance sizes; each test compares the output WAVEFORMS:
  * RMS(ours - oracle) <= 1e-4 * max(1, RMS(oracle))
  * |SI-SDR(clean, ours) - SI-SDR(clean, oracle)| <= 0.01 dB per utterance (and per channel / speaker).
C2 avse1: STFT -> AVNet -> iSTFT with the noisy phase (test.py:79-89), 3 s @ 16 kHz, lips 3x75x96x96.
C4 avse4: binaural 2 x 5 s @ 16 kHz + 125 lip frames 112x112 (model.py:316-321).
C3 Mamba-TasNet-L: 4 s @ 8 kHz (L = 3999 frames) at full width (N = 512, d_inner 1024); the depth is
cut to 4 of the 32 BiMamba layers so the fp64 CPU oracle (a Python loop over time) finishes in seconds.
"""
import numpy as np
import pytest
import torch

from oracle import avse1_ref, avse4_ref, mamba_ref, stft_ref
from oracle.det_init import det_init_
from oracle.losses_ref import si_sdr_db

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _fp32_exact():
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    torch.set_num_threads(16)
    yield


def check_waveforms(est, ref, clean, what):
    """est / ref / clean: (..., T); RMS and SI-SDR bars of the north star."""
    est, ref, clean = est.double().cpu(), ref.double().cpu(), clean.double().cpu()
    rms = float((est - ref).pow(2).mean().sqrt())
    bar = 1e-4 * max(1.0, float(ref.pow(2).mean().sqrt()))
    assert rms <= bar, f"{what}: RMS waveform error {rms:.3e} > {bar:.1e}"
    d = (si_sdr_db(clean, est) - si_sdr_db(clean, ref)).abs()
    assert float(d.max()) <= 0.01, f"{what}: SI-SDR differs by {float(d.max()):.4f} dB"
    print(f"\n{what}: RMS error {rms:.2e} (bar {bar:.1e}), max |dSI-SDR| {float(d.max()):.2e} dB, "
          f"SI-SDR ours {si_sdr_db(clean, est).flatten().tolist()}")
    return rms, float(d.max())


def test_avse1_enhance_fullsize():
    from avse_challenge_amd import avse1, data
    noisy, clean, lips = data.avse1_batch(2, "cpu", 11, lip_hw=96)
    net = det_init_(avse1.AVNet(), 71).to(DEV).eval()
    ref = det_init_(avse1_ref.AVNet(), 71).double().eval()
    est = net.enhance(noisy.to(DEV), lips.to(DEV))                          # (2, 48000)
    spec = stft_ref.stft(noisy.numpy())                                        # (2, 257, 376) complex
    mag_T = np.swapaxes(np.abs(spec), -1, -2).astype(np.float32)               # dataset.py:112-118
    with torch.no_grad():
        pred = ref({"noisy_audio_spec": torch.from_numpy(mag_T).double()[:, None], "lip_images": lips})[:, 0]
    phase = np.angle(spec)
    est_spec = np.swapaxes(pred.numpy(), -1, -2) * (np.cos(phase) + 1j * np.sin(phase))
    ref_wave = torch.from_numpy(stft_ref.istft(est_spec, length=noisy.shape[-1]))
    check_waveforms(est, ref_wave, clean, "avse1 C2")


def test_avse4_fullsize():
    from avse_challenge_amd import avse4, data
    batch = data.avse4_batch(1, "cpu", 12)                                     # 2 x 80000, 125 x 112 x 112
    m = det_init_(avse4.AVSE4BaselineModule(num_channels=2), 72).to(DEV).eval()
    r = det_init_(avse4_ref.AVSE4BaselineModule(num_channels=2), 72).double().eval()
    with torch.no_grad():
        est = m({k: v.to(DEV) for k, v in batch.items()})
        # forward() casts to fp32 (model.py:316-321): call the parts in fp64
        ref = r.model(batch["noisy_audio"].double(), r.visual_frontend(batch["vis_feat"].double()))
    check_waveforms(est, ref, batch["clean"], "avse4 C4")


def test_mamba_tasnet_L_fullsize_4_layers():
    from avse_challenge_amd import data, mamba_tasnet as M
    mix, tgt = data.wsj0mix_batch(1, "cpu", 13)                                # (1, 32000), (1, 32000, 2)
    ours = det_init_(M.MambaTasNet(N=512, n_mamba=4), 73).to(DEV).eval()
    ref = det_init_(mamba_ref.MambaTasNet(N=512, n_mamba=4), 73).double().eval()
    with torch.no_grad():
        est = ours(mix.to(DEV))
        est_r = ref(mix.double())
    # speaker order is the model's own (no PIT needed: same weights); compare per speaker
    check_waveforms(est.transpose(1, 2), est_r.transpose(1, 2), tgt.transpose(1, 2), "Mamba-TasNet-L C3 (4 layers)")


def test_avse1_audio_only_c1_enhance():
    """C1 (BASELINE configs[0]): audio-only AVNet (model.py:117-118) end to end from 3 s waveforms:
    HIP STFT -> AudioFeatNet -> FusionNet LSTM -> HIP iSTFT with the noisy phase (test.py:71-89)."""
    from avse_challenge_amd import avse1, data
    noisy, clean, _ = data.avse1_batch(2, "cpu", 14, lip_hw=8)
    net = det_init_(avse1.AVNet(a_only=True), 74).to(DEV).eval()
    ref = det_init_(avse1_ref.AVNet(a_only=True), 74).double().eval()
    est = net.enhance(noisy.to(DEV), None)
    spec = stft_ref.stft(noisy.numpy())
    mag_T = np.swapaxes(np.abs(spec), -1, -2).astype(np.float32)
    with torch.no_grad():
        pred = ref({"noisy_audio_spec": torch.from_numpy(mag_T).double()[:, None]})[:, 0]
    phase = np.angle(spec)
    est_spec = np.swapaxes(pred.numpy(), -1, -2) * (np.cos(phase) + 1j * np.sin(phase))
    ref_wave = torch.from_numpy(stft_ref.istft(est_spec, length=noisy.shape[-1]))
    check_waveforms(est, ref_wave, clean, "avse1 C1 audio-only")
