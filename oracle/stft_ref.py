"""librosa 0.8.1 STFT / iSTFT restated in numpy — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The avse1 path calls (citations relative to /root/reference/baseline/avse1):
  dataset.py:112-118  librosa.stft(noisy, win_length=512, n_fft=512, hop_length=128,
                      window="hann", center=True).T  -> |.| as float32  (376, 257) for 48000 samples
  test.py:85-88       librosa.istft(mag * e^{j angle(noisy_stft)}.T, win_length=512,
                      hop_length=128, window="hann", length=len(clean))
librosa is not vendored and not installed (pinned 0.8.1 in baseline/avse1/requirements.txt).
Restated from librosa 0.8.1's published algorithm: periodic Hann window
(scipy.signal.get_window('hann', 512, fftbins=True)); center=True reflect-pads n_fft//2 both
sides (0.8.1 default pad_mode='reflect'); frames every hop; rfft of window*frame computed in
float64 and stored complex64.  istft: irfft each frame, multiply by the window, overlap-add,
divide by the window-sum-square where it exceeds float tiny, trim n_fft//2 and fix length.
Only the frame count (376, config.py:19) is pinned by the reference: numerics parity unpinned.
"""
import numpy as np

N_FFT, HOP, WIN = 512, 128, 512


def hann_periodic(n=WIN):
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def stft(y, n_fft=N_FFT, hop=HOP):
    """y: (..., T) float -> complex64 (..., 1+n_fft//2, n_frames) like librosa.stft."""
    y = np.asarray(y)
    pad = n_fft // 2
    yp = np.pad(y, [(0, 0)] * (y.ndim - 1) + [(pad, pad)], mode="reflect")
    n_frames = 1 + (yp.shape[-1] - n_fft) // hop
    idx = np.arange(n_fft)[None, :] + hop * np.arange(n_frames)[:, None]
    frames = yp[..., idx]                              # (..., n_frames, n_fft)
    spec = np.fft.rfft(hann_periodic(n_fft) * frames.astype(np.float64), axis=-1)
    return np.swapaxes(spec, -1, -2).astype(np.complex64)


def stft_mag_T(y):
    """The avse1 feature: |stft(y)|.T as float32 -> (..., n_frames, 257)."""
    return np.swapaxes(np.abs(stft(y)), -1, -2).astype(np.float32)


def window_sumsquare(n_frames, n_fft=N_FFT, hop=HOP):
    w2 = hann_periodic(n_fft) ** 2
    out = np.zeros(n_fft + hop * (n_frames - 1), dtype=np.float64)
    for i in range(n_frames):
        out[i * hop:i * hop + n_fft] += w2
    return out


def istft(spec, length=None, n_fft=N_FFT, hop=HOP):
    """spec: (..., 1+n_fft//2, n_frames) complex -> (..., length) float32 like librosa.istft."""
    spec = np.asarray(spec)
    n_frames = spec.shape[-1]
    if length is not None:
        n_frames = min(n_frames, int(np.ceil((length + n_fft) / hop)))
    spec = spec[..., :n_frames]
    frames = np.fft.irfft(np.swapaxes(spec, -1, -2).astype(np.complex128), n=n_fft, axis=-1)
    frames = frames * hann_periodic(n_fft)
    out_len = n_fft + hop * (n_frames - 1)
    y = np.zeros(spec.shape[:-2] + (out_len,), dtype=np.float64)
    for i in range(n_frames):
        y[..., i * hop:i * hop + n_fft] += frames[..., i, :]
    wss = window_sumsquare(n_frames, n_fft, hop)
    nz = wss > np.finfo(np.float32).tiny
    y[..., nz] /= wss[nz]
    start = n_fft // 2
    if length is None:
        y = y[..., start:-start]
    else:
        y = y[..., start:]
        if y.shape[-1] >= length:
            y = y[..., :length]
        else:
            y = np.concatenate([y, np.zeros(y.shape[:-1] + (length - y.shape[-1],))], axis=-1)
    return y.astype(np.float32)
