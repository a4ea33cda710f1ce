"""avse_challenge_amd — MI355X-native hot path of shangfuu/avse_challenge.

Hand-written gfx950 HIP kernels (libavse_hip.so, C ABI in include/avse_hip.h) behind the
reference's operator / module surfaces:
  kernels        torch wrappers of the C ABI (selective scan, causal conv1d, add+RMSNorm, STFT/iSTFT)
  dropin         importable stand-ins for selective_scan_cuda / causal_conv1d(_cuda) / mamba_ssm
  mamba_tasnet   Mamba-TasNet separator (Encoder, MaskNet of BiMamba v2 blocks, Decoder)
  avse1          avse1 AVNet with the STFT front-end / iSTFT back-end on the GPU
  losses, data   SI-SNR / PIT objectives; synthetic GPU-resident batches
"""
__version__ = "0.1.0"
