"""Drop-in replacements for the un-vendored native packages the reference imports.

``install()`` puts ``_path`` first on sys.path so the reference's own modules import OUR
implementations under the names they already use (no edit to the reference code):

  selective_scan_cuda.fwd / .bwd             selective_scan_interface.py:16,42,67,218,252
  causal_conv1d_cuda.causal_conv1d_fwd/_bwd  selective_scan_interface.py:15,182,244,286
  causal_conv1d.causal_conv1d_fn             selective_scan_interface.py:14; bimamba.py:20
  mamba_ssm.ops.triton.layernorm.RMSNorm,
  rms_norm_fn                                 bimamba.py:35; mamba_blocks.py:17
  mamba_ssm.Mamba (unidirectional; unused by the bidirectional configs) mamba_blocks.py:12

Everything routes to libavse_hip.so; nothing falls back to CPU.
"""
import os
import sys

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_path")


def install():
    if PATH not in sys.path:
        sys.path.insert(0, PATH)
    return PATH
