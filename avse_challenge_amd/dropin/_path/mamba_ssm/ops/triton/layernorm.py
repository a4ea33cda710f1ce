"""Drop-in for mamba_ssm.ops.triton.layernorm (RMSNorm / rms_norm_fn) on libavse_hip.so."""
from avse_challenge_amd.mamba_tasnet import AddRMSNorm, RMSNorm  # noqa: F401


def rms_norm_fn(x, weight, bias, residual=None, prenorm=False, residual_in_fp32=False, eps=1e-6):
    if bias is not None:
        raise NotImplementedError("RMSNorm has no bias")
    y, res = AddRMSNorm.apply(x, residual, weight, eps)
    return (y, res) if prenorm else y


def layer_norm_fn(*args, **kwargs):
    raise NotImplementedError("LayerNorm blocks are not used (rms_norm: True in every Mamba-TasNet config)")
