"""Drop-in for ``causal_conv1d`` (causal_conv1d_fn with autograd) on libavse_hip.so."""
import torch

from avse_challenge_amd import kernels as _K


class _CausalConv1dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, silu):
        ctx.save_for_backward(x, weight, bias)
        ctx.silu = silu
        return _K.causal_conv1d_fwd(x, weight, bias, silu)

    @staticmethod
    def backward(ctx, dout):
        x, weight, bias = ctx.saved_tensors
        dx, dw, db = _K.causal_conv1d_bwd(x, weight, bias, dout, silu=ctx.silu)
        return dx, dw.view_as(weight), db, None


def causal_conv1d_fn(x, weight, bias=None, seq_idx=None, activation=None):
    if activation not in (None, "silu", "swish"):
        raise NotImplementedError("activation must be None, 'silu' or 'swish'")
    if seq_idx is not None:
        raise NotImplementedError("seq_idx is not used by the reference path")
    return _CausalConv1dFn.apply(x, weight, bias, activation in ("silu", "swish"))


def causal_conv1d_update(*args, **kwargs):
    raise NotImplementedError("single-token decode (causal_conv1d_update) is outside the training/eval hot path")
