"""Deterministic, key-name-driven parameter initialisation — TEST INFRASTRUCTURE ONLY.

Golden fixtures for large modules (ResNet-18 lip encoders, full AVNet) would
be tens of MB if we stored weights.  Instead both the reference module (in the
build container, when the goldens are made) and the restated / HIP modules
(in tests, on any box) are filled by this function, which derives every tensor
from its state_dict KEY and SHAPE only.  Two modules with identical state_dict
keys and shapes therefore get bit-identical weights, which also proves the
checkpoint-key compatibility the drop-in boundary promises.
"""
import math
import zlib

import torch


def _gen(seed: int, key: str) -> torch.Generator:
    g = torch.Generator()
    g.manual_seed((seed * 1000003 + zlib.crc32(key.encode())) & 0x7FFFFFFF)
    return g


def det_tensor(key: str, shape, seed: int = 0) -> torch.Tensor:
    """Value for state_dict entry ``key`` of ``shape`` (fp32, CPU)."""
    g = _gen(seed, key)
    shape = tuple(shape)
    leaf = key.rsplit(".", 1)[-1]
    n = 1
    for s in shape:
        n *= s
    if leaf == "num_batches_tracked":
        return torch.zeros(shape, dtype=torch.long)
    if leaf == "running_mean":
        return 0.1 * torch.randn(shape, generator=g)
    if leaf == "running_var":
        return 0.5 + torch.rand(shape, generator=g)
    if leaf in ("A_log", "A_b_log"):
        d, ns = shape
        base = torch.log(torch.arange(1, ns + 1, dtype=torch.float32)).expand(d, ns)
        return (base + 0.1 * torch.randn(shape, generator=g)).contiguous()
    if leaf in ("D", "D_b"):
        return 1.0 + 0.1 * torch.randn(shape, generator=g)
    if "dt_proj" in key and leaf == "bias":
        # softplus^-1 of dt in [1e-3, 1e-1] as Mamba initialises it (bimamba.py:111-117)
        dt = torch.exp(torch.rand(shape, generator=g) * (math.log(0.1) - math.log(1e-3)) + math.log(1e-3))
        return dt + torch.log(-torch.expm1(-dt))
    if leaf == "weight" and len(shape) == 1:
        # norm scales (BN / RMSNorm / LayerNorm) and PReLU slopes share one rule
        return 0.2 + torch.rand(shape, generator=g)
    if leaf in ("gamma",):
        return 1.0 + 0.1 * torch.randn(shape, generator=g)
    if leaf in ("beta", "bias"):
        return 0.1 * torch.randn(shape, generator=g)
    # conv / linear / lstm weights: fan-in scaled normal
    if len(shape) >= 2:
        fan_in = n // shape[0]
        return torch.randn(shape, generator=g) / math.sqrt(max(fan_in, 1))
    return 0.1 * torch.randn(shape, generator=g)


@torch.no_grad()
def det_init_(module: torch.nn.Module, seed: int = 0) -> torch.nn.Module:
    """Fill every parameter and buffer of ``module`` from its key and shape."""
    sd = module.state_dict(keep_vars=True)
    new, first_key = {}, {}
    for k, v in sd.items():
        # aliased sub-modules (avse1 TemporalBlock.net re-lists conv1/bn1/...) appear under
        # several keys; every alias gets the value of the FIRST key so load order is irrelevant
        ptr = (v.data_ptr(), tuple(v.shape)) if v.numel() else (id(v), ())
        src = first_key.setdefault(ptr, k)
        new[k] = det_tensor(src, v.shape, seed).to(v.dtype)
    module.load_state_dict(new, strict=True)
    return module


def det_input(shape, seed: int, kind: str = "normal", scale: float = 1.0) -> torch.Tensor:
    g = torch.Generator()
    g.manual_seed(seed)
    if kind == "normal":
        return scale * torch.randn(shape, generator=g)
    if kind == "uniform":
        return scale * torch.rand(shape, generator=g)
    if kind == "uint8":
        return torch.randint(0, 256, shape, generator=g, dtype=torch.uint8)
    raise ValueError(kind)
