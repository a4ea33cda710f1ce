"""The drop-in operator boundary, executed: the reference's call sequences into the native modules it imports
(selective_scan_cuda, causal_conv1d_cuda, causal_conv1d.causal_conv1d_fn, mamba_ssm's rms_norm_fn / RMSNorm),
resolved through ``avse_challenge_amd.dropin.install()`` to libavse_hip.so.

The callers are RESTATED here (the reference cannot travel to the GPU box), statement for statement:
  MambaInnerFnNoOutProj.forward / .backward   Mamba-TasNet/modules/mamba/selective_scan_interface.py:160-294
  SelectiveScanFn.forward / .backward          selective_scan_interface.py:18-80
  Mamba.forward (v2 fast path)                 modules/mamba/bimamba.py:176-253
  Mamba.forward (slow path, causal_conv1d_fn)  bimamba.py:271-304
  Block.forward (fused_add_norm True / False)  bimamba.py:436-462
including the layouts the reference hands over: ``xz`` from ``rearrange(W @ h^T, "d (b l) -> b d l")`` (strides
(l, b*l, 1)), the non-contiguous ``delta`` from the same rearrange, 4-D ``B`` / ``C``, ``dz`` as a view of
``dxz`` with ``recompute_out_z=True`` and the 9-value unpack, and ``causal_conv1d_bwd(..., dx, True)`` writing
into the ``dx`` half of ``dxz``. ``dxz`` is poisoned with NaN after ``empty_like`` (test instrumentation, not in
the reference) so an in-place write the drop-in misses cannot pass by luck. Results are compared with the
golden vectors generated from the reference (tests/golden/bimamba_block, mamba_unidir) and with fp64 autograd
through the oracle.
"""
import importlib
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F
from einops import rearrange

from conftest import load_golden
from oracle import mamba_ref
from oracle.det_init import det_init_, det_input

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _fp32_exact():
    torch.backends.cuda.matmul.allow_tf32 = False
    yield


@pytest.fixture(scope="module")
def natives():
    from avse_challenge_amd import dropin
    path = dropin.install()
    names = ("selective_scan_cuda", "causal_conv1d_cuda", "causal_conv1d", "mamba_ssm.ops.triton.layernorm")
    mods = {}
    for n in names:
        sys.modules.pop(n, None)
        mods[n] = importlib.import_module(n)
        assert mods[n].__file__.startswith(path), (n, mods[n].__file__)
    yield mods
    sys.path.remove(path)


def close(a, b, atol, rtol=0.0, what=""):
    a = a.detach().double().cpu().numpy()
    b = b.detach().double().cpu().numpy() if torch.is_tensor(b) else np.asarray(b, np.float64)
    np.testing.assert_allclose(a, b, atol=atol, rtol=rtol, err_msg=what)


def make_inner_fn(ssc, ccc, trace):
    """MambaInnerFnNoOutProj restated (selective_scan_interface.py:160-294; B, C input-dependent, no B/C proj
    bias, delta_softplus=True, checkpoint_lvl=1). ``trace`` records the buffers handed over in place."""

    class MambaInnerFnNoOutProj(torch.autograd.Function):
        @staticmethod
        def forward(ctx, xz, conv1d_weight, conv1d_bias, x_proj_weight, delta_proj_weight, A, D, delta_bias):
            L = xz.shape[-1]
            delta_rank = delta_proj_weight.shape[1]
            d_state = A.shape[-1]
            if torch.is_autocast_enabled():
                x_proj_weight = x_proj_weight.to(dtype=torch.get_autocast_dtype("cuda"))
                delta_proj_weight = delta_proj_weight.to(dtype=torch.get_autocast_dtype("cuda"))
            if xz.stride(-1) != 1:
                xz = xz.contiguous()
            conv1d_weight = rearrange(conv1d_weight, "d 1 w -> d w")
            x, z = xz.chunk(2, dim=1)
            conv1d_bias = conv1d_bias.contiguous()
            conv1d_out = ccc.causal_conv1d_fwd(x, conv1d_weight, conv1d_bias, None, True)
            x_dbl = F.linear(rearrange(conv1d_out, "b d l -> (b l) d"), x_proj_weight)
            delta = rearrange(delta_proj_weight @ x_dbl[:, :delta_rank].t(), "d (b l) -> b d l", l=L)
            trace["delta_contiguous"] = delta.is_contiguous()
            B = rearrange(x_dbl[:, delta_rank:delta_rank + d_state], "(b l) dstate -> b 1 dstate l", l=L).contiguous()
            C = rearrange(x_dbl[:, -d_state:], "(b l) dstate -> b 1 dstate l", l=L).contiguous()
            D = D.contiguous()
            out, scan_intermediates, out_z = ssc.fwd(conv1d_out, delta, A, B, C, D, z, delta_bias, True)
            ctx.save_for_backward(xz, conv1d_weight, conv1d_bias, x_dbl, x_proj_weight, delta_proj_weight,
                                  A, B, C, D, delta_bias, scan_intermediates, out)
            return out_z

        @staticmethod
        def backward(ctx, dout):
            (xz, conv1d_weight, conv1d_bias, x_dbl, x_proj_weight, delta_proj_weight,
             A, B, C, D, delta_bias, scan_intermediates, out) = ctx.saved_tensors
            L = xz.shape[-1]
            delta_rank = delta_proj_weight.shape[1]
            d_state = A.shape[-1]
            x, z = xz.chunk(2, dim=1)
            if dout.stride(-1) != 1:
                dout = dout.contiguous()
            conv1d_out = ccc.causal_conv1d_fwd(x, conv1d_weight, conv1d_bias, None, True)
            delta = rearrange(delta_proj_weight @ x_dbl[:, :delta_rank].t(), "d (b l) -> b d l", l=L)
            dxz = torch.empty_like(xz)
            dxz.fill_(float("nan"))                     # instrumentation: a missed in-place write stays NaN
            dx, dz = dxz.chunk(2, dim=1)
            res = ssc.bwd(conv1d_out, delta, A, B, C, D, z, delta_bias, dout, scan_intermediates, out, dz,
                          True, True)
            dconv1d_out, ddelta, dA, dB, dC, dD, ddelta_bias, dz_ret, out_z = res      # 9-value unpack (:252)
            trace["dz_in_place"] = dz_ret.data_ptr() == dz.data_ptr()
            trace["recomputed_out_z"] = out_z
            dx_dbl = torch.empty_like(x_dbl)
            dB = rearrange(dB, "b 1 dstate l -> (b l) dstate").contiguous()
            dx_dbl[:, delta_rank:delta_rank + d_state] = dB
            dC = rearrange(dC, "b 1 dstate l -> (b l) dstate").contiguous()
            dx_dbl[:, -d_state:] = dC
            ddelta = rearrange(ddelta, "b d l -> d (b l)")
            ddelta_proj_weight = torch.einsum("dB,Br->dr", ddelta, x_dbl[:, :delta_rank])
            dx_dbl[:, :delta_rank] = torch.einsum("dB,dr->Br", ddelta, delta_proj_weight)
            dconv1d_out = rearrange(dconv1d_out, "b d l -> d (b l)")
            dx_proj_weight = torch.einsum("Br,Bd->rd", dx_dbl, rearrange(conv1d_out, "b d l -> (b l) d"))
            dconv1d_out = torch.addmm(dconv1d_out, x_proj_weight.t(), dx_dbl.t(), out=dconv1d_out)
            dconv1d_out = rearrange(dconv1d_out, "d (b l) -> b d l", b=x.shape[0], l=x.shape[-1])
            dx_ret, dconv1d_weight, dconv1d_bias = ccc.causal_conv1d_bwd(x, conv1d_weight, conv1d_bias,
                                                                         dconv1d_out, None, dx, True)
            trace["dx_in_place"] = dx_ret.data_ptr() == dx.data_ptr()
            trace["dxz_finite"] = bool(torch.isfinite(dxz).all())
            dconv1d_weight = rearrange(dconv1d_weight, "d w -> d 1 w")
            return dxz, dconv1d_weight, dconv1d_bias, dx_proj_weight, ddelta_proj_weight, dA, dD, ddelta_bias

    return MambaInnerFnNoOutProj.apply


def mamba_v2_forward(p, h, inner):
    """bimamba.py:176-253 (v2 fast path, if_devide_out=True) over parameter dict ``p`` (keys 'mixer.*')."""
    seqlen = h.shape[1]
    xz = rearrange(p["mixer.in_proj.weight"] @ rearrange(h, "b l d -> d (b l)"), "d (b l) -> b d l", l=seqlen)
    A = -torch.exp(p["mixer.A_log"].float())
    A_b = -torch.exp(p["mixer.A_b_log"].float())
    out = inner(xz, p["mixer.conv1d.weight"], p["mixer.conv1d.bias"], p["mixer.x_proj.weight"],
                p["mixer.dt_proj.weight"], A, p["mixer.D"].float(), p["mixer.dt_proj.bias"].float())
    out_b = inner(xz.flip([-1]), p["mixer.conv1d_b.weight"], p["mixer.conv1d_b.bias"], p["mixer.x_proj_b.weight"],
                  p["mixer.dt_proj_b.weight"], A_b, p["mixer.D_b"].float(), p["mixer.dt_proj_b.bias"].float())
    return F.linear(rearrange(0.5 * out + 0.5 * out_b.flip([-1]), "b d l -> b l d"), p["mixer.out_proj.weight"])


def _block_params(seed=12):
    from avse_challenge_amd import mamba_tasnet as M
    blk = det_init_(M.Block(32, M.BiMambaV2(32)), seed).to(DEV)
    return blk, dict(blk.named_parameters())


@pytest.mark.parametrize("fused_add_norm", [False, True])
def test_block_v2_through_dropins_vs_golden(natives, fused_add_norm):
    """bimamba.Block (Mamba v2, RMSNorm eps 1e-5) with every native call going through the drop-ins; outputs and
    all gradients vs the reference-generated golden ``bimamba_block``."""
    g = load_golden("bimamba_block")
    ln = natives["mamba_ssm.ops.triton.layernorm"]
    trace = {}
    inner = make_inner_fn(natives["selective_scan_cuda"], natives["causal_conv1d_cuda"], trace)
    blk, p = _block_params()
    hs = torch.from_numpy(g["hidden"]).to(DEV).requires_grad_(True)
    res = torch.from_numpy(g["residual"]).to(DEV).requires_grad_(True)
    if fused_add_norm:       # bimamba.py:452-461
        h, r = ln.rms_norm_fn(hs, p["norm.weight"], None, residual=res, prenorm=True, residual_in_fp32=False,
                              eps=1e-5)
    else:                    # bimamba.py:446-450 with the drop-in RMSNorm module
        norm = ln.RMSNorm(32, eps=1e-5).to(DEV)
        norm.weight = p["norm.weight"]
        r = hs + res
        h = norm(r.to(dtype=norm.weight.dtype))
    out = mamba_v2_forward(p, h, inner)
    close(out, g["out_hidden"], 2e-5, 1e-5, "hidden")
    close(r, g["out_residual"], 1e-6, 0, "residual")
    (out * torch.from_numpy(g["gout"]).to(DEV)).sum().backward()
    assert trace == {**trace, "delta_contiguous": False, "dz_in_place": True, "dx_in_place": True, "dxz_finite": True}
    assert trace["recomputed_out_z"] is not None
    close(hs.grad, g["g_hidden"], 5e-5, 1e-4, "g_hidden")
    close(res.grad, g["g_residual"], 5e-5, 1e-4, "g_residual")
    for k, v in p.items():
        ref = g["g_" + k.replace(".", "__")]
        close(v.grad, ref, 1e-4 * max(1.0, float(np.abs(ref).max())), 1e-4, k)


def test_rms_norm_fn_first_layer_and_prenorm_flag(natives):
    """rms_norm_fn with residual=None (first Block) and prenorm False / True vs the oracle RMSNorm."""
    ln = natives["mamba_ssm.ops.triton.layernorm"]
    x = det_input((3, 50, 32), 1501).to(DEV)
    w = (1 + 0.1 * det_input((32,), 1502)).to(DEV)
    y = ln.rms_norm_fn(x, w, None, eps=1e-5)
    y2, r2 = ln.rms_norm_fn(x, w, None, residual=None, prenorm=True, eps=1e-5)
    ref = mamba_ref.rms_norm(x.double().cpu(), w.double().cpu(), 1e-5)
    close(y, ref, 1e-6, 1e-6, "prenorm=False")
    close(y2, ref, 1e-6, 1e-6, "prenorm=True")
    close(r2, x, 0, 0, "residual out == input")


def test_selective_scan_fn_and_causal_conv1d_fn_slow_path_vs_golden(natives):
    """bimamba.py:271-304 slow path (causal_conv1d_fn + selective_scan_fn with 3-D B / C) for the forward direction
    of a Mamba(d_model 32, v2 params) vs the reference-generated golden ``mamba_unidir``; gradients of every input of
    the path vs fp64 autograd through the oracle."""
    ssc, cc = natives["selective_scan_cuda"], natives["causal_conv1d"]

    class SelectiveScanFn(torch.autograd.Function):          # selective_scan_interface.py:18-80 (restated)
        @staticmethod
        def forward(ctx, u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False):
            if u.stride(-1) != 1:
                u = u.contiguous()
            if delta.stride(-1) != 1:
                delta = delta.contiguous()
            D = D.contiguous() if D is not None else None
            B = B.contiguous() if B.stride(-1) != 1 else B
            C = C.contiguous() if C.stride(-1) != 1 else C
            if z is not None and z.stride(-1) != 1:
                z = z.contiguous()
            ctx.squeeze_B = B.dim() == 3
            ctx.squeeze_C = C.dim() == 3
            B = rearrange(B, "b dstate l -> b 1 dstate l") if B.dim() == 3 else B
            C = rearrange(C, "b dstate l -> b 1 dstate l") if C.dim() == 3 else C
            out, x, *rest = ssc.fwd(u, delta, A, B, C, D, z, delta_bias, delta_softplus)
            ctx.delta_softplus = delta_softplus
            ctx.save_for_backward(u, delta, A, B, C, D, z, delta_bias, x, out)
            return rest[0]

        @staticmethod
        def backward(ctx, dout):
            u, delta, A, B, C, D, z, delta_bias, x, out = ctx.saved_tensors
            dout = dout.contiguous() if dout.stride(-1) != 1 else dout
            du, ddelta, dA, dB, dC, dD, ddelta_bias, *rest = ssc.bwd(u, delta, A, B, C, D, z, delta_bias, dout, x,
                                                                     out, None, ctx.delta_softplus, False)
            dz = rest[0]
            dB = dB.squeeze(1) if ctx.squeeze_B else dB
            dC = dC.squeeze(1) if ctx.squeeze_C else dC
            return du, ddelta, dA, dB, dC, dD, dz, ddelta_bias, None

    g = load_golden("mamba_unidir")
    from avse_challenge_amd import mamba_tasnet as M
    m = det_init_(M.BiMambaV2(32), 11).to(DEV)
    h = torch.from_numpy(g["h"]).to(DEV).requires_grad_(True)
    seqlen = h.shape[1]
    xz = rearrange(m.in_proj.weight @ rearrange(h, "b l d -> d (b l)"), "d (b l) -> b d l", l=seqlen)
    x, z = xz.chunk(2, dim=1)
    x = cc.causal_conv1d_fn(x=x, weight=rearrange(m.conv1d.weight, "d 1 w -> d w"), bias=m.conv1d.bias,
                            activation="silu")
    x_dbl = m.x_proj(rearrange(x, "b d l -> (b l) d"))
    dt, B, C = torch.split(x_dbl, [m.dt_rank, 16, 16], dim=-1)
    dt = rearrange(m.dt_proj.weight @ dt.t(), "d (b l) -> b d l", l=seqlen)
    B = rearrange(B, "(b l) dstate -> b dstate l", l=seqlen).contiguous()
    C = rearrange(C, "(b l) dstate -> b dstate l", l=seqlen).contiguous()
    y = SelectiveScanFn.apply(x, dt, -torch.exp(m.A_log.float()), B, C, m.D.float(), z, m.dt_proj.bias.float(), True)
    out = m.out_proj(rearrange(y, "b d l -> b l d"))
    close(out, g["y"], 2e-5, 1e-5, "y")
    gy = det_input(tuple(out.shape), 1503).to(DEV)
    (out * gy).sum().backward()
    # fp64 oracle of the same path (F.conv1d causal conv, sequential scan) on the same weights
    md = det_init_(M.BiMambaV2(32), 11).double()
    hd = torch.from_numpy(g["h"]).double().requires_grad_(True)
    xzd = F.linear(hd, md.in_proj.weight).transpose(1, 2)
    xd, zd = xzd.chunk(2, 1)
    xd = mamba_ref.causal_conv1d(xd, md.conv1d.weight[:, 0], md.conv1d.bias, silu=True)
    xdb = xd.transpose(1, 2).reshape(-1, xd.shape[1]) @ md.x_proj.weight.t()
    r = md.dt_rank
    dtd = (md.dt_proj.weight @ xdb[:, :r].t()).reshape(-1, 2, seqlen).transpose(0, 1)
    Bd = xdb[:, r:r + 16].reshape(2, seqlen, 16).transpose(1, 2)
    Cd = xdb[:, r + 16:].reshape(2, seqlen, 16).transpose(1, 2)
    yd = mamba_ref.selective_scan(xd, dtd, -torch.exp(md.A_log), Bd, Cd, md.D, zd, md.dt_proj.bias, True,
                                  acc_dtype=torch.float64)
    outd = F.linear(yd.transpose(1, 2), md.out_proj.weight)
    (outd * gy.double().cpu()).sum().backward()
    close(h.grad, hd.grad, 1e-5, 1e-4, "dh")
    for (k, p_), (_, q) in zip(m.named_parameters(), md.named_parameters()):
        if q.grad is None:                       # backward-direction parameters: unused on this path
            assert p_.grad is None, k
            continue
        close(p_.grad, q.grad, 1e-5 * max(1.0, float(q.grad.abs().max())), 1e-4, k)


def test_block_v2_dropins_under_bf16_autocast(natives):
    """The same restated Block under bf16 autocast (x_proj / dt_proj weights cast as :174-176, bf16 u / delta / z /
    B / C, dB / dC returned in B's dtype): gradients finite and cosine > 0.99 with the fp32 run."""
    ln = natives["mamba_ssm.ops.triton.layernorm"]
    runs = []
    for bf16 in (False, True):
        trace = {}
        inner = make_inner_fn(natives["selective_scan_cuda"], natives["causal_conv1d_cuda"], trace)
        blk, p = _block_params(13)
        hs = det_input((2, 300, 32), 1504).to(DEV)
        res = det_input((2, 300, 32), 1505).to(DEV)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16, cache_enabled=False):
            h, r = ln.rms_norm_fn(hs, p["norm.weight"], None, residual=res, prenorm=True, eps=1e-5)
            out = mamba_v2_forward(p, h, inner)
        out.float().pow(2).mean().backward()
        assert trace["dz_in_place"] and trace["dx_in_place"] and trace["dxz_finite"], trace
        runs.append({k: v.grad.detach().double().clone() for k, v in p.items()})
    for k in runs[0]:
        a, b = runs[0][k].reshape(-1), runs[1][k].reshape(-1)
        assert torch.isfinite(b).all(), k
        cos = float(torch.dot(a, b) / (a.norm() * b.norm()))
        assert cos > 0.99, (k, cos)
