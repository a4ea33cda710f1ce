"""Mamba-TasNet hot path, CPU restatement — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates (citations relative to /root/reference/Mamba-TasNet):
  selective_scan       modules/mamba/selective_scan_interface.py:91-157 (selective_scan_ref)
  causal_conv1d        semantics of causal_conv1d_cuda.causal_conv1d_fwd as pinned by the
                       in-tree fallback modules/mamba/bimamba.py:278-279 (act(conv1d(x)[..., :L]))
  rms_norm             mamba-ssm 1.1.3.post1 ops/triton/layernorm.py RMSNorm (un-vendored;
                       x * rsqrt(mean(x^2) + eps) * w) — parity unpinned, formula restated
  mamba_inner          MambaInnerFnNoOutProj.forward selective_scan_interface.py:164-229
  BiMambaV2            modules/mamba/bimamba.py:39-174 (params), :176-253 (v2 forward)
  Block                modules/mamba/bimamba.py:409-462 (fused_add_norm=False path)
  MambaBlocksSequential modules/mamba_blocks.py:87-212
  ChannelwiseLayerNorm speechbrain 1.0.0 lobes/models/conv_tasnet.py (un-vendored; EPS 1e-8,
                       biased var over channels) — parity unpinned
  MaskNet              modules/mamba_masknet.py:13-139
  Encoder / Decoder    speechbrain dual_path.Encoder/Decoder, in-tree copies
                       baseline/avse2/model.py:14-37
  compute_forward      train_wsj0mix.py:86-111
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------------------- ops

class _ScanFn(torch.autograd.Function):
    """selective_scan with its backward from the explicit adjoint (selective_scan_grads, pinned against the
    reference's autograd gradients by tests/golden/scan_fp32): autograd through the per-step Python loop costs
    O(L^2) (every step's index backward materialises a full-size gradient), which made a CPU train step of a
    Mamba layer take minutes at L ~ 400."""

    @staticmethod
    def forward(ctx, u, delta, A, B, C, D, z, delta_bias, delta_softplus, acc_dtype):
        ctx.save_for_backward(u, delta, A, B, C, D, z, delta_bias)
        ctx.delta_softplus, ctx.acc_dtype = delta_softplus, acc_dtype
        with torch.no_grad():
            return _selective_scan_loop(u, delta, A, B, C, D, z, delta_bias, delta_softplus, False, acc_dtype)

    @staticmethod
    def backward(ctx, dout):
        u, delta, A, B, C, D, z, delta_bias = ctx.saved_tensors
        acc = torch.float64 if ctx.acc_dtype == torch.float64 else torch.float32
        g = selective_scan_grads(u, delta, A, B, C, D, z, delta_bias, ctx.delta_softplus, dout, acc_dtype=acc)
        cast = lambda v, ref: None if (v is None or ref is None) else v.to(ref.dtype)   # noqa: E731
        return (cast(g["du"], u), cast(g["ddelta"], delta), cast(g["dA"], A), cast(g["dB"], B), cast(g["dC"], C),
                cast(g["dD"], D), cast(g["dz"], z), cast(g["ddelta_bias"], delta_bias), None, None)


def _time_major(x):
    """(b, d, n, l) -> contiguous (l, b, d, n)."""
    return x.permute(3, 0, 1, 2).contiguous()


class _one_thread:
    """The per-step loops work on (b, d, n) slabs of a few hundred KB: intra-op threads cost more than they give
    (a C3-sized fp64 scan: 0.42 s on one thread, 2.3 s on eight)."""

    def __enter__(self):
        self.n = torch.get_num_threads()
        torch.set_num_threads(1)

    def __exit__(self, *exc):
        torch.set_num_threads(self.n)


def selective_scan(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                   return_last_state=False, acc_dtype=torch.float32):
    """Sequential recurrence (selective_scan_ref semantics, see _selective_scan_loop); differentiable through the
    explicit adjoint when gradients are needed."""
    ts = [t for t in (u, delta, A, B, C, D, z, delta_bias) if t is not None]
    if not return_last_state and torch.is_grad_enabled() and any(t.requires_grad for t in ts):
        return _ScanFn.apply(u, delta, A, B, C, D, z, delta_bias, delta_softplus, acc_dtype)
    return _selective_scan_loop(u, delta, A, B, C, D, z, delta_bias, delta_softplus, return_last_state, acc_dtype)


def _selective_scan_loop(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                         return_last_state=False, acc_dtype=torch.float32):
    """Sequential recurrence h_t = exp(dt*A) h_{t-1} + dt*B_t*u_t; y_t = <C_t, h_t>.

    u, delta, z: (b, d, l); A: (d, n); B, C: (b, n, l) or (b, g, n, l); D, delta_bias: (d,).
    Follows selective_scan_ref (selective_scan_interface.py:91-157) for real A.
    """
    dtype_in = u.dtype
    u = u.to(acc_dtype)
    dt = delta.to(acc_dtype)
    if delta_bias is not None:
        dt = dt + delta_bias.to(acc_dtype)[:, None]
    if delta_softplus:
        dt = F.softplus(dt)
    b, d, l = u.shape
    n = A.shape[1]
    A = A.to(acc_dtype)

    def expand_t(M):      # time-major (l, b, d|1, n)
        M = M.to(acc_dtype)
        if M.dim() == 3:  # (b, n, l): shared across d
            return M.permute(2, 0, 1)[:, :, None, :].contiguous()
        g = M.shape[1]    # (b, g, n, l): group g serves d/g channels
        if g == 1:
            return M[:, 0].permute(2, 0, 1)[:, :, None, :].contiguous()
        return _time_major(M.repeat_interleave(d // g, dim=1))

    # the per-step operands time-major (l, b, d, n), built in that layout: each step reads contiguous slabs (the same
    # values and elementwise ops as the (b, d, n, l) form of selective_scan_ref)
    dt_t = dt.permute(2, 0, 1).contiguous()[..., None]                           # (l, b, d, 1)
    dA = torch.exp(dt_t * A)                                                      # (l, b, d, n)
    dBu = (dt * u).permute(2, 0, 1).contiguous()[..., None] * expand_t(B)
    Ct = expand_t(C)
    h = torch.zeros(b, d, n, dtype=acc_dtype, device=u.device)
    ys = []
    with _one_thread():
        for t in range(l):
            h = dA[t] * h + dBu[t]
            ys.append((h * Ct[t]).sum(-1))
    y = torch.stack(ys, dim=-1) if l > 0 else torch.zeros(b, d, 0, dtype=acc_dtype, device=u.device)
    out = y if D is None else y + u * D.to(acc_dtype)[:, None]
    if z is not None:
        out = out * F.silu(z.to(acc_dtype))
    out = out.to(dtype_in)
    return (out, h) if return_last_state else out


@torch.no_grad()
def selective_scan_grads(u, delta, A, B, C, D, z, delta_bias, delta_softplus, dout, acc_dtype=torch.float64):
    """Explicit adjoint of ``selective_scan`` — the gradients autograd computes through selective_scan_ref
    (selective_scan_interface.py:91-157), restated as the backward recurrence with O(L) memory (autograd through the
    per-step Python loop is O(L^2) in time: 400 s at L = 5999). Pinned against the reference's autograd gradients by
    tests/golden/scan_fp32 (test_oracle_golden.py). B, C: (b, 1, n, l) or (b, n, l) shared over d.
    Returns dict(du, ddelta, dA, dB, dC, dD, ddelta_bias, dz), dB / dC shaped like B / C."""
    f = lambda t: None if t is None else t.to(acc_dtype)      # noqa: E731
    u, delta, A, D, z, bias, dout = f(u), f(delta), f(A), f(D), f(z), f(delta_bias), f(dout)
    b, d, l = u.shape
    Bx, Cx = f(B), f(C)
    b4 = Bx.dim() == 4
    Bv = Bx[:, 0] if b4 else Bx                               # (b, n, l)
    Cv = Cx[:, 0] if b4 else Cx
    xpre = delta + (bias[:, None] if bias is not None else 0.0)
    dt = F.softplus(xpre) if delta_softplus else xpre         # (b, d, l)
    dA = torch.exp(dt[:, :, None, :] * A[None, :, :, None])    # (b, d, n, l)
    dBu = (dt * u)[:, :, None, :] * Bv[:, None]               # (b, d, n, l)
    # the recurrences run on time-major copies (l, b, d, n): contiguous per-step slabs, same values and ops
    dAt, dBt = _time_major(dA), _time_major(dBu)
    Ht = torch.empty_like(dAt)
    h = torch.zeros(b, d, A.shape[1], dtype=acc_dtype, device=u.device)
    with _one_thread():
        for t in range(l):
            h = dAt[t] * h + dBt[t]
            Ht[t] = h
    H = Ht.permute(1, 2, 3, 0)                                # (b, d, n, l) view
    y = (H * Cv[:, None]).sum(2)                              # (b, d, l)
    out = y + (u * D[:, None] if D is not None else 0.0)
    if z is not None:
        sz = torch.sigmoid(z)
        g = dout * z * sz                                     # d out_z / d out = silu(z)
        dz = dout * out * sz * (1 + z * (1 - sz))
    else:
        g, dz = dout, None
    lamt = torch.empty_like(dAt)
    gt, Cvt = _time_major(g[:, :, None, :]), _time_major(Cv[:, None])   # (l, b, d, 1), (l, b, 1, n)
    acc = torch.zeros(b, d, A.shape[1], dtype=acc_dtype, device=u.device)
    with _one_thread():
        for t in range(l - 1, -1, -1):                        # lambda_t = g_t C_t + dA_{t+1} lambda_{t+1}
            acc = gt[t] * Cvt[t] + acc
            lamt[t] = acc
            acc = acc * dAt[t]
    lam = lamt.permute(1, 2, 3, 0)
    Hprev = torch.cat([torch.zeros_like(H[..., :1]), H[..., :-1]], -1)
    lam_dA_h = lam * dA * Hprev                               # (b, d, n, l)
    dC = (g[:, :, None, :] * H).sum(1)                        # (b, n, l)
    dB = (lam * (dt * u)[:, :, None, :]).sum(1)
    du = (lam * Bv[:, None]).sum(2) * dt + (g * D[:, None] if D is not None else 0.0)
    ddt = (lam_dA_h * A[None, :, :, None]).sum(2) + (lam * Bv[:, None]).sum(2) * u
    dAm = (lam_dA_h * dt[:, :, None, :]).sum((0, 3))
    ddelta = ddt * torch.sigmoid(xpre) if delta_softplus else ddt
    return {"du": du, "ddelta": ddelta, "dA": dAm, "dB": dB[:, None] if b4 else dB, "dC": dC[:, None] if b4 else dC,
            "dD": (g * u).sum((0, 2)) if D is not None else None,
            "ddelta_bias": ddelta.sum((0, 2)) if bias is not None else None, "dz": dz}


def causal_conv1d(x, weight, bias=None, silu=False):
    """Depthwise causal conv: x (b, d, l), weight (d, w), bias (d,) -> (b, d, l)."""
    d, w = weight.shape
    y = F.conv1d(x, weight[:, None, :], bias, padding=w - 1, groups=d)[..., : x.shape[-1]]
    return F.silu(y) if silu else y


def rms_norm(x, weight, eps=1e-5):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * weight.float()).to(x.dtype)


def mamba_inner(xz, conv_w, conv_b, x_proj_w, dt_proj_w, A, D, dt_bias):
    """MambaInnerFnNoOutProj forward (selective_scan_interface.py:164-229): returns out_z (b, d, l)."""
    b, _, l = xz.shape
    r = dt_proj_w.shape[1]
    n = A.shape[1]
    x, z = xz.chunk(2, dim=1)
    xc = causal_conv1d(x, conv_w.reshape(conv_w.shape[0], -1), conv_b, silu=True)
    x_dbl = xc.transpose(1, 2).reshape(b * l, -1) @ x_proj_w.t()           # (bl, r+2n)
    delta = (dt_proj_w @ x_dbl[:, :r].t()).reshape(-1, b, l).transpose(0, 1)  # (b, d, l)
    Bm = x_dbl[:, r:r + n].reshape(b, l, n).transpose(1, 2)[:, None]         # (b, 1, n, l)
    Cm = x_dbl[:, r + n:].reshape(b, l, n).transpose(1, 2)[:, None]
    return selective_scan(xc, delta, A, Bm, Cm, D, z, dt_bias, delta_softplus=True)


# ----------------------------------------------------------------------------- modules

class RMSNorm(nn.Module):
    def __init__(self, dim, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        return rms_norm(x, self.weight, self.eps)


class BiMambaV2(nn.Module):
    """Parameters / keys of bimamba.Mamba with bimamba_type='v2' (bimamba.py:39-174)."""

    def __init__(self, d_model, d_state=16, d_conv=4, expand=2):
        super().__init__()
        self.d_model, self.d_state, self.d_conv = d_model, d_state, d_conv
        self.d_inner = expand * d_model
        self.dt_rank = math.ceil(d_model / 16)
        di, r, n = self.d_inner, self.dt_rank, d_state
        self.in_proj = nn.Linear(d_model, 2 * di, bias=False)
        self.conv1d = nn.Conv1d(di, di, d_conv, groups=di, padding=d_conv - 1, bias=True)
        self.x_proj = nn.Linear(di, r + 2 * n, bias=False)
        self.dt_proj = nn.Linear(r, di, bias=True)
        self.A_log = nn.Parameter(torch.zeros(di, n))
        self.D = nn.Parameter(torch.ones(di))
        self.A_b_log = nn.Parameter(torch.zeros(di, n))
        self.conv1d_b = nn.Conv1d(di, di, d_conv, groups=di, padding=d_conv - 1, bias=True)
        self.x_proj_b = nn.Linear(di, r + 2 * n, bias=False)
        self.dt_proj_b = nn.Linear(r, di, bias=True)
        self.D_b = nn.Parameter(torch.ones(di))
        self.out_proj = nn.Linear(di, d_model, bias=False)

    def forward(self, h):                       # (b, l, d_model), bimamba.py:176-253
        xz = F.linear(h, self.in_proj.weight).transpose(1, 2)            # (b, 2di, l)
        A = -torch.exp(self.A_log.float())
        A_b = -torch.exp(self.A_b_log.float())
        f = mamba_inner(xz, self.conv1d.weight, self.conv1d.bias, self.x_proj.weight,
                        self.dt_proj.weight, A, self.D.float(), self.dt_proj.bias.float())
        bk = mamba_inner(xz.flip(-1), self.conv1d_b.weight, self.conv1d_b.bias, self.x_proj_b.weight,
                         self.dt_proj_b.weight, A_b, self.D_b.float(), self.dt_proj_b.bias.float())
        y = 0.5 * f + 0.5 * bk.flip(-1)
        return F.linear(y.transpose(1, 2), self.out_proj.weight)


class Block(nn.Module):
    def __init__(self, d_model, mixer, eps=1e-5):
        super().__init__()
        self.mixer = mixer
        self.norm = RMSNorm(d_model, eps)

    def forward(self, h, residual=None):
        residual = h + residual if residual is not None else h
        return self.mixer(self.norm(residual)), residual


class MambaBlocksSequential(nn.Module):
    def __init__(self, n_mamba, d_model, d_state=16, expand=2, d_conv=4, eps=1e-5):
        super().__init__()
        self.layers = nn.Sequential(*[Block(d_model, BiMambaV2(d_model, d_state, d_conv, expand), eps)
                                      for _ in range(n_mamba)])
        self.norm_f = RMSNorm(d_model, eps)

    def forward(self, x):
        h, res = x, None
        for layer in self.layers:
            h, res = layer(h, res)
        res = h + res if res is not None else h
        return self.norm_f(res)


class ChannelwiseLayerNorm(nn.Module):
    """speechbrain conv_tasnet.ChannelwiseLayerNorm: input (M, K, N), stats over N."""

    def __init__(self, channels, eps=1e-8):
        super().__init__()
        self.eps = eps
        self.gamma = nn.Parameter(torch.ones(1, 1, channels))
        self.beta = nn.Parameter(torch.zeros(1, 1, channels))

    def forward(self, y):
        mean = y.mean(dim=2, keepdim=True)
        var = ((y - mean) ** 2).mean(dim=2, keepdim=True)
        return self.gamma * (y - mean) / torch.pow(var + self.eps, 0.5) + self.beta


class ChannelsLastConv1x1(nn.Module):
    """speechbrain nnet.CNN.Conv1d(kernel_size=1, bias=False): (B, L, Cin) -> (B, L, Cout); key conv.weight."""

    def __init__(self, cin, cout):
        super().__init__()
        self.conv = nn.Conv1d(cin, cout, 1, bias=False)

    def forward(self, x):
        return self.conv(x.transpose(1, 2)).transpose(1, 2)


class MaskNet(nn.Module):
    def __init__(self, enc_dim, bot_dim, n_spk=2, n_mamba=16, d_model=256, d_state=16, expand=2, d_conv=4):
        super().__init__()
        self.n_spk = n_spk
        self.layer_norm = ChannelwiseLayerNorm(enc_dim)
        self.bottleneck_conv1x1 = ChannelsLastConv1x1(enc_dim, bot_dim)
        self.mamba_net = MambaBlocksSequential(n_mamba, d_model, d_state, expand, d_conv)
        self.mask_conv1x1 = ChannelsLastConv1x1(bot_dim, n_spk * enc_dim)

    def forward(self, mixture_w):               # (M, N, K) -> (n_spk, M, N, K); mamba_masknet.py:101-139
        x = mixture_w.permute(0, 2, 1)
        Bn, L, D = x.shape
        y = self.mask_conv1x1(self.mamba_net(self.bottleneck_conv1x1(self.layer_norm(x))))
        return F.relu(y.reshape(Bn, L, self.n_spk, D).permute(2, 0, 3, 1))


class Encoder(nn.Module):
    def __init__(self, kernel_size=16, out_channels=512):
        super().__init__()
        self.conv1d = nn.Conv1d(1, out_channels, kernel_size, stride=kernel_size // 2, bias=False)

    def forward(self, x):                       # (B, T) -> (B, N, L)
        return F.relu(self.conv1d(x[:, None, :]))


class Decoder(nn.ConvTranspose1d):
    def forward(self, x):                       # (B, N, L) -> (B, T')
        y = super().forward(x)
        return y.squeeze(1)


class MambaTasNet(nn.Module):
    """Encoder + MaskNet + Decoder with train_wsj0mix.py:86-111 compute_forward semantics."""

    def __init__(self, N=512, kernel_size=16, n_mamba=32, n_spk=2, d_state=16, expand=2, d_conv=4):
        super().__init__()
        self.num_spks = n_spk
        self.encoder = Encoder(kernel_size, N)
        self.masknet = MaskNet(N, N, n_spk, n_mamba, N, d_state, expand, d_conv)
        self.decoder = Decoder(N, 1, kernel_size, stride=kernel_size // 2, bias=False)

    def forward(self, mix):                     # (B, T) -> (B, T, n_spk)
        mix_w = self.encoder(mix)
        est_mask = self.masknet(mix_w)
        sep_h = torch.stack([mix_w] * self.num_spks) * est_mask
        est = torch.stack([self.decoder(sep_h[i]) for i in range(self.num_spks)], dim=-1)
        T = mix.shape[1]
        if T > est.shape[1]:
            est = F.pad(est, (0, 0, 0, T - est.shape[1]))
        else:
            est = est[:, :T, :]
        return est


MAMBA_TASNET_SIZES = {  # hparams/WSJ0Mix/mambatasnet_{XS,S,M,L}.yaml
    "XS": dict(N=128, n_mamba=16),
    "S": dict(N=256, n_mamba=16),
    "M": dict(N=256, n_mamba=32),
    "L": dict(N=512, n_mamba=32),
}
