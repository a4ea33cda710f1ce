"""torch-facing wrappers over the C ABI (include/avse_hip.h).  GPU tensors only; no fallback.

Each wrapper validates shapes/dtypes/strides, allocates its outputs and workspace with torch
(caching allocator, stream-ordered) and enqueues the HIP kernels on torch's current stream.
"""
import functools

import torch

from . import _lib
from ._lib import AVSE_BF16, AVSE_F32, ScanBwdArgs, ScanFwdArgs, check, ptr, stream_ptr

NSTATE = 16

# Launch timing taps (bench.py's in-step roofline): while ``LAUNCH_TAPS`` maps a C entry point's name to a list, each
# eager launch of that entry point appends a (start, end) pair of HIP timing events recorded on its launch stream.
# Entry points whose work differs per launch (the split GEMM's shapes) append it to ``LAUNCH_WORK[name]`` beside the pair.
LAUNCH_TAPS = {}
LAUNCH_WORK = {}


def _tap_begin(name, device):
    taps = LAUNCH_TAPS.get(name)
    if taps is None or torch.cuda.is_current_stream_capturing():
        return None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(torch.cuda.current_stream(device))
    return taps, e0, e1, device, name


def _tap_end(tap, work=None):
    """Called after the launch returned AVSE_OK: only then is the pair appended (a failed launch leaves no
    half-recorded pair behind for bench.roofline's elapsed_time).  work: the launch's algorithmic FLOPs or bytes."""
    if tap is not None:
        taps, e0, e1, device, name = tap
        e1.record(torch.cuda.current_stream(device))
        taps.append((e0, e1))
        if work is not None:
            LAUNCH_WORK.setdefault(name, []).append(float(work))


def _need_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("avse_challenge_amd kernels run on the GPU only (got a CPU tensor); "
                               "the CPU restatement lives in oracle/ and is test infrastructure")


def _dtype_code(dt):
    if dt == torch.float32:
        return AVSE_F32
    if dt == torch.bfloat16:
        return AVSE_BF16
    raise RuntimeError(f"unsupported dtype {dt} (fp32 or bf16)")


# (b, d, l) outputs of the scan / conv kernels (and the Mamba projections feeding them) get a time stride rounded
# up to this many bytes: every row starts on a 128-B cache line, so a 64-step row segment touches 2 lines, not 3
# (L = 3999 fp32 rows were read 1.42x, profiles/r01_traffic.json).  0 = plain contiguous tensors.
TIME_ALIGN_BYTES = 128


def bdl_empty(b, d, l, dtype, dev):
    """An uninitialised (b, d, l) tensor whose time stride is padded to TIME_ALIGN_BYTES (a view when padded)."""
    return _bdl_empty(b, d, l, dtype, dev)


def _bdl_empty(b, d, l, dtype, dev):
    """Rows padded to TIME_ALIGN_BYTES when that costs at most 1/16 of the row (Mamba-TasNet: 3999 -> 4000 fp32,
    5999 -> 6016 bf16; DPMamba intra 250 -> 256); otherwise (DPMamba's 34-step inter rows would grow to 64) to
    4 elements, the vector width of the causal-conv kernels."""
    if TIME_ALIGN_BYTES > 0:
        per = max(1, TIME_ALIGN_BYTES // dtype.itemsize)
        lp = -(-l // per) * per
        if (lp - l) * 16 > l:
            lp = -(-l // 4) * 4
        if lp != l:
            return torch.empty((b, d, lp), device=dev, dtype=dtype)[..., :l]
    return torch.empty((b, d, l), device=dev, dtype=dtype)


def _last_contig(t):
    return t if t.stride(-1) == 1 else t.contiguous()


def _bc4(M, dtype):
    M = M.to(dtype)
    if M.dim() == 3:
        M = M.unsqueeze(1)
    if M.shape[1] != 1:
        raise RuntimeError("only n_groups == 1 B/C are supported (the reference path uses 1)")
    return _last_contig(M)


# ------------------------------------------------------------------------ selective scan

def _sp_mode(delta_softplus, delta_bias):
    """The C ABI's delta_softplus: 0 / 1 (False / True, selective_scan_cuda's flag) or 2 = delta already holds
    softplus(delta_raw + bias) from dtproj(); the backward then returns ddelta and ddelta_bias for delta_raw and the
    bias (so a ddelta_bias is produced although delta_bias is None)."""
    if delta_softplus is not True and delta_softplus == 2:
        if delta_bias is not None:
            raise RuntimeError("delta_softplus=2: the bias is already inside delta (pass delta_bias=None)")
        return 2
    return int(bool(delta_softplus))


def dtproj(w, x, bias=None, softplus=True):
    """delta = softplus(w @ x + bias[:, None]) per batch: w (D, R), x (b, R, l) with unit last stride (e.g. the first R
    rows of x_proj's (b, R + 2n, l) output), bias (D) fp32 or None -> (b, D, l) in x's dtype with the scan layout's
    padded time stride (csrc/dtproj.hip; fp32 accumulation).  The scan takes the result with delta_softplus=2."""
    _need_gpu(w, x, bias)
    dt = x.dtype
    code = _dtype_code(dt)
    if x.dim() != 3 or x.stride(2) != 1 or w.dim() != 2 or w.shape[1] != x.shape[1]:
        raise RuntimeError(f"dtproj: w (D, R) and x (b, R, l) with unit last stride, got {tuple(w.shape)}, "
                           f"{tuple(x.shape)}/{x.stride()}")
    w = w.to(dt)
    if w.stride(1) != 1:
        w = w.contiguous()
    b, R, l = x.shape
    D = w.shape[0]
    bias = None if bias is None else bias.float().contiguous()
    out = _bdl_empty(b, D, l, dt, x.device)
    tap = _tap_begin("avse_dtproj", x.device)
    check(_lib.lib().avse_dtproj(b, D, R, l, code, ptr(w), w.stride(0), ptr(x), x.stride(0) if b > 1 else (R - 1) *
                                 x.stride(1) + l, x.stride(1), ptr(bias), int(bool(softplus)), ptr(out), out.stride(0),
                                 out.stride(1), stream_ptr(x.device)), "avse_dtproj")
    _tap_end(tap)
    return out


def selective_scan_fwd(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False, reverse=False,
                       return_out=True, out_z_acc=None, out_z_max=None):
    """Returns (out, x, out_z|None) — the selective_scan_cuda.fwd contract.
    reverse=True scans time backwards (== flip(scan(flip(inputs))) with no flip copies).
    return_out=False (only with z): skip writing the pre-gate ``out`` (returned as None); the
    backward recomputes it, so training saves one (b, d, l) write and its activation memory.
    out_z_acc (with z): a (b, d, l) tensor of u's dtype, time-contiguous, that the gated output is ADDED to in place
    (the BiMamba v2 direction sum, round 6); returned as out_z.  out_z_max (with z): a zeroed 1-element int32 tensor
    that receives max |out_z| as float bits (the producer-side max of the split GEMM that consumes it)."""
    _need_gpu(u, delta, A, B, C, D, z, delta_bias)
    u = _last_contig(u)
    dt = u.dtype
    delta = _last_contig(delta.to(dt))
    z = None if z is None else _last_contig(z.to(dt))
    B, C = _bc4(B, dt), _bc4(C, dt)
    b, d, l = u.shape
    if A.shape != (d, NSTATE):
        raise RuntimeError(f"A must be ({d}, {NSTATE}), got {tuple(A.shape)}")
    A = A.float().contiguous()
    D = None if D is None else D.float().contiguous()
    delta_bias = None if delta_bias is None else delta_bias.float().contiguous()
    L = _lib.lib()
    nck = L.avse_scan_n_chunks(l)
    if not return_out and z is None:
        raise RuntimeError("return_out=False needs z (the gated output is then the only result)")
    out = _bdl_empty(b, d, l, dt, u.device) if return_out else None
    x = torch.empty((b, d, nck, 2 * NSTATE), device=u.device, dtype=torch.float32)
    out_z = _bdl_empty(b, d, l, dt, u.device) if z is not None else None
    if out_z_acc is not None:
        if z is None or tuple(out_z_acc.shape) != (b, d, l) or out_z_acc.dtype != dt or out_z_acc.stride(2) != 1 \
                or out_z_acc.device != u.device:
            raise RuntimeError("selective_scan_fwd: out_z_acc must be a time-contiguous (b, d, l) tensor of u's dtype "
                               "(and z given)")
        out_z = out_z_acc
    a = ScanFwdArgs()
    a.batch, a.dim, a.seqlen, a.dstate = b, d, l, NSTATE
    a.in_dtype, a.delta_softplus, a.reverse = _dtype_code(dt), _sp_mode(delta_softplus, delta_bias), int(bool(reverse))
    a.u, a.u_bs, a.u_ds = u.data_ptr(), u.stride(0), u.stride(1)
    a.delta, a.delta_bs, a.delta_ds = delta.data_ptr(), delta.stride(0), delta.stride(1)
    a.A = A.data_ptr()
    a.B, a.B_bs, a.B_ns = B.data_ptr(), B.stride(0), B.stride(2)
    a.C, a.C_bs, a.C_ns = C.data_ptr(), C.stride(0), C.stride(2)
    a.D = D.data_ptr() if D is not None else None
    if z is not None:
        a.z, a.z_bs, a.z_ds = z.data_ptr(), z.stride(0), z.stride(1)
        a.out_z, a.out_z_bs, a.out_z_ds = out_z.data_ptr(), out_z.stride(0), out_z.stride(1)
        a.out_z_accumulate = int(out_z_acc is not None)
        a.out_z_max = ptr(out_z_max)
    a.delta_bias = delta_bias.data_ptr() if delta_bias is not None else None
    if out is not None:
        a.out, a.out_bs, a.out_ds = out.data_ptr(), out.stride(0), out.stride(1)
    a.x = x.data_ptr()
    tap = _tap_begin("avse_scan_fwd", u.device)
    check(L.avse_scan_fwd(a, stream_ptr(u.device)), "avse_scan_fwd")
    _tap_end(tap)
    return out, x, out_z


def selective_scan_bwd(u, delta, A, B, C, D, z, delta_bias, dout, x, out=None, dz=None,
                       delta_softplus=False, recompute_out_z=False, reverse=False, dB_out=None, dC_out=None,
                       dz_accumulate=False, dz_max=None):
    """Returns [du, ddelta, dA, dB, dC, dD, ddelta_bias, dz, out_z] — selective_scan_cuda.bwd contract.
    dB, dC are fp32 shaped (b, 1, n, l); a passed-in ``dz`` view is written in place, and so are
    ``dB_out`` / ``dC_out`` (fp32 (b, n, l) or (b, 1, n, l) views with unit last stride, e.g. rows of
    the x_proj output gradient), which are then returned as dB / dC.  dz_accumulate (round 6, with a passed
    ``dz``): dz += the gradient instead of dz = (the serial BiMamba directions' shared xz gradient); dz_max: a zeroed
    1-element int32 tensor that receives max |dz| as float bits."""
    if dz_accumulate and dz is None:
        raise RuntimeError("selective_scan_bwd: dz_accumulate needs the dz to add into")
    _need_gpu(u, delta, A, B, C, D, z, delta_bias, dout, x)
    u = _last_contig(u)
    dt = u.dtype
    delta = _last_contig(delta.to(dt))
    dout = _last_contig(dout.to(dt))
    z = None if z is None else _last_contig(z.to(dt))
    B, C = _bc4(B, dt), _bc4(C, dt)
    b, d, l = u.shape
    A = A.float().contiguous()
    D = None if D is None else D.float().contiguous()
    delta_bias = None if delta_bias is None else delta_bias.float().contiguous()
    x = x.float().contiguous()
    L = _lib.lib()
    if x.shape != (b, d, L.avse_scan_n_chunks(l), 2 * NSTATE):
        raise RuntimeError(f"scan intermediates have shape {tuple(x.shape)}; expected avse layout")
    dev = u.device
    du = _bdl_empty(b, d, l, dt, dev)
    ddelta = _bdl_empty(b, d, l, dt, dev)
    dA = torch.empty((d, NSTATE), device=dev, dtype=torch.float32)
    def _grad_bc(o):
        if o is None:
            return torch.empty((b, 1, NSTATE, l), device=dev, dtype=torch.float32)
        o = o.unsqueeze(1) if o.dim() == 3 else o
        if o.dtype != torch.float32 or o.stride(-1) != 1 or tuple(o.shape) != (b, 1, NSTATE, l):
            raise RuntimeError("dB_out / dC_out must be fp32 (b, [1,] n, l) views with unit last stride")
        return o
    dB, dC = _grad_bc(dB_out), _grad_bc(dC_out)
    dD = torch.empty((d,), device=dev, dtype=torch.float32) if D is not None else None
    mode = _sp_mode(delta_softplus, delta_bias)
    dbias = torch.empty((d,), device=dev, dtype=torch.float32) if (delta_bias is not None or mode == 2) else None
    if z is not None:
        if dz is None:
            dz = _bdl_empty(b, d, l, dt, dev)
        elif dz.stride(-1) != 1 or dz.dtype != dt or tuple(dz.shape) != (b, d, l):
            raise RuntimeError("dz must be a (b, d, l) view with unit last stride and the input dtype")
    else:
        dz = None
    out_z = torch.empty((b, d, l), device=dev, dtype=dt) if (recompute_out_z and z is not None) else None
    ws = torch.empty((L.avse_scan_bwd_workspace_bytes(b, d, l, NSTATE) + 3) // 4, device=dev, dtype=torch.float32)
    a = ScanBwdArgs()
    a.batch, a.dim, a.seqlen, a.dstate = b, d, l, NSTATE
    a.in_dtype, a.delta_softplus = _dtype_code(dt), mode
    a.recompute_out_z = int(out_z is not None)
    a.reverse = int(bool(reverse))
    a.u, a.u_bs, a.u_ds = u.data_ptr(), u.stride(0), u.stride(1)
    a.delta, a.delta_bs, a.delta_ds = delta.data_ptr(), delta.stride(0), delta.stride(1)
    a.A = A.data_ptr()
    a.B, a.B_bs, a.B_ns = B.data_ptr(), B.stride(0), B.stride(2)
    a.C, a.C_bs, a.C_ns = C.data_ptr(), C.stride(0), C.stride(2)
    a.D = D.data_ptr() if D is not None else None
    if z is not None:
        a.z, a.z_bs, a.z_ds = z.data_ptr(), z.stride(0), z.stride(1)
        a.dz, a.dz_bs, a.dz_ds = dz.data_ptr(), dz.stride(0), dz.stride(1)
    if out_z is not None:
        a.out_z, a.out_z_bs, a.out_z_ds = out_z.data_ptr(), out_z.stride(0), out_z.stride(1)
    a.dz_accumulate = int(bool(dz_accumulate) and dz is not None)
    a.dz_max = ptr(dz_max) if dz is not None else None
    a.delta_bias = delta_bias.data_ptr() if delta_bias is not None else None
    a.dout, a.dout_bs, a.dout_ds = dout.data_ptr(), dout.stride(0), dout.stride(1)
    a.x = x.data_ptr()
    a.du, a.du_bs, a.du_ds = du.data_ptr(), du.stride(0), du.stride(1)
    a.ddelta, a.ddelta_bs, a.ddelta_ds = ddelta.data_ptr(), ddelta.stride(0), ddelta.stride(1)
    a.dA = dA.data_ptr()
    a.dB, a.dB_bs, a.dB_ns = dB.data_ptr(), dB.stride(0), dB.stride(2)
    a.dC, a.dC_bs, a.dC_ns = dC.data_ptr(), dC.stride(0), dC.stride(2)
    a.dD = dD.data_ptr() if dD is not None else None
    a.ddelta_bias = dbias.data_ptr() if dbias is not None else None
    a.workspace = ws.data_ptr()
    tap = _tap_begin("avse_scan_bwd", dev)
    check(L.avse_scan_bwd(a, stream_ptr(dev)), "avse_scan_bwd")
    _tap_end(tap)
    return [du, ddelta, dA, dB, dC, dD, dbias, dz, out_z]


# ------------------------------------------------------------------------ causal conv1d

def causal_conv1d_fwd(x, weight, bias=None, silu=False, reverse=False):
    """out = act(depthwise causal conv(x)) in x's dtype (fp32 or bf16; fp32 weights and arithmetic)."""
    _need_gpu(x, weight, bias)
    dt = x.dtype
    _dtype_code(dt)
    x = _last_contig(x)
    if weight.dim() == 3:
        weight = weight.reshape(weight.shape[0], -1)
    weight = weight.float().contiguous()
    bias = None if bias is None else bias.float().contiguous()
    b, d, l = x.shape
    w = weight.shape[1]
    out = _bdl_empty(b, d, l, dt, x.device)
    fn = _lib.lib().avse_cconv_fwd if dt == torch.float32 else _lib.lib().avse_cconv_fwd_bf16
    check(fn(b, d, l, w, ptr(x), x.stride(0), x.stride(1), ptr(weight), ptr(bias), ptr(out), out.stride(0),
             out.stride(1), int(bool(silu)), int(bool(reverse)), stream_ptr(x.device)), "avse_cconv_fwd")
    return out


def causal_conv1d_bwd(x, weight, bias, dout, dx=None, silu=False, reverse=False, dx_accumulate=False, dx_max=None):
    """[dx, dweight, dbias]: dx in x's dtype (fp32 or bf16; a passed ``dx`` view of that dtype with unit last
    stride is written in place), dweight / dbias fp32.  dx_accumulate (round 6, with such a ``dx``): dx += the input
    gradient (the serial BiMamba directions' shared xz gradient); dx_max: a zeroed 1-element int32 tensor that receives
    max |dx| as float bits."""
    _need_gpu(x, weight, bias, dout)
    dt = x.dtype
    _dtype_code(dt)
    x = _last_contig(x)
    wshape = weight.shape
    weight = weight.reshape(wshape[0], -1).float().contiguous()
    bias = None if bias is None else bias.float().contiguous()
    dout = _last_contig(dout.to(dt))
    b, d, l = x.shape
    w = weight.shape[1]
    dx_ret = dx
    if dx_accumulate and (dx is None or dx.dtype != dt or dx.stride(-1) != 1):
        raise RuntimeError("causal_conv1d_bwd: dx_accumulate needs a dx of x's dtype with unit last stride")
    if dx is None or dx.dtype != dt or dx.stride(-1) != 1:
        dx = _bdl_empty(b, d, l, dt, x.device)
    dweight = torch.empty((d, w), device=x.device, dtype=torch.float32)
    dbias = torch.empty((d,), device=x.device, dtype=torch.float32) if bias is not None else None
    ws = torch.empty((_lib.lib().avse_cconv_bwd_workspace_bytes(b, d, w) + 3) // 4, device=x.device,
                     dtype=torch.float32)
    fn = _lib.lib().avse_cconv_bwd if dt == torch.float32 else _lib.lib().avse_cconv_bwd_bf16
    check(fn(b, d, l, w, ptr(x), x.stride(0), x.stride(1), ptr(weight), ptr(bias), ptr(dout), dout.stride(0),
             dout.stride(1), ptr(dx), dx.stride(0), dx.stride(1), ptr(dweight), ptr(dbias), int(bool(silu)),
             int(bool(reverse)), ptr(ws), int(bool(dx_accumulate)), ptr(dx_max), stream_ptr(x.device)),
          "avse_cconv_bwd")
    if dx_ret is not None and dx_ret is not dx:
        dx_ret.copy_(dx)
        dx = dx_ret
    return [dx, dweight, dbias]


# ------------------------------------------------------------------------ add + RMSNorm

def _rows_in(t, n):
    """(rows, n) view of t for the RMSNorm kernels: fp32 or bf16 rows as they are (contiguous), anything else as fp32."""
    if t.dtype not in (torch.float32, torch.bfloat16):
        t = t.float()
    return t.contiguous().view(-1, n)


def add_rmsnorm_fwd(h, res, weight, eps=1e-5, out_dtype=None):
    """(norm(h + res) * w, h + res, rstd) over the last dim; res may be None.  h fp32 or bf16 (read as it is); the output
    in out_dtype (fp32 default, or bf16: rounded once); h + res and the statistics in fp32."""
    _need_gpu(h, res, weight)
    n = h.shape[-1]
    h2 = _rows_in(h, n)
    r2 = None if res is None else res.float().contiguous().view(-1, n)
    w = weight.float().contiguous()
    rows = h2.shape[0]
    out_dtype = out_dtype or torch.float32
    if out_dtype not in (torch.float32, torch.bfloat16):
        raise RuntimeError(f"add_rmsnorm_fwd: output dtype {out_dtype} (fp32 or bf16)")
    y = torch.empty((rows, n), device=h.device, dtype=out_dtype)
    res_out = torch.empty((rows, n), device=h.device, dtype=torch.float32)
    rstd = torch.empty((rows,), device=h.device, dtype=torch.float32)
    ymax = torch.empty(1, device=h.device, dtype=torch.int32)
    dt = lambda t: AVSE_BF16 if t.dtype == torch.bfloat16 else AVSE_F32          # noqa: E731
    check(_lib.lib().avse_add_rmsnorm_fwd2(rows, n, ptr(h2), dt(h2), ptr(r2), ptr(w), float(eps), ptr(y), dt(y),
                                           ptr(res_out), ptr(rstd), ptr(ymax), stream_ptr(h.device)),
          "avse_add_rmsnorm_fwd2")
    y = y.view(h.shape)
    if out_dtype == torch.float32:
        _set_absmax(y, ymax)                  # the producer-side max: the projection's split_planes skips its pass
    return y, res_out.view(h.shape), rstd


def rmsnorm_bwd(dy, dres_out, res_out, weight, rstd):
    """(dx fp32, dweight) of add_rmsnorm_fwd; dy fp32 or bf16 (read as it is)."""
    _need_gpu(dy, dres_out, res_out, weight, rstd)
    n = res_out.shape[-1]
    dy2 = _rows_in(dy, n)
    dr2 = None if dres_out is None else dres_out.float().contiguous().view(-1, n)
    x2 = res_out.float().contiguous().view(-1, n)
    rows = x2.shape[0]
    dx = torch.empty_like(x2)
    dw = torch.empty((n,), device=dy.device, dtype=torch.float32)
    ws = torch.empty((_lib.lib().avse_rmsnorm_bwd_workspace_bytes(rows, n) + 3) // 4, device=dy.device,
                     dtype=torch.float32)
    dxmax = torch.empty(1, device=dy.device, dtype=torch.int32)
    check(_lib.lib().avse_rmsnorm_bwd2(rows, n, ptr(dy2), AVSE_BF16 if dy2.dtype == torch.bfloat16 else AVSE_F32,
                                       ptr(dr2), ptr(x2), ptr(weight.float().contiguous()), ptr(rstd), ptr(dx),
                                       ptr(dw), ptr(ws), ptr(dxmax), stream_ptr(dy.device)), "avse_rmsnorm_bwd2")
    dx = dx.view(res_out.shape)
    _set_absmax(dx, dxmax)
    return dx, dw


# ------------------------------------------------------------------------ STFT / iSTFT

def stft_frames(T):
    return int(_lib.lib().avse_stft_frames(T))


def stft(wave, return_complex=False):
    """wave (B, T) fp32 -> |STFT|.T (B, frames, 257) [and complex (B, frames, 257)]; librosa 0.8.1 semantics."""
    _need_gpu(wave)
    wave = wave.float().contiguous()
    Bn, T = wave.shape
    F = stft_frames(T)
    mag = torch.empty((Bn, F, 257), device=wave.device, dtype=torch.float32)
    spec = torch.empty((Bn, F, 257, 2), device=wave.device, dtype=torch.float32) if return_complex else None
    check(_lib.lib().avse_stft_fwd(Bn, T, ptr(wave), ptr(mag), ptr(spec), stream_ptr(wave.device)), "avse_stft_fwd")
    if return_complex:
        return mag, torch.view_as_complex(spec)
    return mag


def istft(mag, phase_spec, length):
    """mag (B, frames, 257) and the complex spectrum whose angle is used (B, frames, 257) -> (B, length)."""
    _need_gpu(mag, phase_spec)
    mag = mag.float().contiguous()
    ps = torch.view_as_real(phase_spec.to(torch.complex64)).contiguous()
    Bn, F, nb = mag.shape
    if nb != 257 or tuple(ps.shape[:3]) != (Bn, F, 257):
        raise RuntimeError("istft expects (B, frames, 257) magnitude and matching complex phase spectrum")
    fbuf = torch.empty((Bn, F, 512), device=mag.device, dtype=torch.float32)
    out = torch.empty((Bn, length), device=mag.device, dtype=torch.float32)
    check(_lib.lib().avse_istft(Bn, F, length, ptr(mag), ptr(ps), ptr(fbuf), ptr(out), stream_ptr(mag.device)),
          "avse_istft")
    return out


# ------------------------------------------------------------------------ lip front-end Conv3d dW

CONV3D_WGRAD_MAX_WO = 64      # output width the MFMA kernel stages per LDS row (conv3d_wgrad.hip MAX_WO)
# the f16 MFMA weight gradient with dy split (uint8 frames: avse_conv3d_wgrad_u8_split; fp32 frames split too:
# avse_conv3d_wgrad_split); False (a test's comparison): the exact-fp32 kernel
C3W_F16 = True


def _absmax_bits(t):
    """max |t| as float bits in a 1-element int32 device tensor (the split kernels' scale input)."""
    return t.abs().amax().float().reshape(1).view(torch.int32)


def conv3d_wgrad(x, dy, kernel_size, padding, out=None, accumulate=False, xmax=None):
    """dW of Conv3d(Cin, 64, kernel_size, stride (1,2,2), padding, bias=False) -> (64, Cin, KT, KH, KW).
    x: fp32, or the uint8 lip frames as stored (read as their float values, no fp32 copy).  xmax (fp32 x, optional):
    max |x| bits as conv3d_fwd(..., return_xmax=True) returned them; computed here when not given."""
    _need_gpu(x, dy)
    u8 = x.dtype == torch.uint8
    x = x.contiguous() if u8 else x.float().contiguous()
    dymax = _known_absmax(dy) if C3W_F16 else None            # the BatchNorm -> act backward's max |dy|
    dy = dy.float().contiguous()
    if C3W_F16 and dymax is None:
        dymax = _absmax_bits(dy)
    if C3W_F16 and not u8 and xmax is None:
        xmax = _absmax_bits(x)
    Bn, Cin, Tn, H, W = x.shape
    KT, KH, KW = kernel_size
    PT, PH, PW = padding
    if dy.shape[1] != 64:
        raise RuntimeError("conv3d_wgrad is built for 64 output channels (the lip front-ends)")
    N = Cin * KT * KH * KW
    if out is None:
        out = torch.empty((64, Cin, KT, KH, KW), device=x.device, dtype=torch.float32)
        accumulate = False
    L = _lib.lib()
    ws = torch.empty((L.avse_conv3d_wgrad_workspace_bytes(Bn, dy.shape[2], dy.shape[3], N) + 3) // 4,
                     device=x.device, dtype=torch.float32)
    if C3W_F16 and u8:                 # uint8 frames on the f16 MFMA, dy split under its max
        check(L.avse_conv3d_wgrad_u8_split(Bn, Cin, Tn, H, W, KT, KH, KW, PT, PH, PW, ptr(x), ptr(dy), ptr(dymax),
                                           ptr(out), int(bool(accumulate)), ptr(ws), stream_ptr(x.device)),
              "avse_conv3d_wgrad_u8_split")
        return out
    if C3W_F16:                        # fp32 frames: x and dy split under their maxima
        check(L.avse_conv3d_wgrad_split(Bn, Cin, Tn, H, W, KT, KH, KW, PT, PH, PW, ptr(x), ptr(xmax), ptr(dy),
                                        ptr(dymax), ptr(out), int(bool(accumulate)), ptr(ws), stream_ptr(x.device)),
              "avse_conv3d_wgrad_split")
        return out
    fn = L.avse_conv3d_wgrad_u8 if u8 else L.avse_conv3d_wgrad
    check(fn(Bn, Cin, Tn, H, W, KT, KH, KW, PT, PH, PW, ptr(x), ptr(dy), ptr(out),
             int(bool(accumulate)), ptr(ws), stream_ptr(x.device)), "avse_conv3d_wgrad")
    return out


def conv3d_fwd_supported(x, w, stride, padding):
    """True when the MFMA forward (conv3d_fwd.hip) is compiled for this lip front-end shape."""
    return (tuple(stride) == (1, 2, 2) and tuple(padding) == (2, 3, 3) and tuple(w.shape[0:1]) == (64,)
            and tuple(w.shape[2:]) == (5, 7, 7) and x.dim() == 5 and x.shape[1] == w.shape[1]
            and (x.dtype == torch.float32 or (x.dtype == torch.uint8 and x.shape[1] == 3))   # uint8: avse1's f16 path
            and x.numel() * x.element_size() < (1 << 31)          # the kernel's 32-bit buffer offsets
            and _lib.lib().avse_conv3d_fwd_workspace_bytes(x.shape[1], x.shape[3], x.shape[4]) > 0)


def conv3d_fwd(x, w, return_xmax=False):
    """Conv3d(Cin, 64, (5, 7, 7), stride (1, 2, 2), padding (2, 3, 3), bias=False) forward of the lip front-end:
    x (B, Cin, T, H, W) uint8 frames or fp32, w (64, Cin, 5, 7, 7) fp32 -> (B, 64, T, Ho, Wo) fp32.
    return_xmax (fp32 x): also return max |x| bits (1-element int32, from the forward's absmax pass) for
    conv3d_wgrad."""
    _need_gpu(x, w)
    if x.dtype not in (torch.uint8, torch.float32):
        raise RuntimeError(f"conv3d_fwd: x must be uint8 or float32, got {x.dtype}")
    x = x.contiguous()
    w = w.float().contiguous()
    Bn, Cin, Tn, H, W = x.shape
    if tuple(w.shape) != (64, Cin, 5, 7, 7):
        raise RuntimeError(f"conv3d_fwd: weight {tuple(w.shape)} is not (64, {Cin}, 5, 7, 7)")
    L = _lib.lib()
    nb = L.avse_conv3d_fwd_workspace_bytes(Cin, H, W)
    if nb <= 0:
        raise RuntimeError(f"conv3d_fwd: shape Cin={Cin} {H}x{W} is not compiled in (conv3d_fwd.hip)")
    ws = torch.empty((nb + 3) // 4, device=x.device, dtype=torch.float32)
    y = torch.empty((Bn, 64, Tn, (H - 1) // 2 + 1, (W - 1) // 2 + 1), device=x.device, dtype=torch.float32)
    check(L.avse_conv3d_fwd(Bn, Cin, Tn, H, W, 2 if x.dtype == torch.uint8 else 0, ptr(x), ptr(w), ptr(y), ptr(ws),
                            stream_ptr(x.device)), "avse_conv3d_fwd")
    if not return_xmax:
        return y
    # workspace: the split weights (2 * Cin * 5 * 8192 bytes), then max |W|, max |x| (conv3d_fwd.hip ws_bytes)
    xmax = ws.view(torch.int32)[(2 * Cin * 5 * 8192) // 4 + 1:(2 * Cin * 5 * 8192) // 4 + 2]
    return y, (xmax if x.dtype == torch.float32 else None)


# ------------------------------------------------------------------------ dilated Conv2d dW (AudioFeatNet)

DCONV_WGRAD_MAX_DIL = 16       # dconv_wgrad.hip MAX_DIL


def dconv_wgrad(x, dy, dilation, bias_grad=False):
    """dW (64, 64, 5, 5) of Conv2d(64, 64, 5, padding=2*dilation, dilation) from the conv input x and the output
    gradient dy, both (N, 64, H, W) fp32; channels-last memory is read as it lies, anything else is made so.
    bias_grad: return (dW, db) with db = dy summed over (N, H, W), computed in the same pass."""
    _need_gpu(x, dy)
    if x.shape[1] != 64 or dy.shape != x.shape:
        raise RuntimeError(f"dconv_wgrad expects (N, 64, H, W) input and gradient, got {tuple(x.shape)}, {tuple(dy.shape)}")
    cl = torch.channels_last
    x = x.float().contiguous(memory_format=cl)
    dy = dy.float().contiguous(memory_format=cl)
    Bn, _, H, W = x.shape
    L = _lib.lib()
    out = torch.empty((64, 64, 5, 5), device=x.device, dtype=torch.float32)
    ws = torch.empty((L.avse_dconv_wgrad_workspace_bytes(Bn, H, W, dilation) + 3) // 4, device=x.device,
                     dtype=torch.float32)
    db = torch.empty(64, device=x.device, dtype=torch.float32) if bias_grad else None
    tap = _tap_begin("avse_dconv_wgrad", x.device)
    check(L.avse_dconv_wgrad(Bn, H, W, dilation, ptr(x), ptr(dy), ptr(out), ptr(db) if bias_grad else None, ptr(ws),
                             stream_ptr(x.device)), "avse_dconv_wgrad")
    _tap_end(tap)
    return (out, db) if bias_grad else out


# ------------------------------------------------------------------------ dilated Conv2d fwd / dX (split fp16 MFMA)

DCONV_DILATIONS = (2, 4, 8, 16)     # dconv.hip instantiations


def dconv_split_ok(x, dilation):
    """True when csrc/dconv.hip takes conv(x) / its input gradient: (N, 64, H, W >= 256) fp32 GPU tensor, d in 2..16."""
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.shape[1] == 64 and x.shape[3] >= 256
            and dilation in DCONV_DILATIONS and x.shape[0] * x.shape[2] * x.shape[3] * 256 < (1 << 31) - 1024)


def split16(x, maxbits):
    """x (N, 64, H, W) fp32 (channels-last memory is read as it lies, anything else made so) -> its fp16 hi / lo split
    in dconv.hip's Q4 layout (uint8 (N*H*W, 256)); writes max |x| (float bits) into maxbits[0].  A split-output
    tensor (bnact_fwd / bnact_bwd with q_out) already holds those bytes: returned as its uint8 view, no pass."""
    _need_gpu(x)
    known = _known_absmax(x)
    if is_split_q(x):
        maxbits[:1].copy_(known)
        return q_view(x)
    x = x.contiguous(memory_format=torch.channels_last)
    npix = x.shape[0] * x.shape[2] * x.shape[3]
    xq = torch.empty((npix, 256), device=x.device, dtype=torch.uint8)
    if known is not None:                          # the producer's max: the split pass only
        maxbits[:1].copy_(known)
        check(_lib.lib().avse_split16_known(npix, ptr(x), ptr(xq), ptr(maxbits), stream_ptr(x.device)),
              "avse_split16_known")
    else:
        check(_lib.lib().avse_split16(npix, ptr(x), ptr(xq), ptr(maxbits), stream_ptr(x.device)), "avse_split16")
    return xq


def dconv_wprep(w, transposed, maxbits):
    """W (64, 64, 5, 5) fp32 -> dconv.hip's split weight image (transposed: the input gradient's flipped W'); writes
    max |w| into maxbits[1]."""
    _need_gpu(w)
    L = _lib.lib()
    wq = torch.empty(int(L.avse_dconv_wprep_bytes()), device=w.device, dtype=torch.uint8)
    check(L.avse_dconv_wprep(ptr(w.float().contiguous()), int(bool(transposed)), ptr(wq), ptr(maxbits),
                             stream_ptr(w.device)), "avse_dconv_wprep")
    return wq


def dconv_fwd(x, w, dilation, bias=None, transposed=False, split=None):
    """conv2d(x, w, bias, padding=2d, dilation=d) for the 64 -> 64 5x5 AudioFeatNet convs on csrc/dconv.hip (fp16x3
    split MFMA, fp32-accurate); transposed=True: the input gradient conv_transpose(x = dY, w).  x (N, 64, H, W) fp32
    (its shape only, when ``split`` = (xq, maxbits) from split16 is given: maxbits[1] is then overwritten with W's);
    returns (N, 64, H, W) in channels-last memory."""
    _need_gpu(x, w, bias)
    if not dconv_split_ok(x, dilation) or tuple(w.shape) != (64, 64, 5, 5):
        raise RuntimeError(f"dconv_fwd: unsupported shape {tuple(x.shape)} / {tuple(w.shape)} dilation {dilation}")
    N, _, H, W = x.shape
    if split is None:
        maxbits = torch.empty(2, device=x.device, dtype=torch.int32)
        xq = split16(x, maxbits)
    else:
        xq, maxbits = split
    wq = dconv_wprep(w, transposed, maxbits)
    y = torch.empty((N, 64, H, W), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
    tap = _tap_begin("avse_dconv_fwd", x.device)
    check(_lib.lib().avse_dconv_fwd(N, H, W, dilation, ptr(xq), ptr(wq), ptr(maxbits),
                                    ptr(None if bias is None else bias.float().contiguous()), ptr(y),
                                    stream_ptr(x.device)), "avse_dconv_fwd")
    _tap_end(tap)
    return y


def dconv_wgrad16(xs, dys, shape, dilation, bias_grad=False):
    """dW (64, 64, 5, 5) [and db (64)] of Conv2d(64, 64, 5, padding=2d, dilation=d) from the split input and output
    gradient: xs = (xq, x_maxbits), dys = (dyq, dy_maxbits) from split16 (csrc/dconv.hip, fp16x3 split MFMA);
    shape = (N, 64, H, W)."""
    (xq, xm), (dyq, dym) = xs, dys
    _need_gpu(xq, dyq)
    N, _, H, W = shape
    L = _lib.lib()
    dw = torch.empty((64, 64, 5, 5), device=xq.device, dtype=torch.float32)
    db = torch.empty(64, device=xq.device, dtype=torch.float32) if bias_grad else None
    ws = torch.empty((L.avse_dconv_wgrad16_workspace_bytes(N, H, W) + 3) // 4, device=xq.device, dtype=torch.float32)
    tap = _tap_begin("avse_dconv_wgrad16", xq.device)
    check(L.avse_dconv_wgrad16(N, H, W, dilation, ptr(xq), ptr(xm), ptr(dyq), ptr(dym), ptr(dw), ptr(db), ptr(ws),
                               stream_ptr(xq.device)), "avse_dconv_wgrad16")
    _tap_end(tap)
    return (dw, db) if bias_grad else dw


# ------------------------------------------------------------------------ AudioFeatNet.conv1 (1 -> 64, 5x5)

def conv1_fwd(x, w, b=None):
    """conv2d(x, w, b, padding=2) for x (N, 1, H, W) fp32 contiguous, w (64, 1, 5, 5) (csrc/conv1.hip) -> (N, 64, H, W)
    in channels-last memory."""
    _need_gpu(x, w, b)
    n, _, h, wd = x.shape
    y = torch.empty((n, 64, h, wd), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
    tap = _tap_begin("avse_conv1_fwd", x.device)
    check(_lib.lib().avse_conv1_fwd(n, h, wd, ptr(x.contiguous()), ptr(w.float().contiguous()),
                                    ptr(None if b is None else b.float().contiguous()), ptr(y), stream_ptr(x.device)),
          "avse_conv1_fwd")
    _tap_end(tap)
    return y


def conv1_bwd(x, w, dy, need_dx=True, need_dw=True):
    """(dx (N, 1, H, W) or None, dW (64, 1, 5, 5) or None, db (64) or None) of conv1_fwd from its input x and the
    output gradient dy (N, 64, H, W) (read as channels-last memory)."""
    _need_gpu(x, w, dy)
    n, _, h, wd = x.shape
    dy = dy.contiguous(memory_format=torch.channels_last)
    L = _lib.lib()
    dx = dw = db = None
    if need_dx:
        dx = torch.empty((n, 1, h, wd), device=x.device, dtype=torch.float32)
        check(L.avse_conv1_dgrad(n, h, wd, ptr(dy), ptr(w.float().contiguous()), ptr(dx), stream_ptr(x.device)),
              "avse_conv1_dgrad")
    if need_dw:
        dw = torch.empty((64, 1, 5, 5), device=x.device, dtype=torch.float32)
        db = torch.empty(64, device=x.device, dtype=torch.float32)
        ws = torch.empty((L.avse_conv1_wgrad_workspace_bytes(n, h, wd) + 3) // 4, device=x.device, dtype=torch.float32)
        check(L.avse_conv1_wgrad(n, h, wd, ptr(x.contiguous()), ptr(dy), ptr(dw), ptr(db), ptr(ws),
                                 stream_ptr(x.device)), "avse_conv1_wgrad")
    return dx, dw, db


# ------------------------------------------------------------------------ AudioFeatNet.convf (64 -> 4, 1x1)

def convf_fwd(x, w, b=None):
    """conv2d(x, w (4, 64, 1, 1), b) for x (N, 64, H, W) fp32 in channels-last memory (csrc/convf.hip) -> (N, 4, H, W)
    in channels-last memory."""
    _need_gpu(x, w, b)
    n, c, h, wd = x.shape
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.empty((n, 4, h, wd), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
    check(_lib.lib().avse_convf_fwd(n * h * wd, ptr(x), ptr(w.float().contiguous()),
                                    ptr(None if b is None else b.float().contiguous()), ptr(y), stream_ptr(x.device)),
          "avse_convf_fwd")
    return y


def convf_bwd(x, w, dy, need_dx=True, need_dw=True):
    """(dx (N, 64, H, W) channels-last or None, dW (4, 64, 1, 1) or None, db (4) or None) of convf_fwd from its input x
    and the output gradient dy (N, 4, H, W) (read as channels-last memory)."""
    _need_gpu(x, w, dy)
    n, c, h, wd = x.shape
    dy = dy.contiguous(memory_format=torch.channels_last)
    L = _lib.lib()
    dx = dw = db = None
    if need_dx:
        dx = torch.empty((n, c, h, wd), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
        check(L.avse_convf_dgrad(n * h * wd, ptr(dy), ptr(w.float().contiguous()), ptr(dx), stream_ptr(x.device)),
              "avse_convf_dgrad")
    if need_dw:
        x = x.contiguous(memory_format=torch.channels_last)
        dw = torch.empty((4, c, 1, 1), device=x.device, dtype=torch.float32)
        db = torch.empty(4, device=x.device, dtype=torch.float32)
        ws = torch.empty((L.avse_convf_wgrad_workspace_bytes(n * h * wd) + 3) // 4, device=x.device, dtype=torch.float32)
        check(L.avse_convf_wgrad(n * h * wd, ptr(x), ptr(dy), ptr(dw), ptr(db), ptr(ws), stream_ptr(x.device)),
              "avse_convf_wgrad")
    return dx, dw, db


# ------------------------------------------------------------------------ ResNet trunk 3x3 Conv2d (split fp16 MFMA)

def sconv_ok(x, cout, stride):
    """True when csrc/sconv.hip takes Conv2d(cin, cout, 3, stride, padding=1, bias=False) on x: (N, cin, H, W) fp32 GPU
    tensor, cin and cout multiples of 64, stride 1 or 2, the pixel counts inside the kernels' 32-bit offsets."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and stride in (1, 2)):
        return False
    n, cin, h, w = x.shape
    if cin % 64 or cout % 64 or n * h * w * max(cin, cout) * 4 >= (1 << 31) - 4096:
        return False
    return _lib.lib().avse_sconv_wgrad_workspace_bytes(n, h, w, cin, cout, stride) > 0


def split_nhwc(x, maxbits):
    """x (N, C, H, W) fp32, C % 64 == 0 (channels-last memory read as it lies, anything else made so) -> its fp16
    hi / lo split in the Q layout (uint8 (N*H*W, 4 C): per pixel C / 16 chunks of [hi 16][lo 16]); writes max |x| bits
    into maxbits[0] (avse_split16 over the tensor viewed as (N H W C / 64, 64))."""
    _need_gpu(x)
    x = x.contiguous(memory_format=torch.channels_last)
    n, c, h, w = x.shape
    xq = torch.empty((n * h * w, 4 * c), device=x.device, dtype=torch.uint8)
    check(_lib.lib().avse_split16(n * h * w * (c // 64), ptr(x), ptr(xq), ptr(maxbits), stream_ptr(x.device)),
          "avse_split16")
    return xq


def split_q(x):
    """-> (xq, xmax): split_nhwc with the producer's max when x carries one (no absmax pass), else a fresh max; a
    split-output tensor as its uint8 view (no pass)."""
    known = _known_absmax(x)
    if is_split_q(x):
        return q_view(x), known
    if known is None:
        xm = torch.empty(1, device=x.device, dtype=torch.int32)
        return split_nhwc(x, xm), xm
    _need_gpu(x)
    x = x.contiguous(memory_format=torch.channels_last)
    n, c, h, w = x.shape
    if c % 64:
        raise RuntimeError(f"split_q: channels must be a multiple of 64, got {c}")
    xq = torch.empty((n * h * w, 4 * c), device=x.device, dtype=torch.uint8)
    check(_lib.lib().avse_split16_known(n * h * w * (c // 64), ptr(x), ptr(xq), ptr(known), stream_ptr(x.device)),
          "avse_split16_known")
    return xq, known


def sconv_wprep(w, transposed, wmax):
    """W (co, ci, 3, 3) -> sconv.hip's split weight image (transposed: the stride-1 input gradient's flipped W')."""
    _need_gpu(w)
    co, ci = w.shape[0], w.shape[1]
    L = _lib.lib()
    wq = torch.empty(int(L.avse_sconv_wprep_bytes(co, ci)), device=w.device, dtype=torch.uint8)
    check(L.avse_sconv_wprep(co, ci, ptr(w.float().contiguous()), int(bool(transposed)), ptr(wq), ptr(wmax),
                             stream_ptr(w.device)), "avse_sconv_wprep")
    return wq


def sconv_fwd(xs, xshape, w, stride, transposed=False):
    """conv2d(x, w, stride=stride, padding=1) on csrc/sconv.hip from x's split xs = (xq, xmax) (split_nhwc) and shape
    (N, ci, H, W); transposed=True: the stride-1 input gradient (x = dY, w the forward's (co, ci, 3, 3) weight).
    Returns the (N, co, Ho, Wo) output in channels-last memory."""
    xq, xm = xs
    _need_gpu(xq, w)
    n, ci, h, wd = xshape
    co = w.shape[1] if transposed else w.shape[0]
    if transposed and stride != 1:
        raise RuntimeError("sconv_fwd: the transposed (input gradient) form is stride 1 only")
    wm = torch.empty(1, device=w.device, dtype=torch.int32)
    wq = sconv_wprep(w, transposed, wm)
    ho, wo = (h - 1) // stride + 1, (wd - 1) // stride + 1
    y = torch.empty((n, co, ho, wo), device=xq.device, dtype=torch.float32, memory_format=torch.channels_last)
    tap = _tap_begin("avse_sconv_fwd", xq.device)
    check(_lib.lib().avse_sconv_fwd(n, h, wd, ci, co, stride, ptr(xq), ptr(xm), ptr(wq), ptr(wm), ptr(y),
                                    stream_ptr(xq.device)), "avse_sconv_fwd")
    _tap_end(tap)
    return y


def sconv_dgrad2_ok(xshape, cout):
    """True when csrc/sconv.hip's stride-2 input gradient takes Conv2d(ci, cout, 3, 2, padding=1) on an input of shape
    xshape = (N, ci, H, W)."""
    n, ci, h, w = xshape
    return bool(_lib.lib().avse_sconv_dgrad2_supported(n, h, w, ci, cout))


def sconv_dgrad2(dys, xshape, w):
    """Input gradient (N, ci, H, W) (channels-last memory) of conv2d(x, w, stride=2, padding=1) from the split output
    gradient dys = (dyq, dymax) (csrc/sconv.hip: the 4 parity phases of dX as stride-1 split-fp16 MFMA GEMMs over dY,
    only the taps of each phase)."""
    dyq, dym = dys
    _need_gpu(dyq, w)
    n, ci, h, wd = xshape
    co = w.shape[0]
    L = _lib.lib()
    wm = torch.empty(1, device=w.device, dtype=torch.int32)
    wq = torch.empty(int(L.avse_sconv_wprep_bytes(co, ci)), device=w.device, dtype=torch.uint8)
    check(L.avse_sconv_wprep(co, ci, ptr(w.float().contiguous()), 2, ptr(wq), ptr(wm), stream_ptr(w.device)),
          "avse_sconv_wprep")
    dx = torch.empty((n, ci, h, wd), device=dyq.device, dtype=torch.float32, memory_format=torch.channels_last)
    tap = _tap_begin("avse_sconv_dgrad2", dyq.device)
    check(L.avse_sconv_dgrad2(n, h, wd, ci, co, ptr(dyq), ptr(dym), ptr(wq), ptr(wm), ptr(dx), stream_ptr(dyq.device)),
          "avse_sconv_dgrad2")
    _tap_end(tap)
    return dx


def sconv_wgrad(xs, dys, xshape, cout, stride):
    """dW (cout, ci, 3, 3) of Conv2d(ci, cout, 3, stride, padding=1, bias=False) from the splits of the input
    (xs = (xq, xmax), shape xshape = (N, ci, H, W)) and of the output gradient (dys), csrc/sconv.hip."""
    (xq, xm), (dyq, dym) = xs, dys
    _need_gpu(xq, dyq)
    n, ci, h, wd = xshape
    L = _lib.lib()
    nb = L.avse_sconv_wgrad_workspace_bytes(n, h, wd, ci, cout, stride)
    if nb <= 0:
        raise RuntimeError(f"sconv_wgrad: unsupported shape {tuple(xshape)} -> {cout}, stride {stride}")
    dw = torch.empty((cout, ci, 3, 3), device=xq.device, dtype=torch.float32)
    ws = torch.empty((nb + 3) // 4, device=xq.device, dtype=torch.float32)
    tap = _tap_begin("avse_sconv_wgrad", xq.device)
    check(L.avse_sconv_wgrad(n, h, wd, ci, cout, stride, ptr(xq), ptr(xm), ptr(dyq), ptr(dym), ptr(dw), ptr(ws),
                             stream_ptr(xq.device)), "avse_sconv_wgrad")
    _tap_end(tap)
    return dw


# ------------------------------------------------------------------------ PReLU

def _ncs(x):
    N, C = x.shape[0], x.shape[1]
    S = x.numel() // max(1, N * C)
    return N, C, S


def _nhwc(x):
    """(R, C) of a channels-last 4-D activation the NHWC PReLU kernels take, else None."""
    if x.dim() != 4 or x.is_contiguous() or not x.is_contiguous(memory_format=torch.channels_last):
        return None
    C = x.shape[1]
    if C % 4 or 256 % (C // 4):
        return None
    return x.numel() // C, C


def prelu_fwd(x, a):
    _need_gpu(x, a)
    if x.dtype == torch.float32 and _nhwc(x) is not None:
        R, C = _nhwc(x)
        y = torch.empty_like(x)                      # preserves channels-last strides
        check(_lib.lib().avse_prelu_nhwc_fwd(R, C, a.numel(), ptr(x), ptr(a.contiguous()), ptr(y),
                                             stream_ptr(x.device)), "avse_prelu_nhwc_fwd")
        return y
    x = x.contiguous()
    if x.dtype != torch.float32:
        raise RuntimeError("prelu kernels are fp32")
    N, C, S = _ncs(x)
    y = torch.empty_like(x)
    check(_lib.lib().avse_prelu_fwd(N, C, S, a.numel(), ptr(x), ptr(a.contiguous()), ptr(y), stream_ptr(x.device)),
          "avse_prelu_fwd")
    return y


def prelu_bwd(x, a, dy):
    _need_gpu(x, a, dy)
    if x.dtype == torch.float32 and _nhwc(x) is not None:
        R, C = _nhwc(x)
        dy = dy.float().contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x)
        da = torch.empty((a.numel(),), device=x.device, dtype=torch.float32)
        L = _lib.lib()
        ws = torch.empty((max(4, L.avse_prelu_nhwc_bwd_workspace_bytes(R, C)) + 3) // 4, device=x.device,
                         dtype=torch.float32)
        check(L.avse_prelu_nhwc_bwd(R, C, a.numel(), ptr(x), ptr(a.contiguous()), ptr(dy), ptr(dx), ptr(da), ptr(ws),
                                    stream_ptr(x.device)), "avse_prelu_nhwc_bwd")
        return dx, da.view_as(a)
    x, dy = x.contiguous(), dy.contiguous().float()
    N, C, S = _ncs(x)
    dx = torch.empty_like(x)
    da = torch.empty((a.numel(),), device=x.device, dtype=torch.float32)
    ws = torch.empty((N * C,), device=x.device, dtype=torch.float32)
    check(_lib.lib().avse_prelu_bwd(N, C, S, a.numel(), ptr(x), ptr(a.contiguous()), ptr(dy), ptr(dx), ptr(da), ptr(ws),
                                    stream_ptr(x.device)), "avse_prelu_bwd")
    return dx, da.view_as(a)


# ------------------------------------------------------------------------ max pooling over (H, W) planes

def maxpool_planes_fwd(x, k, s, p):
    """x (..., H, W) contiguous fp32, window k = (KH, KW), stride s, padding p -> (y (..., Ho, Wo), idx uint8)."""
    _need_gpu(x)
    x = x.float().contiguous()
    H, W = x.shape[-2], x.shape[-1]
    planes = x.numel() // (H * W)
    L = _lib.lib()
    Ho, Wo = L.avse_maxpool2d_out_size(H, k[0], s[0], p[0]), L.avse_maxpool2d_out_size(W, k[1], s[1], p[1])
    y = torch.empty(x.shape[:-2] + (Ho, Wo), device=x.device, dtype=torch.float32)
    idx = torch.empty(y.shape, device=x.device, dtype=torch.uint8)
    check(L.avse_maxpool2d_fwd(planes, H, W, k[0], k[1], s[0], s[1], p[0], p[1], ptr(x), ptr(y), ptr(idx),
                               stream_ptr(x.device)), "avse_maxpool2d_fwd")
    return y, idx


def transpose_cp(x):
    """x (N, C, P) contiguous fp32 -> y (N, P, C) contiguous with y[n, p, c] = x[n, c, p] (csrc/transpose.hip)."""
    _need_gpu(x)
    if x.dtype != torch.float32 or not x.is_contiguous() or x.dim() != 3:
        raise ValueError("transpose_cp: (N, C, P) contiguous fp32 expected")
    N, C, P = x.shape
    y = torch.empty((N, P, C), device=x.device, dtype=torch.float32)
    check(_lib.lib().avse_transpose_cp(N, C, P, ptr(x), ptr(y), stream_ptr(x.device)), "avse_transpose_cp")
    return y


def maxpool_planes_bwd(dy, idx, in_shape, k, s, p):
    _need_gpu(dy, idx)
    dy = dy.float().contiguous()
    H, W = in_shape[-2], in_shape[-1]
    planes = dy.numel() // (dy.shape[-2] * dy.shape[-1])
    dx = torch.empty(in_shape, device=dy.device, dtype=torch.float32)
    check(_lib.lib().avse_maxpool2d_bwd(planes, H, W, k[0], k[1], s[0], s[1], p[0], p[1], ptr(dy), ptr(idx), ptr(dx),
                                        stream_ptr(dy.device)), "avse_maxpool2d_bwd")
    return dx


# ------------------------------------------------------------------------ BatchNorm -> [+ res] -> act

ACT_NONE, ACT_RELU, ACT_PRELU = 0, 1, 2


def _bn_view(x):
    """(N, C, S) of x as the bnact kernels read it: contiguous (N, C, *spatial) or channels-last (S = 1)."""
    if x.is_contiguous():
        N, C = x.shape[0], x.shape[1]
        return N, C, x.numel() // max(1, N * C)
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        return x.numel() // x.shape[1], x.shape[1], 1
    if x.dim() == 5 and x.is_contiguous(memory_format=torch.channels_last_3d):
        return x.numel() // x.shape[1], x.shape[1], 1
    return None


def _same_layout(t, like):
    if t.stride() == like.stride():
        return t
    fmt = (torch.channels_last if like.dim() == 4 else torch.channels_last_3d) if not like.is_contiguous() \
        else torch.contiguous_format
    return t.contiguous(memory_format=fmt)


def _opt(t):
    return ptr(t) if t is not None else None


# Split-output tensors (round 5): bnact_fwd / bnact_bwd with q_out write their channels-last output directly as the
# fp16 hi / lo split of the split-fp16 convolutions (csrc/bnact.hip, "Q" layout: per pixel C / 16 chunks of [hi 16]
# [lo 16]) into an fp32 tensor of the output's shape (the same bytes), marked with SPLITQ_ATTR and the bound of its
# max |.| (ABSMAX_ATTR).  Only a split consumer may read it (split16 / split_q return its bytes as they are): the
# layers request it where the next convolution (forward) or the previous one (backward) is a split-fp16 kernel.
SPLITQ_ATTR = "_avse_splitq"


def is_split_q(t):
    return getattr(t, SPLITQ_ATTR, False) is True


def q_view(t):
    """The uint8 (N*H*W, 4 C) view of a split-output (N, C, H, W) channels-last tensor."""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c).view(torch.uint8)


def positive(t):
    """t > 0 elementwise (logical shape), for a split-output tensor from its fp16 hi / lo planes (the sign of hi + lo)."""
    if not is_split_q(t):
        return t > 0
    n, c, h, w = t.shape
    q = q_view(t).view(torch.float16).reshape(-1, c // 16, 2, 16)
    pos = (q[:, :, 0, :] > 0) | ((q[:, :, 0, :] == 0) & (q[:, :, 1, :] > 0))
    return pos.reshape(n, h, w, c).permute(0, 3, 1, 2)


def _q_ok(x, res):
    v = _bn_view(x)
    return (res is None and x.dim() == 4 and v is not None and v[2] == 1 and x.shape[1] % 64 == 0
            and not x.is_contiguous() and x.data_ptr() % 16 == 0)


def bnact_fwd(x, gamma, beta, running_mean, running_var, training, momentum, eps, act=ACT_NONE, alpha=None, res=None,
              q_out=False):
    """act(BatchNorm(x) [+ res]); returns (y, stats (C, 4) = mean hi, mean lo, rstd, bound of max |x - mean|).  y keeps
    x's format.  q_out (training, channels-last, C % 64 == 0, no residual; otherwise ignored): y is a split-output
    tensor (SPLITQ_ATTR)."""
    _need_gpu(x)
    if x.dtype != torch.float32:
        raise RuntimeError("bnact kernels are fp32")
    if _bn_view(x) is None:
        x = x.contiguous()
    N, C, S = _bn_view(x)
    if res is not None:
        res = _same_layout(res.float(), x)
    y = torch.empty_like(x)
    stats = torch.empty((C, 4), device=x.device, dtype=torch.float32)
    L = _lib.lib()
    ws = torch.empty((L.avse_bnact_workspace_bytes(N, C, S) + 3) // 4, device=x.device, dtype=torch.float32)
    a = alpha.float().contiguous() if alpha is not None else None
    ymax = torch.empty(1, device=x.device, dtype=torch.int32)
    if q_out and training and _q_ok(x, res):
        check(L.avse_bnact_fwd_q(N, C, S, ptr(x), _opt(gamma), _opt(beta), int(act), _opt(a),
                                 a.numel() if a is not None else 0, float(eps), float(momentum), _opt(running_mean),
                                 _opt(running_var), ptr(stats), ptr(y), ptr(ws), ptr(ymax), stream_ptr(x.device)),
              "avse_bnact_fwd_q")
        _set_absmax(y, ymax)
        setattr(y, SPLITQ_ATTR, True)
        return y, stats
    check(L.avse_bnact_fwd(N, C, S, ptr(x), _opt(res), _opt(gamma), _opt(beta), int(act), _opt(a),
                           a.numel() if a is not None else 0, int(bool(training)), float(eps), float(momentum),
                           _opt(running_mean), _opt(running_var), ptr(stats), ptr(y), ptr(ws), ptr(ymax),
                           stream_ptr(x.device)), "avse_bnact_fwd")
    _set_absmax(y, ymax)
    return y, stats


# The producer-side max |t| of a tensor (float bits in a 1-element int32 device tensor), attached to the tensor object by
# the kernels that compute it in their output pass (bnact fwd / bwd): a split consumer (split16 / split_q) then skips its
# absmax pass.  Only fresh outputs carry it, and nothing writes them in place before their consumers read them.
ABSMAX_ATTR = "_avse_absmax"


def _set_absmax(t, mb):
    setattr(t, ABSMAX_ATTR, mb)


def _known_absmax(t):
    mb = getattr(t, ABSMAX_ATTR, None)
    return mb if isinstance(mb, torch.Tensor) and mb.device == t.device else None


def bnact_bwd(x, res, dy, stats, gamma, beta, act, alpha, training, q_out=False):
    """-> (dx, dres or None, dgamma, dbeta, dalpha (alpha's shape) or None).  q_out (channels-last, C % 64 == 0, no
    residual; otherwise ignored): dx is a split-output tensor (SPLITQ_ATTR)."""
    _need_gpu(x, dy, stats)
    N, C, S = _bn_view(x)
    dy = _same_layout(dy.float(), x)
    if res is not None:
        res = _same_layout(res.float(), x)
    dx = torch.empty_like(x)
    dres = torch.empty_like(x) if res is not None else None
    dgamma = torch.empty((C,), device=x.device, dtype=torch.float32)
    dbeta = torch.empty((C,), device=x.device, dtype=torch.float32)
    a = alpha.float().contiguous() if alpha is not None else None
    dalpha_c = torch.empty((C,), device=x.device, dtype=torch.float32) if a is not None else None
    L = _lib.lib()
    ws = torch.empty((L.avse_bnact_workspace_bytes(N, C, S) + 3) // 4, device=x.device, dtype=torch.float32)
    dxmax = torch.empty(1, device=x.device, dtype=torch.int32)
    q = q_out and _q_ok(x, res) and dy.data_ptr() % 16 == 0
    if q:
        check(L.avse_bnact_bwd_q(N, C, S, ptr(x), ptr(dy), ptr(stats), _opt(gamma), _opt(beta), int(act), _opt(a),
                                 a.numel() if a is not None else 0, int(bool(training)), ptr(dx), ptr(dgamma),
                                 ptr(dbeta), _opt(dalpha_c), ptr(ws), ptr(dxmax), stream_ptr(x.device)),
              "avse_bnact_bwd_q")
        setattr(dx, SPLITQ_ATTR, True)
    else:
        check(L.avse_bnact_bwd(N, C, S, ptr(x), _opt(res), ptr(dy), ptr(stats), _opt(gamma), _opt(beta), int(act),
                               _opt(a), a.numel() if a is not None else 0, int(bool(training)), ptr(dx), _opt(dres),
                               ptr(dgamma), ptr(dbeta), _opt(dalpha_c), ptr(ws), ptr(dxmax), stream_ptr(x.device)),
              "avse_bnact_bwd")
    _set_absmax(dx, dxmax)
    dalpha = None
    if a is not None:
        dalpha = (dalpha_c if a.numel() == C else dalpha_c.sum().reshape(1)).view_as(alpha)
    return dx, dres, dgamma, dbeta, dalpha


# ------------------------------------------------------------------------ PReLU -> gLN (avse4)

def prelu_gln_fwd(x, alpha, gamma, beta, eps=1e-8):
    """gLN(PReLU(x)) on (B, C, K); returns (y, stats (B, 2) = mean, rstd)."""
    _need_gpu(x, alpha, gamma, beta)
    x = x.float().contiguous()
    Bn, C, Kn = x.shape
    y = torch.empty_like(x)
    stats = torch.empty((Bn, 2), device=x.device, dtype=torch.float32)
    L = _lib.lib()
    ws = torch.empty((L.avse_prelu_gln_workspace_bytes(Bn, C) + 3) // 4, device=x.device, dtype=torch.float32)
    tap = _tap_begin("avse_prelu_gln_fwd", x.device)
    check(L.avse_prelu_gln_fwd(Bn, C, Kn, ptr(x), ptr(alpha.float().contiguous()), ptr(gamma.float().contiguous()),
                               ptr(beta.float().contiguous()), float(eps), ptr(y), ptr(stats), ptr(ws),
                               stream_ptr(x.device)), "avse_prelu_gln_fwd")
    _tap_end(tap)
    return y, stats


def prelu_gln_bwd(x, alpha, gamma, stats, dy, planes=False):
    """(dx, dalpha, dgamma, dbeta) of gLN(PReLU(x)).  planes: dx is written only as the split-fp16 planes of the GEMM
    that produced x (avse_prelu_gln_bwd_q) and returned as their carrier (PLANES_ATTR)."""
    _need_gpu(x, alpha, gamma, stats, dy)
    x, dy = x.float().contiguous(), dy.float().contiguous()
    Bn, C, Kn = x.shape
    dalpha = torch.empty((1,), device=x.device, dtype=torch.float32)
    dgamma = torch.empty((C,), device=x.device, dtype=torch.float32)
    dbeta = torch.empty((C,), device=x.device, dtype=torch.float32)
    L = _lib.lib()
    ws = torch.empty((L.avse_prelu_gln_workspace_bytes(Bn, C) + 3) // 4, device=x.device, dtype=torch.float32)
    if planes:
        dx, sp, cp = _planes_carrier((Bn, C, Kn), x.device)
        tap = _tap_begin("avse_prelu_gln_bwd_q", x.device)
        check(L.avse_prelu_gln_bwd_q(Bn, C, Kn, ptr(x), ptr(alpha.float().contiguous()), ptr(gamma.float().contiguous()),
                                     ptr(stats), ptr(dy), ptr(sp.hi), ptr(sp.lo), cp, ptr(sp.mb), ptr(dalpha),
                                     ptr(dgamma), ptr(dbeta), ptr(ws), stream_ptr(x.device)), "avse_prelu_gln_bwd_q")
        _tap_end(tap)
        return dx, dalpha, dgamma, dbeta
    dx = torch.empty_like(x)
    tap = _tap_begin("avse_prelu_gln_bwd", x.device)
    check(L.avse_prelu_gln_bwd(Bn, C, Kn, ptr(x), ptr(alpha.float().contiguous()), ptr(gamma.float().contiguous()),
                               ptr(stats), ptr(dy), ptr(dx), ptr(dalpha), ptr(dgamma), ptr(dbeta), ptr(ws),
                               stream_ptr(x.device)), "avse_prelu_gln_bwd")
    _tap_end(tap)
    return dx, dalpha, dgamma, dbeta


# ------------------------------------------------------------------------ depthwise dilated conv1d

def dwconv_fwd(x, w, dilation):
    _need_gpu(x, w)
    x = x.float().contiguous()
    Bn, C, Kn = x.shape
    w2 = w.reshape(C, -1).float().contiguous()
    y = torch.empty_like(x)
    check(_lib.lib().avse_dwconv_fwd(Bn, C, Kn, w2.shape[1], int(dilation), ptr(x), ptr(w2), ptr(y),
                                     stream_ptr(x.device)), "avse_dwconv_fwd")
    return y


def dwconv_bwd(x, w, dy, dilation):
    _need_gpu(x, w, dy)
    x, dy = x.float().contiguous(), dy.float().contiguous()
    Bn, C, Kn = x.shape
    w2 = w.reshape(C, -1).float().contiguous()
    P = w2.shape[1]
    dx = torch.empty_like(x)
    dw = torch.empty((C, P), device=x.device, dtype=torch.float32)
    L = _lib.lib()
    ws = torch.empty((L.avse_dwconv_bwd_workspace_bytes(Bn, C) + 3) // 4, device=x.device, dtype=torch.float32)
    check(L.avse_dwconv_bwd(Bn, C, Kn, P, int(dilation), ptr(x), ptr(w2), ptr(dy), ptr(dx), ptr(dw), ptr(ws),
                            stream_ptr(x.device)), "avse_dwconv_bwd")
    return dx, dw.view_as(w)


# ------------------------------------------------------------------------ fused dwconv <-> PReLU -> gLN (avse4)

# The split planes a producer wrote for the split-fp16 GEMM that consumes its output (PLANES_ATTR: a Split on an fp32
# "carrier" tensor of the output's shape whose storage holds the two planes; its own elements are not the values, so
# only that GEMM may read it — avse4._PointwiseFn).
PLANES_ATTR = "_avse_planes"


def planes_of(t):
    return getattr(t, PLANES_ATTR, None)


def _planes_carrier(shape, device):
    """(carrier, Split) for a (b, r, c) output written as split planes with rows of cp = c rounded up to 8 elements:
    one allocation of 4 (b r cp + 16) bytes = the hi plane, 16 elements of slack, the lo plane, 16 of slack."""
    b, r, c = shape
    cp = (c + 7) // 8 * 8
    n = b * r * cp + 16
    store = torch.empty(n, device=device, dtype=torch.float32).untyped_storage()
    carrier = torch.empty(0, device=device, dtype=torch.float32).set_(store, 0, (b, r, c), (r * cp, cp, 1))
    hi = torch.empty(0, device=device, dtype=torch.float16).set_(store, 0, (b, r, c), (r * cp, cp, 1))
    lo = torch.empty(0, device=device, dtype=torch.float16).set_(store, n, (b, r, c), (r * cp, cp, 1))
    mb = torch.empty(1, device=device, dtype=torch.int32)
    sp = Split(hi, lo, mb)
    setattr(carrier, PLANES_ATTR, sp)
    return carrier, sp, cp


def dwconv_gln_fwd(x, w, dilation, alpha, gamma, beta, eps=1e-8, planes=False):
    """y1 = depthwise dilated conv1d(x) (w (C, 1, P)), y = gLN(PReLU(y1)); returns (y, y1, stats (B, 2)).  planes: y is
    written only as the split-fp16 planes of its consumer GEMM (avse_dwconv_gln_fwd_q) and returned as their carrier
    (PLANES_ATTR)."""
    _need_gpu(x, w, alpha, gamma, beta)
    x = x.float().contiguous()
    Bn, C, Kn = x.shape
    w2 = w.reshape(C, -1).float().contiguous()
    stats = torch.empty((Bn, 2), device=x.device, dtype=torch.float32)
    L = _lib.lib()
    ws = torch.empty((L.avse_dwconv_gln_workspace_bytes(Bn, C) + 3) // 4, device=x.device, dtype=torch.float32)
    y1 = torch.empty_like(x)
    if planes:
        y, sp, cp = _planes_carrier((Bn, C, Kn), x.device)
        tap = _tap_begin("avse_dwconv_gln_fwd_q", x.device)
        check(L.avse_dwconv_gln_fwd_q(Bn, C, Kn, w2.shape[1], int(dilation), ptr(x), ptr(w2),
                                      ptr(alpha.float().contiguous()), ptr(gamma.float().contiguous()),
                                      ptr(beta.float().contiguous()), float(eps), ptr(y1), ptr(sp.hi), ptr(sp.lo), cp,
                                      ptr(sp.mb), ptr(stats), ptr(ws), stream_ptr(x.device)), "avse_dwconv_gln_fwd_q")
        _tap_end(tap)
        return y, y1, stats
    y = torch.empty_like(x)
    tap = _tap_begin("avse_dwconv_gln_fwd", x.device)
    check(L.avse_dwconv_gln_fwd(Bn, C, Kn, w2.shape[1], int(dilation), ptr(x), ptr(w2), ptr(alpha.float().contiguous()),
                                ptr(gamma.float().contiguous()), ptr(beta.float().contiguous()), float(eps), ptr(y1),
                                ptr(y), ptr(stats), ptr(ws), stream_ptr(x.device)), "avse_dwconv_gln_fwd")
    _tap_end(tap)
    return y, y1, stats


def dwconv_gln_bwd(x, w, dilation, y1, alpha, gamma, stats, dy):
    """-> (dx, dw (like w), dalpha (1,), dgamma (C,), dbeta (C,))."""
    _need_gpu(x, w, y1, alpha, gamma, stats, dy)
    x, dy = x.float().contiguous(), dy.float().contiguous()
    Bn, C, Kn = x.shape
    w2 = w.reshape(C, -1).float().contiguous()
    dx = torch.empty_like(x)
    dw = torch.empty((C, w2.shape[1]), device=x.device, dtype=torch.float32)
    dalpha = torch.empty((1,), device=x.device, dtype=torch.float32)
    dgamma = torch.empty((C,), device=x.device, dtype=torch.float32)
    dbeta = torch.empty((C,), device=x.device, dtype=torch.float32)
    L = _lib.lib()
    ws = torch.empty((L.avse_dwconv_gln_workspace_bytes(Bn, C) + 3) // 4, device=x.device, dtype=torch.float32)
    tap = _tap_begin("avse_dwconv_gln_bwd", x.device)
    check(L.avse_dwconv_gln_bwd(Bn, C, Kn, w2.shape[1], int(dilation), ptr(x), ptr(w2), ptr(y1.contiguous()),
                                ptr(alpha.float().contiguous()), ptr(gamma.float().contiguous()), ptr(stats), ptr(dy),
                                ptr(dx), ptr(dw), ptr(dalpha), ptr(dgamma), ptr(dbeta), ptr(ws), stream_ptr(x.device)),
          "avse_dwconv_gln_bwd")
    _tap_end(tap)
    return dx, dw.view_as(w), dalpha, dgamma, dbeta


# ------------------------------------------------------------------------ LSTM recurrence

def lstm_fwd(gx, w_hh, hout=None, reverse=False):
    """gx (B, T, 4H) = X W_ih^T + b_ih + b_hh; w_hh (4H, H).  Returns (h (B, T, H) [or the passed strided hout
    view, unit stride over H], c (B, T, H), gates (B, T, 4H) post-activation i, f, g, o)."""
    _need_gpu(gx, w_hh)
    gx = gx.float().contiguous()
    Bn, T, H4 = gx.shape
    H = H4 // 4
    if tuple(w_hh.shape) != (H4, H):
        raise RuntimeError(f"w_hh must be ({H4}, {H}), got {tuple(w_hh.shape)}")
    if hout is None:
        hout = torch.empty((Bn, T, H), device=gx.device, dtype=torch.float32)
    elif hout.dtype != torch.float32 or hout.stride(-1) != 1 or tuple(hout.shape) != (Bn, T, H):
        raise RuntimeError("hout must be an fp32 (B, T, H) view with unit stride over H")
    c_all = torch.empty((Bn, T, H), device=gx.device, dtype=torch.float32)
    gates = torch.empty((Bn, T, H4), device=gx.device, dtype=torch.float32)
    L = _lib.lib()
    ws = _lstm_group_ws(L, Bn, H, gx.device, backward=False)
    if ws is not None:      # W_hh resident in LDS, each sequence over G workgroups (csrc/lstm_group.hip)
        check(L.avse_lstm_fwd_group(Bn, T, H, int(bool(reverse)), ptr(gx), ptr(w_hh.float().contiguous()), ptr(hout),
                                    hout.stride(0), hout.stride(1), ptr(c_all), ptr(gates), ptr(ws),
                                    ptr(_kernel_error_flag(gx.device)), stream_ptr(gx.device)), "avse_lstm_fwd_group")
        return hout, c_all, gates
    whhT = w_hh.float().t().contiguous()
    check(L.avse_lstm_fwd(Bn, T, H, int(bool(reverse)), ptr(gx), ptr(whhT), ptr(hout), hout.stride(0),
                          hout.stride(1), ptr(c_all), ptr(gates), stream_ptr(gx.device)), "avse_lstm_fwd")
    return hout, c_all, gates


_GROUP_CAPACITY = {}     # (device index, H, backward) -> workgroups of that grouped kernel the device holds at once
_ERROR_FLAGS = {}        # device index -> int32 sticky error flag of the grouped LSTM launches (never freed)


# While > 0 the grouped LSTM kernels are not launched (lstm.hip's single-workgroup kernels run instead).  ddp.Trainer
# raises it around the backward at world > 1: bucket all-reduces launched from gradient hooks can be in flight then,
# and RCCL's kernels hold CUs the grouped launch needs co-resident (its static capacity query cannot see them).  The
# forward needs no such guard: every collective of the previous step was waited for by the compute stream before it.
NO_GROUPED_LSTM = 0


class no_grouped_lstm:
    """Context manager: lstm.hip's kernels for every LSTM launch inside (process-wide: autograd's device threads run
    the backward, so a thread-local switch would not reach them)."""

    def __enter__(self):
        global NO_GROUPED_LSTM
        NO_GROUPED_LSTM += 1
        return self

    def __exit__(self, *exc):
        global NO_GROUPED_LSTM
        NO_GROUPED_LSTM -= 1
        return False


# the grouped recurrence (csrc/lstm_group.hip) where it applies; False: lstm.hip everywhere (a test's comparison)
LSTM_GROUP = True
# a test hook: pretend the device holds at most this many grouped-LSTM workgroups at once (None: the device's capacity)
LSTM_GROUP_CAPACITY_LIMIT = None


def lstm_group_allowed():
    return NO_GROUPED_LSTM == 0 and LSTM_GROUP


def _lstm_group_ws(L, Bn, H, device, backward):
    """Workspace of the grouped LSTM kernels, or None when they do not apply: LSTM_GROUP False or inside
    no_grouped_lstm(); B * G > 256 or H > 384 (avse_lstm_group_size); or B * G workgroups cannot be co-resident on
    this device (avse_lstm_group_capacity).  Those cases run lstm.hip's one-workgroup-per-sequence kernels."""
    if not lstm_group_allowed():
        return None
    G = int(L.avse_lstm_group_size(Bn, H))
    if G == 0:
        return None
    key = (device.index, H, bool(backward))
    if key not in _GROUP_CAPACITY:
        with torch.cuda.device(device):
            _GROUP_CAPACITY[key] = int(L.avse_lstm_group_capacity(H, int(bool(backward))))
    cap = _GROUP_CAPACITY[key]
    if LSTM_GROUP_CAPACITY_LIMIT is not None:
        cap = min(cap, int(LSTM_GROUP_CAPACITY_LIMIT))
    if Bn * G > cap:
        return None
    nb = int(L.avse_lstm_group_workspace_bytes(Bn, H))
    return torch.empty((nb + 15) // 16 * 4, device=device, dtype=torch.int32)


def _kernel_error_flag(device):
    """The device's sticky error flag (int32, 0 = no error) that the grouped LSTM kernels write a timeout code into.
    Allocated once per device outside any graph pool and never freed, so captured launches keep a valid pointer."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _ERROR_FLAGS:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("the grouped LSTM error flag must be created before graph capture (run the step "
                               "eagerly first)")
        _ERROR_FLAGS[idx] = torch.zeros(1, device=torch.device("cuda", idx), dtype=torch.int32)
    return _ERROR_FLAGS[idx]


class HipKernelError(RuntimeError):
    """A hand-written kernel reported invalid outputs through its sticky error flag."""


def lstm_group_status(device=None):
    """0 when every grouped LSTM launch on `device` (default: all used devices) since the last reset completed its
    hand-offs; else the timeout code one of them wrote (0x71000000 + step): a sequence's workgroups were not
    co-resident and that launch's outputs are invalid.  Synchronises with the flag's device."""
    return max([int(f.item()) & 0xFFFFFFFF for f in _flags_of(device)] + [0])


def _flags_of(device):
    if device is None:
        return list(_ERROR_FLAGS.values())
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    return [f for i, f in _ERROR_FLAGS.items() if i == idx]


def raise_if_kernel_error(device=None, reset=True):
    """Raise HipKernelError when a grouped LSTM launch timed out (see lstm_group_status); with ``reset`` clear the
    flag afterwards (a raised error is reported once)."""
    code = lstm_group_status(device)
    if code and reset:
        for f in _flags_of(device):      # only the flags that were read: another device's error stays reported
            f.zero_()
    if code:
        raise HipKernelError(kernel_error_message(code))


def kernel_error_message(code):
    return (f"grouped LSTM recurrence timed out waiting for its workgroups (code {code:#x}): the grid was not "
            "co-resident on the GPU; the step's outputs and gradients are invalid")


def lstm_bwd(dh, gates, c_all, w_hh, reverse=False):
    """dh (B, T, H) gradient of the h output (any strides with unit stride over H) -> dgates (B, T, 4H), the
    gradient of the pre-activation gates."""
    _need_gpu(dh, gates, c_all, w_hh)
    dh = dh.float()
    if dh.stride(-1) != 1:
        dh = dh.contiguous()
    Bn, T, H = dh.shape
    L = _lib.lib()
    dg = torch.empty((Bn, T, 4 * H), device=dh.device, dtype=torch.float32)
    ws = _lstm_group_ws(L, Bn, H, dh.device, backward=True)
    if ws is not None:
        check(L.avse_lstm_bwd_group(Bn, T, H, int(bool(reverse)), ptr(dh), dh.stride(0), dh.stride(1),
                                    ptr(gates.contiguous()), ptr(c_all.contiguous()), ptr(w_hh.float().contiguous()),
                                    ptr(dg), ptr(ws), ptr(_kernel_error_flag(dh.device)), stream_ptr(dh.device)),
              "avse_lstm_bwd_group")
        return dg
    Hp = int(L.avse_lstm_padded_hidden(H))
    w_pad = torch.nn.functional.pad(w_hh.float(), (0, Hp - H)).contiguous()
    check(L.avse_lstm_bwd(Bn, T, H, int(bool(reverse)), ptr(dh), dh.stride(0), dh.stride(1), ptr(gates.contiguous()),
                          ptr(c_all.contiguous()), ptr(w_pad), ptr(dg), stream_ptr(dh.device)), "avse_lstm_bwd")
    return dg


# ------------------------------------------------------------------------ bf16 projection GEMM (Mamba in/out_proj)


def _extent(t):
    """Elements readable from t.data_ptr() to the end of t's storage."""
    return t.untyped_storage().nbytes() // t.element_size() - t.storage_offset()


def _gemm_operand(t):
    """(batch stride, stride of the row index, stride of k) of a (b|1, rows, k) operand; None when neither of the
    last two strides is 1 or the other one is not a multiple of 8 elements (16 B)."""
    bs = 0 if t.shape[0] == 1 else t.stride(0)
    sx, sk = t.stride(1), t.stride(2)
    if t.shape[1] == 1:                     # one row: either layout reads it
        sx = 8 if sk == 1 else 1
    if sk == 1 and sx % 8 == 0 and sx > 0:
        return bs, sx, sk
    if sx == 1 and sk % 8 == 0 and sk > 0:
        return bs, sx, sk
    return None


def gemm_bf16_supported(P, Q, out, fold=1):
    """True when avse_gemm_bf16 takes out[g, q, p] = sum_{b in group g} sum_k P[b, p, k] Q[b, q, k] as laid out
    (see gemm_bf16)."""
    if not (P.is_cuda and P.dtype == Q.dtype == torch.bfloat16 and out.dtype in (torch.bfloat16, torch.float32)):
        return False
    if P.dim() != 3 or Q.dim() != 3 or out.dim() != 3 or P.shape[2] != Q.shape[2] or P.shape[2] < 1:
        return False
    b = out.shape[0] * fold
    if out.shape[1:] != (Q.shape[1], P.shape[1]) or P.shape[0] not in (1, b) or Q.shape[0] not in (1, b):
        return False
    if max(P.shape[0], Q.shape[0]) != b and fold != 1:
        return False
    if out.stride(2) != 1 or out.stride(1) % 4 or out.data_ptr() % (16 if out.dtype == torch.float32 else 8):
        return False
    if P.data_ptr() % 16 or Q.data_ptr() % 16:
        return False
    return _gemm_operand(P) is not None and _gemm_operand(Q) is not None


def gemm_bf16(P, Q, out, alpha=1.0, fold=1):
    """out[g, q, p] = alpha * sum_{b = g fold .. g fold + fold - 1} sum_k P[b, p, k] * Q[b, q, k] on the bf16 MFMA GEMM
    (csrc/projgemm.hip): bf16 operands, fp32 accumulation, bf16 or fp32 out.  P (b or 1, mp, k), Q (b or 1, mq, k) are
    strided views whose k or row stride is 1 (a batch of 1 is shared by every batch); out (b / fold, mq, mp) with
    stride(2) == 1.  fold > 1 sums groups of batches (the weight gradients).  Returns out."""
    _need_gpu(P, Q, out)
    if not gemm_bf16_supported(P, Q, out, fold):
        raise RuntimeError(f"avse_gemm_bf16: unsupported operands P {tuple(P.shape)}/{P.stride()} "
                           f"Q {tuple(Q.shape)}/{Q.stride()} out {tuple(out.shape)}/{out.stride()} ({P.dtype}, "
                           f"fold {fold})")
    a = _lib.GemmBf16Args()
    a.batch, a.mp, a.mq, a.k, a.fold = out.shape[0] * fold, P.shape[1], Q.shape[1], P.shape[2], fold
    a.p, (a.p_bs, a.p_sx, a.p_sk), a.p_extent = P.data_ptr(), _gemm_operand(P), _extent(P)
    a.q, (a.q_bs, a.q_sx, a.q_sk), a.q_extent = Q.data_ptr(), _gemm_operand(Q), _extent(Q)
    a.c, a.c_bs, a.c_sq = out.data_ptr(), out.stride(0), out.stride(1)
    a.alpha, a.c_dtype = float(alpha), _dtype_code(out.dtype)
    tap = _tap_begin("avse_gemm_bf16", out.device)
    check(_lib.lib().avse_gemm_bf16(a, stream_ptr(out.device)), "avse_gemm_bf16")
    _tap_end(tap)
    return out


# ------------------------------------------------------------------------ fp32 GEMM on split fp16 planes (C3 projections)

class Split:
    """fp16 hi / lo planes of an fp32 tensor (same shape and strides) and its max-|x| bits (split_planes); ``t()`` is the
    transposed (1, 2) view of both planes, for the GEMM operand that reads the tensor transposed."""

    def __init__(self, hi, lo, mb):
        self.hi, self.lo, self.mb = hi, lo, mb

    def t(self):
        return Split(self.hi.transpose(1, 2), self.lo.transpose(1, 2), self.mb)


def add_max(a_full, b_full, l):
    """a + b over two contiguous (b, c, lp) padded storages (kernels.bdl_empty rows) -> (the sum's (b, c, l) view
    carrying max |sum| over the logical columns as its producer-side max, csrc/projgemm.hip avse_add_max)."""
    _need_gpu(a_full, b_full)
    y = torch.empty_like(a_full)
    mb = torch.empty(1, device=a_full.device, dtype=torch.int32)
    nb, c, lp = a_full.shape
    check(_lib.lib().avse_add_max(nb * c, lp, l, ptr(a_full), ptr(b_full), ptr(y), ptr(mb), stream_ptr(a_full.device)),
          "avse_add_max")
    v = y[..., :l]
    _set_absmax(v, mb)
    return v


def add_max_flat(a, b):
    """a + b for two contiguous fp32 tensors of one shape (numel % 4 == 0, 16-B aligned) -> the sum carrying max |sum|
    as its producer-side max (avse_add_max over one row): a residual sum whose consumer splits it skips its absmax pass."""
    _need_gpu(a, b)
    n = a.numel()
    y = torch.empty_like(a)
    mb = torch.empty(1, device=a.device, dtype=torch.int32)
    check(_lib.lib().avse_add_max(1, n, n, ptr(a), ptr(b), ptr(y), ptr(mb), stream_ptr(a.device)), "avse_add_max")
    _set_absmax(y, mb)
    return y


def add_max_flat_ok(a, b):
    return (a.is_cuda and a.dtype == b.dtype == torch.float32 and a.shape == b.shape and a.is_contiguous()
            and b.is_contiguous() and a.numel() % 4 == 0 and a.numel() < (1 << 33) and a.data_ptr() % 16 == 0
            and b.data_ptr() % 16 == 0)


def split_planes(t):
    """t (b, r, c) fp32 view with stride(2) == 1 or stride(1) == 1 -> Split(hi, lo, maxbits): fp16 planes of t's shape and
    strides holding fp16(t 2^e) and the remainder (csrc/projgemm.hip avse_split16_planes), and max |t|'s bits."""
    _need_gpu(t)
    if t.dtype != torch.float32 or t.dim() != 3:
        raise RuntimeError("split_planes: (b, r, c) fp32 views only")
    # flat buffers with 16 elements of slack past the last element: a 16-B DMA starting at any element stays inside the
    # GEMM's buffer range (a load straddling the range's end returns 0 for all of its 8 elements)
    span = 1 + sum((n - 1) * st for n, st in zip(t.size(), t.stride()))
    hi = torch.empty(span + 16, device=t.device, dtype=torch.float16).as_strided(t.size(), t.stride())
    lo = torch.empty(span + 16, device=t.device, dtype=torch.float16).as_strided(t.size(), t.stride())
    known = _known_absmax(t)                  # the producer's max (add_rmsnorm_fwd, rmsnorm_bwd): the split pass only
    mb = known if known is not None else torch.empty(1, device=t.device, dtype=torch.int32)
    v = t if t.stride(2) == 1 else t.transpose(1, 2)
    if v.stride(2) != 1:
        raise RuntimeError(f"split_planes: no unit stride in {t.stride()}")
    b, r, c = v.shape
    fn = _lib.lib().avse_split16_planes_known if known is not None else _lib.lib().avse_split16_planes
    check(fn(b, r, c, ptr(v), v.stride(0) if b > 1 else (r - 1) * v.stride(1) + c, v.stride(1), ptr(hi), ptr(lo),
             ptr(mb), stream_ptr(t.device)), "avse_split16_planes")
    return Split(hi, lo, mb)


def split_rows8(t):
    """t (b, r, c) fp32 with stride(2) == 1 -> Split whose planes are (b, r, c) views of (b, r, cp) storage, cp = c
    rounded up to a multiple of 8 (csrc/projgemm.hip avse_split16_planes_to): an operand of avse_gemm_f32s read along c
    or along r whatever c is (the avse4 (B, C, K) activations, K = 3999).  The pad columns are never written; the GEMM
    only reads them into output rows it does not store (along r) or into the zeroed tail of its last k-stage (along c)."""
    _need_gpu(t)
    if t.dtype != torch.float32 or t.dim() != 3 or t.stride(2) != 1:
        raise RuntimeError("split_rows8: (b, r, c) fp32 views with a unit last stride only")
    b, r, c = t.shape
    cp = (c + 7) // 8 * 8
    n = b * r * cp + 16                        # 16 elements of slack: a 16-B DMA at any element stays in the range
    hi = torch.empty(n, device=t.device, dtype=torch.float16).as_strided((b, r, c), (r * cp, cp, 1))
    lo = torch.empty(n, device=t.device, dtype=torch.float16).as_strided((b, r, c), (r * cp, cp, 1))
    known = _known_absmax(t)
    mb = known if known is not None else torch.empty(1, device=t.device, dtype=torch.int32)
    x_bs = t.stride(0) if b > 1 else (r - 1) * t.stride(1) + c
    check(_lib.lib().avse_split16_planes_to(b, r, c, ptr(t), x_bs, t.stride(1), ptr(hi), ptr(lo), r * cp, cp, ptr(mb),
                                            int(known is not None), stream_ptr(t.device)), "avse_split16_planes_to")
    return Split(hi, lo, mb)


def gemm_f32s_supported(P, Q, out, fold=1):
    """True when avse_gemm_f32s takes out[g, q, p] = sum_{b in g} sum_k P[b, p, k] Q[b, q, k] for these fp32 views."""
    return P.is_cuda and P.dtype == Q.dtype == torch.float32 and _f32s_layout_ok(P, Q, out, fold)


def _f32s_layout_ok(P, Q, out, fold=1):
    """The shape / stride rules of avse_gemm_f32s (P, Q: the operands or their split planes; out fp32)."""
    if out.dtype != torch.float32:
        return False
    if P.dim() != 3 or Q.dim() != 3 or out.dim() != 3 or P.shape[2] != Q.shape[2] or P.shape[2] < 1:
        return False
    b = out.shape[0] * fold
    if out.shape[1:] != (Q.shape[1], P.shape[1]) or P.shape[0] not in (1, b) or Q.shape[0] not in (1, b):
        return False
    if max(P.shape[0], Q.shape[0]) != b and fold != 1:
        return False
    # fp32 rows of any stride without folding (stored per element when not 16-B aligned); folded: 16-B rows
    if out.stride(2) != 1 or (fold != 1 and out.stride(1) % 4) or out.data_ptr() % 16:
        return False
    return _gemm_operand(P) is not None and _gemm_operand(Q) is not None


def gemm_f32s(P, Q, out, alpha=1.0, fold=1, ps=None, qs=None):
    """out[g, q, p] = alpha * sum_{b in group g} sum_k P[b, p, k] * Q[b, q, k] in fp32 on the split-fp16 MFMA GEMM
    (csrc/projgemm.hip avse_gemm_f32s: both operands split into hi / lo fp16 planes, three MFMAs per product, fp32
    accumulation, fp32-accurate).  Same operand rules as gemm_bf16; out fp32.  ps / qs: the operands' Split when the
    caller already made it (an operand used by two GEMMs is split once).  Returns out."""
    _need_gpu(P, Q, out)
    if not gemm_f32s_supported(P, Q, out, fold):
        raise RuntimeError(f"avse_gemm_f32s: unsupported operands P {tuple(P.shape)}/{P.stride()} "
                           f"Q {tuple(Q.shape)}/{Q.stride()} out {tuple(out.shape)}/{out.stride()} (fold {fold})")
    for t, sp in ((P, ps), (Q, qs)):
        if sp is not None and (sp.hi.shape != t.shape or sp.hi.stride() != t.stride()):
            raise RuntimeError(f"gemm_f32s: split planes {tuple(sp.hi.shape)}/{sp.hi.stride()} do not match the operand "
                               f"{tuple(t.shape)}/{t.stride()}")
    return gemm_f32s_split(ps or split_planes(P), qs or split_planes(Q), out, alpha, fold)


def _plane_extent(sp):
    """Elements readable from both planes' starts (one range serves both: the planes of a carrier share a storage, the
    lo plane last)."""
    return min(_extent(sp.hi), _extent(sp.lo))


def gemm_f32s_split(sp, sq, out, alpha=1.0, fold=1):
    """gemm_f32s on operands given only by their Splits (the fp32 tensors need not be kept)."""
    _need_gpu(sp.hi, sq.hi, out)
    if not _f32s_layout_ok(sp.hi, sq.hi, out, fold):
        raise RuntimeError(f"avse_gemm_f32s: unsupported planes P {tuple(sp.hi.shape)}/{sp.hi.stride()} "
                           f"Q {tuple(sq.hi.shape)}/{sq.hi.stride()} out {tuple(out.shape)}/{out.stride()}")
    P, Q = sp.hi, sq.hi
    ph, pl, pm = sp.hi, sp.lo, sp.mb
    qh, ql, qm = sq.hi, sq.lo, sq.mb
    a = _lib.GemmF32sArgs()
    a.batch, a.mp, a.mq, a.k, a.fold = out.shape[0] * fold, P.shape[1], Q.shape[1], P.shape[2], fold
    a.p_hi, a.p_lo, (a.p_bs, a.p_sx, a.p_sk), a.p_extent, a.p_max = ph.data_ptr(), pl.data_ptr(), _gemm_operand(ph), \
        _plane_extent(sp), pm.data_ptr()
    a.q_hi, a.q_lo, (a.q_bs, a.q_sx, a.q_sk), a.q_extent, a.q_max = qh.data_ptr(), ql.data_ptr(), _gemm_operand(qh), \
        _plane_extent(sq), qm.data_ptr()
    a.c, a.c_bs, a.c_sq = out.data_ptr(), out.stride(0), out.stride(1)
    a.alpha = float(alpha)
    a.nsub = 1
    tap = _tap_begin("avse_gemm_f32s", out.device)
    check(_lib.lib().avse_gemm_f32s(a, stream_ptr(out.device)), "avse_gemm_f32s")
    _tap_end(tap, 2.0 * a.batch * a.mp * a.mq * a.k)
    return out


@functools.lru_cache(maxsize=None)
def _chunk_plan(kp, nb, tiles_out, cus=256):
    """(kc, fold) for a weight gradient summed over nb batches of kp time columns: time chunks of kc columns (kc | kp,
    kc % 8 == 0) become nb kp / kc batches, folded by ``fold`` into partial outputs summed afterwards; minimises a
    stage-count model (rounds of workgroups x stages per tile + a partial-sum pass)."""
    best = None
    for kc in range(8, kp + 1, 8):
        if kp % kc:
            continue
        nsb = nb * (kp // kc)
        for fold in range(1, nsb + 1):
            if nsb % fold:
                continue
            g = nsb // fold
            rounds = -(-(g * tiles_out) // cus)
            # us: ~3.5 per 32-column stage (3 f16 MFMA segments of a 256 x 256 tile at ~35 % of the peak), ~10 per
            # tile (ramp, epilogue), the partial outputs written and summed at ~4 TB/s
            cost = rounds * (fold * (-(-kc // 32)) * 3.5 + 10.0) + g * tiles_out * 65536 * 8 / 4e6
            if best is None or cost < best[0]:
                best = (cost, kc, fold)
    return best[1], best[2]


@functools.lru_cache(maxsize=None)
def _rows_plan(rows, units, tiles_out, cus=256):
    """(nb, fold) for a reduction over ``rows`` rows made of ``units`` equal units (utterances, frames): nb | units
    chunks of rows / nb rows each run as batches, folded by ``fold`` into partial outputs (_chunk_plan's cost model)."""
    best = None
    for nb in range(1, units + 1):
        if units % nb:
            continue
        kc = rows // nb
        for fold in range(1, nb + 1):
            if nb % fold:
                continue
            g = nb // fold
            rounds = -(-(g * tiles_out) // cus)
            cost = rounds * (fold * (-(-kc // 32)) * 3.5 + 10.0) + (g * tiles_out * 65536 * 8 / 4e6 if g > 1 else 0.0)
            if best is None or cost < best[0]:
                best = (cost, nb, fold)
    return best[1], best[2]


def _row_chunks(sp, nb):
    """Split of a (1, rows, c) row-major operand -> the (nb, c, rows / nb) views of its planes (p = column, stride 1;
    k = row within the chunk)."""
    _, r, c = sp.hi.shape
    sr = sp.hi.stride(1)
    kc = r // nb
    v = lambda t: t.as_strided((nb, c, kc), (kc * sr, 1, sr), t.storage_offset())          # noqa: E731
    return Split(v(sp.hi), v(sp.lo), sp.mb)


def gemm_f32s_rows_tn(sa, sb, units):
    """sum_r b[r, q] a[r, p] -> (cb, ca) fp32 (a weight gradient b^T a) from the Splits of two (1, rows, c) row-major
    operands (row strides multiples of 8, unit column stride) on the split-fp16 MFMA GEMM: the rows are cut into
    chunks of whole ``units`` (rows % units == 0) that run as batches, folded into partial outputs, then summed —
    the output has few 256 x 256 tiles (512 x 1536, 128 x 64), so the reduction is what the workgroups share."""
    rows, ca, cb = sa.hi.shape[1], sa.hi.shape[2], sb.hi.shape[2]
    if sb.hi.shape[1] != rows or rows % units:
        raise RuntimeError(f"gemm_f32s_rows_tn: {tuple(sa.hi.shape)} / {tuple(sb.hi.shape)} in {units} units")
    nb, fold = _rows_plan(rows, units, -(-ca // 256) * -(-cb // 256))
    out = torch.empty(nb // fold, cb, ca, device=sa.hi.device, dtype=torch.float32)
    gemm_f32s_split(_row_chunks(sa, nb), _row_chunks(sb, nb), out, fold=fold)
    return out[0] if out.shape[0] == 1 else out.sum(0)


def gemm_f32s_time_chunks(sp, sq, alpha=1.0):
    """sum_b sum_t P[b, p, t] Q[b, q, t] -> (mq, mp) fp32 for two (b, rows, K) Splits in the padded-row layout (rows of
    kp % 8 == 0 elements, zero padding: split_rows8 or a gLN planes output) with the same kp: the time axis cut into
    chunks that run as extra batches (avse_gemm_f32s nsub), folded into partial outputs, then summed — a weight gradient
    over 16 x 3999 columns has only 2 output tiles, so its reduction is what the workgroups share."""
    P, Q = sp.hi, sq.hi
    nb, mp, kn = P.shape
    mq = Q.shape[1]
    kp = P.stride(1)
    if (P.stride(2) != 1 or Q.stride(2) != 1 or Q.stride(1) != kp or kp % 8 or kp < kn or Q.shape[0] != nb
            or Q.shape[2] != kn or P.stride(0) != mp * kp or Q.stride(0) != mq * kp):
        raise RuntimeError(f"gemm_f32s_time_chunks: planes {tuple(P.shape)}/{P.stride()} and {tuple(Q.shape)}/"
                           f"{Q.stride()} are not both in the padded-row layout")
    kc, fold = _chunk_plan(kp, nb, -(-mp // 256) * -(-mq // 256))
    nsub = kp // kc
    out = torch.empty(nb * nsub // fold, mq, mp, device=P.device, dtype=torch.float32)
    a = _lib.GemmF32sArgs()
    a.batch, a.mp, a.mq, a.k, a.fold = nb * nsub, mp, mq, kc, fold
    a.p_hi, a.p_lo, a.p_bs, a.p_sx, a.p_sk, a.p_extent, a.p_max = P.data_ptr(), sp.lo.data_ptr(), mp * kp, kp, 1, \
        _plane_extent(sp), sp.mb.data_ptr()
    a.q_hi, a.q_lo, a.q_bs, a.q_sx, a.q_sk, a.q_extent, a.q_max = Q.data_ptr(), sq.lo.data_ptr(), mq * kp, kp, 1, \
        _plane_extent(sq), sq.mb.data_ptr()
    a.c, a.c_bs, a.c_sq = out.data_ptr(), out.stride(0), out.stride(1)
    a.alpha = float(alpha)
    a.nsub, a.p_bs2, a.q_bs2 = nsub, kc, kc
    tap = _tap_begin("avse_gemm_f32s", out.device)
    check(_lib.lib().avse_gemm_f32s(a, stream_ptr(out.device)), "avse_gemm_f32s")
    _tap_end(tap, 2.0 * nb * mp * mq * kn)
    return out.sum(0)

