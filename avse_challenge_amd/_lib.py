"""ctypes binding of libavse_hip.so (the C ABI declared in include/avse_hip.h).

The product path has NO fallback: if the HIP library is missing or fails to load, every op
raises.  torch is imported first so the HIP runtime torch bundles (soname libamdhip64.so.7)
is the one the library binds to — one runtime, one set of streams.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the library load: shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AVSE_HIP_LIB", os.path.join(_HERE, "libavse_hip.so"))

c_i64, c_i32, c_f32, c_vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_float, ctypes.c_void_p

AVSE_F32, AVSE_BF16 = 0, 1


class ScanFwdArgs(ctypes.Structure):
    _fields_ = [
        ("batch", c_i64), ("dim", c_i64), ("seqlen", c_i64), ("dstate", c_i64),
        ("in_dtype", c_i32), ("delta_softplus", c_i32), ("reverse", c_i32),
        ("u", c_vp), ("u_bs", c_i64), ("u_ds", c_i64),
        ("delta", c_vp), ("delta_bs", c_i64), ("delta_ds", c_i64),
        ("A", c_vp),
        ("B", c_vp), ("B_bs", c_i64), ("B_ns", c_i64),
        ("C", c_vp), ("C_bs", c_i64), ("C_ns", c_i64),
        ("D", c_vp),
        ("z", c_vp), ("z_bs", c_i64), ("z_ds", c_i64),
        ("delta_bias", c_vp),
        ("out", c_vp), ("out_bs", c_i64), ("out_ds", c_i64),
        ("x", c_vp),
        ("out_z", c_vp), ("out_z_bs", c_i64), ("out_z_ds", c_i64),
        ("out_z_accumulate", c_i32),
        ("out_z_max", c_vp),
    ]


class ScanBwdArgs(ctypes.Structure):
    _fields_ = [
        ("batch", c_i64), ("dim", c_i64), ("seqlen", c_i64), ("dstate", c_i64),
        ("in_dtype", c_i32), ("delta_softplus", c_i32), ("recompute_out_z", c_i32), ("reverse", c_i32),
        ("u", c_vp), ("u_bs", c_i64), ("u_ds", c_i64),
        ("delta", c_vp), ("delta_bs", c_i64), ("delta_ds", c_i64),
        ("A", c_vp),
        ("B", c_vp), ("B_bs", c_i64), ("B_ns", c_i64),
        ("C", c_vp), ("C_bs", c_i64), ("C_ns", c_i64),
        ("D", c_vp),
        ("z", c_vp), ("z_bs", c_i64), ("z_ds", c_i64),
        ("delta_bias", c_vp),
        ("dout", c_vp), ("dout_bs", c_i64), ("dout_ds", c_i64),
        ("x", c_vp),
        ("du", c_vp), ("du_bs", c_i64), ("du_ds", c_i64),
        ("ddelta", c_vp), ("ddelta_bs", c_i64), ("ddelta_ds", c_i64),
        ("dA", c_vp),
        ("dB", c_vp), ("dB_bs", c_i64), ("dB_ns", c_i64),
        ("dC", c_vp), ("dC_bs", c_i64), ("dC_ns", c_i64),
        ("dD", c_vp),
        ("ddelta_bias", c_vp),
        ("dz", c_vp), ("dz_bs", c_i64), ("dz_ds", c_i64),
        ("out_z", c_vp), ("out_z_bs", c_i64), ("out_z_ds", c_i64),
        ("workspace", c_vp),
        ("dz_accumulate", c_i32),
        ("dz_max", c_vp),
    ]


class GemmBf16Args(ctypes.Structure):
    _fields_ = [
        ("batch", c_i64), ("mp", c_i64), ("mq", c_i64), ("k", c_i64), ("fold", c_i64),
        ("p", c_vp), ("p_bs", c_i64), ("p_sx", c_i64), ("p_sk", c_i64), ("p_extent", c_i64),
        ("q", c_vp), ("q_bs", c_i64), ("q_sx", c_i64), ("q_sk", c_i64), ("q_extent", c_i64),
        ("c", c_vp), ("c_bs", c_i64), ("c_sq", c_i64),
        ("alpha", c_f32), ("c_dtype", c_i32),
    ]


class GemmF32sArgs(ctypes.Structure):
    _fields_ = [
        ("batch", c_i64), ("mp", c_i64), ("mq", c_i64), ("k", c_i64), ("fold", c_i64),
        ("p_hi", c_vp), ("p_lo", c_vp), ("p_bs", c_i64), ("p_sx", c_i64), ("p_sk", c_i64), ("p_extent", c_i64),
        ("p_max", c_vp),
        ("q_hi", c_vp), ("q_lo", c_vp), ("q_bs", c_i64), ("q_sx", c_i64), ("q_sk", c_i64), ("q_extent", c_i64),
        ("q_max", c_vp),
        ("c", c_vp), ("c_bs", c_i64), ("c_sq", c_i64),
        ("alpha", c_f32),
        ("nsub", c_i64), ("p_bs2", c_i64), ("q_bs2", c_i64),
    ]


# name -> (restype, argtypes); every symbol include/avse_hip.h declares
SIGNATURES = {
    "avse_strerror": (ctypes.c_char_p, [c_i32]),
    "avse_abi_version": (c_i32, []),
    "avse_scan_n_chunks": (c_i64, [c_i64]),
    "avse_scan_bwd_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64, c_i64]),
    "avse_scan_fwd": (c_i32, [ctypes.POINTER(ScanFwdArgs), c_vp]),
    "avse_scan_bwd": (c_i32, [ctypes.POINTER(ScanBwdArgs), c_vp]),
    "avse_dtproj": (c_i32, [c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i32, c_vp, c_i64,
                            c_i64, c_vp]),
    "avse_cconv_bwd_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64]),
    "avse_cconv_fwd": (c_i32, [c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64,
                               c_i32, c_i32, c_vp]),
    "avse_cconv_fwd_bf16": (c_i32, [c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64,
                                    c_i32, c_i32, c_vp]),
    "avse_cconv_bwd": (c_i32, [c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64,
                               c_vp, c_i64, c_i64, c_vp, c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp]),
    "avse_cconv_bwd_bf16": (c_i32, [c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64,
                                    c_vp, c_i64, c_i64, c_vp, c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp]),
    "avse_add_rmsnorm_fwd": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_rmsnorm_bwd_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "avse_rmsnorm_bwd": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_add_rmsnorm_fwd2": (c_i32, [c_i64, c_i64, c_vp, c_i32, c_vp, c_vp, c_f32, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "avse_rmsnorm_bwd2": (c_i32, [c_i64, c_i64, c_vp, c_i32] + [c_vp] * 9),
    "avse_stft_frames": (c_i64, [c_i64]),
    "avse_stft_fwd": (c_i32, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "avse_istft": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_conv3d_wgrad_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64, c_i64]),
    "avse_conv3d_wgrad": (c_i32, [c_i64] * 11 + [c_vp, c_vp, c_vp, c_i32, c_vp, c_vp]),
    "avse_conv3d_wgrad_u8": (c_i32, [c_i64] * 11 + [c_vp, c_vp, c_vp, c_i32, c_vp, c_vp]),
    "avse_conv3d_wgrad_u8_split": (c_i32, [c_i64] * 11 + [c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp]),
    "avse_conv3d_wgrad_split": (c_i32, [c_i64] * 11 + [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp]),
    "avse_conv3d_fwd_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64]),
    "avse_conv3d_fwd": (c_i32, [c_i64] * 5 + [c_i32] + [c_vp] * 5),
    "avse_dconv_wgrad_workspace_bytes": (c_i64, [c_i64] * 4),
    "avse_dconv_wgrad": (c_i32, [c_i64] * 4 + [c_vp] * 6),
    "avse_prelu_fwd": (c_i32, [c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "avse_prelu_bwd_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "avse_prelu_bwd": (c_i32, [c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_maxpool2d_out_size": (c_i64, [c_i64] * 4),
    "avse_maxpool2d_fwd": (c_i32, [c_i64] * 9 + [c_vp, c_vp, c_vp, c_vp]),
    "avse_maxpool2d_bwd": (c_i32, [c_i64] * 9 + [c_vp, c_vp, c_vp, c_vp]),
    "avse_transpose_cp": (c_i32, [c_i64] * 3 + [c_vp, c_vp, c_vp]),
    "avse_bnact_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64]),
    "avse_bnact_fwd": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32, c_i32, c_f32, c_f32,
                               c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_bnact_bwd": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32, c_i32,
                               c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_bnact_fwd_q": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32, c_f32, c_f32, c_vp, c_vp,
                                 c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_bnact_bwd_q": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32, c_i32, c_vp,
                                 c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_prelu_nhwc_fwd": (c_i32, [c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "avse_prelu_nhwc_bwd_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "avse_prelu_nhwc_bwd": (c_i32, [c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_prelu_gln_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "avse_prelu_gln_fwd": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp]),
    "avse_prelu_gln_bwd": (c_i32, [c_i64, c_i64, c_i64] + [c_vp] * 11),
    "avse_prelu_gln_bwd_q": (c_i32, [c_i64, c_i64, c_i64] + [c_vp] * 7 + [c_i64] + [c_vp] * 6),
    "avse_dwconv_bwd_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "avse_dwconv_fwd": (c_i32, [c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "avse_dwconv_bwd": (c_i32, [c_i64, c_i64, c_i64, c_i64, c_i64] + [c_vp] * 7),
    "avse_dwconv_gln_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "avse_dwconv_gln_fwd": (c_i32, [c_i64] * 5 + [c_vp] * 5 + [c_f32] + [c_vp] * 5),
    "avse_dwconv_gln_fwd_q": (c_i32, [c_i64] * 5 + [c_vp] * 5 + [c_f32] + [c_vp] * 3 + [c_i64] + [c_vp] * 4),
    "avse_dwconv_gln_bwd": (c_i32, [c_i64] * 5 + [c_vp] * 14),
    "avse_lstm_padded_hidden": (c_i64, [c_i64]),
    "avse_lstm_group_size": (c_i64, [c_i64, c_i64]),
    "avse_lstm_group_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "avse_lstm_group_capacity": (c_i64, [c_i64, c_i32]),
    "avse_lstm_fwd_group": (c_i32, [c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp,
                                    c_vp]),
    "avse_lstm_bwd_group": (c_i32, [c_i64, c_i64, c_i64, c_i32, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                    c_vp]),
    "avse_lstm_fwd": (c_i32, [c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "avse_lstm_bwd": (c_i32, [c_i64, c_i64, c_i64, c_i32, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_gemm_bf16": (c_i32, [ctypes.POINTER(GemmBf16Args), c_vp]),
    "avse_gemm_f32s": (c_i32, [ctypes.POINTER(GemmF32sArgs), c_vp]),
    "avse_split16_planes": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "avse_add_max": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_split16_planes_known": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "avse_split16_planes_to": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_i32,
                                       c_vp]),
    "avse_dconv_wprep_bytes": (c_i64, []),
    "avse_split16": (c_i32, [c_i64, c_vp, c_vp, c_vp, c_vp]),
    "avse_split16_known": (c_i32, [c_i64, c_vp, c_vp, c_vp, c_vp]),
    "avse_dconv_wprep": (c_i32, [c_vp, c_i32, c_vp, c_vp, c_vp]),
    "avse_dconv_fwd": (c_i32, [c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_dconv_wgrad16_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64]),
    "avse_dconv_wgrad16": (c_i32, [c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "avse_conv1_fwd": (c_i32, [c_i64] * 3 + [c_vp] * 5),
    "avse_conv1_dgrad": (c_i32, [c_i64] * 3 + [c_vp] * 4),
    "avse_conv1_wgrad_workspace_bytes": (c_i64, [c_i64] * 3),
    "avse_conv1_wgrad": (c_i32, [c_i64] * 3 + [c_vp] * 6),
    "avse_convf_fwd": (c_i32, [c_i64] + [c_vp] * 5),
    "avse_convf_dgrad": (c_i32, [c_i64] + [c_vp] * 4),
    "avse_convf_wgrad_workspace_bytes": (c_i64, [c_i64]),
    "avse_convf_wgrad": (c_i32, [c_i64] + [c_vp] * 6),
    "avse_sconv_wprep_bytes": (c_i64, [c_i64, c_i64]),
    "avse_sconv_wprep": (c_i32, [c_i64, c_i64, c_vp, c_i32, c_vp, c_vp, c_vp]),
    "avse_sconv_fwd": (c_i32, [c_i64] * 6 + [c_vp] * 6),
    "avse_sconv_wgrad_workspace_bytes": (c_i64, [c_i64] * 6),
    "avse_sconv_wgrad": (c_i32, [c_i64] * 6 + [c_vp] * 7),
    "avse_sconv_dgrad2_supported": (c_i32, [c_i64] * 5),
    "avse_sconv_dgrad2": (c_i32, [c_i64] * 5 + [c_vp] * 6),
}

_lib = None


class HipLibraryError(RuntimeError):
    pass


ABI_VERSION = 2          # include/avse_hip.h avse_abi_version (2, round 6: the scan out_z / dz and cconv dx accumulate)


def lib():
    """The loaded library; raises HipLibraryError (never falls back) when it is unavailable."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HipLibraryError(
                f"libavse_hip.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (make -C avse_challenge_amd/csrc)")
        try:
            L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise HipLibraryError(f"failed to load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.avse_abi_version() != ABI_VERSION:        # the argument structs above are this version's layout
            raise HipLibraryError(f"{LIB_PATH} has C-ABI version {L.avse_abi_version()}, the bindings expect "
                                  f"{ABI_VERSION}: rebuild it (make -C avse_challenge_amd/csrc)")
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {lib().avse_strerror(rc).decode()} (code {rc})")


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())
