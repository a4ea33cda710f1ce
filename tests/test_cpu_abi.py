"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports every symbol the
header declares, validates arguments on the host, and the product never routes through oracle/."""
import ast
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "avse_hip.h")
PKG = os.path.join(REPO, "avse_challenge_amd")
LIB = os.path.join(PKG, "libavse_hip.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(avse_[a-z0-9_]+)\s*\(", src)))


needs_lib = pytest.mark.skipif(not os.path.exists(LIB), reason="libavse_hip.so not built (run __graft_entry__.build)")


@needs_lib
def test_library_exports_every_declared_symbol():
    from avse_challenge_amd import _lib
    L = _lib.lib()
    decl = declared_functions()
    assert len(decl) >= 15
    for name in decl:
        assert hasattr(L, name), name
        assert name in _lib.SIGNATURES, f"{name} not bound in _lib.SIGNATURES"


@needs_lib
def test_host_side_validation_without_gpu():
    from avse_challenge_amd import _lib
    L = _lib.lib()
    assert L.avse_abi_version() == 2                 # round 6: avse_scan_fwd_args.out_z_accumulate
    assert L.avse_scan_n_chunks(3999) == 125 and L.avse_scan_n_chunks(64) == 2 and L.avse_scan_n_chunks(65) == 3
    assert L.avse_stft_frames(48000) == 376           # baseline/avse1/config.py:19
    a = _lib.ScanFwdArgs()
    assert L.avse_scan_fwd(a, None) == -1             # null pointers -> EINVAL before any launch
    dummy = ctypes.c_void_p(16)
    for f in ("u", "delta", "A", "B", "C", "out", "x"):
        setattr(a, f, dummy)
    a.batch, a.dim, a.seqlen, a.dstate = 1, 64, 10, 8
    assert L.avse_scan_fwd(a, None) == -2             # dstate != 16 -> ESHAPE
    a.dstate, a.in_dtype = 16, 7
    assert L.avse_scan_fwd(a, None) == -3             # dtype -> EDTYPE
    assert L.avse_cconv_fwd(1, 1, 10, 5, dummy, 10, 10, dummy, None, dummy, 10, 10, 0, 0, None) == -2   # width > 4
    assert L.avse_add_rmsnorm_fwd(4, 6, dummy, None, dummy, 1e-5, dummy, dummy, dummy, None, None) == -2   # n % 4
    assert b"shape" in L.avse_strerror(-2)
    ws = L.avse_scan_bwd_workspace_bytes(2, 128, 100, 16)
    assert ws == 4 * (2 * 2 * 32 * 100 + 2 * 128 * 18)
    # dilated Conv2d weight gradient: null pointers, dilation range
    assert L.avse_dconv_wgrad(2, 10, 257, 4, None, dummy, dummy, None, dummy, None) == -1
    assert L.avse_dconv_wgrad(2, 10, 257, 0, dummy, dummy, dummy, None, dummy, None) == -2
    assert L.avse_dconv_wgrad(2, 10, 257, 17, dummy, dummy, dummy, dummy, dummy, None) == -2
    assert L.avse_dconv_wgrad_workspace_bytes(32, 376, 257, 16) % (4 * (25 * 64 * 64 + 64)) == 0
    # lip Conv3d forward: compiled shape table, null pointers, unsupported shape / dtype
    # the fp32 path's prepped weights, or the f16 path's split weights (15 planes x 4 k-steps x 64 x 16 x hi/lo) + max
    # split weights (hi + lo: 2 x planes x 4 k16-steps x 64 x 16 fp16) | max |W|, max |x| (16 B) | 512 partial maxima
    assert L.avse_conv3d_fwd_workspace_bytes(3, 96, 96) == 2 * 15 * 4 * 64 * 16 * 2 + 16 + 4 * 512
    assert L.avse_conv3d_fwd_workspace_bytes(1, 112, 112) == 2 * 5 * 4 * 64 * 16 * 2 + 16 + 4 * 512
    assert L.avse_conv3d_fwd_workspace_bytes(1, 88, 88) == 0
    assert L.avse_conv3d_fwd(2, 3, 75, 96, 96, 2, None, dummy, dummy, dummy, None) == -1
    assert L.avse_conv3d_fwd(2, 1, 75, 88, 88, 2, dummy, dummy, dummy, dummy, None) == -2
    assert L.avse_conv3d_fwd(0, 3, 75, 96, 96, 2, dummy, dummy, dummy, dummy, None) == -2
    assert L.avse_conv3d_fwd(2, 3, 75, 96, 96, 1, dummy, dummy, dummy, dummy, None) == -3
    assert L.avse_conv3d_wgrad_u8(2, 3, 5, 96, 96, 5, 7, 7, 2, 3, 3, None, dummy, dummy, 0, dummy, None) == -1
    # bf16 projection GEMM: null pointers, dtype, batch % fold, neither stride unit, alignment
    g = _lib.GemmBf16Args()
    assert L.avse_gemm_bf16(g, None) == -1
    g.p = g.q = g.c = 4096
    g.batch, g.mp, g.mq, g.k, g.fold = 2, 300, 200, 512, 1
    g.p_sx, g.p_sk, g.q_sx, g.q_sk, g.c_sq = 512, 1, 512, 1, 304
    g.p_extent = g.q_extent = 1 << 20
    g.c_dtype = 2                                       # AVSE_U8
    assert L.avse_gemm_bf16(g, None) == -3
    g.c_dtype = _lib.AVSE_BF16
    g.fold = 3
    assert L.avse_gemm_bf16(g, None) == -2
    g.fold, g.q_sx, g.q_sk = 1, 3, 512
    assert L.avse_gemm_bf16(g, None) == -2
    g.q_sx, g.q_sk, g.p_sx = 512, 1, 516
    assert L.avse_gemm_bf16(g, None) == -5


def test_product_never_imports_oracle():
    for root, _, files in os.walk(PKG):
        for f in files:
            if f.endswith(".py"):
                tree = ast.parse(open(os.path.join(root, f)).read())
                for node in ast.walk(tree):
                    if isinstance(node, ast.Import):
                        names = [a.name for a in node.names]
                    elif isinstance(node, ast.ImportFrom):
                        names = [node.module or ""]
                    else:
                        continue
                    assert not any(n == "oracle" or n.startswith("oracle.") for n in names), (f, names)


def test_kernels_fail_loudly_without_gpu():
    import torch
    from avse_challenge_amd import kernels
    with pytest.raises(RuntimeError):
        kernels.selective_scan_fwd(*(torch.zeros(1, 64, 8),) * 2, torch.zeros(64, 16), torch.zeros(1, 16, 8),
                                   torch.zeros(1, 16, 8))


def test_missing_library_raises(monkeypatch, tmp_path):
    from avse_challenge_amd import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.HipLibraryError):
        _lib.lib()


def test_dropin_modules_resolve_reference_import_names():
    import importlib
    import sys
    from avse_challenge_amd import dropin
    path = dropin.install()
    try:
        for name in ("selective_scan_cuda", "causal_conv1d_cuda", "causal_conv1d", "mamba_ssm",
                     "mamba_ssm.ops.triton.layernorm", "mamba_ssm.ops.triton.selective_state_update"):
            m = importlib.import_module(name)
            assert m.__file__.startswith(path), (name, m.__file__)
        ssc = importlib.import_module("selective_scan_cuda")
        assert callable(ssc.fwd) and callable(ssc.bwd)
        cc = importlib.import_module("causal_conv1d")
        assert callable(cc.causal_conv1d_fn)
        ln = importlib.import_module("mamba_ssm.ops.triton.layernorm")
        assert ln.RMSNorm(8, eps=1e-5).weight.shape == (8,)
    finally:
        sys.path.remove(path)


def test_avse4_dropin_keys_match_oracle():
    """The product avse4 module tree loads the reference's state_dict unchanged (keys and shapes)."""
    from avse_challenge_amd import avse4
    from oracle import avse4_ref
    a = avse4.AVSE4BaselineModule(num_channels=2).state_dict()
    b = avse4_ref.AVSE4BaselineModule(num_channels=2).state_dict()
    assert list(a) == list(b)
    assert all(a[k].shape == b[k].shape for k in a)
