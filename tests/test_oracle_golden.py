"""Pin the CPU oracle (oracle/) against the golden vectors made from the reference itself."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import avse1_ref, avse4_ref, losses_ref, mamba_ref, stft_ref
from oracle.det_init import det_init_, det_input

T = torch.from_numpy


def _close(a, b, atol, rtol=0.0):
    a = a.detach().double().numpy() if torch.is_tensor(a) else np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    np.testing.assert_allclose(a, b, atol=atol, rtol=rtol)


def test_scan_fp32_forward_and_grads():
    g = load_golden("scan_fp32")
    ins = {k: T(g[k]) for k in ("u", "delta", "A", "B", "C", "D", "z", "delta_bias")}
    out = mamba_ref.selective_scan(**ins, delta_softplus=True)
    _close(out, g["out_z"], 5e-5, 1e-5)
    out, last = mamba_ref.selective_scan(**{**ins, "z": None}, delta_softplus=True, return_last_state=True)
    _close(out, g["out_noz"], 5e-5, 1e-5)
    out3 = mamba_ref.selective_scan(ins["u"], ins["delta"].abs(), ins["A"], ins["B"][:, 0], ins["C"][:, 0])
    _close(out3, g["out_3d_nodz"], 5e-5, 1e-5)
    leaves = {k: v.clone().requires_grad_(True) for k, v in ins.items()}
    mamba_ref.selective_scan(**leaves, delta_softplus=True).backward(T(g["dout"]))
    for k, v in leaves.items():
        _close(v.grad, g["d" + k], 1e-4, 1e-4)


def test_scan_bf16():
    g = load_golden("scan_bf16")
    bf = lambda k: T(g[k]).to(torch.bfloat16)
    out = mamba_ref.selective_scan(bf("u"), bf("delta"), T(g["A"]), bf("B"), bf("C"), T(g["D"]), bf("z"),
                                   T(g["delta_bias"]), True)
    ref = g["out_z"]
    rel = np.abs(out.float().numpy() - ref) / (np.abs(ref) + 1e-3)
    assert rel.max() <= 2 ** -7 + 1e-6   # at most one bf16 ulp apart


def test_bimamba_block_and_grads():
    g = load_golden("bimamba_block")
    blk = det_init_(mamba_ref.Block(32, mamba_ref.BiMambaV2(32)), 12)
    hs = T(g["hidden"]).requires_grad_(True)
    res = T(g["residual"]).requires_grad_(True)
    oh, orr = blk(hs, res)
    _close(oh, g["out_hidden"], 1e-5)
    _close(orr, g["out_residual"], 1e-6)
    (oh * T(g["gout"])).sum().backward()
    _close(hs.grad, g["g_hidden"], 1e-5)
    for k, p in blk.named_parameters():
        _close(p.grad, g["g_" + k.replace(".", "__")], 1e-4, 1e-4)


def test_mamba_unidir_pins_causal_conv():
    g = load_golden("mamba_unidir")
    m = det_init_(mamba_ref.BiMambaV2(32), 11)
    h = T(g["h"])
    with torch.no_grad():
        xz = torch.nn.functional.linear(h, m.in_proj.weight).transpose(1, 2)
        di = m.d_inner
        out = mamba_ref.mamba_inner(xz, m.conv1d.weight, m.conv1d.bias, m.x_proj.weight, m.dt_proj.weight,
                                    -torch.exp(m.A_log), m.D, m.dt_proj.bias)
        y = torch.nn.functional.linear(out.transpose(1, 2), m.out_proj.weight)
    assert di == 64
    _close(y, g["y"], 1e-5)


def test_masknet_and_encdec():
    g = load_golden("masknet_small")
    mn = det_init_(mamba_ref.MaskNet(64, 64, 2, 2, 64), 13)
    with torch.no_grad():
        _close(mn(T(g["mixture_w"])), g["est_mask"], 1e-5)
    g = load_golden("encdec")
    enc = det_init_(mamba_ref.Encoder(16, 64), 14)
    dec = det_init_(mamba_ref.Decoder(64, 1, 16, stride=8, bias=False), 15)
    with torch.no_grad():
        w = enc(T(g["mix"]))
        _close(w, g["mix_w"], 1e-6)
        _close(dec(w), g["dec"], 1e-5)


def test_si_snr():
    g = load_golden("si_snr")
    _close(losses_ref.cal_si_snr(T(g["source"]), T(g["estimate"])), g["neg_si_snr"], 1e-4)


def test_avse4_pieces():
    g = load_golden("avse4_ola")
    _close(avse4_ref.overlap_and_add(T(g["frames"]), 20), g["out"], 1e-6)
    g = load_golden("avse4_tblock")
    tb = det_init_(avse4_ref.TemporalBlock(256, 512, 3, 1, 4, 4), 41)
    x = T(g["x"]).requires_grad_(True)
    y = tb(x)
    _close(y, g["y"], 1e-5)
    (y * T(g["gy"])).sum().backward()
    _close(x.grad, g["gx"], 1e-4)
    for k, p in tb.named_parameters():
        key = "g_" + k.replace(".", "__")
        if key in g:
            _close(p.grad, g[key], 1e-3, 1e-4)
        else:
            _close(p.grad.reshape(-1)[::97], g[key + "__sub97"], 1e-3, 1e-4)


def test_avse4_separator_and_frontend():
    g = load_golden("avse4_separator_small")
    sep = det_init_(avse4_ref.Separator(N=64, L=40, B=64, H=128, P=3, X=2, R=2, C=2, num_channels=2), 42)
    for mode in ("eval", "train"):
        sep.train(mode == "train")
        with torch.no_grad():
            _close(sep(T(g["mixture"]), T(g["visual"])), g["est_" + mode], 1e-5)
    g = load_golden("avse4_visual_frontend")
    vf = det_init_(avse4_ref.VisualFrontend(), 43)
    for mode in ("eval", "train"):
        vf.train(mode == "train")
        with torch.no_grad():
            _close(vf(T(g["lips"])), g["feat_" + mode], 1e-4)


@pytest.mark.slow
def test_avse4_full():
    g = load_golden("avse4_full")
    m = det_init_(avse4_ref.AVSE4BaselineModule(num_channels=2), 44).eval()
    batch = {"noisy_audio": 0.1 * det_input((1, 2, 16000), 407),
             "vis_feat": det_input((1, 1, 25, 112, 112), 408, "uniform"),
             "clean": 0.1 * det_input((1, 2, 16000), 409)}
    assert abs(batch["vis_feat"].double().sum().item() - float(g["vis_checksum"])) < 1e-6
    with torch.no_grad():
        _close(m(batch), g["out"], 1e-5)
        _close(m.cal_loss(batch), g["loss"], 1e-4)


def test_avse1_pieces():
    g = load_golden("avse1_audiofeat")
    af = det_init_(avse1_ref.AudioFeatNet(), 51)
    for mode in ("eval", "train"):
        af.train(mode == "train")
        with torch.no_grad():
            _close(af(T(g["spec"])), g["feat_" + mode], 1e-4)
    g = load_golden("avse1_fusion")
    fu = det_init_(avse1_ref.FusionNet(), 52)
    comb = T(g["comb"]).requires_grad_(True)
    y = fu(comb)
    _close(y, g["mask"], 1e-6)
    (y * T(g["gy"])).sum().backward()
    _close(comb.grad, g["gcomb"], 1e-5)
    g = load_golden("avse1_visualfeat")
    vis = det_init_(avse1_ref.VisualFeatNet(), 53)
    lips = T(g["lips"]).float()
    for mode in ("eval", "train"):
        vis.train(mode == "train")
        for mm in vis.modules():
            if isinstance(mm, torch.nn.Dropout):
                mm.eval()
        with torch.no_grad():
            _close(vis(lips), g["feat_" + mode], 1e-4)


@pytest.mark.slow
def test_avse1_full():
    g = load_golden("avse1_full")
    net = det_init_(avse1_ref.AVNet(), 54).eval()
    batch = {"noisy_audio_spec": det_input((1, 1, 376, 257), 505).abs(),
             "lip_images": det_input((1, 3, 75, 96, 96), 506, "uint8"),
             "mask": det_input((1, 1, 376, 257), 507).abs()}
    assert batch["lip_images"].double().sum().item() == float(g["lips_checksum"])
    with torch.no_grad():
        _close(net(batch), g["pred"], 1e-5)
        _close(net.cal_loss(batch), g["loss"], 1e-6)


def test_stft_frame_count_and_roundtrip():
    # pinned: 48000 samples -> 376 frames x 257 bins (baseline/avse1/config.py:19, dataset.py:112-118)
    y = det_input((48000,), 601).numpy() * 0.1
    S = stft_ref.stft(y)
    assert S.shape == (257, 376) and S.dtype == np.complex64
    assert stft_ref.stft_mag_T(y).shape == (376, 257)
    # istft(stft(y)) reconstructs y (COLA of the periodic Hann at hop 128)
    yr = stft_ref.istft(S, length=48000)
    np.testing.assert_allclose(yr, y, atol=2e-6)
    # numpy rfft agrees with a direct DFT on one frame
    frame = np.pad(y, 256, mode="reflect")[128:128 + 512]
    k = np.arange(257)[:, None]
    dft = (stft_ref.hann_periodic() * frame * np.exp(-2j * np.pi * k * np.arange(512) / 512)).sum(1)
    np.testing.assert_allclose(S[:, 1], dft, atol=1e-4)


def test_avse2_sepblock_and_full():
    from oracle import avse2_ref
    g = load_golden("avse2_sepblock")
    sb = det_init_(avse2_ref.SeparatorBlock(64, 128, True), 81)
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    y = sb(x)
    _close(y, g["y"], 1e-6)
    (y * torch.from_numpy(g["gy"])).sum().backward()
    _close(x.grad, g["gx"], 1e-5)
    for k, p in sb.named_parameters():
        key = "g_" + k.replace(".", "__")
        if key in g:
            _close(p.grad, g[key], 1e-4)
        else:
            _close(p.grad.reshape(-1)[::97], g[key + "__sub97"], 1e-4)
    g = load_golden("avse2_full")
    m = det_init_(avse2_ref.AVSEModule(), 82).eval()
    batch = {"noisy_audio": 0.1 * det_input((2, 16000), 803), "video_frames": det_input((2, 1, 25, 64, 64), 804, "uniform"),
             "clean": 0.1 * det_input((2, 16000), 805)}
    assert abs(batch["video_frames"].double().sum().item() - float(g["vis_checksum"])) < 1e-6
    with torch.no_grad():
        _close(m(batch), g["out"], 1e-6)
        _close(m.cal_loss(batch), g["loss"], 1e-5)


def test_avse1_audio_only_c1():
    """BASELINE configs[0] (C1): audio-only AVNet (reference train.py:28-30, model.py:117-118), eval and
    train BN, and the L1 loss gradients of every parameter."""
    g = load_golden("avse1_aonly")
    net = det_init_(avse1_ref.AVNet(a_only=True), 55)
    batch = {"noisy_audio_spec": det_input((1, 1, 376, 257), 508).abs(),
             "mask": det_input((1, 1, 376, 257), 509).abs()}
    for mode in ("eval", "train"):
        net.train(mode == "train")
        pred = net(batch)
        _close(pred, g["pred_" + mode], 1e-5)
        loss = net.cal_loss(batch)
        _close(loss, g["loss_" + mode], 1e-6)
    loss.backward()
    for k, p in net.named_parameters():
        key = "g_" + k.replace(".", "__")
        ref = g[key] if key in g else g[key + "__sub97"]
        got = p.grad if key in g else p.grad.reshape(-1)[::97]
        _close(got, ref, 1e-5 * max(1.0, float(np.abs(ref).max())), 1e-4)


def test_dpmamba_wrapper_pinned():
    """oracle/dpmamba_ref.Dual_Path_Model vs the reference's in-tree dual-path forward
    (modules/dual_path.py:53-150) run over the same components, skip_around_intra True and False."""
    from oracle import dpmamba_ref
    g = load_golden("dpmamba_wrapper")
    for sia in (True, False):
        m = det_init_(dpmamba_ref.Dual_Path_Model(64, 64, dpmamba_ref.MambaBlocksSequential(1, 64),
                                                  dpmamba_ref.MambaBlocksSequential(1, 64), 2, 10, 2, sia), 91)
        with torch.no_grad():
            _close(m(T(g["mixture_w"])), g["est_mask_" + ("sia" if sia else "nosia")], 1e-5)


def test_scan_explicit_adjoint_matches_reference_autograd():
    """oracle.mamba_ref.selective_scan_grads (the O(L) explicit backward the full-length GPU tests use as truth)
    against the gradients of autograd through the reference's selective_scan_ref (golden scan_fp32)."""
    g = load_golden("scan_fp32")
    ins = {k: T(g[k]) for k in ("u", "delta", "A", "B", "C", "D", "z", "delta_bias")}
    r = mamba_ref.selective_scan_grads(**ins, delta_softplus=True, dout=T(g["dout"]))
    for k in ("u", "delta", "A", "B", "C", "D", "z", "delta_bias"):
        ref = g["d" + k]
        _close(r["d" + k], ref, 2e-5 * max(1.0, float(np.abs(ref).max())), 1e-5)
