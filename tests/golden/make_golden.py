"""Generate the golden vectors under tests/golden/ by importing the REFERENCE (build container only).

Run:  python tests/golden/make_golden.py        (needs /root/reference; never runs on the GPU box)

What it does, per case:
  1. imports the reference module from /root/reference (third-party packages that are not
     installed are replaced by the stubs in _install_stubs(); every stub is either a no-op
     framework base class or a restatement that is itself recorded as "parity unpinned"),
  2. builds the oracle restatement (oracle/*.py) with the same constructor arguments,
  3. fills BOTH from oracle.det_init (values derived from state_dict key + shape only, so equal
     keys => equal weights; strict loading proves key compatibility),
  4. runs both on identical seeded inputs, asserts agreement, and writes the REFERENCE outputs
     (and small inputs) to tests/golden/<case>.npz plus tests/golden/manifest.json.
No reference source is copied: only numeric inputs/outputs are written.
"""
import json
import os
import sys
import types
from functools import partial

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from oracle import avse1_ref, avse2_ref, avse4_ref, losses_ref, mamba_ref  # noqa: E402
from oracle.det_init import det_init_, det_input  # noqa: E402

torch.set_num_threads(8)
MANIFEST = {}


def _mod(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _LM(nn.Module):
    """pytorch_lightning.LightningModule stand-in: a plain nn.Module (framework glue only)."""

    def log(self, *a, **k):
        pass

    def save_hyperparameters(self, *a, **k):
        pass


def _install_stubs():
    _mod("pytorch_lightning", LightningModule=_LM, LightningDataModule=object, Trainer=object)
    _mod("librosa")
    # causal-conv1d 1.1.3.post1 (un-vendored): restated definition
    _mod("causal_conv1d",
         causal_conv1d_fn=lambda x, weight, bias=None, activation=None, **k:
         mamba_ref.causal_conv1d(x, weight, bias, silu=activation in ("silu", "swish")),
         causal_conv1d_update=None)
    _mod("causal_conv1d_cuda",
         causal_conv1d_fwd=lambda x, w, b, seq_idx, silu: mamba_ref.causal_conv1d(x, w, b, silu))
    # selective_scan_cuda.fwd bound to the REFERENCE's own selective_scan_ref (imported lazily)
    _mod("selective_scan_cuda")
    class RMSNormStub(mamba_ref.RMSNorm):   # mamba-ssm Triton RMSNorm(hidden, eps, device, dtype)
        def __init__(self, hidden_size, eps=1e-5, device=None, dtype=None):
            super().__init__(hidden_size, eps)

    tri = _mod("mamba_ssm.ops.triton.layernorm", RMSNorm=RMSNormStub, layer_norm_fn=None, rms_norm_fn=None)
    ssu = _mod("mamba_ssm.ops.triton.selective_state_update", selective_state_update=None)
    _mod("mamba_ssm.ops.triton", layernorm=tri, selective_state_update=ssu)
    _mod("mamba_ssm.ops")
    _mod("mamba_ssm", Mamba=nn.Module)
    # speechbrain 1.0.0 (un-vendored): cLN + channels-last Conv1d restated; cal_si_snr = in-tree copy
    sys.path.insert(0, os.path.join(REF, "baseline/avse2"))
    import utils.dnn as avse2_dnn  # baseline/avse2/utils/dnn.py (in-tree speechbrain copy)
    del sys.modules["utils"], sys.modules["utils.dnn"]
    sys.path.pop(0)

    class SBConv1d(mamba_ref.ChannelsLastConv1x1):
        def __init__(self, in_channels, out_channels, kernel_size=1, bias=False):
            assert kernel_size == 1 and not bias
            super().__init__(in_channels, out_channels)

    cnn = _mod("speechbrain.nnet.CNN", Conv1d=SBConv1d)
    losses = _mod("speechbrain.nnet.losses", cal_si_snr=avse2_dnn.cal_si_snr)
    nnet = _mod("speechbrain.nnet", CNN=cnn, losses=losses)
    ct = _mod("speechbrain.lobes.models.conv_tasnet", ChannelwiseLayerNorm=mamba_ref.ChannelwiseLayerNorm)
    _mod("speechbrain.lobes.models", conv_tasnet=ct)
    _mod("speechbrain.lobes")
    _mod("speechbrain", nnet=nnet)
    return avse2_dnn


SUB = 97  # arrays above BIG elements are stored as flat[::SUB] under "<key>__sub97"
BIG = 60000


def _save(name, arrays, note, diffs):
    path = os.path.join(HERE, name + ".npz")
    out = {}
    for k, v in arrays.items():
        a = v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)
        if a.size > BIG and k.startswith("g_"):
            out[k + "__sub97"] = a.reshape(-1)[::SUB].copy()
        else:
            out[k] = a
    np.savez_compressed(path, **out)
    MANIFEST[name] = {"note": note, "oracle_vs_reference_maxabs": diffs,
                      "bytes": os.path.getsize(path)}
    print(f"{name}: {diffs}")


def _maxabs(a, b):
    return float((a.detach().double() - b.detach().double()).abs().max())


def _same_keys(ref_mod, our_mod):
    rk, ok = list(ref_mod.state_dict().keys()), list(our_mod.state_dict().keys())
    assert rk == ok, (set(rk) ^ set(ok))


def _import_from(subdir, modname):
    path = os.path.join(REF, subdir)
    sys.path.insert(0, path)
    try:
        for k in list(sys.modules):
            if k in ("model", "utils", "config") or k.startswith("utils.") or k.startswith("modules"):
                del sys.modules[k]
        mod = __import__(modname, fromlist=["*"])
    finally:
        sys.path.pop(0)
    return mod


# ============================================================================ Mamba-TasNet

def gen_mamba():
    ssi = _import_from("Mamba-TasNet", "modules.mamba.selective_scan_interface")
    ref_scan = ssi.selective_scan_ref

    def ss_fwd(u, delta, A, B, C, D, z, delta_bias, delta_softplus):
        out, last = ref_scan(u, delta, A, B, C, D, None, delta_bias, delta_softplus, return_last_state=True)
        x = torch.stack([torch.zeros_like(last), last], -1).reshape(last.shape[0], last.shape[1], 1, -1)
        res = [out, x]
        if z is not None:
            res.append(out * F.silu(z.float()).to(out.dtype))
        return res
    sys.modules["selective_scan_cuda"].fwd = ss_fwd

    # ---- a1: selective scan forward, several argument combinations
    b, d, l, n = 2, 64, 300, 16
    cases = {}
    g = 100
    u = det_input((b, d, l), g + 1)
    delta = 0.5 * det_input((b, d, l), g + 2)
    A = -torch.exp(0.5 * det_input((d, n), g + 3))
    Bv = det_input((b, 1, n, l), g + 4)
    Cv = det_input((b, 1, n, l), g + 5)
    D = det_input((d,), g + 6)
    z = det_input((b, d, l), g + 7)
    dbias = 0.3 * det_input((d,), g + 8)
    ins = dict(u=u, delta=delta, A=A, B=Bv, C=Cv, D=D, z=z, delta_bias=dbias)
    out_full, last = ref_scan(u, delta, A, Bv, Cv, D, z, dbias, True, return_last_state=True)
    out_noz = ref_scan(u, delta, A, Bv, Cv, D, None, dbias, True)
    out_3d = ref_scan(u, delta.abs(), A, Bv[:, 0], Cv[:, 0], None, None, None, False)
    ours = mamba_ref.selective_scan(u, delta, A, Bv, Cv, D, z, dbias, True)
    ours3 = mamba_ref.selective_scan(u, delta.abs(), A, Bv[:, 0], Cv[:, 0], None, None, None, False)
    # gradients through the reference's pure-torch scan (autograd)
    leaves = {k: v.clone().requires_grad_(True) for k, v in ins.items()}
    dout = det_input((b, d, l), g + 9)
    o = ref_scan(leaves["u"], leaves["delta"], leaves["A"], leaves["B"], leaves["C"], leaves["D"],
                 leaves["z"], leaves["delta_bias"], True)
    o.backward(dout)
    grads = {"d" + k: v.grad for k, v in leaves.items()}
    leaves2 = {k: v.clone().requires_grad_(True) for k, v in ins.items()}
    o2 = mamba_ref.selective_scan(leaves2["u"], leaves2["delta"], leaves2["A"], leaves2["B"], leaves2["C"],
                                  leaves2["D"], leaves2["z"], leaves2["delta_bias"], True)
    o2.backward(dout)
    gd = max(_maxabs(leaves2[k].grad, grads["d" + k]) for k in ins)
    _save("scan_fp32", dict(**ins, out_z=out_full, last_state=last, out_noz=out_noz, out_3d_nodz=out_3d,
                            dout=dout, **grads),
          "selective_scan_ref (selective_scan_interface.py:91-157), fp32, b2 d64 l300 n16; grads via autograd",
          {"out_z": _maxabs(ours, out_full), "out_3d": _maxabs(ours3, out_3d), "grads": gd})

    # bf16 inputs (u, delta, z, B, C bf16; A, D, bias fp32), as under torch.autocast bf16
    ub, db_, zb, Bb, Cb = (t.to(torch.bfloat16) for t in (u, delta, z, Bv, Cv))
    out_bf = ref_scan(ub, db_, A, Bb, Cb, D, zb, dbias, True)
    ours_bf = mamba_ref.selective_scan(ub, db_, A, Bb, Cb, D, zb, dbias, True)
    _save("scan_bf16", dict(u=ub.float(), delta=db_.float(), z=zb.float(), B=Bb.float(), C=Cb.float(),
                            A=A, D=D, delta_bias=dbias, out_z=out_bf.float()),
          "selective_scan_ref with bf16 u/delta/z/B/C (values stored as fp32, exactly bf16-representable)",
          {"out_z_max_rel": float(((ours_bf.double() - out_bf.double()).abs() /
                                   (out_bf.double().abs() + 1e-3)).max())})

    # ---- a3/a4: single-direction Mamba through the reference fallback (pins causal conv semantics)
    bim = _import_from("Mamba-TasNet", "modules.mamba.bimamba")
    bim.selective_scan_fn = ref_scan          # bimamba imported the CUDA autograd fn; use the ref
    bim.causal_conv1d_fn = None               # forces act(conv1d(x)[..., :L]) (bimamba.py:278-279)
    dm, L = 32, 64
    ref_m = bim.Mamba(dm, bimamba_type="v2", use_fast_path=False)
    det_init_(ref_m, 11)
    h = det_input((2, L, dm), 201)
    with torch.no_grad():
        y_uni = ref_m(h)
    ours_m = mamba_ref.BiMambaV2(dm)
    _same_keys(ref_m, ours_m)
    det_init_(ours_m, 11)
    with torch.no_grad():
        x = F.linear(h, ours_m.in_proj.weight).transpose(1, 2)
        xi, zi = x.chunk(2, 1)
        xc = mamba_ref.causal_conv1d(xi, ours_m.conv1d.weight[:, 0], ours_m.conv1d.bias, silu=True)
        xd = xc.transpose(1, 2).reshape(-1, xc.shape[1]) @ ours_m.x_proj.weight.t()
        r = ours_m.dt_rank
        dt = (ours_m.dt_proj.weight @ xd[:, :r].t()).reshape(-1, 2, L).transpose(0, 1)
        Bm = xd[:, r:r + 16].reshape(2, L, 16).transpose(1, 2)
        Cm = xd[:, r + 16:].reshape(2, L, 16).transpose(1, 2)
        yy = mamba_ref.selective_scan(xc, dt, -torch.exp(ours_m.A_log), Bm, Cm, ours_m.D, zi,
                                      ours_m.dt_proj.bias, True)
        y_ours = F.linear(yy.transpose(1, 2), ours_m.out_proj.weight)
    _save("mamba_unidir", dict(h=h, y=y_uni),
          "bimamba.Mamba(d_model=32, v2 params) with use_fast_path=False and causal_conv1d_fn=None: "
          "reference in-tree conv fallback (bimamba.py:271-304); det_init seed 11",
          {"y": _maxabs(y_ours, y_uni)})

    # ---- a4/a5: bidirectional v2 Block forward (fast path with shimmed natives) + grads
    def inner_no_out_proj_ref(xz, cw, cb, xw, dw, A, B=None, C=None, D=None, delta_bias=None,
                              delta_softplus=True, **k):
        # reference composition mamba_inner_ref (selective_scan_interface.py:651-684) with an
        # identity out_proj, differentiable through the reference's selective_scan_ref
        di = xz.shape[1] // 2
        eye = torch.eye(di, dtype=xz.dtype)
        return ssi.mamba_inner_ref(xz, cw, cb, xw, dw, eye, None, A, B, C, D, delta_bias,
                                   delta_softplus=delta_softplus).transpose(1, 2)
    ssi.selective_scan_fn = ref_scan
    bim.mamba_inner_fn_no_out_proj = inner_no_out_proj_ref
    blk = bim.Block(dm, partial(bim.Mamba, bimamba_type="v2"), norm_cls=partial(mamba_ref.RMSNorm, eps=1e-5),
                    fused_add_norm=False)
    det_init_(blk, 12)
    ours_blk = mamba_ref.Block(dm, mamba_ref.BiMambaV2(dm))
    _same_keys(blk, ours_blk)
    det_init_(ours_blk, 12)
    hs = det_input((2, L, dm), 202).requires_grad_(True)
    res = det_input((2, L, dm), 203).requires_grad_(True)
    gout = det_input((2, L, dm), 204)
    o_h, o_r = blk(hs, res)
    (o_h * gout).sum().backward()
    ref_grads = {"g_" + k.replace(".", "__"): p.grad.clone() for k, p in blk.named_parameters()}
    g_hs, g_res = hs.grad.clone(), res.grad.clone()
    hs2 = hs.detach().clone().requires_grad_(True)
    res2 = res.detach().clone().requires_grad_(True)
    p_h, p_r = ours_blk(hs2, res2)
    (p_h * gout).sum().backward()
    gmax = max(_maxabs(p.grad, ref_grads["g_" + k.replace(".", "__")]) for k, p in ours_blk.named_parameters())
    _save("bimamba_block", dict(hidden=hs.detach(), residual=res.detach(), gout=gout, out_hidden=o_h.detach(),
                                out_residual=o_r.detach(), g_hidden=g_hs, g_residual=g_res, **ref_grads),
          "bimamba.Block(d_model=32, Mamba v2, RMSNorm eps 1e-5, fused_add_norm=False), L=64, det_init seed 12",
          {"out": _maxabs(p_h, o_h), "param_grads": gmax, "g_hidden": _maxabs(hs2.grad, g_hs)})

    # ---- a6/a7: MaskNet (2 layers, enc=bot=d_model=64) forward via the real MambaInnerFnNoOutProj.forward
    bim.mamba_inner_fn_no_out_proj = ssi.mamba_inner_fn_no_out_proj
    mn_mod = _import_from("Mamba-TasNet", "modules.mamba_masknet")
    ref_mn = mn_mod.MaskNet(enc_dim=64, bot_dim=64, n_spk=2, n_mamba=2, bidirectional=True, d_model=64,
                            fused_add_norm=False, rms_norm=True)
    ours_mn = mamba_ref.MaskNet(64, 64, 2, 2, 64)
    _same_keys(ref_mn, ours_mn)
    det_init_(ref_mn, 13)
    det_init_(ours_mn, 13)
    mw = det_input((2, 64, 50), 205).abs()
    with torch.no_grad():
        m_ref = ref_mn(mw)
        m_ours = ours_mn(mw)
    _save("masknet_small", dict(mixture_w=mw, est_mask=m_ref),
          "mamba_masknet.MaskNet(enc=bot=d_model=64, n_mamba=2, n_spk=2), fast path (MambaInnerFnNoOutProj.forward "
          "with selective_scan_cuda.fwd -> selective_scan_ref), det_init seed 13",
          {"est_mask": _maxabs(m_ours, m_ref)})

    # ---- a8: Encoder / Decoder = speechbrain dual_path copies in baseline/avse2/model.py:14-37
    av2 = _import_from("baseline/avse2", "model")
    enc_r = av2.AudioEncoder(kernel_size=16, out_channels=64)
    dec_r = av2.AudioDecoder(in_channels=64, out_channels=1, kernel_size=16, stride=8, bias=False)
    enc_o, dec_o = mamba_ref.Encoder(16, 64), mamba_ref.Decoder(64, 1, 16, stride=8, bias=False)
    _same_keys(enc_r, enc_o)
    _same_keys(dec_r, dec_o)
    for mdl in (enc_r, enc_o):
        det_init_(mdl, 14)
    for mdl in (dec_r, dec_o):
        det_init_(mdl, 15)
    mix = det_input((2, 800), 206)
    with torch.no_grad():
        w_r = enc_r(mix)
        y_r = dec_r(w_r)
        w_o = enc_o(mix)
        y_o = dec_o(w_o)
    _save("encdec", dict(mix=mix, mix_w=w_r, dec=y_r),
          "SpeechBrain dual_path Encoder(k16,s8)/Decoder(ConvTranspose1d k16 s8) via in-tree copies "
          "baseline/avse2/model.py:14-37, det_init seeds 14/15",
          {"enc": _maxabs(w_o, w_r), "dec": _maxabs(y_o, y_r)})


# ============================================================================ losses

def gen_losses(avse2_dnn):
    src = det_input((1000, 3, 2), 301)
    est = src + 0.3 * det_input((1000, 3, 2), 302)
    ref = avse2_dnn.cal_si_snr(src.clone(), est.clone())
    ours = losses_ref.cal_si_snr(src, est)
    _save("si_snr", dict(source=src, estimate=est, neg_si_snr=ref),
          "cal_si_snr baseline/avse2/utils/dnn.py:15-57 (speechbrain copy), [T,B,C]",
          {"neg_si_snr": _maxabs(ours, ref)})


# ============================================================================ avse4

def gen_avse4():
    m4 = _import_from("baseline/avse4", "model")
    sig = det_input((2, 3, 50, 40), 401)
    ola_r = m4.overlap_and_add(sig, 20)
    ola_o = avse4_ref.overlap_and_add(sig, 20)
    _save("avse4_ola", dict(frames=sig, out=ola_r), "overlap_and_add model.py:19-66, step 20",
          {"out": _maxabs(ola_o, ola_r)})

    # full-size TemporalBlock (256 -> 512, k3, dil 4) fwd + grads
    tb_r = m4.TemporalBlock(256, 512, 3, stride=1, padding=4, dilation=4)
    tb_o = avse4_ref.TemporalBlock(256, 512, 3, 1, 4, 4)
    _same_keys(tb_r, tb_o)
    det_init_(tb_r, 41)
    det_init_(tb_o, 41)
    x = det_input((2, 256, 300), 402).requires_grad_(True)
    gy = det_input((2, 256, 300), 403)
    y_r = tb_r(x)
    (y_r * gy).sum().backward()
    grads = {"g_" + k.replace(".", "__"): p.grad.clone() for k, p in tb_r.named_parameters()}
    gx = x.grad.clone()
    x2 = x.detach().clone().requires_grad_(True)
    y_o = tb_o(x2)
    (y_o * gy).sum().backward()
    gmax = max(_maxabs(p.grad, grads["g_" + k.replace(".", "__")]) for k, p in tb_o.named_parameters())
    _save("avse4_tblock", dict(x=x.detach(), gy=gy, y=y_r.detach(), gx=gx, **grads),
          "TemporalBlock(256,512,k3,dil4) model.py:255-293 (conv1x1,PReLU,gLN,dwconv,PReLU,gLN,conv1x1,+res), "
          "det_init seed 41",
          {"y": _maxabs(y_o, y_r), "gx": _maxabs(x2.grad, gx), "param_grads": gmax})

    # reduced separator (N=B=64, H=128, X=2, R=2), binaural 1 s
    sep_r = m4.avse4_separator(N=64, L=40, B=64, H=128, P=3, X=2, R=2, C=2, num_channels=2)
    sep_o = avse4_ref.Separator(N=64, L=40, B=64, H=128, P=3, X=2, R=2, C=2, num_channels=2)
    _same_keys(sep_r, sep_o)
    det_init_(sep_r, 42)
    det_init_(sep_o, 42)
    mixture = 0.1 * det_input((2, 2, 16000), 404)
    visual = det_input((2, 25, 512), 405)
    out = {}
    diffs = {}
    for mode in ("eval", "train"):
        sep_r.train(mode == "train")
        sep_o.train(mode == "train")
        with torch.no_grad():
            a = sep_r(mixture, visual)
            bb = sep_o(mixture, visual)
        out["est_" + mode] = a
        diffs[mode] = _maxabs(bb, a)
    _save("avse4_separator_small", dict(mixture=mixture, visual=visual, **out),
          "avse4_separator(N=64,L=40,B=64,H=128,P=3,X=2,R=2,C=2,ch=2) model.py:73-94, eval and train BN, seed 42",
          diffs)

    # VisualFrontend (ResNet-18 lip encoder) on 5 frames
    ut = _import_from("baseline/avse4", "utils")
    vf_r, vf_o = ut.VisualFrontend(), avse4_ref.VisualFrontend()
    _same_keys(vf_r, vf_o)
    det_init_(vf_r, 43)
    det_init_(vf_o, 43)
    lips = det_input((2, 1, 5, 112, 112), 406, "uniform")
    out, diffs = {}, {}
    for mode in ("eval", "train"):
        vf_r.train(mode == "train")
        vf_o.train(mode == "train")
        with torch.no_grad():
            a = vf_r(lips)
            bb = vf_o(lips)
        out["feat_" + mode] = a
        diffs[mode] = _maxabs(bb, a)
    _save("avse4_visual_frontend", dict(lips=lips, **out),
          "VisualFrontend utils.py:97-118 on (2,1,5,112,112), eval/train BN, det_init seed 43", diffs)

    # full AVSE4BaselineModule forward + cal_loss at 1 s binaural, 25 lip frames (weights from det_init)
    full_r = m4.AVSE4BaselineModule(num_channels=2)
    full_o = avse4_ref.AVSE4BaselineModule(num_channels=2)
    _same_keys(full_r, full_o)
    det_init_(full_r, 44)
    det_init_(full_o, 44)
    full_r.eval()
    full_o.eval()
    batch = {"noisy_audio": 0.1 * det_input((1, 2, 16000), 407), "vis_feat": det_input((1, 1, 25, 112, 112), 408, "uniform"),
             "clean": 0.1 * det_input((1, 2, 16000), 409)}
    with torch.no_grad():
        a = full_r(batch)
        la = full_r.cal_loss(batch)
        bb = full_o(batch)
        lb = full_o.cal_loss(batch)
    _save("avse4_full", dict(out=a, loss=la, vis_checksum=batch["vis_feat"].double().sum()),
          "AVSE4BaselineModule(num_channels=2) eval forward + cal_loss; inputs det_input seeds 407-409 "
          "(noisy/clean scaled 0.1, vis uniform) regenerated in tests; det_init seed 44",
          {"out": _maxabs(bb, a), "loss": abs(float(la) - float(lb))})


# ============================================================================ avse1

def gen_avse1():
    os.environ.setdefault("MPLBACKEND", "Agg")
    m1 = _import_from("baseline/avse1", "model")
    af_r, af_o = m1.build_audiofeat_net(), avse1_ref.AudioFeatNet()
    _same_keys(af_r, af_o)
    det_init_(af_r, 51)
    det_init_(af_o, 51)
    spec = det_input((2, 1, 40, 257), 501).abs()
    out, diffs = {}, {}
    for mode in ("eval", "train"):
        af_r.train(mode == "train")
        af_o.train(mode == "train")
        with torch.no_grad():
            a = af_r(spec)
            bb = af_o(spec)
        out["feat_" + mode] = a
        diffs[mode] = _maxabs(bb, a)
    _save("avse1_audiofeat", dict(spec=spec, **out),
          "AudioFeatNet model.py:181-267 on (2,1,40,257), eval/train BN, det_init seed 51", diffs)

    fu_r, fu_o = m1.FusionNet(a_only=False), avse1_ref.FusionNet()
    _same_keys(fu_r, fu_o)
    det_init_(fu_r, 52)
    det_init_(fu_o, 52)
    comb = det_input((2, 20, 1540), 502).requires_grad_(True)
    gy = det_input((2, 20, 257), 503)
    yr = fu_r(comb)
    (yr * gy).sum().backward()
    grads = {"g_" + k.replace(".", "__"): p.grad.clone() for k, p in fu_r.named_parameters()}
    gcomb = comb.grad.clone()
    comb2 = comb.detach().clone().requires_grad_(True)
    yo = fu_o(comb2)
    (yo * gy).sum().backward()
    gmax = max(_maxabs(p.grad, grads["g_" + k.replace(".", "__")]) for k, p in fu_o.named_parameters())
    _save("avse1_fusion", dict(comb=comb.detach(), gy=gy, mask=yr.detach(), gcomb=gcomb, **grads),
          "FusionNet model.py:81-96 (LSTM 1540->257 + Linear + sigmoid), T=20, grads, det_init seed 52",
          {"mask": _maxabs(yo, yr), "gcomb": _maxabs(comb2.grad, gcomb), "param_grads": gmax})

    vis_r = m1.build_visualfeat_net(extract_feats=True)
    vis_o = avse1_ref.VisualFeatNet()
    _same_keys(vis_r, vis_o)
    det_init_(vis_r, 53)
    det_init_(vis_o, 53)
    lips = det_input((2, 3, 8, 64, 64), 504, "uint8").float()
    out, diffs = {}, {}
    for mode in ("eval", "train"):
        vis_r.train(mode == "train")
        vis_o.train(mode == "train")
        if mode == "train":   # dropout off so the comparison is deterministic (BN still in batch mode)
            for mm in list(vis_r.modules()) + list(vis_o.modules()):
                if isinstance(mm, nn.Dropout):
                    mm.eval()
        with torch.no_grad():
            a = vis_r(lips, 8)
            bb = vis_o(lips)
        out["feat_" + mode] = a
        diffs[mode] = _maxabs(bb, a)
    _save("avse1_visualfeat", dict(lips=lips.to(torch.uint8), **out),
          "VisualFeatNet model.py:17-58 (Conv3d+BN+PReLU+MaxPool, ResNet-18 PReLU, TCN 4x512) on raw uint8 "
          "lips (2,3,8,64,64); train mode has Dropout disabled; det_init seed 53", diffs)

    # full AVNet, B=1, 3 s (376 STFT frames) + 75 lip frames 96x96 (the BASELINE C2 utterance shape)
    net_r = m1.AVNet((m1.build_visualfeat_net(extract_feats=True), m1.build_audiofeat_net(), m1.FusionNet()), "l1")
    net_o = avse1_ref.AVNet()
    _same_keys(net_r, net_o)
    det_init_(net_r, 54)
    det_init_(net_o, 54)
    net_r.eval()
    net_o.eval()
    batch = {"noisy_audio_spec": det_input((1, 1, 376, 257), 505).abs(),
             "lip_images": det_input((1, 3, 75, 96, 96), 506, "uint8"),
             "mask": det_input((1, 1, 376, 257), 507).abs()}
    with torch.no_grad():
        a = net_r(batch)
        la = net_r.cal_loss(batch)
        bb = net_o(batch)
        lb = net_o.cal_loss(batch)
    _save("avse1_full", dict(pred=a, loss=la, lips_checksum=batch["lip_images"].double().sum()),
          "AVNet eval forward + cal_loss(l1) on (1,1,376,257) spec + (1,3,75,96,96) uint8 lips; inputs det_input "
          "seeds 505-507 regenerated in tests; det_init seed 54",
          {"pred": _maxabs(bb, a), "loss": abs(float(la) - float(lb))})


def gen_avse1_aonly():
    """BASELINE configs[0] (C1): audio-only AVNet, as train.py:28-30 builds it — nets = (None, AudioFeatNet,
    FusionNet(a_only=True)), model.py:117-118 — on one 3 s utterance (376 STFT frames), eval and train BN,
    plus the train-mode L1 loss gradients of every parameter."""
    m1 = _import_from("baseline/avse1", "model")
    net_r = m1.AVNet((None, m1.build_audiofeat_net(a_only=True), m1.FusionNet(a_only=True)), "l1", a_only=True)
    net_o = avse1_ref.AVNet(a_only=True)
    _same_keys(net_r, net_o)
    det_init_(net_r, 55)
    det_init_(net_o, 55)
    batch = {"noisy_audio_spec": det_input((1, 1, 376, 257), 508).abs(),
             "mask": det_input((1, 1, 376, 257), 509).abs()}
    out, diffs = {}, {}
    for mode in ("eval", "train"):
        net_r.train(mode == "train")
        net_o.train(mode == "train")
        net_r.zero_grad()
        net_o.zero_grad()
        a = net_r(batch)
        la = net_r.cal_loss(batch)
        bb = net_o(batch)
        lb = net_o.cal_loss(batch)
        out["pred_" + mode], out["loss_" + mode] = a.detach(), la.detach()
        diffs[mode] = {"pred": _maxabs(bb, a), "loss": abs(float(la) - float(lb))}
        if mode == "train":
            la.backward()
            lb.backward()
            grads = {"g_" + k.replace(".", "__"): p.grad.clone() for k, p in net_r.named_parameters()}
            diffs["param_grads"] = max(_maxabs(p.grad, grads["g_" + k.replace(".", "__")])
                                       for k, p in net_o.named_parameters())
    _save("avse1_aonly", dict(**out, **grads),
          "AVNet audio-only (train.py:28-30, model.py:117-118): AudioFeatNet -> FusionNet(a_only, LSTM 1028->257) "
          "on (1,1,376,257) det_input seeds 508/509 (abs; regenerated in tests), eval + train BN, L1 loss grads "
          "in train mode; det_init seed 55", diffs)


# ============================================================================ DPMamba wrapper

def gen_dpmamba():
    """Pins the dual-path forward the reference holds in-tree (modules/dual_path.py:53-150,
    Dual_Path_Model_Skip.forward, skip_n_block=0) over a stub base class: speechbrain 1.0.0's
    Dual_Path_Model.__init__ / _Segmentation / _over_add / Dual_Computation_Block are not vendored, so the
    stub binds them to oracle/dpmamba_ref.py's restatement (those helpers stay "parity unpinned"); the
    intra / inter models are the reference's own MambaBlocksSequential (fast path with shimmed natives)."""
    from oracle import dpmamba_ref

    class SBDualPath(dpmamba_ref.Dual_Path_Model):
        def __init__(self, in_channels, out_channels, intra_model, inter_model, num_layers=1, norm="ln", K=200,
                     num_spks=2, skip_around_intra=True, linear_layer_after_inter_intra=True,
                     use_global_pos_enc=False, max_length=20000):
            assert norm == "ln" and not linear_layer_after_inter_intra and not use_global_pos_enc
            super().__init__(in_channels, out_channels, intra_model, inter_model, num_layers, K, num_spks,
                             skip_around_intra)
            self.use_global_pos_enc = use_global_pos_enc
    _mod("speechbrain.lobes.models.dual_path", Dual_Path_Model=SBDualPath)
    # the fast path of the reference's MambaBlocksSequential (as in gen_mamba's masknet case)
    ssi = _import_from("Mamba-TasNet", "modules.mamba.selective_scan_interface")
    ref_scan = ssi.selective_scan_ref

    def ss_fwd(u, delta, A, B, C, D, z, delta_bias, delta_softplus):
        out, last = ref_scan(u, delta, A, B, C, D, None, delta_bias, delta_softplus, return_last_state=True)
        x = torch.stack([torch.zeros_like(last), last], -1).reshape(last.shape[0], last.shape[1], 1, -1)
        return [out, x, out * F.silu(z.float()).to(out.dtype)]
    sys.modules["selective_scan_cuda"].fwd = ss_fwd
    dp_mod = _import_from("Mamba-TasNet", "modules.dual_path")
    mb = sys.modules["modules.mamba_blocks"] if "modules.mamba_blocks" in sys.modules else \
        _import_from("Mamba-TasNet", "modules.mamba_blocks")
    N, K = 64, 10
    out, diffs = {}, {}
    mix_w = det_input((2, N, 47), 901).abs()         # L=47: chunking pads (gap > 0)
    for sia in (True, False):
        mk = lambda: mb.MambaBlocksSequential(1, bidirectional=True, d_model=N, fused_add_norm=False,  # noqa: E731
                                              rms_norm=True)
        ref_dp = dp_mod.Dual_Path_Model_Skip(N, N, mk(), mk(), num_layers=2, norm="ln", K=K, num_spks=2,
                                             skip_around_intra=sia, skip_n_block=0,
                                             linear_layer_after_inter_intra=False)
        ours = dpmamba_ref.Dual_Path_Model(N, N, dpmamba_ref.MambaBlocksSequential(1, N),
                                           dpmamba_ref.MambaBlocksSequential(1, N), 2, K, 2, sia)
        _same_keys(ref_dp, ours)
        det_init_(ref_dp, 91)
        det_init_(ours, 91)
        with torch.no_grad():
            a = ref_dp(mix_w)
            bb = ours(mix_w)
        tag = "sia" if sia else "nosia"
        out["est_mask_" + tag] = a
        diffs[tag] = _maxabs(bb, a)
    _save("dpmamba_wrapper", dict(mixture_w=mix_w, **out),
          "modules/dual_path.py:53-150 Dual_Path_Model_Skip.forward (skip_n_block=0) on a stub speechbrain base "
          "(oracle restatement of __init__/_Segmentation/_over_add/Dual_Computation_Block), intra/inter = reference "
          "MambaBlocksSequential(1 BiMamba v2, d_model 64), 2 dual-path layers, K=10, L=47, skip_around_intra "
          "True/False, det_init seed 91", diffs)


# ============================================================================ avse2

def gen_avse2():
    m2 = _import_from("baseline/avse2", "model")
    # DPRNN separator block (bidirectional LSTMs, K=20 chunks x S=5) fwd + every gradient
    sb_r, sb_o = m2.SeparatorBlock(64, 128, bidirectional=True), avse2_ref.SeparatorBlock(64, 128, True)
    _same_keys(sb_r, sb_o)
    det_init_(sb_r, 81)
    det_init_(sb_o, 81)
    x = det_input((2, 64, 20, 5), 801).requires_grad_(True)
    gy = det_input((2, 64, 20, 5), 802)
    y_r = sb_r(x)
    (y_r * gy).sum().backward()
    grads = {"g_" + k.replace(".", "__"): p.grad.clone() for k, p in sb_r.named_parameters()}
    gx = x.grad.clone()
    x2 = x.detach().clone().requires_grad_(True)
    y_o = sb_o(x2)
    (y_o * gy).sum().backward()
    gmax = max(_maxabs(p.grad, grads["g_" + k.replace(".", "__")]) for k, p in sb_o.named_parameters())
    _save("avse2_sepblock", dict(x=x.detach(), gy=gy, y=y_r.detach(), gx=gx, **grads),
          "SeparatorBlock(64, 128, bidirectional) model.py:88-123 (DPRNN intra/inter LSTM + Linear + GroupNorm), "
          "fwd + grads, det_init seed 81", {"y": _maxabs(y_o, y_r), "gx": _maxabs(x2.grad, gx), "param_grads": gmax})

    # full AVSEModule: 1 s @ 16 kHz (1999 encoder frames -> 20 chunks of 200) + 25 lip frames 64x64, eval
    full_r, full_o = m2.AVSEModule(), avse2_ref.AVSEModule()
    _same_keys(full_r, full_o)
    det_init_(full_r, 82)
    det_init_(full_o, 82)
    full_r.eval()
    full_o.eval()
    batch = {"noisy_audio": 0.1 * det_input((2, 16000), 803), "video_frames": det_input((2, 1, 25, 64, 64), 804, "uniform"),
             "clean": 0.1 * det_input((2, 16000), 805)}
    with torch.no_grad():
        a = full_r(batch)
        la = full_r.cal_loss({k: v.clone() for k, v in batch.items()})
        bb = full_o(batch)
        lb = full_o.cal_loss({k: v.clone() for k, v in batch.items()})
    _save("avse2_full", dict(out=a, loss=la, vis_checksum=batch["video_frames"].double().sum()),
          "AVSEModule eval forward + cal_loss (SI-SNR clamp -30) on (2,16000) audio + (2,1,25,64,64) lips; inputs "
          "det_input seeds 803-805 regenerated in tests; det_init seed 82",
          {"out": _maxabs(bb, a), "loss": abs(float(la) - float(lb))})


def main():
    """python make_golden.py [case ...]: all cases, or only the named ones (merged into manifest.json)."""
    global MANIFEST
    avse2_dnn = _install_stubs()
    gens = {"losses": partial(gen_losses, avse2_dnn), "mamba": gen_mamba, "avse4": gen_avse4, "avse1": gen_avse1,
            "avse2": gen_avse2, "avse1_aonly": gen_avse1_aonly, "dpmamba": gen_dpmamba}
    only = sys.argv[1:] or list(gens)
    if sys.argv[1:]:
        with open(os.path.join(HERE, "manifest.json")) as f:
            MANIFEST = json.load(f)
    for name in only:
        gens[name]()
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(MANIFEST, f, indent=1, sort_keys=True)
    print("total bytes", sum(v["bytes"] for v in MANIFEST.values()))


if __name__ == "__main__":
    main()
