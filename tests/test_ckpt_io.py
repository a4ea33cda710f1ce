"""CPU tests of the checkpoint / wav compatibility layer (avse_challenge_amd/ckpt_io.py).

Formats follow the reference's call sites: Lightning `.ckpt` (`baseline/avse4/test.py:32`), SpeechBrain
`CKPT+*/<name>.ckpt` + CKPTMETA.yaml (`Mamba-TasNet/train_wsj0mix.py:414-416`, `inference.ipynb` cell 1),
PCM_16 wavs (`baseline/avse4/test.py:47`, `evaluation/avse4/objective_evaluation.py:23-35`).  The reference's
shipped `hyperparams.yaml` files are read as data when /root/reference is present (skipped otherwise).
"""
import os
import struct

import numpy as np
import pytest
import torch

from avse_challenge_amd import ckpt_io

REF_CKPTS = "/root/reference/Mamba-TasNet/ckpts/WSJ0Mix"


def _perturb(module, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in module.parameters():
            p.copy_(torch.randn(p.shape, generator=g))


def _same_state(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    return sa.keys() == sb.keys() and all(torch.equal(sa[k], sb[k]) for k in sa)


def test_wav_pcm16_layout_and_scaling(tmp_path):
    x = np.stack([np.linspace(-1, 1, 101), 0.5 * np.sin(np.arange(101))], axis=1)   # (frames, channels)
    p = ckpt_io.write_wav(str(tmp_path / "a.wav"), x, 16000)
    raw = open(p, "rb").read()
    assert raw[:4] == b"RIFF" and raw[8:16] == b"WAVEfmt " and raw[36:40] == b"data"
    assert struct.unpack("<HHIIHH", raw[20:36]) == (1, 2, 16000, 16000 * 4, 4, 16)
    assert struct.unpack("<I", raw[4:8])[0] == len(raw) - 8 and struct.unpack("<I", raw[40:44])[0] == 101 * 4
    pcm = np.frombuffer(raw[44:], "<i2").reshape(101, 2)                   # interleaved frames
    assert np.array_equal(pcm, np.rint(x * 32767).astype(np.int16))
    y, sr = ckpt_io.read_wav(p)
    assert sr == 16000 and y.shape == (101, 2) and y.dtype == np.float64
    assert np.array_equal(y, pcm / 32768.0)
    assert np.abs(y - x).max() <= 1.0 / 32768 + 1.0 / 65536


def test_wav_mono_float_and_clipping(tmp_path):
    x = np.array([0.0, 0.25, -0.75, 1.5, -2.0])
    y, _ = ckpt_io.read_wav(ckpt_io.write_wav(str(tmp_path / "m.wav"), x, 8000))
    assert y.shape == (5,)
    assert np.array_equal(y, np.array([0, 8192, -24575, 32767, -32767]) / 32768.0)   # saturates out of range
    f, sr = ckpt_io.read_wav(ckpt_io.write_wav(str(tmp_path / "f.wav"), x, 8000, subtype="FLOAT"))
    assert sr == 8000 and np.array_equal(f, x.astype(np.float32).astype(np.float64))
    with pytest.raises(ValueError):
        ckpt_io.read_wav(__file__)              # not RIFF/WAVE


def test_enhance_output_round_trip_binaural(tmp_path):
    """avse4 test.py:47 writes `estimated_audio.T` of a peak-normalised (2, T) estimate; the evaluation reads
    it back as (T, 2)."""
    est = np.random.default_rng(0).standard_normal((2, 4000))
    est /= np.abs(est).max()
    y, _ = ckpt_io.read_wav(ckpt_io.write_wav(str(tmp_path / "scene.wav"), est.T, 16000))
    assert y.shape == (4000, 2) and np.abs(y - est.T).max() <= 1.5 / 32768   # 32767 / 32768 scale + rounding


def test_lightning_checkpoint_avse4(tmp_path):
    from avse_challenge_amd.avse4 import AVSE4BaselineModule
    m = AVSE4BaselineModule(lr=3e-4, num_channels=1)
    _perturb(m, 1)
    hp = {"lr": 3e-4, "a_only": False, "val_dataset": None, "loss": "si_snr", "batch_size": 4,
          "frontend_ckpt_path": None, "num_channels": 1}            # model.py:296-316 save_hyperparameters()
    p = ckpt_io.save_lightning_checkpoint(m, str(tmp_path / "epoch=1.ckpt"), hp, epoch=1, global_step=10)
    ck = torch.load(p, weights_only=True)
    assert ck["epoch"] == 1 and ck["global_step"] == 10 and ck["hyper_parameters"]["batch_size"] == 4
    m2 = AVSE4BaselineModule.load_from_checkpoint(p)
    assert m2.lr == 3e-4 and m2.num_channels == 1 and _same_state(m, m2)
    with pytest.raises(RuntimeError):          # strict: a binaural module does not take a mono checkpoint
        AVSE4BaselineModule.load_from_checkpoint(p, num_channels=2)


def test_lightning_checkpoint_avse1_default_hparams(tmp_path):
    from avse_challenge_amd.avse1 import AVNet
    m = AVNet(a_only=True, lr=1e-3)
    _perturb(m, 2)
    p = ckpt_io.save_lightning_checkpoint(m, str(tmp_path / "last.ckpt"))
    assert torch.load(p, weights_only=True)["hyper_parameters"] == {"a_only": True, "lr": 1e-3}
    m2 = AVNet.load_from_checkpoint(p, nets=None)           # test.py:47 passes nets=; not a ctor arg here
    assert m2.a_only and m2.lr == 1e-3 and _same_state(m, m2)


def test_speechbrain_checkpointer_round_trip_and_selection(tmp_path):
    from avse_challenge_amd.mamba_tasnet import MambaTasNet
    save = str(tmp_path / "save")
    m = MambaTasNet(N=32, n_mamba=2)
    dirs = []
    for i, sisnr in enumerate([-10.0, -14.5, -12.0]):
        _perturb(m, 10 + i)
        dirs.append(ckpt_io.save_speechbrain_checkpoint(save, ckpt_io.speechbrain_modules(m), {"-si-snr": sisnr}))
        if i == 1:
            best = {k: v.clone() for k, v in m.state_dict().items()}
    names = [os.path.basename(d) for d in dirs]
    assert all(n.startswith("CKPT+") for n in names) and len(set(names)) == 3
    assert sorted(os.listdir(dirs[0])) == ["CKPTMETA.yaml", "decoder.ckpt", "encoder.ckpt", "masknet.ckpt"]
    assert ckpt_io.find_speechbrain_checkpoint(save, min_key="-si-snr") == dirs[1]
    assert ckpt_io.find_speechbrain_checkpoint(save, max_key="-si-snr") == dirs[0]
    assert ckpt_io.find_speechbrain_checkpoint(save) == dirs[2]                       # most recent
    assert ckpt_io.find_speechbrain_checkpoint(str(tmp_path / "none")) is None
    m2 = MambaTasNet(N=32, n_mamba=2)
    meta = ckpt_io.load_speechbrain_checkpoint(dirs[1], ckpt_io.speechbrain_modules(m2))
    assert meta["-si-snr"] == -14.5 and meta["end-of-epoch"] is True
    assert all(torch.equal(best[k], v) for k, v in m2.state_dict().items())
    # inference.ipynb cell 1 style: plain torch.load of each <name>.ckpt into the module
    m3 = MambaTasNet(N=32, n_mamba=2)
    for name, mod in ckpt_io.speechbrain_modules(m3).items():
        mod.load_state_dict(torch.load(os.path.join(dirs[1], name + ".ckpt"), weights_only=True))
    assert _same_state(m2, m3)


@pytest.mark.skipif(not os.path.isdir(REF_CKPTS), reason="reference checkpoints dir not present")
@pytest.mark.parametrize("size", ["XS", "S", "M", "L"])
def test_hparams_of_reference_checkpoints(size):
    """The reference's saved hyperparams.yaml (hyperpyyaml tags read as data) describe the same architecture
    this package builds: the model's encoder / masknet / decoder shapes match the yaml's module entries."""
    from avse_challenge_amd.dpmamba import DPMAMBA_SIZES
    for family in ("mambatasnet", "dpmamba"):
        hp = ckpt_io.read_hparams(os.path.join(REF_CKPTS, f"{family}_{size}", "1234", "hyperparams.yaml"))
        kind, kw = ckpt_io.model_kwargs_from_hparams(hp)
        assert kind == family
        assert hp["Encoder"]["out_channels"] == kw["N"] and hp["Decoder"]["stride"] == kw["kernel_size"] // 2
        if family == "dpmamba":
            assert hp["MaskNet"]["num_layers"] == kw["n_dp"] and hp["MaskNet"]["K"] == kw["chunk_size"]
            assert {k: kw[k] for k in DPMAMBA_SIZES[size]} == DPMAMBA_SIZES[size]
        else:
            assert hp["MaskNet"]["n_mamba"] == kw["n_mamba"] and hp["MaskNet"]["d_model"] == kw["N"]
        if size == "XS":                      # build only the small ones on CPU
            m = ckpt_io.model_from_hparams(hp)
            assert m.encoder.conv1d.weight.shape == (kw["N"], 1, kw["kernel_size"])


def test_hparams_ref_arithmetic_resolved(tmp_path):
    """The training recipes (hparams/WSJ0Mix/*.yaml) carry hyperpyyaml `!ref` arithmetic, e.g.
    `kernel_stride: !ref <kernel_size> // 2` and `n_mamba: !ref <n_mamba_dp> // 2`: resolved as data."""
    p = tmp_path / "recipe.yaml"
    p.write_text("N_encoder_out: 64\nout_channels: !ref <N_encoder_out>\nkernel_size: 16\n"
                 "kernel_stride: !ref <kernel_size> // 2\nnum_spks: 2\nssm_dim: 16\nmamba_expand: 2\nmamba_conv: 4\n"
                 "n_mamba: !ref (<kernel_size> - 12) * 2\n")
    kind, kw = ckpt_io.model_kwargs_from_hparams(str(p))
    assert kind == "mambatasnet" and kw["n_mamba"] == 8 and kw["N"] == 64 and kw["kernel_size"] == 16
    p.write_text(p.read_text().replace("out_channels: !ref <N_encoder_out>", "out_channels: 32"))
    with pytest.raises(ValueError, match="out_channels"):
        ckpt_io.model_kwargs_from_hparams(str(p))
    p.write_text(p.read_text().replace("out_channels: 32", "out_channels: 64").replace("// 2", "// 4"))
    with pytest.raises(ValueError, match="stride"):
        ckpt_io.model_kwargs_from_hparams(str(p))


RECIPES = "/root/reference/Mamba-TasNet/hparams/WSJ0Mix"


@pytest.mark.skipif(not os.path.isdir(RECIPES), reason="reference recipes not present")
@pytest.mark.parametrize("name", ["mambatasnet_XS", "mambatasnet_L", "dpmamba_S", "dpmamba_L"])
def test_reference_training_recipes_parse(name):
    from avse_challenge_amd.dpmamba import DPMAMBA_SIZES
    from avse_challenge_amd.mamba_tasnet import MAMBA_TASNET_SIZES
    kind, kw = ckpt_io.model_kwargs_from_hparams(os.path.join(RECIPES, name + ".yaml"))
    fam, size = name.split("_")
    assert kind == fam
    ref = (DPMAMBA_SIZES if fam == "dpmamba" else MAMBA_TASNET_SIZES)[size]
    assert {k: kw[k] for k in ref} == ref
