"""Checkpoint and wav I/O compatible with the reference's trainers and evaluation scripts.

Host-side only (no kernels).  Three formats, each read and written here so that the reference's tools consume
this package's outputs unchanged and this package consumes theirs:

- **Lightning `.ckpt`** (avse1 / avse4): `AVSE4BaselineModule.load_from_checkpoint(cfg.ckpt_path)` at
  `baseline/avse4/test.py:32`, `baseline/avse1/test.py:47`; the module calls `self.save_hyperparameters()`
  (`baseline/avse4/model.py:316`), so the file holds `state_dict` (the module's own keys, which this package
  keeps identical) and `hyper_parameters` (the constructor's arguments).
- **SpeechBrain checkpoint directories** (Mamba-TasNet / DPMamba): `Checkpointer(checkpoints_dir=save_folder,
  recoverables={encoder, decoder, masknet, counter, lr_scheduler})` at
  `Mamba-TasNet/hparams/WSJ0Mix/mambatasnet_L.yaml:188-195`; saved by `save_and_keep_only(meta={"-si-snr": v},
  min_keys=["-si-snr"])` (`train_wsj0mix.py:414-416`) into `CKPT+<date>+<time>+00/` with one
  `<name>.ckpt` state_dict per recoverable and a `CKPTMETA.yaml`; loaded module by module with
  `mod.load_state_dict(torch.load(CKPT_PATH/name.ckpt))` (`inference.ipynb` cell 1).
- **Enhanced / estimated wavs**: `sf.write(path, estimated_audio.T, samplerate=16000)` (`baseline/avse4/test.py:47`,
  libsndfile's default WAV subtype PCM_16) and `SoundFile(f).read()` (`evaluation/avse4/objective_evaluation.py:23-35`,
  float64 frames x channels).  `soundfile` is absent from this image, so `write_wav` / `read_wav` restate
  libsndfile's normalised conversions (write: rint(x * 32767); read: s / 32768).  Parity unpinned against
  libsndfile itself (not importable here); the CPU tests pin the byte layout and the scaling.

Loads default to `torch.load(weights_only=True)`: checkpoints are data, nothing in them is executed.
"""
import ast
import datetime
import inspect
import os
import re
import struct
import time

import numpy as np
import torch

import yaml

# ---------------------------------------------------------------------------------------------- Lightning


def save_lightning_checkpoint(module, path, hyper_parameters=None, epoch=0, global_step=0, optimizer=None):
    """Write `module` as a Lightning checkpoint dict (the layout `LightningModule.load_from_checkpoint` reads)."""
    ckpt = {
        "epoch": int(epoch),
        "global_step": int(global_step),
        "pytorch-lightning_version": "2.1.0",
        "state_dict": {k: v.detach().cpu() for k, v in module.state_dict().items()},
        "hyper_parameters": dict(hyper_parameters or _ctor_hparams(module)),
        "optimizer_states": [optimizer.state_dict()] if optimizer is not None else [],
        "lr_schedulers": [],
        "callbacks": {},
    }
    torch.save(ckpt, path)
    return path


def load_lightning_checkpoint(cls, path, map_location="cpu", strict=True, weights_only=True, **overrides):
    """`cls.load_from_checkpoint(path, **overrides)`: build `cls` from the saved `hyper_parameters` (arguments
    `cls.__init__` does not name are dropped: the reference's `val_dataset`, `loss`, `batch_size`,
    `frontend_ckpt_path` configure its trainer, not the network) and load `state_dict` (strict by default,
    as Lightning)."""
    ckpt = torch.load(path, map_location=map_location, weights_only=weights_only)
    if "state_dict" not in ckpt:
        raise KeyError(f"{path}: not a Lightning checkpoint (no 'state_dict')")
    hp = dict(ckpt.get("hyper_parameters", {}))
    hp.update(overrides)
    params = inspect.signature(cls.__init__).parameters
    named = {n for n, p in params.items() if n != "self" and p.kind not in (p.VAR_KEYWORD, p.VAR_POSITIONAL)}
    model = cls(**{k: v for k, v in hp.items() if k in named})
    model.load_state_dict(ckpt["state_dict"], strict=strict)
    return model


def _ctor_hparams(module):
    """Constructor arguments of `module` that are stored as attributes of the same name (save_hyperparameters)."""
    params = inspect.signature(type(module).__init__).parameters
    return {n: getattr(module, n) for n, p in params.items()
            if n != "self" and p.kind == p.POSITIONAL_OR_KEYWORD and hasattr(module, n)
            and isinstance(getattr(module, n), (bool, int, float, str, type(None)))}


# ---------------------------------------------------------------------------------------------- SpeechBrain

CKPT_PREFIX = "CKPT"
METAFNAME = "CKPTMETA.yaml"


def speechbrain_modules(model):
    """The recoverables of the reference's hparams (`encoder`, `decoder`, `masknet`) on a MambaTasNet /
    DPMambaTasNet of this package (same submodule trees and state_dict keys)."""
    return {"encoder": model.encoder, "decoder": model.decoder, "masknet": model.masknet}


def save_speechbrain_checkpoint(save_dir, modules, meta=None, end_of_epoch=True, name=None):
    """One `CKPT+YYYY-MM-DD+HH-MM-SS+00/` directory: `<name>.ckpt` = torch.save(state_dict) per module and
    `CKPTMETA.yaml` = meta + `end-of-epoch` + `unixtime`."""
    now = time.time()
    if name is None:
        stamp = datetime.datetime.fromtimestamp(now, datetime.timezone.utc).strftime("%Y-%m-%d+%H-%M-%S")
        name = f"{CKPT_PREFIX}+{stamp}+00"
        base, k = name, 0
        while os.path.exists(os.path.join(save_dir, name)):
            k += 1
            name = f"{base}_{k}"
    ckpt_dir = os.path.join(save_dir, name)
    os.makedirs(ckpt_dir)
    for mod_name, mod in modules.items():
        torch.save({k: v.detach().cpu() for k, v in mod.state_dict().items()},
                   os.path.join(ckpt_dir, f"{mod_name}.ckpt"))
    full_meta = {**(meta or {}), "end-of-epoch": bool(end_of_epoch), "unixtime": now}
    with open(os.path.join(ckpt_dir, METAFNAME), "w") as f:
        yaml.safe_dump({k: (float(v) if isinstance(v, (np.floating, torch.Tensor)) else v)
                        for k, v in full_meta.items()}, f)
    return ckpt_dir


def list_speechbrain_checkpoints(save_dir):
    """[(ckpt_dir, meta)] for every `CKPT+*` directory holding a CKPTMETA.yaml."""
    out = []
    if not os.path.isdir(save_dir):
        return out
    for name in sorted(os.listdir(save_dir)):
        d = os.path.join(save_dir, name)
        mf = os.path.join(d, METAFNAME)
        if name.startswith(CKPT_PREFIX + "+") and os.path.isfile(mf):
            with open(mf) as f:
                out.append((d, yaml.safe_load(f) or {}))
    return out


def find_speechbrain_checkpoint(save_dir, min_key=None, max_key=None):
    """The checkpoint `Checkpointer.recover_if_possible(min_key=..., max_key=...)` would pick: the lowest
    `meta[min_key]`, the highest `meta[max_key]`, or else the most recent (`unixtime`).  Checkpoints whose meta
    lacks the key are skipped.  Returns the directory, or None if there is none."""
    if min_key is not None and max_key is not None:
        raise ValueError("give at most one of min_key / max_key")
    cks = list_speechbrain_checkpoints(save_dir)
    if min_key is not None:
        cks = [(d, m) for d, m in cks if min_key in m]
        key = lambda dm: -float(dm[1][min_key])  # noqa: E731
    elif max_key is not None:
        cks = [(d, m) for d, m in cks if max_key in m]
        key = lambda dm: float(dm[1][max_key])  # noqa: E731
    else:
        key = lambda dm: float(dm[1].get("unixtime", 0.0))  # noqa: E731
    return max(cks, key=key)[0] if cks else None


def load_speechbrain_checkpoint(ckpt_dir, modules, map_location="cpu", strict=True):
    """inference.ipynb cell 1: `mod.load_state_dict(torch.load(ckpt_dir/<name>.ckpt))` for each module.
    Returns the CKPTMETA dict."""
    for mod_name, mod in modules.items():
        path = os.path.join(ckpt_dir, f"{mod_name}.ckpt")
        if not os.path.isfile(path):
            raise FileNotFoundError(f"{path}: recoverable '{mod_name}' missing from checkpoint")
        mod.load_state_dict(torch.load(path, map_location=map_location, weights_only=True), strict=strict)
    mf = os.path.join(ckpt_dir, METAFNAME)
    if os.path.isfile(mf):
        with open(mf) as f:
            return yaml.safe_load(f) or {}
    return {}


class _TagTolerantLoader(yaml.SafeLoader):
    """SafeLoader that reads hyperpyyaml tags (`!new:`, `!name:`, `!ref`, `!apply:` ...) as plain data: tagged
    mappings become dicts with the tag under `__tag__`.  Nothing named by a tag is imported or called."""


def _tagged(loader, tag_suffix, node):
    if isinstance(node, yaml.MappingNode):
        d = loader.construct_mapping(node, deep=True)
        return {"__tag__": "!" + tag_suffix, **d}
    if isinstance(node, yaml.SequenceNode):
        return loader.construct_sequence(node, deep=True)
    return loader.construct_scalar(node)


_TagTolerantLoader.add_multi_constructor("!", _tagged)


def read_hparams(path):
    """Parse a SpeechBrain `hyperparams.yaml` (as saved next to the reference's checkpoints) as data."""
    with open(path) as f:
        return yaml.load(f, Loader=_TagTolerantLoader)  # noqa: S506 (SafeLoader subclass)


_REF = re.compile(r"<([A-Za-z_][A-Za-z0-9_]*)>")


def _resolve(hp, key, seen=()):
    """A top-level hparams value with hyperpyyaml's `!ref` resolved as data: `<name>` references are substituted
    (recursively) and simple integer arithmetic (+ - * // / and parentheses, e.g. `<kernel_size> // 2`) is
    evaluated on a parsed expression tree — nothing is imported or executed."""
    v = hp[key]
    if not isinstance(v, str) or "<" not in v:
        return v
    if key in seen:
        raise ValueError(f"cyclic !ref at {key}")

    def sub(m):
        r = _resolve(hp, m.group(1), seen + (key,))
        if not isinstance(r, (int, float)) or isinstance(r, bool):
            raise ValueError(f"!ref <{m.group(1)}> is not a number: {r!r}")
        return repr(r)
    return _arith(_REF.sub(sub, v))


def _arith(expr):
    ops = {ast.Add: lambda a, b: a + b, ast.Sub: lambda a, b: a - b, ast.Mult: lambda a, b: a * b,
           ast.FloorDiv: lambda a, b: a // b, ast.Div: lambda a, b: a / b}

    def ev(n):
        if isinstance(n, ast.Expression):
            return ev(n.body)
        if isinstance(n, ast.Constant) and isinstance(n.value, (int, float)) and not isinstance(n.value, bool):
            return n.value
        if isinstance(n, ast.BinOp) and type(n.op) in ops:
            return ops[type(n.op)](ev(n.left), ev(n.right))
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, ast.USub):
            return -ev(n.operand)
        raise ValueError(f"unsupported !ref expression {expr!r}")
    return ev(ast.parse(expr.strip(), mode="eval"))


def model_kwargs_from_hparams(hp):
    """Constructor kwargs of this package's MambaTasNet / DPMambaTasNet from the reference's hparams: the
    training recipes `mambatasnet_*.yaml` / `dpmamba_*.yaml` (hparams/WSJ0Mix/, `!ref` arithmetic such as
    `kernel_stride: !ref <kernel_size> // 2` resolved) or a saved `hyperparams.yaml`.  Returns (kind, kwargs),
    kind in {"mambatasnet", "dpmamba"}.  The MaskNet bottleneck / d_model come from `out_channels`, which this
    package's models tie to the encoder width `N_encoder_out` (as every reference recipe does)."""
    if isinstance(hp, str):
        hp = read_hparams(hp)
    g = lambda k: _resolve(hp, k)                                                      # noqa: E731
    common = dict(N=int(g("N_encoder_out")), kernel_size=int(g("kernel_size")), n_spk=int(g("num_spks")),
                  d_state=int(g("ssm_dim")), expand=int(g("mamba_expand")), d_conv=int(g("mamba_conv")))
    if "out_channels" in hp and int(g("out_channels")) != common["N"]:
        raise ValueError(f"out_channels ({g('out_channels')}) != N_encoder_out ({common['N']}): the MaskNet "
                         "bottleneck width must equal the encoder width in this package's models")
    stride = int(g("kernel_stride")) if "kernel_stride" in hp else common["kernel_size"] // 2
    if stride != common["kernel_size"] // 2:
        raise ValueError("encoder stride must be kernel_size // 2 (the reference's Encoder / Decoder)")
    if "n_dp" in hp:
        return "dpmamba", dict(common, n_dp=int(g("n_dp")), chunk_size=int(g("chunk_size")),
                               skip_around_intra=bool(g("skip_around_intra")), n_mamba_dp=int(g("n_mamba_dp")))
    return "mambatasnet", dict(common, n_mamba=int(g("n_mamba")))


def model_from_hparams(hp):
    """A MambaTasNet / DPMambaTasNet with the architecture the hparams file describes (random init)."""
    kind, kw = model_kwargs_from_hparams(hp)
    if kind == "dpmamba":
        from .dpmamba import DPMambaTasNet
        return DPMambaTasNet(**kw)
    from .mamba_tasnet import MambaTasNet
    return MambaTasNet(**kw)


# ---------------------------------------------------------------------------------------------- wav

_WAVE_FORMAT_PCM, _WAVE_FORMAT_IEEE_FLOAT, _WAVE_FORMAT_EXTENSIBLE = 1, 3, 0xFFFE


def write_wav(path, audio, samplerate, subtype="PCM_16"):
    """`soundfile.write(path, audio, samplerate)`: `audio` is (frames,) or (frames, channels) (the reference
    passes `estimated_audio.T`).  PCM_16 stores rint(x * 32767) (libsndfile's normalised float->short
    scale); values outside [-1, 1] saturate (libsndfile without SFC_SET_CLIPPING would wrap them).
    FLOAT stores IEEE float32."""
    a = np.asarray(audio)
    if a.ndim == 1:
        a = a[:, None]
    if a.ndim != 2:
        raise ValueError(f"audio must be (frames,) or (frames, channels), got {a.shape}")
    frames, ch = a.shape
    if subtype == "PCM_16":
        data = np.rint(np.clip(a.astype(np.float64), -1.0, 1.0) * 32767.0).astype("<i2").tobytes()
        fmt, bits = _WAVE_FORMAT_PCM, 16
    elif subtype == "FLOAT":
        data = a.astype("<f4").tobytes()
        fmt, bits = _WAVE_FORMAT_IEEE_FLOAT, 32
    else:
        raise ValueError(f"unsupported subtype {subtype!r} (PCM_16, FLOAT)")
    block = ch * bits // 8
    fmt_chunk = struct.pack("<HHIIHH", fmt, ch, int(samplerate), int(samplerate) * block, block, bits)
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 4 + 8 + len(fmt_chunk) + 8 + len(data)) + b"WAVE")
        f.write(b"fmt " + struct.pack("<I", len(fmt_chunk)) + fmt_chunk)
        f.write(b"data" + struct.pack("<I", len(data)) + data)
    return path


def read_wav(path, always_2d=False):
    """`SoundFile(path).read()`: float64 (frames,) for mono, (frames, channels) otherwise; PCM scaled by
    1 / 2**(bits-1) (libsndfile's normalised read), float data as stored.  Returns (audio, samplerate)."""
    with open(path, "rb") as f:
        raw = f.read()
    if raw[:4] != b"RIFF" or raw[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt = 12, None
    while pos + 8 <= len(raw):
        cid, size = raw[pos:pos + 4], struct.unpack("<I", raw[pos + 4:pos + 8])[0]
        body = raw[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, sr, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == _WAVE_FORMAT_EXTENSIBLE and len(body) >= 26:
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, sr, bits)
        elif cid == b"data":
            if fmt is None:
                raise ValueError(f"{path}: data chunk before fmt chunk")
            tag, ch, sr, bits = fmt
            if tag == _WAVE_FORMAT_PCM and bits == 16:
                a = np.frombuffer(body, "<i2").astype(np.float64) / 32768.0
            elif tag == _WAVE_FORMAT_PCM and bits == 32:
                a = np.frombuffer(body, "<i4").astype(np.float64) / 2147483648.0
            elif tag == _WAVE_FORMAT_PCM and bits == 24:
                b = np.frombuffer(body[:len(body) // 3 * 3], np.uint8).reshape(-1, 3).astype(np.int32)
                v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
                a = np.where(v >= 1 << 23, v - (1 << 24), v).astype(np.float64) / 8388608.0
            elif tag == _WAVE_FORMAT_IEEE_FLOAT and bits in (32, 64):
                a = np.frombuffer(body, "<f4" if bits == 32 else "<f8").astype(np.float64)
            else:
                raise ValueError(f"{path}: unsupported WAV format tag {tag} / {bits} bits")
            a = a[:len(a) // ch * ch].reshape(-1, ch)
            return (a if (always_2d or ch > 1) else a[:, 0]), sr
        pos += 8 + size + (size & 1)
    raise ValueError(f"{path}: no data chunk")
