"""Throughput bench: utterances/s of the avse1 AV training step on MI355X (BASELINE configs[1]).

python bench.py [--gpus N --steps K --warmup W --workload avse1|mamba]
For N > 1 launch under torch.distributed.run (one rank per GPU, RCCL); every rank trains on
its own synthetic batch (weak scaling, DDP gradient all-reduce overlapped with backward).

A step = one pass of the hot path over one batch, inputs already resident in HBM:
  avse1 (default, C2): HIP STFT of the noisy + clean waveforms (B x 48000 @ 16 kHz)
          -> AVNet forward (75 lip frames 96x96 uint8) -> L1 loss -> backward -> Adam.
  mamba (C3):  Mamba-TasNet (XS/S/M/L) on B x 4 s @ 8 kHz mixtures -> PIT SI-SNR -> bwd -> Adam.
  avse4 (C4):  binaural AVSE4BaselineModule on B x 2ch x 5 s @ 16 kHz + 125 lip frames 112x112
               -> SI-SNR loss -> bwd -> Adam (C4: 16 per GPU).
  avmamba (C5): Mamba-TasNet-L + avse4 lip encoder, bf16 autocast, B x 3 s @ 16 kHz (L = 5999) + 75 lip
               frames 112x112 -> SI-SNR loss -> bwd -> Adam (C5: 32 per GPU).
Rank 0 prints ONE JSON line (plus "roofline" for the dominant kernel, timed live with HIP
events on torch's current stream, and "cpu_baseline": the oracle restatement on host cores).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
import avse_challenge_amd  # noqa: E402,F401  (sets MIOPEN_USER_DB_PATH before the first convolution)

# MIOpen convolutions / batch norms on channels_last tensors run as NHWC kernels instead of being
# transposed around NCHW ones (read by PyTorch-ROCm per call)
os.environ.setdefault("PYTORCH_MIOPEN_SUGGEST_NHWC", "1")
os.environ.setdefault("PYTORCH_MIOPEN_SUGGEST_NHWC_BATCHNORM", "1")

METRIC = "utterances/sec (3s@16kHz + 75 lip frames)"
# HBM bytes per launch of each roofline kernel, from rocprofv3 PMC passes (tools/pmc_traffic.sh:
# FETCH_SIZE and WRITE_SIZE in separate passes, corrected as MI355X_MICROARCH.md prescribes)
TRAFFIC_FILE = os.path.join(REPO, "profiles", "r01_traffic.json")
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP32_PEAK_TFS = 157.3          # FP32 matrix (= vector) peak, spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="avse1", choices=["avse1", "mamba", "avse4", "dpmamba", "avse2", "avmamba"])
    p.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the BASELINE config's)")
    p.add_argument("--size", default="L", choices=["XS", "S", "M", "L"], help="Mamba-TasNet / DPMamba size")
    p.add_argument("--lip-hw", type=int, default=96)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--no-graph", action="store_true", help="eager launches instead of captured HIP graphs")
    return p.parse_args()


def setup_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, torch.device("cuda", local)


def barrier(world):
    if world > 1:
        dist.barrier()


# ------------------------------------------------------------------------------ workloads

class Avse1Step:
    unit_desc = "3s@16kHz utterance + 75 lip frames"
    # MIOpen's LSTM (FusionNet) issues hipBLASLt calls that are illegal under stream capture, and the
    # step is kernel-bound at B=32 anyway: avse1 runs with eager launches.
    graph_ok = False

    def __init__(self, B, dev, rank, world, lip_hw):
        from avse_challenge_amd import avse1, data
        self.B, self.lip_hw = B, lip_hw
        self.model = avse1.AVNet().to(dev).train()
        if int(os.environ.get("AVSE_CHANNELS_LAST", "1")):      # NHWC audio convs (+4.5% step rate)
            self.model.net_audiofeat.use_channels_last()
        self.lr, self.clip = self.model.lr, None
        self.noisy, self.clean, self.lips = data.avse1_batch(B, dev, 1234 + rank, lip_hw)
        self.avse1 = avse1

    def loss(self):
        batch = self.avse1.AVNet.features_from_waves(self.noisy, self.clean)
        batch["lip_images"] = self.lips
        return self.model.loss(self.model(batch), batch["mask"])

    def config(self, world):
        return {"workload": "avse1 AV baseline train step (BASELINE configs[1]): HIP STFT front-end + AVNet "
                            "(ResNet18 lip enc + TCN, dilated Conv2d audio net, LSTM fusion) fwd/bwd + Adam",
                "global_batch": self.B * world, "per_gpu_batch": self.B, "seq_len": 48000,
                "stft_frames": 376, "lip_frames": 75, "lip_hw": self.lip_hw, "parallelism": f"dp{world}"}

    def roofline(self, dev):
        """Dominant kernel class of the step: the 64->64 5x5 dilated Conv2d of AudioFeatNet (MFMA-bound).
        Times conv3 (dilation 4) forward at the step's shape with HIP events; FLOPs = 2*B*64*64*25*376*257."""
        conv = self.model.net_audiofeat.conv3
        x = torch.randn(self.B, 64, 376, 257, device=dev)
        if getattr(self.model.net_audiofeat, "channels_last", False):
            x = x.to(memory_format=torch.channels_last)        # the layout the step runs the conv in
        with torch.no_grad():
            for _ in range(3):
                conv(x)
            torch.cuda.synchronize()
            n = 10
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                conv(x)
            e1.record()
            torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        flops = 2.0 * self.B * 64 * 64 * 25 * 376 * 257
        ach = flops / (ms * 1e-3) / 1e12
        return _with_traffic({"kernel": "AudioFeatNet.conv3 fwd (Conv2d 64->64 5x5 dil 4, MIOpen)", "bound": "mfma",
                              "achieved": round(ach, 2), "peak": FP32_PEAK_TFS, "unit": "TFLOP/s",
                              "frac": round(ach / FP32_PEAK_TFS, 4), "traffic": None, "avg_ms": round(ms, 4),
                              "algorithmic_flops_per_launch": flops}, "conv3" if self.B == 32 else "-")

    def cpu_baseline(self):
        from oracle import avse1_ref, stft_ref
        nthreads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
        torch.set_num_threads(max(1, min(nthreads, 64)))
        B = 2
        m = avse1_ref.AVNet().train()
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        g = torch.Generator().manual_seed(0)
        noisy = 0.1 * torch.randn(B, 48000, generator=g)
        clean = 0.1 * torch.randn(B, 48000, generator=g)
        lips = torch.randint(0, 256, (B, 3, 75, self.lip_hw, self.lip_hw), generator=g, dtype=torch.uint8)

        def step():
            batch = {"noisy_audio_spec": torch.from_numpy(stft_ref.stft_mag_T(noisy.numpy()))[:, None],
                     "mask": torch.from_numpy(stft_ref.stft_mag_T(clean.numpy()))[:, None], "lip_images": lips}
            loss = m.cal_loss(batch)
            opt.zero_grad()
            loss.backward()
            opt.step()
        step()
        t0 = time.perf_counter()
        iters = 0
        while iters < 2 or (time.perf_counter() - t0 < 10.0 and iters < 6):
            step()
            iters += 1
        dt = time.perf_counter() - t0
        return {"value": round(B * iters / dt, 4), "unit": "utt/s", "cores": torch.get_num_threads(), "kind": "port",
                "sample": f"oracle/avse1_ref AVNet train step (numpy librosa-0.8.1 STFT + fwd + bwd + Adam), "
                          f"batch {B}, {iters} steps after 1 warm-up, lips {self.lip_hw}x{self.lip_hw}"}


class MambaStep:
    unit_desc = "4s@8kHz WSJ0-2mix utterance"
    graph_ok = True

    def __init__(self, B, dev, rank, world, size):
        from avse_challenge_amd import data, losses, mamba_tasnet
        self.B, self.size = B, size
        self.model = mamba_tasnet.MambaTasNet(**mamba_tasnet.MAMBA_TASNET_SIZES[size]).to(dev).train()
        self.lr, self.clip = 1.5e-4, 5.0
        self.mix, self.tgt = data.wsj0mix_batch(B, dev, 4321 + rank)
        self.losses = losses

    def loss(self):
        return self.losses.si_snr_pit(self.tgt, self.model(self.mix)).mean()

    def config(self, world):
        return {"workload": f"Mamba-TasNet-{self.size} train step (BASELINE configs[2])", "global_batch": self.B * world,
                "per_gpu_batch": self.B, "seq_len": 32000, "frames": 3999, "parallelism": f"dp{world}"}

    def roofline(self, dev):
        from avse_challenge_amd import kernels as K
        d = 2 * self.model.masknet.mamba_net.layers[0].mixer.d_model
        b, l = self.B, 3999
        u = torch.randn(b, d, l, device=dev)
        dl = 0.1 * torch.randn(b, d, l, device=dev)
        z = torch.randn(b, d, l, device=dev)
        A = -torch.rand(d, 16, device=dev) - 0.5
        Bm, Cm = torch.randn(b, 16, l, device=dev), torch.randn(b, 16, l, device=dev)
        D, bias = torch.ones(d, device=dev), torch.zeros(d, device=dev)
        for _ in range(2):
            K.selective_scan_fwd(u, dl, A, Bm, Cm, D, z, bias, True, return_out=False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 5
        e0.record()
        for _ in range(n):
            K.selective_scan_fwd(u, dl, A, Bm, Cm, D, z, bias, True, return_out=False)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        byts = 4.0 * b * l * (4 * d + 2 * 16)     # u, delta, z, B, C read; out_z written
        ach = byts / (ms * 1e-3) / 1e9
        roof = {"kernel": "avse_scan_fwd (selective scan, fp32, training fwd: out_z + chunk states)", "bound": "hbm",
                "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": None, "avg_ms": round(ms, 4), "algorithmic_bytes_per_launch": byts}
        return _with_traffic(roof, "scan") if b == 64 else roof

    def cpu_baseline(self):
        from oracle import losses_ref, mamba_ref
        torch.set_num_threads(max(1, min(len(os.sched_getaffinity(0)), 64)))
        m = mamba_ref.MambaTasNet(**mamba_ref.MAMBA_TASNET_SIZES[self.size], n_spk=2)
        m.masknet.mamba_net.layers = m.masknet.mamba_net.layers[:1]      # 1 of n layers, scaled below
        n_layers = mamba_ref.MAMBA_TASNET_SIZES[self.size]["n_mamba"]
        g = torch.Generator().manual_seed(0)
        mix = 0.1 * torch.randn(1, 32000, generator=g)
        tgt = 0.1 * torch.randn(1, 32000, 2, generator=g)
        t0 = time.perf_counter()
        with torch.no_grad():
            m(mix)
        dt = (time.perf_counter() - t0) * n_layers      # forward only, 1 layer timed, scaled to all layers
        return {"value": round(1.0 / dt, 6), "unit": "utt/s", "cores": torch.get_num_threads(), "kind": "port",
                "sample": f"oracle/mamba_ref forward of 1 of {n_layers} BiMamba layers on one 4 s utterance, "
                          f"scaled x{n_layers} (forward only; the training step is >=3x slower)"}


class DPMambaStep(MambaStep):
    """DPMamba: the same BiMamba kernels on 250-frame chunks (intra) and across chunks
    (inter); 4 s @ 8 kHz WSJ0-2mix-shaped mixtures, PIT SI-SNR, bwd, Adam."""

    def __init__(self, B, dev, rank, world, size):
        from avse_challenge_amd import data, dpmamba, losses
        self.B, self.size = B, size
        self.model = dpmamba.DPMambaTasNet(**dpmamba.DPMAMBA_SIZES[size]).to(dev).train()
        self.lr, self.clip = 1.5e-4, 5.0
        self.mix, self.tgt = data.wsj0mix_batch(B, dev, 4321 + rank)
        self.losses = losses

    def config(self, world):
        return {"workload": f"DPMamba-{self.size} train step (SURVEY 8f row 2; dpmamba_{self.size}.yaml)",
                "global_batch": self.B * world, "per_gpu_batch": self.B, "seq_len": 32000, "frames": 3999,
                "chunk_size": 250, "chunks": 34, "parallelism": f"dp{world}"}

    def roofline(self, dev):
        """Intra-chunk selective scan fwd at the step's shape: (B*34 chunks, d_inner, 250)."""
        from avse_challenge_amd import kernels as K
        d = 2 * self.model.masknet.dual_mdl[0].intra_mdl.layers[0].mixer.d_model
        b, l = self.B * 34, 250
        u, dl, z = (torch.randn(b, d, l, device=dev) for _ in range(3))
        dl.mul_(0.1)
        A = -torch.rand(d, 16, device=dev) - 0.5
        Bm, Cm = torch.randn(b, 16, l, device=dev), torch.randn(b, 16, l, device=dev)
        D, bias = torch.ones(d, device=dev), torch.zeros(d, device=dev)
        return _time_hbm(lambda: K.selective_scan_fwd(u, dl, A, Bm, Cm, D, z, bias, True, return_out=False),
                         4.0 * b * l * (4 * d + 2 * 16), f"avse_scan_fwd (DPMamba intra, {b} x {d} x {l}, training fwd)")

    def cpu_baseline(self):
        from oracle import dpmamba_ref
        torch.set_num_threads(max(1, min(len(os.sched_getaffinity(0)), 64)))
        kw = dict(dpmamba_ref.DPMAMBA_SIZES[self.size])
        n_dp = kw.pop("n_dp")
        m = dpmamba_ref.DPMambaTasNet(n_dp=1, **kw)
        g = torch.Generator().manual_seed(0)
        mix = 0.1 * torch.randn(1, 32000, generator=g)
        t0 = time.perf_counter()
        with torch.no_grad():
            m(mix)
        dt = (time.perf_counter() - t0) * n_dp
        return {"value": round(1.0 / dt, 6), "unit": "utt/s", "cores": torch.get_num_threads(), "kind": "port",
                "sample": f"oracle/dpmamba_ref forward with 1 of {n_dp} dual-path layers on one 4 s utterance, "
                          f"scaled x{n_dp} (forward only)"}


class AVMambaStep:
    """C5 (BASELINE configs[4]): Mamba-TasNet-L conditioned on an avse4 lip encoder, bf16 autocast, 3 s @ 16 kHz
    (L = 5999 encoder frames), 75 gray lip frames 112x112, SI-SNR loss, 32 utterances per GPU."""
    unit_desc = "3s@16kHz utterance + 75 lip frames 112x112"
    graph_ok = True
    dtype = "bf16"

    def __init__(self, B, dev, rank, world, size):
        from avse_challenge_amd import avmamba, data
        self.B, self.size = B, size
        self.model = avmamba.AVMambaTasNet(**avmamba.AV_MAMBA_SIZES[size]).to(dev).train()
        self.lr, self.clip = 1.5e-4, 5.0
        g = torch.Generator(device=dev).manual_seed(999 + rank)
        noisy, clean, _ = data.avse1_batch(B, dev, 999 + rank, lip_hw=8)
        self.batch = {"noisy_audio": noisy, "clean": clean,
                      "vis_feat": torch.rand((B, 1, 75, 112, 112), device=dev, generator=g)}

    def loss(self):
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            return self.model.cal_loss(self.batch)

    def config(self, world):
        return {"workload": f"AV Mamba-TasNet-{self.size} train step (BASELINE configs[4]): avse4 lip encoder (fp32) + "
                            "Mamba-TasNet separator under bf16 autocast (bf16 scan / conv activations, fp32 state)",
                "global_batch": self.B * world, "per_gpu_batch": self.B, "seq_len": 48000, "frames": 5999,
                "lip_frames": 75, "lip_hw": 112, "parallelism": f"dp{world}"}

    def roofline(self, dev):
        """Selective scan fwd at the step's shape, bf16 u/delta/z/B/C/out_z: (B, 1024, 5999)."""
        from avse_challenge_amd import kernels as K
        d = 2 * self.model.masknet.mamba_net.layers[0].mixer.d_model
        b, l, bf = self.B, 5999, torch.bfloat16
        u, z = torch.randn(b, d, l, device=dev, dtype=bf), torch.randn(b, d, l, device=dev, dtype=bf)
        dl = (0.1 * torch.randn(b, d, l, device=dev)).to(bf)
        A = -torch.rand(d, 16, device=dev) - 0.5
        Bm, Cm = torch.randn(b, 16, l, device=dev, dtype=bf), torch.randn(b, 16, l, device=dev, dtype=bf)
        D, bias = torch.ones(d, device=dev), torch.zeros(d, device=dev)
        return _time_hbm(lambda: K.selective_scan_fwd(u, dl, A, Bm, Cm, D, z, bias, True, return_out=False),
                         2.0 * b * l * (4 * d + 2 * 16), f"avse_scan_fwd (bf16, {b} x {d} x {l}, training fwd)")

    def cpu_baseline(self):
        """oracle/avmamba_ref forward (fp32) of one 3 s utterance: the whole model with 0 and with 1 BiMamba layer
        timed, the per-layer time scaled to all n layers."""
        from oracle import avmamba_ref
        torch.set_num_threads(max(1, min(len(os.sched_getaffinity(0)), 64)))
        kw = avmamba_ref.AV_MAMBA_SIZES[self.size]
        m = avmamba_ref.AVMambaTasNet(**kw).eval()
        layers = m.masknet.mamba_net.layers
        g = torch.Generator().manual_seed(0)
        mix, lips = 0.1 * torch.randn(1, 48000, generator=g), torch.rand(1, 1, 75, 112, 112, generator=g)
        ts = []
        with torch.no_grad():
            for n in (0, 1):
                m.masknet.mamba_net.layers = layers[:n]
                t0 = time.perf_counter()
                m(mix, lips)
                ts.append(time.perf_counter() - t0)
        dt = ts[0] + kw["n_mamba"] * max(ts[1] - ts[0], 0.0)
        return {"value": round(1.0 / dt, 6), "unit": "utt/s", "cores": torch.get_num_threads(), "kind": "port",
                "sample": f"oracle/avmamba_ref fp32 forward of one 3 s utterance: front/back end {ts[0]:.2f} s + "
                          f"{kw['n_mamba']} x one BiMamba layer ({ts[1] - ts[0]:.2f} s); forward only"}


class Avse2Step:
    """avse2: time-domain AV separator, 3 s @ 16 kHz + 75 gray lip frames 224x224
    (baseline/avse2/config.py), DPRNN separator, SI-SNR loss, batch 16 (train.py:28)."""
    unit_desc = "3s@16kHz utterance + 75 lip frames 224x224"
    graph_ok = False            # MIOpen LSTM: not capturable (as avse1)

    def __init__(self, B, dev, rank, world):
        from avse_challenge_amd import avse2, data
        self.B = B
        self.model = avse2.AVSEModule().to(dev).train()
        self.lr, self.clip = self.model.lr, None
        g = torch.Generator(device=dev).manual_seed(555 + rank)
        noisy, clean, _ = data.avse1_batch(B, dev, 555 + rank, lip_hw=8)
        self.batch = {"noisy_audio": noisy, "clean": clean,
                      "video_frames": torch.rand((B, 1, 75, 224, 224), device=dev, generator=g)}

    def loss(self):
        return self.model.cal_loss(self.batch)

    def config(self, world):
        return {"workload": "avse2 AV separator train step (SURVEY 8f row 3): Swish ResNet-18 lip encoder + DPRNN "
                            "(bidirectional LSTMs, K=200) fwd/bwd + Adam", "global_batch": self.B * world,
                "per_gpu_batch": self.B, "seq_len": 48000, "lip_frames": 75, "lip_hw": 224, "parallelism": f"dp{world}"}

    def roofline(self, dev):
        return None

    def cpu_baseline(self):
        return None


class Avse4Step:
    unit_desc = "5s@16kHz binaural utterance + 125 lip frames"
    graph_ok = True

    def __init__(self, B, dev, rank, world):
        from avse_challenge_amd import avse4, data
        self.B = B
        self.model = avse4.AVSE4BaselineModule(num_channels=2).to(dev).train()
        self.lr, self.clip = self.model.lr, None
        self.batch = data.avse4_batch(B, dev, 777 + rank)

    def loss(self):
        return self.model.training_step(self.batch)

    def config(self, world):
        return {"workload": "avse4 binaural AV baseline train step (BASELINE configs[3]): ResNet18 lip encoder + "
                            "Conv-TasNet TCN (8x4 blocks, fused PReLU/gLN, depthwise dilated conv) fwd/bwd + Adam",
                "global_batch": self.B * world, "per_gpu_batch": self.B, "seq_len": 80000, "channels": 2,
                "frames": 3999, "lip_frames": 125, "lip_hw": 112, "parallelism": f"dp{world}"}

    def roofline(self, dev):
        """HBM-bound TCN kernel at the step's shape: depthwise dilated conv1d fwd on (B, 512, 3999), dil 128.
        Algorithmic bytes = read x + write y = 8 B per element."""
        from avse_challenge_amd import kernels as K
        x = torch.randn(self.B, 512, 3999, device=dev)
        w = torch.randn(512, 1, 3, device=dev)
        roof = _time_hbm(lambda: K.dwconv_fwd(x, w, 128), 8.0 * x.numel(),
                         "avse_dwconv_fwd (depthwise dilated conv1d, H=512, K=3999, dil 128)")
        return _with_traffic(roof, "dwconv") if self.B == 16 else roof

    def cpu_baseline(self):
        from oracle import avse4_ref
        torch.set_num_threads(max(1, min(len(os.sched_getaffinity(0)), 64)))
        m = avse4_ref.AVSE4BaselineModule(num_channels=2).train()
        opt = torch.optim.Adam(m.parameters(), lr=1e-4)
        g = torch.Generator().manual_seed(0)
        batch = {"noisy_audio": 0.1 * torch.randn(1, 2, 80000, generator=g),
                 "clean": 0.1 * torch.randn(1, 2, 80000, generator=g),
                 "vis_feat": torch.rand(1, 1, 125, 112, 112, generator=g)}

        def step():
            loss = m.cal_loss(batch)
            opt.zero_grad()
            loss.backward()
            opt.step()
        step()
        t0 = time.perf_counter()
        iters = 0
        while iters < 1 or (time.perf_counter() - t0 < 10.0 and iters < 4):
            step()
            iters += 1
        dt = time.perf_counter() - t0
        return {"value": round(iters / dt, 4), "unit": "utt/s", "cores": torch.get_num_threads(), "kind": "port",
                "sample": f"oracle/avse4_ref train step (fwd + bwd + Adam), batch 1, {iters} steps after 1 warm-up"}


class Trainer:
    """One training step = forward + loss + backward (+ gradient all-reduce over RCCL when N > 1)
    + optional grad-norm clip + Adam.  Gradients live in ONE flat fp32 buffer (param.grad are views):
    the data-parallel exchange is a single large all-reduce of it (ring over xGMI), and with
    --graph (default) the launch-bound forward/backward and the optimizer are each replayed as a
    captured HIP graph; the collective stays outside the graphs."""

    def __init__(self, step, world, dev, use_graph):
        self.step, self.world, self.use_graph = step, world, use_graph
        self.params = [p for p in step.model.parameters() if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(n, device=dev)
        off = 0
        for p in self.params:
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        if world > 1:                      # identical initial weights on every rank (DDP semantics)
            for p in step.model.parameters():
                dist.broadcast(p.data, 0)
            for b in step.model.buffers():
                dist.broadcast(b, 0)
        self.opt = torch.optim.Adam(self.params, lr=step.lr, capturable=use_graph, foreach=True)
        self.g_fb = self.g_opt = None
        self.loss = None

    def _fwd_bwd(self):
        self.flat.zero_()
        loss = self.step.loss()
        loss.backward()
        return loss.detach()

    def _opt(self):
        if self.world > 1:
            self.flat.mul_(1.0 / self.world)
        if self.step.clip is not None:
            torch.nn.utils.clip_grad_norm_(self.params, self.step.clip, foreach=True)
        self.opt.step()

    def _allreduce(self):
        if self.world > 1:
            dist.all_reduce(self.flat)

    def eager(self):
        self.loss = self._fwd_bwd()
        self._allreduce()
        self._opt()
        return self.loss

    def capture(self):
        """Capture after eager warm-up (lazy MIOpen / hipBLASLt / Adam-state init done)."""
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.g_fb, self.g_opt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_fb, stream=s):
                self.loss = self._fwd_bwd()
            with torch.cuda.graph(self.g_opt, stream=s):
                self._opt()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()

    def __call__(self):
        if self.g_fb is None:
            return self.eager()
        self.g_fb.replay()
        self._allreduce()
        self.g_opt.replay()
        return self.loss


def pmc_traffic(phase):
    """(bytes per launch, source) for a roofline kernel, or (None, reason) without a PMC summary."""
    try:
        with open(TRAFFIC_FILE) as f:
            rec = json.load(f)[phase]
        return rec["traffic_bytes"], f"{os.path.relpath(TRAFFIC_FILE, REPO)}[{phase}] ({rec['kernel'][:60]})"
    except (OSError, KeyError, ValueError):
        return None, "no PMC summary"


def _with_traffic(roof, phase):
    t, src = pmc_traffic(phase)
    roof["traffic"] = t
    roof["traffic_source"] = src
    return roof


def _time_hbm(fn, byts, name, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    ach = byts / (ms * 1e-3) / 1e9
    return {"kernel": name, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "avg_ms": round(ms, 4),
            "algorithmic_bytes_per_launch": byts}


def heartbeat(rank, period=60.0):
    """Progress line every minute: the first step JIT-compiles MIOpen kernels on a fresh box (minutes)."""
    import threading

    def run():
        t0 = time.time()
        while True:
            time.sleep(period)
            print(f"[bench] rank {rank} alive {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()


def main():
    args = parse()
    world, rank, dev = setup_dist()
    heartbeat(rank)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    # MIOpen immediate mode: find mode (benchmark=True, as avse1 train.py:11 sets for cuDNN) JIT-compiles
    # every candidate solver on a fresh box (minutes); immediate mode compiles only the chosen one.
    torch.backends.cudnn.benchmark = bool(int(os.environ.get("AVSE_MIOPEN_FIND", "0")))
    if args.workload == "avse1":
        B = args.batch or 32
        step = Avse1Step(B, dev, rank, world, args.lip_hw)
    elif args.workload == "avse4":
        B = args.batch or 16
        step = Avse4Step(B, dev, rank, world)
    elif args.workload == "avse2":
        B = args.batch or 16
        step = Avse2Step(B, dev, rank, world)
    elif args.workload == "avmamba":
        B = args.batch or 32
        step = AVMambaStep(B, dev, rank, world, args.size)
    elif args.workload == "dpmamba":
        B = args.batch or 32
        step = DPMambaStep(B, dev, rank, world, args.size)
    else:
        B = args.batch or 64
        step = MambaStep(B, dev, rank, world, args.size)

    work = step
    use_graph = work.graph_ok and not args.no_graph
    step = Trainer(work, world, dev, use_graph=use_graph)
    for i in range(max(args.warmup, 1 if use_graph else 0)):
        t = time.perf_counter()
        step()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] warmup {i + 1}/{args.warmup}: {time.perf_counter() - t:.2f}s", file=sys.stderr, flush=True)
    graph = False
    if use_graph:
        try:
            step.capture()
            step()
            torch.cuda.synchronize()
            graph = True
        except Exception as e:      # noqa: BLE001 - report and fall back to eager launches
            print(f"[bench] HIP graph capture failed ({type(e).__name__}: {e}); eager launches", file=sys.stderr,
                  flush=True)
            step.g_fb = step.g_opt = None
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    mark = bool(int(os.environ.get("AVSE_PROFILE_MARK", "0")))   # tools/ktrace_window.py brackets the timed steps
    if mark:
        torch.cuda._sleep(1000)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    if mark:
        torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    if not torch.isfinite(loss.detach()).all():
        raise RuntimeError("non-finite loss in the timed region")

    roof = None if args.no_roofline or rank != 0 else work.roofline(dev)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = work.cpu_baseline()
    if rank == 0:
        value = world * B * args.steps / dt
        rec = {"metric": {"avse1": METRIC, "mamba": "utterances/sec (4s@8kHz WSJ0-2mix, Mamba-TasNet)",
                          "avse4": "utterances/sec (5s@16kHz binaural + 125 lip frames, avse4)",
                          "dpmamba": "utterances/sec (4s@8kHz WSJ0-2mix, DPMamba)",
                          "avse2": "utterances/sec (3s@16kHz + 75 lip frames 224x224, avse2)",
                          "avmamba": "utterances/sec (3s@16kHz + 75 lip frames, AV Mamba-TasNet-L bf16)"}[args.workload],
               "value": round(value, 3), "unit": "utt/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": getattr(work, "dtype", "fp32"),
               "data": "synthetic (speech-like noise with 4 Hz envelope at SNR {0,3,6,9} dB, uint8 lips; "
                       "random-init weights)",
               "config": {**work.config(world), "hip_graph": graph, "max_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2)},
               "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
