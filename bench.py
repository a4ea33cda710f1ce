"""Throughput bench: utterances/s of the avse1 AV training step on MI355X (BASELINE configs[1]).

python bench.py [--gpus N --steps K --warmup W --workload avse1|mamba|avse4|avmamba|dpmamba|avse2]
One rank per GPU over RCCL: under torch.distributed.run (RANK / WORLD_SIZE in the env), or, with
--gpus N > 1 and no WORLD_SIZE, bench.py starts N ranks itself (a torch.distributed.run child
process launched before anything touches the GPU) and exits with its status. Every rank trains on
its own synthetic batch (weak scaling); gradients are all-reduced in buckets launched from autograd
hooks as they become ready, overlapping the backward, and rank 0's BatchNorm buffers are broadcast
before every forward (avse_challenge_amd/ddp.py). --device cpu (gloo) with --workload plumbing is
the CPU test hook of that distributed path.

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
import socket
import statistics
import subprocess
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
TRAFFIC_FILE = os.path.join(REPO, "profiles", "r06_traffic.json")   # tools/runs/r06ad.sh (final round-6 tree)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP32_PEAK_TFS = 157.3          # FP32 matrix (= vector) peak, spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="avse1",
                   choices=["avse1", "mamba", "avse4", "dpmamba", "avse2", "avmamba", "plumbing"])
    p.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                   help="cpu: gloo test hook of the distributed plumbing (--workload plumbing only)")
    p.add_argument("--bucket-mb", type=float, default=25.0, help="gradient all-reduce bucket size (world > 1)")
    p.add_argument("--no-roofline-hip", action="store_true", help="skip the north-star kernel roofline list")
    p.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the BASELINE config's)")
    p.add_argument("--size", default="L", choices=["XS", "S", "M", "L"], help="Mamba-TasNet / DPMamba size")
    p.add_argument("--lip-hw", type=int, default=96)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-parity", action="store_true", help="skip the output-waveform parity check vs the oracle")
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--no-graph", action="store_true", help="eager launches instead of captured HIP graphs")
    p.add_argument("--secondary", default="mamba,avse4,avmamba",
                   help="with the default avse1 workload at one rank: also time these BASELINE configs (C3 Mamba-TasNet-L "
                        "B=64, C4 avse4 B=16, C5 AV Mamba-TasNet-L bf16 B=32), each as a child bench run after the "
                        "headline's measurement, reported under 'secondary' in the same JSON line ('' = none)")
    p.add_argument("--secondary-steps", type=int, default=4)
    p.add_argument("--direction-streams", default="auto", choices=["auto", "on", "off"],
                   help="Mamba workloads: BiMamba v2's backward direction on a second HIP stream (auto: off, "
                        "the measured default)")
    return p.parse_args()


def run_secondary(args):
    """The other BASELINE configs, each in a child process (fresh device memory; a failure is reported, not raised)
    started after this process's measurement is complete; returns one record per config."""
    out = []
    for wl in [w for w in args.secondary.split(",") if w]:
        # 2 warm-up steps: the in-step roofline taps the last one, past the first step's one-time work (MIOpen's
        # first-call solver selection ran its naive fallback kernels there: 0.5 s per C4 / C5 step, r06i profiles)
        cmd = [sys.executable, os.path.abspath(__file__), "--workload", wl, "--steps", str(args.secondary_steps),
               "--warmup", "2", "--secondary", "", "--no-cpu-baseline", "--no-roofline-hip"]
        t = time.perf_counter()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not lines:
                out.append({"workload": wl, "error": f"rc {r.returncode}: {r.stderr[-400:]}"})
                continue
            rec = json.loads(lines[-1])
            keep = {k: rec.get(k) for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "dtype")}
            keep["config"] = {k: rec["config"].get(k) for k in ("workload", "global_batch", "hip_graph", "max_mem_gb")
                              if k in rec["config"]}
            keep["roofline"] = rec.get("roofline")
            keep["parity"] = rec.get("parity")
            keep["wall_s"] = round(time.perf_counter() - t, 1)
            out.append({"workload": wl, **keep})
        except Exception as e:      # noqa: BLE001 - the headline line must still print
            out.append({"workload": wl, "error": f"{type(e).__name__}: {e}"})
        print(f"[bench] secondary {wl}: {out[-1].get('value', out[-1].get('error'))}", file=sys.stderr, flush=True)
    return out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args):
    """--gpus N > 1 without a launcher: start N ranks via torch.distributed.run as a CHILD process (this process
    has not touched the GPU) and return its exit status; rank 0 of the child prints the JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")       # dmabuf IPC for RCCL on this driver
    return subprocess.call(cmd, env=env)


def setup_dist(device):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if device == "cpu":
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
        return world, rank, dev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    return world, rank, dev


def sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def barrier(world):
    if world > 1:
        dist.barrier()


# ------------------------------------------------------------------------------ parity (the CPU-baseline leg's checker)

def _wave_parity(est, ref, clean, n_utt, what):
    """North-star parity of output WAVEFORMS (BASELINE.json: "within 1e-4 RMS waveform error (SI-SDR within 0.01 dB)"):
    est (GPU path) / ref (fp64 CPU oracle) / clean: (..., T).  RMS(est - ref) against the bar 1e-4 * max(1, RMS(ref)),
    and |SI-SDR(clean, est) - SI-SDR(clean, ref)| per utterance (channel, speaker)."""
    from oracle.losses_ref import si_sdr_db
    est, ref, clean = est.double().cpu(), ref.double().cpu(), clean.double().cpu()
    rms = float((est - ref).pow(2).mean().sqrt())
    bar = 1e-4 * max(1.0, float(ref.pow(2).mean().sqrt()))
    s_est, s_ref = si_sdr_db(clean, est), si_sdr_db(clean, ref)
    d = float((s_est - s_ref).abs().max())
    return {"what": what, "utterances": n_utt, "rms": float(f"{rms:.3e}"), "rms_bar": float(f"{bar:.1e}"),
            "dsisdr_db": float(f"{d:.3e}"), "si_sdr_db": [round(v, 3) for v in s_est.flatten().tolist()],
            "ok": bool(rms <= bar and d <= 0.01)}


def _oracle_from(model, ref):
    """The fp64 oracle module ``ref`` with the product model's current weights and buffers (identical state_dict
    keys, tests/test_ckpt_io.py), in the product model's train / eval mode."""
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    return ref.double().train(model.training)


def _avse1_oracle_enhance(ref, noisy, lips):
    """test.py:79-89 on the oracle: librosa-0.8.1 STFT (numpy) -> AVNet (fp64) -> iSTFT with the noisy phase."""
    import numpy as np
    from oracle import stft_ref
    spec = stft_ref.stft(noisy.numpy())
    mag_t = np.swapaxes(np.abs(spec), -1, -2).astype(np.float32)              # dataset.py:112-118
    inp = {"noisy_audio_spec": torch.from_numpy(mag_t).double()[:, None]}
    if lips is not None:
        inp["lip_images"] = lips
    with torch.no_grad():
        pred = ref(inp)[:, 0]
    phase = np.angle(spec)
    est = np.swapaxes(pred.numpy(), -1, -2) * (np.cos(phase) + 1j * np.sin(phase))
    return torch.from_numpy(stft_ref.istft(est, length=noisy.shape[-1]))


def _parity_leg(fn):
    """Run a workload's parity check (eval mode, no grad) and restore the model's mode; a failure is reported."""
    def wrapped(self, dev):
        was = self.model.training
        t = time.perf_counter()
        try:
            self.model.eval()
            with torch.no_grad():
                rec = fn(self, dev)
            rec["wall_s"] = round(time.perf_counter() - t, 1)
            return rec
        except Exception as e:      # noqa: BLE001 - the bench line must still print
            return {"error": f"{type(e).__name__}: {e}"}
        finally:
            self.model.train(was)
            torch.cuda.empty_cache()
    return wrapped



# ------------------------------------------------------------------------------ workloads

class Avse1Step:
    unit_desc = "3s@16kHz utterance + 75 lip frames"
    # the FusionNet LSTM is the HIP recurrence (layers.HipLSTM), so the whole step captures as HIP graphs
    graph_ok = True

    def __init__(self, B, dev, rank, world, lip_hw):
        from avse_challenge_amd import avse1, data
        self.B, self.lip_hw = B, lip_hw
        self.model = avse1.AVNet().to(dev).train()
        # channels-last audio net and lip trunk: the layouts of the split-fp16 conv kernels (dconv.hip, sconv.hip)
        self.model.net_audiofeat.use_channels_last()
        self.model.net_visualfeat.use_channels_last()
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
        """Dominant hand-written kernel class of the step: the AudioFeatNet 64->64 5x5 dilated Conv2d (conv2..5, d = 2,
        4, 8, 16).  With the split-fp16 path (csrc/dconv.hip, default) its forward + input-gradient launches
        (avse_dconv_fwd, 8 per step) and its weight gradient (avse_dconv_wgrad16, 4 per step); otherwise the fp32-MFMA
        weight gradient (avse_dconv_wgrad).  Algorithmic FLOPs per launch = 2*B*64*64*25*376*257 (fp32 math); the split
        kernels run 3 f16 MFMAs per fp32 product, so their peak is the dense f16 peak / 3 (833 TFLOP/s), the fp32-MFMA
        kernel's the fp32 peak (157.3).
          * ``achieved`` / ``frac`` / ``avg_ms``: IN-STEP, AS THE TIMED STEPS RUN — every launch inside 3 eager train
            steps of the benchmarked model with the lip branch on its side stream (the timed schedule), each bracketed
            by HIP events on its launch stream (kernels.LAUNCH_TAPS): a launch's event time is its duration while it
            shares the CUs with the lip branch (the rocprofv3 timed window, profiles/*_avse1_timed_window_stats.csv,
            shows the same per-launch average); ``roofline`` is the entry point with the most kernel time in them;
          * ``in_step_serial``: the same with the lip branch on the launch stream for 3 more steps (a launch's event
            time is then its kernel time alone on the GPU); AVSE_PROFILE_MARK=1 brackets these steps (the rocprof window
            that must agree);
          * ``isolated``: conv3's launch (d = 4) alone on the idle GPU, random operands of the step's shape;
          * ``roofline_library``: the MIOpen forward of the same conv, alone."""
        from avse_challenge_amd import kernels as K
        from avse_challenge_amd import layers
        cl = torch.channels_last
        flops = 2.0 * self.B * 64 * 64 * 25 * 376 * 257
        names = ("avse_dconv_fwd", "avse_dconv_wgrad16")
        peak = BF16_PEAK_TFS / 3
        mark = os.environ.get("AVSE_PROFILE_MARK", "0") == "1"        # tools/ktrace_window.py OUT_ROOF.csv

        def taps(serial):
            for n in names:
                K.LAUNCH_TAPS[n] = []
            old = self.avse1.set_branch_streams(not serial)         # serial: the lip branch on the launch stream
            try:
                if mark and serial:
                    torch.cuda._sleep(1000)
                for _ in range(3):
                    self.loss().backward()
                if mark and serial:
                    torch.cuda._sleep(1000)
                torch.cuda.synchronize()
                return {n: [a.elapsed_time(b) for a, b in K.LAUNCH_TAPS[n]] for n in names}
            finally:
                for n in names:
                    K.LAUNCH_TAPS.pop(n, None)
                self.avse1.set_branch_streams(old)
        per2 = taps(False)
        per = taps(True)
        x = torch.randn(self.B, 64, 376, 257, device=dev).contiguous(memory_format=cl)
        dy = torch.randn(self.B, 64, 376, 257, device=dev).contiguous(memory_format=cl)
        w = 0.05 * torch.randn(64, 64, 5, 5, device=dev)
        recs = []
        for n in names:
            v, vs = per2[n], per[n]                   # two streams (the timed schedule), serial
            if not v:
                continue
            ms_in = sum(v) / len(v)
            ach_in = flops / (ms_in * 1e-3) / 1e12
            if n == "avse_dconv_fwd":
                mb = torch.empty(2, device=dev, dtype=torch.int32)
                xq = K.split16(x, mb)
                wq = K.dconv_wprep(w, False, mb)
                y = torch.empty_like(x)
                L = K._lib.lib()
                iso = lambda: K.check(L.avse_dconv_fwd(self.B, 376, 257, 4, K.ptr(xq), K.ptr(wq), K.ptr(mb), None,  # noqa: E731
                                                       K.ptr(y), K.stream_ptr(dev)), "avse_dconv_fwd")
                desc = ("avse_dconv_fwd (AudioFeatNet conv2..5 forward and input gradient: Conv2d 64->64 5x5 dil "
                        "2/4/8/16 as a split-fp16 MFMA implicit GEMM, fp32-accurate)")
            else:
                xm, dm = torch.empty(2, device=dev, dtype=torch.int32), torch.empty(2, device=dev, dtype=torch.int32)
                xq, dq = K.split16(x, xm), K.split16(dy, dm)
                iso = lambda: K.dconv_wgrad16((xq, xm[:1]), (dq, dm[:1]), tuple(x.shape), 4)  # noqa: E731
                desc = "avse_dconv_wgrad16 (AudioFeatNet conv2..5 weight gradient, split-fp16 MFMA implicit GEMM)"
            ms = _event_ms(iso, n=10, warm=3)
            ach = flops / (ms * 1e-3) / 1e12
            vs = vs or [float("nan")]
            ms_s = sum(vs) / len(vs)
            recs.append({"kernel": desc, "bound": "mfma", "achieved": round(ach_in, 2), "peak": round(peak, 1),
                         "unit": "TFLOP/s", "frac": round(ach_in / peak, 4), "traffic": None, "avg_ms": round(ms_in, 4),
                         "launches": len(v), "step_ms": round(sum(v) / 3, 3),
                         "measured": f"in-step, timed schedule: {len(v)} launches in 3 eager train steps of the "
                                     "benchmarked model with the lip branch on its side stream, HIP events on the "
                                     "launch stream",
                         "in_step_serial": {"avg_ms": round(ms_s, 4),
                                            "frac": round(flops / (ms_s * 1e-3) / 1e12 / peak, 4),
                                            "note": "lip branch on the launch stream (3 more eager steps): the launch "
                                                    "alone on the GPU"},
                         "per_launch_ms": [round(t, 3) for t in v[:4]], "algorithmic_flops_per_launch": flops,
                         "isolated": {"what": "conv3 (d = 4) alone on the idle GPU", "avg_ms": round(ms, 4),
                                      "achieved": round(ach, 2), "frac": round(ach / peak, 4)}})
        if not recs:
            return None
        roof = dict(max(recs, key=lambda r: r["step_ms"]))
        roof["peak_note"] = ("split-fp16 kernels: 3 f16 MFMAs per fp32 product, peak = dense f16 2500 TFLOP/s / 3; "
                             "achieved counts the fp32 algorithmic FLOPs")
        roof["other_conv_kernels"] = [{k: r[k] for k in ("kernel", "avg_ms", "achieved", "frac", "launches",
                                                         "step_ms")} for r in recs if r is not roof]
        _with_traffic(roof, "-")
        conv = self.model.net_audiofeat.conv3
        with torch.no_grad(), _dconv_library():
            ms_f = _event_ms(lambda: conv(x), n=10, warm=3)
        ach_f = flops / (ms_f * 1e-3) / 1e12
        roof["roofline_library"] = {"kernel": "AudioFeatNet.conv3 fwd (MIOpen), alone", "achieved": round(ach_f, 2),
                                    "frac_fp32": round(ach_f / FP32_PEAK_TFS, 4), "avg_ms": round(ms_f, 4)}
        return roof

    def cpu_baseline(self):
        """the oracle's full train step (numpy librosa-0.8.1 STFT + AVNet fwd + bwd + Adam) on the
        same synthetic inputs, batch min(32, 4) = 4, 1 warm-up + median of 5."""
        from avse_challenge_amd import data
        from oracle import avse1_ref, stft_ref
        _cpu_threads()
        B = 4
        m = avse1_ref.AVNet().train()
        opt = torch.optim.Adam(m.parameters(), lr=self.lr)
        noisy, clean, lips = data.avse1_batch(B, "cpu", 1234, self.lip_hw)

        def step():
            batch = {"noisy_audio_spec": torch.from_numpy(stft_ref.stft_mag_T(noisy.numpy()))[:, None],
                     "mask": torch.from_numpy(stft_ref.stft_mag_T(clean.numpy()))[:, None], "lip_images": lips}
            _cpu_train_step(m, opt, m.cal_loss(batch))
        return _cpu_record(step, B, 1.0, f"oracle/avse1_ref AVNet train step (numpy librosa-0.8.1 STFT + fwd + bwd + "
                                         f"Adam), batch {B}, lips {self.lip_hw}x{self.lip_hw}")


    @_parity_leg
    def parity(self, dev):
        """C2 (and C1): the benchmarked model's enhanced waveforms (HIP STFT -> AVNet in eval mode -> HIP iSTFT with
        the noisy phase, test.py:79-89) on the batch's first 2 utterances vs the fp64 CPU oracle with the same weights
        and buffers; C1 (BASELINE configs[0]): the audio-only AVNet (model.py:117-118, det-init weights) on the first
        utterance, the same comparison."""
        from avse_challenge_amd import avse1
        from oracle import avse1_ref
        from oracle.det_init import det_init_
        _cpu_threads()
        P = min(2, self.B)
        noisy, clean, lips = self.noisy[:P], self.clean[:P], self.lips[:P]
        est = self.model.enhance(noisy, lips)
        ref = _avse1_oracle_enhance(_oracle_from(self.model, avse1_ref.AVNet()), noisy.cpu(), lips.cpu())
        out = {"c2": _wave_parity(est, ref, clean, P, "avse1 AV enhance (trained bench weights, eval) vs fp64 oracle")}
        net = det_init_(avse1.AVNet(a_only=True), 74).to(dev).eval()
        est1 = net.enhance(self.noisy[:1], None)
        ref1 = _avse1_oracle_enhance(_oracle_from(net, avse1_ref.AVNet(a_only=True)), self.noisy[:1].cpu(), None)
        out["c1"] = _wave_parity(est1, ref1, self.clean[:1], 1, "avse1 audio-only enhance (det-init, eval) vs fp64 "
                                                                "oracle")
        return out


DIRECTION_STREAMS_ARG = "auto"     # --direction-streams


def _apply_direction_streams(work):
    """--direction-streams on / off overrides the workload's default (auto)."""
    from avse_challenge_amd import mamba_tasnet
    if DIRECTION_STREAMS_ARG != "auto":
        work.direction_streams = DIRECTION_STREAMS_ARG == "on"
        mamba_tasnet.set_direction_streams(work.direction_streams)


class MambaStep:
    unit_desc = "4s@8kHz WSJ0-2mix utterance"
    graph_ok = True

    def __init__(self, B, dev, rank, world, size):
        from avse_challenge_amd import data, losses, mamba_tasnet
        self.B, self.size = B, size
        # the v2 backward direction on a second stream (mamba_tasnet._direction_stream) needs record_stream on the
        # shared xz, and blocks with pending stream uses are not reusable inside a graph capture: at B >= 48 the
        # captured Mamba-TasNet-L step then exceeds 288 GB, so large batches run both directions on one stream
        # (measured at B=64: captured 1 stream 1402 ms/step; eager at ~200 GB allocator churn 6993 ms/step)
        # the two BiMamba directions serially on one stream (mamba_tasnet.DIRECTION_STREAMS): at B >= 48 the side
        # stream's pending record_stream uses would also keep blocks out of the graph pool (the captured C3 step then
        # exceeds 288 GB); --direction-streams on runs the side stream where it fits
        self.direction_streams = False
        mamba_tasnet.set_direction_streams(False)
        _apply_direction_streams(self)
        if self.direction_streams and B >= 48:
            raise SystemExit("--direction-streams on needs B < 48 (the captured step's memory, see above)")
        self.model = mamba_tasnet.MambaTasNet(**mamba_tasnet.MAMBA_TASNET_SIZES[size]).to(dev).train()
        self.lr, self.clip = 1.5e-4, 5.0
        self.mix, self.tgt = data.wsj0mix_batch(B, dev, 4321 + rank)
        self.losses = losses

    def loss(self):
        return self.losses.si_snr_pit(self.tgt, self.model(self.mix)).mean()

    def config(self, world):
        return {"workload": f"Mamba-TasNet-{self.size} train step (BASELINE configs[2])", "global_batch": self.B * world,
                "per_gpu_batch": self.B, "seq_len": 32000, "frames": 3999, "parallelism": f"dp{world}",
                "direction_streams": self.direction_streams}

    # the step's dominant hand-written kernels (rocprofv3 window: the scan backward, then the forward)
    tap_kernels = ("avse_scan_bwd", "avse_scan_fwd")
    scan_dtype, scan_len = torch.float32, 3999

    def roofline(self, dev):
        """In-step figure of the step's dominant kernel, the selective-scan backward (main._in_step_hbm): bytes as
        MambaInnerNoOutProj calls it (u, delta, z, dout, B, C read; du, ddelta, dz and fp32 dB, dC written); the
        forward's in-step figure and each kernel's isolated launch at the step's shape beside it."""
        d = 2 * self.model.masknet.mamba_net.layers[0].mixer.d_model
        b, l = self.B, self.scan_len
        s = 2 if self.scan_dtype == torch.bfloat16 else 4
        bwd = b * l * (7 * s * d + 2 * s * 16 + 2 * 4 * 16)
        fwd = s * b * l * (4 * d + 2 * 16)
        tag = "bf16" if s == 2 else "fp32"
        roof = _in_step_hbm(self, "avse_scan_bwd", bwd, f"avse_scan_bwd (selective scan backward, {tag}, "
                            f"{b} x {d} x {l}; entry point: main kernel + dB/dC and dA/dD/dbias reductions)")
        f = _in_step_hbm(self, "avse_scan_fwd", fwd, f"avse_scan_fwd (training fwd, {tag}, out_z + checkpoints)")
        if roof is None:
            return None
        roof["in_step_fwd"] = {k: f[k] for k in ("avg_ms", "achieved", "frac", "launches")} if f else None
        return roof

    def cpu_baseline(self):
        """The oracle's full train step (every BiMamba layer, PIT SI-SNR, bwd, Adam), 1 warm-up + median of 3 — on
        ONE utterance cut to 1/32 of its length (1000 samples, L = 124 frames): the oracle's scan is a Python loop
        over frames (its train step at batch 4 x 2000 samples took 84-100 s on 8 cores), so the step time, linear
        in L, is scaled x32 to the 4 s utterance. Deviates from BASELINE.md §4's batch 4 / median of 5 to stay a
        bounded sample (~30 s)."""
        from avse_challenge_amd import data
        from oracle import losses_ref, mamba_ref
        _cpu_threads()
        B, cut = 1, 32
        m = mamba_ref.MambaTasNet(**mamba_ref.MAMBA_TASNET_SIZES[self.size], n_spk=2).train()
        opt = torch.optim.Adam(m.parameters(), lr=self.lr)
        mix, tgt = data.wsj0mix_batch(B, "cpu", 4321, T=32000 // cut)

        def step():
            _cpu_train_step(m, opt, losses_ref.si_snr_pit(tgt, m(mix)).mean(), self.clip)
        return _cpu_record(step, B, cut, f"oracle/mamba_ref Mamba-TasNet-{self.size} train step (all layers, PIT "
                                         f"SI-SNR, bwd, Adam), batch {B} x {32000 // cut} samples (1/{cut} of 4 s), "
                                         f"time scaled x{cut}", runs=3)


    @_parity_leg
    def parity(self, dev):
        """C3: the benchmarked separator (eval) on the batch's first 4 s mixture vs the fp64 CPU oracle with the same
        weights; per speaker in the model's own output order (same weights: no PIT needed)."""
        from oracle import mamba_ref
        _cpu_threads()
        mix, tgt = self.mix[:1], self.tgt[:1]
        est = self.model(mix)                                        # (1, T, n_spk)
        ref = _oracle_from(self.model, mamba_ref.MambaTasNet(**mamba_ref.MAMBA_TASNET_SIZES[self.size], n_spk=2))
        est_r = ref(mix.double().cpu())
        return {"c3": _wave_parity(est.transpose(1, 2), est_r.transpose(1, 2), tgt.transpose(1, 2), 1,
                                   f"Mamba-TasNet-{self.size} separation (trained bench weights, eval) vs fp64 oracle")}


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

    parity = None

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
        """The oracle's full train step on one 4 s utterance with 1 and with 2 of the n dual-path layers (1 warm-up +
        median of 3 each), the per-layer time (2-layer step minus 1-layer step) scaled to all n layers."""
        from avse_challenge_amd import data
        from oracle import dpmamba_ref, losses_ref
        _cpu_threads()
        B = 1
        kw = dict(dpmamba_ref.DPMAMBA_SIZES[self.size])
        n_dp = kw.pop("n_dp")
        mix, tgt = data.wsj0mix_batch(B, "cpu", 4321)
        recs = []
        for n in (1, 2):
            m = dpmamba_ref.DPMambaTasNet(n_dp=n, **kw).train()
            opt = torch.optim.Adam(m.parameters(), lr=self.lr)

            def step():
                _cpu_train_step(m, opt, losses_ref.si_snr_pit(tgt, m(mix)).mean(), self.clip)
            recs.append(_cpu_record(step, B, 1.0, "", runs=3))
        t1, t2 = (B / r["value"] for r in recs)
        dt = t1 + (n_dp - 1) * max(t2 - t1, 0.0)
        rec = recs[1]
        rec.update(value=round(B / dt, 6), sample=f"oracle/dpmamba_ref DPMamba-{self.size} train step (PIT SI-SNR, "
                   f"bwd, Adam), batch {B} x 4 s: 1-layer {t1:.2f} s, 2-layer {t2:.2f} s (median of 3 each), "
                   f"extrapolated to {n_dp} dual-path layers")
        return rec


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
        self.model.visual_frontend.use_channels_last()
        from avse_challenge_amd import mamba_tasnet
        self.direction_streams = False                         # C5 B=32: 552.5 vs 571.7 ms/step with the side stream
        mamba_tasnet.set_direction_streams(False)
        _apply_direction_streams(self)         # NHWC lip ResNet: 3x3 convs on csrc/sconv.hip
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
                "lip_frames": 75, "lip_hw": 112, "parallelism": f"dp{world}", "direction_streams": self.direction_streams}

    tap_kernels = ("avse_scan_bwd", "avse_scan_fwd")
    scan_dtype, scan_len = torch.bfloat16, 5999
    roofline = MambaStep.roofline

    def cpu_baseline(self):
        """The oracle's full fp32 train step (lip encoder + all BiMamba layers, SI-SNR, bwd, Adam), 1 warm-up + median
        of 3, on ONE utterance cut to 1/32 with its lip track (1500 samples, L = 186 frames, 3 lip frames), the step
        time scaled x32 to the 3 s utterance (linear in length: the oracle's scan is a Python loop over frames, the
        lip encoder is per frame). A bounded sample (~30 s), not BASELINE.md §4's batch 4 / median of 5."""
        from avse_challenge_amd import data
        from oracle import avmamba_ref
        from oracle.losses_ref import avse4_loss
        _cpu_threads()
        B, cut = 1, 32
        m = avmamba_ref.AVMambaTasNet(**avmamba_ref.AV_MAMBA_SIZES[self.size]).train()
        opt = torch.optim.Adam(m.parameters(), lr=self.lr)
        noisy, clean, _ = data.avse1_batch(B, "cpu", 999, lip_hw=8, T=48000 // cut)
        lips = torch.rand((B, 1, 75 // cut + 1, 112, 112), generator=torch.Generator().manual_seed(999))

        def step():
            _cpu_train_step(m, opt, avse4_loss(clean[:, None], m(noisy, lips)[:, None]), self.clip)
        return _cpu_record(step, B, cut, f"oracle/avmamba_ref AV Mamba-TasNet-{self.size} fp32 train step, batch {B} x "
                                         f"{48000 // cut} samples + {75 // cut + 1} lip frames (1/{cut} of 3 s), time "
                                         f"scaled x{cut}", runs=3)


    @_parity_leg
    def parity(self, dev):
        """C5 has no reference model: the assembly of reference components (oracle/avmamba_ref.py) is the
        checker.  The benchmarked model (eval) on the first utterance with its lip track, in fp32 (autocast off: the
        kernels' parity) vs the fp64 oracle with the same weights; the bf16-autocast output's SI-SDR vs the same oracle
        beside it (bf16 keeps 8 mantissa bits: the precision choice of the config, not a parity claim)."""
        from oracle import avmamba_ref
        from oracle.losses_ref import si_sdr_db
        _cpu_threads()
        noisy, clean, vis = self.batch["noisy_audio"][:1], self.batch["clean"][:1], self.batch["vis_feat"][:1]
        est = self.model(noisy, vis)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            est16 = self.model(noisy, vis).float()
        ref = _oracle_from(self.model, avmamba_ref.AVMambaTasNet(**avmamba_ref.AV_MAMBA_SIZES[self.size]))
        est_r = ref(noisy.double().cpu(), vis.double().cpu())
        rec = _wave_parity(est, est_r, clean, 1, f"AV Mamba-TasNet-{self.size} (trained bench weights, eval, fp32 "
                                                 "kernels) vs fp64 oracle assembly")
        c = clean.double().cpu()
        d16 = (si_sdr_db(c, est16.double().cpu()) - si_sdr_db(c, est_r)).abs().max()
        rec["bf16_autocast"] = {"rms": float(f"{float((est16.double().cpu() - est_r).pow(2).mean().sqrt()):.3e}"),
                                "dsisdr_db": float(f"{float(d16):.3e}")}
        return {"c5": rec}


class Avse2Step:
    """avse2: time-domain AV separator, 3 s @ 16 kHz + 75 gray lip frames 224x224
    (baseline/avse2/config.py), DPRNN separator, SI-SNR loss, batch 16 (train.py:28)."""
    unit_desc = "3s@16kHz utterance + 75 lip frames 224x224"
    graph_ok = True             # DPRNN LSTMs on the HIP recurrence (layers.HipLSTM)

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

    parity = None


class Avse4Step:
    unit_desc = "5s@16kHz binaural utterance + 125 lip frames"
    graph_ok = True

    def __init__(self, B, dev, rank, world):
        from avse_challenge_amd import avse4, data
        self.B = B
        self.model = avse4.AVSE4BaselineModule(num_channels=2).to(dev).train()
        self.model.visual_frontend.use_channels_last()         # NHWC lip ResNet: 3x3 convs on csrc/sconv.hip
        self.lr, self.clip = self.model.lr, None
        self.batch = data.avse4_batch(B, dev, 777 + rank)

    def loss(self):
        return self.model.training_step(self.batch)

    def config(self, world):
        return {"workload": "avse4 binaural AV baseline train step (BASELINE configs[3]): ResNet18 lip encoder + "
                            "Conv-TasNet TCN (8x4 blocks, fused PReLU/gLN, depthwise dilated conv) fwd/bwd + Adam",
                "global_batch": self.B * world, "per_gpu_batch": self.B, "seq_len": 80000, "channels": 2,
                "frames": 3999, "lip_frames": 125, "lip_hw": 112, "parallelism": f"dp{world}"}

    # the TCN's hand-written kernels (32 TemporalBlocks: fused dwconv -> PReLU -> gLN and PReLU -> gLN, each way) and
    # the split-fp16 GEMM of its 1x1 convs (forward, input and weight gradients: the step's most kernel time)
    tap_kernels = ("avse_dwconv_gln_bwd", "avse_dwconv_gln_fwd", "avse_prelu_gln_bwd", "avse_prelu_gln_fwd",
                   "avse_gemm_f32s")

    def roofline(self, dev):
        """In-step figures of the TCN's hand-written kernels (main._in_step_hbm) on (B, 512, 3999): algorithmic bytes
        per element dwconv_gln fwd 12 (x read, y1 + y written), bwd 16 (x, y1, dy read, dx written), prelu_gln fwd 8,
        bwd 12; and of every avse_gemm_f32s launch of the step (the 1x1 convs 256 <-> 512 and the bottleneck / mask
        convs, forward + both gradients): the launches' fp32 algorithmic FLOPs (2 M N K each) over their summed
        HIP-event time against the split peak.  ``roofline`` is the one with the most kernel time in the step (the
        GEMM); the TCN kernels are listed beside it."""
        ne = self.B * 512 * 3999
        recs = []
        for name, bpe, desc in (("avse_dwconv_gln_bwd", 16, "fused dwconv <- PReLU <- gLN backward"),
                                ("avse_dwconv_gln_fwd", 12, "fused dwconv -> PReLU -> gLN forward"),
                                ("avse_prelu_gln_bwd", 12, "PReLU <- gLN backward (after the 1x1 conv)"),
                                ("avse_prelu_gln_fwd", 8, "PReLU -> gLN forward (after the 1x1 conv)")):
            r = _in_step_hbm(self, name, bpe * ne, f"{name} ({desc}, {self.B} x 512 x 3999)")
            if r is not None:
                recs.append(r)
        if not recs:
            return None
        tcn = [{k: r[k] for k in ("kernel", "avg_ms", "achieved", "frac", "launches", "step_ms")} for r in recs]
        gemm = _in_step_flops(self, "avse_gemm_f32s", round(BF16_PEAK_TFS / 3, 1),
                              "avse_gemm_f32s (TCN 1x1 convs and the bottleneck / mask convs on the split-fp16 GEMM: "
                              "forward, input and weight gradients)")
        top = max(recs + ([gemm] if gemm else []), key=lambda r: r["step_ms"])
        roof = dict(top)
        roof["tcn_kernels"] = tcn
        if gemm is not None and top is not gemm:
            roof["gemm"] = gemm
        return roof

    def cpu_baseline(self):
        """the oracle's train step (fwd + SI-SNR + bwd + Adam) on the same synthetic inputs,
        batch min(16, 4) = 4 binaural 5 s utterances + 125 lip frames, 1 warm-up + median of 5."""
        from avse_challenge_amd import data
        from oracle import avse4_ref
        _cpu_threads()
        B = 4
        m = avse4_ref.AVSE4BaselineModule(num_channels=2).train()
        opt = torch.optim.Adam(m.parameters(), lr=self.lr)
        batch = data.avse4_batch(B, "cpu", 777)

        def step():
            _cpu_train_step(m, opt, m.cal_loss(batch))
        return _cpu_record(step, B, 1.0, f"oracle/avse4_ref train step (fwd + bwd + Adam), batch {B} x 2 ch x 5 s "
                                         f"+ 125 lip frames 112x112")


    @_parity_leg
    def parity(self, dev):
        """C4: the benchmarked model (eval) on the batch's first binaural utterance + lip track vs the fp64 oracle with
        the same weights and buffers (forward() casts to fp32, model.py:316-321: the oracle's parts are called in
        fp64)."""
        from oracle import avse4_ref
        _cpu_threads()
        b1 = {k: v[:1] for k, v in self.batch.items()}
        est = self.model(b1)
        r = _oracle_from(self.model, avse4_ref.AVSE4BaselineModule(num_channels=2))
        ref = r.model(b1["noisy_audio"].double().cpu(), r.visual_frontend(b1["vis_feat"].double().cpu()))
        return {"c4": _wave_parity(est, ref, b1["clean"], 1, "avse4 binaural enhancement (trained bench weights, "
                                                             "eval) vs fp64 oracle")}


from avse_challenge_amd.ddp import Trainer  # noqa: E402  (the data-parallel step; re-exported for tests)


class _PlumbingNet(torch.nn.Module):
    """avse1 AudioFeatNet's module tree (bn0, 5 dilated 5x5 Conv2d + BatchNorm2d + ReLU, 1x1 -> 4) in stock
    PyTorch ops: the product's version runs its BatchNorms on the HIP kernels, which the CPU test cannot."""

    def __init__(self, filters=64, k=5):
        super().__init__()
        self.bn0 = torch.nn.BatchNorm2d(1)
        for i in range(5):
            dil = 2 ** i
            setattr(self, f"conv{i + 1}", torch.nn.Conv2d(1 if i == 0 else filters, filters, k,
                                                          padding=(k - 1) * dil // 2, dilation=dil))
            setattr(self, f"bn{i + 1}", torch.nn.BatchNorm2d(filters))
        self.convf = torch.nn.Conv2d(filters, 4, 1)
        self.bn_last = torch.nn.BatchNorm2d(4)

    def forward(self, spec):
        T, Fb = spec.shape[2], spec.shape[3]
        x = self.bn0(spec)
        for i in range(1, 6):
            x = torch.relu(getattr(self, f"bn{i}")(getattr(self, f"conv{i}")(x)))
        x = torch.relu(self.bn_last(self.convf(x)))
        return x.permute(0, 2, 1, 3).reshape(-1, T, Fb * 4)


class PlumbingStep:
    """--device cpu test hook of the distributed path (launch, bucketed all-reduce, BatchNorm-buffer broadcast,
    max-over-ranks timing) under gloo: an AudioFeatNet-shaped net (dilated Conv2d + BatchNorm2d) on a reduced
    spectrogram (B x 1 x 40 x 257) + a 1028 -> 257 sigmoid mask head, L1 loss.  Not a throughput workload."""
    unit_desc = "reduced spectrogram (plumbing test)"
    graph_ok = False

    def __init__(self, B, dev, rank, world):
        torch.manual_seed(5 + rank)                   # different init per rank: the Trainer broadcasts rank 0's
        self.B = B
        self.model = torch.nn.ModuleDict({"net": _PlumbingNet(), "head": torch.nn.Linear(1028, 257)}).to(dev)
        self.lr, self.clip = 1e-3, 1.0
        g = torch.Generator().manual_seed(300 + rank)
        self.spec = torch.rand((B, 1, 40, 257), generator=g).to(dev)
        self.target = torch.rand((B, 1, 40, 257), generator=g).to(dev)

    def loss(self):
        mask = torch.sigmoid(self.model["head"](self.model["net"](self.spec)))
        return torch.nn.functional.l1_loss(self.spec * mask[:, None], self.target)

    def config(self, world):
        return {"workload": "plumbing (CPU test hook of the data-parallel path)", "global_batch": self.B * world,
                "per_gpu_batch": self.B, "parallelism": f"dp{world}"}

    def roofline(self, dev):
        return None

    def cpu_baseline(self):
        return None

    parity = None


# ------------------------------------------------------------------------------ CPU baseline helpers

def _cpu_threads():
    """The host cores this process may use: OMP_NUM_THREADS when the launcher sets it (the GPU box sets the
    box's CPU share there; affinity / cpu_count show the whole machine), else the affinity mask."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    torch.set_num_threads(max(1, n))


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_train_step(m, opt, loss, clip=None):
    opt.zero_grad(set_to_none=True)
    loss.backward()
    if clip is not None:
        torch.nn.utils.clip_grad_norm_(m.parameters(), clip)
    opt.step()


def _cpu_record(step, batch, scale, sample, runs=5):
    """1 warm-up + median of ``runs`` timed steps; utt/s = batch / (median * scale)."""
    step()
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    return {"value": round(batch / (med * scale), 6), "unit": "utt/s", "cores": torch.get_num_threads(),
            "cpu_model": _cpu_model(), "kind": "port", "sample": sample,
            "step_s": [round(t, 3) for t in ts], "median_step_s": round(med, 3), "time_scale": scale}


def pmc_traffic(phase):
    """(bytes per launch, source) for a roofline kernel, or (None, reason) without a PMC summary."""
    try:
        with open(TRAFFIC_FILE) as f:
            rec = json.load(f)[phase]
        return rec["traffic_bytes"], f"{os.path.relpath(TRAFFIC_FILE, REPO)}[{phase}] ({rec['kernel'][:60]})"
    except (OSError, KeyError, ValueError):
        return None, "no PMC summary"


def pmc_valu_busy(fname, kernel_prefix):
    """(VALU-busy share of SIMD cycles, source) of a scan kernel from a committed tools/pmc_scan.sh summary: the
    scan kernels are VALU-throughput bound, so this is their compute-roofline fraction."""
    path = os.path.join(REPO, "profiles", fname)
    try:
        lines = open(path).read().split("\n")
    except OSError:
        return None, "no PMC summary"
    for i, ln in enumerate(lines):
        if ln.startswith(kernel_prefix):
            for nxt in lines[i + 1:i + 4]:
                if "VALU busy" in nxt:
                    return float(nxt.split("VALU busy")[1].split()[0]), f"profiles/{fname} ({kernel_prefix[:48]})"
    return None, "kernel not in PMC summary"


def _with_traffic(roof, phase):
    t, src = pmc_traffic(phase)
    roof["traffic"] = t
    roof["traffic_source"] = src
    return roof


def _in_step_hbm(work, name, byts, desc, isolated=None, traffic_phase=None):
    """roofline record of one tapped entry point from the last eager warm-up step (main: ``tap_kernels``): algorithmic
    bytes per launch over the mean HIP-event duration of its launches in the step."""
    per = getattr(work, "step_taps", {}).get(name) or []
    if not per:
        return None
    ms = sum(per) / len(per)
    ach = byts / (ms * 1e-3) / 1e9
    rec = {"kernel": desc, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "avg_ms": round(ms, 4),
           "launches": len(per), "step_ms": round(sum(per), 3), "per_launch_ms": [round(v, 3) for v in per[:4]],
           "measured": f"in-step: all {len(per)} launches of {name} in the last eager warm-up train step of the "
                       "benchmarked model (same kernels, streams and concurrency as the captured timed step), HIP "
                       "events on each launch's stream",
           "algorithmic_bytes_per_launch": byts}
    if traffic_phase:
        _with_traffic(rec, traffic_phase)
    if isolated is not None:
        rec["isolated"] = isolated
    return rec


def _in_step_flops(work, name, peak_tflops, desc):
    """roofline record of an entry point whose launches differ in size (kernels.LAUNCH_WORK: the fp32 algorithmic
    FLOPs of each launch): the step's FLOPs over the launches' summed HIP-event time."""
    per = getattr(work, "step_taps", {}).get(name) or []
    flops = getattr(work, "step_work", {}).get(name) or []
    if not per or len(flops) != len(per):
        return None
    tot_ms = sum(per)
    ach = sum(flops) / (tot_ms * 1e-3) / 1e12
    return {"kernel": desc, "bound": "mfma", "achieved": round(ach, 2), "peak": peak_tflops, "unit": "TFLOP/s",
            "frac": round(ach / peak_tflops, 4), "traffic": None, "avg_ms": round(tot_ms / len(per), 4),
            "launches": len(per), "step_ms": round(tot_ms, 3),
            "per_launch_ms": [round(v, 3) for v in per[:4]],
            "measured": f"in-step: all {len(per)} launches of {name} in the last eager warm-up train step of the "
                        "benchmarked model, HIP events on each launch's stream; achieved = the step's fp32 algorithmic "
                        "FLOPs (2 M N K per launch) / the launches' summed time",
            "algorithmic_flops_per_step": sum(flops),
            "peak_note": "split-fp16: 3 f16 MFMAs per fp32 product, peak = dense f16 2500 TFLOP/s / 3"}


class _dconv_library:
    """Context: the dilated convs on MIOpen (layers.HIP_DCONV off) — the library figure beside the own kernels."""

    def __enter__(self):
        from avse_challenge_amd import layers
        self.prev, layers.HIP_DCONV = layers.HIP_DCONV, False

    def __exit__(self, *exc):
        from avse_challenge_amd import layers
        layers.HIP_DCONV = self.prev
        return False


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


def _event_ms(fn, n=10, warm=3):
    """Average duration of fn's launches, HIP events on torch's current stream (where the kernels run)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


BF16_PEAK_TFS = 2500.0         # dense bf16 MFMA peak, MI355X_MICROARCH.md (no sparsity)


def roofline_hip(dev):
    """The north-star kernels at their BASELINE shapes, timed live (HIP events) in the same run as the bench line:
    hand-written HBM-bound kernels against 8 TB/s (algorithmic bytes of each launch AS THE MODELS MAKE IT, DESIGN.md
    §3) and the Mamba projections' MFMA rate against the dense peak of their dtype. Returns (hbm_list, projections)."""
    from avse_challenge_amd import kernels as K
    from avse_challenge_amd import mamba_tasnet as M
    hbm, proj = [], []
    g = torch.Generator(device=dev).manual_seed(7)

    def rnd(*shape, dtype=torch.float32, scale=1.0):
        """(b, d, l) operands in the product's layout: 128-B aligned time stride (kernels.bdl_empty)."""
        v = (scale * torch.randn(shape, device=dev, generator=g)).to(dtype)
        if len(shape) != 3:
            return v
        t = K.bdl_empty(*shape, dtype, dev)
        t.copy_(v)
        return t

    def add_hbm(name, shape, dtype, byts, fn, pmc=None, valu=None):
        ms = _event_ms(fn)
        ach = byts / (ms * 1e-3) / 1e9
        rec = {"kernel": name, "shape": shape, "dtype": dtype, "bound": "hbm", "algorithmic_bytes_per_launch": byts,
               "avg_ms": round(ms, 4), "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(ach / HBM_PEAK_GBS, 4)}
        if pmc:
            rec["traffic"], rec["traffic_source"] = pmc_traffic(pmc)
        if valu:
            rec["valu_busy"], rec["valu_busy_source"] = pmc_valu_busy(*valu)
        hbm.append(rec)

    n = 16
    for tag, b, l, dt in (("C3", 64, 3999, torch.float32), ("C5", 32, 5999, torch.bfloat16)):
        d, s = 1024, (2 if dt == torch.bfloat16 else 4)
        name = "fp32" if s == 4 else "bf16"
        pmcf = "r03b_scan_pmc_c3_fp32.txt" if tag == "C3" else "r03e_scan_pmc_c5_bf16.txt"
        ktype = "float" if s == 4 else "avse::bf16_t"
        u, z, dout = rnd(b, d, l, dtype=dt), rnd(b, d, l, dtype=dt), rnd(b, d, l, dtype=dt)
        A = -torch.rand(d, n, device=dev, generator=g) - 0.5
        Bm, Cm = rnd(b, n, l, dtype=dt), rnd(b, n, l, dtype=dt)
        D = torch.ones(d, device=dev)
        # the step sizes as the model makes them (mamba_tasnet._delta): dt_proj with the softplus in its epilogue
        # (csrc/dtproj.hip, K = dt_rank = 32, the first 32 rows of x_proj's (b, 64, l) output), scanned in mode 2
        xdbl = rnd(b, 64, l, dtype=dt)
        wdt = ((32 ** -0.5) * torch.randn(d, 32, device=dev, generator=g)).to(dt)
        bdt = torch.log(torch.expm1(0.001 + 0.099 * torch.rand(d, device=dev, generator=g)))   # dt init 1e-3 .. 0.1
        add_hbm(f"avse_dtproj ({tag}, dt_proj + bias + softplus: 32 rows of x read, delta written)", [b, d, l], name,
                s * b * l * (d + 32), lambda: K.dtproj(wdt, xdbl[:, :32], bdt))
        delta = K.dtproj(wdt, xdbl[:, :32], bdt)
        _, x, _ = K.selective_scan_fwd(u, delta, A, Bm, Cm, D, z, None, 2, return_out=False)
        # training fwd: reads u, delta, z, B, C; writes out_z
        add_hbm(f"avse_scan_fwd ({tag}, training fwd, out_z only; delta from avse_dtproj)", [b, d, l], name,
                s * b * l * (4 * d + 2 * n),
                lambda: K.selective_scan_fwd(u, delta, A, Bm, Cm, D, z, None, 2, return_out=False),
                "scan" if tag == "C3" else "scan_c5", (pmcf, f"void avse::scan::fwd_kernel<{ktype},"))
        # bwd as the model calls it (out=None, no out_z recompute): reads u, delta, z, dout, B, C; writes du,
        # ddelta, dz (input dtype) and fp32 dB, dC
        add_hbm(f"avse_scan_bwd ({tag}, as MambaInnerNoOutProj calls it)", [b, d, l], name,
                b * l * (7 * s * d + 2 * s * n + 2 * 4 * n),
                lambda: K.selective_scan_bwd(u, delta, A, Bm, Cm, D, z, None, dout, x, None, None, 2, False),
                "scan_bwd" if tag == "C3" else "scan_bwd_c5",
                (pmcf, f"void avse::scan::bwd_kernel<{ktype},"))
        if tag == "C3":
            w, cb = rnd(d, 4, scale=0.5), rnd(d)
            add_hbm("avse_cconv_fwd (C3, k4 + SiLU)", [b, d, l], name, 2 * s * b * d * l,
                    lambda: K.causal_conv1d_fwd(u, w, cb, True), "cconv")
            add_hbm("avse_cconv_bwd (C3, k4 + SiLU)", [b, d, l], name, 3 * s * b * d * l,
                    lambda: K.causal_conv1d_bwd(u, w, cb, dout, silu=True))
        del u, z, dout, delta, Bm, Cm, x, xdbl
        torch.cuda.empty_cache()
    xd = torch.randn(16, 512, 3999, device=dev, generator=g)          # the TCN kernels take contiguous (B, C, K)
    wd, gy = rnd(512, 1, 3), torch.randn(16, 512, 3999, device=dev, generator=g)
    add_hbm("avse_dwconv_fwd (C4 TCN, H=512, K=3999, dil 128)", [16, 512, 3999], "fp32", 8 * xd.numel(),
            lambda: K.dwconv_fwd(xd, wd, 128), "dwconv")
    add_hbm("avse_dwconv_bwd (C4 TCN, H=512, K=3999, dil 128)", [16, 512, 3999], "fp32", 12 * xd.numel(),
            lambda: K.dwconv_bwd(xd, wd, gy, 128))
    al = torch.full((1,), 0.25, device=dev)
    gm, bt = 1 + 0.1 * torch.randn(1, 512, 1, device=dev, generator=g), 0.1 * torch.randn(1, 512, 1, device=dev, generator=g)
    _, y1, st = K.dwconv_gln_fwd(xd, wd, 128, al, gm, bt)
    add_hbm("avse_dwconv_gln_fwd (C4 TCN fused dwconv -> PReLU -> gLN: x read, y1 + y written)", [16, 512, 3999], "fp32",
            12 * xd.numel(), lambda: K.dwconv_gln_fwd(xd, wd, 128, al, gm, bt), "dwconv_gln")
    add_hbm("avse_dwconv_gln_bwd (C4 TCN fused: x, y1, dy read, dx written)", [16, 512, 3999], "fp32",
            16 * xd.numel(), lambda: K.dwconv_gln_bwd(xd, wd, 128, y1, al, gm, st, gy), "dwconv_gln_bwd")
    _, st2 = K.prelu_gln_fwd(xd, al, gm, bt)
    add_hbm("avse_prelu_gln_fwd (C4 TCN PReLU -> gLN after the 1x1 conv: x read, y written)", [16, 512, 3999], "fp32",
            8 * xd.numel(), lambda: K.prelu_gln_fwd(xd, al, gm, bt), "prelu_gln")
    add_hbm("avse_prelu_gln_bwd (C4 TCN: x, dy read, dx written)", [16, 512, 3999], "fp32",
            12 * xd.numel(), lambda: K.prelu_gln_bwd(xd, al, gm, st2, gy), "prelu_gln_bwd")
    del xd, gy, y1
    # avse1 C2 lip front-end: BatchNorm3d -> PReLU (bnact) and the (1,3,3) max pool on (32, 64, 75, 48, 48), and the
    # ResNet layer4 bn2 + shortcut -> PReLU site on (2400, 512, 3, 3).  Two passes each way: fwd reads x twice and
    # writes y (12 B/elem, +4 with the residual); bwd reads x, dy twice, writes dx (20 B/elem; with the residual
    # x, dy, res -> dres then x, dres -> dx: 28 B/elem).  Max pool: x read, y and the byte argmax written (fwd),
    # dy and argmax read, dx written (bwd): 4 + 4/4 + 1/4 B per input element each way.
    for tag, shape, res in (("C2 frontend BatchNorm3d -> PReLU", (32, 64, 75, 48, 48), False),
                            ("C2 ResNet layer4 bn2 + shortcut -> PReLU", (2400, 512, 3, 3), True)):
        xb = torch.randn(shape, device=dev, generator=g)
        rb = torch.randn(shape, device=dev, generator=g) if res else None
        gb = torch.randn(shape, device=dev, generator=g)
        C = shape[1]
        gam, bet, alp = torch.ones(C, device=dev), torch.zeros(C, device=dev), torch.full((C,), 0.25, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        _, stt = K.bnact_fwd(xb, gam, bet, rm, rv, True, 0.1, 1e-5, K.ACT_PRELU, alp, rb)
        ne = xb.numel()
        add_hbm(f"avse_bnact_fwd ({tag})", list(shape), "fp32", (16 if res else 12) * ne,
                lambda: K.bnact_fwd(xb, gam, bet, rm, rv, True, 0.1, 1e-5, K.ACT_PRELU, alp, rb))
        add_hbm(f"avse_bnact_bwd ({tag})", list(shape), "fp32", (28 if res else 20) * ne,
                lambda: K.bnact_bwd(xb, rb, gb, stt, gam, bet, K.ACT_PRELU, alp, True))
        if not res:
            yp, ip = K.maxpool_planes_fwd(xb, (3, 3), (2, 2), (1, 1))
            add_hbm("avse_maxpool2d_fwd (C2 frontend (1,3,3)/(1,2,2))", list(shape), "fp32", int(5.25 * ne),
                    lambda: K.maxpool_planes_fwd(xb, (3, 3), (2, 2), (1, 1)))
            add_hbm("avse_maxpool2d_bwd (C2 frontend (1,3,3)/(1,2,2))", list(shape), "fp32", int(5.25 * ne),
                    lambda: K.maxpool_planes_bwd(yp, ip, xb.shape, (3, 3), (2, 2), (1, 1)))
            del yp, ip
        del xb, rb, gb
        torch.cuda.empty_cache()
    # projections (MFMA): BiMambaV2's in_proj (_InProj) and out_proj (_BiOutProj) at C3 (fp32) and C5 (bf16)
    for tag, b, l, dt, peak in (("C3", 64, 3999, torch.float32, FP32_PEAK_TFS),
                                ("C5", 32, 5999, torch.bfloat16, BF16_PEAK_TFS)):
        dm, di = 512, 1024
        h, f, bk = rnd(b, l, dm, dtype=dt), rnd(b, di, l, dtype=dt), rnd(b, di, l, dtype=dt)
        w_in, w_out = rnd(2 * di, dm, scale=0.05), rnd(dm, di, scale=0.05)
        on = dt == torch.bfloat16
        for pname, flops, fn in (("in_proj", 2.0 * b * l * dm * 2 * di, lambda: M._InProj.apply(h, w_in)),
                                 ("out_proj", 2.0 * b * l * di * dm, lambda: M._BiOutProj.apply(f, bk, w_out))):
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=on, cache_enabled=False):
                ms = _event_ms(fn)
            ach = flops / (ms * 1e-3) / 1e12
            split = not on
            pk = BF16_PEAK_TFS / 3 if split else peak
            proj.append({"gemm": f"BiMambaV2 {pname} ({tag})", "shape": [b, l, dm, di], "dtype": str(dt)[6:],
                         "path": ("avse_gemm_bf16 (csrc/projgemm.hip)" if on and pname == "in_proj"
                                  else "avse_gemm_f32s (csrc/projgemm.hip: split-fp16 planes, 3 f16 MFMAs per product; "
                                       "time includes splitting the activation)" if split
                                  else "hipBLASLt (torch.bmm)"),
                         "bound": "mfma", "flops_per_launch": flops, "avg_ms": round(ms, 4),
                         "achieved": round(ach, 2), "peak": pk, "unit": "TFLOP/s", "frac": round(ach / pk, 4)}
                        | ({"peak_note": "dense f16 2500 TFLOP/s / 3 (three f16 MFMAs per fp32 product); achieved "
                                         "counts the fp32 algorithmic FLOPs"} if split else {}))
        del h, f, bk
        torch.cuda.empty_cache()
    # avse4 1x1 Conv1d (avse4._PointwiseFn, baseline/avse4/model.py:255-293) at C4: TemporalBlock's first conv
    # (256 -> 512 channels, B = 16, K = 3999) on avse_gemm_f32s
    from avse_challenge_amd import avse4 as A4
    b, cin, cout, kk = 16, 256, 512, 3999
    x4 = torch.randn(b, cin, kk, device=dev, generator=g)                  # contiguous, as the model's activations
    g4 = torch.randn(b, cout, kk, device=dev, generator=g)
    w4 = rnd(cout, cin, scale=0.05)
    xs4, ws4, gs4 = K.split_rows8(x4), K.split_planes(w4[None]), K.split_rows8(g4)
    y4 = torch.empty(b, cout, kk, device=dev)
    flops = 2.0 * b * kk * cin * cout
    for pname, fn, note in (
            ("forward (incl. splitting x and W)", lambda: A4._PointwiseFn.apply(w4, x4), "time includes the operand splits"),
            ("forward GEMM", lambda: K.gemm_f32s_split(xs4.t(), ws4, y4), "planes given"),
            ("weight gradient over time chunks", lambda: K.gemm_f32s_time_chunks(xs4, gs4),
             "planes given; time chunks as batches + the partial-output sum")):
        with torch.no_grad():
            ms = _event_ms(fn)
        ach = flops / (ms * 1e-3) / 1e12
        pk = BF16_PEAK_TFS / 3
        proj.append({"gemm": f"avse4 1x1 Conv1d {pname} (C4)", "shape": [b, cin, cout, kk], "dtype": "float32",
                     "path": f"avse_gemm_f32s (csrc/projgemm.hip: split-fp16 planes, 3 f16 MFMAs per product; {note})",
                     "bound": "mfma", "flops_per_launch": flops, "avg_ms": round(ms, 4), "achieved": round(ach, 2),
                     "peak": pk, "unit": "TFLOP/s", "frac": round(ach / pk, 4),
                     "peak_note": "dense f16 2500 TFLOP/s / 3 (three f16 MFMAs per fp32 product); achieved counts the "
                                  "fp32 algorithmic FLOPs"})
    del x4, w4, g4, xs4, ws4, gs4, y4
    torch.cuda.empty_cache()
    return hbm, proj


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    if args.device == "cpu" and args.workload != "plumbing":
        raise SystemExit("--device cpu runs --workload plumbing only (the HIP kernels are GPU-only)")
    world, rank, dev = setup_dist(args.device)
    if world != args.gpus and rank == 0:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE {world}: timing {world} rank(s)", file=sys.stderr, flush=True)
    heartbeat(rank)
    if dev.type == "cuda":
        torch.backends.cuda.matmul.allow_tf32 = False
        torch.backends.cudnn.allow_tf32 = False
        # MIOpen immediate mode: find mode (benchmark=True, as avse1 train.py:11 sets for cuDNN) JIT-compiles
        # every candidate solver on a fresh box (minutes); immediate mode compiles only the chosen one.
        torch.backends.cudnn.benchmark = bool(int(os.environ.get("AVSE_MIOPEN_FIND", "0")))
    global DIRECTION_STREAMS_ARG
    DIRECTION_STREAMS_ARG = args.direction_streams
    if args.workload == "avse1":
        B = args.batch or 32
        work = Avse1Step(B, dev, rank, world, args.lip_hw)
    elif args.workload == "avse4":
        B = args.batch or 16
        work = Avse4Step(B, dev, rank, world)
    elif args.workload == "avse2":
        B = args.batch or 16
        work = Avse2Step(B, dev, rank, world)
    elif args.workload == "avmamba":
        B = args.batch or 32
        work = AVMambaStep(B, dev, rank, world, args.size)
    elif args.workload == "dpmamba":
        # B=16: the 16-step scan checkpoints (1 fp32 per step; 64 per 34-step inter row) take ~0.8 GB per utterance
        # more than round 1's 64-step ones, and B=32 no longer fits 288 GB
        B = args.batch or 16
        work = DPMambaStep(B, dev, rank, world, args.size)
    elif args.workload == "plumbing":
        B = args.batch or 2
        work = PlumbingStep(B, dev, rank, world)
    else:
        B = args.batch or 64
        work = MambaStep(B, dev, rank, world, args.size)

    use_graph = work.graph_ok and not args.no_graph and dev.type == "cuda"
    step = Trainer(work, world, dev, use_graph=use_graph, bucket_mb=args.bucket_mb)
    # in-step roofline of C3 / C4 / C5: every launch of the workload's dominant hand-written kernels inside the last
    # eager warm-up step (the same kernels, streams and concurrency the captured step replays), HIP events on each
    # launch's stream (kernels.LAUNCH_TAPS).  AVSE_PROFILE_MARK=roof brackets that step with marker kernels instead of
    # the timed region (tools/profile_bench.sh: the window's kernel averages are the line's in-step avg_ms).
    taps = getattr(work, "tap_kernels", ()) if (dev.type == "cuda" and rank == 0 and not args.no_roofline) else ()
    roof_mark = os.environ.get("AVSE_PROFILE_MARK", "0") == "roof"
    nwarm = max(args.warmup, 1 if use_graph else 0)
    for i in range(nwarm):
        t = time.perf_counter()
        tapping = bool(taps) and i == nwarm - 1
        if tapping:
            from avse_challenge_amd import kernels as K
            for n in taps:
                K.LAUNCH_TAPS[n] = []
                K.LAUNCH_WORK.pop(n, None)
            if roof_mark:
                torch.cuda._sleep(1000)
        try:
            step()
            if tapping and roof_mark:
                torch.cuda._sleep(1000)
            sync(dev)
            if tapping:
                work.step_taps = {n: [a.elapsed_time(b) for a, b in K.LAUNCH_TAPS[n]] for n in taps}
                work.step_work = {n: list(K.LAUNCH_WORK.get(n, [])) for n in taps}
        finally:
            if tapping:
                for n in taps:
                    K.LAUNCH_TAPS.pop(n, None)
                    K.LAUNCH_WORK.pop(n, None)
        if rank == 0:
            print(f"[bench] warmup {i + 1}/{args.warmup}: {time.perf_counter() - t:.2f}s", file=sys.stderr, flush=True)
    graph = False
    if use_graph:
        try:
            step.capture()
            step()
            sync(dev)
            graph = "fwd+bwd+opt" if step.g_fb is not None else "opt"
        except Exception as e:      # noqa: BLE001 - report and fall back to eager launches
            print(f"[bench] HIP graph capture failed ({type(e).__name__}: {e}); eager launches", file=sys.stderr,
                  flush=True)
            step.drop_graphs()
            import gc
            gc.collect()                       # the half-captured graph's private pool goes back to the device
            torch.cuda.empty_cache()
            sync(dev)
    sync(dev)
    barrier(world)
    sync(dev)
    mark = os.environ.get("AVSE_PROFILE_MARK", "0") == "1"   # tools/ktrace_window.py brackets the timed steps
    if mark:
        torch.cuda._sleep(1000)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    if mark:
        torch.cuda._sleep(1000)
    sync(dev)
    barrier(world)
    sync(dev)
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    if not torch.isfinite(loss.detach()).all():
        raise RuntimeError("non-finite loss in the timed region")
    step.check_kernel_errors()          # a grouped-LSTM launch that was not co-resident raises here (ddp.py)

    cuda = dev.type == "cuda"
    roof = None if args.no_roofline or rank != 0 or not cuda else work.roofline(dev)
    hbm_list = proj = None
    if rank == 0 and world == 1 and cuda and not args.no_roofline_hip:
        hbm_list, proj = roofline_hip(dev)
    # the CPU-baseline leg (rank 0, one rank): the oracle restatement on the host cores, timed (cpu_baseline), and the
    # same oracle as the CHECKER of the benchmarked model's output waveforms on the batch's first utterances (parity,
    # the "SI-SDR vs ref" half of the BASELINE metric)
    cpu = par = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = work.cpu_baseline()
    if rank == 0 and world == 1 and dev.type == "cuda" and not args.no_parity and getattr(work, "parity", None) is not None:
        par = work.parity(dev)
    secondary = None
    if rank == 0 and world == 1 and cuda and args.workload == "avse1" and args.secondary:
        secondary = run_secondary(args)
    if rank == 0:
        value = world * B * args.steps / dt
        cfg = {**work.config(world), "hip_graph": graph}
        if cuda:
            cfg["max_mem_gb"] = round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2)
        if world > 1:
            cfg["ddp"] = {"backend": dist.get_backend(), "grad_buckets": step.n_buckets, "bucket_mb": args.bucket_mb,
                          "allreduce": "async per bucket from post-accumulate-grad hooks (overlaps backward)",
                          "broadcast_buffers": step.broadcast_buffers}
        rec = {"metric": {"avse1": METRIC, "mamba": "utterances/sec (4s@8kHz WSJ0-2mix, Mamba-TasNet)",
                          "avse4": "utterances/sec (5s@16kHz binaural + 125 lip frames, avse4)",
                          "dpmamba": "utterances/sec (4s@8kHz WSJ0-2mix, DPMamba)",
                          "avse2": "utterances/sec (3s@16kHz + 75 lip frames 224x224, avse2)",
                          "avmamba": "utterances/sec (3s@16kHz + 75 lip frames, AV Mamba-TasNet-L bf16)",
                          "plumbing": "steps/sec (CPU plumbing test hook)"}[args.workload],
               "value": round(value, 3), "unit": "utt/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": getattr(work, "dtype", "fp32"),
               "data": "synthetic (speech-like noise with 4 Hz envelope at SNR {0,3,6,9} dB, uint8 lips; "
                       "random-init weights)",
               "config": cfg, "roofline": roof, "roofline_hip": hbm_list, "projections": proj, "cpu_baseline": cpu,
               "parity": par}
        if secondary is not None:
            rec["secondary"] = secondary
        if not cuda:
            rec["device"] = "cpu (gloo ranks; n_gpus counts ranks)"
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
