"""Two data-parallel ranks on ONE GPU (gloo on CUDA tensors, both ranks on cuda:0): the hook-launched bucket
all-reduce of avse_challenge_amd.ddp.Trainer must wait for EVERY stream that wrote a bucket's gradients.

The avse1 step runs its lip branch (forward and backward) on a side stream and Mamba-TasNet at B < 48 runs the
BiMamba reverse direction on one, so single buckets hold gradients of two streams (ddp.py:_launch).
Gloo's CUDA all-reduce, like RCCL's, orders itself after the current stream only.  Each rank records, on the
second step (every bucket launched from a hook during the backward), the weights the step started from and the
summed gradient the collectives produced; it then recomputes both shards' gradients from those weights in one
process on one stream, eagerly, and the two must agree.  A bucket reduced before its side-stream gradients
landed would be O(1) off.  Reference semantics: Lightning DDP, baseline/avse4/train.py:28-42, conf/train.yaml:16-18;
SpeechBrain DDP, Mamba-TasNet/train_wsj0mix.py:160,718.

avse1: the one-process reference runs with the 2-rank run's activation patterns imposed (the technique of
tests/avse1_parity.py, here on the product model itself): every ReLU / PReLU sign and every L1 sign that rank r's
step took is recorded and shard r's reference evaluation follows it, so a pre-activation within rounding of 0 cannot
take the other branch (which the lip trunk's BatchNorm backward amplifies to ~3e-3 of a branch).

What each rank checks, so a failure names the leg that moved (GPUTEST_r05: rank 0 5.7e-5, rank 1 2.9e-3 in one run):
  * the ranks' all-reduced sums are bitwise equal (sha256 of the flat buffer, all-gathered);
  * the grouped-LSTM sticky error flag is 0 after the 2-rank step and after each reference leg;
  * the reference legs run in turn (a barrier between the ranks), so neither process's reference shares the GPU with
    the other's; the concurrent evaluation is kept as a diagnostic, with each branch's forward output compared across
    the two processes and the two legs;
  * both processes run the per-sequence LSTM recurrence (csrc/lstm.hip): two processes on one GPU break the grouped
    recurrence's premise that its workgroups are co-resident on a device no other process holds (one process per GPU
    in production), and a 1-s hand-off timeout there is the likeliest cause of round 5's rank-1 deviation;
  * total <= 2e-3 and every branch <= 2e-3 of its norm (measured: ~1e-6)."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _make(workload, rank, world):
    import bench
    dev = torch.device("cuda", 0)
    torch.manual_seed(7)                                  # same init on both ranks (rank 0's is broadcast anyway)
    if workload == "avse1":
        st = bench.Avse1Step(2, dev, rank, world, 64)
    else:
        st = bench.MambaStep(2, dev, rank, world, "XS")
    for m in st.model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    return st


def _capture(model, masks):
    """Record (into masks, CPU bool tensors keyed by module name) the sign pattern of every activation of the avse1
    product model while active: bn_act ReLU / PReLU outputs, PReLU modules, and the prediction ("pred")."""
    from avse_challenge_amd import avse1, layers
    names = {id(m): n for n, m in model.named_modules()}
    orig = avse1.bn_act

    def spy(x, bn, act=None, res=None, folded_bias=None, **kw):
        y = orig(x, bn, act, res, folded_bias=folded_bias, **kw)
        if act is not None:
            masks[names[id(bn)] if act == "relu" else names[id(act)]] = layers.K.positive(y).detach().cpu()
        return y
    hs = [m.register_forward_hook(lambda mod, i, o, n=n: masks.__setitem__(n, (o > 0).detach().cpu()))
          for n, m in model.named_modules() if isinstance(m, layers.PReLU)]
    hs.append(model.register_forward_hook(lambda mod, i, o: masks.__setitem__("pred", o.detach().cpu())))
    avse1.bn_act = spy

    def undo():
        avse1.bn_act = orig
        for h in hs:
            h.remove()
    return undo


def _impose(model, masks):
    """Make the avse1 product model follow ``masks`` at every activation (ReLU: where(mask, z, 0); PReLU: where(mask, z,
    a z)); returns the undo callable."""
    from avse_challenge_amd import avse1, layers
    names = {id(m): n for n, m in model.named_modules()}
    orig = avse1.bn_act

    def forced(x, bn, act=None, res=None, folded_bias=None, **split_output_flags):   # fp32 outputs: masks applied below
        if act is None:
            return orig(x, bn, None, res, folded_bias=folded_bias)
        z = orig(x, bn, None, res, folded_bias=folded_bias)
        key = names[id(bn)] if act == "relu" else names[id(act)]
        m = masks[key].to(z.device)
        assert m.shape == z.shape, (key, tuple(m.shape), tuple(z.shape))
        if act == "relu":
            return torch.where(m, z, torch.zeros_like(z))
        a = act.weight.view([1, -1] + [1] * (z.dim() - 2)) if act.weight.numel() > 1 else act.weight
        return torch.where(m, z, a * z)
    hs = []
    for n, mod in model.named_modules():
        if isinstance(mod, layers.PReLU):
            def hook(m_, inp, out, n=n):
                z = inp[0]
                a = m_.weight.view([1, -1] + [1] * (z.dim() - 2)) if m_.weight.numel() > 1 else m_.weight
                return torch.where(masks[n].to(z.device), z, a * z)
            hs.append(mod.register_forward_hook(hook))
    avse1.bn_act = forced

    def undo():
        avse1.bn_act = orig
        for h in hs:
            h.remove()
    return undo


def _reference(workload, shard, world, weights, masks, taps):
    """Shard ``shard``'s gradient (flat, parameter order) on the product model in THIS process, on one stream, from
    ``weights``; avse1 follows ``masks`` (rank shard's activation / L1 signs).  ``taps`` collects the forward outputs of
    the branches (CPU copies) so two processes' reference legs can be compared stage by stage."""
    ref = _make(workload, shard, world)
    params = [p for p in ref.model.parameters() if p.requires_grad]
    with torch.no_grad():
        for p, w in zip(params, weights):
            p.copy_(w.to(p.device))
    hs = []
    if workload == "avse1":
        m = ref.model
        for name, mod in (("visual", m.net_visualfeat), ("audio", m.net_audiofeat), ("lstm", m.net_fusion.lstm_conv)):
            hs.append(mod.register_forward_hook(
                lambda mod_, i, o, name=name: taps.__setitem__(f"{shard}/{name}",
                                                               (o[0] if isinstance(o, tuple) else o).detach().cpu())))
        undo = _impose(ref.model, masks)
        try:
            batch = ref.avse1.AVNet.features_from_waves(ref.noisy, ref.clean)
            batch["lip_images"] = ref.lips
            pred = ref.model(batch)
            taps[f"{shard}/pred"] = pred.detach().cpu()
            sgn = torch.sign(masks["pred"].to(pred.device) - batch["mask"])      # the rank's L1 signs
            loss = (sgn * (pred - batch["mask"])).mean()
        finally:
            undo()
    else:
        loss = ref.loss()
    for h in hs:
        h.remove()
    grads = torch.autograd.grad(loss, params, allow_unused=True)
    flat = torch.cat([(torch.zeros_like(p) if g is None else g).reshape(-1) for p, g in zip(params, grads)]).cpu()
    names = [n for n, p in ref.model.named_parameters() if p.requires_grad]
    return flat, params, names


def _branch_errs(workload, names, params, a, b):
    """Per branch ||a - b|| / ||b|| over the flat (parameter-order) gradient vectors."""
    out, off = {}, 0
    for name, p in zip(names, params):
        n = p.numel()
        key = ".".join(name.split(".")[:2]) if workload == "mamba" else name.split(".")[0]
        e, r = out.get(key, (0.0, 0.0))
        out[key] = (e + float((a[off:off + n] - b[off:off + n]).double().norm()) ** 2,
                    r + float(b[off:off + n].double().norm()) ** 2)
        off += n
    return {k: (e / max(r, 1e-60)) ** 0.5 for k, (e, r) in out.items()}


def _worker(rank, world, port, q, workload, bucket_mb):
    try:
        sys.path.insert(0, REPO)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import hashlib

        import bench  # noqa: F401  (imports the package before the GPU is touched)
        import torch.distributed as dist
        from avse_challenge_amd import kernels
        from avse_challenge_amd.ddp import _dense
        torch.cuda.set_device(0)
        # Two processes share ONE GPU here, so the grouped LSTM recurrence's premise (its workgroups co-resident on a
        # device no other process holds) does not hold: both legs run the per-sequence recurrence (csrc/lstm.hip).
        # The sticky error flag is still read after every leg.
        kernels.no_grouped_lstm().__enter__()
        dist.init_process_group("gloo", rank=rank, world_size=world)
        st = _make(workload, rank, world)
        from avse_challenge_amd import mamba_tasnet
        mamba_tasnet.set_direction_streams(True)          # buckets holding gradients of two streams (module docstring)
        tr = bench.Trainer(st, world, torch.device("cuda", 0), use_graph=False, bucket_mb=bucket_mb)
        rec = {}
        orig_opt, orig_launch = tr._opt, tr._launch
        hook_launches = []

        def spy_launch(b):
            hook_launches.append(tr._armed)
            orig_launch(b)

        def spy_opt():
            torch.cuda.synchronize()
            rec["grad_sum"] = tr.flat.detach().clone().cpu()
            rec["weights"] = [p.detach().clone().cpu() for p in tr.params]
            orig_opt()

        tr._opt, tr._launch = spy_opt, spy_launch
        tr()                                              # first step: learns which parameters get gradients
        hook_launches.clear()
        masks = {}
        undo = _capture(st.model, masks) if workload == "avse1" else (lambda: None)
        tr()                                              # second step: every bucket launched from a hook
        torch.cuda.synchronize()
        undo()
        n_buckets = tr.n_buckets
        in_hooks = sum(hook_launches)
        step_flag = kernels.lstm_group_status()
        all_masks = [None] * world
        dist.all_gather_object(all_masks, masks)          # shard s's reference follows rank s's activation signs
        got = rec["grad_sum"]
        # the Trainer's flat buffer holds each gradient with its parameter's strides: parameter order, logical layout
        got_l, off = [], 0
        for p in tr.params:
            n = p.numel()
            seg = got[off:off + n]
            got_l.append((seg.as_strided(p.shape, p.stride()) if _dense(p) else seg.view(p.shape)).reshape(-1))
            off += n
        got_l = torch.cat(got_l)
        # (ii): the ranks must hold bitwise the same all-reduced sum
        digests = [None] * world
        dist.all_gather_object(digests, hashlib.sha256(got.numpy().tobytes()).hexdigest())

        # one-process, one-stream reference on the same weights: the sum of both shards' gradients.  The two ranks
        # evaluate it in turn (a barrier between them), so neither process's reference shares the GPU with the
        # other's; the concurrent evaluation (both at once, as round 5 ran it) is kept as a diagnostic.
        from avse_challenge_amd import avse1, mamba_tasnet
        avse1.set_branch_streams(False)
        mamba_tasnet.set_direction_streams(False)

        def ref_leg():
            taps, tot = {}, None
            for shard in range(world):
                flat, params, names = _reference(workload, shard, world, rec["weights"], all_masks[shard], taps)
                tot = flat if tot is None else tot + flat
            return tot, params, names, taps, kernels.lstm_group_status()

        conc, params, names, taps_c, flag_c = ref_leg()
        dist.barrier()
        ser = taps_s = flag_s = None
        for turn in range(world):
            if turn == rank:
                ser, _, _, taps_s, flag_s = ref_leg()
            dist.barrier()
        # (i): did the two processes compute the same reference?  Gather the other rank's serialized one.
        refs = [torch.empty_like(ser) for _ in range(world)]
        dist.all_gather(refs, ser)
        tap_keys = sorted(taps_s)
        tap_list = [None] * world
        dist.all_gather_object(tap_list, {k: taps_s[k] for k in tap_keys})
        diag = {
            "digests_equal": len(set(digests)) == 1,
            "step_flag": step_flag, "flag_conc": flag_c, "flag_serial": flag_s,
            "conc_vs_serial": _branch_errs(workload, names, params, conc, ser),
            "serial_vs_rank0": _branch_errs(workload, names, params, ser, refs[0]),
            "taps_vs_rank0": {k: float((taps_s[k] - tap_list[0][k]).double().norm() /
                                       max(float(tap_list[0][k].double().norm()), 1e-30)) for k in tap_keys},
            "taps_conc_vs_serial": {k: float((taps_c[k] - taps_s[k]).double().norm() /
                                             max(float(taps_s[k].double().norm()), 1e-30)) for k in tap_keys},
            "got_vs_conc": _branch_errs(workload, names, params, got_l, conc),
        }
        dist.destroy_process_group()
        errs, off = [], 0                                 # per parameter
        for p in params:
            n = p.numel()
            seg = got_l[off:off + n].view(p.shape)
            r = ser[off:off + n].view(p.shape)
            errs.append((float((seg - r).norm()), float(r.norm())))
            off += n
        tot = (float((torch.tensor([e for e, _ in errs]) ** 2).sum().sqrt()),
               float((torch.tensor([r for _, r in errs]) ** 2).sum().sqrt()))
        q.put((rank, {"errs": errs, "names": names, "total": tot, "n_buckets": n_buckets, "in_hooks": in_hooks,
                      "diag": diag}))
    except Exception as e:                                # surface the failure instead of a queue timeout
        import traceback
        q.put((rank, {"error": repr(e) + "\n" + traceback.format_exc()}))
        raise


@pytest.mark.parametrize("workload", ["avse1", "mamba"])
def test_two_ranks_one_gpu_side_stream_buckets(workload):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, workload, 0.5)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=400) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in res[r], res[r].get("error")
    for p in procs:
        assert p.exitcode == 0
    for r in range(world):
        rec = res[r]
        assert rec["n_buckets"] > 2 and rec["in_hooks"] == rec["n_buckets"], (rec["n_buckets"], rec["in_hooks"])
        e, n = rec["total"]
        print(f"{workload} rank {r} diagnostics: {rec['diag']}")
        worst = sorted(((ei / max(ni, 1e-30), i) for i, (ei, ni) in enumerate(rec["errs"])), reverse=True)[:3]
        print(f"{workload} rank {r}: total rel err {e / n:.2e}, worst params {worst}")
        # With the activation signs imposed (module docstring) the runs differ by fp32 rounding only (MIOpen may still
        # round differently: its solver depends on the workspace the caching allocator can hand it).  A bucket reduced
        # before a side stream's gradients landed leaves whole parameters stale or zero: O(1) of their norm, so a
        # bucket holding 4e-6 of a branch's squared gradient norm already moves that branch past 2e-3.  Per branch:
        # the avse1 lip / audio / fusion nets, the Mamba encoder / masknet / decoder.
        branches = {}
        for name, (ei, ni) in zip(rec["names"], rec["errs"]):
            key = ".".join(name.split(".")[:2]) if workload == "mamba" else name.split(".")[0]
            be, bn = branches.get(key, (0.0, 0.0))
            branches[key] = (be + ei ** 2, bn + ni ** 2)
        for key, (be, bn) in branches.items():
            print(f"    branch {key}: rel err {(be / max(bn, 1e-60)) ** 0.5:.2e}")
        top = sorted(((ei, ni, name) for name, (ei, ni) in zip(rec["names"], rec["errs"])), reverse=True)[:4]
        print("    largest absolute errors: " + ", ".join(f"{nm} {ei:.2e} of {ni:.2e}" for ei, ni, nm in top))
        d = rec["diag"]
        assert d["digests_equal"], "the ranks' all-reduced gradient sums differ"
        assert d["step_flag"] == 0 and d["flag_conc"] == 0 and d["flag_serial"] == 0, d
        assert e <= 2e-3 * n, (workload, r, e, n)
        for key, (be, bn) in branches.items():
            assert be ** 0.5 <= 2e-3 * bn ** 0.5 + 1e-6 * n, (workload, r, key, be ** 0.5, bn ** 0.5)
        for i, (ei, ni) in enumerate(rec["errs"]):
            assert ei <= 5e-2 * ni + 1e-4 * n, (workload, r, i, ei, ni)
