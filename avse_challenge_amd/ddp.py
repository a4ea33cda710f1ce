"""Batch-sharded data-parallel training step: one process per GPU, RCCL over xGMI.

What Lightning DDP does for the reference (baseline/avse4/train.py:28-42 with conf/train.yaml:16-18 strategy
ddp; Mamba-TasNet/train_wsj0mix.py:160,718 via SpeechBrain's DDP wrapper), rebuilt around one flat gradient
buffer instead of DDP's reducer:
  * every parameter's ``.grad`` is a view into ONE flat fp32 buffer; the buffer is cut into contiguous
    buckets of ~``bucket_mb`` in reverse registration order (the order backward produces gradients);
  * a post-accumulate-grad hook per parameter counts arrivals; the moment a bucket is complete its
    all-reduce is launched asynchronously (RCCL runs it on its own stream after an event wait on the
    current stream), so the exchange overlaps the rest of the backward; each hook records an event on the
    stream that accumulated its gradient, and the launch first makes the current stream wait for the events
    of every other stream in the bucket (the avse1 lip branch and the BiMamba reverse direction run their
    backward on a side stream, so one bucket can hold gradients written by two streams);
  * a parameter that got no gradient on the first step (its bucket is sized without it) and gets one later
    raises, as DDP without find_unused_parameters does, instead of going un-averaged;
  * after backward the remaining buckets (parameters without a gradient this step) are launched, the
    current stream waits for every collective, and the sum is scaled by 1/world (mean, as DDP);
  * DDP's ``broadcast_buffers=True``: rank 0's buffers (BatchNorm running stats, num_batches_tracked) are
    broadcast to every rank before each forward, as two flat tensors (floating / integer) that the modules'
    buffers are views of; per-rank batch statistics otherwise (no SyncBN, as the reference);
  * identical initial weights: rank 0's parameters are broadcast once at construction.
With ``use_graph`` (single GPU) the forward/backward and the optimizer step are each replayed as a captured
HIP graph; with world > 1 the forward/backward stays eager (the collectives are launched from autograd hooks)
and only the optimizer step is captured.
Kernel errors: the grouped LSTM recurrence (csrc/lstm_group.hip) writes a sticky device flag when its workgroups
were not co-resident (its outputs are then invalid).  The optimizer update is gated on that flag ON THE DEVICE: the
step's ``found`` scalar (the flag, with world > 1 max-all-reduced together with the gradient buckets so every rank
sees the same value) is fused Adam's ``found_inf``, so a step whose gradients are invalid updates no parameter and
no Adam moment on any rank — nor does any later step while the flag stays set.  Every step enqueues a 4-byte copy
of ``found`` into pinned memory and checks the previous copy once it has landed (no synchronisation); when it is
set, every rank raises ``kernels.HipKernelError`` in the same step and the flag is cleared.
``check_kernel_errors()`` is the blocking form.  The parameters are those from before the failed step.
"""
import functools

import torch
import torch.distributed as dist


class Trainer:
    """One training step = [buffer broadcast] + forward + loss + backward (+ overlapped bucketed gradient
    all-reduce when world > 1) + optional grad-norm clip + Adam.  ``step`` provides ``model``, ``loss()``,
    ``lr`` and ``clip``."""

    def __init__(self, step, world, dev, use_graph, bucket_mb=25.0, broadcast_buffers=True, sync_loss=True):
        self.step, self.world, self.dev = step, world, dev
        # the returned loss is the mean over ranks (Lightning ``self.log(..., sync_dist=True)``,
        # baseline/avse4/model.py:325): one 4-byte all-reduce per step, overlapped with the optimizer
        self.sync_loss = sync_loss and world > 1
        self.use_graph = bool(use_graph) and dev.type == "cuda"
        self.params = [p for p in step.model.parameters() if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        # world > 1: every .grad is a view of one flat buffer (the bucketed all-reduce's operand), zeroed per step,
        # into which autograd accumulates (one add per parameter).  world == 1 (round 6): no flat buffer -- each
        # .grad is reset to None before the backward, so autograd hands the computed gradient over without an add
        # (~120 add launches per avse1 step, ~1.5 ms); under graph capture the gradients then live in the graph's pool
        # at fixed addresses, which the captured optimizer step reads
        self.flat = torch.zeros(n, device=dev) if world > 1 else None
        ranges, off = [], 0
        for p in self.params:
            if self.flat is not None:
                # same strides as the parameter (channels_last conv weights too): autograd accumulates in place
                # without a layout copy (dense, non-overlapping parameters only)
                seg = self.flat[off:off + p.numel()]
                p.grad = seg.as_strided(p.size(), p.stride()) if _dense(p) else seg.view_as(p)
            ranges.append((off, off + p.numel()))
            off += p.numel()
        self.buf_f = self.buf_i = None
        self.broadcast_buffers = broadcast_buffers and world > 1
        if world > 1:
            for p in step.model.parameters():          # identical initial weights (DDP semantics)
                dist.broadcast(p.data, 0)
            self.buf_f, self.buf_i = _flatten_buffers(step.model, dev)
            self.sync_buffers()
            self._make_buckets(ranges, bucket_mb)
            for i, p in enumerate(self.params):
                p.register_post_accumulate_grad_hook(functools.partial(self._grad_ready, i))
        self._armed = False
        self._flag = self._found = None
        if dev.type == "cuda":
            from . import kernels
            # created here, outside any graph pool: captured launches and the captured optimizer keep its pointer
            self._flag = kernels._kernel_error_flag(dev)
            self._found = torch.zeros((), device=dev, dtype=torch.float32)   # 0-dim: Adam's found_inf
            self.opt = torch.optim.Adam(self.params, lr=step.lr, capturable=self.use_graph, fused=True)
            self.opt.found_inf = self._found          # read by Adam.step (fused): skip the update when nonzero
        else:
            self.opt = torch.optim.Adam(self.params, lr=step.lr, foreach=True)
        self.g_fb = self.g_opt = None
        self.loss = None
        self._err_host = self._err_ev = None

    # ------------------------------------------------------------------ kernel error flag
    def _poll_kernel_errors(self):
        """Lagged, non-blocking check of the step's ``found`` scalar (ddp module docstring)."""
        if self._found is None:
            return
        if self._err_host is None:
            self._err_host = torch.zeros((), dtype=torch.float32, pin_memory=True)
            self._err_ev = torch.cuda.Event()
        elif self._err_ev.query() and float(self._err_host) != 0.0:
            self._raise_kernel_error()
        self._err_host.copy_(self._found, non_blocking=True)   # the flag is sticky: a later copy misses nothing
        self._err_ev.record()

    def _raise_kernel_error(self):
        from . import kernels
        code = int(self._flag.item()) & 0xFFFFFFFF           # this rank's own code (0: another rank's launch failed)
        self._flag.zero_()
        self._found.zero_()
        if self._err_host is not None:
            self._err_host.zero_()
        raise kernels.HipKernelError(kernels.kernel_error_message(code) if code else
                                     "a grouped LSTM launch on another rank timed out; this step's update was skipped "
                                     "on every rank")

    def check_kernel_errors(self):
        """Blocking: raise kernels.HipKernelError if any kernel of the steps so far reported invalid outputs."""
        if self._found is not None:
            torch.cuda.synchronize(self.dev)
            if float(self._found.item()) != 0.0 or int(self._flag.item()) != 0:
                self._raise_kernel_error()

    # ------------------------------------------------------------------ buckets
    def _make_buckets(self, ranges, bucket_mb):
        cap = max(1, int(bucket_mb * 2 ** 20 / 4))
        self.bucket_of = [0] * len(ranges)
        self.bucket_range, self.bucket_params = [], []
        cur, lo, hi = [], None, None
        for i in reversed(range(len(ranges))):
            a, b = ranges[i]
            cur.append(i)
            lo, hi = a, (b if hi is None else hi)
            if hi - lo >= cap:
                self._close_bucket(cur, lo, hi)
                cur, lo, hi = [], None, None
        if cur:
            self._close_bucket(cur, lo, hi)
        self.expected = [len(ps) for ps in self.bucket_params]
        self.seen = [False] * len(ranges)
        self.used = [True] * len(ranges)
        self.first_step = True
        self._events = {}

    def _close_bucket(self, idx, lo, hi):
        for i in idx:
            self.bucket_of[i] = len(self.bucket_range)
        self.bucket_range.append((lo, hi))
        self.bucket_params.append(list(idx))

    def _arm(self):
        self.ready = [0] * len(self.bucket_range)
        self.launched = [False] * len(self.bucket_range)
        self.works = []
        # per bucket: the streams its gradients were accumulated on this step, each with an event recorded after
        # the latest of them (the avse1 lip branch and the BiMamba reverse direction run their backward on a side
        # stream, so one bucket can hold gradients of two streams)
        self.bucket_streams = [{} for _ in self.bucket_range]
        self._armed = True

    def _grad_ready(self, i, _param):
        if not self._armed:
            return
        if not self.first_step and not self.used[i]:
            # its bucket was sized on the first step without it and may already be reduced: DDP without
            # find_unused_parameters raises here too, instead of leaving this gradient un-averaged
            raise RuntimeError(f"parameter {i} received a gradient after getting none on the first step; its "
                               "bucket's all-reduce may already have been launched")
        self.seen[i] = True
        b = self.bucket_of[i]
        if self.dev.type == "cuda":
            s = torch.cuda.current_stream(self.dev)     # autograd runs the hook on the stream that accumulated
            ev = self._events.get((b, s.stream_id))
            if ev is None:
                ev = self._events[(b, s.stream_id)] = torch.cuda.Event()
            ev.record(s)
            self.bucket_streams[b][s.stream_id] = ev
        self.ready[b] += 1
        if not self.first_step and self.ready[b] == self.expected[b]:
            self._launch(b)

    def _launch(self, b):
        lo, hi = self.bucket_range[b]
        if self.dev.type == "cuda":
            # the collective is ordered after the CURRENT stream only: make that stream wait for every other
            # stream that wrote a gradient of this bucket
            cur = torch.cuda.current_stream(self.dev)
            for sid, ev in self.bucket_streams[b].items():
                if sid != cur.stream_id:
                    cur.wait_event(ev)
        self.works.append(dist.all_reduce(self.flat[lo:hi], async_op=True))
        self.launched[b] = True

    def _finish_allreduce(self):
        """Launch what the hooks did not (unused parameters; everything on the first step, which also learns
        which parameters receive gradients), then make the current stream wait for every collective."""
        self._armed = False
        for b in range(len(self.bucket_range)):
            if not self.launched[b]:
                self._launch(b)
        if self.sync_loss:
            self.loss = self.loss.clone()
            self.works.append(dist.all_reduce(self.loss, async_op=True))
        if self._found is not None:
            # every rank skips the update when any rank's kernels reported invalid outputs (found is Adam's found_inf)
            self._found.copy_(self._flag.ne(0)[0])       # Adam skips on found_inf == 1 exactly
            self.works.append(dist.all_reduce(self._found, op=dist.ReduceOp.MAX, async_op=True))
        for w in self.works:
            w.wait()
        self.works = []
        if self.sync_loss:
            self.loss.div_(self.world)
        if self.first_step:
            self.expected = [sum(self.seen[i] for i in ps) for ps in self.bucket_params]
            self.used = list(self.seen)
            self.first_step = False

    @property
    def n_buckets(self):
        return len(self.bucket_range) if self.world > 1 else 0

    # ------------------------------------------------------------------ buffers
    def sync_buffers(self):
        """DDP broadcast_buffers: rank 0's BatchNorm running stats (and counters) to every rank."""
        if self.buf_f is not None:
            dist.broadcast(self.buf_f, 0)
        if self.buf_i is not None:
            dist.broadcast(self.buf_i, 0)

    # ------------------------------------------------------------------ step
    def _fwd_bwd(self, out=None):
        if self.flat is not None:
            self.flat.zero_()
        else:
            for p in self.params:
                p.grad = None
        if self.world > 1:
            self._arm()
        loss = self.step.loss()
        if out is not None:
            out.copy_(loss.detach())
        if self.world > 1:
            from . import kernels
            with kernels.no_grouped_lstm():         # bucket all-reduces may be in flight (kernels.NO_GROUPED_LSTM)
                loss.backward()
        else:
            loss.backward()
        return loss.detach() if out is None else out

    def _opt(self):
        if self.world > 1:
            self.flat.mul_(1.0 / self.world)
        elif self._found is not None:
            self._found.copy_(self._flag.ne(0)[0])    # world > 1: max over ranks, set in _finish_allreduce
        if self.step.clip is not None:
            torch.nn.utils.clip_grad_norm_(self.params, self.step.clip, foreach=True)
        self.opt.step()

    def eager(self):
        if self.broadcast_buffers:
            self.sync_buffers()
        self.loss = self._fwd_bwd()
        if self.world > 1:
            self._finish_allreduce()
        self._opt()
        self._poll_kernel_errors()
        return self.loss

    def capture(self):
        """Capture after eager warm-up (lazy MIOpen / hipBLASLt / Adam-state init done). world > 1: the
        optimizer step only (the forward/backward launches its collectives from autograd hooks)."""
        if not self.use_graph:
            return
        from . import GRAPH_CAPTURE_SAFE
        if not GRAPH_CAPTURE_SAFE:          # replays could run kernels with another node's arguments (__init__.py)
            self.use_graph = False
            return
        torch.cuda.synchronize()
        # hand the eager warm-up's cached blocks back: the graphs allocate from a private pool, which cannot reuse
        # them (Mamba-TasNet-L at B=64 keeps ~200 GB of activations and checkpoints per step)
        torch.cuda.empty_cache()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            if self.world == 1:
                # the step's loss lands in a buffer allocated outside the graph's private pool: the pool's block of
                # the in-graph loss tensor is not guaranteed to hold it after replay (observed on the avse1 step)
                loss_buf = torch.zeros((), device=self.dev, dtype=torch.float32)
                self.g_fb = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.g_fb, stream=s):
                    self._fwd_bwd(loss_buf)
                self.loss = loss_buf
            self.g_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_opt, stream=s):
                self._opt()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()

    def drop_graphs(self):
        self.g_fb = self.g_opt = None

    def __call__(self):
        if self.g_fb is None and self.g_opt is None:
            return self.eager()
        if self.broadcast_buffers:
            self.sync_buffers()
        if self.g_fb is not None:
            self.g_fb.replay()
        else:
            self.loss = self._fwd_bwd()
            self._finish_allreduce()
        self.g_opt.replay()
        self._poll_kernel_errors()
        return self.loss


def _dense(t):
    """t's strides address exactly numel() distinct elements (a permutation of a contiguous block)."""
    if t.numel() == 0:
        return False
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.size()) if sz > 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True


def _flatten_buffers(model, dev):
    """Rebind every floating / integer buffer of ``model`` to a view of one flat tensor per kind (shared
    buffers stay shared); returns (flat_float | None, flat_int | None)."""
    groups = {"f": [], "i": []}
    seen = {}
    for mod in model.modules():
        for name, buf in mod._buffers.items():
            if buf is None:
                continue
            key = id(buf)
            if key not in seen:
                kind = "f" if buf.is_floating_point() else "i"
                seen[key] = (kind, len(groups[kind]), buf)
                groups[kind].append(buf)
    flats = {}
    for kind, bufs in groups.items():
        if not bufs:
            flats[kind] = None
            continue
        if kind == "f" and any(b.dtype != torch.float32 for b in bufs) or \
                kind == "i" and any(b.dtype != torch.int64 for b in bufs):
            raise RuntimeError("buffer broadcast expects fp32 floating and int64 integer buffers")
        flat = torch.empty(sum(b.numel() for b in bufs), device=dev, dtype=bufs[0].dtype)
        views, off = [], 0
        for b in bufs:
            v = flat[off:off + b.numel()].view(b.shape)
            v.copy_(b)
            views.append(v)
            off += b.numel()
        flats[kind] = (flat, views)
    for mod in model.modules():
        for name, buf in list(mod._buffers.items()):
            if buf is not None:
                kind, j, _ = seen[id(buf)]
                mod._buffers[name] = flats[kind][1][j]
    return tuple(None if flats[k] is None else flats[k][0] for k in ("f", "i"))
