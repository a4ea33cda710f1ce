"""Data-parallel training harness (bench.Trainer) on CPU with gloo, world_size 2: one flat-gradient
all-reduce per step must give every rank the same weights, equal to single-process training on the
union of the ranks' batches (mean of per-rank gradients, i.e. DDP semantics)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _ToyStep:
    def __init__(self, x, y, clip=None):
        torch.manual_seed(0)
        self.model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 2))
        self.model.register_buffer("seen", torch.zeros(1))
        self.x, self.y, self.lr, self.clip = x, y, 1e-2, clip

    def loss(self):
        return torch.nn.functional.mse_loss(self.model(self.x), self.y)


def _data(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(4, 8, generator=g), torch.randn(4, 2, generator=g)


def _worker(rank, world, port, clip, q):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    if rank == 1:                                   # different init on rank 1: Trainer must broadcast rank 0's
        torch.manual_seed(123)
    st = _ToyStep(*_data(rank), clip)
    if rank == 1:
        with torch.no_grad():
            for p in st.model.parameters():
                p.add_(1.0)
    tr = bench.Trainer(st, world, torch.device("cpu"), use_graph=False)
    for _ in range(3):
        tr()
    q.put((rank, [p.detach().numpy().copy() for p in st.model.parameters()]))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("clip", [None, 0.05])
def test_trainer_gloo_world2_matches_single_process(clip):
    sys.path.insert(0, REPO)
    import bench
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, clip, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = {r: [torch.from_numpy(a) for a in v] for r, v in res.items()}
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)
    # single process on the union batch: mean-of-means == mean over the concatenation (equal batch sizes)
    xs, ys = zip(*(_data(r) for r in range(2)))
    st = _ToyStep(torch.cat(xs), torch.cat(ys), clip)
    tr = bench.Trainer(st, 1, torch.device("cpu"), use_graph=False)
    for _ in range(3):
        tr()
    for a, b in zip(res[0], st.model.parameters()):
        torch.testing.assert_close(a, b.detach(), atol=1e-6, rtol=1e-5)
