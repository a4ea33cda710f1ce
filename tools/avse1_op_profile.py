"""torch.profiler view of one eager avse1 C2 train step (bench.Avse1Step, B=32; --workload: C3 / C4 / C5): device time per aten op and input
shapes, to attribute the copy / transpose / add kernels of the step to their callers.
python tools/avse1_op_profile.py [--batch 32] [--top 40] [--kernels PATTERN]
--kernels PAT[/PAT...]: instead of the op table, list every launch of a kernel whose name contains PATTERN with the
aten op that launched it, its input shapes and the innermost avse_challenge_amd / bench source line on the stack."""
import argparse
import collections
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _site(ev):
    for fr in ev.stack or []:
        if "avse_challenge_amd" in fr or "bench.py" in fr:
            return fr.split("/")[-1]
    return "?"


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--top", type=int, default=40)
    p.add_argument("--kernels", default=None)
    p.add_argument("--workload", default="avse1", choices=["avse1", "mamba", "avse4", "avmamba"],
                   help="the bench step to profile (batch: --batch, default the BASELINE config's)")
    a = p.parse_args()
    # the profiler's post-processing (with stacks) can run for minutes without output: keep a heartbeat on stdout
    threading.Thread(target=lambda: [print(f"alive {i * 30}s", flush=True) or time.sleep(30) for i in range(10 ** 6)],
                     daemon=True).start()
    dev = torch.device("cuda")
    if a.workload == "avse1":
        st = bench.Avse1Step(a.batch, dev, 0, 1, 96)
    elif a.workload == "avse4":
        st = bench.Avse4Step(a.batch if a.batch != 32 else 16, dev, 0, 1)
    else:
        cls = bench.MambaStep if a.workload == "mamba" else bench.AVMambaStep
        st = cls(a.batch if a.batch != 32 or a.workload == "avmamba" else 64, dev, 0, 1, "L")
    params = [q for q in st.model.parameters()]

    def step():
        for q in params:
            q.grad = None
        st.loss().backward()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=a.kernels is not None) as prof:
        step()
        torch.cuda.synchronize()
    if a.kernels is None:
        print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=a.top,
                                                                 max_name_column_width=60,
                                                                 max_shapes_column_width=90))
        return
    # kernel -> launching op: the innermost CPU op whose kernels list holds it (autograd backward ops run on a
    # separate thread; their stack is empty, so the site column names the forward op's node instead)
    for pat in a.kernels.split("/"):
        rows = collections.defaultdict(lambda: [0, 0.0])
        for ev in prof.events():
            for k in ev.kernels:
                if pat not in k.name:
                    continue
                key = (k.name[:50], ev.name, str(ev.input_shapes)[:110], _site(ev))
                rows[key][0] += 1
                rows[key][1] += k.duration / 1000.0
        total = sum(v[1] for v in rows.values())
        print(f"\nkernels matching {pat!r}: {sum(v[0] for v in rows.values())} launches, {total:.3f} ms")
        for key, (n, ms) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:a.top]:
            print(f"{ms:9.3f} ms {n:4d}x  {key[1]:32s} {key[3]:28s} {key[2]}  [{key[0]}]")


if __name__ == "__main__":
    main()
