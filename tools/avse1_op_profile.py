"""torch.profiler view of one eager avse1 C2 train step (bench.Avse1Step, B=32): device time per aten op and input
shapes, to attribute the copy / transpose / add kernels of the step to their callers.
python tools/avse1_op_profile.py [--batch 32] [--top 40]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--top", type=int, default=40)
    a = p.parse_args()
    st = bench.Avse1Step(a.batch, torch.device("cuda"), 0, 1, 96)
    params = [q for q in st.model.parameters()]

    def step():
        for q in params:
            q.grad = None
        st.loss().backward()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=a.top,
                                                             max_name_column_width=60, max_shapes_column_width=90))


if __name__ == "__main__":
    main()
