"""avse1 captured step (one stream): where does the in-graph loss tensor's block get overwritten? (diagnostic)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
os.environ["AVSE_AVSE1_STREAMS"] = "0"


def run(variant):
    torch.manual_seed(5)
    st = bench.Avse1Step(2, dev, 0, 1, 96)
    tr = bench.Trainer(st, 1, dev, use_graph=True)
    losses = [float(tr())]
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    before, after = torch.zeros((), device=dev), torch.zeros((), device=dev)
    keep = {}
    with torch.cuda.stream(s):
        tr.g_fb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(tr.g_fb, stream=s):
            tr.flat.zero_()
            loss = st.loss()
            before.copy_(loss.detach())
            if variant == "no_bwd_graph":
                pass
            else:
                loss.backward()
            after.copy_(loss.detach())
            keep["loss"] = loss.detach()
        tr.g_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(tr.g_opt, stream=s):
            tr._opt()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    for _ in range(3):
        tr.g_fb.replay()
        torch.cuda.synchronize()
        a, b, c = float(before), float(after), float(keep["loss"])
        tr.g_opt.replay()
        torch.cuda.synchronize()
        d = float(keep["loss"])
        losses.append((round(a, 6), round(b, 6), round(c, 6), round(d, 6)))
    print(variant, "eager0", losses[0], "(before bwd, after bwd, tensor after fb, tensor after opt):", losses[1:],
          "loss ptr", hex(keep["loss"].data_ptr()), flush=True)


run("full")
