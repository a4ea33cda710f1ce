"""avse1 train step: eager vs captured-graph losses for the branch-stream / channels-last variants (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
for cl in ("1", "0"):
    for streams in ("0", "1"):
        for graph in (False, True):
            os.environ["AVSE_AVSE1_STREAMS"] = streams
            os.environ["AVSE_CHANNELS_LAST"] = cl
            torch.manual_seed(5)
            st = bench.Avse1Step(2, dev, 0, 1, 96)
            tr = bench.Trainer(st, 1, dev, use_graph=graph)
            losses = [float(tr())]
            if graph:
                tr.capture()
            for _ in range(3):
                losses.append(float(tr()))
            torch.cuda.synchronize()
            pm = max(float(p.detach().abs().max()) for p in st.model.parameters())
            fin = all(bool(torch.isfinite(p).all()) for p in st.model.parameters())
            with torch.no_grad():
                chk = float(st.loss())
            print(f"cl={cl} streams={streams} graph={graph}: losses {[round(x, 6) for x in losses]} "
                  f"param max {pm:.4f} finite {fin} eager-loss-after {chk:.6f}", flush=True)
            del tr, st
            torch.cuda.empty_cache()
