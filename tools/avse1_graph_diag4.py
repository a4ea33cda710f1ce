"""avse1 captured fwd+bwd on one stream: which in-graph values are wrong on replay? (diagnostic)"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
os.environ["AVSE_AVSE1_STREAMS"] = "0"
torch.manual_seed(5)
st = bench.Avse1Step(2, dev, 0, 1, 96)
for m in st.model.modules():
    if isinstance(m, torch.nn.Dropout):
        m.p = 0.0
tr = bench.Trainer(st, 1, dev, use_graph=True)
tr()                                            # eager warm-up step
torch.cuda.synchronize()
torch.cuda.empty_cache()
av = st.avse1.AVNet
out = {k: torch.zeros((), device=dev) for k in ("l1", "sum_abs", "pred_sum", "mask_sum", "spec_sum")}
keep = {}


def fb():
    tr.flat.zero_()
    batch = av.features_from_waves(st.noisy, st.clean)
    batch["lip_images"] = st.lips
    pred = st.model(batch)
    l1 = F.l1_loss(pred, batch["mask"])
    out["l1"].copy_(l1.detach())
    out["sum_abs"].copy_((pred - batch["mask"]).abs().sum().detach() / pred.numel())
    out["pred_sum"].copy_(pred.detach().sum())
    out["mask_sum"].copy_(batch["mask"].sum())
    out["spec_sum"].copy_(batch["noisy_audio_spec"].sum())
    keep["pred"] = pred.detach()
    l1.backward()


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fb()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
for r in range(3):
    g.replay()
    torch.cuda.synchronize()
    got = {k: round(float(v), 6) for k, v in out.items()}
    pg = keep["pred"].clone()
    fb()                                        # eager, same weights (no optimizer step in between)
    torch.cuda.synchronize()
    ref = {k: round(float(v), 6) for k, v in out.items()}
    print(f"replay {r}: graph {got}\n          eager {ref}\n          max|pred_graph - pred_eager| "
          f"{float((pg - keep['pred']).abs().max()):.3e}", flush=True)
