"""Times the lip-trunk shortcut input-gradient GEMMs (hipBLASLt vs the split-fp16 GEMM, alone on the GPU) and the avse1 FusionNet LSTM GEMMs at C2 (B = 32, T = 376, I = 1540, H = 257) one by one, to attribute the step's
once-per-step library GEMMs (profiles/r06u_avse1_timed_window_stats.csv) and A/B the weight-gradient forms."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402


def ev_ms(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def shortcut_dgrad(dev):
    for rows, cout, cin in ((21600, 512, 256), (86400, 256, 128), (345600, 128, 64)):
        dy2 = torch.randn(rows, cout, device=dev)
        wm = torch.randn(cout, cin, device=dev)
        sd = K.split_planes(dy2[None])
        out = torch.empty((1, rows, cin), device=dev)
        lib = ev_ms(lambda: dy2 @ wm)
        own = ev_ms(lambda: K.gemm_f32s_split(K.split_planes(wm[None]).t(), sd, out))
        own_split = ev_ms(lambda: K.gemm_f32s_split(K.split_planes(wm[None]).t(), K.split_planes(dy2[None]), out))
        ref = dy2.double() @ wm.double()
        K.gemm_f32s_split(K.split_planes(wm[None]).t(), sd, out)
        err = float((out[0].double() - ref).abs().max() / ref.abs().max())
        print(json.dumps({"shortcut_dgrad": [rows, cout, cin], "hipblaslt_ms": round(lib, 4),
                          "split_gemm_ms": round(own, 4), "split_gemm_with_dy_split_ms": round(own_split, 4),
                          "split_rel_err": err}), flush=True)


def main():
    dev = torch.device("cuda")
    shortcut_dgrad(dev)
    B, T, I, H = 32, 376, 1540, 257
    x2 = torch.randn(B * T, I, device=dev)
    w_ih = torch.randn(4 * H, I, device=dev)
    b = torch.randn(4 * H, device=dev)
    dg = torch.randn(B * T, 4 * H, device=dev)
    hprev = torch.randn(B, T, H, device=dev)
    rows = {
        "fwd addmm x2 w_ih^T": lambda: torch.addmm(b, x2, w_ih.t()),
        "bwd dx = dg w_ih": lambda: dg @ w_ih,
        "bwd dw_ih = dg^T x2": lambda: dg.t() @ x2,
        "bwd dw_ih bmm+sum": lambda: torch.bmm(dg.view(B, T, 4 * H).transpose(1, 2), x2.view(B, T, I)).sum(0),
        "bwd dw_hh = dg^T hprev (one GEMM)": lambda: dg.t() @ hprev.view(B * T, H),
        "bwd dw_hh bmm+sum": lambda: torch.bmm(dg.view(B, T, 4 * H).transpose(1, 2), hprev).sum(0),
        "bwd db = dg.sum(0)": lambda: dg.sum(0),
    }
    ref = (dg.double().t() @ hprev.view(B * T, H).double())
    err = float(((torch.bmm(dg.view(B, T, 4 * H).transpose(1, 2), hprev).sum(0).double() - ref).abs().max()
                 / ref.abs().max()))
    for k, f in rows.items():
        print(json.dumps({"gemm": k, "ms": round(ev_ms(f), 4)}), flush=True)
    print(json.dumps({"dw_hh_bmm_rel_err_vs_fp64": err}))


if __name__ == "__main__":
    main()
