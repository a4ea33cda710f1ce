"""Launch the bench's roofline kernels at the bench shapes (for rocprofv3 PMC passes: tools/pmc_traffic.sh).

python tools/roofline_kernels.py PHASE [--n N]
PHASE: scan (Mamba-L C3 training scan fwd, B=64), scan_bwd (its backward as the model calls it), dwconv (avse4 C4 TCN dwconv fwd, B=16, dil 128),
       cconv (causal conv fwd, B=64, D=1024: the dword-access calibration kernel, known bytes),
       conv3 (avse1 C2 AudioFeatNet conv3 fwd, B=32, NHWC, MIOpen),
       dconv_wgrad (the same conv's weight gradient on csrc/dconv_wgrad.hip: the step's largest kernel class).
Inputs are created before a device sync, then the kernel runs N times; the PMC summary counts only
non-PyTorch kernels, so input generation does not enter the per-launch numbers.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avse_challenge_amd import kernels as K  # noqa: E402

SHAPES = {"scan": (64, 1024, 3999), "scan_bwd": (64, 1024, 3999), "dwconv": (16, 512, 3999), "cconv": (64, 1024, 3999),
          "conv3": (32, 64, 376, 257), "dconv_wgrad": (32, 64, 376, 257),
          "scan_c5": (32, 1024, 5999), "scan_bwd_c5": (32, 1024, 5999),
          "dwconv_gln": (16, 512, 3999), "dwconv_gln_bwd": (16, 512, 3999),
          "prelu_gln": (16, 512, 3999), "prelu_gln_bwd": (16, 512, 3999)}


def aligned(b, d, l, g, scale=1.0, dtype=torch.float32):
    """(b, d, l) with the product's 128-B aligned time stride (kernels.bdl_empty), filled N(0, scale^2)."""
    t = K.bdl_empty(b, d, l, dtype, "cuda")
    t.copy_(scale * torch.randn(b, d, l, device="cuda", generator=g))
    return t


def main():
    p = argparse.ArgumentParser()
    p.add_argument("phase", choices=sorted(SHAPES))
    p.add_argument("--n", type=int, default=5)
    a = p.parse_args()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    if a.phase.startswith("scan"):
        b, d, l = SHAPES[a.phase]
        dt = torch.bfloat16 if a.phase.endswith("_c5") else torch.float32
        u, dl, z = aligned(b, d, l, g, dtype=dt), aligned(b, d, l, g, 0.1, dt), aligned(b, d, l, g, dtype=dt)
        A = -torch.rand(d, 16, device=dev, generator=g) - 0.5
        Bm, Cm = aligned(b, 16, l, g, dtype=dt), aligned(b, 16, l, g, dtype=dt)
        D = torch.ones(d, device=dev)
        # as the model calls it (round 5): delta already softplus(dt_proj + bias) from avse_dtproj, mode 2
        dl.copy_(torch.nn.functional.softplus(dl.float()))
        fn = lambda: K.selective_scan_fwd(u, dl, A, Bm, Cm, D, z, None, 2, return_out=False)  # noqa: E731
        if a.phase.startswith("scan_bwd"):
            _, x, _ = fn()
            dout = aligned(b, d, l, g, dtype=dt)
            fn = lambda: K.selective_scan_bwd(u, dl, A, Bm, Cm, D, z, None, dout, x, None, None, 2, False)  # noqa: E731
    elif a.phase.startswith("prelu_gln"):
        x = torch.randn(*SHAPES["prelu_gln"], device=dev, generator=g)
        al, gm, bt = torch.full((1,), 0.25, device=dev), torch.ones(1, 512, 1, device=dev), torch.zeros(1, 512, 1, device=dev)
        fn = lambda: K.prelu_gln_fwd(x, al, gm, bt)  # noqa: E731
        if a.phase == "prelu_gln_bwd":
            _, st = fn()
            gy = torch.randn(*SHAPES["prelu_gln"], device=dev, generator=g)
            fn = lambda: K.prelu_gln_bwd(x, al, gm, st, gy)  # noqa: E731
    elif a.phase.startswith("dwconv_gln"):
        x = torch.randn(*SHAPES["dwconv_gln"], device=dev, generator=g)
        w = 0.5 * torch.randn(512, 1, 3, device=dev, generator=g)
        al, gm, bt = torch.full((1,), 0.25, device=dev), torch.ones(1, 512, 1, device=dev), torch.zeros(1, 512, 1, device=dev)
        fn = lambda: K.dwconv_gln_fwd(x, w, 128, al, gm, bt)  # noqa: E731
        if a.phase == "dwconv_gln_bwd":
            _, y1, st = fn()
            gy = torch.randn(*SHAPES["dwconv_gln"], device=dev, generator=g)
            fn = lambda: K.dwconv_gln_bwd(x, w, 128, y1, al, gm, st, gy)  # noqa: E731
    elif a.phase == "dwconv":
        x = torch.randn(*SHAPES["dwconv"], device=dev, generator=g)
        w = torch.randn(512, 1, 3, device=dev, generator=g)
        fn = lambda: K.dwconv_fwd(x, w, 128)  # noqa: E731
    elif a.phase == "cconv":
        b, d, l = SHAPES["cconv"]
        x = torch.randn(b, d, l, device=dev, generator=g)
        w, cb = torch.randn(d, 4, device=dev, generator=g), torch.randn(d, device=dev, generator=g)
        fn = lambda: K.causal_conv1d_fwd(x, w, cb, True)  # noqa: E731
    elif a.phase == "dconv_wgrad":
        cl = torch.channels_last
        x = torch.randn(*SHAPES["dconv_wgrad"], device=dev, generator=g).to(memory_format=cl)
        dy = torch.randn(*SHAPES["dconv_wgrad"], device=dev, generator=g).to(memory_format=cl)
        fn = lambda: K.dconv_wgrad(x, dy, 4)  # noqa: E731
    else:
        from avse_challenge_amd import avse1
        conv = avse1.AVNet().to(dev).net_audiofeat
        conv.use_channels_last()
        conv3 = conv.conv3
        x = torch.randn(*SHAPES["conv3"], device=dev, generator=g).to(memory_format=torch.channels_last)
        fn = lambda: conv3(x)  # noqa: E731
    with torch.no_grad():
        fn()
        torch.cuda.synchronize()
        for _ in range(a.n):
            fn()
        torch.cuda.synchronize()
    print(f"{a.phase}: {a.n + 1} launches", flush=True)


if __name__ == "__main__":
    main()
