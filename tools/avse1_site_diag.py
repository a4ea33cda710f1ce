"""Per-site diagnosis of the avse1 train-step gradient error (the test_avse1_wave_frontend_and_train_step_vs_oracle
setting: det_init 55, inputs 603-605, lips 2x3x75x64x64, dropout 0).

For every BatchNorm -> [+res] -> act site of the lip ResNet trunk (and the front-end), in OUR run (HIP bn_act,
channels-last or NCHW trunk) and in the stock PyTorch-ROCm run of the oracle (torch-GPU), against the fp64 oracle:
  ex     max|x - x64| / max|x64|         (the site's BN input: forward error accumulated upstream)
  edy    max|dy - dy64| / max|dy64|      (the gradient reaching the site's output: backward error upstream)
  flips  elements whose pre-activation sign differs from fp64's (activation-mask flips at this site)
  eloc   the site's bias gradient vs fp64 arithmetic on the SAME (x, res, dy) the run fed it (kernel error)
  eup    fp64 arithmetic on the run's (x, res, dy) vs the fp64 truth (error carried in by x / dy)
  ebias  the run's bias gradient vs truth (what the test bounds), all relative to max|truth|.
Usage: python tools/avse1_site_diag.py [cl|nchw]"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import avse_challenge_amd  # noqa: E402,F401
from avse_challenge_amd import avse1  # noqa: E402
from oracle import avse1_ref, stft_ref  # noqa: E402
from oracle.det_init import det_init_, det_input  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
LAYOUT = sys.argv[1] if len(sys.argv) > 1 else "cl"
noisy = 0.1 * det_input((2, 48000), 603)
clean = 0.1 * det_input((2, 48000), 604)
lips = det_input((2, 3, 75, 64, 64), 605, "uint8")
rb = {"noisy_audio_spec": torch.from_numpy(stft_ref.stft_mag_T(noisy.numpy()))[:, None],
      "mask": torch.from_numpy(stft_ref.stft_mag_T(clean.numpy()))[:, None], "lip_images": lips}
rbg = {k: v.cuda() for k, v in rb.items()}


def nodrop(m):
    for x in m.modules():
        if isinstance(x, torch.nn.Dropout):
            x.p = 0.0
    return m


def hook_ref(model):
    """Capture (x, res, dy) at every BN site of the oracle's VisualFeatNet (BN input, shortcut, act-output grad)."""
    cap = {}
    vf = model.net_visualfeat
    names = {id(m): n for n, m in vf.named_modules()}

    def grab_in(n):
        def h(mod, inp, out):
            cap.setdefault(n, {})["x"] = inp[0].detach().double().cpu()
        return h

    def grab_dy(n):
        def h(mod, inp, out):
            out.register_hook(lambda g: cap.setdefault(n, {}).__setitem__("dy", g.detach().double().cpu()))
        return h

    fe = vf.frontend3D
    fe[1].register_forward_hook(grab_in("frontend3D.1"))
    fe[2].register_forward_hook(grab_dy("frontend3D.1"))
    for n, m in vf.trunk.named_modules():
        if isinstance(m, avse1_ref.BasicBlock):
            p = "trunk." + n
            m.bn1.register_forward_hook(grab_in(p + ".bn1"))
            m.relu1.register_forward_hook(grab_dy(p + ".bn1"))
            m.bn2.register_forward_hook(grab_in(p + ".bn2"))
            m.relu2.register_forward_hook(grab_dy(p + ".bn2"))
            if m.downsample is not None:
                m.downsample[1].register_forward_hook(grab_in(p + ".downsample.1"))
                m.downsample[1].register_forward_hook(grab_dy(p + ".downsample.1"))

                def shortcut(mod, inp, out, p=p):
                    cap.setdefault(p + ".bn2", {})["res"] = out.detach().double().cpu()
                m.downsample.register_forward_hook(shortcut)
            else:
                def shortcut_id(mod, inp, out, p=p):
                    cap.setdefault(p + ".bn2", {})["res"] = inp[0].detach().double().cpu()
                m.register_forward_hook(shortcut_id)
    del names
    return cap


def run_ours():
    m = nodrop(det_init_(avse1.AVNet(), 55).cuda().train())
    if LAYOUT == "cl":
        m.net_audiofeat.use_channels_last()
        m.net_visualfeat.use_channels_last()
    vf = m.net_visualfeat
    names = {id(mod): n for n, mod in vf.named_modules()}
    cap = {}
    orig = avse1.bn_act

    def spy(x, bn, act=None, res=None):
        y = orig(x, bn, act, res)
        n = names.get(id(bn))
        if n is not None:
            d = cap.setdefault(n, {})
            d["x"] = x.detach().double().cpu()
            if res is not None:
                d["res"] = res.detach().double().cpu()
            y.register_hook(lambda g, d=d: d.__setitem__("dy", g.detach().double().cpu()))
        return y

    avse1.bn_act = spy
    try:
        m.training_step(dict(rbg)).backward()
    finally:
        avse1.bn_act = orig
    torch.cuda.synchronize()
    return m, cap


def local_grads(x, res, dy, bn, act_w):
    """fp64 BN(train) [+res] -> act backward on the given tensors: (dbeta, dgamma, z)."""
    g = bn.weight.detach().double().cpu().clone().requires_grad_(True)
    b = bn.bias.detach().double().cpu().clone().requires_grad_(True)
    dims = [0] + list(range(2, x.dim()))
    mean = x.mean(dims, keepdim=True)
    var = x.var(dims, unbiased=False, keepdim=True)
    shp = [1, -1] + [1] * (x.dim() - 2)
    z = (x - mean) / torch.sqrt(var + bn.eps) * g.view(shp) + b.view(shp)
    if res is not None:
        z = z + res
    if act_w is None:
        y = z
    else:
        y = F.prelu(z, act_w.detach().double().cpu())
    y.backward(dy)
    return b.grad, g.grad, z.detach()


r64 = nodrop(det_init_(avse1_ref.AVNet(), 55).double().train())
c64 = hook_ref(r64)
r64.cal_loss({k: (v.double() if v.dtype == torch.float32 else v) for k, v in rb.items()}).backward()
tg = nodrop(det_init_(avse1_ref.AVNet(), 55).cuda().train())
ctg = hook_ref(tg)
tg.cal_loss(dict(rbg)).backward()
ours, co = run_ours()

mods64 = dict(r64.net_visualfeat.named_modules())
modso = dict(ours.net_visualfeat.named_modules())
modstg = dict(tg.net_visualfeat.named_modules())


def act_of(mods, site):
    if site == "frontend3D.1":
        return mods["frontend3D.2"].weight
    if site.endswith("downsample.1"):
        return None
    blk = site.rsplit(".", 1)[0]
    return mods[blk + (".relu1" if site.endswith("bn1") else ".relu2")].weight


print(f"layout {LAYOUT}")
print(f"{'site':26s} {'run':5s} {'ex':>9s} {'edy':>9s} {'flips':>6s} {'eloc':>9s} {'eup':>9s} {'ebias':>9s} "
      f"{'edgam':>9s} {'n':>8s}")
for site in c64:
    t = c64[site]
    truth_b = mods64[site].bias.grad
    truth_g = mods64[site].weight.grad
    sc_b = float(truth_b.abs().max())
    sc_g = float(truth_g.abs().max())
    _, _, z64 = local_grads(t["x"], t.get("res"), t["dy"], mods64[site], act_of(mods64, site))
    for run, cap, mods in (("ours", co, modso), ("tgpu", ctg, modstg)):
        c = cap.get(site)
        if c is None or "dy" not in c:
            print(f"{site:26s} {run:5s} (not captured)")
            continue
        x = c["x"]
        if x.shape != t["x"].shape:
            print(f"{site:26s} {run:5s} shape {tuple(x.shape)} vs {tuple(t['x'].shape)}")
            continue
        ex = float((x - t["x"]).abs().max() / t["x"].abs().max())
        edy = float((c["dy"] - t["dy"]).abs().max() / t["dy"].abs().max())
        db_loc, dg_loc, z = local_grads(x, c.get("res"), c["dy"], mods[site], act_of(mods, site))
        flips = int(((z > 0) != (z64 > 0)).sum()) if act_of(mods, site) is not None else 0
        gb = mods[site].bias.grad.double().cpu()
        gg = mods[site].weight.grad.double().cpu()
        eloc = float((gb - db_loc).abs().max()) / sc_b
        eup = float((db_loc - truth_b).abs().max()) / sc_b
        ebias = float((gb - truth_b).abs().max()) / sc_b
        edg = float((gg - truth_g).abs().max()) / sc_g
        print(f"{site:26s} {run:5s} {ex:9.2e} {edy:9.2e} {flips:6d} {eloc:9.2e} {eup:9.2e} {ebias:9.2e} {edg:9.2e} "
              f"{x.numel():8d}", flush=True)
    # where the largest bias error sits for ours: channel, and the fp64 |z| of the flipped elements there
    c = co.get(site)
    if c is not None and "dy" in c and c["x"].shape == t["x"].shape and act_of(modso, site) is not None:
        gb = modso[site].bias.grad.double().cpu()
        ch = int((gb - truth_b).abs().argmax())
        _, _, z = local_grads(c["x"], c.get("res"), c["dy"], modso[site], act_of(modso, site))
        fl = ((z > 0) != (z64 > 0))
        nfl_ch = int(fl[:, ch].sum())
        zabs = float(z64[:, ch][fl[:, ch]].abs().max()) if nfl_ch else 0.0
        print(f"{'':26s} worst channel {ch}: flips there {nfl_ch}, max |z64| of flipped {zabs:.2e}, "
              f"truth {float(truth_b[ch]):.3e} ours {float(gb[ch]):.3e} |dy64| max there "
              f"{float(t['dy'][:, ch].abs().max()):.3e}", flush=True)
