"""DPMamba (dual-path Mamba) on the HIP kernels vs the fp64 CPU oracle on identical
det_init weights.  The BiMamba blocks are pinned by tests/golden; the dual-path wrapper (speechbrain's
Dual_Path_Model, un-vendored) is a restatement on both sides: parity of that part is unpinned."""
import pytest
import torch

from oracle import dpmamba_ref, losses_ref
from oracle.det_init import det_init_, det_input

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _fp32_exact():
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    yield


def close(a, b, atol, rtol, what=""):
    torch.testing.assert_close(a.detach().double().cpu(), b.detach().double().cpu(), atol=atol, rtol=rtol, msg=what)


@pytest.mark.parametrize("skip", [True, False])
def test_dpmamba_train_step_vs_oracle(skip):
    """Whole separator (N=64, 2 dual-path layers, chunk 250, 50 % overlap) fwd + every gradient vs fp64."""
    from avse_challenge_amd import dpmamba, losses as PL
    ours = det_init_(dpmamba.DPMambaTasNet(N=64, n_dp=2, skip_around_intra=skip), 31).to(DEV)
    ref = det_init_(dpmamba_ref.DPMambaTasNet(N=64, n_dp=2, skip_around_intra=skip), 31).double()
    mix = 0.1 * det_input((2, 4000), 701)                # L = 499 frames -> S = 5 chunks of 250
    tgt = 0.1 * det_input((2, 4000, 2), 702)
    est = ours(mix.to(DEV))
    est_r = ref(mix.double())
    close(est, est_r, 5e-5, 1e-4, "separated")
    loss = PL.si_snr_pit(tgt.to(DEV), est).mean()
    loss_r = losses_ref.si_snr_pit(tgt.double(), est_r).mean()
    assert abs(float(loss) - float(loss_r)) < 1e-3
    loss.backward()
    loss_r.backward()
    rp = dict(ref.named_parameters())
    for k, p in ours.named_parameters():
        r = rp[k].grad
        scale = max(1e-3, float(r.abs().max()))
        close(p.grad, r, 2e-3 * scale, 2e-3, k)


def test_dpmamba_L_width_fullsize_2_layers():
    """DPMamba-L widths (N=512, d_inner 1024) on a 4 s @ 8 kHz mixture (L=3999 -> 34 chunks of 250), 2 of the
    16 dual-path layers: RMS waveform error <= 1e-4 and SI-SDR within 0.01 dB of the fp64 oracle."""
    from test_gpu_fullsize import check_waveforms
    from avse_challenge_amd import data, dpmamba
    mix, tgt = data.wsj0mix_batch(1, "cpu", 14)
    ours = det_init_(dpmamba.DPMambaTasNet(N=512, n_dp=2), 74).to(DEV).eval()
    ref = det_init_(dpmamba_ref.DPMambaTasNet(N=512, n_dp=2), 74).double().eval()
    with torch.no_grad():
        est = ours(mix.to(DEV))
        est_r = ref(mix.double())
    check_waveforms(est.transpose(1, 2), est_r.transpose(1, 2), tgt.transpose(1, 2), "DPMamba-L (2 layers)")
