"""MI355X parity at feature widths that are not multiples of 8 (dfcsa/chanpad.py) against the
reference's own runs (tests/golden/oddw_*.npz, make_golden.py gen_oddwidth): features 10, 12, 20,
27 (stored padded to 16, 16, 24, 32; bottleneck 54 -> 56; attention q/k widths 1..6 -> 8), pool
4, 32x32, batch 2, one train-mode forward + backward and one clip + SGD step.

Tolerances as for the other model fixtures (fp32 compute mode): logits 1e-4 relative, loss 1e-4,
Dice 1e-6, running statistics 1e-4, gradients by check_grads against the float64 reference (tol
2e-3, scaled by the reference's own fp32 noise).  The padded channels' gradients must be exactly
zero (that is what keeps the padding inert through training).
"""
import types

import numpy as np
import pytest
import torch

from test_cpu_oddwidth import ODD, odd_model, sd_of
from test_gpu_fra_unet import LP, T, check_grads, rel

pytestmark = pytest.mark.gpu


def _step(name, fx, precision="fp32"):
    from dfcsa.loss import sigmoid
    from utils.metrics import calculate_metrics
    m = odd_model(name)
    m.set_precision(precision)
    m.load_state_dict(sd_of(fx, "sd0."))
    m = m.cuda().train()
    logits = m(T(fx["x"]))
    met = calculate_metrics(sigmoid(logits), T(fx["t"]), "bce_dice", LP)
    return m, logits, met


@pytest.mark.parametrize("name", ODD)
def test_odd_width_model_fp32_matches_reference(golden, name):
    from dfcsa import chanpad
    from dfcsa.optim import FusedSGD
    fx = golden(f"oddw_{name}.npz")
    m, logits, met = _step(name, fx)
    met["loss"].backward()
    torch.cuda.synchronize()
    assert tuple(logits.shape) == tuple(fx["logits"].shape)
    assert rel(logits, fx["logits"]) < 1e-4
    assert abs(met["loss"].item() - float(fx["loss"])) < 1e-4 * abs(float(fx["loss"]))
    assert abs(met["dice"] - float(fx["dice"])) < 1e-6
    sd = m.state_dict()
    for k in fx:
        if k.startswith("buf.") and "running" in k:
            assert rel(sd[k[4:]], fx[k]) < 1e-4, k
    named = []
    for n, p in m.named_parameters():
        g = chanpad.logical(p, p.grad)
        if hasattr(p, "_dfcsa_pad"):
            assert torch.equal(p._dfcsa_pad.pad(g), p.grad), f"{n}: nonzero gradient in a padded channel"
        named.append((n, types.SimpleNamespace(grad=g)))
    check_grads(named, fx, prefix="grad64.", tol=2e-3)

    # one clip(1.0) + SGD(0.05, 0.9, 1e-4) step through the fused optimizer
    opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    opt.step(max_norm=1.0)
    torch.cuda.synchronize()
    assert abs(opt.last_norm.item() - float(fx["norm"])) < 2e-3 * float(fx["norm"])
    mom_ref = sd_of(fx, "mom1.")
    osd = opt.state_dict()
    params = opt.param_groups[0]["params"]
    names = [n for n, _ in m.named_parameters()]
    ours = torch.cat([osd["state"][i]["momentum_buffer"].double().cpu().reshape(-1) for i in range(len(params))])
    ref = torch.cat([mom_ref[n].double().reshape(-1) for n in names])
    assert ours.numel() == ref.numel()
    assert rel(ours, ref) < 2e-3
    sd1 = m.state_dict()
    sd0 = sd_of(fx, "sd0.")
    new = torch.cat([sd1[n].double().cpu().reshape(-1) for n in names])
    exp = torch.cat([(sd0[n].double() - 0.05 * mom_ref[n].double()).reshape(-1) for n in names])
    assert rel(new, exp) < 1e-5
    for n, p in m.named_parameters():   # the padding is still exactly zero after the step
        if hasattr(p, "_dfcsa_pad"):
            assert torch.equal(p._dfcsa_pad.pad(chanpad.logical(p)), p.data), n


@pytest.mark.parametrize("name", ["UNetDFCSARes", "UNet_FullResAttention"])
def test_odd_width_model_bf16_near_reference(golden, name):
    """The bf16 compute mode at odd widths: logits and loss within the bf16 model-level bounds the
    other fixtures use (5e-2 relative)."""
    fx = golden(f"oddw_{name}.npz")
    m, logits, met = _step(name, fx, "bf16")
    met["loss"].backward()
    torch.cuda.synchronize()
    assert rel(logits, fx["logits"]) < 5e-2
    assert abs(met["loss"].item() - float(fx["loss"])) < 5e-2 * abs(float(fx["loss"]))
    assert all(torch.isfinite(p.grad).all() for p in m.parameters())



STANDALONE = ("oddw_lsa_C12_P4.npz", "oddw_lsa_C20_P8.npz", "oddw_lsa_C27_P16.npz", "oddw_block_5to12_P4.npz",
              "oddw_block_12to20_P8.npz", "oddw_block_16to27_P4.npz")


def standalone_module(fname):
    """The module of a standalone odd-width fixture, built as the reference built it (same seed)."""
    from models.unet_dfc_sa_res import DynamicFusionConvAttnBlock, LightSelfAttention
    parts = fname[:-4].split("_")
    P = int(parts[-1][1:])
    if parts[1] == "lsa":
        C = int(parts[2][1:])
        torch.manual_seed(9700 + C)
        return LightSelfAttention(C, pool_size=P, ablation_on_qk_channels=8)
    cin, cout = (int(v) for v in parts[2].split("to"))
    torch.manual_seed(9900 + cin * 10 + cout)
    return DynamicFusionConvAttnBlock(cin, cout, pool_size=P, ablation_on_qk_channels=8)


@pytest.mark.parametrize("fname", STANDALONE)
def test_standalone_odd_width_matches_reference(golden, fname):
    """A LightSelfAttention / DynamicFusionConvAttnBlock built on its own at a width that is not a
    multiple of 8 (reference models/unet_dfc_sa_res.py:5-116 accepts any; chanpad.pad_standalone pads
    it at construction, the NCHW forward returns the logical channels) against the reference's own
    run (tests/golden/oddw_lsa_* / oddw_block_*, make_golden.gen_oddwidth_standalone): fp32 mode,
    train-mode forward + backward; y 1e-5 relative, dx 1e-4 against the float64 reference, parameter
    gradients by check_grads (tol 2e-3, scaled by the reference's own fp32 noise); the padded
    channels' gradients exactly zero."""
    from dfcsa import chanpad
    fx = golden(fname)
    m = standalone_module(fname)
    m.load_state_dict(sd_of(fx, "sd0."))
    with torch.no_grad():
        (m.gamma if hasattr(m, "gamma") else m.attn_branch[3].gamma).fill_(0.6 if hasattr(m, "gamma") else 0.5)
    m = m.cuda().train()
    m.compute_dtype = torch.float32
    x = T(fx["x"]).requires_grad_(True)
    y = m(x)
    assert tuple(y.shape) == tuple(fx["y"].shape)
    y.backward(T(fx["g"]))
    torch.cuda.synchronize()
    assert rel(y, fx["y64"]) < 1e-5
    assert rel(x.grad, fx["dx64"]) < 1e-4
    named = []
    for n, p in m.named_parameters():
        g = chanpad.logical(p, p.grad)
        if hasattr(p, "_dfcsa_pad"):
            assert torch.equal(p._dfcsa_pad.pad(g), p.grad), f"{n}: nonzero gradient in a padded channel"
        named.append((n, types.SimpleNamespace(grad=g)))
    check_grads(named, fx, prefix="grad64.", tol=2e-3)
    if "sd1.running_mean" in str(list(fx)):
        sd = m.state_dict()
        for k in fx:
            if k.startswith("sd1.") and "running" in k:
                assert rel(sd[k[4:]], fx[k]) < 1e-4, k
