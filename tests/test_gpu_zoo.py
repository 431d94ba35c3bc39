"""MI355X parity of the ablation model zoo (reference unet_dfc_sa_ablation_branches.py, _fusion.py,
_placement.py; model_factory.py:160-187) against the reference's own fp32 / float64 runs
(tests/golden/zoo_*.npz, make_golden.py gen_zoo): one train-mode forward + backward of every
model at features 8..64, pool 4, 32x32, through ModelFactory.

Tolerances as for the other model fixtures (fp32 compute mode): logits 1e-4 relative, loss 1e-4,
Dice 1e-6, BatchNorm running statistics 1e-4; gradients by check_grads against the float64
reference (tol 2e-3, scaled by the reference's own fp32 noise).
"""
import numpy as np
import pytest
import torch

from test_gpu_fra_unet import LP, T, check_grads, rel, sd_from

pytestmark = pytest.mark.gpu

ZOO = ("UNet_Baseline", "UNet_AttentionOnly", "UNet_AdditionFusion", "UNet_ConcatFusion", "UNet_EncoderOnlyDFC",
       "UNet_DecoderOnlyDFC", "UNet_BothStandardConv")


@pytest.mark.parametrize("name", ZOO)
def test_zoo_model_fp32_matches_reference(golden, name):
    from dfcsa.loss import sigmoid
    from models.model_factory import ModelFactory
    from utils.metrics import calculate_metrics
    fx = golden(f"zoo_{name}.npz")
    model = ModelFactory.get_model({"model": {"name": name, "features": [8, 16, 32, 64], "pool_size": 4,
                                              "precision": "fp32"}, "training": {}})
    model.load_state_dict(sd_from(fx, "sd0."))
    model = model.cuda().train()
    logits = model(T(fx["x"]))
    met = calculate_metrics(sigmoid(logits), T(fx["t"]), "bce_dice", LP)
    met["loss"].backward()
    torch.cuda.synchronize()
    assert rel(logits, fx["logits"]) < 1e-4
    assert abs(met["loss"].item() - float(fx["loss"])) < 1e-4 * abs(float(fx["loss"]))
    assert abs(met["dice"] - float(fx["dice"])) < 1e-6
    sd = model.state_dict()
    for k in fx:
        if k.startswith("buf.") and "running" in k:
            assert rel(sd[k[4:]], fx[k]) < 1e-4, k
    check_grads(model.named_parameters(), fx, tol=2e-3)


@pytest.mark.parametrize("name", ["UNet_ConcatFusion", "UNet_DecoderOnlyDFC"])
def test_zoo_model_bf16_train_steps(name):
    """bf16 at the default width (features 64..512) on 64x64: logits near the fp32 path on the
    same weights, finite decreasing loss over fused clip+SGD steps."""
    from dfcsa.loss import sigmoid
    from dfcsa.optim import FusedSGD
    from models.model_factory import ModelFactory
    from utils.metrics import calculate_metrics_device
    torch.manual_seed(5)
    cfg = {"model": {"name": name, "pool_size": 4, "precision": "fp32"}, "training": {}}
    m32 = ModelFactory.get_model(cfg)
    with torch.no_grad():
        for n, p in m32.named_parameters():
            if n.endswith("gamma"):
                p.fill_(0.5)
    m16 = ModelFactory.get_model({"model": dict(cfg["model"], precision="bf16"), "training": {}})
    m16.load_state_dict(m32.state_dict())
    m32, m16 = m32.cuda().train(), m16.cuda().train()
    x = torch.randn(4, 3, 64, 64, device="cuda")
    t = (torch.rand(4, 1, 64, 64, device="cuda") > 0.5).float()
    assert rel(m16(x), m32(x)) < 5e-2
    opt = FusedSGD(m16.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    losses = []
    for _ in range(6):
        opt.zero_grad()
        met = calculate_metrics_device(sigmoid(m16(x)), t, "bce_dice", LP)
        met["loss"].backward()
        opt.step(max_norm=1.0, skip_if_nan=met["loss"])
        losses.append(met["loss"].item())
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses
