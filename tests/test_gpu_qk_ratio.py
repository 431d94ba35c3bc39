"""The attention query/key width ratio (``ablation_on_qk_channels``, reference
models/unet_dfc_sa_res.py:8-13 and model_factory.py:87-91: q/k are C -> C // ratio 1x1 convs) at
ratios other than the shipped 8, including odd query widths (ratio 3: 5, 10, 16, 21, 42 channels)
and a width of 1 (ratio 16 at C = 16).

No reference run covers these ratios (every shipped config uses 8), so the check is against the
oracle (oracle/dfcsa_oracle.py, pinned to the reference's fixtures at ratio 8; it takes every width
from the state-dict shapes) run in float64 on the CPU on the same weights and batch: one train-mode
forward + backward of UNetDFCSARes at features 16, 32, 48, 64, pool 4, 32x32, batch 2, fp32 mode.
Tolerances as for the model fixtures: logits 1e-4 relative, loss 1e-4, gradients by check_grads
(tol 2e-3, scaled by the oracle's own fp32 distance to its float64 run) against the float64 run,
with an absolute floor of 1e-5 of the whole gradient's norm per tensor (see _fixture).
"""
import numpy as np
import pytest
import torch

from test_gpu_fra_unet import LP, T, check_grads, rel

pytestmark = pytest.mark.gpu


def _fixture(sd, x, t, pool, grads64):
    """check_grads' fixture layout from the float64 oracle run.  noise.<name> is the oracle's own
    fp32 distance to its float64 run (as make_golden.fp64_noise records the reference's), floored
    at 2e-6 |g_all| / |g_name|: check_grads then admits an error of 1e-5 of the whole gradient's
    norm on any tensor (round 6: 10x tighter than round 5's 2e-5 floor, which let a small-norm
    tensor -- gamma, res_scale, an attention bias -- be off by several percent).  The
    floor still matters for those block scalars, one cancelling sum each, whose fp32 error swings
    by 100x with the batch's composition (measured: the oracle's own fp32 error on one gamma is
    3e-2 at B = 15 and 4e-4 at B = 17 of the same images; tools/pool_path_diag2.py)."""
    from oracle import dfcsa_oracle as O
    _, _, grads32, _ = O.forward_backward(sd, x, t, pool, LP)
    fx, a, b = {}, [], []
    gall = torch.cat([g.reshape(-1) for g in grads64.values()]).norm().item()
    for k, g in grads64.items():
        fx["grad." + k] = g.float().numpy()
        fx["grad64." + k] = g.numpy()
        fx["noise." + k] = max(rel(grads32[k], g), 2e-6 * gall / max(g.norm().item(), 1e-30))
        a.append(grads32[k].double().reshape(-1))
        b.append(g.reshape(-1))
    fx["noise.all"] = rel(torch.cat(a), torch.cat(b))
    return fx


def _check(model, fx):
    check_grads(model.named_parameters(), fx, tol=2e-3)


@pytest.mark.parametrize("ratio", [2, 3, 4, 16])
def test_qk_ratio_model_matches_oracle(ratio):
    from dfcsa.loss import sigmoid
    from models.unet_dfc_sa_res import UNetDFCSARes
    from oracle import dfcsa_oracle as O
    from utils.metrics import calculate_metrics
    torch.manual_seed(4100 + ratio)
    m = UNetDFCSARes(3, 1, [16, 32, 48, 64], pool_size=4, ablation_on_qk_channels=ratio, precision="fp32")
    with torch.no_grad():
        for i, (n, p) in enumerate(sorted(m.named_parameters())):
            if n.endswith("gamma"):
                p.fill_(0.2 + 0.05 * (i % 9))
    assert m.down1.attn_branch[3].query_conv.out_channels == 16 // ratio
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    gen = torch.Generator().manual_seed(4200 + ratio)
    x = torch.randn(2, 3, 32, 32, generator=gen)
    t = (torch.rand(2, 1, 32, 32, generator=gen) > 0.5).float()

    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    logits64, met64, grads64, _ = O.forward_backward(sd64, x.double(), t.double(), 4, LP)

    m = m.cuda().train()
    logits = m(T(x.numpy()))
    met = calculate_metrics(sigmoid(logits), T(t.numpy()), "bce_dice", LP)
    met["loss"].backward()
    torch.cuda.synchronize()
    assert rel(logits, logits64) < 1e-4
    assert abs(met["loss"].item() - met64["loss"].item()) < 1e-4 * abs(met64["loss"].item())
    fx = _fixture(sd, x, t, 4, grads64)
    _check(m, fx)
    assert np.isfinite(met["loss"].item())


@pytest.mark.parametrize("P,B", [(16, 2), (32, 2), (16, 17), (32, 5)])
def test_large_pool_model_matches_oracle(P, B):
    """configs/config_dfc-sa-res-block-p16.yaml / -p32.yaml (pool_size 16 / 32): P x P pooled tokens
    (up to 1024), larger than the deeper levels' maps at 64 x 64 input (the adaptive pool then repeats
    pixels, reference :20-24), against the float64 oracle as above.  B * P^2 above 4096 takes the
    attention-entry backward off the projection kernel's extra rows (and, for P = 32, off the
    pool-fused finalize, which holds at most 256 tokens)."""
    from dfcsa.loss import sigmoid
    from models.unet_dfc_sa_res import UNetDFCSARes
    from oracle import dfcsa_oracle as O
    from utils.metrics import calculate_metrics
    torch.manual_seed(4300 + P)
    m = UNetDFCSARes(3, 1, [16, 32, 48, 64], pool_size=P, precision="fp32")
    with torch.no_grad():
        for i, (n, p) in enumerate(sorted(m.named_parameters())):
            if n.endswith("gamma"):
                p.fill_(0.2 + 0.05 * (i % 9))
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    gen = torch.Generator().manual_seed(4400 + P)
    x = torch.randn(B, 3, 64, 64, generator=gen)
    t = (torch.rand(B, 1, 64, 64, generator=gen) > 0.5).float()
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    logits64, met64, grads64, _ = O.forward_backward(sd64, x.double(), t.double(), P, LP)
    m = m.cuda().train()
    logits = m(T(x.numpy()))
    met = calculate_metrics(sigmoid(logits), T(t.numpy()), "bce_dice", LP)
    met["loss"].backward()
    torch.cuda.synchronize()
    assert rel(logits, logits64) < 1e-4
    assert abs(met["loss"].item() - met64["loss"].item()) < 1e-4 * abs(met64["loss"].item())
    fx = _fixture(sd, x, t, P, grads64)
    _check(m, fx)
