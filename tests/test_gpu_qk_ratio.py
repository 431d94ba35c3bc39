"""The attention query/key width ratio (``ablation_on_qk_channels``, reference
models/unet_dfc_sa_res.py:8-13 and model_factory.py:87-91: q/k are C -> C // ratio 1x1 convs) at
ratios other than the shipped 8, including odd query widths (ratio 3: 5, 10, 16, 21, 42 channels)
and a width of 1 (ratio 16 at C = 16).

No reference run covers these ratios (every shipped config uses 8), so the check is against the
oracle (oracle/dfcsa_oracle.py, pinned to the reference's fixtures at ratio 8; it takes every width
from the state-dict shapes) run in float64 on the CPU on the same weights and batch: one train-mode
forward + backward of UNetDFCSARes at features 16, 32, 48, 64, pool 4, 32x32, batch 2, fp32 mode.
Tolerances as for the model fixtures: logits 1e-4 relative, loss 1e-4, gradients by check_grads
(tol 2e-3) against the float64 run.
"""
import numpy as np
import pytest
import torch

from test_gpu_fra_unet import LP, T, check_grads, rel

pytestmark = pytest.mark.gpu


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
    fx = {}
    for k, g in grads64.items():
        fx["grad." + k] = g.float().numpy()
        fx["grad64." + k] = g.numpy()
    check_grads(m.named_parameters(), fx, tol=2e-3)
    assert np.isfinite(met["loss"].item())
