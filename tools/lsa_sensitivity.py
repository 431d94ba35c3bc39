"""Is the P = 16, B = 2 model gradient of tests/test_gpu_qk_ratio.py::test_large_pool_model_matches_oracle
well conditioned?  The float64 oracle's forward + backward, with the pooled attention's output o of
every block perturbed by relative noise of size eps (fp32 rounding is ~6e-8), against the unperturbed
float64 run: a smooth function moves its gradient by O(eps); a ReLU / max-pool decision that a
perturbation this small flips moves it by O(1) on the tensors that sum over the flipped element.

  python tools/lsa_sensitivity.py [P B eps nseeds]
"""
import sys

import torch

sys.path[:0] = ["dfc-sa-unet_amd", ".", "tests"]
from models.unet_dfc_sa_res import UNetDFCSARes  # noqa: E402
from oracle import dfcsa_oracle as O  # noqa: E402

P, B = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (16, 2)
eps = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-7
nseeds = int(sys.argv[4]) if len(sys.argv) > 4 else 4
LP = {"bce_weight": 0.5, "dice_weight": 0.5}
torch.manual_seed(4300 + P)
m0 = UNetDFCSARes(3, 1, [16, 32, 48, 64], pool_size=P, precision="fp32")
with torch.no_grad():
    for i, (n, p) in enumerate(sorted(m0.named_parameters())):
        if n.endswith("gamma"):
            p.fill_(0.2 + 0.05 * (i % 9))
sd = {k: (v.detach().double() if v.is_floating_point() else v) for k, v in m0.state_dict().items()}
gen = torch.Generator().manual_seed(4400 + P)
x = torch.randn(B, 3, 64, 64, generator=gen).double()
t = (torch.rand(B, 1, 64, 64, generator=gen) > 0.5).double()
orig = O.light_self_attention


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-300)).item()


_, _, g0, _ = O.forward_backward(sd, x, t, P, LP)
for s in range(nseeds):
    ng = torch.Generator().manual_seed(s)

    def noisy(a, sd_, name, pool_size, _g=ng):
        y = orig(a, sd_, name, pool_size)
        att = y - a
        return a + att * (1 + eps * torch.randn(att.shape, generator=_g, dtype=att.dtype))

    O.light_self_attention = noisy
    _, _, g1, _ = O.forward_backward(sd, x, t, P, LP)
    O.light_self_attention = orig
    worst = sorted(((rel(g1[n], g0[n]), n) for n in g0 if not n.endswith(
        ("conv_branch.0.bias", "attn_branch.0.bias", "gate.0.bias", "fusion_conv.0.bias", "key_conv.bias"))), reverse=True)
    print(f"P={P} B={B} eps={eps:g} seed {s}: " + ", ".join(f"{r:.1e} {n}" for r, n in worst[:3]), flush=True)
