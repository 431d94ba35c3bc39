"""Near-ties of the encoder max-pools in the float64 oracle forward (the setup of
tools/lsa_bmm_diag.py / tests/test_gpu_qk_ratio.py::test_large_pool_model_matches_oracle): for every
2x2 window, (max - second max) / max |value| of the map; the smallest margins are where a rounding
difference between two correct fp32 implementations can move the max-pool gradient to another
pixel (a discrete change of the backward).

  python tools/pool_tie_margins.py [P B]
"""
import sys

import torch
import torch.nn.functional as F

sys.path[:0] = ["dfc-sa-unet_amd", "."]
from models.unet_dfc_sa_res import UNetDFCSARes  # noqa: E402
from oracle import dfcsa_oracle as O  # noqa: E402

P, B = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (16, 2)
torch.manual_seed(4300 + P)
m0 = UNetDFCSARes(3, 1, [16, 32, 48, 64], pool_size=P, precision="fp32")
with torch.no_grad():
    for i, (n, p) in enumerate(sorted(m0.named_parameters())):
        if n.endswith("gamma"):
            p.fill_(0.2 + 0.05 * (i % 9))
sd = {k: (v.detach().double() if v.is_floating_point() else v) for k, v in m0.state_dict().items()}
gen = torch.Generator().manual_seed(4400 + P)
x = torch.randn(B, 3, 64, 64, generator=gen).double()
with torch.no_grad():
    t = x
    for name in ("down1", "down2", "down3", "down4"):
        d = O.dfc_block(t, sd, name, P, True, {})
        w = F.unfold(d.reshape(-1, 1, *d.shape[2:]), 2, stride=2)          # [B*C, 4, windows]
        top = w.topk(2, dim=1).values
        gap = (top[:, 0] - top[:, 1]) / d.abs().max()
        v, i = gap.flatten().sort()
        print(f"{name} out {tuple(d.shape)}: smallest top-2 gaps / max|d| {[f'{g:.1e}' for g in v[:4].tolist()]}")
        t = F.max_pool2d(d, 2, 2)
