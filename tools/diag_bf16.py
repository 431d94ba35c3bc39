"""Per-parameter gradient error of bf16 compute vs fp32 compute (same weights/batch)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
from models.unet_dfc_sa_res import UNetDFCSARes
from dfcsa.loss import sigmoid
from utils.metrics import calculate_metrics

fx = dict(np.load(os.path.join(ROOT, "tests/golden/model_small.npz")))
sd = {k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("sd0.")}
feats = [int(a) for a in (sys.argv[1].split(",") if len(sys.argv) > 1 else "8,16,32,64".split(","))]
res = {}
for prec in ("fp32", "bf16"):
    torch.manual_seed(0)
    m = UNetDFCSARes(3, 1, feats, pool_size=4, precision=prec)
    if feats == [8, 16, 32, 64]:
        m.load_state_dict(sd)
    else:
        torch.manual_seed(0); m = UNetDFCSARes(3, 1, feats, pool_size=4, precision=prec)
    m = m.cuda().train()
    g = torch.Generator().manual_seed(5)
    H = int(os.environ.get("H", 32)); B = int(os.environ.get("B", 2))
    x = torch.randn(B, 3, H, H, generator=g).cuda()
    t = (torch.rand(B, 1, H, H, generator=g) > 0.5).float().cuda()
    lg = m(x)
    met = calculate_metrics(sigmoid(lg), t, "bce_dice", {})
    met["loss"].backward()
    res[prec] = (lg.detach().cpu(), {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()})
l32, g32 = res["fp32"]; l16, g16 = res["bf16"]
print("logits rel", ((l16 - l32).norm() / l32.norm()).item())
ZERO = ("conv_branch.0.bias", "attn_branch.0.bias", "gate.0.bias", "fusion_conv.0.bias", "key_conv.bias")
rows = []
for n in g32:
    if n.endswith(ZERO):
        continue
    a, b = g16[n].double(), g32[n].double()
    rows.append((((a - b).norm() / (b.norm() + 1e-30)).item(), b.norm().item(), n))
rows.sort(reverse=True)
for r in rows[:25]:
    print(f"{r[0]:.4f} norm={r[1]:.3e} {r[2]}")
keep = [n for n in g32 if not n.endswith(ZERO)]
ga = torch.cat([g16[n].flatten().double() for n in keep]); gb = torch.cat([g32[n].flatten().double() for n in keep])
print("cos", (ga @ gb / ga.norm() / gb.norm()).item())
