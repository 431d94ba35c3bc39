"""Error budget of the bf16 pooled attention (LightSelfAttention at P = 16 / 32, bf16 mode): the flash
MFMA path, the fp32 per-row path on the same bf16 input, and the reference's own CPU bf16 autocast,
each against the oracle in float64 (y - x, dx, parameter gradients); plus the energy range.

  python tools/lsa_flash_err.py [C P H B scale]
"""
import os
import sys

import torch

sys.path[:0] = ["dfc-sa-unet_amd", "."]
from dfcsa import block  # noqa: E402
from models.unet_dfc_sa_res import LightSelfAttention  # noqa: E402
from oracle import dfcsa_oracle as O  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


C, P, H, B = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (64, 16, 28, 2)))
scale = float(sys.argv[5]) if len(sys.argv) > 5 else 2.0
torch.manual_seed(100 + C + P)
m = LightSelfAttention(C, pool_size=P)
with torch.no_grad():
    m.gamma.fill_(0.7)
    for conv in (m.query_conv, m.key_conv, m.value_conv):
        conv.weight.mul_(scale)
g0 = torch.Generator().manual_seed(7 + C)
x = torch.randn(B, C, H, H + 1, generator=g0).bfloat16().float()
gy = torch.randn(B, C, H, H + 1, generator=g0)
sd = {"a." + k: v.detach().double().clone().requires_grad_(True) for k, v in m.state_dict().items()}
xr = x.double().clone().requires_grad_(True)
yr = O.light_self_attention(xr, sd, "a", P)
yr.backward(gy.double())
with torch.no_grad():
    p = torch.nn.functional.adaptive_avg_pool2d(x.double(), (P, P))
    q = O.conv(p, sd, "a.query_conv").reshape(B, -1, P * P)
    k = O.conv(p, sd, "a.key_conv").reshape(B, -1, P * P)
    e = torch.bmm(q.transpose(1, 2), k)
    print(f"C={C} P={P} H={H} B={B} scale={scale}: energy range [{e.min():.1f}, {e.max():.1f}], "
          f"row max - row 2nd max median {(e.topk(2, -1).values[..., 0] - e.topk(2, -1).values[..., 1]).median():.2f}")


def report(tag, y, dx, grads):
    gs = " ".join(f"{n.split('.')[0][:5]}.{n.split('.')[-1][0]} {rel(grads[n], sd['a.' + n].grad):.1e}"
                  for n in grads if n != "key_conv.bias")
    print(f"  {tag:10s} y-x {rel(y - x, (yr - xr).detach()):.2e}  dx {rel(dx - gy, xr.grad - gy.double()):.2e}  {gs}",
          flush=True)


sa = {k: v.detach().float().clone().requires_grad_(True) for k, v in sd.items()}
xa = x.clone().requires_grad_(True)
with torch.autocast("cpu", dtype=torch.bfloat16):
    ya = O.light_self_attention(xa, sa, "a", P)
ya.float().backward(gy)
report("ref-amp", ya.float(), xa.grad, {k[2:]: v.grad for k, v in sa.items()})
for tag, dtype, min_n in (("flash-bf16", torch.bfloat16, 64), ("row-bf16", torch.bfloat16, 1 << 30),
                          ("flash-fp32", torch.float32, 64), ("row-fp32", torch.float32, 1 << 30)):
    block.LSA_FLASH_MIN_N[0] = min_n
    block.LSA_FLASH_FP32[0] = True
    mg = LightSelfAttention(C, pool_size=P)
    mg.load_state_dict(m.state_dict())
    mg = mg.cuda()
    mg.compute_dtype = dtype
    xg = x.cuda().requires_grad_(True)
    y = mg(xg)
    y.backward(gy.cuda())
    torch.cuda.synchronize()
    report(tag, y.float().cpu(), xg.grad.cpu(), {n: p.grad for n, p in mg.named_parameters()})
