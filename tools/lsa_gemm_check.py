"""LightSelfAttention (standalone, fp32) at pool 16: forward and gradients with the pooled attention
on the batched-GEMM path (N > LSA_GEMM_MIN_N) and on the per-row kernels, each against the float64
oracle (oracle/dfcsa_oracle.py light_self_attention)."""
import sys

import torch

sys.path[:0] = ["dfc-sa-unet_amd", ".", "tests"]
import dfcsa.block as blk  # noqa: E402
from models.unet_dfc_sa_res import LightSelfAttention  # noqa: E402
from oracle import dfcsa_oracle as O  # noqa: E402


def rel(a, b):
    return ((a.double().cpu() - b.double().cpu()).norm() / b.double().cpu().norm()).item()


import os
torch.manual_seed(0)
C, P = int(os.environ.get("C", 64)), 16
m = LightSelfAttention(C, pool_size=P)
with torch.no_grad():
    m.gamma.fill_(0.7)
x = torch.randn(2, C, 32, 32)
g = torch.randn(2, C, 32, 32)
sd = {k: v.detach().double().clone().requires_grad_(True) for k, v in m.state_dict().items()}
x64 = x.double().requires_grad_(True)
y64 = O.light_self_attention(x64, {"." + k if not k.startswith(".") else k: v for k, v in sd.items()}, "", P)
(y64 * g.double()).sum().backward()
for min_n in (256, 64):
    blk.LSA_GEMM_MIN_N = min_n
    mm = LightSelfAttention(C, pool_size=P).cuda()
    mm.load_state_dict(m.state_dict())
    mm.compute_dtype = torch.float32
    xx = x.cuda().requires_grad_(True)
    y = mm(xx)
    (y * g.cuda()).sum().backward()
    torch.cuda.synchronize()
    print(f"MIN_N={min_n}: y {rel(y, y64.detach()):.2e} dx {rel(xx.grad, x64.grad):.2e}", flush=True)
    for n, p in mm.named_parameters():
        print(f"   {n}: {rel(p.grad, sd[n].grad):.2e}", flush=True)
