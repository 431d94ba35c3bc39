"""Run one conv-GEMM shape repeatedly with a given tile config (for rocprofv3 counter passes).
usage: one_gemm.py H Cseg nsrc ntaps N cfg [reps]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch
from dfcsa import ops
from dfcsa._lib import LIB
H, Cs, nsrc, ntaps, N, cfg = (int(v) for v in sys.argv[1:7])
reps = int(sys.argv[7]) if len(sys.argv) > 7 else 5
B = 16
bf = torch.bfloat16
xs = [torch.randn(B, H, H, Cs, device="cuda").to(bf) for _ in range(nsrc)]
if ntaps == 9:
    segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]
else:
    segs = [(x, 0, 0) for x in xs]
Kp = ops.rup(len(segs) * Cs, 64)
w = (torch.randn(N, Kp, device="cuda") * 0.05).to(bf)
y = torch.empty((B, H, H, N), device="cuda", dtype=bf)
LIB.dfcsa_set_tuning(1, cfg)
for _ in range(reps):
    ops.conv_gemm(bf, segs, Cs, (B, H, H), (H, H), w, Kp, N, [y], N)
torch.cuda.synchronize()
print("done")
