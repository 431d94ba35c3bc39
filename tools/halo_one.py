"""One 3x3 GEMM of the benchmark (L1 up_conv1 forward by default), N launches, on the halo kernel
(HALO=1) or the row-tile kernel (HALO=0): for rocprofv3 counter passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch  # noqa: E402
from dfcsa import ops  # noqa: E402
from dfcsa._lib import LIB  # noqa: E402

B, H, Cs, nsrc, C = 16, int(os.environ.get("H", 224)), int(os.environ.get("CS", 64)), 2, int(os.environ.get("C", 64))
bf = torch.bfloat16
xs = [torch.randn(B, H, H, Cs, device="cuda").to(bf) for _ in range(nsrc)]
segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]
Kp = ops.rup(9 * nsrc * Cs, 64)
w = (torch.randn(C, Kp, device="cuda") * 0.03).to(bf)
y = torch.empty(B, H, H, C, device="cuda", dtype=bf)
LIB.dfcsa_set_tuning(19, 1 if os.environ.get("HALO", "1") == "1" else 0)
for _ in range(int(os.environ.get("N", 5))):
    ops.conv_gemm(bf, segs, Cs, (B, H, H), (H, H), w, Kp, C, [y], C)
torch.cuda.synchronize()
print("ok")
