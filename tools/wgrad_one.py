"""One 3x3 weight gradient of the benchmark (L1 up_conv1 by default: B = 16, 224^2, two 64-channel
sources, 64 output channels), N launches on the row-tile LDS-DMA kernel: for rocprofv3 counter
passes (tools/gpu_r03_pmc_wgrad.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch  # noqa: E402
from dfcsa import ops  # noqa: E402

B, H, Cs, nsrc, C = 16, int(os.environ.get("H", 224)), int(os.environ.get("CS", 64)), 2, int(os.environ.get("C", 64))
bf = torch.bfloat16
xs = [torch.randn(B, H, H, Cs, device="cuda").to(bf) for _ in range(nsrc)]
dy = torch.randn(B, H, H, C, device="cuda").to(bf)
segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]
gw = torch.zeros(C, nsrc * Cs, 3, 3, device="cuda")
for _ in range(int(os.environ.get("N", 5))):
    ops.conv_wgrad_into(bf, [dy], C, segs, Cs, (B, H, H), (H, H), [gw], 9, nsrc * Cs, nsrc * Cs)
torch.cuda.synchronize()
print("ok")
