"""Timing experiment: the default conv GEMM kernel with its A and/or B LDS-DMA pointed at a 1-KB
zero page (knob 15; results meaningless) -- separates operand-fetch time from the MFMA/LDS loop."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch
from dfcsa import ops
from dfcsa._lib import LIB
B = 16
bf = torch.bfloat16
SHAPES = [("L2 3x3 dgrad", 112, 128, 1, 11, 256), ("L3 3x3 fwd up_conv3", 56, 256, 2, 9, 256),
          ("L4 3x3 dgrad up_conv4", 28, 512, 1, 11, 1024), ("L3 dgrad", 56, 256, 1, 11, 512),
          ("L2 3x3 fwd up_conv2 (128x128)", 112, 128, 2, 9, 128), ("L4 3x3 fwd up_conv4 (128x128)", 28, 512, 2, 9, 512)]
for name, H, Cs, nsrc, ntaps, N in SHAPES:
    xs = [torch.randn(B, H, H, Cs, device="cuda").to(bf) for _ in range(nsrc)]
    if ntaps == 9:
        segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]
    else:
        segs = [(xs[0], 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)] + [(xs[0], 0, 0), (xs[0], 0, 0)]
    K = len(segs) * Cs
    Kp = ops.rup(K, 64)
    w = (torch.randn(N, Kp, device="cuda") * 0.05).to(bf)
    y = torch.empty((B, H, H, N), device="cuda", dtype=bf)
    M = B * H * H
    row = {"shape": name, "M": M, "N": N, "K": K}
    for dbg in (0, 1, 2, 3):
        LIB.dfcsa_set_tuning(15, dbg)
        run = lambda: ops.conv_gemm(bf, segs, Cs, (B, H, H), (H, H), w, Kp, N, [y], N)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 50
        row[dbg] = (round(us, 1), round(2.0 * M * N * K / us / 1e6, 1))
    LIB.dfcsa_set_tuning(15, 0)
    print(json.dumps(row), flush=True)
