"""Time the implicit-GEMM conv kernel on the model's real shapes (B=16, 224^2) per tile config."""
import ctypes, os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch
from dfcsa import ops
from dfcsa._lib import LIB

B = 16
bf = torch.bfloat16
# name, H, Cseg, nsrc, ntaps(1|9), N
SHAPES = [("L1 3x3 fwd up_conv1", 224, 64, 2, 9, 64), ("L1 3x3 dgrad up_conv1", 224, 64, 1, 11, 128),
          ("L1 1x1 gate", 224, 64, 2, 1, 64), ("L1 1x1 fusion", 224, 64, 3, 1, 64),
          ("L1 1x1 entry+res", 224, 64, 2, 1, 128), ("L1 3x3 down1 (Cin 8)", 224, 8, 1, 9, 64),
          ("L2 3x3 fwd up_conv2", 112, 128, 2, 9, 128), ("L2 3x3 dgrad", 112, 128, 1, 11, 256),
          ("L3 3x3 fwd up_conv3", 56, 256, 2, 9, 256), ("L4 3x3 fwd up_conv4", 28, 512, 2, 9, 512),
          ("BN 3x3 fwd bottleneck", 14, 512, 1, 9, 1024), ("L4 3x3 dgrad up_conv4", 28, 512, 1, 11, 1024),
          ("BN 3x3 dgrad bottleneck", 14, 1024, 1, 11, 512), ("L4 3x3 dgrad down4", 28, 512, 1, 11, 256),
          ("L2 3x3 dgrad N64", 112, 128, 1, 11, 64), ("L3 3x3 dgrad up_conv3", 56, 256, 1, 11, 512),
          ("L3 3x3 dgrad down3", 56, 256, 1, 11, 128), ("L3 3x3 fwd down3", 56, 128, 1, 9, 256)]
if os.environ.get("GEMM_SHAPES"):
    keep = os.environ["GEMM_SHAPES"].split(",")
    SHAPES = [s for s in SHAPES if any(k in s[0] for k in keep)]
cfgs = [int(c) for c in (sys.argv[1].split(",") if len(sys.argv) > 1 else "1,2,3,4,5,6".split(","))]
res = []
for name, H, Cs, nsrc, ntaps, N in SHAPES:
    xs = [torch.randn(B, H, H, Cs, device="cuda").to(bf) for _ in range(nsrc)]
    if ntaps == 9:
        segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]
    elif ntaps == 11:
        segs = [(xs[0], 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)] + [(xs[0], 0, 0), (xs[0], 0, 0)]
    else:
        segs = [(x, 0, 0) for x in xs]
    K = len(segs) * Cs
    Kp = ops.rup(K, 64)
    w = (torch.randn(N, Kp, device="cuda") * 0.05).to(bf)
    y = torch.empty((B, H, H, N), device="cuda", dtype=bf)
    M = B * H * H
    stats = torch.empty(ops.ntiles_gemm(M) * 2 * N, device="cuda")
    flops = 2.0 * M * N * K
    row = {"shape": name, "M": M, "N": N, "K": K}
    ref = None
    for c in cfgs:
        LIB.dfcsa_set_tuning(1, c)
        run = lambda: ops.conv_gemm(bf, segs, Cs, (B, H, H), (H, H), w, Kp, N, [y], N, stats=stats)
        if os.environ.get("GEMM_CHECK"):
            y.zero_()
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            else:
                row[f"{c}_maxdiff"] = (y.float() - ref.float()).abs().max().item()
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 100
        row[c] = (round(us, 1), round(flops / us / 1e6, 1))
    LIB.dfcsa_set_tuning(1, 0)
    res.append(row)
    print(json.dumps(row), flush=True)
