"""Time the memory-bound 1x1 GEMM shapes of the step: streaming kernel (per-CU workgroup counts)
vs the generic tile kernel (tuning knob 1 = 7).  Prints us and effective HBM GB/s."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch
from dfcsa import ops
from dfcsa._lib import LIB
bf = torch.bfloat16
B = 16
# H, Cseg, nsrc, N, ndest, accumulate
SHAPES = [(224, 64, 3, 64, 1, False), (224, 64, 2, 64, 1, False), (112, 128, 2, 128, 1, False),
          (56, 256, 1, 512, 2, False), (56, 256, 2, 256, 1, False), (28, 512, 1, 1024, 2, False), (224, 64, 1, 128, 2, True), (224, 64, 1, 192, 3, False), (224, 64, 3, 64, 1, False),
          (224, 64, 2, 64, 1, False), (224, 64, 2, 128, 2, False), (224, 8, 1, 128, 2, False),
          (112, 128, 1, 256, 2, False), (112, 128, 3, 128, 1, False), (112, 128, 1, 384, 3, False),
          (112, 128, 2, 128, 1, False)]
if os.environ.get("STREAM_H"):
    SHAPES = [s for s in SHAPES if s[0] == int(os.environ["STREAM_H"])]
if os.environ.get("STREAM_NOSTATS"):
    SHAPES = [s[:5] + (s[5],) for s in SHAPES]
variants = [("tile", 7, 0)] + [(f"stream{w}", 0, w) for w in (0, 2, 3)] + [("force0", -1, 0), ("force2", -1, 2)]
for H, Cs, nsrc, N, nd, acc in SHAPES:
    M = B * H * H
    xs = [torch.randn(B, H, H, Cs, device="cuda").to(bf) for _ in range(nsrc)]
    segs = [(x, 0, 0) for x in xs]
    Kp = ops.rup(nsrc * Cs, 64)
    w = (torch.randn(N, Kp, device="cuda") * 0.05).to(bf)
    C = N // nd
    dests = [torch.zeros((B, H, H, C), device="cuda", dtype=bf) for _ in range(nd)]
    stats = torch.empty(ops.ntiles_gemm(M) * 2 * N, device="cuda")
    byts = 2 * M * (nsrc * Cs + N * (2 if acc else 1))
    row = {"M": M, "N": N, "K": nsrc * Cs, "acc": acc}
    for name, knob1, wgs in variants:
        LIB.dfcsa_set_tuning(1, max(knob1, 0))
        LIB.dfcsa_set_tuning(5, 1 if knob1 < 0 else 0)
        LIB.dfcsa_set_tuning(3, wgs)
        run = lambda: ops.conv_gemm(bf, segs, Cs, (B, H, H), (H, H), w, Kp, N, dests, C, accumulate=acc,
                                    stats=None if (acc or os.environ.get("STREAM_NOSTATS")) else stats)
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
        row[name] = (round(us, 1), round(byts / us / 1e3, 0))
    LIB.dfcsa_set_tuning(1, 0)
    LIB.dfcsa_set_tuning(3, 0)
    LIB.dfcsa_set_tuning(5, 0)
    print(json.dumps(row), flush=True)
