"""Check + time the 256x256 ping-pong conv GEMM (tuning knob 1 = 20) against the default tile
choice on the model's N % 256 == 0 shapes: outputs must be bit-identical (same per-accumulator
MFMA order), BN partial statistics equal to fp32 rounding."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch
from dfcsa import ops
from dfcsa._lib import LIB

B = int(os.environ.get("PP_B", "16"))
bf = torch.bfloat16
SHAPES = [("L2 3x3 dgrad", 112, 128, 1, 11, 256), ("L3 3x3 fwd up_conv3", 56, 256, 2, 9, 256),
          ("L4 3x3 fwd up_conv4", 28, 512, 2, 9, 512), ("BN 3x3 fwd bottleneck", 14, 512, 1, 9, 1024),
          ("L4 3x3 dgrad up_conv4", 28, 512, 1, 11, 1024), ("BN 3x3 dgrad bottleneck", 14, 1024, 1, 11, 512),
          ("L3 dgrad", 56, 256, 1, 11, 512), ("L4 3x3 dgrad down4", 28, 512, 1, 11, 256),
          ("L3 3x3 fwd down3", 56, 128, 1, 9, 256), ("odd 1x1", 20, 64, 3, 1, 256)]
cfgs = [int(c) for c in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,20".split(","))]
torch.manual_seed(0)
ok_all = True
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
    bias = torch.randn(N, device="cuda")
    M = B * H * H
    flops = 2.0 * M * N * K
    row = {"shape": name, "M": M, "N": N, "K": K}
    outs = {}
    for c in cfgs:
        y = torch.full((B, H, H, N), float("nan"), device="cuda", dtype=bf)
        stats = torch.full((ops.ntiles_gemm(M) * 2 * N,), float("nan"), device="cuda")
        LIB.dfcsa_set_tuning(1, c)
        run = lambda: ops.conv_gemm(bf, segs, Cs, (B, H, H), (H, H), w, Kp, N, [y], N, bias=bias, stats=stats)
        run(); torch.cuda.synchronize()
        outs[c] = (y.clone(), stats.clone())
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
        row[c] = (round(us, 1), round(flops / us / 1e6, 1))
    LIB.dfcsa_set_tuning(1, 0)
    y0, s0 = outs[cfgs[0]]
    for c in cfgs[1:]:
        y1, s1 = outs[c]
        same = bool(torch.equal(y0, y1))
        serr = ((s1 - s0).abs().max() / s0.abs().max()).item()
        row[f"eq{c}"] = same
        row[f"stat_err{c}"] = serr
        ok_all &= same and serr < 1e-5
    print(json.dumps(row), flush=True)
print("ALL_OK" if ok_all else "MISMATCH")
