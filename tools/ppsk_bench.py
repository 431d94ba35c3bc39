"""Stream-K ping-pong conv (knob 40) against the tile choice without it, on the model's B = 16 shapes
where it applies; one JSON line per shape: microseconds per launch (20 launches after 3 warm-ups)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

import dfcsa  # noqa: E402
from dfcsa import ops  # noqa: E402
from gemm_bench_shapes import SHAPES  # noqa: E402

B = 16
bf = torch.bfloat16


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, H, Cs, nsrc, ntaps, N in SHAPES:
    if N % 256 or H > 56:
        continue
    xs = [(torch.rand(B, H, H, Cs, device="cuda") * 2 - 1).to(bf) for _ in range(nsrc)]
    if ntaps == 9:
        segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]
    elif ntaps == 11:
        segs = [(xs[0], 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)] + [(xs[0], 0, 0), (xs[0], 0, 0)]
    else:
        segs = [(x, 0, 0) for x in xs]
    K = len(segs) * Cs
    Kp = ops.rup(K, 64)
    w = ((torch.rand(N, Kp, device="cuda") * 2 - 1) * 0.05).to(bf)
    y = torch.empty((B, H, H, N), device="cuda", dtype=bf)
    M = B * H * H
    stats = torch.empty(ops.ntiles_gemm(M) * 2 * N, device="cuda")
    row = {"shape": name, "M": M, "N": N, "K": K}
    for lab, v in (("sk", 1), ("nosk", 0)):
        dfcsa.set_tuning(40, v)
        us = timeit(lambda: ops.conv_gemm(bf, segs, Cs, (B, H, H), (H, H), w, Kp, N, [y], N, stats=stats))
        row[lab + "_us"] = round(us, 1)
        row[lab + "_frac"] = round(2.0 * M * N * K / us / 2.5e9, 3)
    dfcsa.set_tuning(40, 1)
    print(json.dumps(row), flush=True)
