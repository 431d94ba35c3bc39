"""Calibration: the vendor GEMM (torch.mm -> hipBLASLt / rocBLAS) on the plain GEMM of every conv shape of
tools/gemm_bench.py (same M, N, K; explicit operands, no im2col) beside our implicit-GEMM conv kernel
(automatic tile choice) -- what a tuned library reaches on these sizes, the ceiling claim of
cdna_hip_programming.md rule 10.  Prints one JSON line per shape."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

from dfcsa import ops  # noqa: E402
from dfcsa._lib import LIB  # noqa: E402

B = 16
bf = torch.bfloat16
import gemm_bench_shapes as S  # noqa: E402


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


LIB.dfcsa_set_tuning(1, 0)
for name, H, Cs, nsrc, ntaps, N in S.SHAPES:
    M = B * H * H
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
    stats = torch.empty(ops.ntiles_gemm(M) * 2 * N, device="cuda")
    ours = timeit(lambda: ops.conv_gemm(bf, segs, Cs, (B, H, H), (H, H), w, Kp, N, [y], N, stats=stats))
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(bf)
    bt = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(bf)
    out = {}
    for lib in ("hipblaslt", "rocblas"):
        try:
            torch.backends.cuda.preferred_blas_library(lib)
            out[lib] = timeit(lambda: torch.mm(a, bt.t()))
        except Exception as e:  # noqa: BLE001
            out[lib] = str(e)[:80]
    fl = 2.0 * M * N * K
    row = {"shape": name, "M": M, "N": N, "K": K, "ours_us": round(ours, 1), "ours_frac": round(fl / ours / 2.5e9, 3)}
    for k, v in out.items():
        if isinstance(v, float):
            row[k + "_us"] = round(v, 1)
            row[k + "_frac"] = round(fl / v / 2.5e9, 3)
    print(json.dumps(row), flush=True)
