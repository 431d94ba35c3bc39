"""Time the ConvTranspose2d(2, 2) forward GEMMs and the mid-M 1x1 GEMMs of the step on the streaming
kernel against the tile kernels (knob 34: shuffle store on the streaming kernel; knob 33: smallest
M it takes).  Prints us and effective HBM GB/s per variant (one JSON line per shape)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch
from dfcsa import ops
from dfcsa._lib import LIB
bf = torch.bfloat16
B = 16


def timeit(run):
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 50


VARIANTS = [("tile", 65536, 0), ("stream", 65536, 1), ("stream_allm", 0, 1)]
# ConvTranspose2d: input h, Cin, Cout
for h, Cin, Cout in [(112, 128, 64), (56, 256, 128), (28, 512, 256), (14, 1024, 512)]:
    M, N = B * h * h, 4 * Cout
    x = torch.randn(B, h, h, Cin, device="cuda").to(bf)
    w = (torch.randn(N, Cin, device="cuda") * 0.05).to(bf)
    bias = torch.randn(N, device="cuda")
    y = torch.empty(B, 2 * h, 2 * h, Cout, device="cuda", dtype=bf)
    byts = 2 * M * (Cin + N)
    row = {"convT": True, "M": M, "N": N, "K": Cin}
    for name, k33, k34 in VARIANTS:
        LIB.dfcsa_set_tuning(33, k33)
        LIB.dfcsa_set_tuning(34, k34)
        us = timeit(lambda: ops.conv_gemm(bf, [(x, 0, 0)], Cin, (B, h, h), (h, h), w, Cin, N, [y], Cout, bias=bias,
                                          mode=1, out_hw=(2 * h, 2 * h)))
        row[name] = (round(us, 1), round(byts / us / 1e3))
    print(json.dumps(row), flush=True)
# 1x1 convs with M < 65536 (H, Cseg, nsrc, N, ndest)
for H, Cs, nsrc, N, nd in [(56, 256, 1, 512, 2), (56, 128, 1, 512, 2), (28, 256, 1, 1024, 2), (56, 128, 2, 256, 1)]:
    M = B * H * H
    xs = [torch.randn(B, H, H, Cs, device="cuda").to(bf) for _ in range(nsrc)]
    Kp = ops.rup(nsrc * Cs, 64)
    if Kp > 256:
        continue
    w = (torch.randn(N, Kp, device="cuda") * 0.05).to(bf)
    C = N // nd
    dests = [torch.empty((B, H, H, C), device="cuda", dtype=bf) for _ in range(nd)]
    stats = torch.empty(ops.ntiles_gemm(M) * 2 * N, device="cuda")
    byts = 2 * M * (nsrc * Cs + N)
    row = {"convT": False, "M": M, "N": N, "K": nsrc * Cs}
    for name, k33, k34 in VARIANTS:
        LIB.dfcsa_set_tuning(33, k33)
        us = timeit(lambda: ops.conv_gemm(bf, [(x, 0, 0) for x in xs], Cs, (B, H, H), (H, H), w, Kp, N, dests, C,
                                          stats=stats))
        row[name] = (round(us, 1), round(byts / us / 1e3))
    print(json.dumps(row), flush=True)
LIB.dfcsa_set_tuning(33, 65536)
LIB.dfcsa_set_tuning(34, 1)
