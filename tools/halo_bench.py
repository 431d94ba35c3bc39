"""Per-layer timing of the benchmark's 3x3 GEMMs (B = 16, 224^2 model): the 2-D halo-tile kernels
(conv fwd / fused dgrad: knob 19; weight gradient: knob 20) against the row-tile kernels.
Prints one JSON line per (layer, kernel) with microseconds per launch and TFLOP/s."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch  # noqa: E402
from dfcsa import ops  # noqa: E402
from dfcsa._lib import LIB  # noqa: E402

B = 16
bf = torch.bfloat16
# name, H, Cs (source channels), nsrc, C (block width)
LAYERS = [("L1 up_conv1", 224, 64, 2, 64), ("L2 down2", 112, 64, 1, 128), ("L2 up_conv2", 112, 128, 2, 128),
          ("L3 down3", 56, 128, 1, 256), ("L3 up_conv3", 56, 256, 2, 256), ("L4 down4", 28, 256, 1, 512),
          ("L4 up_conv4", 28, 512, 2, 512), ("L5 bottleneck", 14, 512, 1, 1024)]
which = sys.argv[1].split(",") if len(sys.argv) > 1 else ["fwd", "dgrad", "wgrad"]
h19, h20 = LIB.dfcsa_get_tuning(19), LIB.dfcsa_get_tuning(20)


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


for name, H, Cs, nsrc, C in LAYERS:
    M = B * H * H
    xs = [torch.randn(B, H, H, Cs, device="cuda").to(bf) for _ in range(nsrc)]
    Cin = nsrc * Cs
    segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]
    if "fwd" in which:
        Kp = ops.rup(9 * Cin, 64)
        w = (torch.randn(C, Kp, device="cuda") * 0.03).to(bf)
        y = torch.empty(B, H, H, C, device="cuda", dtype=bf)
        st = torch.empty(ops.ntiles_gemm(M) * 2 * C, device="cuda")
        fl = 2.0 * M * C * 9 * Cin
        for knob in (0, 32768):
            LIB.dfcsa_set_tuning(19, knob)
            us = timeit(lambda: ops.conv_gemm(bf, segs, Cs, (B, H, H), (H, H), w, Kp, C, [y], C, stats=st))
            print(json.dumps({"layer": name, "op": "fwd", "halo": knob, "us": round(us, 1),
                              "tflops": round(fl / us / 1e6, 1)}), flush=True)
        LIB.dfcsa_set_tuning(19, h19)
    if "dgrad" in which:
        dy = [torch.randn(B, H, H, C, device="cuda").to(bf) for _ in range(3)]
        dsegs = [(dy[0], 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)] + [(dy[1], 0, 0), (dy[2], 0, 0)]
        Kp = ops.rup(11 * C, 64)
        w = (torch.randn(Cin, Kp, device="cuda") * 0.03).to(bf)
        dxs = [torch.empty(B, H, H, Cs, device="cuda", dtype=bf) for _ in range(nsrc)]
        fl = 2.0 * M * Cin * 11 * C
        for knob in (0, 32768):
            LIB.dfcsa_set_tuning(19, knob)
            us = timeit(lambda: ops.conv_gemm(bf, dsegs, C, (B, H, H), (H, H), w, Kp, Cin, dxs, Cs))
            print(json.dumps({"layer": name, "op": "dgrad", "halo": knob, "us": round(us, 1),
                              "tflops": round(fl / us / 1e6, 1)}), flush=True)
        LIB.dfcsa_set_tuning(19, h19)
    if "wgrad" in which:
        g = torch.randn(B, H, H, C, device="cuda").to(bf)
        gw = torch.zeros(C, Cin, 3, 3, device="cuda")
        fl = 2.0 * M * C * 9 * Cin
        for knob in (0, 1):
            LIB.dfcsa_set_tuning(20, knob)
            us = timeit(lambda: ops.conv_wgrad_into(bf, [g], C, segs, Cs, (B, H, H), (H, H), [gw], 9, Cin, Cin))
            print(json.dumps({"layer": name, "op": "wgrad", "halo": knob, "us": round(us, 1),
                              "tflops": round(fl / us / 1e6, 1)}), flush=True)
        LIB.dfcsa_set_tuning(20, h20)
