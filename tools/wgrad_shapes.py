"""Per-launch timing of every weight-gradient GEMM of the headline step (DFC-SA-Res 64..512,
B=16, 224^2, bf16), each timed as 10 calls captured in one HIP graph (pure device time): the
complete gradient update (ops.conv_wgrad_into: wgrad kernel + split-K reduction into the weight
gradient) under each tuning mode of MODES (WGRAD_MODES=a,b selects), with each mode's result
checked against the first mode's (relative max difference).  One JSON line per shape + totals.  Usage: python tools/wgrad_shapes.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch  # noqa: E402

import dfcsa  # noqa: E402
from dfcsa import ops  # noqa: E402

B = 16
bf = torch.bfloat16
BLOCKS = [(8, 64, 224, 1), (64, 128, 112, 1), (128, 256, 56, 1), (256, 512, 28, 1), (512, 1024, 14, 1),
          (512, 512, 28, 2), (256, 256, 56, 2), (128, 128, 112, 2), (64, 64, 224, 2)]
# mode -> {tuning knob: value} (knobs 12/13: in-kernel split reduction, 14: LDS ring depth,
# 2: workgroups per launch target); every knob is reset to its default after each shape
MODES = {"default": {}, "fuse16": {13: 16}, "unfused": {12: -1},
         "nst3": {14: 3}, "nst4": {14: 4}, "nst3_t256": {14: 3, 2: 256}, "nst4_t256": {14: 4, 2: 256},
         "nst3_t1024": {14: 3, 2: 1024}, "t1024": {2: 1024},
         "big1": {17: 1}, "big1_t256": {17: 1, 2: 256}, "big1_t1024": {17: 1, 2: 1024}, "big2": {17: 2},
         "big2_t256": {17: 2, 2: 256}, "big3": {17: 3}, "big3_t256": {17: 3, 2: 256}, "big1_f16": {17: 1, 13: 16}, "wide192": {18: 1}}
DEFAULTS = {2: 512, 12: 0, 13: 0, 14: 2, 17: 0, 18: 0}
if os.environ.get("WGRAD_MODES"):
    MODES = {k: v for k, v in MODES.items() if k in os.environ["WGRAD_MODES"].split(",")}


def shapes():
    for cin, c, H, nsrc in BLOCKS:
        cs = cin // nsrc
        yield f"W4 H{H}", H, [c], [(s, 0, 0) for s in range(3)], c, c, 1
        yield f"W3 H{H}", H, [c], [(s, 0, 0) for s in range(2)], c, c, 1
        yield f"W1 H{H}", H, [c], [(s, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for s in range(nsrc)], cs, c, 9
        yield f"W2res H{H}", H, [c, c], [(s, 0, 0) for s in range(nsrc)], cs, c, 1


def graph_time(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


def main():
    tot = {m: 0.0 for m in MODES}
    for name, H, gch, segdesc, cs, c, ntaps in shapes():
        M = B * H * H
        gs = [torch.randn(B, H, H, g, device="cuda").to(bf) for g in gch]
        nsrc = max(s for s, _, _ in segdesc) + 1
        xs = [torch.randn(B, H, H, cs, device="cuda").to(bf) for _ in range(nsrc)]
        segs = [(xs[s], dh, dw) for s, dh, dw in segdesc]
        NI, NJ = len(gs) * c, len(segs) * cs
        Cin = nsrc * cs
        dsts = [torch.zeros(c, Cin, 3, 3, device="cuda") if ntaps == 9 else torch.zeros(c, NJ, device="cuda")
                for _ in gs]
        Ctot = Cin if ntaps == 9 else NJ
        row = {"shape": name, "M": M, "NI": NI, "NJ": NJ, "gflop": round(2.0 * M * NI * NJ / 1e9, 2)}
        ref = None
        for mode, knobs in MODES.items():
            for k, v in knobs.items():
                dfcsa.set_tuning(k, v)
            us = graph_time(lambda: ops.conv_wgrad_into(bf, gs, c, segs, cs, (B, H, H), (H, H), dsts, ntaps, Ctot, Ctot))
            for d in dsts:
                d.zero_()
            ops.conv_wgrad_into(bf, gs, c, segs, cs, (B, H, H), (H, H), dsts, ntaps, Ctot, Ctot)
            out = torch.cat([d.flatten() for d in dsts])
            if ref is None:
                ref = out.clone()
            row[mode] = round(us, 1)
            row[mode + "_maxdiff"] = float((out - ref).abs().max() / (ref.abs().max() + 1e-30))
            tot[mode] += us
            for k in knobs:
                dfcsa.set_tuning(k, DEFAULTS[k])
        print(json.dumps(row), flush=True)
    print(json.dumps({k: round(v, 1) for k, v in tot.items()}))


if __name__ == "__main__":
    main()
