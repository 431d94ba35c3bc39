"""Per-launch timing of every weight-gradient GEMM of the headline step (DFC-SA-Res 64..512,
B=16, 224^2, bf16), each timed as 10 calls captured in one HIP graph (pure device time): the
complete gradient update (ops.conv_wgrad_into: wgrad kernel + split-K reduction into the weight
gradient) with the in-kernel reduction threshold at its default, at 16 splits, and disabled.
One JSON line per shape + totals.  Usage: python tools/wgrad_shapes.py"""
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
MODES = {"default": (0, 0), "fuse16": (0, 16), "unfused": (-1, 0)}   # knobs 12, 13
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
        for mode, (k12, k13) in MODES.items():
            dfcsa.set_tuning(12, k12)
            dfcsa.set_tuning(13, k13)
            us = graph_time(lambda: ops.conv_wgrad_into(bf, gs, c, segs, cs, (B, H, H), (H, H), dsts, ntaps, Ctot, Ctot))
            row[mode] = round(us, 1)
            tot[mode] += us
        dfcsa.set_tuning(12, 0)
        dfcsa.set_tuning(13, 0)
        print(json.dumps(row), flush=True)
    print(json.dumps({k: round(v, 1) for k, v in tot.items()}))


if __name__ == "__main__":
    main()
