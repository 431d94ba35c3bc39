"""Time the weight-gradient GEMM (+ its split-K reduction) on the headline step's shapes (B=16,
224^2 DFC-SA-Res) under tuning-knob settings; outputs compared with the first setting.
usage: python tools/wgrad_bench.py "base:" "nst3:14=3" "nst64_3:24=3" ...   (label:knob=v;knob=v)"""
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
# name, H, Cs (per source), nsrc, taps (1 | 9), NI, NG (dY tensors)
SHAPES = [("L1 3x3 up_conv1", 224, 64, 2, 9, 64, 1), ("L1 1x1 fusion", 224, 64, 3, 1, 64, 1),
          ("L1 1x1 gate", 224, 64, 2, 1, 64, 1), ("L1 1x1 entry+res (128 in)", 224, 128, 1, 1, 64, 2),
          ("L1 3x3 down1 (Cin 8)", 224, 8, 1, 9, 64, 1), ("L2 3x3 up_conv2", 112, 128, 2, 9, 128, 1),
          ("L2 1x1 fusion", 112, 128, 3, 1, 128, 1), ("L2 1x1 gate", 112, 128, 2, 1, 128, 1),
          ("L3 3x3 up_conv3", 56, 256, 2, 9, 256, 1), ("L4 3x3 up_conv4", 28, 512, 2, 9, 512, 1),
          ("BN 3x3", 14, 512, 1, 9, 1024, 1)]
if os.environ.get("WG_SHAPES"):
    keep = os.environ["WG_SHAPES"].split(",")
    SHAPES = [s for s in SHAPES if any(k in s[0] for k in keep)]


def parse(arg):
    lab, _, kv = arg.partition(":")
    return lab, [tuple(int(x) for x in p.split("=")) for p in kv.split(";") if p]


arms = [parse(a) for a in sys.argv[1:]] or [("base", [])]
for name, H, Cs, nsrc, taps, NI, NG in SHAPES:
    xs = [torch.randn(B, H, H, Cs, device="cuda").to(bf) for _ in range(nsrc)]
    gs = [(torch.randn(B, H, H, NI, device="cuda") * 0.1).to(bf) for _ in range(NG)]
    if taps == 9:
        segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]
    else:
        segs = [(x, 0, 0) for x in xs]
    grads = [torch.zeros(NI, nsrc * Cs, 3 if taps == 9 else 1, 3 if taps == 9 else 1, device="cuda") for _ in range(NG)]
    flops = 2.0 * B * H * H * NI * NG * len(segs) * Cs
    row = {"shape": name, "M": B * H * H, "NI": NI * NG, "NJ": len(segs) * Cs}
    ref = None
    for lab, kvs in arms:
        for k, v in kvs:
            dfcsa.set_tuning(k, v)
        try:
            def run():
                ops.conv_wgrad_into(bf, gs, NI, segs, Cs, (B, H, H), (H, H), grads, taps, nsrc * Cs, nsrc * Cs)
            for gr in grads:
                gr.zero_()
            run()
            torch.cuda.synchronize()
            out = torch.cat([gr.flatten() for gr in grads]).clone()
            if ref is None:
                ref = out
            else:
                row[f"{lab}_maxdiff"] = (out - ref).abs().max().item()
            for _ in range(2):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 100
            row[lab] = (round(us, 1), round(flops / us / 1e6, 1))
        finally:
            for k, v in kvs:
                dfcsa.set_tuning(k, {14: 2, 2: 512, 8: 1}.get(k, 0))
    print(json.dumps(row), flush=True)
