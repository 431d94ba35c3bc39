"""Time the weight-gradient GEMM (+ its slab reduction) on the model's shapes for tuning
variants: knob 6 (waves per workgroup) x knob 2 (target workgroups)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch
from dfcsa import ops
from dfcsa._lib import LIB
bf = torch.bfloat16
B = 16
# H, Cg, ng, Cseg, nsrc, 3x3?
SHAPES = [(224, 64, 1, 64, 2, True), (112, 128, 1, 128, 2, True), (56, 256, 1, 256, 2, True),
          (28, 512, 1, 512, 2, True), (14, 1024, 1, 512, 1, True), (224, 64, 1, 64, 3, False),
          (224, 64, 2, 64, 1, False), (112, 128, 1, 64, 1, True)]
variants = [(8, 512, 0), (8, 512, 1), (8, 1024, 0)]
NOGLDS = int(os.environ.get("NOGLDS", "0"))
LIB.dfcsa_set_tuning(7, NOGLDS)
for H, Cg, ng, Cs, nsrc, k3 in SHAPES:
    M = B * H * H
    gs = [torch.randn(B, H, H, Cg, device="cuda").to(bf) for _ in range(ng)]
    xs = [torch.randn(B, H, H, Cs, device="cuda").to(bf) for _ in range(nsrc)]
    segs = [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs] if k3 else [(x, 0, 0) for x in xs]
    NI, NJ = ng * Cg, len(segs) * Cs
    fl = 2.0 * M * NI * NJ
    row = {"M": M, "NI": NI, "NJ": NJ}
    for w, t, nar in variants:
        LIB.dfcsa_set_tuning(6, w)
        LIB.dfcsa_set_tuning(2, t)
        LIB.dfcsa_set_tuning(8, nar)
        def run():
            slab, sp, ni, nj = ops.wgrad(bf, gs, Cg, segs, Cs, (B, H, H), (H, H))
            return slab, sp
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            slab, sp = run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 200
        row[f"w{w}t{t}n{nar}"] = (round(us, 1), round(fl / us / 1e6, 1), sp)
    print(json.dumps(row), flush=True)
LIB.dfcsa_set_tuning(6, 4)
LIB.dfcsa_set_tuning(2, 512)
