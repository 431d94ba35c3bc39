"""TransUNet (config 4) ViT GEMMs at the bench batch (M = 8 x 196 = 1568 rows): our 1x1 implicit
GEMM (forward / dgrad shapes) and weight-gradient GEMM (+ its split reduction) under tuning-knob
arms, beside torch.mm (hipBLASLt) on the same M, N, K.  One JSON line per shape and arm.
usage: python tools/vit_gemm_bench.py "base:" "sk24:37=24" ...   (label:knob=v;knob=v)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch  # noqa: E402

import dfcsa  # noqa: E402
from dfcsa import ops  # noqa: E402

bf = torch.bfloat16
B, H = 8, 14
M = B * H * H
CONV = [("qkv fwd", 768, 2304), ("proj fwd", 768, 768), ("fc1 fwd", 768, 3072), ("fc2 fwd", 3072, 768),
        ("qkv dgrad", 2304, 768), ("fc1 dgrad", 3072, 768), ("fc2 dgrad", 768, 3072)]   # (K, N)
WG = [("qkv wgrad", 2304, 768), ("proj wgrad", 768, 768), ("fc1 wgrad", 3072, 768), ("fc2 wgrad", 768, 3072)]  # (NI, NJ)


def parse(arg):
    lab, _, kv = arg.partition(":")
    return lab, [tuple(int(x) for x in p.split("=")) for p in kv.split(";") if p]


def timeit(fn, reps=30):
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


arms = [parse(a) for a in sys.argv[1:]] or [("base", [])]
for name, K, N in CONV:
    x = (torch.rand(B, H, H, K, device="cuda") * 2 - 1).to(bf)
    Kp = ops.rup(K, 64)
    w = ((torch.rand(N, Kp, device="cuda") * 2 - 1) * 0.05).to(bf)
    y = torch.empty((B, H, H, N), device="cuda", dtype=bf)
    fl = 2.0 * M * N * K
    row = {"shape": name, "M": M, "N": N, "K": K}
    a2, b2 = x.reshape(M, K), w[:, :K]
    row["hipblaslt_us"] = round(timeit(lambda: torch.mm(a2, b2.t())), 1)
    ref = None
    for lab, kvs in arms:
        for k, v in kvs:
            dfcsa.set_tuning(k, v)
        try:
            run = lambda: ops.conv_gemm(bf, [(x, 0, 0)], K, (B, H, H), (H, H), w, Kp, N, [y], N)  # noqa: E731
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            row[lab + "_maxdiff"] = (y.float() - ref.float()).abs().max().item()
            row[lab + "_us"] = round(timeit(run), 1)
        finally:
            for k, _ in kvs:
                dfcsa.set_tuning(k, 0)
    row.update({k.replace("_us", "_frac"): round(fl / v / 2.5e9, 3) for k, v in list(row.items()) if k.endswith("_us")})
    print(json.dumps(row), flush=True)
for name, NI, NJ in WG:
    g = (torch.rand(B, H, H, NI, device="cuda") * 0.2 - 0.1).to(bf)
    x = (torch.rand(B, H, H, NJ, device="cuda") * 2 - 1).to(bf)
    dst = torch.zeros(NI, NJ, 1, 1, device="cuda")
    fl = 2.0 * M * NI * NJ
    row = {"shape": name, "M": M, "NI": NI, "NJ": NJ}
    g2, x2 = g.reshape(M, NI), x.reshape(M, NJ)
    row["hipblaslt_us"] = round(timeit(lambda: torch.mm(g2.t(), x2)), 1)
    ref = None
    for lab, kvs in arms:
        for k, v in kvs:
            dfcsa.set_tuning(k, v)
        try:
            def run():
                ops.conv_wgrad_into(bf, [g], NI, [(x, 0, 0)], NJ, (B, H, H), (H, H), [dst], 1, NJ, NJ)
            dst.zero_()
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = dst.clone()
            row[lab + "_maxdiff"] = (dst - ref).abs().max().item()
            row[lab + "_us"] = round(timeit(run), 1)
        finally:
            for k, _ in kvs:
                dfcsa.set_tuning(k, 0)
    row.update({k.replace("_us", "_frac"): round(fl / v / 2.5e9, 3) for k, v in list(row.items()) if k.endswith("_us")})
    print(json.dumps(row), flush=True)
