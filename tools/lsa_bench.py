"""LightSelfAttention full-resolution kernels at the bench's level shapes (B=16, P=4):
dfcsa_lsa_pool and dfcsa_lsa_up_bwd_rows (with its A/B knob 28), timed with HIP
events over 50 launches.  Prints one JSON line per (kernel, level, variant) with us and GB/s of
the full-resolution tensor read."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dfc-sa-unet_amd"))
import torch  # noqa: E402
import dfcsa  # noqa: E402
from dfcsa._lib import LIB, call  # noqa: E402
from dfcsa.ops import P as ptr, stream, dt  # noqa: E402

B, P = 16, 4
LEVELS = [(224, 64), (112, 128), (56, 256), (28, 512), (14, 1024)]


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for H, C in LEVELS:
    x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
    nbytes = x.numel() * 2
    sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
    S = LIB.dfcsa_lsa_pool_splits(H, P)
    part = torch.empty(B * P * P * S * C, device="cuda")
    rows = torch.empty(B * H * P * C, device="cuda")
    for knob, name, fn in [
        (None, "pool", lambda: call("dfcsa_lsa_pool", dt(torch.bfloat16), B, H, H, C, ptr(x), ptr(sc), ptr(sh), P, 1,
                                  ptr(part), stream())),
        (28, "up_bwd_rows", lambda: call("dfcsa_lsa_up_bwd_rows", dt(torch.bfloat16), B, H, H, C, ptr(x), P,
                                         ptr(rows), stream()))]:
        for old in ((0, 1) if knob else (0,)):
            if knob:
                dfcsa.set_tuning(knob, old)
            us = timeit(fn)
            if knob:
                dfcsa.set_tuning(knob, 0)
            print(json.dumps({"kernel": name, "H": H, "C": C, "old": old, "us": round(us, 2),
                              "GBps": round(nbytes / us / 1e3, 1)}), flush=True)
