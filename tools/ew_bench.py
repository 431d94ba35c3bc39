"""HBM rate of the block elementwise / reduction passes at the level-1 and level-2 shapes of the
B=16 step (bf16), timed with HIP events; compare with tools/hbm_copy_bench.py (~7 TB/s copy)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch
from dfcsa import ops
from dfcsa._lib import LIB, call
from dfcsa.ops import P, S, stream
bf = torch.bfloat16


def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


TILES = [int(v) for v in os.environ.get("EW_TILES", "16384").split(",")]
for tile, (B, H, C) in [(tl, s) for s in [(16, 224, 64), (16, 112, 128), (16, 56, 256), (16, 28, 512)] for tl in TILES]:
    LIB.dfcsa_set_tuning(11, tile)
    M = B * H * H
    t = lambda: torch.randn(B, H, H, C, device="cuda").to(bf)
    a, b, c, d, e, f, h = t(), t(), t(), t(), t(), t(), t()
    sc = torch.rand(C, device="cuda") + 0.5
    sh = torch.randn(C, device="cuda")
    mean, inv = torch.randn(C, device="cuda"), torch.rand(C, device="cuda") + 0.5
    coef = torch.randn(3 * C, device="cuda")
    nt = ops.ntiles_ew(M, C)
    part = torch.empty(nt * 3 * C, device="cuda")
    o = torch.randn(B, 4, 4, C, device="cuda")
    g = torch.ones(1, device="cuda")
    E = M * C * 2
    rows = {}
    rows["bn_bwd_apply 2R1W"] = (bench(lambda: call("dfcsa_bn_bwd_apply", 1, M, C, P(a), P(b), P(mean), P(inv), P(sc), P(coef), P(c), None, 0, stream())), 3 * E)
    rows["bwd_relu_bn 2R1W+sums"] = (bench(lambda: call("dfcsa_bwd_relu_bn", 1, M, C, P(a), P(b), P(sc), P(sh), P(mean), P(inv), P(c), *S(part), stream())), 3 * E)
    rows["bwd_relu_bn (no dz) 2R+sums"] = (bench(lambda: call("dfcsa_bwd_relu_bn", 1, M, C, P(a), P(b), P(sc), P(sh), P(mean), P(inv), None, *S(part), stream())), 2 * E)
    rows["bn_bwd_apply_relu 2R1W"] = (bench(lambda: call("dfcsa_bn_bwd_apply_relu", 1, M, C, P(a), P(b), P(sc), P(sh), P(mean), P(inv), P(sc), P(coef), P(c), None, 0, stream())), 3 * E)
    rows["bwd_gate 6R3W+sums"] = (bench(lambda: call("dfcsa_bwd_gate", 1, M, C, P(a), P(b), P(sc), P(sh), P(mean), P(inv), P(c), P(d), P(e), P(f), P(h), *S(part), stream())), 9 * E)
    rows["bwd_block_out 3R2W+sums"] = (bench(lambda: call("dfcsa_bwd_block_out", 1, M, C, P(a), P(b), P(sc), P(sh), P(mean), P(inv), P(c), P(g), P(d), P(e), *S(part), stream())), 5 * E)
    rows["local_attn 2R2W"] = (bench(lambda: call("dfcsa_block_local_attn", 1, B, H, H, C, P(a), P(sc), P(sh), P(b), P(sc), P(sh), P(o), 4, P(g), 1, P(c), P(d), stream())), 4 * E)
    rows["gate_fuse 3R1W"] = (bench(lambda: call("dfcsa_gate_fuse", 1, M, C, P(a), P(sc), P(sh), P(b), P(c), P(d), stream())), 4 * E)
    rows["block_out 2R1W"] = (bench(lambda: call("dfcsa_block_out", 1, M, C, P(a), P(sc), P(sh), P(b), P(g), P(c), stream())), 3 * E)
    rows["copy 1R1W (torch)"] = (bench(lambda: c.copy_(a)), 2 * E)
    print(json.dumps({"shape": [B, H, H, C], "tile_elems": tile, **{k: [round(us, 1), round(by / us / 1e3)] for k, (us, by) in rows.items()}}),
          flush=True)
LIB.dfcsa_set_tuning(11, 16384)
