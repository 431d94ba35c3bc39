"""Per-call GEMM timing of one training step (B=16, 224^2, bf16): wraps dfcsa.ops.conv_gemm /
ops.wgrad with synchronising HIP events and prints time and TFLOP/s per call shape."""
import collections, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch
from dfcsa import ops
from dfcsa.loss import bce_dice, sigmoid
from dfcsa.optim import FusedSGD
from models.model_factory import ModelFactory

rec = []
def timed(fn, kind):
    def w(dtype, *a, **k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); r = fn(dtype, *a, **k); e1.record(); torch.cuda.synchronize()
        if kind == "conv":
            segs, Cseg, grid, N = a[0], a[1], a[2], a[6]
            M, K = grid[0] * grid[1] * grid[2], len(segs) * Cseg
            key = (kind, str(dtype)[6:], M, N, K, len(segs))
        else:
            gs, Cg, segs, Cseg, grid = a[0], a[1], a[2], a[3], a[4]
            M = grid[0] * grid[1] * grid[2]
            key = (kind, str(dtype)[6:], M, len(gs) * Cg, len(segs) * Cseg, len(segs))
        rec.append((key, e0.elapsed_time(e1), 2.0 * key[2] * key[3] * key[4]))
        return r
    return w
ops.conv_gemm = timed(ops.conv_gemm, "conv")
ops.wgrad = timed(ops.wgrad, "wgrad")
import dfcsa.block, dfcsa.functions
dfcsa.block.ops = ops; dfcsa.functions.ops = ops

cfg = {"model": {"name": "DFC-SA-Res-Block", "features": [64, 128, 256, 512], "pool_size": 4, "precision": "bf16"}, "training": {}}
model = ModelFactory.get_model(cfg).cuda().train()
opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
x = torch.randn(16, 3, 224, 224, device="cuda"); t = (torch.rand(16, 1, 224, 224, device="cuda") > 0.5).float()
def step():
    opt.zero_grad(); loss, _ = bce_dice(sigmoid(model(x)), t); loss.backward(); opt.step(max_norm=1.0)
step(); torch.cuda.synchronize(); rec.clear()
step(); torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for k, ms, fl in rec:
    agg[k][0] += 1; agg[k][1] += ms; agg[k][2] += fl
tot = sum(v[1] for v in agg.values())
print(f"GEMM total {tot:.3f} ms/step over {len(rec)} calls")
def roof_ms(k, n):
    kind, _, M, N, K, nseg = k
    if kind == "conv":
        cin = K // nseg * (nseg // 9 if nseg >= 9 and nseg % 9 == 0 else nseg)
        by = 2 * (M * cin + N * K + M * N)
    else:
        by = 2 * (M * N + M * K // max(1, (nseg // 9 if nseg % 9 == 0 else 1))) + 4 * N * K
    return n * max(2.0 * M * N * K / 2.5e15, by / 6.3e12) * 1e3
tr = 0.0
for k, (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    r = roof_ms(k, n); tr += r
    print(f"{ms:7.3f} ms  {fl/ms/1e9:7.1f} TF  roof {r:6.3f} ms ({r/ms*100:5.1f}%)  n={n}  {k}")
print(f"sum of per-call roofline times {tr:.3f} ms ({tr/tot*100:.1f}% of measured)")
