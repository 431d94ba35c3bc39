"""Graph-timed ops.wgrad (partials only, no reduction) on a few headline shapes; runs against
whichever tree's dfcsa package is first on sys.path (A/B of kernel builds)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TREE = os.environ.get("TREE", ROOT)
sys.path[:0] = [TREE, os.path.join(TREE, "dfc-sa-unet_amd")]
import torch  # noqa: E402

from dfcsa import ops  # noqa: E402

bf = torch.bfloat16
B = 16
res = {}
for name, H, Cg, ng, Cs, nseg, k3 in (("W1 H28", 28, 512, 1, 512, 1, True), ("W4 H28", 28, 512, 1, 512, 3, False),
                                      ("W1 H56", 56, 256, 1, 256, 1, True), ("W4 H14", 14, 1024, 1, 1024, 3, False),
                                      ("W1 H224", 224, 64, 1, 64, 1, True), ("W3 H224", 224, 64, 1, 64, 2, False)):
    gs = [torch.randn(B, H, H, Cg, device="cuda").to(bf) for _ in range(ng)]
    xs = [torch.randn(B, H, H, Cs, device="cuda").to(bf) for _ in range(nseg if not k3 else 1)]
    segs = [(xs[0], kh - 1, kw - 1) for kh in range(3) for kw in range(3)] if k3 else [(x, 0, 0) for x in xs]
    fn = lambda: ops.wgrad(bf, gs, Cg, segs, Cs, (B, H, H), (H, H))  # noqa: E731
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        fn()
    torch.cuda.current_stream().wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    res[name] = round(e0.elapsed_time(e1) * 1000 / 30, 1)
print(json.dumps({"tree": TREE, **res}))
