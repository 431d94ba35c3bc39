"""Per-launch time of the BatchNorm-backward finalize (dfcsa_bn_bwd_finalize) at the step's
(ntiles, C) shapes: 200 back-to-back launches captured in a HIP graph and replayed (the step's
launch mode), and the same launches eager."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch  # noqa: E402

from dfcsa._lib import call  # noqa: E402
from dfcsa.ops import P, stream  # noqa: E402

N = 200
for T, C, ns in [(3136, 64, 2), (3136, 64, 3), (1568, 128, 2), (784, 256, 2), (392, 512, 2), (196, 1024, 2),
                 (98, 1024, 3)]:
    part = torch.randn(T * ns * C, device="cuda")
    coef = torch.empty(3 * C, device="cuda")
    dg = torch.zeros(C, device="cuda")
    db = torch.zeros(C, device="cuda")
    ex = torch.zeros(1, device="cuda")

    def launch():
        call("dfcsa_bn_bwd_finalize", P(part), T, ns, C, 1000, P(coef), P(dg), P(db), P(ex) if ns == 3 else None,
             stream())
    for _ in range(10):
        launch()
    torch.cuda.synchronize()
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    for _ in range(N):
        launch()
    s1.record()
    torch.cuda.synchronize()
    eager = s0.elapsed_time(s1) * 1e3 / N
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        with torch.cuda.graph(g):
            for _ in range(N):
                launch()
    torch.cuda.current_stream().wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    s0.record()
    g.replay()
    s1.record()
    torch.cuda.synchronize()
    print(json.dumps({"ntiles": T, "C": C, "nsum": ns, "eager_us": round(eager, 2),
                      "graph_us": round(s0.elapsed_time(s1) * 1e3 / N, 2)}), flush=True)
