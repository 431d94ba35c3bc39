"""Diagnostic: P = 16, B = 17 fp32 model step, run twice in one process (bitwise determinism of
every gradient), worst per-tensor errors against the float64 oracle; run under different stream
switches (DFCSA_SIDE_STREAM / DFCSA_BRANCH_STREAM) to separate ordering from arithmetic."""
import os
import sys

import torch

sys.path[:0] = ["dfc-sa-unet_amd", ".", "tests"]
from dfcsa.loss import sigmoid  # noqa: E402
from models.unet_dfc_sa_res import UNetDFCSARes  # noqa: E402
from oracle import dfcsa_oracle as O  # noqa: E402
from test_gpu_fra_unet import LP, T, rel  # noqa: E402
from utils.metrics import calculate_metrics  # noqa: E402

P, B = int(os.environ.get("P", 16)), int(os.environ.get("B", 17))
torch.manual_seed(4300 + 16)
m0 = UNetDFCSARes(3, 1, [16, 32, 48, 64], pool_size=P, precision="fp32")
with torch.no_grad():
    for i, (n, p) in enumerate(sorted(m0.named_parameters())):
        if n.endswith("gamma"):
            p.fill_(0.2 + 0.05 * (i % 9))
sd = {k: v.detach().clone() for k, v in m0.state_dict().items()}
gen = torch.Generator().manual_seed(4400 + 16)
BG = int(os.environ.get("BG", B))   # generate BG images, use the first B (same data across B)
x = torch.randn(BG, 3, 64, 64, generator=gen)[:B].contiguous()
t = (torch.rand(BG, 1, 64, 64, generator=gen) > 0.5).float()[:B].contiguous()
sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
_, _, g64, _ = O.forward_backward(sd64, x.double(), t.double(), P, LP)
_, _, g32, _ = O.forward_backward(sd, x, t, P, LP)
runs = []
for r in range(2):
    m = UNetDFCSARes(3, 1, [16, 32, 48, 64], pool_size=P, precision="fp32")
    m.load_state_dict(sd)
    m = m.cuda().train()
    logits = m(T(x.numpy()))
    met = calculate_metrics(sigmoid(logits), T(t.numpy()), "bce_dice", LP)
    met["loss"].backward()
    torch.cuda.synchronize()
    runs.append({n: p.grad.detach().double().cpu().clone() for n, p in m.named_parameters()})
diff = [n for n in runs[0] if not torch.equal(runs[0][n], runs[1][n])]
print(f"P={P} B={B} side={os.environ.get('DFCSA_SIDE_STREAM', '1')} branch={os.environ.get('DFCSA_BRANCH_STREAM', '1')}"
      f" nondeterministic tensors: {len(diff)} {diff[:4]}", flush=True)
rows = sorted(((rel(runs[0][n], g64[n]), n) for n in runs[0]
               if not n.endswith(("conv_branch.0.bias", "attn_branch.0.bias", "gate.0.bias", "fusion_conv.0.bias",
                                  "key_conv.bias"))), reverse=True)
for r, n in rows[:5]:
    print(f"   {r:.2e} (torch fp32 {rel(g32[n], g64[n]):.2e}) {n}", flush=True)
