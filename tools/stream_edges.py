"""Count the cross-stream edges (Stream.wait_stream / wait_event calls) one eager bench step issues,
by call site: each becomes an inter-queue dependency of the captured HIP graph."""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
import torch  # noqa: E402

from dfcsa.loss import bce_dice, sigmoid  # noqa: E402
from dfcsa.optim import FusedSGD  # noqa: E402
from models.unet_dfc_sa_res import UNetDFCSARes  # noqa: E402

calls = collections.Counter()
orig = torch.cuda.Stream.wait_stream


def counted(self, other):
    fr = [f for f in traceback.extract_stack()[:-1] if "dfc-sa-unet_amd" in f.filename]
    site = f"{os.path.basename(fr[-1].filename)}:{fr[-1].lineno}" if fr else "?"
    caller = f"{os.path.basename(fr[-2].filename)}:{fr[-2].lineno}" if len(fr) > 1 else "?"
    calls[(site, caller)] += 1
    return orig(self, other)


torch.manual_seed(0)
dev = torch.device("cuda")
m = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=4, precision="bf16").to(dev).train()
opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4, zero_after_step=True)
x = torch.randn(16, 3, 224, 224, device=dev)
t = (torch.rand(16, 1, 224, 224, device=dev) > 0.5).float()
one = torch.ones((), device=dev)


def step():
    opt.zero_grad()
    loss, stats = bce_dice(sigmoid(m(x)), t, 1.0, 1.0)
    loss.backward(one)
    opt.step(max_norm=1.0, skip_if_nan=loss)


step()
torch.cuda.synchronize()
torch.cuda.Stream.wait_stream = counted
step()
torch.cuda.synchronize()
torch.cuda.Stream.wait_stream = orig
print("wait_stream calls per step:", sum(calls.values()))
for (site, caller), n in calls.most_common():
    print(f"{n:4d}  {site:28s} <- {caller}")
