"""Per-tensor gradient error at the config-2 geometry (GPU diagnostic, not a test).

Builds the cfg2_step.npz model (seed 12000, 64..512, P=4, gammas 0.5), runs one fp32 forward +
backward on the HIP kernels and the CPU oracle, and prints per parameter tensor: the reference's
own fp32-vs-fp64 error ("noise"), our gradient-norm error against the float64 reference, and our
full-tensor error against the oracle.  Usage: python tools/cfg2_diag.py [--precision fp32]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]

from dfcsa.loss import sigmoid  # noqa: E402
from models.unet_dfc_sa_res import UNetDFCSARes  # noqa: E402
from oracle import dfcsa_oracle as O  # noqa: E402
from utils.metrics import calculate_metrics_device  # noqa: E402

LP = {"bce_weight": 0.5, "dice_weight": 0.5}


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp32")
    a = ap.parse_args()
    fx = dict(np.load(os.path.join(ROOT, "tests/golden/cfg2_step.npz")))
    torch.manual_seed(12000)
    m = UNetDFCSARes(3, 1, [64, 128, 256, 512], pool_size=4, precision=a.precision)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("gamma"):
                p.fill_(0.5)
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.cuda().train()
    x, t = torch.from_numpy(fx["x"]).cuda(), torch.from_numpy(fx["t"]).cuda()
    lg = m(x)
    met = calculate_metrics_device(sigmoid(lg), t, "bce_dice", LP)
    met["loss"].backward()
    torch.cuda.synchronize()
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    lo, _, grads, _ = O.forward_backward(sd0, x.cpu(), t.cpu(), 4, LP)
    print(json.dumps({"logits_rel_fixture": rel(lg, torch.from_numpy(fx["logits"])),
                      "oracle_logits_rel_fixture": rel(lo, torch.from_numpy(fx["logits"]))}))
    zero = ("conv_branch.0.bias", "attn_branch.0.bias", "gate.0.bias", "fusion_conv.0.bias", "key_conv.bias")
    rows = []
    for n, p in m.named_parameters():
        if n.endswith(zero):   # true gradient 0: both sides hold rounding noise
            continue
        g64 = float(fx["gnorm64." + n])
        rows.append({"name": n, "numel": p.numel(), "noise": float(fx["noise." + n]),
                     "ours_norm_err": abs(p.grad.double().norm().item() - g64) / (g64 + 1e-30),
                     "oracle_norm_err": abs(grads[n].double().norm().item() - g64) / (g64 + 1e-30),
                     "ours_vs_oracle": rel(p.grad, grads[n])})
    rows.sort(key=lambda r: -r["ours_norm_err"] / max(r["noise"], 1e-7))
    for r in rows[:40]:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
