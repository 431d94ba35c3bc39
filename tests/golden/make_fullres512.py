"""Config 5 at its geometry (UNet_FullResAttention, features 64..512, 512^2, B = 1): the oracle's
train-mode forward (oracle/dfcsa_oracle.py, fp32, the FRA formed 8192 query rows at a time) on a
seeded model and input -> fullres512_fwd.npz (logits, BCE+Dice loss, a checksum of the initial
parameters).  The reference itself cannot run this size on a CPU (its attention map is 275 GB); the
oracle's FRA, block and model are pinned to the reference at small N by fra_C*.npz, frablock_*.npz
and fullres_model.npz (make_golden.py gen_fullres).  Takes ~6 min on 8 threads.

    python tests/golden/make_fullres512.py
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]

from oracle import dfcsa_oracle as O  # noqa: E402


def seeded_model_and_batch():
    """The weights (torch.manual_seed(13), attention gammas 0.5) and batch (generator seed 14) the
    fixture and its GPU test share."""
    from models.unet_dfc_sa_ablation_attention import UNet_FullResAttention
    torch.manual_seed(13)
    m = UNet_FullResAttention(3, 1, [64, 128, 256, 512], precision="fp32")
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("gamma"):
                p.fill_(0.5)
    g = torch.Generator().manual_seed(14)
    x = torch.randn(1, 3, 512, 512, generator=g)
    t = (torch.rand(1, 1, 512, 512, generator=g) > 0.5).float()
    return m, x, t


def param_checksum(m):
    return np.array([float(sum(p.detach().double().sum() for p in m.parameters())),
                     float(sum(p.detach().double().abs().sum() for p in m.parameters()))])


if __name__ == "__main__":
    torch.set_num_threads(os.cpu_count() or 8)
    m, x, t = seeded_model_and_batch()
    sd = {k: v.detach().float() for k, v in m.state_dict().items()}
    t0 = time.time()
    with torch.no_grad():
        logits = O.unet_dfc_sa_res(x, sd, 4, training=True, bufs={}, full_res=True)
        loss = O.calculate_metrics(torch.sigmoid(logits), t)["loss"]
    print(f"oracle forward {time.time() - t0:.1f} s, loss {float(loss):.6f}")
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "fullres512_fwd.npz"),
                        logits=logits.numpy().astype(np.float32), loss=np.float64(loss),
                        param_checksum=param_checksum(m))
