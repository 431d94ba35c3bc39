"""One rank of the SyncBN rehearsal (tests/test_gpu_syncbn.py): W processes share one GPU through a
gloo group; each runs DFC-SA-Res (fp32 mode, features 8..64, P=4) on its shard of a fixed batch
with dfcsa.ops.set_sync_bn() on, under a per-sample-additive loss sum(logits * R) (so the rank
gradients must SUM to the single-process full-batch gradients), and writes its logits, gradients
and BN running statistics to an .npz.

  python tools/syncbn_check.py RANK WORLD PORT OUT.npz
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]

BATCH, HW = 4, 32


def build_model(dev):
    from models.unet_dfc_sa_res import UNetDFCSARes
    torch.manual_seed(0)
    m = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4, precision="fp32").to(dev).train()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("gamma") or n.endswith("res_scale"):
                p.fill_(0.5)
    return m


def batch(dev):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(BATCH, 3, HW, HW, generator=g)
    r = torch.randn(BATCH, 1, HW, HW, generator=g)
    return x.to(dev), r.to(dev)


def run(model, x, r):
    """forward + backward of sum(logits * r); returns logits, {name: grad}, {name: buffer}"""
    for p in model.parameters():
        p.grad = None
    logits = model(x)
    (logits * r).sum().backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().cpu().numpy().copy() for n, p in model.named_parameters()}
    bufs = {n: b.detach().cpu().numpy().copy() for n, b in model.named_buffers() if "running" in n}
    return logits.detach().cpu().numpy(), grads, bufs


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from dfcsa import ops
    ops.set_sync_bn()
    model = build_model(dev)
    x, r = batch(dev)
    per = BATCH // world
    logits, grads, bufs = run(model, x[rank * per:(rank + 1) * per], r[rank * per:(rank + 1) * per])
    np.savez(out, logits=logits, **{"grad." + k: v for k, v in grads.items()},
             **{"buf." + k: v for k, v in bufs.items()})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
