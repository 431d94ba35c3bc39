"""Rehearsal of bench.py's multi-GPU step on a one-GPU box: an RCCL process group of world size 1,
the bucketed gradient reducer (dfcsa.ddp) forced on, and the whole step captured in one HIP graph.
The graph replays must reproduce the eager steps (same parameters after 3 steps), which checks
that the async RCCL all-reduces on the side stream are captured and ordered correctly.

  python tools/rccl_graph_check.py   -> one JSON line
"""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    # world size 1: an in-process store (no TCP rendezvous, no port to race for)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    from dfcsa.ddp import GradBucketReducer
    from dfcsa.loss import bce_dice, sigmoid
    from dfcsa.optim import FusedSGD
    from models.unet_dfc_sa_res import UNetDFCSARes

    def build():
        torch.manual_seed(0)
        m = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4, precision="fp32").to(dev).train()
        with torch.no_grad():
            for n, p in m.named_parameters():
                if n.endswith("gamma"):
                    p.fill_(0.5)
        return m

    g = torch.Generator().manual_seed(1)
    x = torch.randn(4, 3, 64, 64, generator=g).to(dev)
    t = (torch.rand(4, 1, 64, 64, generator=g) > 0.5).float().to(dev)

    def make_step(model):
        opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
        model(x)
        red = GradBucketReducer(model, bucket_mb=0.05)   # several buckets even at this width

        def step():
            opt.zero_grad()
            loss, stats = bce_dice(sigmoid(model(x)), t, 1.0, 1.0)
            red.start()
            loss.backward()
            skip = red.finish(loss)   # all-reduced NaN flag of the loss (every rank skips together)
            opt.step(max_norm=1.0, grad_scale=red.grad_scale, skip_if_nan=skip)
            return stats
        return step, len(red.buckets)

    m_eager = build()
    step_e, nb = make_step(m_eager)
    for _ in range(3):
        step_e()
    torch.cuda.synchronize()

    m_graph = build()
    step_g, _ = make_step(m_graph)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step_g()                      # step 1 (eager warm-up, as bench.py does)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step_g()                      # captured, not executed
    graph.replay()                    # step 2
    graph.replay()                    # step 3
    torch.cuda.synchronize()
    worst = 0.0
    for (n, a), (_, b) in zip(m_eager.named_parameters(), m_graph.named_parameters()):
        worst = max(worst, ((a - b).norm() / (a.norm() + 1e-30)).item())
    print(json.dumps({"buckets": nb, "world": dist.get_world_size(), "max_rel_param_diff_after_3_steps": worst,
                      "ok": worst < 1e-6 and nb >= 4}), flush=True)
    # leave without tearing the communicator down under the live graph (destroy_process_group
    # aborts while a captured RCCL graph still references the communicator); the OS releases it
    os._exit(0)


if __name__ == "__main__":
    main()
