"""Rehearsal of the multi-GPU step on a one-GPU box: an RCCL process group of world size 1 with the
bucketed gradient reducer (dfcsa.ddp) forced on and the whole step captured in one HIP graph -- the
code path bench.py and utils.trainer.Trainer run at N > 1, teardown included.

  1. bench-style step: one eager warm-up step, then capture (dfcsa.ddp.capture_step: thread_local
     mode, NCCL watchdog drained first) and two replays must reproduce three eager steps;
  2. the drop-in Trainer with ``training.data_parallel: true`` (reducer, NaN agreement, metric
     all-reduce, graph capture on the second batch) over 4 batches against the same Trainer with
     graphs off;
  3. teardown exactly as bench.py does it (dfcsa.ddp.shutdown: graphs released, device drained,
     barrier, destroy_process_group) and a normal exit with status 0.

  python tools/rccl_graph_check.py   -> one JSON line, exit status 0 iff ok
"""
import contextlib
import io
import json
import os
import sys
import tempfile

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    # world size 1: an in-process store (no TCP rendezvous, no port to race for)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    from dfcsa.ddp import GradBucketReducer, capture_step, shutdown
    from dfcsa.loss import bce_dice, sigmoid
    from dfcsa.optim import FusedSGD
    from models.unet_dfc_sa_res import UNetDFCSARes
    from utils.trainer import Trainer

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

    def worst_diff(ma, mb):
        w = 0.0
        for (_, a), (_, b) in zip(ma.named_parameters(), mb.named_parameters()):
            w = max(w, ((a - b).norm() / (a.norm() + 1e-30)).item())
        return w

    # 1. bench-style step
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
    graph, _ = capture_step(step_g)   # captured, not executed
    graph.replay()                    # step 2
    graph.replay()                    # step 3
    torch.cuda.synchronize()
    bench_worst = worst_diff(m_eager, m_graph)

    # 2. the drop-in Trainer, data parallel, graph capture on the second batch vs graphs off
    batches = []
    for i in range(4):
        gi = torch.Generator().manual_seed(10 + i)
        batches.append({"image": torch.randn(4, 3, 64, 64, generator=gi),
                        "mask": (torch.rand(4, 1, 64, 64, generator=gi) > 0.5).float()})
    trainers, res = [], []
    with tempfile.TemporaryDirectory() as tmp, contextlib.redirect_stdout(io.StringIO()):
        for graphs in (False, True):
            m = build()
            opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
            cfg = {"training": {"num_epochs": 1, "loss": {"type": "bce_dice", "params": {}}, "data_parallel": True,
                                "cuda_graph": graphs, "bucket_mb": 0.05},
                   "logging": {"log_dir": os.path.join(tmp, f"l{graphs}"), "images_dir": os.path.join(tmp, f"i{graphs}")}}
            tr = Trainer(m, batches, batches[:1], opt, dev, cfg)
            res.append(tr.train_epoch(0))
            torch.cuda.synchronize()
            trainers.append(tr)
    trainer_worst = worst_diff(trainers[0].model, trainers[1].model)
    trainer_graphs = len(trainers[1]._graphs or {})
    loss_diff = max(abs(a - b) for a, b in zip(res[0], res[1]))

    ok = bench_worst < 1e-6 and nb >= 4 and trainer_worst < 1e-6 and loss_diff < 1e-6 and trainer_graphs >= 1 \
        and trainers[1].reducer is not None
    print(json.dumps({"buckets": nb, "world": dist.get_world_size(), "max_rel_param_diff_after_3_steps": bench_worst,
                      "trainer_max_rel_param_diff_4_batches": trainer_worst, "trainer_epoch_metric_diff": loss_diff,
                      "trainer_graphs_captured": trainer_graphs, "ok": ok}), flush=True)
    # 3. bench.py's teardown: graphs released before the communicator goes
    for tr in trainers:
        tr.close()
    shutdown(graph)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
