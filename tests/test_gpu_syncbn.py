"""Opt-in SyncBatchNorm (dfcsa.ops.set_sync_bn) against the single-process
full-batch step.

Two ranks (separate processes on the one GPU, gloo group) each run DFC-SA-Res in fp32 mode on half
of a fixed batch with SyncBN on, under the per-sample-additive loss sum(logits * R).  With global
batch statistics the distributed step is the same function as the full-batch step, so:
  * each rank's logits equal the full-batch logits of its rows;
  * the rank gradients SUM to the full-batch gradients (BN weight/bias/res_scale gradients are
    local sums, the input gradients use the all-reduced sums);
  * every rank's BN running statistics equal the full-batch ones.
Without SyncBN (the default) the per-rank statistics differ, which the last check confirms.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tools", "syncbn_check.py")


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


def test_syncbn_two_ranks_equal_full_batch(tmp_path):
    sys.path[:0] = [os.path.dirname(WORKER)]
    import syncbn_check as W
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = str(sk.getsockname()[1])
    sk.close()
    outs = [str(tmp_path / f"r{r}.npz") for r in range(2)]
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, WORKER, str(r), "2", port, outs[r]], env=env, cwd=ROOT)
             for r in range(2)]
    for p in procs:
        assert p.wait(timeout=240) == 0
    ranks = [dict(np.load(o)) for o in outs]

    from dfcsa import ops
    assert not ops.sync_bn_enabled()
    dev = torch.device("cuda:0")
    model = W.build_model(dev)
    x, r = W.batch(dev)
    logits, grads, bufs = W.run(model, x, r)

    per = W.BATCH // 2
    for k in range(2):
        assert rel(ranks[k]["logits"], logits[k * per:(k + 1) * per]) < 1e-5, k
        for n, v in bufs.items():
            assert rel(ranks[k]["buf." + n], v) < 1e-5, (k, n)
    worst = 0.0
    for n, g in grads.items():
        if not np.any(g) or n.endswith("key_conv.bias"):   # true gradient 0 (softmax shift invariance)
            continue
        e = rel(ranks[0]["grad." + n] + ranks[1]["grad." + n], g)
        worst = max(worst, e)
        assert e < 2e-4, (n, e)
    print(f"SyncBN 2 ranks vs full batch: worst per-tensor grad rel {worst:.2e}")

    # without SyncBN the two halves would normalise with their own statistics
    part, _, _ = W.run(W.build_model(dev), x[:per], r[:per])
    assert rel(part, logits[:per]) > 1e-3
