"""The drop-in Trainer (utils/trainer.py) on the MI355X: HIP-graph replay against eager stepping
over many batches, the reference's pinned-memory DataLoader feeding a graph-captured step, and data
parallelism through the unchanged Trainer API (two gloo ranks on the one GPU).

Reference: utils/trainer.py:105-170 (train_epoch), :172-265 (validate_epoch), :267-324
(checkpoints), train.py:73-88 (SGD + Trainer wiring).
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
GOLDEN = os.path.join(ROOT, "tests", "golden")
LP = {"bce_weight": 0.5, "dice_weight": 0.5}
ZERO = ("conv_branch.0.bias", "attn_branch.0.bias", "gate.0.bias", "fusion_conv.0.bias", "key_conv.bias")


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


def small_model(precision="fp32"):
    from models.unet_dfc_sa_res import UNetDFCSARes
    fx = dict(np.load(os.path.join(GOLDEN, "model_small.npz")))
    m = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4, precision=precision)
    m.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("sd0.")})
    return m


def cfg_for(tmp, graphs, epochs=1):
    return {"training": {"num_epochs": epochs, "save_checkpoint_freq": 100, "cuda_graph": graphs,
                         "loss": {"type": "bce_dice", "params": LP}},
            "logging": {"log_dir": str(tmp / "logs"), "images_dir": str(tmp / "img"), "save_best_worst_samples": 0}}


def batches(n, bs, last=None, seed=7):
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(n):
        b = last if (last and i == n - 1) else bs
        out.append({"image": torch.randn(b, 3, 32, 32, generator=g),
                    "mask": (torch.rand(b, 1, 32, 32, generator=g) > 0.5).float(), "filename": [f"{i}_{j}" for j in range(b)]})
    return out


def state(model, opt):
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    mom = {n: opt.state[p]["momentum_buffer"].detach().cpu().clone() for n, p in model.named_parameters()}
    return sd, mom


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_graph_replay_equals_eager_over_epochs(tmp_path, precision):
    """Trainer.train_epoch over 6 batches with a short last batch (a second graph shape),
    twice, with training.cuda_graph on and off from the same start: replays 2..n (resumed momentum,
    BN running stats and num_batches_tracked, packs rebuilt from updated weights) must give the
    eager step's losses, parameters, momentum and buffers bit for bit (same kernels, same order).
    Between the epochs a second model is built and run (a new PackSet: the model's pack plan goes
    stale) and the model is validated (eager forward), as a training script does."""
    from utils.trainer import Trainer
    data = batches(6, 4, last=2)
    runs = []
    for graphs in (False, True):
        model = small_model(precision)
        opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
        tr = Trainer(model, data, data[:2], opt, torch.device("cuda"), cfg_for(tmp_path / str(graphs), graphs))
        e1 = tr.train_epoch(0)
        other = small_model(precision).cuda()     # bumps the pack-plan epoch
        with torch.no_grad():
            other(data[0]["image"].cuda())
        va = tr.validate_epoch(data[:2])
        e2 = tr.train_epoch(1)
        torch.cuda.synchronize()
        if graphs:
            assert tr._graphs, "the step was never captured"
        runs.append((e1, e2, va["dice"]) + state(model, tr.optimizer))
    (a1, a2, ad, asd, am), (b1, b2, bd, bsd, bm) = runs
    assert a1 == b1 and a2 == b2 and ad == bd, (a1, b1, a2, b2)
    for k in asd:
        assert torch.equal(asd[k], bsd[k]), k
    for k in am:
        assert torch.equal(am[k], bm[k]), k


def test_graph_capture_with_pinned_dataloader(tmp_path):
    """the reference's DataLoader path (pin_memory=True, two worker processes: the
    pin-memory thread runs during the capture) feeding the graph-captured step over 4 batches,
    against the same batches (unshuffled loader order) stepped eagerly from host copies."""
    from utils.data_loader import DataLoaderFactory
    from utils.trainer import Trainer
    cfg = {"dataset": {"synthetic": 64, "img_size": [32, 32]}, "training": {"batch_size": 4, "num_workers": 2}}
    loader = DataLoaderFactory(cfg).get_val_loader()          # 16 images, fixed order
    assert loader.pin_memory and len(loader) == 4
    host = [{"image": b["image"].clone(), "mask": b["mask"].clone()} for b in DataLoaderFactory(
        dict(cfg, training={"batch_size": 4, "num_workers": 0})).get_val_loader()]
    out = []
    for graphs, src in ((True, loader), (False, host)):
        model = small_model("fp32")
        opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
        tr = Trainer(model, src, host[:1], opt, torch.device("cuda"), cfg_for(tmp_path / str(graphs), graphs))
        out.append((tr.train_epoch(0), state(model, tr.optimizer)[0]))
        if graphs:
            assert tr._graphs, "the step was never captured"
    (l1, s1), (l2, s2) = out
    assert l1 == l2
    for k in s1:
        assert torch.equal(s1[k], s2[k]), k


def test_trainer_data_parallel_two_ranks(tmp_path):
    """two gloo ranks on the one GPU run Trainer.train_epoch on the 8-image global
    batch of tests/golden/ddp_shards.npz through the reference's wiring (torch.optim.SGD + Trainer).
    The clipped gradient every rank applies is the clip of the reference's mean of per-shard
    gradients (w2.mean_grad); parameters after the step equal the reference SGD step from it; the
    replicas are identical (parameters after the step, BN statistics after validation's broadcast);
    the reported loss is the mean of the per-shard reference losses and IoU / Dice are the global
    batch's counts; only rank 0 writes a checkpoint."""
    from oracle import dfcsa_oracle as O
    worker = os.path.join(ROOT, "tools", "trainer_ddp_check.py")
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = str(sk.getsockname()[1])
    sk.close()
    outs = [str(tmp_path / f"r{r}.npz") for r in range(2)]
    procs = [subprocess.Popen([sys.executable, worker, str(r), "2", port, outs[r], str(tmp_path / "logs")],
                              env=dict(os.environ), cwd=ROOT) for r in range(2)]
    for p in procs:
        assert p.wait(timeout=240) == 0
    r0, r1 = (dict(np.load(o)) for o in outs)
    dd = dict(np.load(os.path.join(GOLDEN, "ddp_shards.npz")))
    fx = dict(np.load(os.path.join(GOLDEN, "model_small.npz")))
    sd0 = {k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("sd0.")}
    mean = {n: torch.from_numpy(dd[f"w2.mean_grad.{n}"]) for n in O.param_names(sd0)}
    sd1, _, _, clipped = O.clip_and_sgd(sd0, mean, {})
    for n in O.param_names(sd0):
        assert np.array_equal(r0["param." + n], r1["param." + n]), n       # identical replicas
        if n.endswith(ZERO):
            continue
        assert rel(r0["grad." + n], clipped[n].numpy()) < 2e-3, n
        upd, upd_ref = r0["param." + n] - sd0[n].numpy(), (sd1[n] - sd0[n]).numpy()
        assert rel(upd, upd_ref) < 3e-3, n
    for k in r0:
        if k.startswith("buf."):
            assert np.array_equal(r0[k], r1[k]), k                          # broadcast before validation
    assert any(not np.array_equal(r0[k], r1[k]) for k in r0 if k.startswith("trainbuf."))  # per-replica BN
    # metrics: mean of the per-shard losses, IoU / Dice of the global batch's counts
    x, t = torch.from_numpy(dd["x"]), torch.from_numpy(dd["t"])
    losses, inter, sb, st = [], 0.0, 0.0, 0.0
    for r in range(2):
        logits, met, _, _ = O.forward_backward(sd0, x[4 * r:4 * r + 4], t[4 * r:4 * r + 4], 4, LP)
        losses.append(met["loss"].item())
        b = (torch.sigmoid(logits) > 0.5).float()
        inter += (b * t[4 * r:4 * r + 4]).sum().item()
        sb += b.sum().item()
        st += t[4 * r:4 * r + 4].sum().item()
    assert abs(float(r0["loss"]) - np.mean(losses)) < 1e-4 * abs(np.mean(losses))
    assert float(r0["loss"]) == float(r1["loss"]) and float(r0["dice"]) == float(r1["dice"])
    assert abs(float(r0["dice"]) - 2 * inter / (sb + st + 1e-7)) < 1e-3
    assert abs(float(r0["iou"]) - inter / (sb + st - inter + 1e-7)) < 1e-3
    assert os.path.exists(tmp_path / "logs" / "r0" / "checkpoints" / "checkpoint_epoch_1.pth")
    assert not os.path.exists(tmp_path / "logs" / "r1" / "checkpoints" / "checkpoint_epoch_1.pth")


def test_trainer_data_parallel_ragged_batches(tmp_path):
    """data-parallel training over global batches that do not divide over the ranks.  Two
    gloo ranks run one epoch of a 7-image batch (rows 4 / 3) and a 1-image batch (rank 1 without rows,
    stepping with zero gradients through the same collectives); rank 1 starts from perturbed weights,
    which the reducer's broadcast from rank 0 replaces.  Expected: each step applies the row-weighted
    mean of the per-replica reference gradients, sum_r (n_r / n) g_r (the CPU oracle: clip + SGD with
    momentum over both steps), and the replicas end identical."""
    from oracle import dfcsa_oracle as O
    worker = os.path.join(ROOT, "tools", "trainer_ddp_check.py")
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = str(sk.getsockname()[1])
    sk.close()
    outs = [str(tmp_path / f"r{r}.npz") for r in range(2)]
    procs = [subprocess.Popen([sys.executable, worker, str(r), "2", port, outs[r], str(tmp_path / "logs"), "ragged"],
                              env=dict(os.environ), cwd=ROOT) for r in range(2)]
    for p in procs:
        assert p.wait(timeout=240) == 0
    r0, r1 = (dict(np.load(o)) for o in outs)
    dd = dict(np.load(os.path.join(GOLDEN, "ddp_shards.npz")))
    fx = dict(np.load(os.path.join(GOLDEN, "model_small.npz")))
    sd = {k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("sd0.")}
    sd0 = dict(sd)
    x, t = torch.from_numpy(dd["x"]), torch.from_numpy(dd["t"])
    mom = {}
    for rows in ([(0, 4), (4, 7)], [(7, 8)]):
        n = sum(b - a for a, b in rows)
        g = None
        for a, b in rows:   # rank 0's shard first: its BN buffers are the ones rank 0 keeps
            _, _, gr, _ = O.forward_backward(sd, x[a:b], t[a:b], 4, LP)
            w = (b - a) / n
            g = {k: w * v for k, v in gr.items()} if g is None else {k: g[k] + w * v for k, v in gr.items()}
        sd, mom, _, _ = O.clip_and_sgd(sd, g, mom)
    for n in O.param_names(sd0):
        assert np.array_equal(r0["param." + n], r1["param." + n]), n       # identical replicas
        if n.endswith(ZERO):
            continue
        upd, upd_ref = r0["param." + n] - sd0[n].numpy(), (sd[n] - sd0[n]).numpy()
        assert rel(upd, upd_ref) < 3e-3, n
