"""End-to-end training parity: 20 training steps of the HIP Trainer (fp32 compute mode, the
HIP-graph-replayed step, fused clip + SGD) against the same 20 steps of the CPU oracle
(oracle/dfcsa_oracle.py: train_step = utils/trainer.py:115-151 + train.py:73-78 restated), then the
validation epoch of both (eval-mode BatchNorm with the trained running statistics,
utils/trainer.py:153-200): per-step training loss, validation loss and validation Dice / IoU.

SyntheticEllipses 64 x 64, features 16..128, pool_size 4, batch 4, momentum 0.9, weight decay 1e-4,
clip 1.0, lr 0.05 (at the reference's 0.01 twenty steps leave the validation Dice at ~1e-4: nothing
to compare; at 0.05 it is ~0.08).

Twenty SGD steps amplify rounding: the reference's own fp32 run and its float64 run (the same
oracle in float64) drift apart by up to 1e-3 in the step loss and 3e-4 in validation Dice by step
20 here (4e-3 / 5e-3 at lr 0.1).  Bars: validation Dice and IoU within max(1e-3, 3 x that fp32-vs-
float64 distance) of the oracle's fp32 run; step losses and the validation loss within
max(1e-3, 3 x the largest fp32-vs-float64 distance of the reference up to that step) relative; parameters after
20 steps within max(1e-3, 3 x the reference's fp32-vs-float64 distance) over the whole state
vector."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

LP = {"bce_weight": 0.5, "dice_weight": 0.5}
STEPS, BATCH, NVAL, LR = 20, 4, 3, 0.05


def batches(seed, nb):
    from utils.data_loader import SyntheticEllipses
    ds = SyntheticEllipses(nb * BATCH, (64, 64), seed=seed)
    out = []
    for b in range(nb):
        items = [ds[b * BATCH + i] for i in range(BATCH)]
        out.append({"image": torch.stack([s["image"] for s in items]), "mask": torch.stack([s["mask"] for s in items]),
                    "filename": [s["filename"] for s in items]})
    return out


def oracle_run(sd0, train, val, dt=torch.float32):
    from oracle import dfcsa_oracle as O
    sd, mom, losses = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in sd0.items()}, {}, []
    for b in train:
        sd, mom, r = O.train_step(sd, mom, b["image"].to(dt), b["mask"].to(dt), 4, LP, lr=LR)
        losses.append(r["loss"].item())
    vl = vi = vd = 0.0
    with torch.no_grad():
        for b in val:
            logits = O.unet_dfc_sa_res(b["image"].to(dt), sd, 4, training=False)
            m = O.calculate_metrics(torch.sigmoid(logits), b["mask"].to(dt), "bce_dice", LP)
            vl, vi, vd = vl + m["loss"].item(), vi + m["iou"], vd + m["dice"]
    n = len(val)
    return sd, losses, (vl / n, vi / n, vd / n)


def test_twenty_steps_then_validation_match_the_oracle(tmp_path):
    from models.unet_dfc_sa_res import UNetDFCSARes
    from utils.trainer import Trainer
    torch.manual_seed(2024)
    model = UNetDFCSARes(3, 1, [16, 32, 64, 128], pool_size=4, precision="fp32")
    sd0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    opt = torch.optim.SGD(model.parameters(), lr=LR, momentum=0.9, weight_decay=1e-4)
    cfg = {"training": {"num_epochs": 1, "loss": {"type": "bce_dice", "params": LP}},
           "logging": {"log_dir": str(tmp_path / "logs"), "images_dir": str(tmp_path / "img")}}
    train, val = batches(7, STEPS), batches(8, NVAL)
    tr = Trainer(model, train, val, opt, torch.device("cuda"), cfg)
    losses = []
    model.train()
    for b in train:           # train_epoch's loop, keeping every step's loss
        met = tr.train_step(b["image"].cuda(), b["mask"].cuda())
        losses.append(float(met["stats"][0].item()))
    assert tr._graphs, "the HIP-graph-replayed step was not exercised"
    va = tr.validate_epoch(val)
    torch.cuda.synchronize()

    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    sd_ref, losses_ref, (vl, vi, vd) = oracle_run(sd0, train, val)
    sd64, losses64, (vl64, vi64, vd64) = oracle_run(sd0, train, val, torch.float64)
    print(f"val dice HIP {va['dice']:.6f} oracle fp32 {vd:.6f} (oracle float64 {vd64:.6f}); val loss "
          f"{va['loss']:.6f} / {vl:.6f}; last train loss {losses[-1]:.6f} / {losses_ref[-1]:.6f}")
    print("step loss rel, HIP vs oracle fp32:   ", " ".join(f"{abs(a - b) / b:.1e}" for a, b in zip(losses, losses_ref)))
    print("step loss rel, oracle fp32 vs fp64:  ", " ".join(f"{abs(a - b) / b:.1e}" for a, b in zip(losses_ref, losses64)))
    env = 0.0   # the reference's fp32-vs-float64 drift so far (its envelope: one step's value is noisy)
    for i, (a, b, c) in enumerate(zip(losses, losses_ref, losses64)):
        env = max(env, abs(b - c) / abs(c))
        assert abs(a - b) <= max(1e-3, 3 * env) * abs(b), (i, a, b, c)
    assert abs(va["loss"] - vl) <= max(1e-3, 3 * abs(vl - vl64) / abs(vl64)) * abs(vl)
    assert vd > 0.05, "the validation Dice is trivial: nothing is compared"
    assert abs(va["dice"] - vd) <= max(1e-3, 3 * abs(vd - vd64))
    assert abs(va["iou"] - vi) <= max(1e-3, 3 * abs(vi - vi64))
    sd = model.state_dict()
    keys = [k for k in sd0 if sd0[k].is_floating_point()]
    vec = lambda d: torch.cat([d[k].detach().double().cpu().reshape(-1) for k in keys])  # noqa: E731
    a, b, c = vec(sd), vec(sd_ref), vec(sd64)
    d_ours, d_ref = ((a - b).norm() / b.norm()).item(), ((b - c).norm() / c.norm()).item()
    print(f"parameters after {STEPS} steps: HIP vs oracle fp32 {d_ours:.2e}, oracle fp32 vs float64 {d_ref:.2e}")
    assert d_ours <= max(1e-3, 3 * d_ref)
