"""One rank of the data-parallel Trainer rehearsal (tests/test_gpu_trainer.py): W processes share one
GPU through a gloo group and run the reference's wiring unchanged -- torch.optim.SGD + Trainer over
dict batches (train.py:73-88) -- on the global batch of tests/golden/ddp_shards.npz (8 images).  The
Trainer shards each batch by rank, all-reduces the flat gradient buffer, applies 1/W in the fused
clip + SGD, sums the metric vector over the ranks, broadcasts rank 0's BatchNorm statistics before
validating and writes checkpoints on rank 0 only.  Writes this rank's results to an .npz.

  python tools/trainer_ddp_check.py RANK WORLD PORT OUT.npz LOGDIR [ragged]

``ragged``: one epoch of two global batches that do not divide over the ranks -- the first 7 images
(rows 4 / 3 at world 2) and the 8th image alone (rank 1 has no rows: zero gradients through the same
collectives) -- with rank 1's replica deliberately started from perturbed weights (the reducer's
broadcast from rank 0 must undo that).  Writes the parameters after the epoch.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]
LP = {"bce_weight": 0.5, "dice_weight": 0.5}


def main():
    rank, world, port, out, logdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from models.unet_dfc_sa_res import UNetDFCSARes
        from utils.trainer import Trainer
        fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "model_small.npz")))
        dd = dict(np.load(os.path.join(ROOT, "tests", "golden", "ddp_shards.npz")))
        model = UNetDFCSARes(3, 1, [8, 16, 32, 64], pool_size=4, precision="fp32")
        model.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("sd0.")})
        opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
        cfg = {"training": {"num_epochs": 1, "save_checkpoint_freq": 1, "loss": {"type": "bce_dice", "params": LP}},
               "logging": {"log_dir": os.path.join(logdir, f"r{rank}"), "images_dir": os.path.join(logdir, f"i{rank}"),
                           "save_best_worst_samples": 1}}
        batches = [{"image": torch.from_numpy(dd["x"]), "mask": torch.from_numpy(dd["t"]),
                    "filename": [f"s{i}" for i in range(8)]}]
        if len(sys.argv) > 6 and sys.argv[6] == "ragged":
            x, t = torch.from_numpy(dd["x"]), torch.from_numpy(dd["t"])
            rb = [{"image": x[:7], "mask": t[:7]}, {"image": x[7:], "mask": t[7:]}]
            if rank == 1:
                with torch.no_grad():
                    for p in model.parameters():
                        p.add_(0.01)
            model.cuda()
            tr = Trainer(model, rb, rb[:1], opt, dev, cfg)
            loss, iou, dice = tr.train_epoch(0)
            torch.cuda.synchronize()
            res = {"loss": np.float64(loss), "iou": np.float64(iou), "dice": np.float64(dice)}
            res.update({"param." + n: p.detach().cpu().numpy() for n, p in model.named_parameters()})
            np.savez(out, **res)
            return
        tr = Trainer(model, batches, batches, opt, dev, cfg)
        loss, iou, dice = tr.train_epoch(0)
        torch.cuda.synchronize()
        res = {"loss": np.float64(loss), "iou": np.float64(iou), "dice": np.float64(dice)}
        res.update({"grad." + n: p.grad.detach().cpu().numpy() for n, p in model.named_parameters()})
        res.update({"param." + n: p.detach().cpu().numpy() for n, p in model.named_parameters()})
        res.update({"trainbuf." + n: b.detach().cpu().numpy() for n, b in model.named_buffers() if "running" in n})
        va = tr.validate_epoch(batches)
        res["val_dice"] = np.float64(va["dice"])
        res.update({"buf." + n: b.detach().cpu().numpy() for n, b in model.named_buffers() if "running" in n})
        tr.save_checkpoint(0, va, is_best=True)
        np.savez(out, **res)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
