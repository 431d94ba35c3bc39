"""Where does the bf16 mode's error come from?  (GPU diagnostic, not a test.)

For the small model fixture (tests/golden/model_small.npz, weights sd0, batch x1) and a few extra
seeded batches this prints, as JSON lines:
  * logits / loss / IoU / Dice error of bf16 compute against fp32 compute (fp32 == reference to 1e-5);
  * per block, the ACCUMULATED error of the block output (bf16 run vs fp32 run);
  * per block and per stage (y1..y4, local, attn, fused, out), the LOCAL error: the bf16 block fed
    the fp32 block's exact inputs (rounded to bf16), against the fp32 block.
Usage: python tools/bf16_diag.py [--feats 8,16,32,64] [--img 32] [--batch 2] [--seeds 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dfc-sa-unet_amd")]

import dfcsa.block as Bk  # noqa: E402
from dfcsa.loss import metrics_from_stats, sigmoid  # noqa: E402
from models.unet_dfc_sa_res import UNetDFCSARes  # noqa: E402
from utils.metrics import calculate_metrics_device  # noqa: E402

STAGES = ("y1", "y2", "local", "attn", "y3", "fused", "y4")


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--feats", default="8,16,32,64")
    ap.add_argument("--img", type=int, default=32)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--seeds", type=int, default=5)
    ap.add_argument("--pool", type=int, default=4)
    a = ap.parse_args()
    feats = [int(v) for v in a.feats.split(",")]
    small = feats == [8, 16, 32, 64] and a.img == 32
    fx = dict(np.load(os.path.join(ROOT, "tests/golden/model_small.npz")))
    torch.manual_seed(0)
    model = UNetDFCSARes(3, 1, feats, pool_size=a.pool, precision="fp32")
    if small:
        model.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("sd0.")})
    else:
        with torch.no_grad():
            for n, p in model.named_parameters():
                if n.endswith("gamma"):
                    p.fill_(0.5)
    model = model.cuda().train()

    rec = []
    orig = Bk.block_forward

    def hook(blk, xs, pool, training, dtype):
        out, s = orig(blk, xs, pool, training, dtype)
        rec.append((blk, [x.detach().clone() for x in xs], out.detach().clone(),
                    {k: getattr(s, k).detach().clone() for k in STAGES}))
        return out, s

    Bk.block_forward = hook
    batches = []
    if small:
        batches.append(("fixture_x1", torch.from_numpy(fx["x1"]), torch.from_numpy(fx["t1"])))
    for sd in range(a.seeds):
        g = torch.Generator().manual_seed(100 + sd)
        x = torch.randn(a.batch, 3, a.img, a.img, generator=g)
        t = (torch.rand(a.batch, 1, a.img, a.img, generator=g) > 0.5).float()
        batches.append((f"seed{100 + sd}", x, t))
    for tag, x, t in batches:
        x, t = x.cuda(), t.cuda()
        res = {}
        for prec in (torch.float32, torch.bfloat16):
            model.compute_dtype = prec
            rec.clear()
            with torch.no_grad():
                lg = model(x)
                st = calculate_metrics_device(sigmoid(lg), t, "bce_dice", {})["stats"]
            iou, dice = metrics_from_stats(st)
            res[prec] = (lg.float().cpu(), float(st[0].item()), iou, dice, list(rec))
        l32, loss32, iou32, d32, rec32 = res[torch.float32]
        l16, loss16, iou16, d16, rec16 = res[torch.bfloat16]
        line = {"batch": tag, "logits_rel": rel(l16, l32), "loss_rel": abs(loss16 - loss32) / abs(loss32),
                "iou": [iou32, iou16], "dice": [d32, d16],
                "acc_block_out_rel": [round(rel(b[2].float(), f[2].float()), 5) for b, f in zip(rec16, rec32)]}
        if tag in ("fixture_x1", "seed100"):
            local = []
            with torch.no_grad():
                for blk, xs, out, st32 in rec32:
                    o16, s16 = orig(blk, [v.bfloat16() for v in xs], blk.pool_size, True, torch.bfloat16)
                    d = {k: round(rel(getattr(s16, k).float(), st32[k].float()), 5) for k in STAGES}
                    d["out"] = round(rel(o16.float(), out.float()), 5)
                    local.append(d)
            line["local_stage_rel"] = local
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
