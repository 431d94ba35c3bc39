"""Sliding-window inference and segmentation counts (drop-in for the reference's inference.py
:73-153: ``calculate_segmentation_metrics``, ``predict_single_image``, ``predict_large_image``;
the global metrics of :346-353 as ``global_metrics``).

MI355X path:
  * the whole image is uploaded once (uint8 HWC) and stays in HBM;
  * ``dfcsa_tiles_gather`` cuts every tile, applies ToTensor + ImageNet Normalize
    (inference.py:116-119) and, with TTA, also writes the h- and v-flipped tile
    (:136-139), straight into the model's NCHW fp32 input batch;
  * the model runs on batches of tiles.  It is in eval mode, so BatchNorm uses running
    statistics and a tile's logits do not depend on its batch-mates;
  * ``dfcsa_tiles_accumulate`` applies the sigmoid, averages the TTA variants, un-flipping them,
    and overlap-averages the canvas (:132-151).  Every pixel sums its tiles in the reference's
    y-major loop order, so the fp32 sums are formed in the same order;
  * ``dfcsa_seg_counts`` thresholds and counts TP/FP/FN exactly (TN by difference).

The folder CLI, file IO and visualisation of inference.py:155-398 are out of scope.
"""
import ctypes

import numpy as np
import torch

from dfcsa._lib import call
from dfcsa.loss import sigmoid
from dfcsa.ops import P, stream

IMAGENET_MEAN_STD = (0.485, 0.456, 0.406, 0.229, 0.224, 0.225)


def _cuda(device):
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError("inference runs on the MI355X kernels only; pass device='cuda'")
    return dev


def tile_grid(h, w, tile_size, overlap):
    """Tile origins of inference.py:121-131.  y and x run over range(0, extent, stride); a tile ends
    at min(start + tile, extent) and starts at max(0, end - tile), so every tile is
    min(tile, h) x min(tile, w).  Returns (ys, xs, th, tw); tile t = iy * len(xs) + ix."""
    stride = tile_size - overlap
    if stride <= 0:
        raise ValueError(f"overlap ({overlap}) must be smaller than tile_size ({tile_size})")
    ys = [max(0, min(y + tile_size, h) - tile_size) for y in range(0, h, stride)]
    xs = [max(0, min(x + tile_size, w) - tile_size) for x in range(0, w, stride)]
    return ys, xs, min(tile_size, h), min(tile_size, w)


def _image_u8(image, dev):
    t = image if isinstance(image, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(image))
    if t.dtype != torch.uint8 or t.dim() != 3:
        raise TypeError("expected a uint8 H x W x C image (load_image's original_image)")
    return t.to(dev).contiguous()


def _gt_u8(gt, dev):
    t = gt if isinstance(gt, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(gt))
    if t.dtype != torch.uint8 or t.dim() not in (2, 3):
        raise TypeError("expected a uint8 H x W or H x W x 3 ground-truth mask")
    return (t.unsqueeze(-1) if t.dim() == 2 else t).to(dev).contiguous()


@torch.no_grad()
def predict_large_image(model, image, tile_size, overlap, device, use_tta=False, tiles_per_batch=32,
                        return_tensor=False):
    """Probability canvas [H, W] of ``image`` (uint8 H x W x 3) by overlapping tiles
    (inference.py:104-153).  ``tiles_per_batch`` tiles (x3 with TTA) go through the model per
    launch sequence.  Returns numpy fp32 like the reference, or the device tensor."""
    model.eval()
    dev = _cuda(device)
    img = _image_u8(image, dev)
    H, W, C = img.shape
    ys, xs, th, tw = tile_grid(H, W, tile_size, overlap)
    ny, nx = len(ys), len(xs)
    T, V = ny * nx, (3 if use_tta else 1)
    ty = torch.tensor([y for y in ys for _ in xs], dtype=torch.int32, device=dev)
    tx = torch.tensor([x for _ in ys for x in xs], dtype=torch.int32, device=dev)
    ms = (ctypes.c_float * (2 * C))(*(IMAGENET_MEAN_STD[:C] + IMAGENET_MEAN_STD[3:3 + C]))
    per = max(1, int(tiles_per_batch))
    batch = torch.empty((min(per, T) * V, C, th, tw), dtype=torch.float32, device=dev)
    logits = torch.empty((T * V, th, tw), dtype=torch.float32, device=dev)
    for t0 in range(0, T, per):
        n = min(per, T - t0)
        inp = batch[:n * V]
        call("dfcsa_tiles_gather", P(img), H, W, C, P(ty[t0:]), P(tx[t0:]), n, th, tw, V, ms, P(inp), stream())
        out = model(inp)
        if out.shape[1] != 1:
            raise ValueError("sliding-window inference expects a single-channel (binary) model")
        logits[t0 * V:(t0 + n) * V].copy_(out.reshape(n * V, th, tw))
    canvas = torch.empty((H, W), dtype=torch.float32, device=dev)
    ys_d = torch.tensor(ys, dtype=torch.int32, device=dev)
    xs_d = torch.tensor(xs, dtype=torch.int32, device=dev)
    call("dfcsa_tiles_accumulate", P(logits), P(ys_d), ny, P(xs_d), nx, th, tw, V, H, W, P(canvas), stream())
    return canvas if return_tensor else canvas.cpu().numpy()


@torch.no_grad()
def predict_single_image(model, image_tensor, device):
    """inference.py:93-102: sigmoid of the model output for one [1, 3, H, W] tensor -> [H, W]."""
    model.eval()
    out = model(image_tensor.to(_cuda(device)))
    return sigmoid(out).squeeze(0).squeeze(0).cpu().numpy()


def segmentation_counts(prob, gt, threshold=0.5, gt_threshold=128):
    """TP/FP/FN/TN of (prob > threshold) against (gt > gt_threshold) on the device.  ``gt`` is
    uint8 [H, W] or [H, W, 3] (3 channels: OpenCV RGB2GRAY first, inference.py:300-305)."""
    if not (isinstance(prob, torch.Tensor) and prob.is_cuda):
        raise RuntimeError("segmentation_counts needs the probability map on the GPU")
    dev = prob.device
    p = prob.contiguous().float()
    g = _gt_u8(gt, dev)
    n = p.numel()
    if g.shape[0] * g.shape[1] != n:
        raise ValueError(f"ground truth {tuple(g.shape)} does not match the prediction {tuple(p.shape)}")
    counts = torch.empty(4, dtype=torch.int64, device=dev)
    call("dfcsa_seg_counts", p.data_ptr(), ctypes.c_int64(n), ctypes.c_float(threshold), P(g), g.shape[2],
         int(gt_threshold), P(counts), stream())
    tp, fp, fn, _ = (int(v) for v in counts.tolist())
    return {"tp": tp, "fp": fp, "fn": fn, "tn": n - tp - fp - fn}


def calculate_segmentation_metrics(pred_binary, gt_binary):
    """inference.py:73-91: counts of (pred > 0) against (gt > 0) for two binary maps (numpy or
    device tensors); computed on the GPU."""
    dev = _cuda("cuda")
    pb = pred_binary if isinstance(pred_binary, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(pred_binary))
    gb = gt_binary if isinstance(gt_binary, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(gt_binary))
    gb = (gb.to(dev) > 0).to(torch.uint8)
    return segmentation_counts(pb.to(dev).float(), gb, threshold=0.0, gt_threshold=0)


def per_image_metrics(c):
    """The per-file metrics of inference.py:317-321 from one image's counts."""
    tp, fp, fn, tn = c["tp"], c["fp"], c["fn"], c["tn"]
    return {"iou": tp / (tp + fp + fn + 1e-7), "dice_f1": (2 * tp) / (2 * tp + fp + fn + 1e-7),
            "accuracy": (tp + tn) / (tp + tn + fp + fn + 1e-7), "recall": tp / (tp + fn + 1e-7),
            "precision": tp / (tp + fp + 1e-7), **c}


def global_metrics(counts_list):
    """Global IoU / Dice / accuracy / recall / precision over summed counts (inference.py:346-353)."""
    tot = {k: sum(c[k] for c in counts_list) for k in ("tp", "fp", "fn", "tn")}
    m = per_image_metrics(tot)
    return {k: m[k] for k in ("iou", "dice_f1", "accuracy", "recall", "precision")}


@torch.no_grad()
def evaluate_image(model, image, gt, tile_size=224, overlap=50, threshold=0.5, use_tta=False, device="cuda"):
    """Sliding-window prediction + counts of one image against its mask, device-resident end to end
    (inference.py:284-314 in sliding-window mode: the mask needs no resize).  Returns
    (probability canvas as a device tensor, per-image metrics dict)."""
    prob = predict_large_image(model, image, tile_size, overlap, device, use_tta=use_tta, return_tensor=True)
    c = segmentation_counts(prob, gt, threshold=threshold, gt_threshold=128)
    return prob, per_image_metrics(c)
