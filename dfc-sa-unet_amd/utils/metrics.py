"""Loss and metrics (drop-in for the reference's utils/metrics.py) on libdfcsa kernels.

``calculate_metrics(pred, target, loss_type, loss_params)`` keeps the reference's contract
(utils/metrics.py:211-264): pred are probabilities (after sigmoid), the result is
{'loss': 0-d tensor with grad, 'iou': float, 'dice': float}; the 'bce_dice' weights are read
from 'weight_bce' / 'weight_dice' (defaults 1.0) -- NOT from the yaml's 'bce_weight' /
'dice_weight' keys, exactly like the reference.  The thresholded IoU/Dice are counted over
the whole flattened batch.

'bce_dice' (the loss every config uses) and 'dice' (the reference's default when a config names no
loss, :251-252 -> dice_loss :6-24, smooth 1) run on the MI355X kernels -- 'dice' is the same fused
reduction with the BCE weight 0; the reference's 'tversky' and 'joint' losses (no config uses them)
are not built and raise NotImplementedError; an unknown type raises ValueError as in the reference.
"""
import torch
import torch.nn as nn

from dfcsa.loss import bce_dice, metrics_from_stats

_NOT_BUILT = ("tversky", "joint")


def dice_loss(pred, target, smooth=1.0):
    """1 - (2 sum pt + smooth) / (sum p + sum t + smooth) over the flattened batch (reference :6-24)."""
    if smooth != 1.0:
        raise NotImplementedError("dice_loss kernel uses the reference's smooth = 1")
    loss, _ = bce_dice(pred, target, 0.0, 1.0)
    return loss


class BCEDiceLoss(nn.Module):
    """w_bce * BCELoss + w_dice * dice_loss (reference :52-78)."""

    def __init__(self, weight_bce=1.0, weight_dice=1.0):
        super().__init__()
        self.weight_bce = weight_bce
        self.weight_dice = weight_dice

    def forward(self, inputs, targets, smooth=1.0):
        if smooth != 1.0:
            raise NotImplementedError("BCEDiceLoss kernel uses the reference's smooth = 1")
        loss, _ = bce_dice(inputs, targets, self.weight_bce, self.weight_dice)
        return loss


def calculate_metrics_device(pred, target, loss_type="dice", loss_params=None):
    """Like calculate_metrics but keeps everything on the device: returns
    {'loss': 0-d tensor, 'stats': fp32[8] device vector} (no host synchronisation)."""
    if loss_params is None:
        loss_params = {}
    if loss_type == "bce_dice":
        loss, stats = bce_dice(pred, target, loss_params.get("weight_bce", 1.0), loss_params.get("weight_dice", 1.0))
        return {"loss": loss, "stats": stats}
    if loss_type == "dice":   # reference :251-252: dice_loss(pred, target) = 1 - (2 sum pt + 1)/(sum p + sum t + 1)
        loss, stats = bce_dice(pred, target, 0.0, 1.0)
        return {"loss": loss, "stats": stats}
    if loss_type in _NOT_BUILT:
        raise NotImplementedError(f"loss type {loss_type!r} is not built on the MI355X path (only 'bce_dice' and 'dice')")
    raise ValueError(f"不支持的損失函數類型: {loss_type}")


def calculate_metrics(pred, target, loss_type="dice", loss_params=None):
    out = calculate_metrics_device(pred, target, loss_type, loss_params)
    iou, dice = metrics_from_stats(out["stats"])
    return {"loss": out["loss"], "iou": iou, "dice": dice}
