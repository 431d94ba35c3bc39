"""torch.sigmoid (utils/trainer.py:124) and BCE+Dice loss with IoU/Dice counts
(utils/metrics.py:6-24, 52-78, 211-264) on libdfcsa kernels.

The reduction produces one fp32 device vector
  stats = [loss, sum bce, sum p*t, sum p, sum t, sum b*t, sum b, finite]   (b = p > 0.5)
so the loss stays on the device (no host sync) and the metrics can be read lazily.
"""
import ctypes

import torch

from ._lib import LIB, call
from .ops import P, stream


class Sigmoid(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous().float()
        y = torch.empty_like(x)
        call("dfcsa_sigmoid", ctypes.c_int64(x.numel()), P(x), P(y), stream())
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        dx = torch.empty_like(y)
        call("dfcsa_sigmoid_bwd", ctypes.c_int64(y.numel()), P(y), P(g.contiguous().float()), P(dx), stream())
        return dx


def sigmoid(x):
    return Sigmoid.apply(x)


class BCEDice(torch.autograd.Function):
    """loss = w_bce * mean BCE(p, t) (log clamped at -100) + w_dice * (1 - (2 sum pt + 1)/(sum p + sum t + 1))."""

    @staticmethod
    def forward(ctx, p, t, w_bce, w_dice):
        p = p.contiguous().float()
        t = t.contiguous().float()
        if p.shape != t.shape:
            raise ValueError(f"prediction {tuple(p.shape)} and target {tuple(t.shape)} differ in shape")
        n = p.numel()
        part = torch.empty(LIB.dfcsa_bce_dice_partial_count(n) * 6, dtype=torch.float32, device=p.device)
        stats = torch.empty(8, dtype=torch.float32, device=p.device)
        call("dfcsa_bce_dice_fwd", ctypes.c_int64(n), P(p), P(t), P(part), float(w_bce), float(w_dice), P(stats),
             stream())
        ctx.save_for_backward(p, t, stats)
        ctx.w = (float(w_bce), float(w_dice))
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)   # no zero-filled gradient for the stats output
        return stats[0], stats

    @staticmethod
    def backward(ctx, gloss, gstats):
        p, t, stats = ctx.saved_tensors
        dp = torch.empty_like(p)
        gl = gloss.contiguous().float() if gloss is not None else None
        call("dfcsa_bce_dice_bwd", ctypes.c_int64(p.numel()), P(p), P(t), P(stats), ctx.w[0], ctx.w[1], P(gl),
             P(dp), stream())
        return dp, None, None, None


def bce_dice(p, t, w_bce=1.0, w_dice=1.0):
    """Returns (loss 0-d tensor with grad, stats device vector)."""
    return BCEDice.apply(p, t, w_bce, w_dice)


def metrics_from_stats(stats):
    """IoU / Dice of the thresholded prediction exactly as utils/metrics.py:228-236 forms them
    (python floats from the fp32 sums).  One device->host copy."""
    s = stats.tolist()
    inter, sum_b, sum_t = s[5], s[6], s[4]
    union = (sum_b + sum_t) - inter
    iou = inter / (union + 1e-7)
    dice = (2.0 * inter) / (sum_b + sum_t + 1e-7)
    return iou, dice
