"""autograd nodes of the plain U-Net (reference models/unet.py, BASELINE config 1) on libdfcsa.

  ConvBNReLU      nn.Conv2d(3x3, p1) -> BatchNorm2d -> ReLU (DoubleConv, unet.py:9-16); the input
                  is the channel concat of NHWC sources (never materialised)
  MaxPool2x2Ceil  nn.MaxPool2d(2, ceil_mode=True)                          unet.py:26
  Crop            the crop-to-match of Up.forward                          unet.py:47-55
"""
import torch

from . import ops
from ._lib import call
from .block import grad_of, raise_eval_backward
from .ddp import notify_grads_ready
from .ops import P, S, dt, rup, stream
from .packs import get_packset, param_key
from .streams import side_or_main


def _taps(xs, k=3):
    if k == 1:
        return [(x, 0, 0) for x in xs]
    return [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]


def _dgrad_taps(dy, k=3):
    if k == 1:
        return [(dy, 0, 0)]
    return [(dy, 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)]


def _conv3_packs(ps, conv, dtype, Cin_p, C, k=3):
    """Wf [C][Kpad]: forward rows (k = tap*Cin_p + ci); Wt [Cin_p][Kpad(ntaps*C)]: dgrad rows,
    Wt[ci][tap*C + co] = Wf[co][tap*Cin_p + ci]."""
    nt = k * k
    Wf = ps.rows("Wf", dtype, conv.weight, Cin_p, rup(nt * Cin_p, ops.KALIGN))
    shape = (Cin_p, rup(nt * C, ops.KALIGN))
    for tap in range(nt):
        ps.transpose(Wf, 0, tap * Cin_p, C, Cin_p, "Wt", shape, dc0=tap * C)


class ConvBNReLU(torch.autograd.Function):
    """forward: y = conv(cat(xs)) (+bias, BN partial sums in the GEMM epilogue) -> BN (train: batch
    statistics; eval: running) -> ReLU.  backward: ReLU/BN backward with the per-channel sums,
    weight gradient GEMM, dgrad GEMM split back over the sources.  3x3/p1 or 1x1 convs."""

    @staticmethod
    def forward(ctx, conv, bn, dtype, nsrc, *args):
        xs = list(args[:nsrc])
        B, H, W, Cs = xs[0].shape
        if any(tuple(x.shape) != (B, H, W, Cs) for x in xs):
            raise ValueError("ConvBNReLU sources must share one NHWC shape")
        Cin_p, C = nsrc * Cs, conv.out_channels
        k = conv.kernel_size[0]
        if conv.in_channels > Cin_p or C % 8 or conv.kernel_size not in ((3, 3), (1, 1)) \
                or conv.padding != ((1, 1) if k == 3 else (0, 0)) or conv.stride != (1, 1):
            raise ValueError(f"ConvBNReLU: 3x3/p1 or 1x1 conv {conv.in_channels}->{C} over {Cin_p} source channels")
        M, dev = B * H * W, xs[0].device
        training = bn.training
        pk = get_packset(conv, (dtype, nsrc, Cs, param_key(conv)),
                         lambda ps: _conv3_packs(ps, conv, dtype, Cin_p, C, k))
        nt = ops.ntiles_gemm(M)
        st = torch.empty(nt * 2 * C, device=dev, dtype=torch.float32) if training else None
        y = torch.empty((B, H, W, C), dtype=dtype, device=dev)
        fold = ops.bn_fold_ok(training)
        ntw = ops.conv_gemm(dtype, _taps(xs, k), Cs, (B, H, W), (H, W), pk["Wf"], rup(k * k * Cin_p, ops.KALIGN), C,
                            [y], C, bias=conv.bias, stats=st, bn=(bn, conv.bias, C) if fold else None)
        if fold:
            ntw, bnst = ntw
        else:
            bnst = ops.bn_finalize(bn, conv.bias, st, ntw if training else nt, C, C, M, training)
        out = ops.bn_act(dtype, y, bnst, 1)
        ctx.conv, ctx.bn, ctx.dtype, ctx.nsrc, ctx.np = conv, bn, dtype, nsrc, len(args) - nsrc
        ctx.xs, ctx.y, ctx.bnst, ctx.pk = xs, y, bnst, pk
        ctx.training = training
        return out

    @staticmethod
    def backward(ctx, dout):
        if not ctx.training:
            raise_eval_backward()
        conv, bn, dtype, xs, y, bnst = ctx.conv, ctx.bn, ctx.dtype, ctx.xs, ctx.y, ctx.bnst
        B, H, W, C = y.shape
        Cs = xs[0].shape[-1]
        M = B * H * W
        nte = ops.ntiles_ew(M, C)
        dz = torch.empty_like(y)
        part = torch.empty(nte * 2 * C, device=y.device, dtype=torch.float32)
        call("dfcsa_bwd_relu_bn", dt(dtype), M, C, P(dout.contiguous()), P(y), P(bnst.scale), P(bnst.shift),
             P(bnst.mean), P(bnst.invstd), P(dz), *S(part), stream())
        coef = ops.bn_bwd_finalize(part, nte, 2, C, M, grad_of(bn.weight), grad_of(bn.bias))
        dy = ops.bn_bwd_apply(dtype, dz, y, bnst, bn.weight, coef,
                              grad_of(conv.bias) if conv.bias is not None else None)
        del dz
        grid, hw = (B, H, W), (H, W)
        k = conv.kernel_size[0]
        # the weight gradient on the side stream beside the input-gradient GEMM (dfcsa.streams)
        with side_or_main(y.device, dy, *xs):
            ops.conv_wgrad_into(dtype, [dy], C, _taps(xs, k), Cs, grid, hw, [grad_of(conv.weight)], k * k,
                                ctx.nsrc * Cs, conv.in_channels)
        notify_grads_ready(conv)
        dxs = [None] * ctx.nsrc
        if any(ctx.needs_input_grad[4:4 + ctx.nsrc]):
            dxs = [torch.empty((B, H, W, Cs), dtype=dtype, device=y.device) for _ in range(ctx.nsrc)]
            ops.conv_gemm(dtype, _dgrad_taps(dy, k), C, grid, hw, ctx.pk["Wt"], rup(k * k * C, ops.KALIGN),
                          ctx.nsrc * Cs, dxs, Cs)
        ctx.xs = ctx.y = None
        return (None, None, None, None, *dxs, *([None] * ctx.np))


class MaxPool2x2Ceil(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        B, H, W, C = x.shape
        out = torch.empty((B, (H + 1) // 2, (W + 1) // 2, C), dtype=dtype, device=x.device)
        call("dfcsa_maxpool2_ceil_fwd", dt(dtype), B, H, W, C, P(x), P(out), stream())
        ctx.save_for_backward(x)
        ctx.dtype = dtype
        return out

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        B, H, W, C = x.shape
        dx = torch.empty_like(x)
        call("dfcsa_maxpool2_ceil_bwd", dt(ctx.dtype), B, H, W, C, P(x), P(g.contiguous()), P(dx), stream())
        return dx, None


class Crop(torch.autograd.Function):
    """out = x[:, oy:oy+Ho, ox:ox+Wo, :] (NHWC copy); backward pads the gradient back with zeros."""

    @staticmethod
    def forward(ctx, x, oy, ox, Ho, Wo, dtype):
        B, H, W, C = x.shape
        out = torch.empty((B, Ho, Wo, C), dtype=dtype, device=x.device)
        call("dfcsa_window_copy", dt(dtype), B, C, H, W, P(x), Ho, Wo, P(out), oy, ox, stream())
        ctx.geo, ctx.dtype = (B, H, W, C, oy, ox, Ho, Wo), dtype
        return out

    @staticmethod
    def backward(ctx, g):
        B, H, W, C, oy, ox, Ho, Wo = ctx.geo
        dx = torch.empty((B, H, W, C), dtype=ctx.dtype, device=g.device)
        call("dfcsa_window_copy", dt(ctx.dtype), B, C, Ho, Wo, P(g.contiguous()), H, W, P(dx), -oy, -ox, stream())
        return dx, None, None, None, None, None
