"""autograd nodes of the ablation-zoo blocks (reference models/unet_dfc_sa_ablation_branches.py,
_fusion.py, _placement.py) on libdfcsa.  The blocks are compositions of:

  ConvBNReLU (dfcsa.unet_ops)  conv_branch (3x3) and the attention entry (1x1): Conv -> BN -> ReLU
  LSAFunction (dfcsa.block)    LightSelfAttention on the activated entry
  Conv1x1                      residual_conv (1x1, no bias) over the NHWC sources
  SumOut                       out = a (+ b) + res_scale * res  (branches :62-70, :93-101,
                               fusion :35-49, :86-100)
  BlockGate                    identity on the block inputs whose backward runs after every node
                               of the block, so it reports the block's gradients as final to the
                               data-parallel bucket reducer
"""
import ctypes

import torch

from . import ops
from ._lib import call
from .block import grad_of
from .ddp import notify_grads_ready
from .ops import P, S, dt, rup, stream
from .packs import get_packset, param_key


def _conv1_packs(ps, conv, dtype, Cin_p, C):
    Wf = ps.rows("Wf", dtype, conv.weight, Cin_p, rup(Cin_p, ops.KALIGN))
    ps.transpose(Wf, 0, 0, C, Cin_p, "Wt", (Cin_p, rup(C, ops.KALIGN)), dc0=0)


class Conv1x1(torch.autograd.Function):
    """y = conv1x1(cat(xs)) (+ bias); backward: weight gradient GEMM (+ bias column sums) and the
    dgrad GEMM split back over the sources."""

    @staticmethod
    def forward(ctx, conv, dtype, nsrc, *args):
        xs = list(args[:nsrc])
        B, H, W, Cs = xs[0].shape
        Cin_p, C = nsrc * Cs, conv.out_channels
        if conv.kernel_size != (1, 1) or conv.in_channels > Cin_p or C % 8:
            raise ValueError(f"Conv1x1: 1x1 conv {conv.in_channels}->{C} over {Cin_p} source channels")
        pk = get_packset(conv, (dtype, nsrc, Cs, param_key(conv)), lambda ps: _conv1_packs(ps, conv, dtype, Cin_p, C))
        y = torch.empty((B, H, W, C), dtype=dtype, device=xs[0].device)
        ops.conv_gemm(dtype, [(x, 0, 0) for x in xs], Cs, (B, H, W), (H, W), pk["Wf"], rup(Cin_p, ops.KALIGN), C,
                      [y], C, bias=conv.bias)
        ctx.conv, ctx.dtype, ctx.nsrc, ctx.np, ctx.xs, ctx.pk = conv, dtype, nsrc, len(args) - nsrc, xs, pk
        return y

    @staticmethod
    def backward(ctx, dout):
        conv, dtype, xs = ctx.conv, ctx.dtype, ctx.xs
        dout = dout.contiguous()
        B, H, W, Cs = xs[0].shape
        C = conv.out_channels
        grid, hw = (B, H, W), (H, W)
        ops.conv_wgrad_into(dtype, [dout], C, [(x, 0, 0) for x in xs], Cs, grid, hw, [grad_of(conv.weight)], 1,
                            ctx.nsrc * Cs, conv.in_channels)
        if conv.bias is not None:
            ops.channel_sum_into(dtype, dout, grad_of(conv.bias))
        dxs = [None] * ctx.nsrc
        if any(ctx.needs_input_grad[3:3 + ctx.nsrc]):
            dxs = [torch.empty((B, H, W, Cs), dtype=dtype, device=dout.device) for _ in range(ctx.nsrc)]
            ops.conv_gemm(dtype, [(dout, 0, 0)], C, grid, hw, ctx.pk["Wt"], rup(C, ops.KALIGN), ctx.nsrc * Cs, dxs,
                          Cs)
        ctx.xs = None
        return (None, None, None, *dxs, *([None] * ctx.np))


class SumOut(torch.autograd.Function):
    """out = a (+ b) + res_scale * res; grad(res_scale) += sum(dout * res)."""

    @staticmethod
    def forward(ctx, dtype, res_scale, a, b, res):
        B, H, W, C = a.shape
        out = torch.empty_like(a)
        call("dfcsa_sum_out", dt(dtype), B * H * W, C, P(a), P(b), P(res), P(res_scale), P(out), stream())
        ctx.dtype, ctx.rs, ctx.res, ctx.has_b = dtype, res_scale, res, b is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        dout = dout.contiguous()
        res = ctx.res
        B, H, W, C = dout.shape
        M = B * H * W
        nte = ops.ntiles_ew(M, C)
        part = torch.empty(nte * C, device=dout.device, dtype=torch.float32)
        dres = torch.empty_like(res) if ctx.needs_input_grad[4] else None
        call("dfcsa_bwd_sum_out", dt(ctx.dtype), M, C, P(dout), P(res), P(ctx.rs), P(dres), *S(part), stream())
        call("dfcsa_sum_into", P(part), nte * C, P(grad_of(ctx.rs)), stream())
        ctx.res = None
        return None, None, dout, (dout if ctx.has_b else None), dres


class BlockGate(torch.autograd.Function):
    """Identity on the block inputs; its backward fires once every node of the block has run."""

    @staticmethod
    def forward(ctx, block, nsrc, *args):
        ctx.block, ctx.nsrc, ctx.np = block, nsrc, len(args) - nsrc
        return tuple(x.view_as(x) for x in args[:nsrc])

    @staticmethod
    def backward(ctx, *grads):
        notify_grads_ready(ctx.block)
        return (None, None, *grads, *([None] * ctx.np))


def gate_inputs(block, xs):
    out = BlockGate.apply(block, len(xs), *xs, *block.parameters())
    return list(out) if isinstance(out, tuple) else [out]
