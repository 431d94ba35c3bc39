"""autograd nodes for the U-Net plumbing around the DFC blocks (all on libdfcsa kernels).

  InputToNHWC    NCHW fp32 images -> NHWC dtype (channels zero-padded to a multiple of 8)
  MaxPool2x2     nn.MaxPool2d(2, 2)                          unet_dfc_sa_res.py:132-141
  ConvTranspose  nn.ConvTranspose2d(k=2, s=2) as one GEMM    unet_dfc_sa_res.py:147-156
  ResizeBilinear F.interpolate(bilinear) shape fix          unet_dfc_sa_res.py:180-199
  Head1x1        final_conv -> NCHW fp32 logits              unet_dfc_sa_res.py:159, 203
"""
import torch

from . import ops
from ._lib import call
from .block import grad_of
from .ddp import notify_grads_ready
from .ops import P, dt, rup, stream
from .packs import get_packset, param_key
from .streams import on_side


class InputToNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype, cpad):
        B, Cin, H, W = x.shape
        x = x.contiguous().float()
        out = torch.empty((B, H, W, cpad), dtype=dtype, device=x.device)
        call("dfcsa_pack_input", dt(dtype), B, Cin, H, W, P(x), cpad, P(out), stream())
        ctx.cin = Cin
        return out

    @staticmethod
    def backward(ctx, g):
        # only standalone block/attention modules need this (the U-Net input needs no grad)
        return g[..., :ctx.cin].permute(0, 3, 1, 2).float(), None, None


class MaxPool2x2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        B, H, W, C = x.shape
        out = torch.empty((B, H // 2, W // 2, C), dtype=dtype, device=x.device)
        call("dfcsa_maxpool2_fwd", dt(dtype), B, H, W, C, P(x), P(out), stream())
        ctx.save_for_backward(x)
        ctx.dtype = dtype
        return out

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        B, H, W, C = x.shape
        dx = torch.zeros_like(x)
        call("dfcsa_maxpool2_bwd", dt(ctx.dtype), B, H, W, C, P(x), P(g.contiguous()), P(dx), stream())
        return dx, None


class MaxPoolFork(torch.autograd.Function):
    """d -> (maxpool2x2(d), d): an encoder output feeds both the next level (reference
    models/unet_dfc_sa_res.py:165-172, pool1..pool4) and the decoder skip (:179-201).  Its backward
    forms dd = dskip + maxpool_bwd(dpooled) in one pass: the pooling-gradient kernel accumulates
    into the skip gradient (a fresh tensor from the decoder block's dgrad GEMM) instead of a
    zero-filled buffer that autograd would then add to the skip gradient."""

    @staticmethod
    def forward(ctx, x, dtype):
        B, H, W, C = x.shape
        out = torch.empty((B, H // 2, W // 2, C), dtype=dtype, device=x.device)
        call("dfcsa_maxpool2_fwd", dt(dtype), B, H, W, C, P(x), P(out), stream())
        ctx.save_for_backward(x)
        ctx.dtype = dtype
        return out, x.view_as(x)

    @staticmethod
    def backward(ctx, g_pool, g_skip):
        (x,) = ctx.saved_tensors
        B, H, W, C = x.shape
        if g_skip is None:
            dx = torch.zeros_like(x)
        elif g_skip.is_contiguous() and g_skip.dtype == x.dtype and g_skip.shape == x.shape:
            dx = g_skip
        else:
            dx = g_skip.to(x.dtype).contiguous().clone()
        if g_pool is not None:
            call("dfcsa_maxpool2_bwd", dt(ctx.dtype), B, H, W, C, P(x), P(g_pool.contiguous()), P(dx), stream())
        return dx, None


class ConvTranspose2x2(torch.autograd.Function):
    """out[b, 2h+i, 2w+j, co] = sum_ci x[b,h,w,ci] W[ci,co,i,j] + bias[co]: one GEMM with N = 4*Cout
    and a pixel-shuffle epilogue; dgrad = stride-2 gather GEMM; wgrad = pixel reduction."""

    @staticmethod
    def forward(ctx, x, mod, dtype, *params):
        B, h, w, Cin = x.shape
        Cout = mod.out_channels
        dev = x.device
        Kf = rup(Cin, ops.KALIGN)
        Kb = rup(4 * Cout, ops.KALIGN)
        pk = get_packset(mod, (dtype, param_key(mod)), lambda ps: _convT_packs(ps, mod, dtype, Kf, Kb))
        Wf, Wb, b4 = pk["Wf"], pk["Wb"], pk["b4"]
        out = torch.empty((B, 2 * h, 2 * w, Cout), dtype=dtype, device=dev)
        ops.conv_gemm(dtype, [(x, 0, 0)], Cin, (B, h, w), (h, w), Wf, Kf, 4 * Cout, [out], Cout, bias=b4,
                      mode=1, out_hw=(2 * h, 2 * w))
        ctx.save_for_backward(x)
        ctx.mod, ctx.dtype, ctx.Wb, ctx.Kb, ctx.np = mod, dtype, Wb, Kb, len(params)
        return out

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        mod, dtype = ctx.mod, ctx.dtype
        B, h, w, Cin = x.shape
        Cout = mod.out_channels
        g = g.contiguous()
        segs = [(g, i, j) for i in range(2) for j in range(2)]
        # input gradient first (critical path), then the weight / bias gradients on the side stream
        # (see dfcsa.block.block_backward: the dgrad launched first keeps its CUs)
        from .block import DX_FIRST
        dx = None
        if ctx.needs_input_grad[0] and DX_FIRST[0]:
            dx = torch.empty_like(x)
            ops.conv_gemm(dtype, segs, Cout, (B, h, w), (2 * h, 2 * w), ctx.Wb, ctx.Kb, Cin, [dx], Cin, stride=2)
        with on_side(x.device, x, g):
            ops.conv_wgrad_into(dtype, [x], Cin, segs, Cout, (B, h, w), (2 * h, 2 * w), [grad_of(mod.weight)],
                                ntaps=4, Ctot=Cout, Creal=Cout, layout=1, stride=2)
            ops.channel_sum_into(dtype, g, grad_of(mod.bias))
        if ctx.needs_input_grad[0] and not DX_FIRST[0]:
            dx = torch.empty_like(x)
            ops.conv_gemm(dtype, segs, Cout, (B, h, w), (2 * h, 2 * w), ctx.Wb, ctx.Kb, Cin, [dx], Cin, stride=2)
        notify_grads_ready(mod)
        return (dx, None, None, *([None] * ctx.np))


def _convT_packs(ps, mod, dtype, Kf, Kb):
    """Wb[ci][ij*Cout + co] = W[ci][co][ij] (dgrad operand, phase A); Wf = Wb^T (forward operand,
    rows ij*Cout + co, phase B); b4[ij*Cout + co] = bias[co]."""
    Cin, Cout = mod.weight.shape[0], mod.weight.shape[1]
    Wb = ps.rows("Wb", dtype, mod.weight, Cout, Kb)
    ps.transpose(Wb, 0, 0, Cin, 4 * Cout, "Wf", (4 * Cout, Kf))
    ps.bias4("b4", mod.bias)


class ResizeBilinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, size, dtype):
        B, Hi, Wi, C = x.shape
        Ho, Wo = size
        out = torch.empty((B, Ho, Wo, C), dtype=dtype, device=x.device)
        call("dfcsa_resize_bilinear", dt(dtype), B, C, Hi, Wi, Ho, Wo, P(x), P(out), stream())
        ctx.shape, ctx.dtype = (B, Hi, Wi, C, Ho, Wo), dtype
        return out

    @staticmethod
    def backward(ctx, g):
        B, Hi, Wi, C, Ho, Wo = ctx.shape
        acc = torch.zeros((B, Hi, Wi, C), dtype=torch.float32, device=g.device)
        call("dfcsa_resize_bilinear_bwd", dt(ctx.dtype), B, C, Hi, Wi, Ho, Wo, P(g.contiguous()), P(acc), stream())
        dx = torch.empty((B, Hi, Wi, C), dtype=ctx.dtype, device=g.device)
        call("dfcsa_cast_f32", dt(ctx.dtype), acc.numel(), P(acc), P(dx), 0, stream())
        return dx, None, None


class Head1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, dtype, *params):
        B, H, W, C = x.shape
        Cout = mod.out_channels
        logits = torch.empty((B, Cout, H, W), dtype=torch.float32, device=x.device)
        call("dfcsa_head_fwd", dt(dtype), B, H * W, C, Cout, P(x), P(mod.weight), P(mod.bias), P(logits), stream())
        ctx.save_for_backward(x)
        ctx.mod, ctx.dtype, ctx.np = mod, dtype, len(params)
        return logits

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        mod, dtype = ctx.mod, ctx.dtype
        B, H, W, C = x.shape
        Cout = mod.out_channels
        import ctypes
        nt = ctypes.c_int()
        call("dfcsa_head_bwd", dt(dtype), B, H * W, C, Cout, None, None, None, None, None, None,
             ctypes.addressof(nt), stream())
        pw = torch.empty(nt.value * Cout * C, dtype=torch.float32, device=x.device)
        pb = torch.empty(nt.value * Cout, dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x)
        call("dfcsa_head_bwd", dt(dtype), B, H * W, C, Cout, P(x), P(mod.weight), P(g.contiguous()), P(dx), P(pw),
             P(pb), None, stream())
        ops.colsum_into(pw, nt.value, Cout * C, grad_of(mod.weight))
        ops.colsum_into(pb, nt.value, Cout, grad_of(mod.bias))
        notify_grads_ready(mod)
        return (dx if ctx.needs_input_grad[0] else None, None, None, *([None] * ctx.np))
