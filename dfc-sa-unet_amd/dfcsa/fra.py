"""Full-resolution self-attention (reference models/unet_dfc_sa_ablation_attention.py:7-26) on the
flash-style kernels of csrc/fra.hip.

forward (a = the NHWC attention input, C channels, Cq = C // 8):
    qkv = a @ [Wq | Wk | Wv]^T + [bq | bk | bv]   one implicit GEMM (1x1), [M][Jp] compute dtype
    O, lse = flash(q, k, v)                        dfcsa_fra_fwd; y = gamma * O + a in its epilogue
backward (dy at y):
    r = rowsum(dy * O)                             dfcsa_fra_bwd_prep; dgamma = sum r
    dqkv = flash_bwd(q, k, v, dy, lse, r)          dfcsa_fra_bwd (P recomputed from lse); C > 256:
                                                   dfcsa_fra_bwd_wide (value-column chunks of 128)
    dW = dqkv^T a, db = colsum(dqkv)               weight-gradient GEMM + channel sums
    da = dy + dqkv @ Wqkv                          dgrad GEMM accumulated onto dy
Jp = 2 Cq + C rounded up to a multiple of 8 (zero weight rows; only the tiny test widths pad).
"""
import ctypes

import torch

from . import _lib, ops
from ._lib import call
from .ops import P, S, dt, rup, stream
from .packs import get_packset, param_key


def _grad_of(p):
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


def widths(mod):
    """(C, Cq, J, Jp) of a FullResolutionAttention module."""
    C = mod.value_conv.out_channels
    Cq = mod.query_conv.out_channels
    J = 2 * Cq + C
    return C, Cq, J, rup(J, 8)


def build_packs(ps, mod, dtype):
    """Wqkv [Jp][Kpad(C)] (rows q | k | v, forward operand), WqkvT [C][Kpad(Jp)] (dgrad operand),
    bqkv [Jp] fp32."""
    C, Cq, J, Jp = widths(mod)
    for w, off in ((mod.query_conv.weight, 0), (mod.key_conv.weight, Cq), (mod.value_conv.weight, 2 * Cq)):
        Wf = ps.rows("Wqkv", dtype, w, C, rup(C, ops.KALIGN), row0=off, rows=Jp)
    ps.concat("bqkv", [mod.query_conv.bias, mod.key_conv.bias, mod.value_conv.bias], Jp)
    ps.transpose(Wf, 0, 0, Jp, C, "WqkvT", (C, rup(Jp, ops.KALIGN)))


def core_forward(mod, a, dtype, pk):
    """a: NHWC [B,H,W,C] -> (y = gamma * attention(a) + a, saved)."""
    B, H, W, C = a.shape
    _, Cq, J, Jp = widths(mod)
    if C != mod.value_conv.in_channels:
        raise ValueError(f"attention over {mod.value_conv.in_channels} channels got {C}")
    dev = a.device
    N = H * W
    qkv = torch.empty((B, H, W, Jp), dtype=dtype, device=dev)
    ops.conv_gemm(dtype, [(a, 0, 0)], C, (B, H, W), (H, W), pk["Wqkv"], rup(C, ops.KALIGN), Jp, [qkv], Jp,
                  bias=pk["bqkv"])
    o = torch.empty_like(a)
    y = torch.empty_like(a)
    lse = torch.empty(B * N, device=dev, dtype=torch.float32)
    call("dfcsa_fra_fwd", dt(dtype), B, N, C, Cq, Jp, P(qkv), P(a), P(mod.gamma), P(o), P(y), P(lse), stream())
    return y, (a, qkv, o, lse)


def core_backward(mod, saved, dy, dtype, pk):
    """dy: gradient at the attention output; it is consumed (becomes the input gradient da, which
    includes the residual path).  Accumulates the q/k/v weight, bias and gamma gradients."""
    a, qkv, o, lse = saved
    B, H, W, C = a.shape
    _, Cq, J, Jp = widths(mod)
    M, N = B * H * W, H * W
    dev = a.device
    f32 = torch.float32
    T = dt(dtype)
    r = torch.empty(M, device=dev, dtype=f32)
    call("dfcsa_fra_bwd_prep", T, M, C, P(dy), P(o), P(r), stream())
    call("dfcsa_sum_to_scalar", P(r), M, P(_grad_of(mod.gamma)), stream())
    dqkv = torch.empty_like(qkv)
    if _lib.LIB.dfcsa_fra_path(T, C, Cq, Jp, 1) == 2:
        nb = ctypes.c_int64()
        call("dfcsa_fra_bwd_wide_bytes", B, N, C, Cq, ctypes.byref(nb))
        work = torch.empty(nb.value // 4, device=dev, dtype=f32)
        call("dfcsa_fra_bwd_wide", T, B, N, C, Cq, Jp, P(qkv), P(dy), P(mod.gamma), P(lse), P(r), P(dqkv),
             P(work), stream())
    else:
        call("dfcsa_fra_bwd", T, B, N, C, Cq, Jp, P(qkv), P(dy), P(mod.gamma), P(lse), P(r), P(dqkv), stream())
    grid, hw = (B, H, W), (H, W)
    ops.conv_wgrad_into(dtype, [dqkv], Jp, [(a, 0, 0)], C, grid, hw,
                        [_grad_of(mod.query_conv.weight), _grad_of(mod.key_conv.weight),
                         _grad_of(mod.value_conv.weight)], 1, Cq, C, layout=2)
    nt = ops.ntiles_ew(M, Jp)
    part = torch.empty(nt * Jp, device=dev, dtype=f32)
    call("dfcsa_channel_sum", T, M, Jp, P(dqkv), *S(part), stream())
    dbv = _grad_of(mod.value_conv.bias)
    tail = dbv if Jp == J else torch.zeros(Jp - 2 * Cq, device=dev, dtype=f32)
    call("dfcsa_slab_colsum3", P(part), nt, Jp, Cq, Cq, P(_grad_of(mod.query_conv.bias)),
         P(_grad_of(mod.key_conv.bias)), P(tail), stream())
    if tail is not dbv:
        call("dfcsa_cast_f32", _lib.DT_F32, C, P(tail), P(dbv), 1, stream())
    ops.conv_gemm(dtype, [(dqkv, 0, 0)], Jp, grid, hw, pk["WqkvT"], rup(Jp, ops.KALIGN), C, [dy], C, accumulate=True)
    return dy


class FRAFunction(torch.autograd.Function):
    """Standalone FullResolutionAttention on an NHWC tensor (no BatchNorm/ReLU in front)."""

    @staticmethod
    def forward(ctx, mod, dtype, x, *params):
        pk = get_packset(mod, ("fra", dtype, param_key(mod)), lambda ps: build_packs(ps, mod, dtype))
        y, saved = core_forward(mod, x, dtype, pk)
        ctx.mod, ctx.saved, ctx.dtype, ctx.pk, ctx.np = mod, saved, dtype, pk, len(params)
        return y

    @staticmethod
    def backward(ctx, g):
        da = core_backward(ctx.mod, ctx.saved, g.contiguous().clone(), ctx.dtype, ctx.pk)
        ctx.saved = None
        return (None, None, da, *([None] * ctx.np))
