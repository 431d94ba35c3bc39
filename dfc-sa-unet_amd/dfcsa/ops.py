"""Thin tensor-level wrappers over the libdfcsa C ABI.

Every wrapper enqueues on torch's current HIP stream and takes/returns torch tensors that live
on the GPU.  NHWC activations are torch tensors of shape [B, H, W, C] (dtype bf16 or fp32);
all statistics / parameters / gradients are fp32.  Nothing here computes on the host and
there is no fallback: a CPU tensor is rejected.
"""
import ctypes
import os

import torch

from . import _lib
from ._lib import call

KALIGN = 64          # Kpad granularity (64 bf16 / 32 f32 per K stage -> 64 serves both)
GEMM_MTILE = 64      # rows per conv_gemm stats tile (dfcsa_conv_gemm_mtile)


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def dt(dtype):
    if dtype == torch.bfloat16:
        return _lib.DT_BF16
    if dtype == torch.float32:
        return _lib.DT_F32
    raise TypeError(f"dfcsa supports bf16/fp32 activations, got {dtype}")


def S(t):
    """(device pointer, capacity in elements) of a slab tensor for the C ABI's `ptr, ptr_floats`
    argument pairs (None -> NULL, 0)."""
    return (None, 0) if t is None else (P(t), t.numel())


def P(t):
    """device pointer of a tensor (None -> NULL); rejects host tensors."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("dfcsa kernels need GPU tensors (MI355X/ROCm); got a CPU tensor")
    return t.data_ptr()


def rup(x, a):
    return (x + a - 1) // a * a


def ntiles_gemm(M):
    return (M + GEMM_MTILE - 1) // GEMM_MTILE


def ntiles_ew(M, C):
    return _lib.LIB.dfcsa_ew_ntiles(M, C)


# --------------------------------------------------------------------------- GEMMs
_SPLITK_MAX_M = 65536   # split-K applies to few-tile launches only (dfcsa_conv_work_floats decides)


# the train-mode BatchNorm finalisation folded into the producing conv's launch (dfcsa_conv_gemm_bn;
# the finalize is launched separately when the picked kernel cannot fold); DFCSA_BN_FOLD=0 disables
BN_FOLD = [os.environ.get("DFCSA_BN_FOLD", "1") == "1"]


def conv_gemm(dtype, segs, Cseg, grid, in_hw, weight, Kpad, N, dests, Nd, bias=None, stride=1,
              mode=0, accumulate=False, stats=None, out_hw=(0, 0), bn=None):
    """segs: list of (tensor, dh, dw); grid: (B, Ho, Wo) output pixel grid; in_hw: (Hi, Wi).
    With `stats` (>= ceil(M/64) rows of [2][N] fp32) returns the number of statistics rows the
    launch wrote (ntiles for bn_finalize; the 3x3 halo-tile kernel writes one per 2-D tile).
    bn = (bn_module, conv_bias, C): the train-mode BatchNorm of output columns [0, C) finalised by the
    launch itself (dfcsa_conv_gemm_bn); returns (rows, BNState) then."""
    B, Ho, Wo = grid
    d = _lib.ConvDesc()
    d.dtype = dt(dtype)
    d.M, d.N, d.Kpad, d.Cseg, d.nseg = B * Ho * Wo, N, Kpad, Cseg, len(segs)
    if len(segs) > _lib.MAX_SEG:
        raise ValueError("too many GEMM segments")
    for i, (t, dh, dw) in enumerate(segs):
        d.seg_ptr[i] = P(t)
        d.seg_dh[i] = dh
        d.seg_dw[i] = dw
    d.Ho, d.Wo = Ho, Wo
    d.Hi, d.Wi = in_hw
    d.stride = stride
    d.weight = P(weight)
    d.bias = P(bias)
    d.mode = mode
    d.ndest = len(dests)
    for i, t in enumerate(dests):
        d.dest[i] = P(t)
    d.Nd = Nd
    d.accumulate = int(bool(accumulate))
    d.stats = P(stats)
    d.stats_floats = stats.numel() if stats is not None else 0
    d.Hout, d.Wout = out_hw
    work = None
    if d.dtype == _lib.DT_BF16 and d.M <= _SPLITK_MAX_M:
        # split-K workspace of a few-tile, long-K launch (stream-ordered torch allocation, graph-safe)
        wf = _lib.LIB.dfcsa_conv_work_floats(ctypes.addressof(d))
        if wf > 0:
            work = torch.empty(wf, device=weight.device, dtype=torch.float32)
            d.work, d.work_floats = P(work), wf
    if bn is not None:
        bn_mod, conv_bias, C = bn
        f, st = bn_fold_desc(bn_mod, conv_bias, C, d.M)
        call("dfcsa_conv_gemm_bn", ctypes.addressof(d), ctypes.addressof(f), stream())
        return _lib.LIB.dfcsa_conv_stats_rows(ctypes.addressof(d)), st
    call("dfcsa_conv_gemm", ctypes.addressof(d), stream())
    if stats is not None:   # statistics rows written (the ntiles of bn_finalize)
        return _lib.LIB.dfcsa_conv_stats_rows(ctypes.addressof(d))
    return None


def bn_fold_desc(bn_mod, conv_bias, C, count):
    """(dfcsa_bn_fold, BNState): the train-mode BatchNorm of C channels over `count` values that a
    producing launch finalises in its tail (dfcsa_conv_gemm_bn, dfcsa_*_fwd_bn)."""
    st = BNState(C, bn_mod.weight.device)
    f = _lib.BnFold()
    f.C, f.count = C, count
    f.conv_bias, f.gamma, f.beta = P(conv_bias), P(bn_mod.weight), P(bn_mod.bias)
    f.running_mean, f.running_var = P(bn_mod.running_mean), P(bn_mod.running_var)
    f.num_batches_tracked = P(bn_mod.num_batches_tracked)
    f.momentum = float(bn_mod.momentum if bn_mod.momentum is not None else 0.1)
    f.eps = float(bn_mod.eps)
    f.scale, f.shift, f.mean, f.invstd = P(st.scale), P(st.shift), P(st.mean), P(st.invstd)
    return f, st


def bn_fold_ok(training):
    """whether a BatchNorm after a conv is finalised inside the conv's launch (conv_gemm(bn=...))"""
    return training and BN_FOLD[0] and _SYNC_BN is None and not _SKIP_FIN


def _wgrad_desc(dtype, gs, Cg, segs, Cseg, grid, in_hw, stride, layout=0):
    """The weight-gradient descriptor and its launch plan (dfcsa_wgrad_plan_desc: the 3x3 halo-tile
    kernel plans its own pixel splits)."""
    B, Ho, Wo = grid
    M = B * Ho * Wo
    NI, NJ = len(gs) * Cg, len(segs) * Cseg
    splits, mchunk, floats = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
    d = _lib.WgradDesc()
    d.dtype = dt(dtype)
    d.M, d.ng, d.Cg = M, len(gs), Cg
    for i, t in enumerate(gs):
        d.g_ptr[i] = P(t)
    d.nseg, d.Cseg = len(segs), Cseg
    for i, (t, dh, dw) in enumerate(segs):
        d.seg_ptr[i] = P(t)
        d.seg_dh[i] = dh
        d.seg_dw[i] = dw
    d.Ho, d.Wo = Ho, Wo
    d.Hi, d.Wi = in_hw
    d.stride = stride
    d.layout = layout
    call("dfcsa_wgrad_plan_desc", ctypes.addressof(d), ctypes.addressof(splits), ctypes.addressof(mchunk),
         ctypes.addressof(floats))
    d.splits, d.mchunk = splits.value, mchunk.value
    return d, floats.value, NI, NJ


def wgrad(dtype, gs, Cg, segs, Cseg, grid, in_hw, stride=1):
    """Split-K partials only: returns (slab, splits, NI, NJ) with slab [splits][NI][NJ] fp32 (the
    caller reduces with wgrad_reduce)."""
    d, floats, NI, NJ = _wgrad_desc(dtype, gs, Cg, segs, Cseg, grid, in_hw, stride, layout=-1)
    slab = torch.empty(floats, device=gs[0].device, dtype=torch.float32)
    d.slab = P(slab)
    d.slab_floats = slab.numel()
    d.ndst = 0
    call("dfcsa_conv_wgrad", ctypes.addressof(d), stream())
    return slab, d.splits, NI, NJ


def wgrad_reduce(slab, splits, NI, NJ, layout, ntaps, Ctot, Creal, dsts):
    arr = (ctypes.c_void_p * len(dsts))(*[P(t) for t in dsts])
    call("dfcsa_wgrad_reduce", P(slab), splits, NI, NJ, layout, ntaps, Ctot, Creal, len(dsts),
         ctypes.addressof(arr), stream())


def conv_wgrad_into(dtype, gs, Cg, segs, Cseg, grid, in_hw, grads, ntaps, Ctot, Creal, layout=0, stride=1,
                    bias_grads=None):
    """grads[d] += the weight gradient in the reference layout, in one dfcsa_conv_wgrad call (the
    split-K reduction runs inside the kernel, or as its second launch at high split counts).
    bias_grads (layout 2: three tensors): += the pixel sums of G, the stacked 1x1 biases' gradients."""
    d, floats, NI, NJ = _wgrad_desc(dtype, gs, Cg, segs, Cseg, grid, in_hw, stride, layout=layout)
    slab = torch.empty(floats, device=gs[0].device, dtype=torch.float32) if d.splits > 1 else None
    d.slab = P(slab)
    d.slab_floats = slab.numel() if slab is not None else 0
    d.layout, d.ntaps, d.Ctot, d.Creal, d.ndst = layout, ntaps, Ctot, Creal, len(grads)
    for i, t in enumerate(grads):
        d.dst[i] = P(t)
    if bias_grads is not None:
        for i, t in enumerate(bias_grads):
            d.bias_dst[i] = P(t)
    call("dfcsa_conv_wgrad", ctypes.addressof(d), stream())


def conv_wgrad_dgrad1x1(dtype, g, Cg, x, Cx, M, grads, ntaps, Ctot, Creal, wt, kpad, N, dx, layout=0,
                        bias_grads=None, pool=None):
    """conv_wgrad_into over G = g [M][Cg], X = x [M][Cx] (1x1, one row grid of M pixels) and, in the
    same launch where the small fp32 kernels apply, dx [M][N] = g * wt^T (the 1x1 conv's input
    gradient; wt [N][kpad] is its dfcsa_conv_gemm operand).  pool = (wsum, mean, invstd, rows, H, W,
    P): also the attention entry's pool-backward BatchNorm rows (dfcsa_conv_wgrad_dgrad1x1_pool)."""
    d, floats, NI, NJ = _wgrad_desc(dtype, [g], Cg, [(x, 0, 0)], Cx, (1, M, 1), (M, 1), 1, layout=layout)
    slab = torch.empty(floats, device=g.device, dtype=torch.float32) if d.splits > 1 else None
    d.slab = P(slab)
    d.slab_floats = slab.numel() if slab is not None else 0
    d.layout, d.ntaps, d.Ctot, d.Creal, d.ndst = layout, ntaps, Ctot, Creal, len(grads)
    for i, t in enumerate(grads):
        d.dst[i] = P(t)
    if bias_grads is not None:
        for i, t in enumerate(bias_grads):
            d.bias_dst[i] = P(t)
    if pool is None:
        call("dfcsa_conv_wgrad_dgrad1x1", ctypes.addressof(d), P(wt), kpad, N, P(dx), stream())
        return
    wsum, mean, invstd, rows, H, W, P_ = pool
    pc = _lib.PoolContract()
    pc.wsum, pc.mean, pc.invstd, pc.rows = P(wsum), P(mean), P(invstd), rows
    pc.H, pc.W, pc.P = H, W, P_
    call("dfcsa_conv_wgrad_dgrad1x1_pool", ctypes.addressof(d), P(wt), kpad, N, P(dx), ctypes.addressof(pc), stream())


# --------------------------------------------------------------------------- packing
def pack_conv_w(dtype, w, Cpad, Kpad, out=None, row0=0, rows=None):
    Cout, Cin = w.shape[0], w.shape[1]
    ntaps = w.shape[2] * w.shape[3] if w.dim() == 4 else 1
    if out is None:
        out = torch.empty((rows or Cout, Kpad), device=w.device, dtype=dtype)
    call("dfcsa_pack_conv_w", dt(dtype), P(w), Cout, Cin, ntaps, Cpad, Kpad, row0, P(out), stream())
    return out


def pack_conv_w_t(dtype, w, Kpad, out, col0):
    Cout, Cin = w.shape[0], w.shape[1]
    ntaps = w.shape[2] * w.shape[3] if w.dim() == 4 else 1
    call("dfcsa_pack_conv_w_t", dt(dtype), P(w), Cout, Cin, ntaps, Kpad, col0, P(out), stream())
    return out


def zeros(shape, dtype, device):
    return torch.zeros(shape, dtype=dtype, device=device)


# --------------------------------------------------------------------------- BatchNorm
class BNState:
    """Per-forward BatchNorm coefficients (fp32 [C] each)."""
    __slots__ = ("scale", "shift", "mean", "invstd")

    def __init__(self, C, device):
        buf = torch.empty(4, C, device=device, dtype=torch.float32)
        self.scale, self.shift, self.mean, self.invstd = buf[0], buf[1], buf[2], buf[3]


REDUCE_GROUPS = 256


def rows_reduce(src, T, rowlen):
    """First stage of a per-tile slab reduction: [T][rowlen] -> [G][rowlen] (G <= 256)."""
    if T <= REDUCE_GROUPS // 4:
        return src, T
    G = REDUCE_GROUPS
    dst = torch.empty(G * rowlen, device=src.device, dtype=torch.float32)
    call("dfcsa_rows_reduce", P(src), T, rowlen, P(dst), G, stream())
    return dst, G


# ---------------------------------------------------------------------------- SyncBN (opt-in)
# BatchNorm stays per-replica by default (standard DDP).  set_sync_bn(group)
# switches every BatchNorm of the MI355X path to SyncBatchNorm semantics over `group`: the forward
# statistics (sum x, sum x^2) and the backward sums (sum dz, sum dz*xhat) are all-reduced, so mean,
# variance, running statistics and the input gradient use the global batch; the BN weight/bias (and
# res_scale) gradients stay local sums, as in torch.nn.SyncBatchNorm (DDP then averages them).
# Shards must be equal-sized (the global count is world * local count).  One all-reduce of 2*C
# floats per BatchNorm forward and nsum*C per backward, on the current stream (graph-capturable
# with RCCL).
_SYNC_BN = None


def set_sync_bn(group=None, enabled=True):
    """Enable (group = a torch.distributed process group, None = WORLD) or disable SyncBN."""
    global _SYNC_BN
    if not enabled:
        _SYNC_BN = None
        return
    import torch.distributed as dist
    g = group if group is not None else dist.group.WORLD
    _SYNC_BN = (g, dist.get_world_size(g))


def sync_bn_enabled():
    return _SYNC_BN is not None


def _allreduce_(t):
    import torch.distributed as dist
    g = _SYNC_BN[0]
    if dist.get_backend(g) == "gloo":   # host-staged (CPU rehearsals / tests; synchronises)
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=g)
        t.copy_(h)
    else:                                # RCCL on the current stream
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=g)


# timing experiment only (results are garbage): DFCSA_SKIP_FINALIZE=1 launches no BatchNorm
# finalize kernel -- the upper bound of what folding them into their consumers could save
_SKIP_FIN = os.environ.get("DFCSA_SKIP_FINALIZE", "0") == "1"


def bn_finalize(bn_mod, conv_bias, stats, ntiles, C, ld, count, training):
    st = BNState(C, bn_mod.weight.device)
    if _SKIP_FIN and training:
        return st
    if training and _SYNC_BN is not None:
        # global column sums [2][ld] (fp64 inside the kernel, one fp32 total per column), summed
        # over the ranks, then finalised as a single row with the global count
        tot = torch.zeros(2 * ld, device=stats.device, dtype=torch.float32)
        call("dfcsa_slab_colsum", P(stats), ntiles, 2 * ld, P(tot), stream())
        _allreduce_(tot)
        stats, ntiles, count = tot, 1, count * _SYNC_BN[1]
    nbt = bn_mod.num_batches_tracked if training else None
    call("dfcsa_bn_finalize", P(stats) if training else None, ntiles, C, ld, count, P(conv_bias),
         P(bn_mod.weight), P(bn_mod.bias), P(bn_mod.running_mean), P(bn_mod.running_var), P(nbt),
         float(bn_mod.momentum if bn_mod.momentum is not None else 0.1), float(bn_mod.eps), int(training),
         P(st.scale), P(st.shift), P(st.mean), P(st.invstd), stream())
    return st


def bn_act(dtype, y, bn, act):
    """act(y * scale + shift): act 0 none, 1 relu, 2 sigmoid (NHWC, new tensor)."""
    out = torch.empty_like(y)
    C = y.shape[-1]
    call("dfcsa_bn_act", dt(dtype), y.numel() // C, C, P(y), P(bn.scale), P(bn.shift), int(act), P(out), stream())
    return out


def bn_bwd_finalize(partial, ntiles, nsum, C, count, dgamma, dbeta, extra=None):
    coef = torch.empty(3 * C, device=partial.device, dtype=torch.float32)
    if _SKIP_FIN:
        return coef
    if _SYNC_BN is not None:
        # local sums -> the parameter gradients (dgamma, dbeta, res_scale); global sums -> coef
        tot = torch.zeros(nsum * C, device=partial.device, dtype=torch.float32)
        call("dfcsa_slab_colsum", P(partial), ntiles, nsum * C, P(tot), stream())
        scratch = torch.empty(3 * C, device=partial.device, dtype=torch.float32)
        call("dfcsa_bn_bwd_finalize", P(tot), 1, nsum, C, count, P(scratch), P(dgamma), P(dbeta), P(extra),
             stream())
        _allreduce_(tot)
        call("dfcsa_bn_bwd_finalize", P(tot), 1, nsum, C, count * _SYNC_BN[1], P(coef), None, None, None,
             stream())
        return coef
    call("dfcsa_bn_bwd_finalize", P(partial), ntiles, nsum, C, count, P(coef), P(dgamma), P(dbeta), P(extra),
         stream())
    return coef


def bn_bwd_finalize_pool(partial, ntiles, C, count, dgamma, dbeta, dpooled, wsum, B, H, W, P_, bn):
    """bn_bwd_finalize (2 sums) of a DFC block's attention entry: `partial` holds the dattn part of
    the sums, the pool-backward part comes from the forward pool's window sums (dfcsa_bn_bwd_finalize_pool)."""
    coef = torch.empty(3 * C, device=partial.device, dtype=torch.float32)
    if _SKIP_FIN:
        return coef
    if _SYNC_BN is not None:
        raise NotImplementedError("the window-sum entry statistics are per replica (SyncBN uses the entry pass)")
    call("dfcsa_bn_bwd_finalize_pool", P(partial), ntiles, C, count, P(coef), P(dgamma), P(dbeta), P(dpooled),
         P(wsum), B, H, W, P_, P(bn.mean), P(bn.invstd), stream())
    return coef


# The gradient of a conv bias that feeds a train-mode BatchNorm is exactly zero:
#   sum_m dy_m = gamma*invstd*(sum_m dz_m - M*mean(dz) - mean(dz*xh)*sum_m xh_m) = 0  (sum xh = 0).
# The reference's autograd evaluates it in floating point (rounding noise ~1e-7 of the weight
# gradients); by default it is left at its exact value (no reduction pass).  Set
# DFCSA_NUMERIC_BN_BIAS_GRAD=1 to accumulate the floating-point column sums instead.
NUMERIC_BN_BIAS_GRAD = os.environ.get("DFCSA_NUMERIC_BN_BIAS_GRAD", "0") == "1"


def bn_bwd_apply(dtype, dz, y, bn, gamma, coef, bias_grad):
    M, C = dz.numel() // dz.shape[-1], dz.shape[-1]
    dy = torch.empty_like(dz)
    part = None
    if bias_grad is not None and NUMERIC_BN_BIAS_GRAD:
        nt = ntiles_ew(M, C)
        part = torch.empty(nt * C, device=dz.device, dtype=torch.float32)
    call("dfcsa_bn_bwd_apply", dt(dtype), M, C, P(dz), P(y), P(bn.mean), P(bn.invstd), P(gamma), P(coef), P(dy),
         *S(part), stream())
    if part is not None:
        colsum_into(part, nt, C, bias_grad)
    return dy


def bn_bwd_apply_relu(dtype, dact, y, bn, gamma, coef, bias_grad):
    """bn_bwd_apply with dz = relu'(bn y) * dact recomputed in the kernel (the producing
    dfcsa_bwd_relu_bn / dfcsa_bwd_block_out call then passes dz = None): no dz tensor."""
    M, C = dact.numel() // dact.shape[-1], dact.shape[-1]
    dy = torch.empty_like(dact)
    part = None
    if bias_grad is not None and NUMERIC_BN_BIAS_GRAD:
        nt = ntiles_ew(M, C)
        part = torch.empty(nt * C, device=dact.device, dtype=torch.float32)
    call("dfcsa_bn_bwd_apply_relu", dt(dtype), M, C, P(dact), P(y), P(bn.scale), P(bn.shift), P(bn.mean),
         P(bn.invstd), P(gamma), P(coef), P(dy), *S(part), stream())
    if part is not None:
        colsum_into(part, nt, C, bias_grad)
    return dy


def bn_bwd_apply_entry(dtype, dattn, dpooled, P_, y, bn, relu, gamma, coef, bias_grad):
    """bn_bwd_apply for the attention entry with dz = act'(bn y) * (dattn + pool backward of
    dpooled) recomputed in the kernel (dfcsa_bwd_attn_entry then passes dz = None)."""
    B, H, W, C = dattn.shape
    M = B * H * W
    dy = torch.empty_like(dattn)
    part = None
    if bias_grad is not None and NUMERIC_BN_BIAS_GRAD:
        nt = ntiles_ew(M, C)
        part = torch.empty(nt * C, device=dattn.device, dtype=torch.float32)
    # dpooled in bf16: the flash layers' projection dgrad output, read as it is
    fn = "dfcsa_bn_bwd_apply_entry16" if dpooled.dtype == torch.bfloat16 else "dfcsa_bn_bwd_apply_entry"
    call(fn, dt(dtype), B, H, W, C, P(dattn), P(dpooled), P_, P(y), P(bn.scale),
         P(bn.shift), P(bn.mean), P(bn.invstd), int(relu), P(gamma), P(coef), P(dy), *S(part), stream())
    if part is not None:
        colsum_into(part, nt, C, bias_grad)
    return dy


def colsum_into(slab, nt, C, out):
    """out[c] += sum_t slab[t][c]"""
    call("dfcsa_slab_colsum", P(slab), nt, C, P(out), stream())


def channel_sum_into(dtype, x, out):
    M, C = x.numel() // x.shape[-1], x.shape[-1]
    nt = ntiles_ew(M, C)
    part = torch.empty(nt * C, device=x.device, dtype=torch.float32)
    call("dfcsa_channel_sum", dt(dtype), M, C, P(x), *S(part), stream())
    colsum_into(part, nt, C, out)


def pack_t3(dtype, Cin, Kpad, segs, identity_last=False, out=None, device=None):
    """Transposed packing of up to three weights side by side (full rows, zero tail):
    segs = [w0, w1, w2] (None = absent); with identity_last the third segment is I (Cout=Cin)."""
    ws = list(segs) + [None] * (3 - len(segs))
    wcin = next(w.shape[1] for w in ws if w is not None)
    args = []
    for i, w in enumerate(ws):
        if w is None:
            cout = Cin if (i == 2 and identity_last) else 0
            args += [None, cout, 1]
        else:
            args += [P(w), w.shape[0], (w.shape[2] * w.shape[3]) if w.dim() == 4 else 1]
    if out is None:
        out = torch.empty((Cin, Kpad), dtype=dtype, device=device or ws[0].device)
    call("dfcsa_pack_t3", dt(dtype), Cin, Kpad, wcin, *args, int(identity_last), P(out), stream())
    return out
