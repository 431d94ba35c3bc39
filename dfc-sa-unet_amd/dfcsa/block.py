"""DynamicFusionConvAttnBlock forward and backward on the libdfcsa kernels.

Reference: models/unet_dfc_sa_res.py:41-116 (block) and :5-39 (LightSelfAttention).  The
backward is written out by hand (no autograd inside): every tensor the reference's autograd
graph would touch is produced by one of our kernels, parameter gradients are accumulated
straight into ``param.grad`` (fp32), and the block input gradient is one implicit GEMM that
fuses the 3x3 dgrad with both 1x1 dgrads (attention entry + residual).

FullResAttnDFCBlock (models/unet_dfc_sa_ablation_attention.py:29-92) runs the same flow with the
pooled LSA replaced by full-resolution attention on a = relu(bn2 y2) (dfcsa/fra.py).

Activation flow per block (NHWC, dtype T; M = B*H*W pixels; C = out channels):
  GEMM 3x3            x -> y1 (+bias, BN1 stats)
  GEMM 1x1 (N = 2C)   x -> [y2 (+bias, BN2 stats) | res]        (one launch)
  LSA                 pool(relu(bn2 y2)) -> q,k,v -> softmax -> o      (pooled P x P, fp32)
  EW                  local = relu(bn1 y1); attn = gamma*up(o) + relu(bn2 y2)
  GEMM 1x1            [local, attn] -> y3 (+bias, BN3 stats)   (no concat materialised)
  EW                  fused = s*local + (1-s)*attn, s = sigmoid(bn3 y3)
  GEMM 1x1            [fused, local, attn] -> y4 (+bias, BN4 stats)
  EW                  out = relu(bn4 y4) + res_scale * res
"""
import ctypes
import os

import torch
import torch.nn as nn

from . import _lib, fra, ops, streams
from ._lib import call
from .ddp import ARMED, notify_grads_ready
from .ops import P, S, dt, rup, stream
from .packs import get_packset, param_key
from .streams import join_branch, on_branch, on_side

# bf16 blocks with C % 64 == 0, C <= 256: the fusion conv's input-gradient GEMM carries the gate
# backward in its epilogue (dfcsa_dgrad_gate), the gate conv's accumulating one the BN1-backward
# sums (dfcsa_dgrad_acc_relu_bn); C == 64 (train mode): the fusion conv's forward GEMM computes the
# gate fusion in its A-operand prologue (dfcsa_gate_fusion_fwd).  DFCSA_DGRAD_GATE=0 selects the
# separate GEMM + elementwise launches everywhere
FUSED_DGRAD_GATE = [os.environ.get("DFCSA_DGRAD_GATE", "1") == "1"]
# encoder blocks: the 2x2 max-pool fused into the block-output pass and its backward (DFCSA_POOL_FUSION=0: separate)
POOL_FUSION = [os.environ.get("DFCSA_POOL_FUSION", "1") == "1"]
# C == 64: BatchNorm-backward applies in the dgrad GEMMs' A prologue (DFCSA_APPLY_PROLOGUE=<dy4><dy3> flags, "00": separate)
# [dy4 into the fusion-conv dgrad, dy3 into the gate-conv dgrad]: per-launch traces put the first at
# 205 us against 131 + 55 us for the separate pair (the longer prologue between the DMA wait and the
# MFMAs) and the second at 137 against 103 + ~50 us, so only the second is on by default
APPLY_PROLOGUE = [os.environ.get("DFCSA_APPLY_PROLOGUE", "01")[:1] == "1",
                  os.environ.get("DFCSA_APPLY_PROLOGUE", "01")[-1:] == "1"]
# bf16 blocks with C <= 128: the fusion conv's and the gate conv's weight gradients as one GEMM over
# [fused | local | attn] (wgrad layout 3; DFCSA_PAIR_WGRAD=0: two launches)
PAIR_WGRAD = [os.environ.get("DFCSA_PAIR_WGRAD", "1") == "1"]
# P <= 4: the pooled-attention backward (upsample column pass + softmax attention) in one
# token-parallel launch with last-arriver dk / dv (DFCSA_LSA_CORE_BWD=1).  Off: measured slower
# than the three launches (1416 / 1420 vs 1433 / 1435 img/s; a one-workgroup-per-image version
# 1409 vs 1434): the last arriver's write-through hand-off costs more than the launches it saves
# (profiles/r03b_ab_lsa_core_bwd.jsonl)
LSA_CORE_BWD = [os.environ.get("DFCSA_LSA_CORE_BWD", "0") == "1"]
# backward: DFCSA_DX_FIRST=1 issues the block input-gradient GEMM before the input-side weight
# gradients on the side stream (default: after them).  Same-box A/B, 150 steps x 3: 1526 / 1528 /
# 1526 img/s first against 1550 / 1540 / 1547 after -- the weight gradients started early overlap the
# latency-bound stretches that follow better than they hurt the dgrad they start beside
DX_FIRST = [os.environ.get("DFCSA_DX_FIRST", "0") == "1"]
# block widths whose gate conv takes the local/attention prologue (DFCSA_LOCAL_ATTN_WIDTHS=64,128)
LOCAL_ATTN_WIDTHS = tuple(int(c) for c in os.environ.get("DFCSA_LOCAL_ATTN_WIDTHS", "64,128").split(",") if c)
# block widths whose fusion conv takes the gate-fusion prologue (DFCSA_GATE_FUSION_WIDTHS=64,128)
GATE_FUSION_WIDTHS = tuple(int(c) for c in os.environ.get("DFCSA_GATE_FUSION_WIDTHS", "64,128").split(",") if c)


def grad_of(p):
    """fp32 gradient buffer of a parameter (created zeroed if absent)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


def raise_eval_backward():
    """The backward kernels implement train-mode BatchNorm (batch statistics: dz is centred by
    mean(dz) and mean(dz*xh), the pre-BN conv bias gets its exact-zero gradient).  An eval-mode
    forward (running statistics) would need the per-channel affine backward instead, so it is
    refused rather than answered with wrong gradients."""
    raise NotImplementedError("backward through an eval-mode (running-statistics) BatchNorm forward is not "
                              "implemented by the dfcsa kernels; run the forward in train mode or under "
                              "torch.no_grad()")


def _conv3x3_segments(xs):
    return [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3) for x in xs]


class _Saved:
    pass


def block_forward(blk, xs, pool_size, training, dtype, pool=False):
    """Returns (out, saved), or with pool=True ((pooled, out), saved): the encoder's 2x2 max-pool
    of the block output (reference :165-172) fused into the block-output pass when H, W are even."""
    B, H, W, Cs = xs[0].shape
    nsrc = len(xs)
    Cin_p = nsrc * Cs
    conv1, bn1m = blk.conv_branch[0], blk.conv_branch[1]
    conv2, bn2m = blk.attn_branch[0], blk.attn_branch[1]
    lsa = blk.attn_branch[3]
    conv3, bn3m = blk.gate[0], blk.gate[1]
    conv4, bn4m = blk.fusion_conv[0], blk.fusion_conv[1]
    has_res = not isinstance(blk.residual_conv, nn.Identity)
    C = conv1.out_channels
    Cin_real = conv1.in_channels
    if Cin_real > Cin_p:
        raise ValueError(f"block expects {Cin_real} input channels, got {Cin_p}")
    if not has_res and (nsrc != 1 or Cs != C):
        raise ValueError("identity residual needs a single source with out_channels channels")
    M = B * H * W
    dev = xs[0].device
    nt = ops.ntiles_gemm(M)
    s = _Saved()

    # ---- weights -> persistent GEMM operands (one pack-plan launch per forward) ----
    N2 = 2 * C if has_res else C
    Kp1, Kp2 = rup(9 * Cin_p, ops.KALIGN), rup(Cin_p, ops.KALIGN)
    Kp3, Kp4 = rup(2 * C, ops.KALIGN), rup(3 * C, ops.KALIGN)
    pk = get_packset(blk, (dtype, nsrc, Cs, LSA_FLASH_MIN_N[0], param_key(blk)),
                     lambda ps: _build_block_packs(ps, blk, dtype, Cin_p, C, has_res))
    W1p, W2p, W3p, W4p = pk["W1p"], pk["W2p"], pk["W3p"], pk["W4p"]
    b2 = pk["b2"] if has_res else conv2.bias

    def stats(n):
        return torch.empty(nt * 2 * n, device=dev, dtype=torch.float32) if training else None

    # ---- attention entry / residual 1x1 conv, then the local branch 3x3 conv ----
    Cq = lsa.query_conv.out_channels
    fullres = getattr(lsa, "full_resolution", False)
    # the pooled attention chain (bn2 statistics -> pool -> q/k/v -> softmax core) runs on the branch
    # stream beside the 3x3 conv (streams.on_branch); on maps of >= ENTRY_ON_BRANCH_HW pixels the
    # attention entry / residual 1x1 conv runs there too (at small maps the chain's fixed launch
    # latencies already outlast the 3x3 conv)
    branch = not fullres and ops._SYNC_BN is None
    entry_on_branch = H * W >= ENTRY_ON_BRANCH_HW[0]

    fold = ops.bn_fold_ok(training)   # BatchNorm finalisations inside the producing conv launches

    def entry_conv():
        y2_ = torch.empty((B, H, W, C), dtype=dtype, device=dev)
        res_ = torch.empty((B, H, W, C), dtype=dtype, device=dev) if has_res else xs[0]
        st2_ = stats(N2)
        r = ops.conv_gemm(dtype, [(x, 0, 0) for x in xs], Cs, (B, H, W), (H, W), W2p, Kp2, N2,
                          [y2_, res_] if has_res else [y2_], C, bias=b2, stats=st2_,
                          bn=(bn2m, conv2.bias, C) if fold else None)
        return y2_, res_, st2_, r

    if not entry_on_branch:
        y2, res, st2, nt2 = entry_conv()
    with on_branch(dev, branch, *xs):
        if entry_on_branch:
            y2, res, st2, nt2 = entry_conv()
        if fold:
            nt2, bn2 = nt2
        else:
            bn2 = ops.bn_finalize(bn2m, conv2.bias, st2, nt2 if training else nt, C, N2, M, training)
        if not fullres:
            Pp = pool_size
            lsa_saved = lsa_core_forward(lsa, y2, bn2.scale, bn2.shift, True, Pp, dtype, pk,
                                         window_sums=training and ENTRY_WS[0] and ops._SYNC_BN is None)
    y1 = torch.empty((B, H, W, C), dtype=dtype, device=dev)
    st1 = stats(C)
    nt1 = ops.conv_gemm(dtype, _conv3x3_segments(xs), Cs, (B, H, W), (H, W), W1p, Kp1, C, [y1], C,
                        bias=conv1.bias, stats=st1,   # (3x3 halo tiles: one statistics row per 2-D tile)
                        bn=(bn1m, conv1.bias, C) if fold else None)
    if fold:
        nt1, bn1 = nt1
    else:
        bn1 = ops.bn_finalize(bn1m, conv1.bias, st1, nt1 if training else nt, C, C, M, training)
    join_branch(dev, branch, bn2, None if fullres else lsa_saved, y2, res if has_res else None)

    if fullres:
        # ---- FullResolutionAttention (unet_dfc_sa_ablation_attention.py:42-47, :71-75) on the
        #      unpooled map a = relu(bn2 y2): flash-style kernels, no N x N tensor ----
        Pp, J, N = 0, 2 * Cq + C, H * W
        local = ops.bn_act(dtype, y1, bn1, 1)
        a = ops.bn_act(dtype, y2, bn2, 1)
        attn, s.fra = fra.core_forward(lsa, a, dtype, pk)
        pooled = qkv = A = o = Wqkv = None
    else:
        # ---- LightSelfAttention on the pooled map ----
        s.fra = None
        J, N = 2 * Cq + C, Pp * Pp
        pooled, qkv, A, o, Wqkv = lsa_saved[:5]
        s.wsum = lsa_saved[5] if len(lsa_saved) > 5 else None
        local = torch.empty((B, H, W, C), dtype=dtype, device=dev)
        attn = torch.empty((B, H, W, C), dtype=dtype, device=dev)
    y3 = torch.empty((B, H, W, C), dtype=dtype, device=dev)
    st3 = stats(C)
    nt3 = nt
    if not fullres and dtype == torch.bfloat16 and C in LOCAL_ATTN_WIDTHS and Kp3 == 2 * C and training and \
            FUSED_DGRAD_GATE[0]:
        # the local/attention merge runs in the gate conv's A-operand prologue (one statistics row
        # per workgroup)
        nt3 = _lib.LIB.dfcsa_fwd_pro_parts(M, C, 1)
        args3 = (B, H, W, C, P(y1), P(bn1.scale), P(bn1.shift), P(y2), P(bn2.scale), P(bn2.shift), P(o), Pp,
                 P(lsa.gamma), P(W3p), Kp3, P(conv3.bias), P(local), P(attn), P(y3), *S(st3))
        if fold:   # BN3 finalised in the launch's tail
            f3, bn3f = ops.bn_fold_desc(bn3m, conv3.bias, C, M)
            call("dfcsa_local_attn_gate_fwd_bn", *args3, ctypes.addressof(f3), stream())
            nt3 = (nt3, bn3f)
        else:
            call("dfcsa_local_attn_gate_fwd", *args3, stream())
    else:
        if not fullres:
            call("dfcsa_block_local_attn", dt(dtype), B, H, W, C, P(y1), P(bn1.scale), P(bn1.shift), P(y2),
                 P(bn2.scale), P(bn2.shift), P(o), Pp, P(lsa.gamma), 1, P(local), P(attn), stream())
        # ---- gate conv ----
        nt3 = ops.conv_gemm(dtype, [(local, 0, 0), (attn, 0, 0)], C, (B, H, W), (H, W), W3p, Kp3, C, [y3], C,
                            bias=conv3.bias, stats=st3, bn=(bn3m, conv3.bias, C) if fold else None) or nt
    if isinstance(nt3, tuple):
        nt3, bn3 = nt3
    else:
        bn3 = ops.bn_finalize(bn3m, conv3.bias, st3, nt3, C, C, M, training)
    fused = torch.empty((B, H, W, C), dtype=dtype, device=dev)
    y4 = torch.empty((B, H, W, C), dtype=dtype, device=dev)
    st4 = stats(C)
    nt4 = nt
    if dtype == torch.bfloat16 and C in GATE_FUSION_WIDTHS and Kp4 == 3 * C and training and FUSED_DGRAD_GATE[0]:
        # the gate fusion runs in the fusion conv's A-operand prologue (dfcsa_gate_fusion_fwd; one
        # statistics row per workgroup)
        nt4 = _lib.LIB.dfcsa_fwd_pro_parts(M, C, 0)
        args4 = (M, C, P(y3), P(bn3.scale), P(bn3.shift), P(local), P(attn), P(W4p), Kp4, P(conv4.bias), P(fused),
                 P(y4), *S(st4))
        if fold:   # BN4 finalised in the launch's tail
            f4, bn4f = ops.bn_fold_desc(bn4m, conv4.bias, C, M)
            call("dfcsa_gate_fusion_fwd_bn", *args4, ctypes.addressof(f4), stream())
            nt4 = (nt4, bn4f)
        else:
            call("dfcsa_gate_fusion_fwd", *args4, stream())
    else:
        call("dfcsa_gate_fuse", dt(dtype), M, C, P(y3), P(bn3.scale), P(bn3.shift), P(local), P(attn), P(fused),
             stream())
        nt4 = ops.conv_gemm(dtype, [(fused, 0, 0), (local, 0, 0), (attn, 0, 0)], C, (B, H, W), (H, W), W4p, Kp4, C,
                            [y4], C, bias=conv4.bias, stats=st4, bn=(bn4m, conv4.bias, C) if fold else None) or nt
    if isinstance(nt4, tuple):
        nt4, bn4 = nt4
    else:
        bn4 = ops.bn_finalize(bn4m, conv4.bias, st4, nt4, C, C, M, training)
    out = torch.empty((B, H, W, C), dtype=dtype, device=dev)
    pooled_out = None
    if pool:
        pooled_out = torch.empty((B, H // 2, W // 2, C), dtype=dtype, device=dev)
    if pool and H % 2 == 0 and W % 2 == 0 and POOL_FUSION[0]:
        call("dfcsa_block_out_pool", dt(dtype), B, H, W, C, P(y4), P(bn4.scale), P(bn4.shift), P(res),
             P(blk.res_scale), P(out), P(pooled_out), stream())
    else:
        call("dfcsa_block_out", dt(dtype), M, C, P(y4), P(bn4.scale), P(bn4.shift), P(res), P(blk.res_scale),
             P(out), stream())
        if pool:
            call("dfcsa_maxpool2_fwd", dt(dtype), B, H, W, C, P(out), P(pooled_out), stream())

    s.shape = (B, H, W, C, Cs, nsrc, Cin_p, Cin_real, has_res, Pp, Cq, J, N)
    s.xs = xs
    s.y1, s.y2, s.res, s.local, s.attn, s.y3, s.fused, s.y4 = y1, y2, res, local, attn, y3, fused, y4
    s.bn = (bn1, bn2, bn3, bn4)
    s.pooled, s.qkv, s.A, s.o, s.Wqkv = pooled, qkv, A, o, Wqkv
    s.pk = pk
    if pool:
        s.out = out   # the max-pool's argmax source in backward
        return (pooled_out, out), s
    return out, s


def _build_block_packs(ps, blk, dtype, Cin_p, C, has_res):
    """Entries of one DFC block.  Phase A: forward operands from the fp32 weights; phase B:
    the dgrad operands as transposes of those (W4t = W4p^T, W3t = W3p^T, and the fused block-input
    dgrad operand Wdx = [W1p(tap)^T for 9 taps | W2p^T | Wres^T or I])."""
    conv1, conv2, conv3, conv4 = blk.conv_branch[0], blk.attn_branch[0], blk.gate[0], blk.fusion_conv[0]
    N2 = 2 * C if has_res else C
    Kp2 = rup(Cin_p, ops.KALIGN)
    W1p = ps.rows("W1p", dtype, conv1.weight, Cin_p, rup(9 * Cin_p, ops.KALIGN))
    W2p = ps.rows("W2p", dtype, conv2.weight, Cin_p, Kp2, row0=0, rows=N2)
    if has_res:
        ps.rows("W2p", dtype, blk.residual_conv.weight, Cin_p, Kp2, row0=C)
        ps.concat("b2", [conv2.bias], N2)
    W3p = ps.rows("W3p", dtype, conv3.weight, 2 * C, rup(2 * C, ops.KALIGN))
    W4p = ps.rows("W4p", dtype, conv4.weight, 3 * C, rup(3 * C, ops.KALIGN))
    KpC = rup(C, ops.KALIGN)
    ps.transpose(W4p, 0, 0, C, 3 * C, "W4t", (3 * C, KpC))
    ps.transpose(W3p, 0, 0, C, 2 * C, "W3t", (2 * C, KpC))
    att = blk.attn_branch[3]
    if not getattr(att, "full_resolution", False) and SPLIT_DX[0]:
        # the block-input gradient in two GEMMs (block_backward): WdxA = [W1p(tap)^T for 9 taps | Wres^T
        # or I] before the attention chain's dy2 arrives, WdxB = W2p^T accumulated after it
        wa, wb = (Cin_p, rup(10 * C, ops.KALIGN)), (Cin_p, rup(C, ops.KALIGN))
        for tap in range(9):
            ps.transpose(W1p, 0, tap * Cin_p, C, Cin_p, "WdxA", wa, dc0=tap * C)
        if has_res:
            ps.transpose(W2p, C, 0, C, Cin_p, "WdxA", wa, dc0=9 * C)
        else:  # identity residual: constant identity block (written once)
            ps.buffer("WdxA", wa, dtype)[:, 9 * C:10 * C].copy_(torch.eye(C, dtype=dtype, device=ps.device))
        ps.transpose(W2p, 0, 0, C, Cin_p, "WdxB", wb)
    else:
        wdx = (Cin_p, rup(11 * C, ops.KALIGN))
        for tap in range(9):
            ps.transpose(W1p, 0, tap * Cin_p, C, Cin_p, "Wdx", wdx, dc0=tap * C)
        ps.transpose(W2p, 0, 0, C, Cin_p, "Wdx", wdx, dc0=9 * C)
        if has_res:
            ps.transpose(W2p, C, 0, C, Cin_p, "Wdx", wdx, dc0=10 * C)
        else:  # identity residual: constant identity block (written once)
            ps.buffer("Wdx", wdx, dtype)[:, 10 * C:11 * C].copy_(torch.eye(C, dtype=dtype, device=ps.device))
    if getattr(att, "full_resolution", False):
        fra.build_packs(ps, att, dtype)
    else:
        _build_lsa_packs(ps, att, dtype, blk.pool_size)


def _build_lsa_packs(ps, lsa, dtype=None, pool_size=None):
    f32 = torch.float32
    C = lsa.value_conv.out_channels
    Cq = lsa.query_conv.out_channels
    J = 2 * Cq + C
    qw, kw, vw = lsa.query_conv.weight, lsa.key_conv.weight, lsa.value_conv.weight
    ps.concat("bqkv", [lsa.query_conv.bias, lsa.key_conv.bias, lsa.value_conv.bias], J)
    if _lsa_gemm_ok(C, J):
        Kp = rup(C, ops.KALIGN)
        for w, off in ((qw, 0), (kw, Cq), (vw, 2 * Cq)):
            Wp = ps.rows("Wp", f32, w, C, Kp, row0=off, rows=J)
        ps.transpose(Wp, 0, 0, J, C, "WT", (C, rup(J, ops.KALIGN)))
        if pool_size is not None and flash16_layer(dtype, C, Cq, pool_size):
            # the bf16 projection operands of a flash layer (forward rows, dgrad transposes)
            for w, off in ((qw, 0), (kw, Cq), (vw, 2 * Cq)):
                Wp16 = ps.rows("Wp16", torch.bfloat16, w, C, Kp, row0=off, rows=J)
            ps.transpose(Wp16, 0, 0, J, C, "WT16", (C, rup(J, ops.KALIGN)))
    else:
        for w, off in ((qw, 0), (kw, Cq), (vw, 2 * Cq)):
            Wq = ps.rows("Wqkv", f32, w, C, C, row0=off, rows=J)
        ps.transpose(Wq, 0, 0, J, C, "WqkvT", (C, J))


def block_backward(blk, s, dout, need_dx, dtype, pool_grads=None):
    """pool_grads = (dpooled, dskip) for a block run with pool=True (dout unused): the block-output
    gradient is dskip + the max-pool backward of dpooled, formed in the block-output backward pass."""
    B, H, W, C, Cs, nsrc, Cin_p, Cin_real, has_res, Pp, Cq, J, N = s.shape
    conv1, bn1m = blk.conv_branch[0], blk.conv_branch[1]
    conv2, bn2m = blk.attn_branch[0], blk.attn_branch[1]
    lsa = blk.attn_branch[3]
    conv3, bn3m = blk.gate[0], blk.gate[1]
    conv4, bn4m = blk.fusion_conv[0], blk.fusion_conv[1]
    bn1, bn2, bn3, bn4 = s.bn
    M = B * H * W
    dev = s.y4.device
    T = dt(dtype)
    grid, hw = (B, H, W), (H, W)
    nte = ops.ntiles_ew(M, C)
    f32 = torch.float32
    nbo = nte
    dres = torch.empty_like(s.y4)
    if pool_grads is not None:
        dpool, dskip = pool_grads
        dskip = dskip.contiguous() if dskip is not None else None
        if dpool is not None and H % 2 == 0 and W % 2 == 0 and POOL_FUSION[0]:
            # ---- max-pool backward + block output backward in one pass ----
            dout = torch.empty_like(s.y4)
            nbo = _lib.LIB.dfcsa_bwd_block_out_pool_ntiles(B, H, W, C)
            part = torch.empty(nbo * 3 * C, device=dev, dtype=f32)
            call("dfcsa_bwd_block_out_pool", T, B, H, W, C, P(dskip), P(s.out), P(dpool.contiguous()), P(s.y4),
                 P(bn4.scale), P(bn4.shift), P(bn4.mean), P(bn4.invstd), P(s.res), P(blk.res_scale), P(dout),
                 P(dres), *S(part), stream())
        else:
            dout = dskip if dskip is not None else torch.zeros_like(s.y4)
            if dpool is not None:
                call("dfcsa_maxpool2_bwd", T, B, H, W, C, P(s.out), P(dpool.contiguous()), P(dout), stream())
            dpool = None
    else:
        dpool = None
        dout = dout.contiguous()
    if dpool is None:
        # ---- block output: relu(bn4 y4) + res_scale * res ----
        # (dz4 = relu'(bn4 y4) * dout is not materialised: the apply recomputes it)
        part = torch.empty(nte * 3 * C, device=dev, dtype=f32)
        call("dfcsa_bwd_block_out", T, M, C, P(dout), P(s.y4), P(bn4.scale), P(bn4.shift), P(bn4.mean),
             P(bn4.invstd), P(s.res), P(blk.res_scale), None, P(dres), *S(part), stream())
    coef = ops.bn_bwd_finalize(part, nbo, 3, C, M, grad_of(bn4m.weight), grad_of(bn4m.bias),
                               extra=grad_of(blk.res_scale))
    KpC = rup(C, ops.KALIGN)
    W4t = s.pk["W4t"]
    dlocal = torch.empty_like(s.y4)
    dattn = torch.empty_like(s.y4)
    dz3 = torch.empty_like(s.y3)
    fused = dtype == torch.bfloat16 and C % 64 == 0 and C <= 256 and FUSED_DGRAD_GATE[0]
    # C == 64: the BatchNorm-backward applies (dy4, dy3) run in the A-operand prologue of the fused
    # input-gradient GEMMs below (the conv-bias gradient is the analytic zero there)
    apro_ok = fused and C == 64 and not ops.NUMERIC_BN_BIAS_GRAD
    apro = apro_ok and APPLY_PROLOGUE[0]           # dy4 in the fusion-conv dgrad (measured slower: off)
    apro3 = apro_ok and APPLY_PROLOGUE[1]          # dy3 in the gate-conv dgrad
    # ---- gate: s = sigmoid(bn3 y3); fused = s*local + (1-s)*attn ----
    if apro:
        # dy4 in the prologue, the gate backward in the epilogue of the fusion conv's dgrad GEMM
        dy4 = torch.empty_like(dout)
        npart = _lib.LIB.dfcsa_dgrad_apply_parts(M, 0)
        part = torch.empty(npart * 2 * C, device=dev, dtype=f32)
        call("dfcsa_dgrad_gate_apply", M, P(dout), P(s.y4), P(bn4m.weight), P(coef), P(bn4.mean), P(bn4.invstd),
             P(bn4.scale), P(bn4.shift), P(dy4), P(W4t), P(s.y3), P(bn3.scale), P(bn3.shift), P(bn3.mean),
             P(bn3.invstd), P(s.local), P(s.attn), P(dlocal), P(dattn), P(dz3), *S(part), stream())
    else:
        dy4 = ops.bn_bwd_apply_relu(dtype, dout, s.y4, bn4, bn4m.weight, coef, grad_of(conv4.bias))
    # fusion conv: dW4 (side stream) and d[fused, local, attn].  C <= 128 (HBM-bound 1x1 weight
    # gradients at 224^2 / 112^2): dW4 waits for dy3 and runs as ONE GEMM with the gate conv's dW3
    # (G = [dy4 | dy3] over [fused | local | attn], layout 3): local and attn are read once
    pair_wgrad = dtype == torch.bfloat16 and C <= 128 and PAIR_WGRAD[0]
    dy4_keep = dy4 if pair_wgrad else None
    if not pair_wgrad:
        with on_side(dev, dy4, s.fused, s.local, s.attn):
            ops.conv_wgrad_into(dtype, [dy4], C, [(s.fused, 0, 0), (s.local, 0, 0), (s.attn, 0, 0)], C, grid, hw,
                                [grad_of(conv4.weight)], 1, 3 * C, 3 * C)
    if apro:
        del dy4
    elif fused:
        # the gate backward runs in the epilogue of the fusion conv's input-gradient GEMM
        # (dfused never stored; dfcsa_dgrad_gate)
        npart = _lib.LIB.dfcsa_dgrad_gate_parts(M, C)
        part = torch.empty(npart * 2 * C, device=dev, dtype=f32)
        call("dfcsa_dgrad_gate", M, C, P(dy4), P(W4t), KpC, P(s.y3), P(bn3.scale), P(bn3.shift), P(bn3.mean),
             P(bn3.invstd), P(s.local), P(s.attn), P(dlocal), P(dattn), P(dz3), *S(part), stream())
        del dy4
    else:
        npart = nte
        dfused = torch.empty_like(s.y4)
        ops.conv_gemm(dtype, [(dy4, 0, 0)], C, grid, hw, W4t, KpC, 3 * C, [dfused, dlocal, dattn], C)
        del dy4
        part = torch.empty(nte * 2 * C, device=dev, dtype=f32)
        call("dfcsa_bwd_gate", T, M, C, P(dfused), P(s.y3), P(bn3.scale), P(bn3.shift), P(bn3.mean),
             P(bn3.invstd), P(s.local), P(s.attn), P(dlocal), P(dattn), P(dz3), *S(part), stream())
        del dfused
    coef = ops.bn_bwd_finalize(part, npart, 2, C, M, grad_of(bn3m.weight), grad_of(bn3m.bias))
    W3t = s.pk["W3t"]
    fused_bn1 = fused
    if apro3:
        # dy3 in the prologue, the accumulate + BN1 sums in the epilogue of the gate conv's dgrad GEMM
        dy3 = torch.empty_like(dz3)
        npart1 = _lib.LIB.dfcsa_dgrad_apply_parts(M, 1)
        part1 = torch.empty(npart1 * 2 * C, device=dev, dtype=f32)
        call("dfcsa_dgrad_acc_relu_bn_apply", M, P(dz3), P(s.y3), P(bn3m.weight), P(coef), P(bn3.mean),
             P(bn3.invstd), P(dy3), P(W3t), P(s.y1), P(bn1.scale), P(bn1.shift), P(bn1.mean), P(bn1.invstd),
             P(dlocal), P(dattn), *S(part1), stream())
        del dz3
    else:
        dy3 = ops.bn_bwd_apply(dtype, dz3, s.y3, bn3, bn3m.weight, coef, grad_of(conv3.bias))
        del dz3
    if pair_wgrad:
        def gate_wgrads(dy4k=dy4_keep, dy3k=dy3, fused_=s.fused, local_=s.local, attn_=s.attn):
            with on_side(dev, dy4k, dy3k, fused_, local_, attn_):
                ops.conv_wgrad_into(dtype, [dy4k, dy3k], C, [(fused_, 0, 0), (local_, 0, 0), (attn_, 0, 0)], C,
                                    grid, hw, [grad_of(conv4.weight), grad_of(conv3.weight)], 1, C, 3 * C, layout=3)
        del dy4_keep
    else:
        def gate_wgrads(dy3k=dy3, local_=s.local, attn_=s.attn):
            with on_side(dev, dy3k):
                ops.conv_wgrad_into(dtype, [dy3k], C, [(local_, 0, 0), (attn_, 0, 0)], C, grid, hw,
                                    [grad_of(conv3.weight)], 1, 2 * C, 2 * C)
    if not WGRAD_LATE[0] or (not need_dx and LAST_EARLY[0] >= 2):
        gate_wgrads()
        gate_wgrads = None
    if apro3:
        pass
    elif fused_bn1:
        # accumulate GEMM with the local branch's BN1-backward sums in its epilogue
        npart1 = _lib.LIB.dfcsa_dgrad_acc_relu_bn_parts(M, C)
        part1 = torch.empty(npart1 * 2 * C, device=dev, dtype=f32)
        call("dfcsa_dgrad_acc_relu_bn", M, C, P(dy3), P(W3t), KpC, P(s.y1), P(bn1.scale), P(bn1.shift), P(bn1.mean),
             P(bn1.invstd), P(dlocal), P(dattn), *S(part1), stream())
    else:
        ops.conv_gemm(dtype, [(dy3, 0, 0)], C, grid, hw, W3t, KpC, 2 * C, [dlocal, dattn], C, accumulate=True)
    del dy3

    # the attention chain (LightSelfAttention backward -> attention entry -> bn2 backward) runs
    # on the branch stream beside the local branch's bn1 backward (streams.on_branch)
    branch = s.fra is None and ops._SYNC_BN is None
    wsum = getattr(s, "wsum", None)
    local_part = None
    if s.fra is None and wsum is not None:
        # the attention chain's statistics without a pass after it: the dattn part of the entry's
        # BN2-backward sums on this stream, beside the attention backward on the branch; the
        # pool part is a [B][N][C] contraction with the forward pool's window sums, inside the
        # finalize (dfcsa_bn_bwd_finalize_pool)
        # the pool part as extra partial rows written by the projection backward (B*P*P <= 4096: the
        # one-launch small kernel) or after the bf16 projection backward of a flash layer
        # (dfcsa_lsa_pool_rows), else by the finalize (dfcsa_bn_bwd_finalize_pool)
        Np = Pp * Pp
        flash16 = isinstance(s.A, FlashSaved) and s.A.qkv16 is not None
        rows_in_proj = _lsa_gemm_ok(C, 2 * lsa.query_conv.out_channels + C) and (B * Np <= 4096 or flash16)
        ncr = (B * Np + 15) // 16 if rows_in_proj else 0
        part2 = torch.empty((nte + ncr) * 2 * C, device=dev, dtype=f32)
        pool_rows = (wsum, bn2.mean, bn2.invstd, P(part2) + nte * 2 * C * 4, H, W) if rows_in_proj else None
        with on_branch(dev, branch, dattn, part2, wsum):
            dpooled = lsa_core_backward(lsa, (s.pooled, s.qkv, s.A, s.o, s.Wqkv), dattn, Pp, dtype, s.pk,
                                        pool_rows=pool_rows)
    if s.fra is None and wsum is not None:
        if fused_bn1:
            call("dfcsa_bwd_relu_bn", T, M, C, P(dattn), P(s.y2), P(bn2.scale), P(bn2.shift), P(bn2.mean),
                 P(bn2.invstd), None, *S(part2), stream())
        else:   # with the local branch's BN1-backward sums in the same launch
            local_part = torch.empty(nte * 2 * C, device=dev, dtype=f32)
            call("dfcsa_bwd_relu_bn_pair", T, M, C, P(dattn), P(s.y2), P(bn2.scale), P(bn2.shift), P(bn2.mean),
                 P(bn2.invstd), P(part2), P(dlocal), P(s.y1), P(bn1.scale), P(bn1.shift), P(bn1.mean),
                 P(bn1.invstd), P(local_part), part2.numel(), stream())
        with on_branch(dev, branch, part2, dattn, wsum):
            if rows_in_proj:
                coef2 = ops.bn_bwd_finalize(part2, nte + ncr, 2, C, M, grad_of(bn2m.weight), grad_of(bn2m.bias))
            else:
                coef2 = ops.bn_bwd_finalize_pool(part2, nte, C, M, grad_of(bn2m.weight), grad_of(bn2m.bias),
                                                 dpooled, wsum, B, H, W, Pp, bn2)
            dy2 = ops.bn_bwd_apply_entry(dtype, dattn, dpooled, Pp, s.y2, bn2, 1, bn2m.weight, coef2,
                                         grad_of(conv2.bias))
            del dpooled, coef2
        del part2
        s.wsum = None
    else:
        with on_branch(dev, branch, dattn):
            # (dz2 is not materialised: the apply recomputes it from the same inputs)
            part2 = torch.empty(nte * 2 * C, device=dev, dtype=f32)
            if s.fra is not None:
                # ---- full-resolution attention: da = dattn + projections' dgrad; then relu(bn2 y2) ----
                da = fra.core_backward(lsa, s.fra, dattn, dtype, s.pk)
                s.fra = None
                call("dfcsa_bwd_relu_bn", T, M, C, P(da), P(s.y2), P(bn2.scale), P(bn2.shift), P(bn2.mean),
                     P(bn2.invstd), None, *S(part2), stream())
                coef2 = ops.bn_bwd_finalize(part2, nte, 2, C, M, grad_of(bn2m.weight), grad_of(bn2m.bias))
                dy2 = ops.bn_bwd_apply_relu(dtype, da, s.y2, bn2, bn2m.weight, coef2, grad_of(conv2.bias))
                del da
            else:
                # ---- LightSelfAttention ----
                dpooled = lsa_core_backward(lsa, (s.pooled, s.qkv, s.A, s.o, s.Wqkv), dattn, Pp, dtype, s.pk)
                # ---- attention entry: a = relu(bn2 y2) feeds the pool and the attn residual ----
                call("dfcsa_bwd_attn_entry", T, B, H, W, C, P(dattn), P(dpooled), Pp, P(s.y2), P(bn2.scale),
                     P(bn2.shift), P(bn2.mean), P(bn2.invstd), 1, None, *S(part2), stream())
                coef2 = ops.bn_bwd_finalize(part2, nte, 2, C, M, grad_of(bn2m.weight), grad_of(bn2m.bias))
                dy2 = ops.bn_bwd_apply_entry(dtype, dattn, dpooled, Pp, s.y2, bn2, 1, bn2m.weight, coef2,
                                             grad_of(conv2.bias))
                del dpooled
            del part2, coef2
    del dattn

    # ---- local branch: relu(bn1 y1) (dz1 recomputed by the apply, not materialised) ----
    if local_part is not None:   # formed beside the attention entry's sums (dfcsa_bwd_relu_bn_pair)
        part, npart = local_part, nte
    elif fused_bn1:
        part, npart = part1, npart1
    else:
        part, npart = torch.empty(nte * 2 * C, device=dev, dtype=f32), nte
        call("dfcsa_bwd_relu_bn", T, M, C, P(dlocal), P(s.y1), P(bn1.scale), P(bn1.shift), P(bn1.mean),
             P(bn1.invstd), None, *S(part), stream())
    coef = ops.bn_bwd_finalize(part, npart, 2, C, M, grad_of(bn1m.weight), grad_of(bn1m.bias))
    dy1 = ops.bn_bwd_apply_relu(dtype, dlocal, s.y1, bn1, bn1m.weight, coef, grad_of(conv1.bias))
    del dlocal
    xs = s.xs
    if "WdxA" in s.pk.t:
        # ---- split input gradient: the 3x3 dgrad over dy1 (+ the residual's 1x1 / identity over dres)
        #      and conv1's weight gradient start while the attention chain still runs on the branch
        #      stream; dy2's 1x1 dgrad is accumulated after the join ----
        with on_side(dev, dy1, *xs):
            ops.conv_wgrad_into(dtype, [dy1], C, _conv3x3_segments(xs), Cs, grid, hw, [grad_of(conv1.weight)], 9,
                                Cin_p, Cin_real)
        dxs = None
        if need_dx:
            segs = [(dy1, 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)] + [(dres, 0, 0)]
            dxs = [torch.empty((B, H, W, Cs), dtype=dtype, device=dev) for _ in range(nsrc)]
            ops.conv_gemm(dtype, segs, C, grid, hw, s.pk["WdxA"], rup(10 * C, ops.KALIGN), Cin_p, dxs, Cs)
        join_branch(dev, branch, dy2)
        if gate_wgrads is not None:
            gate_wgrads()
        if need_dx:
            ops.conv_gemm(dtype, [(dy2, 0, 0)], C, grid, hw, s.pk["WdxB"], rup(C, ops.KALIGN), Cin_p, dxs, Cs,
                          accumulate=True)
        with on_side(dev, dy2, dres, *xs):
            if has_res:
                ops.conv_wgrad_into(dtype, [dy2, dres], C, [(x, 0, 0) for x in xs], Cs, grid, hw,
                                    [grad_of(conv2.weight), grad_of(blk.residual_conv.weight)], 1, Cin_p, Cin_real)
            else:
                ops.conv_wgrad_into(dtype, [dy2], C, [(x, 0, 0) for x in xs], Cs, grid, hw,
                                    [grad_of(conv2.weight)], 1, Cin_p, Cin_real)
        streams.flush_deferred()
        return dxs
    # the last block of the backward (no input gradient): the main stream has nothing left to do, so
    # conv1's weight gradient (dy1 is final) starts before the join instead of after it (LAST_EARLY)
    early1 = not need_dx and LAST_EARLY[0] >= 1
    if early1:
        with on_side(dev, dy1, *xs):
            ops.conv_wgrad_into(dtype, [dy1], C, _conv3x3_segments(xs), Cs, grid, hw, [grad_of(conv1.weight)], 9,
                                Cin_p, Cin_real)
    join_branch(dev, branch, dy2)
    if gate_wgrads is not None:
        gate_wgrads()

    # ---- input gradient: 3x3 dgrad + both 1x1 dgrads in one implicit GEMM (critical path) ----
    # (order against the side-stream weight gradients: DX_FIRST)
    dxs = None

    def input_grad():
        Kx = rup(11 * C, ops.KALIGN)
        Wdx = s.pk["Wdx"]  # [W1^T | W2^T | Wres^T or I] side by side
        segs = [(dy1, 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)] + [(dy2, 0, 0), (dres, 0, 0)]
        out = [torch.empty((B, H, W, Cs), dtype=dtype, device=dev) for _ in range(nsrc)]
        ops.conv_gemm(dtype, segs, C, grid, hw, Wdx, Kx, Cin_p, out, Cs)
        return out

    if need_dx and DX_FIRST[0]:
        dxs = input_grad()

    # ---- weight gradients of the input-side convs (side stream) ----
    def input_wgrads(dy1_=dy1, dy2_=dy2, dres_=dres, xs_=xs):
        with on_side(dev, dy1_, dy2_, dres_, *xs_):
            if not early1:
                ops.conv_wgrad_into(dtype, [dy1_], C, _conv3x3_segments(xs_), Cs, grid, hw,
                                    [grad_of(conv1.weight)], 9, Cin_p, Cin_real)
            if has_res:
                ops.conv_wgrad_into(dtype, [dy2_, dres_], C, [(x, 0, 0) for x in xs_], Cs, grid, hw,
                                    [grad_of(conv2.weight), grad_of(blk.residual_conv.weight)], 1, Cin_p, Cin_real)
            else:
                ops.conv_wgrad_into(dtype, [dy2_], C, [(x, 0, 0) for x in xs_], Cs, grid, hw,
                                    [grad_of(conv2.weight)], 1, Cin_p, Cin_real)

    defer = DEFER_WGRAD[0] and ARMED[0] == 0 and streams.ENABLED[0]
    if not defer:
        input_wgrads()
    if need_dx and not DX_FIRST[0]:
        dxs = input_grad()
    streams.flush_deferred()     # the previous block's deferred weight gradients (DEFER_WGRAD)
    if defer:
        streams.defer(input_wgrads)
    return dxs


# the backward's last block (no input gradient): conv1's weight gradient issued before the attention
# chain's join (DFCSA_LAST_EARLY=1, the default: same-box A/B 1645.3 / 1645.4 / 1646.0 against
# 1644.1 / 1642.8 / 1638.7 img/s for 0), and the gate / fusion weight gradients too (=2: 1640.5 /
# 1636.6 / 1640.9)
LAST_EARLY = [int(os.environ.get("DFCSA_LAST_EARLY", "1"))]

# the input-side convs' weight gradients of a block issued one block later in the backward (after the
# next block's input-gradient GEMM) instead of right after its own join: DFCSA_DEFER_WGRAD=1
DEFER_WGRAD = [os.environ.get("DFCSA_DEFER_WGRAD", "0") == "1"]

# smallest H*W whose attention entry conv runs on the branch stream (block_forward);
# DFCSA_ENTRY_ON_BRANCH_HW, 0 = every level
ENTRY_ON_BRANCH_HW = [int(os.environ.get("DFCSA_ENTRY_ON_BRANCH_HW", "0"))]

# the block-input gradient split around the attention chain's join (block_backward), opt-in with
# DFCSA_SPLIT_DX=1: measured slower (same-box A/B 1531 vs 1566 img/s) -- the 3x3 dgrad GEMM issued
# before the join takes the CUs the latency-bound attention chain needs, so the join comes later
SPLIT_DX = [os.environ.get("DFCSA_SPLIT_DX", "0") == "1"]

# the gate / fusion convs' weight gradients are issued on the side stream after the attention chain's
# join, not before it: their GEMM then stays off the CUs the latency-bound chain needs (same-box A/B
# 1594 vs 1565 img/s); DFCSA_WGRAD_LATE=0 restores the early issue
WGRAD_LATE = [os.environ.get("DFCSA_WGRAD_LATE", "1") == "1"]

# the attention-entry BN2-backward statistics from the forward pool's window sums (no full-resolution
# pass after the attention backward); DFCSA_ENTRY_WS=0 restores the dfcsa_bwd_attn_entry pass
ENTRY_WS = [os.environ.get("DFCSA_ENTRY_WS", "1") == "1"]


# pooled attention above this many tokens (N = P*P) in bf16 mode on the flash kernels
# (dfcsa_lsa_flash_fwd / _bwd: bf16 MFMA, online softmax, P recomputed from the row log-sum-exp in the
# backward, nothing N x N stored); at and below it, and in fp32 (parity) mode, the per-row fp32 kernels
# (dfcsa_lsa_attn / dfcsa_lsa_attn_bwd).  DFCSA_LSA_FLASH_MIN_N; same-box bench at 224^2, B = 16: P = 8
# 1484 -> 1533 img/s with its 64 tokens on the flash kernels, P = 4 1620 -> 1600 (profiles/r06g_pools.jsonl)
LSA_FLASH_MIN_N = [int(os.environ.get("DFCSA_LSA_FLASH_MIN_N", "32"))]
# the flash kernels' fp32 variant (generic, one wave per row) for fp32 mode and for the widths the
# MFMA kernels do not take: off by default (the per-row kernels are the fp32 path); tests switch it on
LSA_FLASH_FP32 = [os.environ.get("DFCSA_LSA_FLASH_FP32", "0") == "1"]


# bf16 flash layers on the window-sum path: the projection dgrad's bf16 dpooled is read as it is by the
# entry's pool rows and BatchNorm apply (DFCSA_LSA_DP16=0: widened to fp32 first; same-box +0.4-0.7 % at
# P = 8 / 16 / 32, profiles/r06dp16_ab.txt; gradients bitwise equal)
LSA_DP16 = [os.environ.get("DFCSA_LSA_DP16", "1") == "1"]

# pooled attention with N > 64 tokens: dgamma of the upsample backward as a separate sum over per-token
# partials instead of the in-kernel ticket (DFCSA_LSA_DGAMMA_SPLIT=0: in-kernel, N / 64 tokens per
# workgroup)
LSA_DGAMMA_SPLIT = [os.environ.get("DFCSA_LSA_DGAMMA_SPLIT", "1") == "1"]


class FlashSaved:
    """What the flash path keeps for the backward in place of A: the row log-sum-exp and, on the bf16
    MFMA kernels, qkv and the pooled map in bf16 (the projection GEMMs' operands; None on the fp32
    kernels)."""
    __slots__ = ("lse", "qkv16", "pooled16")

    def __init__(self, lse, qkv16=None, pooled16=None):
        self.lse, self.qkv16, self.pooled16 = lse, qkv16, pooled16


def flash16_layer(dtype, C, Cq, pool_size):
    """True when this layer's pooled attention runs on the bf16 flash kernels (with bf16 q/k/v
    projection GEMMs)."""
    J = 2 * Cq + C
    return (dtype == torch.bfloat16 and pool_size * pool_size > LSA_FLASH_MIN_N[0] and _lsa_gemm_ok(C, J)
            and _lib.LIB.dfcsa_lsa_flash_path(C, Cq, J) == 1)


def _flash_mode(dtype, C, Cq, J, N):
    """None (per-row kernels) or (storage dtype code, bf16?) of the flash kernels for this layer."""
    if N <= LSA_FLASH_MIN_N[0]:
        return None
    if dtype == torch.bfloat16 and _lib.LIB.dfcsa_lsa_flash_path(C, Cq, J) == 1:
        return _lib.DT_BF16, True
    if LSA_FLASH_FP32[0] and C <= 1024 and C % 4 == 0:
        return _lib.DT_F32, False
    return None


def _lsa_gemm_ok(C, J):
    return C % 8 == 0 and J % 8 == 0 and C >= 64


def lsa_core_forward(lsa, y, scale, shift, relu, pool_size, dtype, pk, window_sums=False):
    """LightSelfAttention up to the pooled output o (unet_dfc_sa_res.py:24-34): pool of
    act(y*scale + shift) -> q/k/v 1x1 convs -> softmax(q k^T) -> o = v A^T (all fp32).
    window_sums: also return the pool windows' sums of the relu mask r and of r*y ([B][N][2][C],
    dfcsa_lsa_pooled_ws) for the attention-entry backward (dfcsa_bn_bwd_finalize_pool); on the
    projection-GEMM path only (otherwise the 6th element is None)."""
    B, H, W, C = y.shape
    dev = y.device
    f32 = torch.float32
    Pp = pool_size
    N = Pp * Pp
    Cq = lsa.query_conv.out_channels
    J = 2 * Cq + C
    fm = _flash_mode(dtype, C, Cq, J, N)
    f16 = fm is not None and fm[1]
    # the window sums feed the projection backward's extra rows (B*N <= 4096, fp32 projections), the
    # pool-rows kernel (bf16 flash layers, dfcsa_lsa_pool_rows) or the pool-fused finalize
    # (dfcsa_bn_bwd_finalize_pool: N <= 256); otherwise the entry pass computes them
    ws = window_sums and _lsa_gemm_ok(C, J) and (f16 or N <= 256 or B * N <= 4096)
    wsum = torch.empty((B, N, 2, C), device=dev, dtype=f32) if ws else None
    pooled16 = torch.empty((B, N, C), device=dev, dtype=torch.bfloat16) if f16 else None
    # large pools on the projection-GEMM path: one wave per window, pooled (+ its bf16 copy, + the window
    # sums) written by the pool launch itself (dfcsa_lsa_pool_direct); the bf16 flash layers keep only
    # the bf16 copy (their backward reads pooled16)
    direct = _lsa_gemm_ok(C, J) and _lib.LIB.dfcsa_lsa_pool_direct_ok(C, Pp, H, W) == 1
    pooled = None if (direct and f16) else torch.empty((B, N, C), device=dev, dtype=f32)
    if direct:
        call("dfcsa_lsa_pool_direct", dt(dtype), B, H, W, C, P(y), P(scale), P(shift), Pp, int(relu), P(pooled),
             P(pooled16), P(wsum), stream())
    else:
        S = ops._lib.LIB.dfcsa_lsa_pool_splits(H, Pp)
        part = torch.empty(B * N * S * C, device=dev, dtype=f32)
        wpart = torch.empty(B * N * S * 2 * C, device=dev, dtype=f32) if ws else None
        call("dfcsa_lsa_pool_ws", dt(dtype), B, H, W, C, P(y), P(scale), P(shift), Pp, int(relu), P(part),
             P(wpart), stream())
    bqkv = pk["bqkv"]
    o = torch.empty((B, N, C), device=dev, dtype=f32)
    Wqkv = None
    if f16:
        # bf16 mode, large pools: the q/k/v projections as one bf16 implicit GEMM (the reference's 1x1
        # convs under bf16 autocast) whose output feeds the bf16 flash kernels directly; the backward
        # recomputes P from the row log-sum-exp (nothing N x N is stored)
        bf = torch.bfloat16
        if not direct:
            call("dfcsa_lsa_pooled_ws", B, H, W, C, Pp, P(part), P(pooled), P(wpart), P(wsum), stream())
            call("dfcsa_cast_f32", _lib.DT_BF16, ctypes.c_int64(B * N * C), P(pooled), P(pooled16), 0, stream())
        qkv16 = torch.empty((B, N, J), device=dev, dtype=bf)
        ops.conv_gemm(bf, [(pooled16, 0, 0)], C, (1, B * N, 1), (B * N, 1), pk["Wp16"], rup(C, ops.KALIGN), J,
                      [qkv16], J, bias=bqkv)
        lse = torch.empty(B * N, device=dev, dtype=f32)
        call("dfcsa_lsa_flash_fwd", _lib.DT_BF16, B, N, C, Cq, J, P(qkv16), P(o), P(lse), stream())
        A = FlashSaved(lse, qkv16, pooled16)
        qkv = None
    else:
        qkv = torch.empty((B, N, J), device=dev, dtype=f32)
        if _lsa_gemm_ok(C, J):
            # projections on the MFMA implicit GEMM (fp32 operands, f32 MFMA): [B*N, C] x [C, J]
            if not direct:
                call("dfcsa_lsa_pooled_ws", B, H, W, C, Pp, P(part), P(pooled), P(wpart), P(wsum), stream())
            ops.conv_gemm(f32, [(pooled, 0, 0)], C, (1, B * N, 1), (B * N, 1), pk["Wp"], rup(C, ops.KALIGN), J, [qkv],
                          J, bias=bqkv)
        else:
            Wqkv, WqkvT = pk["Wqkv"], pk["WqkvT"]
            call("dfcsa_lsa_qkv", B, H, W, C, Cq, Pp, P(part), P(WqkvT), P(bqkv), P(pooled), P(qkv), stream())
        if fm is not None:   # the flash kernels' fp32 variant (opt-in: LSA_FLASH_FP32)
            lse = torch.empty(B * N, device=dev, dtype=f32)
            call("dfcsa_lsa_flash_fwd", _lib.DT_F32, B, N, C, Cq, J, P(qkv), P(o), P(lse), stream())
            A = FlashSaved(lse)
        else:
            A = torch.empty((B, N, N), device=dev, dtype=f32)
            call("dfcsa_lsa_attn", B, N, C, Cq, P(qkv), P(A), P(o), stream())
    if window_sums:
        return pooled, qkv, A, o, Wqkv, wsum
    return pooled, qkv, A, o, Wqkv


def lsa_core_backward(lsa, saved, dattn, pool_size, dtype, pk, pool_rows=None):
    """Backward of gamma * bilinear(o) (unet_dfc_sa_res.py:36-38) through the attention core;
    accumulates gamma/q/k/v parameter gradients and returns d(pooled) [B][N][C] fp32.
    pool_rows = (wsum, mean, invstd, rows_ptr, H, W): the projection backward also writes the attention
    entry's pool-backward BatchNorm rows (dfcsa_conv_wgrad_dgrad1x1_pool)."""
    pooled, qkv, A, o, Wqkv = saved
    B, H, W, C = dattn.shape
    dev = dattn.device
    f32 = torch.float32
    Pp = pool_size
    N = Pp * Pp
    Cq = lsa.query_conv.out_channels
    J = 2 * Cq + C
    rows = torch.empty(B * H * Pp * C, device=dev, dtype=f32)
    call("dfcsa_lsa_up_bwd_rows", dt(dtype), B, H, W, C, P(dattn), Pp, P(rows), stream())
    dqkv = torch.empty((B, N, J), device=dev, dtype=f32)
    if Pp <= 4 and C % 8 == 0 and Cq % 2 == 0 and C <= 1024 and LSA_CORE_BWD[0]:
        # upsample column pass + attention backward in one launch (dk / dv and dgamma by last arrivers)
        dO = torch.empty((B, N, C), device=dev, dtype=f32)
        dE = torch.empty((B, N, N), device=dev, dtype=f32)
        gpart = torch.empty(B * N, device=dev, dtype=f32)
        call("dfcsa_lsa_core_bwd", B, H, C, Cq, Pp, P(rows), P(o), P(lsa.gamma), P(qkv), P(A), P(dqkv), P(dO), P(dE),
             P(gpart), P(grad_of(lsa.gamma)), stream())
    elif (isinstance(A, FlashSaved) and A.qkv16 is not None and H <= 29 * Pp
          and _lib.LIB.dfcsa_get_tuning(49) == 1):
        # bf16 flash layer: the column pass writes the bf16 dO and r of the flash backward itself (one
        # wave per token; no fp32 dO, no prep pass), then the MFMA kernels (dfcsa_lsa_flash_bwd_up)
        gpart = torch.empty(B * N, device=dev, dtype=f32)
        nb = ctypes.c_int64()
        call("dfcsa_lsa_flash_bwd_bytes", _lib.DT_BF16, B, N, C, Cq, J, ctypes.byref(nb))
        work = torch.empty((nb.value + 15) // 16 * 4, device=dev, dtype=f32)
        dqkv = torch.empty((B, N, J), device=dev, dtype=torch.bfloat16)
        call("dfcsa_lsa_flash_bwd_up", B, H, C, Cq, Pp, P(rows), P(o), P(lsa.gamma), P(A.qkv16), P(A.lse), P(dqkv),
             P(gpart), P(work), ctypes.c_int64(work.numel() * 4), stream())
        del work
        call("dfcsa_sum_to_scalar", P(gpart), B * N, P(grad_of(lsa.gamma)), stream())
        # with the entry's pool rows (the window-sum path) the bf16 dpooled is consumed as it is (the
        # rows kernel here, dfcsa_bn_bwd_apply_entry16 after the finalize): no fp32 widening pass
        dpooled = _lsa_proj_bwd_bf16(lsa, A.pooled16, dqkv, B, N, C, Cq, pk,
                                     widen=pool_rows is None or not LSA_DP16[0])
        if pool_rows is not None:   # the attention entry's pool-backward BatchNorm rows
            wsum, mean, invstd, rows_ptr, Hh, Ww = pool_rows
            call("dfcsa_lsa_pool_rows", dt(dpooled.dtype), B * N, C, Pp, Hh, Ww, P(dpooled), P(wsum), P(mean),
                 P(invstd), rows_ptr, ctypes.c_int64((B * N + 15) // 16 * 2 * C), stream())
        return dpooled
    else:
        dO = torch.empty((B, N, C), device=dev, dtype=f32)
        if N > 64 and LSA_DGAMMA_SPLIT[0]:
            # large pools: dgamma as a separate fixed-order sum of the column pass's partials (the
            # in-kernel last-arriver sum takes one ticket atomic per workgroup)
            gpart = torch.empty(B * N, device=dev, dtype=f32)
            call("dfcsa_lsa_up_bwd_cols", B, H, C, Pp, P(rows), P(o), P(lsa.gamma), P(dO), P(gpart), None, None,
                 stream())
            call("dfcsa_sum_to_scalar", P(gpart), B * N, P(grad_of(lsa.gamma)), stream())
        else:
            gpart = torch.empty(B * N, device=dev, dtype=f32)
            call("dfcsa_lsa_up_bwd_cols", B, H, C, Pp, P(rows), P(o), P(lsa.gamma), P(dO), P(gpart), None,
                 P(grad_of(lsa.gamma)), stream())    # dgamma summed in-kernel
        if isinstance(A, FlashSaved):
            f16 = A.qkv16 is not None
            T = _lib.DT_BF16 if f16 else _lib.DT_F32
            nb = ctypes.c_int64()
            call("dfcsa_lsa_flash_bwd_bytes", T, B, N, C, Cq, J, ctypes.byref(nb))
            work = torch.empty((nb.value + 15) // 16 * 4, device=dev, dtype=f32)
            if f16:
                dqkv = torch.empty((B, N, J), device=dev, dtype=torch.bfloat16)
            call("dfcsa_lsa_flash_bwd", T, B, N, C, Cq, J, P(A.qkv16 if f16 else qkv), P(dO), P(o), P(A.lse),
                 P(dqkv), P(work), ctypes.c_int64(work.numel() * 4), stream())
            del work
            if f16:
                dpooled = _lsa_proj_bwd_bf16(lsa, A.pooled16, dqkv, B, N, C, Cq, pk,
                                             widen=pool_rows is None or not LSA_DP16[0])
                if pool_rows is not None:   # the attention entry's pool-backward BatchNorm rows
                    wsum, mean, invstd, rows_ptr, Hh, Ww = pool_rows
                    call("dfcsa_lsa_pool_rows", dt(dpooled.dtype), B * N, C, Pp, Hh, Ww, P(dpooled), P(wsum),
                         P(mean), P(invstd), rows_ptr, ctypes.c_int64((B * N + 15) // 16 * 2 * C), stream())
                return dpooled
        else:
            dE = torch.empty((B, N, N), device=dev, dtype=f32)
            call("dfcsa_lsa_attn_bwd", B, N, C, Cq, P(qkv), P(A), P(dO), P(dE), P(dqkv), stream())
    dpooled = torch.empty((B, N, C), device=dev, dtype=f32)
    qw, kw, vw = lsa.query_conv.weight, lsa.key_conv.weight, lsa.value_conv.weight
    if _lsa_gemm_ok(C, J):
        BN = B * N
        # dW = dqkv^T pooled (pixel reduction GEMM), db = column sums and dpooled = dqkv Wqkv, all
        # in one launch; the stacked q/k/v rows go straight into the three weight / bias gradients
        ops.conv_wgrad_dgrad1x1(f32, dqkv, J, pooled, C, BN, [grad_of(qw), grad_of(kw), grad_of(vw)], 1, Cq, C,
                                pk["WT"], rup(J, ops.KALIGN), C, dpooled, layout=2,
                                bias_grads=[grad_of(lsa.query_conv.bias), grad_of(lsa.key_conv.bias),
                                            grad_of(lsa.value_conv.bias)],
                                pool=None if pool_rows is None else pool_rows + (Pp,))
    else:
        call("dfcsa_lsa_proj_bwd", B, N, C, Cq, P(dqkv), P(pooled), P(Wqkv),
             P(grad_of(qw)), P(grad_of(kw)), P(grad_of(vw)), P(grad_of(lsa.query_conv.bias)),
             P(grad_of(lsa.key_conv.bias)), P(grad_of(lsa.value_conv.bias)), P(dpooled), stream())
    return dpooled


def _lsa_proj_bwd_bf16(lsa, pooled16, dqkv16, B, N, C, Cq, pk, widen=True):
    """Backward of the bf16 q/k/v projections of a flash layer: dW = dqkv^T pooled (bf16 weight-gradient
    GEMM into the fp32 gradients, stacked q/k/v rows -> three tensors), db = column sums of dqkv,
    dpooled = dqkv Wqkv (bf16 implicit GEMM; widened to fp32 for the attention-entry backward unless
    widen is False -- the window-sum path's consumers read the bf16 values as they are)."""
    dev = dqkv16.device
    f32, bf = torch.float32, torch.bfloat16
    J, BN = 2 * Cq + C, B * N
    qw, kw, vw = lsa.query_conv.weight, lsa.key_conv.weight, lsa.value_conv.weight
    ops.conv_wgrad_into(bf, [dqkv16], J, [(pooled16, 0, 0)], C, (1, BN, 1), (BN, 1),
                        [grad_of(qw), grad_of(kw), grad_of(vw)], 1, Cq, C, layout=2)
    nt = ops.ntiles_ew(BN, J)
    part = torch.empty(nt * J, device=dev, dtype=f32)
    call("dfcsa_channel_sum", _lib.DT_BF16, BN, J, P(dqkv16), *S(part), stream())
    call("dfcsa_slab_colsum3", P(part), nt, J, Cq, Cq, P(grad_of(lsa.query_conv.bias)),
         P(grad_of(lsa.key_conv.bias)), P(grad_of(lsa.value_conv.bias)), stream())
    dp16 = torch.empty((B, N, C), device=dev, dtype=bf)
    ops.conv_gemm(bf, [(dqkv16, 0, 0)], J, (1, BN, 1), (BN, 1), pk["WT16"], rup(J, ops.KALIGN), C, [dp16], C)
    if not widen:
        return dp16
    dpooled = torch.empty((B, N, C), device=dev, dtype=f32)
    call("dfcsa_bf16_to_f32", ctypes.c_int64(BN * C), P(dp16), P(dpooled), stream())
    return dpooled


class LSAFunction(torch.autograd.Function):
    """Standalone LightSelfAttention on an NHWC tensor (no BatchNorm/ReLU in front)."""

    @staticmethod
    def forward(ctx, lsa, pool_size, dtype, x, *params):
        B, H, W, C = x.shape
        dev = x.device
        one = torch.ones(C, device=dev)
        zero = torch.zeros(C, device=dev)
        pk = get_packset(lsa, ("lsa", dtype, pool_size, LSA_FLASH_MIN_N[0], param_key(lsa)),
                         lambda ps: _build_lsa_packs(ps, lsa, dtype, pool_size))
        saved = lsa_core_forward(lsa, x, one, zero, False, pool_size, dtype, pk)
        out = torch.empty_like(x)
        call("dfcsa_block_local_attn", dt(dtype), B, H, W, C, None, None, None, P(x), P(one), P(zero),
             P(saved[3]), pool_size, P(lsa.gamma), 0, None, P(out), stream())
        ctx.lsa, ctx.saved, ctx.ps, ctx.dtype, ctx.np = lsa, saved, pool_size, dtype, len(params)
        ctx.x, ctx.pk = x, pk
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        x = ctx.x
        B, H, W, C = x.shape
        dev = x.device
        dpooled = lsa_core_backward(ctx.lsa, ctx.saved, g, ctx.ps, ctx.dtype, ctx.pk)
        one = torch.ones(C, device=dev)
        zero = torch.zeros(C, device=dev)
        dx = torch.empty_like(x)
        part = torch.empty(ops.ntiles_ew(B * H * W, C) * 2 * C, device=dev, dtype=torch.float32)
        call("dfcsa_bwd_attn_entry", dt(ctx.dtype), B, H, W, C, P(g), P(dpooled), ctx.ps, P(x), P(one), P(zero),
             P(zero), P(one), 0, P(dx), *S(part), stream())
        ctx.saved = None
        return (None, None, None, dx, *([None] * ctx.np))


def block_params(blk):
    return [p for p in blk.parameters()]


class DFCBlockPoolFunction(torch.autograd.Function):
    """DFCBlockFunction for an encoder block followed by MaxPool2d(2,2) (reference :165-172):
    returns (pooled, out) -- out is the decoder skip -- like MaxPoolFork after the block."""

    @staticmethod
    def forward(ctx, blk, pool_size, dtype, nsrc, *args):
        xs = list(args[:nsrc])
        training = blk.training
        (pooled, out), saved = block_forward(blk, xs, pool_size, training, dtype, pool=True)
        ctx.blk, ctx.saved, ctx.dtype, ctx.nsrc, ctx.nparams = blk, saved, dtype, nsrc, len(args) - nsrc
        ctx.training = training
        return pooled, out

    @staticmethod
    def backward(ctx, dpooled, dskip):
        if not ctx.training:
            raise_eval_backward()
        need_dx = any(ctx.needs_input_grad[4:4 + ctx.nsrc])
        dxs = block_backward(ctx.blk, ctx.saved, None, need_dx, ctx.dtype, pool_grads=(dpooled, dskip))
        ctx.saved = None
        notify_grads_ready(ctx.blk)
        grads = list(dxs) if dxs is not None else [None] * ctx.nsrc
        return (None, None, None, None, *grads, *([None] * ctx.nparams))


class DFCBlockFunction(torch.autograd.Function):
    """autograd node for one DFC block: inputs = NHWC sources (+ the block's parameters, passed
    only so the graph knows they are upstream; their gradients are accumulated in place)."""

    @staticmethod
    def forward(ctx, blk, pool_size, dtype, nsrc, *args):
        xs = list(args[:nsrc])
        training = blk.training
        out, saved = block_forward(blk, xs, pool_size, training, dtype)
        ctx.blk, ctx.saved, ctx.dtype, ctx.nsrc, ctx.nparams = blk, saved, dtype, nsrc, len(args) - nsrc
        ctx.training = training
        return out

    @staticmethod
    def backward(ctx, dout):
        if not ctx.training:
            raise_eval_backward()
        need_dx = any(ctx.needs_input_grad[4:4 + ctx.nsrc])
        dxs = block_backward(ctx.blk, ctx.saved, dout, need_dx, ctx.dtype)
        ctx.saved = None
        notify_grads_ready(ctx.blk)
        grads = list(dxs) if dxs is not None else [None] * ctx.nsrc
        return (None, None, None, None, *grads, *([None] * ctx.nparams))
