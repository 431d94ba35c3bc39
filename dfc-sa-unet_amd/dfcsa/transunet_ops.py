"""autograd nodes of TransUNet (reference models/transformer_unet.py, BASELINE config 4) on libdfcsa.

  StdWeights     weight standardisation of every StdConv2d of a model, one launch each way
                 (StdConv2d.forward, transformer_unet.py:21-27)
  RootStem       ResNetV2 root: StdConv2d 7x7/s2 as input gather + GEMM -> GroupNorm -> ReLU (:76-80)
  MaxPool3x3s2   nn.MaxPool2d(3, stride 2, padding 1)                                       (:101)
  Bottleneck     PreActBottleneck unit: 1x1 -> 3x3/s -> 1x1 StdConvs with GroupNorms and the
                 projection (or identity) residual                                           (:40-68)
  PatchEmbed     patch_embeddings 1x1 conv + position embeddings + dropout               (:186-199)
  ViTBlock       LN -> multi-head attention -> +h -> LN -> MLP(GELU) -> +h                (:202-220)
  LayerNormOut   encoder_norm                                                              (:236)
  Upsample2x     nn.UpsamplingBilinear2d(scale_factor=2)                                   (:262)
  ConcatC        torch.cat([x, skip], 1) when the widths differ (otherwise the decoder conv
                 takes both as GEMM source segments)                                        (:267)
  SegHead3x3     SegmentationHead conv 3x3 + bias -> NCHW fp32 logits                      (:272-276)

Every backward is written out by hand; parameter gradients are accumulated straight into
``param.grad`` (flat fp32 views).  StdConv2d weight gradients go to a scratch dL/d(w_hat) first and
are mapped through the standardisation by one table launch at the end of the backward pass (the
root stem is the last node autograd runs).  The ViT residual stream is fp32 in every precision.
"""
import math
import os

import torch

from . import _lib, ops, streams
from ._lib import LIB, call
from .block import grad_of
from .ddp import notify_grads_ready
from .ops import P, dt, rup, stream
from .packs import get_packset, param_key
from .streams import side_or_main
from .unet_ops import ConvBNReLU  # noqa: F401  (decoder convs: Conv2dReLU = conv + BN + ReLU)

KA = ops.KALIGN
SITE_EMBED = 1            # dropout call sites (the mask key); layer i uses 16 + 4*i + {0, 1, 2}


def _taps3(x):
    return [(x, kh - 1, kw - 1) for kh in range(3) for kw in range(3)]


def _f32(shape, dev):
    return torch.empty(shape, device=dev, dtype=torch.float32)


# ------------------------------------------------------------------ weight standardisation
class StdWeights:
    """Standardised weights of every StdConv2d (module order) in persistent fp32 buffers
    (``conv._what``, read by the pack plans), their rstd, and one flat scratch for dL/d(w_hat)
    (``conv._dwhat``, zeroed at every training forward)."""

    def __init__(self, convs, device):
        self.convs = list(convs)
        total = sum(c.weight.numel() for c in self.convs)
        self.g_flat = torch.zeros(total, device=device, dtype=torch.float32)
        entries, row0, off = [], 0, 0
        for c in self.convs:
            w = c.weight
            c._what = torch.empty_like(w)
            c._rstd = _f32((w.shape[0],), device)
            c._dwhat = self.g_flat[off:off + w.numel()].view_as(w)
            off += w.numel()
            e = _lib.WstdEntry()
            e.w, e.what, e.rstd, e.g, e.dw = P(w), P(c._what), P(c._rstd), P(c._dwhat), P(grad_of(w))
            e.K, e.rows, e.row0 = w.numel() // w.shape[0], w.shape[0], row0
            row0 += w.shape[0]
            entries.append(e)
        arr = (_lib.WstdEntry * len(entries))(*entries)
        self.table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(device)
        self.n, self.rows = len(entries), row0
        self.key = self._key()

    def _key(self):
        return tuple((c.weight.data_ptr(), c.weight.grad.data_ptr() if c.weight.grad is not None else 0)
                     for c in self.convs)

    def valid(self):
        return self.key == self._key()

    def forward(self, training):
        call("dfcsa_wstd_fwd", P(self.table), self.n, self.rows, stream())
        if training:
            call("dfcsa_zero", P(self.g_flat), self.g_flat.numel() * 4, stream())

    def backward(self):
        call("dfcsa_wstd_bwd", P(self.table), self.n, self.rows, stream())


def _what_key(*convs):
    return tuple(c._what.data_ptr() for c in convs)


# ------------------------------------------------------------------ GroupNorm helpers
class GNState:
    __slots__ = ("mr", "scsh", "G", "S")


# GroupNorm with the reductions finished inside the stats / backward-reduce launches (no separate
# finalize launches; dfcsa_gn_stats_fused / dfcsa_gn_bwd_reduce_fused, C <= 1024).  DFCSA_GN_FUSED=0
# restores the four-launch path.
GN_FUSED = [os.environ.get("DFCSA_GN_FUSED", "1") == "1"]


def _gn_fused(C, G):
    return GN_FUSED[0] and C <= 1024 and G <= 256 and C % G == 0


def gn_forward(dtype, y, gn):
    B, H, W, C = y.shape
    G = gn.num_groups
    st = GNState()
    st.mr, st.scsh = _f32((B * 2 * G,), y.device), _f32((B * 2 * C,), y.device)
    if _gn_fused(C, G):
        S = LIB.dfcsa_gn_nslices_fused(B, H * W, C)
        rows = _f32((B * S * 2 * C,), y.device)
        call("dfcsa_gn_stats_fused", dt(dtype), B, H * W, C, G, S, P(y), P(rows), P(gn.weight), P(gn.bias),
             float(gn.eps), P(st.mr), P(st.scsh), stream())
        st.G, st.S = G, S
        return st
    S = LIB.dfcsa_gn_nslices(H * W, C)
    part = _f32((B * S * 2 * C,), y.device)
    call("dfcsa_gn_stats", dt(dtype), B, H * W, C, S, P(y), P(part), stream())
    st.G, st.S = G, S
    call("dfcsa_gn_finalize", B, H * W, C, G, S, P(part), P(gn.weight), P(gn.bias), float(gn.eps), P(st.mr),
         P(st.scsh), stream())
    return st


def gn_apply(dtype, y, st, act, res=None, st_res=None):
    B, H, W, C = y.shape
    out = torch.empty_like(y)
    call("dfcsa_gn_apply", dt(dtype), B, H * W, C, P(y), P(st.scsh), P(res), P(st_res.scsh) if st_res else None,
         int(act), P(out), stream())
    return out


def gn_backward(dtype, dout, mask, y, st, gn, dz_out=None):
    """dy for y -> GroupNorm(gn) given dL/d(out) where out = relu(...) is `mask` (None: no ReLU)."""
    B, H, W, C = y.shape
    coef = _f32((B * 2 * st.G,), y.device)
    if _gn_fused(C, st.G):
        S = LIB.dfcsa_gn_nslices_fused(B, H * W, C)
        rows = _f32((B * S * 2 * C + B * 4 * C,), y.device)   # hand-off rows + [B][2][C] doubles
        call("dfcsa_gn_bwd_reduce_fused", dt(dtype), B, H * W, C, st.G, S, P(dout), P(mask), P(y), P(st.mr),
             P(gn.weight), P(rows), P(rows) + B * S * 2 * C * 4, P(coef), P(grad_of(gn.weight)),
             P(grad_of(gn.bias)), stream())
    else:
        part = _f32((B * st.S * 2 * C,), y.device)
        call("dfcsa_gn_bwd_reduce", dt(dtype), B, H * W, C, st.G, st.S, P(dout), P(mask), P(y), P(st.mr), P(part),
             stream())
        call("dfcsa_gn_bwd_finalize", B, H * W, C, st.G, st.S, P(part), P(gn.weight), P(coef),
             P(grad_of(gn.weight)), P(grad_of(gn.bias)), stream())
    dy = torch.empty_like(y)
    call("dfcsa_gn_bwd_apply", dt(dtype), B, H * W, C, st.G, P(dout), P(mask), P(y), P(st.mr), P(gn.weight), P(coef),
         P(dy), P(dz_out), stream())
    return dy


def _wgrad_1x1(dtype, dy, x, grid, in_hw, dst, stride=1):
    ops.conv_wgrad_into(dtype, [dy], dy.shape[-1], [(x, 0, 0)], x.shape[-1], grid, in_hw, [dst], 1, x.shape[-1],
                        x.shape[-1], stride=stride)


def _gemm_1x1(dtype, x, w, K, N, out, bias=None, accumulate=False):
    B, H, W, C = x.shape
    ops.conv_gemm(dtype, [(x, 0, 0)], C, (B, H, W), (H, W), w, K, N, [out], N, bias=bias, accumulate=accumulate)
    return out


def _linear_packs(ps, w, dtype, name):
    """rows [out][Kpad(in)] and the transposed (data-gradient) operand [in][Kpad(out)]."""
    cout, cin = w.shape[0], w.shape[1]
    W = ps.rows(name, dtype, w, cin, rup(cin, KA))
    ps.transpose(W, 0, 0, cout, cin, name + "t", (cin, rup(cout, KA)))


def channel_sum3_into(dtype, x, n0, n1, d0, d1=None, d2=None):
    """column sums of x [M][C] (any width) added to d0 [0, n0), d1 [n0, n0+n1), d2 [n0+n1, C)."""
    M, C = x.numel() // x.shape[-1], x.shape[-1]
    nt = LIB.dfcsa_colsum_ntiles(M)
    part = _f32((nt * C,), x.device)
    call("dfcsa_colsum_partial", dt(dtype), M, C, P(x), P(part), stream())
    call("dfcsa_slab_colsum3", P(part), nt, C, n0, n1, P(d0), P(d1), P(d2), stream())


def _drop_bwd_cs(dtype, M, C, dout, p, rng, site, out, x=None):
    """dropout backward (x given: GELU + dropout backward) of dout [M][C] into out, returning the
    64-row column partials of out (the bias gradient of the GEMM whose dY out is; dfcsa_colsum_partial).
    (Round 5 measured partials formed inside the dropout pass, dfcsa_drop_bwd_cs: slower, 600 vs 609
    img/s on config 4 bf16, and dropped.)"""
    if x is None:
        call("dfcsa_drop_bwd", dt(dtype), M * C, P(dout), float(p), P(rng), site, P(out), stream())
    else:
        call("dfcsa_gelu_drop_bwd", dt(dtype), M * C, P(x), P(dout), float(p), P(rng), site, P(out), stream())
    nt = LIB.dfcsa_colsum_ntiles(M)
    part = _f32((nt * C,), out.device)
    call("dfcsa_colsum_partial", dt(dtype), M, C, P(out), P(part), stream())
    return part


def _colsum_rows_into(part, M, C, out):
    """out[c] += the sum of the column-partial rows of _drop_bwd_cs."""
    call("dfcsa_slab_colsum3", P(part), part.numel() // C, C, C, 0, P(out), None, None, stream())


def bias_grad_into(dtype, dy, bias):
    channel_sum3_into(dtype, dy, dy.shape[-1], 0, grad_of(bias))


def _ln_forward(dtype, h, ln, out_shape):
    M, C = h.numel() // h.shape[-1], h.shape[-1]
    y = torch.empty(out_shape, dtype=dtype, device=h.device)
    mr = _f32((2 * M,), h.device)
    call("dfcsa_ln_fwd", dt(dtype), M, C, P(h), P(ln.weight), P(ln.bias), float(ln.eps), P(y), P(mr), stream())
    return y, mr


def _ln_backward(dtype, dy, h, mr, ln, dres):
    """dx (fp32) = LayerNorm backward + dres; dgamma/dbeta accumulated."""
    M, C = h.numel() // h.shape[-1], h.shape[-1]
    nt = LIB.dfcsa_ln_bwd_ntiles(M)
    part = _f32((nt * 2 * C,), h.device)
    dx = torch.empty_like(h)
    call("dfcsa_ln_bwd", dt(dtype), M, C, P(dy), P(h), P(mr), P(ln.weight), P(dres), P(dx), P(part), stream())
    call("dfcsa_slab_colsum3", P(part), nt, 2 * C, C, C, P(grad_of(ln.weight)), P(grad_of(ln.bias)), None, stream())
    return dx


# ------------------------------------------------------------------ ResNetV2 hybrid stem
class RootStem(torch.autograd.Function):
    """x NCHW fp32 [B, 1|3, H, W] -> relu(GroupNorm(StdConv 7x7/s2/p3 (x))) NHWC.  The conv runs as
    an input gather (k = tap*3 + ci, K padded to 64) + one GEMM; its backward (the last node of the
    backward pass) also maps every StdConv2d's dL/d(w_hat) to dL/dw (one table launch)."""

    @staticmethod
    def forward(ctx, x, root, dtype, model, *params):
        conv, gn = root.conv, root.gn
        B, Cs, H, W = x.shape
        Cin, C = conv.in_channels, conv.out_channels
        k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        if Cs not in (1, Cin) or C % 8:
            raise ValueError(f"root conv expects 1 or {Cin} input channels, got {Cs}")
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        Kpad = rup(k * k * Cin, KA)
        pk = get_packset(conv, (dtype, Kpad, _what_key(conv)), lambda ps: ps.rows("Wf", dtype, conv._what, Cin, Kpad))
        dev = x.device
        xin = x.contiguous().float()
        cols = torch.empty((B, Ho, Wo, Kpad), dtype=dtype, device=dev)
        call("dfcsa_im2col_input", dt(dtype), B, Cs, Cin, H, W, k, s, p, P(xin), Kpad, P(cols), stream())
        y = torch.empty((B, Ho, Wo, C), dtype=dtype, device=dev)
        ops.conv_gemm(dtype, [(cols, 0, 0)], Kpad, (B, Ho, Wo), (Ho, Wo), pk["Wf"], Kpad, C, [y], C)
        st = gn_forward(dtype, y, gn)
        out = gn_apply(dtype, y, st, 1)
        ctx.geo, ctx.dtype, ctx.root, ctx.model, ctx.np = (B, Ho, Wo, C, k, Cin, Kpad), dtype, root, model, len(params)
        ctx.cols, ctx.y, ctx.out, ctx.st = cols, y, out, st
        return out

    @staticmethod
    def backward(ctx, dout):
        B, Ho, Wo, C, k, Cin, Kpad = ctx.geo
        dtype, conv, gn = ctx.dtype, ctx.root.conv, ctx.root.gn
        dy = gn_backward(dtype, dout.contiguous(), ctx.out, ctx.y, ctx.st, gn)
        with side_or_main(dy.device, dy, ctx.cols):
            ops.conv_wgrad_into(dtype, [dy], C, [(ctx.cols, 0, 0)], Kpad, (B, Ho, Wo), (Ho, Wo), [conv._dwhat], k * k,
                                Cin, Cin)
        # every StdConv2d's dL/d(w_hat) (side-stream weight gradients) is final: map them to dL/dw
        streams.join()
        ctx.model._stdw.backward()
        notify_grads_ready(ctx.model)
        ctx.cols = ctx.y = ctx.out = None
        return (None, None, None, None, *([None] * ctx.np))


class MaxPool3x3s2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        B, H, W, C = x.shape
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        out = torch.empty((B, Ho, Wo, C), dtype=dtype, device=x.device)
        idx = torch.empty((B, Ho, Wo, C), dtype=torch.uint8, device=x.device)
        call("dfcsa_maxpool3s2_fwd", dt(dtype), B, H, W, C, P(x), P(out), P(idx), stream())
        ctx.save_for_backward(idx)
        ctx.shape, ctx.dtype = x.shape, dtype
        return out

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        B, H, W, C = ctx.shape
        dx = torch.empty(ctx.shape, dtype=ctx.dtype, device=g.device)
        call("dfcsa_maxpool3s2_bwd", dt(ctx.dtype), B, H, W, C, P(idx), P(g.contiguous()), P(dx), stream())
        return dx, None


def _unit_convs(unit):
    cs = [unit.conv1, unit.conv2, unit.conv3]
    if hasattr(unit, "downsample"):
        cs.append(unit.downsample)
    return cs


def _unit_packs(ps, unit, dtype, cin, cmid, cout, stride):
    W1 = ps.rows("W1", dtype, unit.conv1._what, cin, rup(cin, KA))
    ps.transpose(W1, 0, 0, cmid, cin, "W1t", (cin, rup(cmid, KA)))
    W2 = ps.rows("W2", dtype, unit.conv2._what, cmid, rup(9 * cmid, KA))
    if stride == 1:   # implicit transposed-conv dgrad: Wt[ci][tap*cmid + co] = W2[co][tap*cmid + ci]
        for tap in range(9):
            ps.transpose(W2, 0, tap * cmid, cmid, cmid, "W2t", (cmid, rup(9 * cmid, KA)), dc0=tap * cmid)
    else:             # column-gradient operand for col2im: Wc[tap*cmid + ci][co]
        ps.transpose(W2, 0, 0, cmid, 9 * cmid, "W2c", (9 * cmid, rup(cmid, KA)))
    W3 = ps.rows("W3", dtype, unit.conv3._what, cmid, rup(cmid, KA))
    ps.transpose(W3, 0, 0, cout, cmid, "W3t", (cmid, rup(cout, KA)))
    if hasattr(unit, "downsample"):
        Wd = ps.rows("Wd", dtype, unit.downsample._what, cin, rup(cin, KA))
        ps.transpose(Wd, 0, 0, cout, cin, "Wdt", (cin, rup(cout, KA)))


class Bottleneck(torch.autograd.Function):
    """PreActBottleneck.forward (transformer_unet.py:58-68):
      y1 = conv1(x) -> a1 = relu(gn1 y1);  y2 = conv2(a1, stride s) -> a2 = relu(gn2 y2)
      y3 = conv3(a2);  out = relu(gn3 y3 + (gn_proj(downsample(x, stride s)) | x))"""

    @staticmethod
    def forward(ctx, x, unit, dtype, *params):
        B, H, W, cin = x.shape
        c1, c2, c3 = unit.conv1, unit.conv2, unit.conv3
        cmid, cout, s = c1.out_channels, c3.out_channels, c2.stride[0]
        ds = hasattr(unit, "downsample")
        if c1.in_channels != cin or cmid % 8 or cout % 8:
            raise ValueError(f"bottleneck unit expects {c1.in_channels} input channels, got {cin}")
        if not ds and (cin != cout or s != 1):
            raise ValueError("identity residual needs cin == cout and stride 1")
        Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
        pk = get_packset(unit, (dtype, cin, param_key(unit), _what_key(*_unit_convs(unit))),
                         lambda ps: _unit_packs(ps, unit, dtype, cin, cmid, cout, s))
        dev = x.device
        y1 = _gemm_1x1(dtype, x, pk["W1"], rup(cin, KA), cmid, torch.empty((B, H, W, cmid), dtype=dtype, device=dev))
        st1 = gn_forward(dtype, y1, unit.gn1)
        a1 = gn_apply(dtype, y1, st1, 1)
        y2 = torch.empty((B, Ho, Wo, cmid), dtype=dtype, device=dev)
        ops.conv_gemm(dtype, _taps3(a1), cmid, (B, Ho, Wo), (H, W), pk["W2"], rup(9 * cmid, KA), cmid, [y2], cmid,
                      stride=s)
        st2 = gn_forward(dtype, y2, unit.gn2)
        a2 = gn_apply(dtype, y2, st2, 1)
        y3 = _gemm_1x1(dtype, a2, pk["W3"], rup(cmid, KA), cout,
                       torch.empty((B, Ho, Wo, cout), dtype=dtype, device=dev))
        st3 = gn_forward(dtype, y3, unit.gn3)
        if ds:
            yd = torch.empty((B, Ho, Wo, cout), dtype=dtype, device=dev)
            ops.conv_gemm(dtype, [(x, 0, 0)], cin, (B, Ho, Wo), (H, W), pk["Wd"], rup(cin, KA), cout, [yd], cout,
                          stride=s)
            std = gn_forward(dtype, yd, unit.gn_proj)
            out = gn_apply(dtype, y3, st3, 1, res=yd, st_res=std)
        else:
            yd = std = None
            out = gn_apply(dtype, y3, st3, 1, res=x)
        ctx.unit, ctx.dtype, ctx.pk, ctx.np = unit, dtype, pk, len(params)
        ctx.geo = (B, H, W, Ho, Wo, cin, cmid, cout, s, ds)
        ctx.t = (x, y1, a1, y2, a2, y3, yd, out)
        ctx.st = (st1, st2, st3, std)
        return out

    @staticmethod
    def backward(ctx, dout):
        unit, dtype, pk = ctx.unit, ctx.dtype, ctx.pk
        B, H, W, Ho, Wo, cin, cmid, cout, s, ds = ctx.geo
        x, y1, a1, y2, a2, y3, yd, out = ctx.t
        st1, st2, st3, std = ctx.st
        dev = x.device
        dout = dout.contiguous()
        dres = dyd = None
        if ds:
            dyd = gn_backward(dtype, dout, out, yd, std, unit.gn_proj)
            dy3 = gn_backward(dtype, dout, out, y3, st3, unit.gn3)
        else:
            dres = torch.empty_like(out)   # relu'(out) * dout: the identity path's gradient
            dy3 = gn_backward(dtype, dout, out, y3, st3, unit.gn3, dz_out=dres)
        with side_or_main(dev, dy3, a2):
            _wgrad_1x1(dtype, dy3, a2, (B, Ho, Wo), (Ho, Wo), unit.conv3._dwhat)
        da2 = _gemm_1x1(dtype, dy3, pk["W3t"], rup(cout, KA), cmid,
                        torch.empty((B, Ho, Wo, cmid), dtype=dtype, device=dev))
        dy2 = gn_backward(dtype, da2, a2, y2, st2, unit.gn2)
        del da2
        with side_or_main(dev, dy2, a1):
            ops.conv_wgrad_into(dtype, [dy2], cmid, _taps3(a1), cmid, (B, Ho, Wo), (H, W), [unit.conv2._dwhat], 9,
                                cmid, cmid, stride=s)
        da1 = torch.empty((B, H, W, cmid), dtype=dtype, device=dev)
        if s == 1:
            segs = [(dy2, 1 - kh, 1 - kw) for kh in range(3) for kw in range(3)]
            ops.conv_gemm(dtype, segs, cmid, (B, H, W), (H, W), pk["W2t"], rup(9 * cmid, KA), cmid, [da1], cmid)
        else:
            dcols = _gemm_1x1(dtype, dy2, pk["W2c"], rup(cmid, KA), 9 * cmid,
                              torch.empty((B, Ho, Wo, 9 * cmid), dtype=dtype, device=dev))
            call("dfcsa_col2im", dt(dtype), B, H, W, cmid, Ho, Wo, 3, s, 1, P(dcols), P(da1), 0, stream())
            del dcols
        dy1 = gn_backward(dtype, da1, a1, y1, st1, unit.gn1)
        del da1
        with side_or_main(dev, dy1, x, dyd):
            _wgrad_1x1(dtype, dy1, x, (B, H, W), (H, W), unit.conv1._dwhat)
            if ds:
                _wgrad_1x1(dtype, dyd, x, (B, Ho, Wo), (H, W), unit.downsample._dwhat, stride=s)
        dx = None
        if ctx.needs_input_grad[0]:
            if ds:
                dx = _gemm_1x1(dtype, dy1, pk["W1t"], rup(cmid, KA), cin, torch.empty_like(x))
                if s == 1:
                    _gemm_1x1(dtype, dyd, pk["Wdt"], rup(cout, KA), cin, dx, accumulate=True)
                else:
                    dc = _gemm_1x1(dtype, dyd, pk["Wdt"], rup(cout, KA), cin,
                                   torch.empty((B, Ho, Wo, cin), dtype=dtype, device=dev))
                    call("dfcsa_col2im", dt(dtype), B, H, W, cin, Ho, Wo, 1, s, 0, P(dc), P(dx), 1, stream())
            else:
                dx = _gemm_1x1(dtype, dy1, pk["W1t"], rup(cmid, KA), cin, dres, accumulate=True)
        ctx.t = ctx.st = None
        return (dx, None, None, *([None] * ctx.np))


# ------------------------------------------------------------------ ViT encoder
class PatchEmbed(torch.autograd.Function):
    """Embeddings.forward after the hybrid stem (:195-199): h = dropout(conv1x1(x) + bias + pos),
    tokens = the NHWC patch grid, fp32 out."""

    @staticmethod
    def forward(ctx, x, emb, dtype, p, rng, *params):
        conv, pos = emb.patch_embeddings, emb.position_embeddings
        B, h, w, Cin = x.shape
        if conv.kernel_size != (1, 1) or conv.stride != (1, 1):
            # patch size = img // 16 // grid > 1: the reference's patch conv gives (h / p) x (w / p)
            # tokens against (img / 16)^2 position embeddings, and its `x + position_embeddings`
            # (models/transformer_unet.py:179-181,196) raises this broadcast error at forward
            # (tests/golden/transunet_patch2_error.json, recorded from the reference)
            ntok = (h // conv.kernel_size[0]) * (w // conv.kernel_size[1])
            raise RuntimeError(f"The size of tensor a ({ntok}) must match the size of tensor b ({pos.shape[1]}) "
                               f"at non-singleton dimension 1")
        D = conv.out_channels
        if pos.shape[1] != h * w:
            raise ValueError(f"position embeddings for {pos.shape[1]} patches, grid has {h * w}")
        pk = get_packset(conv, (dtype, param_key(conv)), lambda ps: _linear_packs(ps, conv.weight, dtype, "W"))
        e = _gemm_1x1(dtype, x, pk["W"], rup(Cin, KA), D, torch.empty((B, h, w, D), dtype=dtype, device=x.device),
                      bias=conv.bias)
        out = _f32((B, h, w, D), x.device)
        call("dfcsa_drop_add_fwd", dt(dtype), e.numel(), P(e), P(pos), h * w * D, None, float(p), P(rng), SITE_EMBED,
             P(out), stream())
        ctx.emb, ctx.dtype, ctx.p, ctx.rng, ctx.pk, ctx.np = emb, dtype, p, rng, pk, len(params)
        ctx.x = x
        return out

    @staticmethod
    def backward(ctx, dout):
        emb, dtype, x = ctx.emb, ctx.dtype, ctx.x
        conv, pos = emb.patch_embeddings, emb.position_embeddings
        B, h, w, Cin = x.shape
        D = conv.out_channels
        de = torch.empty((B, h, w, D), dtype=dtype, device=x.device)
        call("dfcsa_drop_bwd", dt(dtype), de.numel(), P(dout.contiguous()), float(ctx.p), P(ctx.rng), SITE_EMBED,
             P(de), stream())
        call("dfcsa_batch_sum", dt(dtype), B, h * w * D, P(de), P(grad_of(pos)), stream())
        with side_or_main(de.device, de, x):
            bias_grad_into(dtype, de, conv.bias)
            _wgrad_1x1(dtype, de, x, (B, h, w), (h, w), grad_of(conv.weight))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _gemm_1x1(dtype, de, ctx.pk["Wt"], rup(D, KA), Cin, torch.empty_like(x))
        ctx.x = None
        return (dx, None, None, None, None, *([None] * ctx.np))


def _vit_packs(ps, blk, dtype, D, F):
    att, mlp = blk.attn, blk.ffn
    KD = rup(D, KA)
    Wqkv = None
    for i, lin in enumerate((att.query, att.key, att.value)):
        Wqkv = ps.rows("Wqkv", dtype, lin.weight, D, KD, row0=i * D, rows=3 * D)
    ps.transpose(Wqkv, 0, 0, 3 * D, D, "Wqkvt", (D, rup(3 * D, KA)))
    ps.concat("bqkv", [att.query.bias, att.key.bias, att.value.bias], 3 * D)
    _linear_packs(ps, att.out.weight, dtype, "Wo")
    _linear_packs(ps, mlp.fc1.weight, dtype, "W1")
    _linear_packs(ps, mlp.fc2.weight, dtype, "W2")


FLASH_MHA = os.environ.get("DFCSA_MHA_FLASH", "1") != "0"


def _flash_mha(dtype, dh):
    """bf16 heads of width 64 run on the MFMA flash-attention kernels (fwd and bwd)."""
    return (FLASH_MHA and dtype == torch.bfloat16 and dh == 64
            and LIB.dfcsa_fra_path(_lib.DT_BF16, dh, dh, 3 * dh, 0) == 1
            and LIB.dfcsa_fra_path(_lib.DT_BF16, dh, dh, 3 * dh, 1) == 1)


def mha_flash_forward(dtype, qkv, B, N, heads, dh):
    """Attention core (transformer_unet.py:146-154) of token-major qkv [B*N][3*heads*dh] on the bf16
    MFMA flash kernels of fra.hip: a head-major copy of q|k|v with q pre-scaled by 1/sqrt(dh),
    gamma = 1 and x = 0 (so their output is softmax(q k^T) v).  Returns (ctx [B*N][heads*dh], saved)."""
    dev = qkv.device
    Bh, scale = heads * B, 1.0 / math.sqrt(dh)
    qkv_h = torch.empty((Bh, N, 3 * dh), dtype=dtype, device=dev)
    call("dfcsa_heads_relayout", 0, B, N, heads, dh, 3, float(scale), P(qkv), P(qkv_h), stream())
    o_h = torch.empty((Bh, N, dh), dtype=dtype, device=dev)
    y_h = torch.empty_like(o_h)
    one = torch.ones(1, device=dev)
    lse = _f32((Bh * N,), dev)
    call("dfcsa_fra_fwd", dt(dtype), Bh, N, dh, dh, 3 * dh, P(qkv_h), P(torch.zeros_like(o_h)), P(one), P(o_h),
         P(y_h), P(lse), stream())
    del y_h
    cx = torch.empty((B * N, heads * dh), dtype=dtype, device=dev)
    call("dfcsa_heads_relayout", 1, B, N, heads, dh, 1, 1.0, P(o_h), P(cx), stream())
    return cx, (qkv_h, o_h, one, lse)


def mha_flash_backward(dtype, saved, dcx, B, N, heads, dh, col_partial=None):
    """d(qkv) [B*N][3*heads*dh] from d(ctx) (the dQ and dK/dV flash kernels; dq rescaled).  With
    col_partial (fp32 [ceil(B*N/64)][3*heads*dh]) the unpack also writes dqkv's column partials."""
    qkv_h, o_h, one, lse = saved
    dev = o_h.device
    Bh, scale = heads * B, 1.0 / math.sqrt(dh)
    dcx_h = torch.empty_like(o_h)
    call("dfcsa_heads_relayout", 0, B, N, heads, dh, 1, 1.0, P(dcx.contiguous()), P(dcx_h), stream())
    rvec = _f32((Bh * N,), dev)
    call("dfcsa_fra_bwd_prep", dt(dtype), Bh * N, dh, P(dcx_h), P(o_h), P(rvec), stream())
    dqkv_h = torch.empty_like(qkv_h)
    call("dfcsa_fra_bwd", dt(dtype), Bh, N, dh, dh, 3 * dh, P(qkv_h), P(dcx_h), P(one), P(lse), P(rvec), P(dqkv_h),
         stream())
    dqkv = torch.empty((B * N, 3 * heads * dh), dtype=dtype, device=dev)
    if col_partial is not None:
        call("dfcsa_heads_unpack_cs", B, N, heads, dh, 3, float(scale), P(dqkv_h), P(dqkv), P(col_partial),
             col_partial.numel(), stream())
    else:
        call("dfcsa_heads_relayout", 1, B, N, heads, dh, 3, float(scale), P(dqkv_h), P(dqkv), stream())
    return dqkv


class ViTBlock(torch.autograd.Function):
    """Block.forward (:211-220) with Attention (:137-157) and Mlp (:167-173):
      y1 = LN1(h); qkv = y1 [Wq|Wk|Wv]^T + b (one GEMM); ctx = MHA(qkv); h1 = drop(ctx Wo^T + bo) + h
      y2 = LN2(h1); f = y2 W1^T + b1; g = drop(gelu(f)); out = drop(g W2^T + b2) + h1
    h / h1 / out are fp32 NHWC token grids [B, gh, gw, D]."""

    @staticmethod
    def forward(ctx, h, blk, dtype, p, p_attn, rng, site, *params):
        B, gh, gw, D = h.shape
        att, mlp = blk.attn, blk.ffn
        heads, dh = att.num_attention_heads, att.attention_head_size
        F = mlp.fc1.out_features
        if heads * dh != D or D % 8 or F % 8:
            raise ValueError("ViT block: hidden size must equal heads * head size, multiples of 8")
        N, dev = gh * gw, h.device
        pk = get_packset(blk, (dtype, param_key(blk)), lambda ps: _vit_packs(ps, blk, dtype, D, F))
        KD = rup(D, KA)
        y1, mr1 = _ln_forward(dtype, h, blk.attention_norm, (B, gh, gw, D))
        qkv = _gemm_1x1(dtype, y1, pk["Wqkv"], KD, 3 * D, torch.empty((B, gh, gw, 3 * D), dtype=dtype, device=dev),
                        bias=pk["bqkv"])
        scale = 1.0 / math.sqrt(dh)
        flash = None
        probs = None
        if p_attn > 0:
            # attn_dropout on the probabilities (:151): materialised-score path, mask regenerated
            # in the backward from (rng, site + 3)
            cx = torch.empty((B, gh, gw, D), dtype=dtype, device=dev)
            probs = _f32((B * heads * N * N,), dev)
            lse = None
            call("dfcsa_mha_drop_fwd", dt(dtype), B, N, heads, dh, 3 * D, scale, P(qkv), float(p_attn), P(rng),
                 site + 3, P(probs), P(cx), stream())
        elif _flash_mha(dtype, dh):
            cx, flash = mha_flash_forward(dtype, qkv, B, N, heads, dh)
            cx = cx.view(B, gh, gw, D)
            lse = None
        else:
            cx = torch.empty((B, gh, gw, D), dtype=dtype, device=dev)
            lse = _f32((B * heads * N,), dev)
            call("dfcsa_mha_fwd", dt(dtype), B, N, heads, dh, 3 * D, scale, P(qkv), P(cx), P(lse), stream())
        a = _gemm_1x1(dtype, cx, pk["Wo"], KD, D, torch.empty((B, gh, gw, D), dtype=dtype, device=dev),
                      bias=att.out.bias)
        h1 = _f32((B, gh, gw, D), dev)
        call("dfcsa_drop_add_fwd", dt(dtype), a.numel(), P(a), None, 0, P(h), float(p_attn), P(rng), site, P(h1),
             stream())
        del a
        y2, mr2 = _ln_forward(dtype, h1, blk.ffn_norm, (B, gh, gw, D))
        f = _gemm_1x1(dtype, y2, pk["W1"], KD, F, torch.empty((B, gh, gw, F), dtype=dtype, device=dev),
                      bias=mlp.fc1.bias)
        g = torch.empty_like(f)
        call("dfcsa_gelu_drop_fwd", dt(dtype), f.numel(), P(f), float(p), P(rng), site + 1, P(g), stream())
        m = _gemm_1x1(dtype, g, pk["W2"], rup(F, KA), D, torch.empty((B, gh, gw, D), dtype=dtype, device=dev),
                      bias=mlp.fc2.bias)
        out = _f32((B, gh, gw, D), dev)
        call("dfcsa_drop_add_fwd", dt(dtype), m.numel(), P(m), None, 0, P(h1), float(p), P(rng), site + 2, P(out),
             stream())
        ctx.blk, ctx.dtype, ctx.pk, ctx.np = blk, dtype, pk, len(params)
        ctx.cfg = (p, p_attn, rng, site, heads, dh, scale, F)
        ctx.t = (h, y1, mr1, qkv, cx, lse, h1, y2, mr2, f, g)
        ctx.flash = flash
        ctx.probs = probs
        return out

    @staticmethod
    def backward(ctx, dout):
        blk, dtype, pk = ctx.blk, ctx.dtype, ctx.pk
        p, p_attn, rng, site, heads, dh, scale, F = ctx.cfg
        h, y1, mr1, qkv, cx, lse, h1, y2, mr2, f, g = ctx.t
        att, mlp = blk.attn, blk.ffn
        B, gh, gw, D = h.shape
        N, dev = gh * gw, h.device
        grid, hw = (B, gh, gw), (gh, gw)
        KD, KF = rup(D, KA), rup(F, KA)
        dout = dout.contiguous()
        # ---- MLP half: out = drop(fc2(drop(gelu(fc1(LN2 h1))))) + h1
        M = B * N
        dm = torch.empty((B, gh, gw, D), dtype=dtype, device=dev)
        # the dropout backward also forms the fc2 bias gradient's column partials (dfcsa_drop_bwd_cs)
        pm = _drop_bwd_cs(dtype, M, D, dout, p, rng, site + 2, dm)
        with side_or_main(dev, dm, g, pm):
            _wgrad_1x1(dtype, dm, g, grid, hw, grad_of(mlp.fc2.weight))
            _colsum_rows_into(pm, M, D, grad_of(mlp.fc2.bias))
        dg = _gemm_1x1(dtype, dm, pk["W2t"], KD, F, torch.empty_like(f))
        del dm
        df = torch.empty_like(f)
        pf = _drop_bwd_cs(dtype, M, F, dg, p, rng, site + 1, df, x=f)
        del dg
        with side_or_main(dev, df, y2, pf):
            _wgrad_1x1(dtype, df, y2, grid, hw, grad_of(mlp.fc1.weight))
            _colsum_rows_into(pf, M, F, grad_of(mlp.fc1.bias))
        dy2 = _gemm_1x1(dtype, df, pk["W1t"], KF, D, torch.empty((B, gh, gw, D), dtype=dtype, device=dev))
        del df
        dh1 = _ln_backward(dtype, dy2, h1, mr2, blk.ffn_norm, dout)
        # ---- attention half: h1 = drop(out_proj(MHA(qkv(LN1 h)))) + h
        da = torch.empty((B, gh, gw, D), dtype=dtype, device=dev)
        pa = _drop_bwd_cs(dtype, M, D, dh1, p_attn, rng, site, da)
        with side_or_main(dev, da, cx, pa):
            _wgrad_1x1(dtype, da, cx, grid, hw, grad_of(att.out.weight))
            _colsum_rows_into(pa, M, D, grad_of(att.out.bias))
        dcx = _gemm_1x1(dtype, da, pk["Wot"], KD, D, torch.empty_like(cx))
        del da
        if ctx.probs is not None:
            dqkv = torch.empty_like(qkv)
            dscores = _f32((B * heads * N * N,), dev)
            call("dfcsa_mha_drop_bwd", dt(dtype), B, N, heads, dh, 3 * D, scale, P(qkv), P(dcx), P(ctx.probs),
                 float(p_attn), P(rng), site + 3, P(dscores), P(dqkv), stream())
            ctx.probs = None
            del dscores
        elif ctx.flash is not None:
            dqkv = mha_flash_backward(dtype, ctx.flash, dcx, B, N, heads, dh).view_as(qkv)
            ctx.flash = None
        else:
            dqkv = torch.empty_like(qkv)
            dvec = _f32((B * heads * N,), dev)
            call("dfcsa_mha_bwd", dt(dtype), B, N, heads, dh, 3 * D, scale, P(qkv), P(cx), P(dcx), P(lse), P(dvec),
                 P(dqkv), stream())
        del dcx
        with side_or_main(dev, dqkv, y1):
            ops.conv_wgrad_into(dtype, [dqkv], 3 * D, [(y1, 0, 0)], D, grid, hw,
                                [grad_of(att.query.weight), grad_of(att.key.weight), grad_of(att.value.weight)],
                                1, D, D, layout=2)
            channel_sum3_into(dtype, dqkv, D, D, grad_of(att.query.bias), grad_of(att.key.bias),
                              grad_of(att.value.bias))
        dy1 = _gemm_1x1(dtype, dqkv, pk["Wqkvt"], rup(3 * D, KA), D, torch.empty((B, gh, gw, D), dtype=dtype,
                                                                                  device=dev))
        del dqkv
        dx = _ln_backward(dtype, dy1, h, mr1, blk.attention_norm, dh1)
        ctx.t = None
        return (dx, None, None, None, None, None, None, *([None] * ctx.np))


class LayerNormOut(torch.autograd.Function):
    """encoder_norm (:226, :236): fp32 token grid -> dtype (the decoder's GEMM operand)."""

    @staticmethod
    def forward(ctx, h, ln, dtype, *params):
        y, mr = _ln_forward(dtype, h, ln, h.shape)
        ctx.ln, ctx.dtype, ctx.np, ctx.h, ctx.mr = ln, dtype, len(params), h, mr
        return y

    @staticmethod
    def backward(ctx, dy):
        dx = _ln_backward(ctx.dtype, dy.contiguous(), ctx.h, ctx.mr, ctx.ln, None)
        ctx.h = None
        return (dx, None, None, *([None] * ctx.np))


# ------------------------------------------------------------------ decoder plumbing
class Upsample2x(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        B, H, W, C = x.shape
        out = torch.empty((B, 2 * H, 2 * W, C), dtype=dtype, device=x.device)
        call("dfcsa_upsample2_ac", dt(dtype), B, C, H, W, P(x), P(out), stream())
        ctx.shape, ctx.dtype = x.shape, dtype
        return out

    @staticmethod
    def backward(ctx, g):
        B, H, W, C = ctx.shape
        dx = torch.empty(ctx.shape, dtype=ctx.dtype, device=g.device)
        call("dfcsa_upsample2_ac_bwd", dt(ctx.dtype), B, C, H, W, P(g.contiguous()), P(dx), stream())
        return dx, None


class ConcatC(torch.autograd.Function):
    """torch.cat([a, b], 1) in NHWC (channels last), used when the widths differ."""

    @staticmethod
    def forward(ctx, a, b, dtype):
        B, H, W, Ca = a.shape
        Cb = b.shape[-1]
        out = torch.empty((B, H, W, Ca + Cb), dtype=dtype, device=a.device)
        es, M = out.element_size(), B * H * W
        call("dfcsa_copy_cols", dt(dtype), M, Ca, P(a), Ca, P(out), Ca + Cb, 0, stream())
        call("dfcsa_copy_cols", dt(dtype), M, Cb, P(b), Cb, out.data_ptr() + Ca * es, Ca + Cb, 0, stream())
        ctx.shapes, ctx.dtype = (a.shape, b.shape), dtype
        return out

    @staticmethod
    def backward(ctx, g):
        sa, sb = ctx.shapes
        g = g.contiguous()
        Ca, Cb = sa[-1], sb[-1]
        M, es = g.numel() // (Ca + Cb), g.element_size()
        da = torch.empty(sa, dtype=ctx.dtype, device=g.device)
        db = torch.empty(sb, dtype=ctx.dtype, device=g.device)
        call("dfcsa_copy_cols", dt(ctx.dtype), M, Ca, P(g), Ca + Cb, P(da), Ca, 0, stream())
        call("dfcsa_copy_cols", dt(ctx.dtype), M, Cb, g.data_ptr() + Ca * es, Ca + Cb, P(db), Cb, 0, stream())
        return da, db, None


class UpsampleAC(torch.autograd.Function):
    """nn.UpsamplingBilinear2d(scale_factor) (align_corners=True) of fp32 NCHW logits: the
    SegmentationHead's upsampling > 1 (:272-276).  Output size floor(H * s) as F.interpolate."""

    @staticmethod
    def forward(ctx, x, scale):
        x = x.contiguous()
        B, C, H, W = x.shape
        Ho, Wo = int(math.floor(H * float(scale))), int(math.floor(W * float(scale)))
        out = _f32((B, C, Ho, Wo), x.device)
        call("dfcsa_upsample_ac_f32", B * C, H, W, Ho, Wo, P(x), P(out), stream())
        ctx.geom = (B, C, H, W, Ho, Wo)
        return out

    @staticmethod
    def backward(ctx, g):
        B, C, H, W, Ho, Wo = ctx.geom
        dx = _f32((B, C, H, W), g.device)
        call("dfcsa_upsample_ac_f32_bwd", B * C, H, W, Ho, Wo, P(g.contiguous()), P(dx), stream())
        return dx, None


class SegHead3x3(torch.autograd.Function):
    """SegmentationHead (:272-276): conv 3x3 (+bias, padding 1) -> logits NCHW fp32; upsampling 1."""

    @staticmethod
    def forward(ctx, x, conv, dtype, *params):
        B, H, W, C = x.shape
        Cout = conv.out_channels
        if conv.kernel_size != (3, 3) or conv.padding != (1, 1) or conv.in_channels != C:
            raise ValueError("segmentation head: 3x3/p1 conv over the decoder channels")
        logits = _f32((B, Cout, H, W), x.device)
        call("dfcsa_head3_fwd", dt(dtype), B, H, W, C, Cout, P(x), P(conv.weight), P(conv.bias), P(logits), stream())
        ctx.conv, ctx.dtype, ctx.np, ctx.x = conv, dtype, len(params), x
        return logits

    @staticmethod
    def backward(ctx, g):
        x, conv, dtype = ctx.x, ctx.conv, ctx.dtype
        B, H, W, C = x.shape
        Cout = conv.out_channels
        nt = LIB.dfcsa_head3_ntiles(B, H, W)
        pw = _f32((nt * Cout * C * 9,), x.device)
        pb = _f32((nt * Cout,), x.device)
        dx = torch.empty_like(x)
        call("dfcsa_head3_bwd", dt(dtype), B, H, W, C, Cout, P(x), P(conv.weight), P(g.contiguous()), P(dx), P(pw),
             P(pb), stream())
        ops.colsum_into(pw, nt, Cout * C * 9, grad_of(conv.weight))
        ops.colsum_into(pb, nt, Cout, grad_of(conv.bias))
        ctx.x = None
        return (dx if ctx.needs_input_grad[0] else None, None, None, *([None] * ctx.np))
