"""DFC-SA-Res U-Net on the MI355X kernels of libdfcsa.

Drop-in for the reference's models/unet_dfc_sa_res.py:
  * the module tree (attribute names, nn.Sequential indices, parameter shapes, creation order)
    is the reference's, so ``state_dict`` keys (343 for features 64..512) and the default
    initialisation under a given seed are identical -- checkpoints interoperate both ways;
  * ``forward`` runs the hand-written HIP kernels (dfcsa.block / dfcsa.functions) on NHWC
    activations in the compute dtype (bf16 by default, fp32 for parity runs) with fp32 master
    parameters, gradients and statistics.  The nn.Conv2d / nn.BatchNorm2d submodules are only
    parameter holders; their own forward is never called.

Reference classes: LightSelfAttention :5-39, DynamicFusionConvAttnBlock :41-116,
UNetDFCSA :118-204, UNetDFCSARes :207-220.
"""
import torch
import torch.nn as nn

import dfcsa
from dfcsa import chanpad, packs
from dfcsa.block import DFCBlockFunction, DFCBlockPoolFunction, LSAFunction
from dfcsa.flat import FlatParams
from dfcsa.functions import ConvTranspose2x2, Head1x1, InputToNHWC, MaxPoolFork, ResizeBilinear
from dfcsa.ops import rup


def _nchw_to_nhwc(x, dtype):
    return InputToNHWC.apply(x, dtype, rup(x.shape[1], 8))


def _nhwc_to_nchw(y, mod=None):
    """NCHW fp32 view of an NHWC output; a standalone module padded by chanpad.pad_standalone returns
    its logical channels only."""
    y = y.permute(0, 3, 1, 2).float()
    c = getattr(mod, "_dfcsa_out", None)
    return y if c is None else y[:, :c]


class LightSelfAttention(nn.Module):
    """Pooled self-attention (reference :5-39).  Parameters: query/key (C -> C // ratio),
    value (C -> C) 1x1 convs and a scalar gamma initialised to 0."""

    def __init__(self, channels, pool_size=8, ablation_on_qk_channels=8):
        super().__init__()
        self.pool_size = pool_size
        reduced = channels // ablation_on_qk_channels
        self.query_conv = nn.Conv2d(channels, reduced, kernel_size=1)
        self.key_conv = nn.Conv2d(channels, reduced, kernel_size=1)
        self.value_conv = nn.Conv2d(channels, channels, kernel_size=1)
        self.gamma = nn.Parameter(torch.zeros(1))
        self.compute_dtype = torch.bfloat16
        if chanpad.standalone():
            chanpad.pad_standalone(self, channels, channels)

    def forward(self, x):
        """x: [B, C, H, W] (any values) -> gamma * up(attn(pool(x))) + x, NCHW fp32."""
        xh = _nchw_to_nhwc(x, self.compute_dtype)
        y = LSAFunction.apply(self, self.pool_size, self.compute_dtype, xh, *self.parameters())
        return _nhwc_to_nchw(y, self)


class DynamicFusionConvAttnBlock(nn.Module):
    """DFC block (reference :41-116): 3x3 conv branch, 1x1 -> pooled self-attention branch,
    sigmoid fusion gate, 1x1 fusion conv, scaled 1x1 residual."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, pool_size=8,
                 ablation_on_qk_channels=8):
        super().__init__()
        if kernel_size != 3 or stride != 1 or padding != 1:
            raise NotImplementedError("the DFC block kernels implement the reference's 3x3/s1/p1 local branch")
        with chanpad.building():   # the attention module is padded with the block
            self._build(in_channels, out_channels, pool_size, ablation_on_qk_channels)
        if chanpad.standalone():
            chanpad.pad_standalone(self, in_channels, out_channels)

    def _build(self, in_channels, out_channels, pool_size, ablation_on_qk_channels):
        self.pool_size = pool_size
        self.conv_branch = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, kernel_size=3, stride=1, padding=1),
            nn.BatchNorm2d(out_channels), nn.ReLU(inplace=True))
        self.attn_branch = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, kernel_size=1),
            nn.BatchNorm2d(out_channels), nn.ReLU(inplace=True),
            self._make_attention(out_channels, pool_size, ablation_on_qk_channels))
        self.gate = nn.Sequential(
            nn.Conv2d(out_channels * 2, out_channels, kernel_size=1),
            nn.BatchNorm2d(out_channels), nn.Sigmoid())
        self.fusion_conv = nn.Sequential(
            nn.Conv2d(out_channels * 3, out_channels, kernel_size=1),
            nn.BatchNorm2d(out_channels), nn.ReLU(inplace=True))
        if in_channels != out_channels:
            self.residual_conv = nn.Conv2d(in_channels, out_channels, kernel_size=1, bias=False)
        else:
            self.residual_conv = nn.Identity()
        self.res_scale = nn.Parameter(torch.tensor(0.1))
        self.compute_dtype = torch.bfloat16

    def _make_attention(self, channels, pool_size, ablation_on_qk_channels):
        """The attention module of the branch (subclasses swap it; created in the reference's order)."""
        return LightSelfAttention(channels, pool_size=pool_size, ablation_on_qk_channels=ablation_on_qk_channels)

    def forward_nhwc(self, xs, dtype):
        """xs: list of NHWC sources whose channel concat is the block input (skip concat
        never materialised)."""
        return DFCBlockFunction.apply(self, self.pool_size, dtype, len(xs), *xs, *self.parameters())

    def forward_nhwc_pool(self, xs, dtype):
        """Encoder use: (MaxPool2d(2,2)(out), out) with the pooling fused into the block."""
        return DFCBlockPoolFunction.apply(self, self.pool_size, dtype, len(xs), *xs, *self.parameters())

    def forward(self, x):
        """Standalone use on NCHW fp32 input (returns NCHW fp32)."""
        y = self.forward_nhwc([_nchw_to_nhwc(x, self.compute_dtype)], self.compute_dtype)
        return _nhwc_to_nchw(y, self)


class UNetDFCSA(nn.Module):
    """U-Net of DFC blocks (reference :118-204): 4 encoder blocks + 2x2 max pooling, a 2x-wide
    bottleneck block, 4 x (ConvTranspose2d k2 s2 -> [bilinear fix] -> concat skip -> block),
    1x1 head.  ``precision`` selects the activation dtype ('bf16' default, 'fp32')."""

    def __init__(self, in_channels=3, out_channels=1, features=(64, 128, 256, 512), pool_size=8,
                 ablation_on_qk_channels=8, precision=None):
        super().__init__()
        f = list(features)
        # blocks built here are padded by pad_model below, not by themselves (chanpad.pad_standalone)
        blk = lambda i, o: chanpad.build_inside(self._make_block, i, o, pool_size, ablation_on_qk_channels)  # noqa: E731
        self.pool_size = pool_size
        self.in_channels = in_channels
        self.down1 = blk(in_channels, f[0])
        self.pool1 = nn.MaxPool2d(kernel_size=2, stride=2)
        self.down2 = blk(f[0], f[1])
        self.pool2 = nn.MaxPool2d(kernel_size=2, stride=2)
        self.down3 = blk(f[1], f[2])
        self.pool3 = nn.MaxPool2d(kernel_size=2, stride=2)
        self.down4 = blk(f[2], f[3])
        self.pool4 = nn.MaxPool2d(kernel_size=2, stride=2)
        self.bottleneck = blk(f[3], f[3] * 2)
        self.up4 = nn.ConvTranspose2d(f[3] * 2, f[3], kernel_size=2, stride=2)
        self.up_conv4 = blk(f[3] * 2, f[3])
        self.up3 = nn.ConvTranspose2d(f[3], f[2], kernel_size=2, stride=2)
        self.up_conv3 = blk(f[2] * 2, f[2])
        self.up2 = nn.ConvTranspose2d(f[2], f[1], kernel_size=2, stride=2)
        self.up_conv2 = blk(f[1] * 2, f[1])
        self.up1 = nn.ConvTranspose2d(f[1], f[0], kernel_size=2, stride=2)
        self.up_conv1 = blk(f[0] * 2, f[0])
        self.final_conv = nn.Conv2d(f[0], out_channels, kernel_size=1)
        self.compute_dtype = dfcsa.resolve_dtype(precision)
        self._flat = None
        if any(c % 8 for c in f):
            # widths the 16-byte channel chunks cannot address: zero-pad every channel dimension
            # after the reference's construction (same init); state_dict stays logical (chanpad)
            chanpad.pad_model(self, f, in_channels, out_channels)

    def _make_block(self, in_channels, out_channels, pool_size, ablation_on_qk_channels):
        """Block factory (AblationUNetBase's block_func, unet_dfc_sa_ablation_branches.py:105)."""
        return DynamicFusionConvAttnBlock(in_channels, out_channels, kernel_size=3, stride=1, padding=1,
                                          pool_size=pool_size, ablation_on_qk_channels=ablation_on_qk_channels)

    # -------------------------------------------------------------- precision / storage
    def set_precision(self, precision):
        self.compute_dtype = dfcsa.resolve_dtype(precision)
        return self

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._flat = None  # parameters moved: re-flatten lazily on the next forward
        self._dfcsa_plan = None
        return out

    def flat_params(self):
        """The FlatParams storage of this model (created on first use, on the params' device)."""
        if self._flat is None or not self._flat.valid():
            self._flat = FlatParams(self)
        return self._flat

    def grad_units(self):
        """[(module, lo, hi)]: the modules whose backward finalises a contiguous range of the flat
        gradient buffer, in buffer order (used by the data-parallel bucket reducer)."""
        from dfcsa.flat import ALIGN
        flat = self.flat_params()
        index = {id(p): i for i, p in enumerate(flat.params)}
        units = []
        for mod in (self.down1, self.down2, self.down3, self.down4, self.bottleneck, self.up4, self.up_conv4,
                    self.up3, self.up_conv3, self.up2, self.up_conv2, self.up1, self.up_conv1, self.final_conv):
            ps = list(mod.parameters())
            first, last = index[id(ps[0])], index[id(ps[-1])]
            units.append((mod, flat.offsets[first], flat.offsets[last] + rup(ps[-1].numel(), ALIGN)))
        return units

    # -------------------------------------------------------------- forward
    def forward(self, x):
        """x: [B, in_channels, H, W] float -> logits [B, out_channels, H, W] fp32 (no sigmoid)."""
        if not x.is_cuda:
            raise RuntimeError("UNetDFCSARes runs on the MI355X kernels only; move model and input to 'cuda'")
        flat = self.flat_params()
        if torch.is_grad_enabled():
            flat.attach_grads()
        dt = self.compute_dtype
        if getattr(self, "_plan_flat", None) is not flat:  # parameter storage changed: stale plan
            self._dfcsa_plan, self._plan_flat = None, flat
        planned = packs.sync_model_plan(self)  # one launch packs every conv operand of the model
        h = _nchw_to_nhwc(x, dt)

        def enc(blk, t):
            """encoder block + MaxPool2d(2,2) (:165-172) -> (pooled, skip); DFC blocks fuse the pooling
            into their block-output pass, other (ablation) blocks pool through MaxPoolFork"""
            if isinstance(blk, DynamicFusionConvAttnBlock):
                return blk.forward_nhwc_pool([t], dt)
            return MaxPoolFork.apply(blk.forward_nhwc([t], dt), dt)
        p1, d1 = enc(self.down1, h)
        p2, d2 = enc(self.down2, p1)
        p3, d3 = enc(self.down3, p2)
        p4, d4 = enc(self.down4, p3)
        u = self.bottleneck.forward_nhwc([p4], dt)
        for up, block, skip in ((self.up4, self.up_conv4, d4), (self.up3, self.up_conv3, d3),
                                (self.up2, self.up_conv2, d2), (self.up1, self.up_conv1, d1)):
            u = ConvTranspose2x2.apply(u, up, dt, *up.parameters())
            if u.shape[1:3] != skip.shape[1:3]:
                u = ResizeBilinear.apply(u, tuple(skip.shape[1:3]), dt)
            u = block.forward_nhwc([u, skip], dt)  # cat([up, skip]) order, never materialised
        logits = Head1x1.apply(u, self.final_conv, dt, *self.final_conv.parameters())
        if not planned:
            packs.rebuild_model_plan(self, x.device)
        return logits


class UNetDFCSARes(UNetDFCSA):
    """Reference :207-220 -- identical to UNetDFCSA (the residual lives inside each block)."""

    def __init__(self, in_channels=3, out_channels=1, features=(64, 128, 256, 512), pool_size=8,
                 ablation_on_qk_channels=8, precision=None):
        super().__init__(in_channels, out_channels, features, pool_size, ablation_on_qk_channels, precision)
