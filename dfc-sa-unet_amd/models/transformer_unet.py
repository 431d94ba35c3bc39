"""TransUNet R50-ViT-B/16 (reference models/transformer_unet.py; config_transunet.yaml = BASELINE
config 4) on the MI355X kernels.

Module tree, parameter creation order and state_dict keys are the reference's (so a seeded
construction gives its initial weights and checkpoints interoperate), and ``get_r50_b16_config``
returns the same hyper-parameters (``ml_collections`` is replaced by a small attribute dict).
The forward runs NHWC through dfcsa/transunet_ops.py:

  ResNetV2 hybrid stem (:70-106)   RootStem (StdConv 7x7/s2 + GN + ReLU), MaxPool3x3s2, Bottleneck
                                   units (StdConv 1x1/3x3/1x1 + GroupNorms, projection residuals);
                                   all convs are implicit GEMMs on standardised weights
  Embeddings (:175-200)            PatchEmbed: 1x1 conv GEMM + position embeddings + dropout
  Encoder (:222-237)               ViTBlock x L (fused q|k|v GEMM, multi-head attention kernels,
                                   erf-GELU MLP), LayerNormOut; residual stream fp32
  DecoderCup (:278-312)            conv_more + DecoderBlocks (bilinear x2 align_corners, skip concat
                                   as GEMM source segments, Conv2d + BatchNorm + ReLU x 2)
  SegmentationHead (:272-276)      SegHead3x3 -> NCHW fp32 logits

Dropout (rate 0.1 in the stock config) uses counter-based masks on the device (statistically
equivalent to nn.Dropout, not the same random stream); attention-probability dropout (0 in the
reference config) runs for p > 0 on materialised-score kernels (dfcsa_mha_drop_fwd/bwd, N = 196)
with the mask regenerated from the same counter-based key in the backward.
"""
import torch
import torch.nn as nn
from torch.nn.modules.utils import _pair

import dfcsa
from dfcsa import packs
from dfcsa._lib import call
from dfcsa.flat import ALIGN, FlatParams
from dfcsa.ops import P, rup, stream
from dfcsa.transunet_ops import (Bottleneck, ConcatC, ConvBNReLU, LayerNormOut, MaxPool3x3s2, PatchEmbed, RootStem,
                                 SegHead3x3, StdWeights, Upsample2x, UpsampleAC, ViTBlock)


class ConfigDict(dict):
    """Attribute access over a dict (the subset of ml_collections.ConfigDict the reference uses)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def get_r50_b16_config():
    """R50 + ViT-B/16 hyper-parameters (reference :318-342)."""
    c = ConfigDict()
    c.patches = ConfigDict(grid=(14, 14))
    c.resnet = ConfigDict(num_layers=(3, 4, 9), width_factor=1)
    c.hidden_size = 768
    c.transformer = ConfigDict(mlp_dim=3072, num_heads=12, num_layers=12, attention_dropout_rate=0.0,
                               dropout_rate=0.1)
    c.classifier = "seg"
    c.decoder_channels = (256, 128, 64, 16)
    c.skip_channels = [512, 256, 64, 16]
    c.n_classes = 9
    c.n_skip = 3
    c.activation = "softmax"
    return c


# ------------------------------------------------------------------ ResNetV2 (:16-106)
class StdConv2d(nn.Conv2d):
    """Weight-standardised conv (:21-27); standardisation runs in the model-wide StdWeights launch."""


def conv1x1(cin, cout, stride=1, bias=False):
    return StdConv2d(cin, cout, kernel_size=1, stride=stride, padding=0, bias=bias)


def conv3x3(cin, cout, stride=1, groups=1, bias=False):
    return StdConv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=bias, groups=groups)


class PreActBottleneck(nn.Module):
    def __init__(self, cin, cout=None, cmid=None, stride=1):
        super().__init__()
        cout = cout or cin
        cmid = cmid or cout // 4
        self.gn1 = nn.GroupNorm(32, cmid, eps=1e-6)
        self.conv1 = conv1x1(cin, cmid, bias=False)
        self.gn2 = nn.GroupNorm(32, cmid, eps=1e-6)
        self.conv2 = conv3x3(cmid, cmid, stride, bias=False)
        self.gn3 = nn.GroupNorm(32, cout, eps=1e-6)
        self.conv3 = conv1x1(cmid, cout, bias=False)
        self.relu = nn.ReLU(inplace=True)
        if stride != 1 or cin != cout:
            self.downsample = conv1x1(cin, cout, stride, bias=False)
            self.gn_proj = nn.GroupNorm(cout, cout)


class ResNetV2(nn.Module):
    def __init__(self, block_units, width_factor):
        super().__init__()
        width = int(64 * width_factor)
        self.width = width
        self.root = nn.Sequential()
        self.root.add_module("conv", StdConv2d(3, width, kernel_size=7, stride=2, bias=False, padding=3))
        self.root.add_module("gn", nn.GroupNorm(32, width, eps=1e-6))
        self.root.add_module("relu", nn.ReLU(inplace=True))
        self.body = nn.Sequential()
        spec = ((width, width * 4, width, 1), (width * 4, width * 8, width * 2, 2), (width * 8, width * 16, width * 4, 2))
        for bi, (units, (cin, cout, cmid, stride)) in enumerate(zip(block_units, spec)):
            blk = nn.Sequential()
            blk.add_module("unit1", PreActBottleneck(cin=cin, cout=cout, cmid=cmid, stride=stride))
            for i in range(2, units + 1):
                blk.add_module(f"unit{i}", PreActBottleneck(cin=cout, cout=cout, cmid=cmid))
            self.body.add_module(f"block{bi + 1}", blk)

    def forward_nhwc(self, x, dtype, model):
        """x NCHW fp32 -> (NHWC stem output, [block2 out, block1 out, root out]) (:97-106)."""
        h = RootStem.apply(x, self.root, dtype, model, *self.root.parameters())
        feats = [h]
        h = MaxPool3x3s2.apply(h, dtype)
        blocks = list(self.body.children())
        for i, blk in enumerate(blocks):
            for unit in blk.children():
                h = Bottleneck.apply(h, unit, dtype, *unit.parameters())
            if i < len(blocks) - 1:
                feats.append(h)
        return h, feats[::-1]


# ------------------------------------------------------------------ ViT (:111-248)
class Attention(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.num_attention_heads = config.transformer["num_heads"]
        self.attention_head_size = int(config.hidden_size / self.num_attention_heads)
        self.all_head_size = self.num_attention_heads * self.attention_head_size
        self.query = nn.Linear(config.hidden_size, self.all_head_size)
        self.key = nn.Linear(config.hidden_size, self.all_head_size)
        self.value = nn.Linear(config.hidden_size, self.all_head_size)
        self.out = nn.Linear(config.hidden_size, config.hidden_size)
        self.attn_dropout = nn.Dropout(config.transformer["attention_dropout_rate"])
        self.proj_dropout = nn.Dropout(config.transformer["attention_dropout_rate"])
        self.softmax = nn.Softmax(dim=-1)


class Mlp(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.fc1 = nn.Linear(config.hidden_size, config.transformer["mlp_dim"])
        self.fc2 = nn.Linear(config.transformer["mlp_dim"], config.hidden_size)
        self.dropout = nn.Dropout(config.transformer["dropout_rate"])


class Embeddings(nn.Module):
    def __init__(self, config, img_size, in_channels=3):
        super().__init__()
        self.config = config
        img_size = _pair(img_size)
        grid_size = config.patches["grid"]
        patch_size = (img_size[0] // 16 // grid_size[0], img_size[1] // 16 // grid_size[1])
        n_patches = (img_size[0] // 16) * (img_size[1] // 16)
        self.hybrid_model = ResNetV2(block_units=config.resnet.num_layers, width_factor=config.resnet.width_factor)
        in_channels = self.hybrid_model.width * 16
        self.patch_embeddings = nn.Conv2d(in_channels=in_channels, out_channels=config.hidden_size,
                                          kernel_size=patch_size, stride=patch_size)
        self.position_embeddings = nn.Parameter(torch.zeros(1, n_patches, config.hidden_size))
        self.dropout = nn.Dropout(config.transformer["dropout_rate"])


class Block(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.hidden_size = config.hidden_size
        self.attention_norm = nn.LayerNorm(config.hidden_size, eps=1e-6)
        self.ffn_norm = nn.LayerNorm(config.hidden_size, eps=1e-6)
        self.ffn = Mlp(config)
        self.attn = Attention(config)


class Encoder(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.layer = nn.ModuleList()
        self.encoder_norm = nn.LayerNorm(config.hidden_size, eps=1e-6)
        for _ in range(config.transformer["num_layers"]):
            self.layer.append(Block(config))


class Transformer(nn.Module):
    def __init__(self, config, img_size):
        super().__init__()
        self.embeddings = Embeddings(config, img_size=img_size)
        self.encoder = Encoder(config)


# ------------------------------------------------------------------ decoder (:250-312)
class Conv2dReLU(nn.Sequential):
    def __init__(self, in_channels, out_channels, kernel_size, padding=0, stride=1, use_batchnorm=True):
        conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                         bias=not use_batchnorm)
        relu = nn.ReLU(inplace=True)
        bn = nn.BatchNorm2d(out_channels)
        super().__init__(conv, bn, relu)

    def forward_nhwc(self, xs, dtype):
        conv, bn = self[0], self[1]
        return ConvBNReLU.apply(conv, bn, dtype, len(xs), *xs, *conv.parameters(), *bn.parameters())


class DecoderBlock(nn.Module):
    def __init__(self, in_channels, out_channels, skip_channels=0, use_batchnorm=True):
        super().__init__()
        self.conv1 = Conv2dReLU(in_channels + skip_channels, out_channels, kernel_size=3, padding=1,
                                use_batchnorm=use_batchnorm)
        self.conv2 = Conv2dReLU(out_channels, out_channels, kernel_size=3, padding=1, use_batchnorm=use_batchnorm)
        self.up = nn.UpsamplingBilinear2d(scale_factor=2)

    def forward_nhwc(self, x, skip, dtype):
        x = Upsample2x.apply(x, dtype)
        if skip is None:
            xs = [x]
        elif skip.shape[-1] == x.shape[-1]:
            xs = [x, skip]                        # cat([x, skip]) as two GEMM source segments
        else:
            xs = [ConcatC.apply(x, skip, dtype)]
        return self.conv2.forward_nhwc([self.conv1.forward_nhwc(xs, dtype)], dtype)


class SegmentationHead(nn.Sequential):
    """conv 3x3 (+bias) then, for upsampling > 1, nn.UpsamplingBilinear2d(upsampling)
    (reference :272-276; the reference's TransUNet builds it with upsampling = 1).  Standalone
    calls take NCHW float input and run the head conv and the upsample on the HIP kernels."""

    def __init__(self, in_channels, out_channels, kernel_size=3, upsampling=1):
        conv2d = nn.Conv2d(in_channels, out_channels, kernel_size=kernel_size, padding=kernel_size // 2)
        upsampling_m = nn.UpsamplingBilinear2d(scale_factor=upsampling) if upsampling > 1 else nn.Identity()
        super().__init__(conv2d, upsampling_m)
        self.upsampling = upsampling

    def upsample(self, logits):
        """The head's upsampling stage on fp32 NCHW logits (identity at upsampling = 1)."""
        return UpsampleAC.apply(logits, self.upsampling) if self.upsampling > 1 else logits

    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("SegmentationHead runs on the MI355X kernels only; move it and its input to 'cuda'")
        conv = self[0]
        xn = x.to(torch.float32).permute(0, 2, 3, 1).contiguous()
        return self.upsample(SegHead3x3.apply(xn, conv, torch.float32, *conv.parameters()))


class DecoderCup(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        head_channels = 512
        self.conv_more = Conv2dReLU(config.hidden_size, head_channels, kernel_size=3, padding=1, use_batchnorm=True)
        decoder_channels = config.decoder_channels
        in_channels = [head_channels] + list(decoder_channels[:-1])
        out_channels = decoder_channels
        if self.config.n_skip != 0:
            skip_channels = list(self.config.skip_channels)
            for i in range(4 - self.config.n_skip):
                skip_channels[3 - i] = 0
        else:
            skip_channels = [0, 0, 0, 0]
        self.blocks = nn.ModuleList([DecoderBlock(i, o, s) for i, o, s in zip(in_channels, out_channels,
                                                                                skip_channels)])

    def forward_nhwc(self, h, features, dtype):
        x = self.conv_more.forward_nhwc([h], dtype)
        for i, blk in enumerate(self.blocks):
            skip = features[i] if (features is not None and i < self.config.n_skip) else None
            x = blk.forward_nhwc(x, skip, dtype)
        return x


# ------------------------------------------------------------------ the model (:347-368)
class TransUNet(nn.Module):
    def __init__(self, config, img_size=224, num_classes=9, zero_head=False, precision=None):
        super().__init__()
        self.num_classes = num_classes
        self.zero_head = zero_head
        self.classifier = config.classifier
        self.transformer = Transformer(config, img_size)
        self.decoder = DecoderCup(config)
        self.segmentation_head = SegmentationHead(in_channels=config.decoder_channels[-1],
                                                  out_channels=config.n_classes, kernel_size=3)
        self.config = config
        self.compute_dtype = dfcsa.resolve_dtype(precision)
        self._flat = None
        self._stdw = None
        self._rng = None

    def set_precision(self, precision):
        self.compute_dtype = dfcsa.resolve_dtype(precision)
        return self

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._flat = None
        self._stdw = None
        self._dfcsa_plan = None
        self._rng = None
        return out

    def flat_params(self):
        if self._flat is None or not self._flat.valid():
            self._flat = FlatParams(self)
        return self._flat

    def grad_units(self):
        """One data-parallel unit: StdConv2d gradients become final only in the root stem's backward
        (the last node), so the whole flat gradient buffer is one bucket."""
        flat = self.flat_params()
        return [(self, 0, rup(flat.numel, ALIGN))]

    def std_convs(self):
        return [m for m in self.modules() if isinstance(m, StdConv2d)]

    def _std_weights(self, device):
        if self._stdw is None or not self._stdw.valid():
            self._stdw = StdWeights(self.std_convs(), device)
            self._dfcsa_plan = None
        return self._stdw

    def _dropout_rng(self, device):
        if self._rng is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
            self._rng = torch.tensor([seed, 0], dtype=torch.int64, device=device)
        return self._rng

    def forward(self, x):
        """x: [B, 1|3, H, W] float -> logits [B, n_classes, H, W] fp32 (reference :362-368)."""
        if not x.is_cuda:
            raise RuntimeError("TransUNet runs on the MI355X kernels only; move model and input to 'cuda'")
        flat = self.flat_params()
        flat.attach_grads()
        dtype = self.compute_dtype
        training = self.training
        stdw = self._std_weights(x.device)
        stdw.forward(training and torch.is_grad_enabled())
        if getattr(self, "_plan_flat", None) is not flat:
            self._dfcsa_plan, self._plan_flat = None, flat
        planned = packs.sync_model_plan(self)

        emb = self.transformer.embeddings
        tcfg = self.config.transformer
        p = float(tcfg["dropout_rate"]) if training else 0.0
        # attn_dropout + proj_dropout (:139-140, :151, :156): both at attention_dropout_rate
        p_attn = float(tcfg["attention_dropout_rate"]) if training else 0.0
        rng = self._dropout_rng(x.device)
        if p > 0 or p_attn > 0:
            call("dfcsa_rng_advance", P(rng), stream())

        h, features = emb.hybrid_model.forward_nhwc(x, dtype, self)
        t = PatchEmbed.apply(h, emb, dtype, p, rng, *emb.patch_embeddings.parameters(), emb.position_embeddings)
        for i, blk in enumerate(self.transformer.encoder.layer):
            t = ViTBlock.apply(t, blk, dtype, p, p_attn, rng, 16 + 4 * i, *blk.parameters())
        enc = self.transformer.encoder.encoder_norm
        t = LayerNormOut.apply(t, enc, dtype, *enc.parameters())
        y = self.decoder.forward_nhwc(t, features, dtype)
        head = self.segmentation_head[0]
        logits = self.segmentation_head.upsample(SegHead3x3.apply(y, head, dtype, *head.parameters()))
        if not planned:
            packs.rebuild_model_plan(self, x.device)
        return logits
