"""Fusion ablations (reference models/unet_dfc_sa_ablation_fusion.py) on the MI355X kernels.

  AdditionFusionBlock  :7-49    local + attention (no gate), + res_scale * residual
  ConcatFusionBlock    :51-100  1x1 conv -> BN -> ReLU over cat[local, attention] (the concat is
                                never materialised: two GEMM sources), + res_scale * residual
  UNet_AdditionFusion / UNet_ConcatFusion  :103-109  AblationUNetBase of those blocks
"""
import torch
import torch.nn as nn

from dfcsa.ablation import SumOut, gate_inputs
from dfcsa.unet_ops import ConvBNReLU
from models.unet_dfc_sa_ablation_branches import (AblationUNetBase, _AblationBlock, _attn_branch, _conv_branch,
                                                  _residual_conv)


class AdditionFusionBlock(_AblationBlock):
    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, pool_size=8):
        super().__init__()
        self.conv_branch = _conv_branch(in_channels, out_channels)
        self.attn_branch = _attn_branch(in_channels, out_channels, pool_size)
        self.residual_conv = _residual_conv(in_channels, out_channels)
        self.res_scale = nn.Parameter(torch.tensor(0.1))

    def forward_nhwc(self, xs, dtype):
        xs = gate_inputs(self, xs)
        local = self._local(xs, dtype)
        attn = self._attention(xs, dtype)
        return SumOut.apply(dtype, self.res_scale, local, attn, self._residual(xs, dtype))


class ConcatFusionBlock(_AblationBlock):
    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, pool_size=8):
        super().__init__()
        self.conv_branch = _conv_branch(in_channels, out_channels)
        self.attn_branch = _attn_branch(in_channels, out_channels, pool_size)
        self.fusion_conv = nn.Sequential(nn.Conv2d(out_channels * 2, out_channels, kernel_size=1),
                                         nn.BatchNorm2d(out_channels), nn.ReLU(inplace=True))
        self.residual_conv = _residual_conv(in_channels, out_channels)
        self.res_scale = nn.Parameter(torch.tensor(0.1))

    def forward_nhwc(self, xs, dtype):
        xs = gate_inputs(self, xs)
        local = self._local(xs, dtype)
        attn = self._attention(xs, dtype)
        conv, bn = self.fusion_conv[0], self.fusion_conv[1]
        fused = ConvBNReLU.apply(conv, bn, dtype, 2, local, attn, *conv.parameters(), *bn.parameters())
        return SumOut.apply(dtype, self.res_scale, fused, None, self._residual(xs, dtype))


class UNet_AdditionFusion(AblationUNetBase):  # noqa: N801  (reference class names)
    def __init__(self, in_channels, out_channels, features, pool_size=8, precision=None):
        super().__init__(lambda i, o: AdditionFusionBlock(i, o, pool_size=pool_size), in_channels, out_channels,
                         features, pool_size, precision=precision)


class UNet_ConcatFusion(AblationUNetBase):  # noqa: N801
    def __init__(self, in_channels, out_channels, features, pool_size=8, precision=None):
        super().__init__(lambda i, o: ConcatFusionBlock(i, o, pool_size=pool_size), in_channels, out_channels,
                         features, pool_size, precision=precision)
