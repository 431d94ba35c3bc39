"""Branch ablations (reference models/unet_dfc_sa_ablation_branches.py) on the MI355X kernels.

  LocalOnlyBlock      :73-101   3x3 conv -> BN -> ReLU, + res_scale * residual (1x1 or identity)
  AttentionOnlyBlock  :42-70    1x1 conv -> BN -> ReLU -> LightSelfAttention, + res_scale * residual
  AblationUNetBase    :104-164  the U-Net of UNetDFCSA with a block factory
  UNet_Baseline       :166-168  LocalOnlyBlock everywhere (pool_size unused, as in the reference)
  UNet_AttentionOnly  :170-172  AttentionOnlyBlock everywhere

Module trees, parameter creation order and state_dict keys are the reference's (LightSelfAttention
with channels // 8 query/key width, as the reference's copy in this file has).  Blocks run on NHWC
activations through dfcsa.unet_ops.ConvBNReLU, dfcsa.block.LSAFunction and dfcsa.ablation.
"""
import torch
import torch.nn as nn

from dfcsa.ablation import Conv1x1, SumOut, gate_inputs
from dfcsa.block import LSAFunction
from dfcsa.unet_ops import ConvBNReLU
from models.unet_dfc_sa_res import LightSelfAttention, UNetDFCSA, _nchw_to_nhwc, _nhwc_to_nchw


class _AblationBlock(nn.Module):
    """Shared pieces: the residual path and standalone NCHW use."""

    def _residual(self, xs, dtype):
        if isinstance(self.residual_conv, nn.Identity):
            if len(xs) != 1:
                raise ValueError("identity residual needs a single source with out_channels channels")
            return xs[0]
        return Conv1x1.apply(self.residual_conv, dtype, len(xs), *xs, *self.residual_conv.parameters())

    def _local(self, xs, dtype):
        conv, bn = self.conv_branch[0], self.conv_branch[1]
        return ConvBNReLU.apply(conv, bn, dtype, len(xs), *xs, *conv.parameters(), *bn.parameters())

    def _attention(self, xs, dtype):
        conv, bn, lsa = self.attn_branch[0], self.attn_branch[1], self.attn_branch[3]
        a = ConvBNReLU.apply(conv, bn, dtype, len(xs), *xs, *conv.parameters(), *bn.parameters())
        return LSAFunction.apply(lsa, lsa.pool_size, dtype, a, *lsa.parameters())

    def forward(self, x):
        dtype = torch.bfloat16
        y = self.forward_nhwc([_nchw_to_nhwc(x, dtype)], dtype)
        return _nhwc_to_nchw(y)


def _residual_conv(in_channels, out_channels):
    if in_channels != out_channels:
        return nn.Conv2d(in_channels, out_channels, kernel_size=1, bias=False)
    return nn.Identity()


def _attn_branch(in_channels, out_channels, pool_size):
    return nn.Sequential(nn.Conv2d(in_channels, out_channels, kernel_size=1), nn.BatchNorm2d(out_channels),
                         nn.ReLU(inplace=True), LightSelfAttention(out_channels, pool_size=pool_size))


def _conv_branch(in_channels, out_channels):
    return nn.Sequential(nn.Conv2d(in_channels, out_channels, kernel_size=3, stride=1, padding=1),
                         nn.BatchNorm2d(out_channels), nn.ReLU(inplace=True))


class AttentionOnlyBlock(_AblationBlock):
    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, pool_size=8):
        super().__init__()
        self.attn_branch = _attn_branch(in_channels, out_channels, pool_size)
        self.residual_conv = _residual_conv(in_channels, out_channels)
        self.res_scale = nn.Parameter(torch.tensor(0.1))

    def forward_nhwc(self, xs, dtype):
        xs = gate_inputs(self, xs)
        attn = self._attention(xs, dtype)
        return SumOut.apply(dtype, self.res_scale, attn, None, self._residual(xs, dtype))


class LocalOnlyBlock(_AblationBlock):
    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, **kwargs):
        super().__init__()
        if kernel_size != 3 or stride != 1 or padding != 1:
            raise NotImplementedError("the local branch kernels implement the reference's 3x3/s1/p1 conv")
        self.conv_branch = _conv_branch(in_channels, out_channels)
        self.residual_conv = _residual_conv(in_channels, out_channels)
        self.res_scale = nn.Parameter(torch.tensor(0.1))

    def forward_nhwc(self, xs, dtype):
        xs = gate_inputs(self, xs)
        local = self._local(xs, dtype)
        return SumOut.apply(dtype, self.res_scale, local, None, self._residual(xs, dtype))


class AblationUNetBase(UNetDFCSA):
    """Reference :104-164: UNetDFCSA's tree and forward with ``block_func(in, out)`` blocks."""

    def __init__(self, block_func, in_channels, out_channels, features, pool_size=8, precision=None):
        self._block_func = block_func
        super().__init__(in_channels, out_channels, features, pool_size=pool_size, precision=precision)

    def _make_block(self, in_channels, out_channels, pool_size, ablation_on_qk_channels):
        return self._block_func(in_channels, out_channels)


class UNet_Baseline(AblationUNetBase):  # noqa: N801  (reference class names)
    def __init__(self, in_channels, out_channels, features, precision=None, **kwargs):
        super().__init__(lambda i, o: LocalOnlyBlock(i, o), in_channels, out_channels, features, precision=precision)


class UNet_AttentionOnly(AblationUNetBase):  # noqa: N801
    def __init__(self, in_channels, out_channels, features, pool_size=8, precision=None):
        super().__init__(lambda i, o: AttentionOnlyBlock(i, o, pool_size=pool_size), in_channels, out_channels,
                         features, pool_size, precision=precision)
