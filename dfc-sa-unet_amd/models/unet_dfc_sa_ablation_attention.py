"""Full-resolution self-attention ablation (reference models/unet_dfc_sa_ablation_attention.py,
config_ablation3_full_res_attn.yaml = BASELINE config 5) on the MI355X kernels.

  FullResolutionAttention  :7-26   q/k (C -> C//8) and v (C -> C) 1x1 convs over ALL H*W
                                   positions, softmax(q k^T) without scaling, out = gamma*(v A^T) + x
  FullResAttnDFCBlock      :29-92  the DFC block with that attention in its attention branch
  UNet_FullResAttention    :95-97  AblationUNetBase (unet_dfc_sa_ablation_branches.py:104-164) of
                                   those blocks; its module tree and forward equal UNetDFCSA's

Module trees, parameter creation order and state_dict keys are the reference's.  The attention runs
on the flash-style kernels of csrc/fra.hip (dfcsa/fra.py): the reference materialises the
[B, HW, HW] energy (274.9 GB per image at 512^2, so it cannot run config 5); here nothing N^2-sized
is stored.
"""
import torch
import torch.nn as nn

from dfcsa import chanpad
from dfcsa.fra import FRAFunction
from models.unet_dfc_sa_res import DynamicFusionConvAttnBlock, UNetDFCSA, _nchw_to_nhwc, _nhwc_to_nchw


class FullResolutionAttention(nn.Module):
    """Reference :7-26 (pool_size and other kwargs are ignored there too)."""
    full_resolution = True

    def __init__(self, channels, **kwargs):
        super().__init__()
        self.query_conv = nn.Conv2d(channels, channels // 8, kernel_size=1)
        self.key_conv = nn.Conv2d(channels, channels // 8, kernel_size=1)
        self.value_conv = nn.Conv2d(channels, channels, kernel_size=1)
        self.gamma = nn.Parameter(torch.zeros(1))
        self.compute_dtype = torch.bfloat16
        if chanpad.standalone():   # any width on its own (inside a block or U-Net: padded with it)
            chanpad.pad_standalone(self, channels, channels)

    def forward(self, x):
        """x: [B, C, H, W] -> gamma * attention(x) + x, NCHW fp32."""
        y = FRAFunction.apply(self, self.compute_dtype, _nchw_to_nhwc(x, self.compute_dtype), *self.parameters())
        return _nhwc_to_nchw(y, self)


class FullResAttnDFCBlock(DynamicFusionConvAttnBlock):
    """Reference :29-92: local 3x3 branch, 1x1 -> full-resolution attention branch, sigmoid gate,
    1x1 fusion conv, scaled 1x1 residual (forward identical to the DFC block's otherwise)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, **kwargs):
        super().__init__(in_channels, out_channels, kernel_size=kernel_size, stride=stride, padding=padding)

    def _make_attention(self, channels, pool_size, ablation_on_qk_channels):
        return FullResolutionAttention(channels)


class UNet_FullResAttention(UNetDFCSA):  # noqa: N801  (reference class name)
    """Reference :95-97 on AblationUNetBase: 4 encoder blocks + max pooling, 2x-wide bottleneck,
    4 x (ConvTranspose2d -> [bilinear fix] -> cat[up, skip] -> block), 1x1 head."""

    def __init__(self, in_channels, out_channels, features, precision=None, **kwargs):
        super().__init__(in_channels, out_channels, features, precision=precision)

    def _make_block(self, in_channels, out_channels, pool_size, ablation_on_qk_channels):
        return FullResAttnDFCBlock(in_channels, out_channels)
