"""Placement ablations (reference models/unet_dfc_sa_ablation_placement.py) on the MI355X kernels.

  UNet_EncoderOnlyDFC    :85-150   DFC blocks in the encoder and bottleneck, LocalOnlyBlock decoder
  UNet_DecoderOnlyDFC    :152-217  LocalOnlyBlock encoder and bottleneck, DFC blocks in the decoder
  UNet_BothStandardConv  :219-284  LocalOnlyBlock everywhere

The reference's own DynamicFusionConvAttnBlock copy (:7-83) is the DFC block with a
channels // 8 query/key width (ablation_on_qk_channels = 8 here).  The module trees and forwards
equal UNetDFCSA's (blocks created in the order down1..down4, bottleneck, up_conv4..up_conv1).
"""
from models.unet_dfc_sa_ablation_branches import AblationUNetBase, LocalOnlyBlock
from models.unet_dfc_sa_res import DynamicFusionConvAttnBlock


class _PlacementUNet(AblationUNetBase):
    ENCODER_DFC = DECODER_DFC = False

    def __init__(self, in_channels, out_channels, features, pool_size=8, precision=None):
        self._nblocks = 0
        super().__init__(None, in_channels, out_channels, features, pool_size, precision=precision)

    def _make_block(self, in_channels, out_channels, pool_size, ablation_on_qk_channels):
        encoder = self._nblocks < 5   # down1..down4, bottleneck
        self._nblocks += 1
        if (encoder and self.ENCODER_DFC) or (not encoder and self.DECODER_DFC):
            return DynamicFusionConvAttnBlock(in_channels, out_channels, pool_size=pool_size)
        return LocalOnlyBlock(in_channels, out_channels)


class UNet_EncoderOnlyDFC(_PlacementUNet):  # noqa: N801  (reference class names)
    ENCODER_DFC = True


class UNet_DecoderOnlyDFC(_PlacementUNet):  # noqa: N801
    DECODER_DFC = True


class UNet_BothStandardConv(_PlacementUNet):  # noqa: N801
    def __init__(self, in_channels, out_channels, features, precision=None, **kwargs):
        super().__init__(in_channels, out_channels, features, precision=precision)
