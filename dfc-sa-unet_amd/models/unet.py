"""Classic U-Net (reference models/unet.py:6-101; config_unet.yaml = BASELINE config 1) on the
MI355X kernels.

Same module tree, parameter creation order and state_dict keys as the reference (so a seeded
construction gives the reference's initial weights): widths 64..1024 hard-coded (the factory's
``features`` / ``pool_size`` are ignored, model_factory.py:94-100), DoubleConv = 2 x (3x3 conv + BN +
ReLU), Down = MaxPool2d(2, ceil_mode=True) + DoubleConv, Up = ConvTranspose2d(k2, s2) + crop-to-match
+ cat([skip, up]) + DoubleConv, OutConv = 1x1.  Activations are NHWC in the compute dtype; the
convolutions run on the implicit GEMM, the skip concat is a second GEMM source segment.
``bilinear=True`` (nn.Upsample(scale_factor=2, bilinear, align_corners=True) in Up, unet.py:36-37;
down4 and the up blocks at half width, unet.py:78-88) upsamples with dfcsa_upsample2_ac.
"""
import torch
import torch.nn as nn

import dfcsa
from dfcsa import packs
from dfcsa.flat import ALIGN, FlatParams
from dfcsa.functions import ConvTranspose2x2, Head1x1, InputToNHWC
from dfcsa.ops import rup
from dfcsa.transunet_ops import Upsample2x
from dfcsa.unet_ops import ConvBNReLU, Crop, MaxPool2x2Ceil


class DoubleConv(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, kernel_size=3, padding=1), nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True),
            nn.Conv2d(out_channels, out_channels, kernel_size=3, padding=1), nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True))

    def forward_nhwc(self, xs, dtype):
        c0, b0, c1, b1 = self.conv[0], self.conv[1], self.conv[3], self.conv[4]
        h = ConvBNReLU.apply(c0, b0, dtype, len(xs), *xs, *c0.parameters(), *b0.parameters())
        return ConvBNReLU.apply(c1, b1, dtype, 1, h, *c1.parameters(), *b1.parameters())

    def units(self):
        return [(self.conv[0], [self.conv[0], self.conv[1]]), (self.conv[3], [self.conv[3], self.conv[4]])]


class Down(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.mpconv = nn.Sequential(nn.MaxPool2d(2, ceil_mode=True), DoubleConv(in_channels, out_channels))

    def forward_nhwc(self, x, dtype):
        return self.mpconv[1].forward_nhwc([MaxPool2x2Ceil.apply(x, dtype)], dtype)

    def units(self):
        return self.mpconv[1].units()


class Up(nn.Module):
    def __init__(self, in_channels, out_channels, bilinear=True):
        super().__init__()
        if bilinear:
            self.up = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        else:
            self.up = nn.ConvTranspose2d(in_channels, in_channels // 2, kernel_size=2, stride=2)
        self.conv = DoubleConv(in_channels, out_channels)

    def forward_nhwc(self, x1, x2, dtype):
        if isinstance(self.up, nn.Upsample):
            if x1.shape[-1] % 8:
                raise ValueError("bilinear Up needs a channel count divisible by 8")
            x1 = Upsample2x.apply(x1, dtype)
        else:
            x1 = ConvTranspose2x2.apply(x1, self.up, dtype, *self.up.parameters())
        h1, w1, h2, w2 = x1.shape[1], x1.shape[2], x2.shape[1], x2.shape[2]
        dy, dx = h2 - h1, w2 - w1
        if dy < 0 or dx < 0:          # crop the upsampled map (reference :50-51)
            x1 = Crop.apply(x1, 0, 0, min(h1, h2), min(w1, w2), dtype)
        elif dy or dx:                # centred crop of the skip (reference :52-55)
            x2 = Crop.apply(x2, dy // 2, dx // 2, h1, w1, dtype)
        return self.conv.forward_nhwc([x2, x1], dtype)   # torch.cat([x2, x1], dim=1)

    def units(self):
        if isinstance(self.up, nn.Upsample):
            return self.conv.units()
        return [(self.up, [self.up])] + self.conv.units()


class OutConv(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size=1)


class UNet(nn.Module):
    def __init__(self, n_channels, n_classes, bilinear=False, precision=None):
        super().__init__()
        self.n_channels = n_channels
        self.n_classes = n_classes
        self.bilinear = bilinear
        factor = 2 if bilinear else 1
        self.inc = DoubleConv(n_channels, 64)
        self.down1 = Down(64, 128)
        self.down2 = Down(128, 256)
        self.down3 = Down(256, 512)
        self.down4 = Down(512, 1024 // factor)
        self.up1 = Up(1024, 512 // factor, bilinear)
        self.up2 = Up(512, 256 // factor, bilinear)
        self.up3 = Up(256, 128 // factor, bilinear)
        self.up4 = Up(128, 64, bilinear)
        self.outc = OutConv(64, n_classes)
        self.compute_dtype = dfcsa.resolve_dtype(precision)
        self._flat = None

    def set_precision(self, precision):
        self.compute_dtype = dfcsa.resolve_dtype(precision)
        return self

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._flat = None
        self._dfcsa_plan = None
        return out

    def flat_params(self):
        if self._flat is None or not self._flat.valid():
            self._flat = FlatParams(self)
        return self._flat

    def grad_units(self):
        """[(module, lo, hi)] in flat-buffer order: each (conv, BN) pair, each ConvTranspose2d and
        the head finalise a contiguous range of the gradient buffer (data-parallel buckets)."""
        flat = self.flat_params()
        index = {id(p): i for i, p in enumerate(flat.params)}
        groups = self.inc.units()
        for m in (self.down1, self.down2, self.down3, self.down4, self.up1, self.up2, self.up3, self.up4):
            groups += m.units()
        groups.append((self.outc.conv, [self.outc.conv]))
        units = []
        for key, mods in groups:
            ps = [p for m in mods for p in m.parameters()]
            first, last = index[id(ps[0])], index[id(ps[-1])]
            units.append((key, flat.offsets[first], flat.offsets[last] + rup(ps[-1].numel(), ALIGN)))
        return units

    def forward(self, x):
        """x: [B, n_channels, H, W] float -> logits [B, n_classes, H, W] fp32."""
        if not x.is_cuda:
            raise RuntimeError("UNet runs on the MI355X kernels only; move model and input to 'cuda'")
        flat = self.flat_params()
        if torch.is_grad_enabled():
            flat.attach_grads()
        dt = self.compute_dtype
        if getattr(self, "_plan_flat", None) is not flat:
            self._dfcsa_plan, self._plan_flat = None, flat
        planned = packs.sync_model_plan(self)
        h = InputToNHWC.apply(x, dt, rup(x.shape[1], 8))
        x1 = self.inc.forward_nhwc([h], dt)
        x2 = self.down1.forward_nhwc(x1, dt)
        x3 = self.down2.forward_nhwc(x2, dt)
        x4 = self.down3.forward_nhwc(x3, dt)
        x5 = self.down4.forward_nhwc(x4, dt)
        u = self.up1.forward_nhwc(x5, x4, dt)
        u = self.up2.forward_nhwc(u, x3, dt)
        u = self.up3.forward_nhwc(u, x2, dt)
        u = self.up4.forward_nhwc(u, x1, dt)
        logits = Head1x1.apply(u, self.outc.conv, dt, *self.outc.conv.parameters())
        if not planned:
            packs.rebuild_model_plan(self, x.device)
        return logits
