"""Paired image/mask transforms on the GPU: the reference's ExtCompose chain
(utils/data_loader.py:25-73, :119-135) for a whole batch, bit-exact with the Pillow calls the
reference makes (Pillow 12.2.0: Image.resize BILINEAR / NEAREST, Image.rotate BILINEAR / NEAREST
with expand=False and black fill, FLIP_LEFT_RIGHT), then ToTensor + ImageNet Normalize.

Host side (this file): decoding stays on the host (PIL), and so do the random draws, which keep
the reference's call order (``draw_augmentation``).  Per batch, the host computes the integer
resampling tables exactly as Pillow does and uploads the raw uint8 images, the tables and one
descriptor per sample.  Device side: three launches per batch (libdfcsa ``dfcsa_aug_resample``
horizontal and vertical passes, ``dfcsa_aug_finish``) write the NCHW fp32 image batch and the
{0, 1} mask batch the training step consumes.
"""
import ctypes
import math

import numpy as np
import torch

from dfcsa._lib import AugDesc, ResampleDesc, call
from dfcsa.ops import stream

PRECISION_BITS = 22  # Pillow Resample.c: 32 - 8 - 2
IMAGENET_MEAN_STD = (0.485, 0.456, 0.406, 0.229, 0.224, 0.225)


def draw_augmentation(use_augmentation, degrees=90):
    """The reference's random draws for one sample, in its order (data_loader.py:41-53):
    rotation coin, rotation angle (only when the coin says so), flip coin.  Returns (angle, flip)."""
    if not use_augmentation:
        return None, False
    angle = np.random.uniform(-degrees, degrees) if np.random.random() < 0.5 else None
    flip = bool(np.random.random() < 0.5)
    return angle, flip


def resample_coeffs(in_size, out_size):
    """Pillow's precompute_coeffs (bilinear filter, support 1, antialiased when shrinking) and
    normalize_coeffs_8bpc: (bounds [out, 2] = (first tap, tap count), kk [out, ksize] int32)."""
    scale = filterscale = float(in_size) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int32)
    kk = np.zeros((out_size, ksize), dtype=np.int32)
    one = float(1 << PRECISION_BITS)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        inv = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        cnt = min(int(center + support + 0.5), in_size) - xmin
        w = [max(0.0, 1.0 - abs((x + xmin - center + 0.5) * inv)) for x in range(cnt)]
        ww = 0.0
        for v in w:
            ww += v
        for x in range(cnt):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(0.5 + k * one) if k >= 0 else int(-0.5 + k * one)
        bounds[xx] = (xmin, cnt)
    return bounds, kk


def nearest_table(in_size, out_size):
    """Image.resize(NEAREST) source index per output index (Pillow's ImagingScaleAffine: a double
    accumulated from half a step); -1 = outside the source (filled with 0)."""
    a = float(in_size) / out_size
    xo = a * 0.5
    tab = np.empty(out_size, dtype=np.int32)
    for x in range(out_size):
        xin = -1 if xo < 0.0 else int(xo)
        tab[x] = xin if 0 <= xin < in_size else -1
        xo += a
    return tab


def rotation(angle, w, h):
    """Image.rotate(angle) of a w x h image: (mode, inverse affine matrix, 16.16 fixed-point matrix).
    mode 0: no-op (angle % 360 == 0), 2: ROTATE_180, 3/4: ROTATE_90/270 (square images), 1: affine."""
    if angle is None:
        return 0, [0.0] * 6, [0] * 6
    a = angle % 360.0
    if a == 0:
        return 0, [0.0] * 6, [0] * 6
    if a == 180:
        return 2, [0.0] * 6, [0] * 6
    if a in (90, 270) and w == h:
        return (3 if a == 90 else 4), [0.0] * 6, [0] * 6
    r = -math.radians(a)
    m = [round(math.cos(r), 15), round(math.sin(r), 15), 0.0, round(-math.sin(r), 15), round(math.cos(r), 15), 0.0]
    cx, cy = w / 2, h / 2
    m[2], m[5] = m[0] * -cx + m[1] * -cy + m[2], m[3] * -cx + m[4] * -cy + m[5]
    m[2] += cx
    m[5] += cy
    fix = lambda v: int(math.floor(v * 65536.0 + 0.5))  # noqa: E731  (Geometry.c affine_fixed)
    f = [fix(m[0]), fix(m[1]), fix(m[2] + m[0] * 0.5 + m[1] * 0.5),
         fix(m[3]), fix(m[4]), fix(m[5] + m[3] * 0.5 + m[4] * 0.5)]
    return 1, m, f


class PairedTransformGPU:
    """``ExtCompose([ExtResize(size), (ExtRandomRotation(90), ExtRandomHorizontalFlip()),
    ExtToTensor(), ExtNormalize()])`` for a batch, on the GPU.  ``size`` = (width, height) as
    ExtResize / PIL take it.  Call with samples {'image': uint8 [H, W, 3], 'mask': uint8 [H, W],
    'angle': float | None, 'flip': bool}; returns (images fp32 [B, 3, h, w], masks fp32
    [B, 1, h, w]) on ``device``."""

    def __init__(self, size, device="cuda", normalize=True):
        self.w, self.h = (int(v) for v in size)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("PairedTransformGPU runs on the MI355X kernels only")
        self.normalize = normalize
        self._coeffs = {}
        self._near = {}

    def _tables(self, key, fn, cache):
        if key not in cache:
            cache[key] = fn(*key)
        return cache[key]

    def __call__(self, samples):
        B, w, h, dev = len(samples), self.w, self.h, self.device
        imgs = [np.ascontiguousarray(s["image"], dtype=np.uint8) for s in samples]
        masks = [np.ascontiguousarray(s["mask"], dtype=np.uint8) for s in samples]
        for im, mk in zip(imgs, masks):
            if im.ndim != 3 or im.shape[2] != 3 or mk.ndim != 2:
                raise ValueError("samples need an RGB uint8 image [H, W, 3] and an 'L' uint8 mask [H, W]")
        # host tables (int32 arena) and per-sample geometry
        tabs, off = [], 0

        def put(a):
            nonlocal off
            tabs.append(a.reshape(-1))
            o = off
            off += a.size
            return o

        geo = []
        for im, mk in zip(imgs, masks):
            H, W = im.shape[:2]
            bh, kh = self._tables((W, w), resample_coeffs, self._coeffs)
            bv, kv = self._tables((H, h), resample_coeffs, self._coeffs)
            y0, y1 = int(bv[0, 0]), int(bv[-1, 0] + bv[-1, 1])
            bvs = bv.copy()
            bvs[:, 0] -= y0
            xt = self._tables((mk.shape[1], w), nearest_table, self._near)
            yt = self._tables((mk.shape[0], h), nearest_table, self._near)
            geo.append(dict(H=H, W=W, y0=y0, rows=y1 - y0, kh=(put(bh), put(kh), kh.shape[1]),
                            kv=(put(bvs), put(kv), kv.shape[1]), xt=put(xt), yt=put(yt)))
        tab_d = torch.from_numpy(np.concatenate(tabs).astype(np.int32)).to(dev)
        src_off = np.cumsum([0] + [im.size for im in imgs])
        msk_off = np.cumsum([0] + [mk.size for mk in masks])
        src_d = torch.from_numpy(np.concatenate([im.reshape(-1) for im in imgs])).to(dev)
        msk_d = torch.from_numpy(np.concatenate([mk.reshape(-1) for mk in masks])).to(dev)
        tmp_off = np.cumsum([0] + [g["rows"] * w * 3 for g in geo])
        tmp_d = torch.empty(int(tmp_off[-1]), dtype=torch.uint8, device=dev)
        res_d = torch.empty((B, h, w, 3), dtype=torch.uint8, device=dev)
        tb, sb, mb, tp, rb = tab_d.data_ptr(), src_d.data_ptr(), msk_d.data_ptr(), tmp_d.data_ptr(), res_d.data_ptr()

        hd, vd, fd = (ResampleDesc * B)(), (ResampleDesc * B)(), (AugDesc * B)()
        for i, g in enumerate(geo):
            hd[i] = ResampleDesc(sb + int(src_off[i]), tp + int(tmp_off[i]), tb + 4 * g["kh"][0], tb + 4 * g["kh"][1],
                                 w, g["rows"], g["kh"][2], 1, g["W"] * 3, w * 3, g["y0"], 0)
            vd[i] = ResampleDesc(tp + int(tmp_off[i]), rb + i * h * w * 3, tb + 4 * g["kv"][0], tb + 4 * g["kv"][1],
                                 h, w, g["kv"][2], 0, w * 3, w * 3, 0, 0)
            mode, m, fix = rotation(samples[i].get("angle"), w, h)
            fd[i] = AugDesc(rb + i * h * w * 3, mb + int(msk_off[i]), tb + 4 * g["xt"], tb + 4 * g["yt"],
                            (ctypes.c_double * 6)(*m), (ctypes.c_int * 6)(*fix), mode, int(bool(samples[i].get("flip"))),
                            masks[i].shape[1], 0)
        desc_d = torch.from_numpy(np.frombuffer(bytes(hd) + bytes(vd) + bytes(fd), dtype=np.uint8).copy()).to(dev)
        dp, rs = desc_d.data_ptr(), ctypes.sizeof(ResampleDesc) * B
        st = stream()
        call("dfcsa_aug_resample", dp, B, max(w * g["rows"] for g in geo), 3, st)
        call("dfcsa_aug_resample", dp + rs, B, h * w, 3, st)
        images = torch.empty((B, 3, h, w), dtype=torch.float32, device=dev)
        out_masks = torch.empty((B, 1, h, w), dtype=torch.float32, device=dev)
        ms = (ctypes.c_float * 6)(*IMAGENET_MEAN_STD)
        call("dfcsa_aug_finish", dp + 2 * rs, B, h, w, ms, int(self.normalize), images.data_ptr(),
             out_masks.data_ptr(), st)
        # keep the staging buffers alive until the launches that read them have run
        self._keep = (tab_d, src_d, msk_d, tmp_d, res_d, desc_d)
        return images, out_masks
