"""CPU oracle for the paired image/mask transforms.  TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, and only as the checker; the product path
(``dfc-sa-unet_amd/utils/augment.py`` on the ``dfcsa_aug_*`` kernels) never does.

Two layers:
  * ``reference_transform`` -- the reference's ExtCompose chain (utils/data_loader.py:25-73,
    :119-135) run with Pillow itself (the library the reference calls; Pillow 12.2.0 is
    installed here and on the GPU box): ExtResize (image BILINEAR, mask NEAREST),
    ExtRandomRotation (BILINEAR / NEAREST, expand=False, black fill), ExtRandomHorizontalFlip,
    ExtToTensor (uint8 / 255; mask / 255 > 0.5), ExtNormalize (ImageNet mean / std).  The random
    draws are passed in explicitly (angle or None, flip) so the GPU path can be fed the same ones.
  * a numpy restatement of the Pillow arithmetic the kernels implement (Resample.c two-pass
    8-bit fixed-point convolution, Geometry.c affine bilinear / nearest sampling), checked
    against Pillow in tests/test_oracle_golden.py so the kernel design is pinned on the CPU.
"""
import math

import numpy as np
from PIL import Image

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)
PRECISION_BITS = 22  # Resample.c: 32 - 8 - 2


# ------------------------------------------------------------------ reference chain (Pillow)
def reference_transform(img_u8, mask_u8, size, angle=None, flip=False, normalize=True):
    """img_u8 [H, W, 3], mask_u8 [H, W] -> (image fp32 [3, h, w], mask fp32 [1, h, w]); size = (w, h)."""
    img = Image.fromarray(img_u8, "RGB").resize(tuple(size), Image.BILINEAR)
    mask = Image.fromarray(mask_u8, "L").resize(tuple(size), Image.NEAREST)
    if angle is not None:
        img = img.rotate(angle, Image.BILINEAR)
        mask = mask.rotate(angle, Image.NEAREST)
    if flip:
        img = img.transpose(Image.FLIP_LEFT_RIGHT)
        mask = mask.transpose(Image.FLIP_LEFT_RIGHT)
    x = np.asarray(img, dtype=np.uint8).transpose(2, 0, 1).astype(np.float32) / np.float32(255.0)
    m = (np.array(mask, dtype=np.uint8).astype(np.float32)[None] / np.float32(255.0) > 0.5).astype(np.float32)
    if normalize:
        x = (x - MEAN[:, None, None]) / STD[:, None, None]
    return x, m


# ------------------------------------------------------------------ Pillow arithmetic, restated
def resample_coeffs(in_size, out_size):
    """Resample.c precompute_coeffs (bilinear filter, support 1) + normalize_coeffs_8bpc:
    (bounds [out, 2] = (xmin, count), kk [out, ksize] int32 22-bit fixed point)."""
    scale = filterscale = float(in_size) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int32)
    kk = np.zeros((out_size, ksize), dtype=np.int32)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w.append(1.0 - t if t < 1.0 else 0.0)
        ww = sum_seq(w)
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + k * (1 << PRECISION_BITS)) if k < 0 else int(0.5 + k * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def sum_seq(vals):
    s = 0.0
    for v in vals:
        s += v
    return s


def _pass(src, bounds, kk, axis):
    """One 8-bit fixed-point pass along ``axis`` of src [H, W, C] uint8."""
    n_out = bounds.shape[0]
    shape = list(src.shape)
    shape[axis] = n_out
    acc = np.full(shape, 1 << (PRECISION_BITS - 1), dtype=np.int64)
    s = src.astype(np.int64)
    for o in range(n_out):
        lo, cnt = bounds[o]
        idx = [slice(None)] * 3
        oidx = [slice(None)] * 3
        oidx[axis] = o
        for k in range(cnt):
            idx[axis] = lo + k
            acc[tuple(oidx)] += s[tuple(idx)] * int(kk[o, k])
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize_bilinear(img, out_w, out_h):
    """Image.resize(BILINEAR) of an RGB uint8 image (ImagingResample: horizontal pass over the rows
    the vertical pass needs, then the vertical pass)."""
    H, W, _ = img.shape
    bh, kh = resample_coeffs(W, out_w)
    bv, kv = resample_coeffs(H, out_h)
    need_h, need_v = out_w != W, out_h != H
    if need_h:
        y0 = int(bv[0, 0])
        y1 = int(bv[-1, 0] + bv[-1, 1])
        bv = bv.copy()
        bv[:, 0] -= y0
        img = _pass(img[y0:y1], bh, kh, 1)
    if need_v:
        img = _pass(img, bv, kv, 0)
    return img


def scale_nearest_tables(in_size, out_size):
    """ImagingScaleAffine tables for Image.resize(NEAREST): sequential double accumulation of
    (in / out) starting at half a step; -1 marks out-of-range samples (filled with 0)."""
    a = float(in_size) / out_size
    xo = 0.0 + a * 0.5
    tab = np.empty(out_size, dtype=np.int32)
    for x in range(out_size):
        xin = -1 if xo < 0.0 else int(xo)
        tab[x] = xin if 0 <= xin < in_size else -1
        xo += a
    return tab


def rotate_matrix(angle, w, h):
    """Image.rotate's inverse affine matrix (PIL/Image.py rotate, expand=False, centre w/2, h/2)."""
    angle = angle % 360.0
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0, round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]
    cx, cy = w / 2, h / 2
    m[2], m[5] = m[0] * -cx + m[1] * -cy + m[2], m[3] * -cx + m[4] * -cy + m[5]
    m[2] += cx
    m[5] += cy
    return m


def rotate_fixed_coeffs(m):
    """Geometry.c affine_fixed (nearest, 16.16 fixed point) integer coefficients."""
    fix = lambda v: int(math.floor(v * 65536.0 + 0.5))  # noqa: E731
    return (fix(m[0]), fix(m[1]), fix(m[2] + m[0] * 0.5 + m[1] * 0.5),
            fix(m[3]), fix(m[4]), fix(m[5] + m[3] * 0.5 + m[4] * 0.5))


def rotate_nearest(mask, m):
    H, W = mask.shape
    a0, a1, a2, a3, a4, a5 = rotate_fixed_coeffs(m)
    y, x = np.mgrid[0:H, 0:W].astype(np.int64)
    xin = (a2 + y * a1 + x * a0) >> 16
    yin = (a5 + y * a4 + x * a3) >> 16
    ok = (xin >= 0) & (xin < W) & (yin >= 0) & (yin < H)
    out = np.zeros_like(mask)
    out[ok] = mask[yin[ok], xin[ok]]
    return out


def rotate_bilinear(img, m, rounding="trunc"):
    """Geometry.c generic affine transform with the bilinear filter (double arithmetic)."""
    H, W, C = img.shape
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    xi = x + 0.5
    yi = y + 0.5
    xin = m[0] * xi + m[1] * yi + m[2]
    yin = m[3] * xi + m[4] * yi + m[5]
    ok = (xin >= 0.0) & (xin < W) & (yin >= 0.0) & (yin < H)
    xs = xin - 0.5
    ys = yin - 0.5
    x0 = np.floor(xs).astype(np.int64)
    y0 = np.floor(ys).astype(np.int64)
    dx = xs - x0
    dy = ys - y0
    xa, xb = np.clip(x0, 0, W - 1), np.clip(x0 + 1, 0, W - 1)
    ya = np.clip(y0, 0, H - 1)
    yb_ok = (y0 + 1 >= 0) & (y0 + 1 < H)
    yb = np.clip(y0 + 1, 0, H - 1)
    f = img.astype(np.float64)
    out = np.zeros_like(img)
    for c in range(C):
        p = f[..., c]
        v1 = p[ya, xa] + (p[ya, xb] - p[ya, xa]) * dx
        v2 = np.where(yb_ok, p[yb, xa] + (p[yb, xb] - p[yb, xa]) * dx, v1)
        v = v1 + (v2 - v1) * dy
        v = np.floor(v + 0.5) if rounding == "round" else np.trunc(v)
        out[..., c] = np.where(ok, np.clip(v, 0, 255), 0).astype(np.uint8)
    return out
