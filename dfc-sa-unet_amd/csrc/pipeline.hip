// Input/output pipeline kernels either side of the training/inference step.
//
// Sliding-window inference (reference inference.py:104-153, predict_large_image):
//   tiles_gather      uint8 HWC image (resident in HBM) -> the batch of normalised NCHW fp32 tiles
//                     the model consumes, optionally with the two TTA flips of every tile
//                     (ToTensor + Normalize of :116-119, torch.flip of :136-139)
//   tiles_accumulate  per-tile logits -> sigmoid -> TTA average -> overlap-averaged canvas
//                     (:132-151); every canvas pixel gathers its tiles in the reference's
//                     y-major loop order, so the fp32 sums are formed in the same order
//   seg_counts        threshold + TP/FP/FN against a uint8 ground truth (:73-91, :289-314),
//                     integer counts (exact); TN = n - TP - FP - FN on the host
//
// Paired training transforms (reference utils/data_loader.py:25-73, :119-135), bit-exact with the
// Pillow calls the reference makes (Pillow 12.2.0; restated and pinned in oracle/augment_oracle.py):
//   aug_resample      one pass of Image.resize(BILINEAR): Resample.c's separable 8-bit
//                     convolution with 22-bit fixed-point coefficients (host-computed tables);
//                     a batch of per-sample descriptors per launch (horizontal, then vertical)
//   aug_finish        Image.rotate (BILINEAR image: Geometry.c's double-precision affine sampling,
//                     contraction off; NEAREST mask: 16.16 fixed point) + FLIP_LEFT_RIGHT +
//                     ToTensor + Normalize for the image, resize(NEAREST) + rotate + flip +
//                     (/255 > 0.5) for the mask, straight into the NCHW fp32 batch
// All work is bandwidth-bound byte/float streaming; no MFMA.
#include <algorithm>
#include <cmath>

#include "common.h"
#include "dfcsa_internal.h"

namespace {

inline int grid_for(int64_t n, int per = 256, int cap = 16384) {
  int64_t b = (n + per - 1) / per;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, cap));
}

struct NormArgs {
  float mean[4];
  float stdv[4];
};

// One thread per tile pixel: one C-byte read, C * variants fp32 writes (variant 1 is the
// horizontally flipped tile, variant 2 the vertically flipped one).  out = [T*V][C][th][tw].
__global__ void __launch_bounds__(256) tiles_gather_kernel(const uint8_t* __restrict__ img, int W, int C,
                                                           const int* __restrict__ ty, const int* __restrict__ tx,
                                                           int T, int th, int tw, int V, NormArgs na,
                                                           float* __restrict__ out) {
  const int64_t plane = (int64_t)th * tw;
  const int64_t total = (int64_t)T * plane;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(e / plane);
    const int r = (int)(e - (int64_t)t * plane);
    const int i = r / tw, j = r - (r / tw) * tw;
    const int y = ty[t] + i, x = tx[t] + j;
    const uint8_t* px = img + ((int64_t)y * W + x) * C;
    float* o = out + (int64_t)t * V * C * plane;
    for (int c = 0; c < C; ++c) {
      // torchvision ToTensor: float(u8) / 255 (true division), Normalize: (v - mean) / std, fp32
      const float v = ((float)px[c] / 255.0f - na.mean[c]) / na.stdv[c];
      o[(int64_t)c * plane + r] = v;
      if (V == 3) {
        o[(int64_t)(C + c) * plane + (int64_t)i * tw + (tw - 1 - j)] = v;
        o[(int64_t)(2 * C + c) * plane + (int64_t)(th - 1 - i) * tw + j] = v;
      }
    }
  }
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// One thread per canvas pixel.  logits = [T*V][th][tw] (the model's [n,1,th,tw] output), tile
// t = iy * nx + ix.
__global__ void __launch_bounds__(256) tiles_accumulate_kernel(const float* __restrict__ logits,
                                                               const int* __restrict__ ys, int ny,
                                                               const int* __restrict__ xs, int nx, int th, int tw,
                                                               int V, int H, int W, float* __restrict__ canvas) {
  const int64_t plane = (int64_t)th * tw;
  const int64_t total = (int64_t)H * W;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)(e / W), x = (int)(e - (e / W) * W);
    float acc = 0.f, cnt = 0.f;
    for (int iy = 0; iy < ny; ++iy) {
      const int i = y - ys[iy];
      if (i < 0 || i >= th) continue;
      for (int ix = 0; ix < nx; ++ix) {
        const int j = x - xs[ix];
        if (j < 0 || j >= tw) continue;
        const float* L = logits + (int64_t)(iy * nx + ix) * V * plane;
        float p = sigmoidf_(L[(int64_t)i * tw + j]);
        if (V == 3) {
          const float ph = sigmoidf_(L[plane + (int64_t)i * tw + (tw - 1 - j)]);
          const float pv = sigmoidf_(L[2 * plane + (int64_t)(th - 1 - i) * tw + j]);
          p = ((p + ph) + pv) / 3.0f;
        }
        acc += p;
        cnt += 1.0f;
      }
    }
    canvas[e] = acc / (cnt == 0.f ? 1.0f : cnt);
  }
}

// TP/FP/FN.  pred = prob > thr; gt = gray(gt_pixel) > gt_thr, gray = OpenCV's fixed-point
// RGB2GRAY ((R*4899 + G*9617 + B*1868 + 2^13) >> 14) for 3-channel ground truth.
__global__ void __launch_bounds__(256) seg_counts_kernel(const float* __restrict__ prob, int64_t n, float thr,
                                                         const uint8_t* __restrict__ gt, int gc, int gt_thr,
                                                         unsigned long long* __restrict__ counts) {
  uint32_t tp = 0, fp = 0, fn = 0;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const bool p = prob[e] > thr;
    int g;
    if (gc == 3) {
      const uint8_t* q = gt + e * 3;
      g = ((int)q[0] * 4899 + (int)q[1] * 9617 + (int)q[2] * 1868 + (1 << 13)) >> 14;
    } else {
      g = gt[e];
    }
    const bool t = g > gt_thr;
    tp += p && t;
    fp += p && !t;
    fn += !p && t;
  }
  __shared__ uint32_t red[3][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t v[3] = {tp, fp, fn};
  for (int k = 0; k < 3; ++k) {
    uint32_t s = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) red[k][wv] = s;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int k = threadIdx.x;
    const unsigned long long s = (unsigned long long)red[k][0] + red[k][1] + red[k][2] + red[k][3];
    if (s) atomicAdd(counts + k, s);  // integer atomics: order-independent, exact
  }
}

// ---------------------------------------------------------------- paired transforms
// One thread per output element (all channels).  Horizontal pass (axis 1): line = output row
// (source row row0 + line), taps step C bytes.  Vertical pass (axis 0): line = column, taps step
// src_pitch bytes.  acc = 2^21 + sum(pixel * coeff), out = clamp(acc >> 22, 0, 255).
__global__ void __launch_bounds__(256) aug_resample_kernel(const dfcsa_resample_desc* __restrict__ descs, int C) {
  const dfcsa_resample_desc d = descs[blockIdx.y];
  const int64_t total = (int64_t)d.n_out * d.n_lines;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    int o, line;
    if (d.axis) {
      line = (int)(e / d.n_out);
      o = (int)(e - (int64_t)line * d.n_out);
    } else {
      o = (int)(e / d.n_lines);
      line = (int)(e - (int64_t)o * d.n_lines);
    }
    const int first = d.bounds[2 * o], cnt = d.bounds[2 * o + 1];
    const int32_t* k = d.kk + (int64_t)o * d.ksize;
    const uint8_t* s;
    int64_t step;
    uint8_t* out;
    if (d.axis) {
      s = d.src + (int64_t)(d.row0 + line) * d.src_pitch + (int64_t)first * C;
      step = C;
      out = d.dst + (int64_t)line * d.dst_pitch + (int64_t)o * C;
    } else {
      s = d.src + (int64_t)first * d.src_pitch + (int64_t)line * C;
      step = d.src_pitch;
      out = d.dst + (int64_t)o * d.dst_pitch + (int64_t)line * C;
    }
    int acc[4] = {1 << 21, 1 << 21, 1 << 21, 1 << 21};
    for (int t = 0; t < cnt; ++t) {
      const int w = k[t];
      for (int c = 0; c < C; ++c) acc[c] += (int)s[t * step + c] * w;
    }
    for (int c = 0; c < C; ++c) out[c] = (uint8_t)min(max(acc[c] >> 22, 0), 255);
  }
}

// Geometry.c bilinear_filter (8-bit bands): sample at (xin, yin) of the [H][W][3] image.
__device__ __forceinline__ bool bilinear_rgb(const uint8_t* img, int W, int H, double xin, double yin,
                                             int (&v)[3]) {
#pragma clang fp contract(off)
  if (xin < 0.0 || xin >= W || yin < 0.0 || yin >= H) return false;
  xin -= 0.5;
  yin -= 0.5;
  const double fx = floor(xin), fy = floor(yin);
  const int x = (int)fx, y = (int)fy;
  const double dx = xin - fx, dy = yin - fy;
  const int x0 = min(max(x, 0), W - 1), x1 = min(max(x + 1, 0), W - 1);
  const int ya = min(max(y, 0), H - 1);
  const bool yb_ok = y + 1 >= 0 && y + 1 < H;
  const uint8_t* ra = img + (int64_t)ya * W * 3;
  const uint8_t* rb = img + (int64_t)(yb_ok ? y + 1 : ya) * W * 3;
  for (int c = 0; c < 3; ++c) {
    // BILINEAR(v, a, b, d) = a + (b - a) * d with integer (b - a), evaluated in double
    const double v1 = (double)ra[x0 * 3 + c] + (double)((int)ra[x1 * 3 + c] - (int)ra[x0 * 3 + c]) * dx;
    double v2 = v1;
    if (yb_ok) v2 = (double)rb[x0 * 3 + c] + (double)((int)rb[x1 * 3 + c] - (int)rb[x0 * 3 + c]) * dx;
    const double r = v1 + (v2 - v1) * dy;
    v[c] = min(max((int)r, 0), 255);  // (UINT8) cast: truncation
  }
  return true;
}

__global__ void __launch_bounds__(256) aug_finish_kernel(const dfcsa_aug_desc* __restrict__ descs, int H, int W,
                                                         NormArgs na, int normalize, float* __restrict__ images,
                                                         float* __restrict__ masks) {
#pragma clang fp contract(off)
  const dfcsa_aug_desc d = descs[blockIdx.y];
  const int64_t plane = (int64_t)H * W;
  float* oi = images + (int64_t)blockIdx.y * 3 * plane;
  float* om = masks + (int64_t)blockIdx.y * plane;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < plane; e += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)(e / W), xo = (int)(e - (e / W) * W);
    const int x = d.flip ? W - 1 - xo : xo;  // FLIP_LEFT_RIGHT after the rotation
    int v[3] = {0, 0, 0};
    int mx = -1, my = -1;                    // position in the resized mask (-1: fill)
    if (d.rotate == 1) {
      const double xi = x + 0.5, yi = y + 0.5;
      const double xin = d.m[0] * xi + d.m[1] * yi + d.m[2];
      const double yin = d.m[3] * xi + d.m[4] * yi + d.m[5];
      bilinear_rgb(d.img, W, H, xin, yin, v);
      const int64_t xx = (int64_t)d.fix[2] + (int64_t)y * d.fix[1] + (int64_t)x * d.fix[0];
      const int64_t yy = (int64_t)d.fix[5] + (int64_t)y * d.fix[4] + (int64_t)x * d.fix[3];
      const int xin_n = (int)(xx >> 16), yin_n = (int)(yy >> 16);
      if (xin_n >= 0 && xin_n < W && yin_n >= 0 && yin_n < H) {
        mx = xin_n;
        my = yin_n;
      }
    } else {
      int sx = x, sy = y;  // exact transposes: 0 none, 2 ROTATE_180, 3 ROTATE_90, 4 ROTATE_270
      if (d.rotate == 2) {
        sx = W - 1 - x;
        sy = H - 1 - y;
      } else if (d.rotate == 3) {
        sx = W - 1 - y;
        sy = x;
      } else if (d.rotate == 4) {
        sx = y;
        sy = H - 1 - x;
      }
      const uint8_t* p = d.img + ((int64_t)sy * W + sx) * 3;
      v[0] = p[0];
      v[1] = p[1];
      v[2] = p[2];
      mx = sx;
      my = sy;
    }
    uint8_t mv = 0;
    if (mx >= 0) {
      const int sxm = d.xtab[mx], sym = d.ytab[my];  // resize(NEAREST) tables (-1: fill 0)
      if (sxm >= 0 && sym >= 0) mv = d.mask[(int64_t)sym * d.mask_w + sxm];
    }
    for (int c = 0; c < 3; ++c) {
      float f = (float)v[c] / 255.0f;
      if (normalize) f = (f - na.mean[c]) / na.stdv[c];
      oi[c * plane + e] = f;
    }
    om[e] = ((float)mv / 255.0f > 0.5f) ? 1.0f : 0.0f;
  }
}

}  // namespace

extern "C" int dfcsa_aug_resample(const dfcsa_resample_desc* descs_dev, int n, int max_work, int C, void* stream) {
  if (!descs_dev || n <= 0 || max_work <= 0 || C <= 0 || C > 4 || n > 65535) return DFCSA_EINVAL;
  hipLaunchKernelGGL(aug_resample_kernel, dim3(grid_for(max_work, 256, 2048), n), dim3(256), 0, (hipStream_t)stream,
                     descs_dev, C);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_aug_finish(const dfcsa_aug_desc* descs_dev, int n, int H, int W, const float* mean_std,
                                int normalize, float* images, float* masks, void* stream) {
  if (!descs_dev || n <= 0 || n > 65535 || H <= 0 || W <= 0 || !images || !masks || (normalize && !mean_std))
    return DFCSA_EINVAL;
  NormArgs na;
  for (int c = 0; c < 4; ++c) {
    na.mean[c] = (normalize && c < 3) ? mean_std[c] : 0.f;
    na.stdv[c] = (normalize && c < 3) ? mean_std[3 + c] : 1.f;
  }
  hipLaunchKernelGGL(aug_finish_kernel, dim3(grid_for((int64_t)H * W, 256, 2048), n), dim3(256), 0,
                     (hipStream_t)stream, descs_dev, H, W, na, normalize, images, masks);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_tiles_gather(const uint8_t* img, int H, int W, int C, const int* ty, const int* tx, int T, int th,
                                  int tw, int variants, const float* mean_std, float* out, void* stream) {
  if (!img || !ty || !tx || !out || !mean_std || H <= 0 || W <= 0 || C <= 0 || C > 4 || T <= 0 || th <= 0 ||
      tw <= 0 || th > H || tw > W || (variants != 1 && variants != 3))
    return DFCSA_EINVAL;
  NormArgs na;
  for (int c = 0; c < 4; ++c) {
    na.mean[c] = c < C ? mean_std[c] : 0.f;
    na.stdv[c] = c < C ? mean_std[C + c] : 1.f;
  }
  hipLaunchKernelGGL(tiles_gather_kernel, dim3(grid_for((int64_t)T * th * tw)), dim3(256), 0, (hipStream_t)stream,
                     img, W, C, ty, tx, T, th, tw, variants, na, out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_tiles_accumulate(const float* logits, const int* ys, int ny, const int* xs, int nx, int th, int tw,
                                      int variants, int H, int W, float* canvas, void* stream) {
  if (!logits || !ys || !xs || !canvas || ny <= 0 || nx <= 0 || th <= 0 || tw <= 0 || H <= 0 || W <= 0 ||
      (variants != 1 && variants != 3))
    return DFCSA_EINVAL;
  hipLaunchKernelGGL(tiles_accumulate_kernel, dim3(grid_for((int64_t)H * W)), dim3(256), 0, (hipStream_t)stream,
                     logits, ys, ny, xs, nx, th, tw, variants, H, W, canvas);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_seg_counts(const float* prob, int64_t n, float thr, const uint8_t* gt, int gt_channels,
                                int gt_thr, unsigned long long* counts, void* stream) {
  if (!prob || !gt || !counts || n <= 0 || (gt_channels != 1 && gt_channels != 3)) return DFCSA_EINVAL;
  hipError_t e = hipMemsetAsync(counts, 0, 4 * sizeof(unsigned long long), (hipStream_t)stream);
  if (e != hipSuccess) return -(int)e;
  hipLaunchKernelGGL(seg_counts_kernel, dim3(grid_for(n, 256 * 8, 4096)), dim3(256), 0, (hipStream_t)stream, prob, n,
                     thr, gt, gt_channels, gt_thr, counts);
  DFCSA_CHECK_LAUNCH();
  return 0;
}
