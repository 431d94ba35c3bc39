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

}  // namespace

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
