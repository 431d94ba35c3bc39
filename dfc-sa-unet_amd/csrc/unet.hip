// Plain U-Net plumbing (reference models/unet.py, BASELINE config 1), NHWC, C % 8 == 0:
//   nn.MaxPool2d(2, ceil_mode=True)   Down, :26 (+ its backward)
//   the crop-to-match of Up.forward   :47-55 (x1[:, :, :H2, :W2] or the centred crop of x2)
// Everything else of the plain U-Net (3x3 conv + BatchNorm + ReLU, ConvTranspose2d, 1x1 head)
// runs on the shared implicit-GEMM / elementwise kernels.
#include "common.h"
#include "dfcsa_internal.h"

namespace {

inline int grid_n(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

// one thread per (output pixel, 8-channel chunk); window taps (0,0),(0,1),(1,0),(1,1) in order,
// taps past the bottom/right edge skipped (ceil mode, no padding)
template <typename T>
__global__ void __launch_bounds__(256) maxpool2c_fwd_kernel(int B, int H, int W, int C, const T* __restrict__ x,
                                                            T* __restrict__ y) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2, cpp = C >> 3;
  const int64_t total = (int64_t)B * Ho * Wo * cpp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t p = e / cpp;
    const int ow = (int)(p % Wo);
    p /= Wo;
    const int oh = (int)(p % Ho);
    const int b = (int)(p / Ho);
    const int h0 = 2 * oh, w0 = 2 * ow;
    float best[8], v[8];
    load8<T>(x + ((size_t)(b * H + h0) * W + w0) * C + ck * 8, best);
#pragma unroll
    for (int t = 1; t < 4; ++t) {
      const int h = h0 + (t >> 1), w = w0 + (t & 1);
      if (h >= H || w >= W) continue;
      load8<T>(x + ((size_t)(b * H + h) * W + w) * C + ck * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (v[q] > best[q] || isnan(v[q])) best[q] = v[q];
    }
    store8<T>(y + ((size_t)(b * Ho + oh) * Wo + ow) * C + ck * 8, best);
  }
}

// windows tile the input exactly (no overlap), so dx is written, not accumulated
template <typename T>
__global__ void __launch_bounds__(256) maxpool2c_bwd_kernel(int B, int H, int W, int C, const T* __restrict__ x,
                                                            const T* __restrict__ dy, T* __restrict__ dx) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2, cpp = C >> 3;
  const int64_t total = (int64_t)B * Ho * Wo * cpp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t p = e / cpp;
    const int ow = (int)(p % Wo);
    p /= Wo;
    const int oh = (int)(p % Ho);
    const int b = (int)(p / Ho);
    const int h0 = 2 * oh, w0 = 2 * ow;
    float best[8], v[8], g[8];
    int arg[8];
    load8<T>(x + ((size_t)(b * H + h0) * W + w0) * C + ck * 8, best);
#pragma unroll
    for (int q = 0; q < 8; ++q) arg[q] = 0;
#pragma unroll
    for (int t = 1; t < 4; ++t) {
      const int h = h0 + (t >> 1), w = w0 + (t & 1);
      if (h >= H || w >= W) continue;
      load8<T>(x + ((size_t)(b * H + h) * W + w) * C + ck * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (v[q] > best[q] || isnan(v[q])) { best[q] = v[q]; arg[q] = t; }
    }
    load8<T>(dy + ((size_t)(b * Ho + oh) * Wo + ow) * C + ck * 8, g);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int h = h0 + (t >> 1), w = w0 + (t & 1);
      if (h >= H || w >= W) continue;
      float o[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = (arg[q] == t) ? g[q] : 0.f;
      store8<T>(dx + ((size_t)(b * H + h) * W + w) * C + ck * 8, o);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) window_copy_kernel(int B, int C, int Hs, int Ws, const T* __restrict__ src,
                                                          int Hd, int Wd, T* __restrict__ dst, int oy, int ox) {
  const int cpp = C >> 3;
  const int64_t total = (int64_t)B * Hd * Wd * cpp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t p = e / cpp;
    const int w = (int)(p % Wd);
    p /= Wd;
    const int h = (int)(p % Hd);
    const int b = (int)(p / Hd);
    const int sh = h + oy, sw = w + ox;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (sh >= 0 && sh < Hs && sw >= 0 && sw < Ws) load8<T>(src + ((size_t)(b * Hs + sh) * Ws + sw) * C + ck * 8, v);
    store8<T>(dst + ((size_t)(b * Hd + h) * Wd + w) * C + ck * 8, v);
  }
}

}  // namespace

extern "C" int dfcsa_maxpool2_ceil_fwd(int dtype, int B, int H, int W, int C, const void* x, void* out,
                                       void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8) return DFCSA_EINVAL;
  const int64_t n = (int64_t)B * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(maxpool2c_fwd_kernel<bf16_t>, dim3(grid_n(n)), dim3(256), 0, st, B, H, W, C,
                       (const bf16_t*)x, (bf16_t*)out);
  else
    hipLaunchKernelGGL(maxpool2c_fwd_kernel<float>, dim3(grid_n(n)), dim3(256), 0, st, B, H, W, C, (const float*)x,
                       (float*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_maxpool2_ceil_bwd(int dtype, int B, int H, int W, int C, const void* x, const void* dout,
                                       void* dx, void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8) return DFCSA_EINVAL;
  const int64_t n = (int64_t)B * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(maxpool2c_bwd_kernel<bf16_t>, dim3(grid_n(n)), dim3(256), 0, st, B, H, W, C,
                       (const bf16_t*)x, (const bf16_t*)dout, (bf16_t*)dx);
  else
    hipLaunchKernelGGL(maxpool2c_bwd_kernel<float>, dim3(grid_n(n)), dim3(256), 0, st, B, H, W, C, (const float*)x,
                       (const float*)dout, (float*)dx);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_window_copy(int dtype, int B, int C, int Hs, int Ws, const void* src, int Hd, int Wd, void* dst,
                                 int oy, int ox, void* stream) {
  if (B <= 0 || C <= 0 || C % 8 || Hs <= 0 || Ws <= 0 || Hd <= 0 || Wd <= 0) return DFCSA_EINVAL;
  const int64_t n = (int64_t)B * Hd * Wd * (C / 8);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(window_copy_kernel<bf16_t>, dim3(grid_n(n)), dim3(256), 0, st, B, C, Hs, Ws,
                       (const bf16_t*)src, Hd, Wd, (bf16_t*)dst, oy, ox);
  else
    hipLaunchKernelGGL(window_copy_kernel<float>, dim3(grid_n(n)), dim3(256), 0, st, B, C, Hs, Ws, (const float*)src,
                       Hd, Wd, (float*)dst, oy, ox);
  DFCSA_CHECK_LAUNCH();
  return 0;
}
