// U-Net plumbing, weight packing and the loss/metric reduction.
//
// Reference call sites replaced (models/unet_dfc_sa_res.py unless noted):
//   nn.MaxPool2d(2, 2)                       :132-141 (+ its backward)
//   F.interpolate(bilinear) shape fix        :180-199 (only when a decoder size mismatches)
//   final_conv 1x1 head                      :159, :203
//   torch.sigmoid                            utils/trainer.py:124
//   BCELoss + dice_loss + IoU/Dice counts    utils/metrics.py:6-24, 52-78, 228-236
#include <algorithm>

#include "common.h"
#include "dfcsa_internal.h"

namespace {

inline int grid_for(int64_t n, int per = 256, int cap = 4096) {
  int64_t b = (n + per - 1) / per;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, cap));
}

// ---------------------------------------------------------------- max pooling 2x2 / 2
template <typename T>
__global__ void maxpool2_fwd_kernel(int B, int H, int W, int C, const T* __restrict__ x, T* __restrict__ y) {
  const int Ho = H / 2, Wo = W / 2, cpp = C >> 3;
  const int64_t total = (int64_t)B * Ho * Wo * cpp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t p = e / cpp;
    const int ow = (int)(p % Wo);
    p /= Wo;
    const int oh = (int)(p % Ho);
    const int b = (int)(p / Ho);
    float best[8], v[8];
    const T* base = x + ((size_t)(b * H + 2 * oh) * W + 2 * ow) * C + ck * 8;
    load8<T>(base, best);
#pragma unroll
    for (int t = 1; t < 4; ++t) {
      load8<T>(base + ((size_t)(t >> 1) * W + (t & 1)) * C, v);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (v[q] > best[q] || isnan(v[q])) best[q] = v[q];
    }
    store8<T>(y + ((size_t)(b * Ho + oh) * Wo + ow) * C + ck * 8, best);
  }
}

// dx += dout at the first maximum (scan order (0,0),(0,1),(1,0),(1,1); NaN wins), as ATen
template <typename T>
__global__ void maxpool2_bwd_kernel(int B, int H, int W, int C, const T* __restrict__ x, const T* __restrict__ dy,
                                    T* __restrict__ dx) {
  const int Ho = H / 2, Wo = W / 2, cpp = C >> 3;
  const int64_t total = (int64_t)B * Ho * Wo * cpp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t p = e / cpp;
    const int ow = (int)(p % Wo);
    p /= Wo;
    const int oh = (int)(p % Ho);
    const int b = (int)(p / Ho);
    float best[8], v[8], g[8];
    int arg[8];
    const size_t base = ((size_t)(b * H + 2 * oh) * W + 2 * ow) * C + ck * 8;
    load8<T>(x + base, best);
#pragma unroll
    for (int q = 0; q < 8; ++q) arg[q] = 0;
#pragma unroll
    for (int t = 1; t < 4; ++t) {
      load8<T>(x + base + ((size_t)(t >> 1) * W + (t & 1)) * C, v);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (v[q] > best[q] || isnan(v[q])) { best[q] = v[q]; arg[q] = t; }
    }
    load8<T>(dy + ((size_t)(b * Ho + oh) * Wo + ow) * C + ck * 8, g);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      T* dst = dx + base + ((size_t)(t >> 1) * W + (t & 1)) * C;
      float o[8];
      load8<T>(dst, o);
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] += (arg[q] == t) ? g[q] : 0.f;
      store8<T>(dst, o);
    }
  }
}

// ---------------------------------------------------------------- layout conversion
template <typename T>
__global__ void pack_input_kernel(int B, int Cin, int H, int W, const float* __restrict__ x, int Cpad,
                                  T* __restrict__ out) {
  const int64_t total = (int64_t)B * H * W;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < total; p += (int64_t)gridDim.x * 256) {
    const int hw = (int)(p % ((int64_t)H * W));
    const int b = (int)(p / ((int64_t)H * W));
    for (int c0 = 0; c0 < Cpad; c0 += 8) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        int c = c0 + q;
        v[q] = c < Cin ? x[((size_t)b * Cin + c) * H * W + hw] : 0.f;
      }
      store8<T>(out + (size_t)p * Cpad + c0, v);
    }
  }
}

__device__ __forceinline__ void bilin_axis(int dst, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  float scale = (float)in / (float)out;
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  l0 = 1.f - l1;
}

template <typename T>
__global__ void resize_kernel(int B, int C, int Hi, int Wi, int Ho, int Wo, const T* __restrict__ x,
                              T* __restrict__ y) {
  const int cpp = C >> 3;
  const int64_t total = (int64_t)B * Ho * Wo * cpp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t p = e / cpp;
    const int ow = (int)(p % Wo);
    p /= Wo;
    const int oh = (int)(p % Ho);
    const int b = (int)(p / Ho);
    int h0, h1, w0, w1;
    float lh0, lh1, lw0, lw1;
    bilin_axis(oh, Hi, Ho, h0, h1, lh0, lh1);
    bilin_axis(ow, Wi, Wo, w0, w1, lw0, lw1);
    const T* xb = x + (size_t)b * Hi * Wi * C + ck * 8;
    float a[8], bq[8], c[8], d[8], o[8];
    load8<T>(xb + ((size_t)h0 * Wi + w0) * C, a);
    load8<T>(xb + ((size_t)h0 * Wi + w1) * C, bq);
    load8<T>(xb + ((size_t)h1 * Wi + w0) * C, c);
    load8<T>(xb + ((size_t)h1 * Wi + w1) * C, d);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = lh0 * (lw0 * a[q] + lw1 * bq[q]) + lh1 * (lw0 * c[q] + lw1 * d[q]);
    store8<T>(y + (size_t)e * 8, o);
  }
}

template <typename T>
__global__ void resize_bwd_kernel(int B, int C, int Hi, int Wi, int Ho, int Wo, const T* __restrict__ dy,
                                  float* __restrict__ dx) {
  const int cpp = C >> 3;
  const int64_t total = (int64_t)B * Ho * Wo * cpp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t p = e / cpp;
    const int ow = (int)(p % Wo);
    p /= Wo;
    const int oh = (int)(p % Ho);
    const int b = (int)(p / Ho);
    int h0, h1, w0, w1;
    float lh0, lh1, lw0, lw1;
    bilin_axis(oh, Hi, Ho, h0, h1, lh0, lh1);
    bilin_axis(ow, Wi, Wo, w0, w1, lw0, lw1);
    float g[8];
    load8<T>(dy + (size_t)e * 8, g);
    float* xb = dx + (size_t)b * Hi * Wi * C + ck * 8;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      atomicAdd(xb + ((size_t)h0 * Wi + w0) * C + q, lh0 * lw0 * g[q]);
      atomicAdd(xb + ((size_t)h0 * Wi + w1) * C + q, lh0 * lw1 * g[q]);
      atomicAdd(xb + ((size_t)h1 * Wi + w0) * C + q, lh1 * lw0 * g[q]);
      atomicAdd(xb + ((size_t)h1 * Wi + w1) * C + q, lh1 * lw1 * g[q]);
    }
  }
}

template <typename T>
__global__ void cast_f32_kernel(int64_t n, const float* __restrict__ x, T* __restrict__ out, int accumulate) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float v = x[i];
    if (accumulate) v += ElemTraits<T>::to_f(out[i]);
    out[i] = ElemTraits<T>::from_f(v);
  }
}

// ---------------------------------------------------------------- 1x1 head (N = Cout small)
template <typename T>
__global__ void head_fwd_kernel(int B, int HW, int C, int Cout, const T* __restrict__ x, const float* __restrict__ w,
                                const float* __restrict__ bias, float* __restrict__ out) {
  const int64_t M = (int64_t)B * HW;
  for (int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x; m < M; m += (int64_t)gridDim.x * 256) {
    const int b = (int)(m / HW), hw = (int)(m % HW);
    for (int o = 0; o < Cout; ++o) {
      float s = bias ? bias[o] : 0.f;
      for (int c0 = 0; c0 < C; c0 += 8) {
        float v[8];
        load8<T>(x + (size_t)m * C + c0, v);
#pragma unroll
        for (int q = 0; q < 8; ++q) s += v[q] * w[(size_t)o * C + c0 + q];
      }
      out[((size_t)b * Cout + o) * HW + hw] = s;
    }
  }
}

// dx = dlogit @ w ; per-tile partial sums for dw and db (tile = 256 pixels)
template <typename T>
__global__ void __launch_bounds__(256) head_bwd_kernel(int B, int HW, int C, int Cout, const T* __restrict__ x,
                                                       const float* __restrict__ w, const float* __restrict__ dl,
                                                       T* __restrict__ dx, float* __restrict__ pw,
                                                       float* __restrict__ pb) {
  extern __shared__ float sred[];  // [256][Cout]
  const int64_t M = (int64_t)B * HW;
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float g[8];
  for (int o = 0; o < Cout && o < 8; ++o) g[o] = 0.f;
  if (m < M) {
    const int b = (int)(m / HW), hw = (int)(m % HW);
    for (int o = 0; o < Cout; ++o) g[o] = dl[((size_t)b * Cout + o) * HW + hw];
    for (int c0 = 0; c0 < C; c0 += 8) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float s = 0.f;
        for (int o = 0; o < Cout; ++o) s += g[o] * w[(size_t)o * C + c0 + q];
        v[q] = s;
      }
      store8<T>(dx + (size_t)m * C + c0, v);
    }
  }
  for (int o = 0; o < Cout; ++o) sred[threadIdx.x * Cout + o] = g[o];
  __syncthreads();
  // dw[o][c] partial over this tile's pixels: thread t handles (o, c) pairs
  const int64_t m0 = (int64_t)blockIdx.x * 256;
  const int np = (int)std::min<int64_t>(256, M - m0);
  for (int e = threadIdx.x; e < Cout * C; e += 256) {
    const int o = e / C, c = e % C;
    float s = 0.f;
    for (int p = 0; p < np; ++p) s += sred[p * Cout + o] * ElemTraits<T>::to_f(x[(size_t)(m0 + p) * C + c]);
    pw[(size_t)blockIdx.x * Cout * C + e] = s;
  }
  for (int o = threadIdx.x; o < Cout; o += 256) {
    float s = 0.f;
    for (int p = 0; p < np; ++p) s += sred[p * Cout + o];
    pb[(size_t)blockIdx.x * Cout + o] = s;
  }
}

// Fast head paths: cpp = C/8 lanes cooperate on one pixel (cpp a power of two <= 64), so one
// wave-instruction loads 1 KB contiguous; weights live in registers.
template <typename T, int NO>
__global__ void __launch_bounds__(256) head_fwd_fast_kernel(int B, int HW, int C, const T* __restrict__ x,
                                                            const float* __restrict__ w, const float* __restrict__ bias,
                                                            float* __restrict__ out) {
  const int cpp = C >> 3;
  const int lane = threadIdx.x & 63, sub = lane & (cpp - 1);
  const int ppw = 64 / cpp;                                 // pixels per wave
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6, nwaves = gridDim.x * 4;
  float wr[NO][8];
#pragma unroll
  for (int o = 0; o < NO; ++o)
#pragma unroll
    for (int q = 0; q < 8; ++q) wr[o][q] = w[o * C + sub * 8 + q];
  const int64_t M = (int64_t)B * HW;
  for (int64_t m0 = (int64_t)wave * ppw; m0 < M; m0 += (int64_t)nwaves * ppw) {
    const int64_t m = m0 + lane / cpp;
    float v[8];
    float s[NO];
    const bool ok = m < M;
    if (ok) load8<T>(x + m * C + sub * 8, v);
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      float a = 0.f;
      if (ok)
#pragma unroll
        for (int q = 0; q < 8; ++q) a += v[q] * wr[o][q];
      for (int k = 1; k < cpp; k <<= 1) a += __shfl_xor(a, k, 64);
      s[o] = a;
    }
    if (ok && sub == 0) {
      const int b = (int)(m / HW), hw = (int)(m % HW);
#pragma unroll
      for (int o = 0; o < NO; ++o) out[((size_t)b * NO + o) * HW + hw] = s[o] + (bias ? bias[o] : 0.f);
    }
  }
}

// dx = dl @ w; per-block partial dw[o][c] = sum g_o x_c and db[o] = sum g_o over the block's pixels
template <typename T, int NO>
__global__ void __launch_bounds__(256) head_bwd_fast_kernel(int B, int HW, int C, const T* __restrict__ x,
                                                            const float* __restrict__ w, const float* __restrict__ dl,
                                                            T* __restrict__ dx, float* __restrict__ pw,
                                                            float* __restrict__ pb) {
  const int cpp = C >> 3;
  const int lane = threadIdx.x & 63, sub = lane & (cpp - 1);
  const int ppw = 64 / cpp;
  const int wave_in_blk = threadIdx.x >> 6;
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6, nwaves = gridDim.x * 4;
  float wr[NO][8], aw[NO][8], ab[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    ab[o] = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) { wr[o][q] = w[o * C + sub * 8 + q]; aw[o][q] = 0.f; }
  }
  const int64_t M = (int64_t)B * HW;
  for (int64_t m0 = (int64_t)wave * ppw; m0 < M; m0 += (int64_t)nwaves * ppw) {
    const int64_t m = m0 + lane / cpp;
    if (m >= M) continue;
    const int b = (int)(m / HW), hw = (int)(m % HW);
    float g[NO], v[8], d[8];
#pragma unroll
    for (int o = 0; o < NO; ++o) g[o] = dl[((size_t)b * NO + o) * HW + hw];
    load8<T>(x + m * C + sub * 8, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float a = 0.f;
#pragma unroll
      for (int o = 0; o < NO; ++o) { a += g[o] * wr[o][q]; aw[o][q] += g[o] * v[q]; }
      d[q] = a;
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) ab[o] += (sub == 0) ? g[o] : 0.f;
    store8<T>(dx + m * C + sub * 8, d);
  }
  // reduce over the lanes that share `sub` (pixel groups) within the wave, then across waves
#pragma unroll
  for (int o = 0; o < NO; ++o) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      for (int k = cpp; k < 64; k <<= 1) aw[o][q] += __shfl_xor(aw[o][q], k, 64);
    for (int k = 1; k < 64; k <<= 1) ab[o] += __shfl_xor(ab[o], k, 64);
  }
  __shared__ float red[4][NO][512 + 1];
  if (lane < cpp) {
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int q = 0; q < 8; ++q) red[wave_in_blk][o][sub * 8 + q] = aw[o][q];
  }
  if (lane == 0)
#pragma unroll
    for (int o = 0; o < NO; ++o) red[wave_in_blk][o][512] = ab[o];
  __syncthreads();
  for (int e = threadIdx.x; e < NO * C; e += 256) {
    const int o = e / C, c = e % C;
    pw[(size_t)blockIdx.x * NO * C + e] = red[0][o][c] + red[1][o][c] + red[2][o][c] + red[3][o][c];
  }
  if (threadIdx.x < NO)
    pb[(size_t)blockIdx.x * NO + threadIdx.x] =
        red[0][threadIdx.x][512] + red[1][threadIdx.x][512] + red[2][threadIdx.x][512] + red[3][threadIdx.x][512];
}

constexpr int kHeadBwdBlocks = 1024;

inline bool head_fast_ok(int C, int Cout) {
  const int cpp = C / 8;
  return C % 8 == 0 && cpp >= 1 && cpp <= 64 && (cpp & (cpp - 1)) == 0 && Cout >= 1 && Cout <= 4;
}

// ---------------------------------------------------------------- weight packing
template <typename T>
__global__ void pack_conv_w_kernel(const float* __restrict__ w, int Cout, int Cin, int ntaps, int Cpad, int Kpad,
                                   int row0, T* __restrict__ out) {
  const int64_t total = (int64_t)Cout * Kpad;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int co = (int)(e / Kpad), k = (int)(e % Kpad);
    const int tap = k / Cpad, ci = k - tap * Cpad;
    float v = 0.f;
    if (tap < ntaps && ci < Cin) v = w[((size_t)co * Cin + ci) * ntaps + tap];
    out[(size_t)(row0 + co) * Kpad + k] = ElemTraits<T>::from_f(v);
  }
}

template <typename T>
__global__ void pack_conv_w_t_kernel(const float* __restrict__ w, int Cout, int Cin, int ntaps, int Kpad, int col0,
                                     T* __restrict__ out) {
  const int64_t total = (int64_t)Cin * ntaps * Cout;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int co = (int)(e % Cout);
    int64_t r = e / Cout;
    const int tap = (int)(r % ntaps);
    const int ci = (int)(r / ntaps);
    out[(size_t)ci * Kpad + col0 + tap * Cout + co] = ElemTraits<T>::from_f(w[((size_t)co * Cin + ci) * ntaps + tap]);
  }
}

template <typename T>
__global__ void pack_t3_kernel(int Cin, int Kpad, int wcin, const float* __restrict__ w0, int c0, int t0,
                               const float* __restrict__ w1, int c1, int t1, const float* __restrict__ w2, int c2,
                               int t2, int ident2, T* __restrict__ out) {
  const int64_t total = (int64_t)Cin * Kpad;
  const int e0 = t0 * c0, e1 = e0 + t1 * c1, e2 = e1 + t2 * c2;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ci = (int)(e / Kpad), k = (int)(e % Kpad);
    float v = 0.f;
    if (k < e0) {
      const int tap = k / c0, co = k - tap * c0;
      if (ci < wcin) v = w0[((size_t)co * wcin + ci) * t0 + tap];
    } else if (k < e1) {
      const int kk = k - e0, tap = kk / c1, co = kk - tap * c1;
      if (ci < wcin) v = w1[((size_t)co * wcin + ci) * t1 + tap];
    } else if (k < e2) {
      const int kk = k - e1, tap = kk / c2, co = kk - tap * c2;
      if (ident2) v = (ci == co ? 1.f : 0.f);
      else if (ci < wcin) v = w2[((size_t)co * wcin + ci) * t2 + tap];
    }
    out[e] = ElemTraits<T>::from_f(v);
  }
}

template <typename T>
__global__ void pack_convT_kernel(const float* __restrict__ w, const float* __restrict__ bias, int Cin, int Cout,
                                  T* __restrict__ fwd, T* __restrict__ bwd, float* __restrict__ bias4) {
  const int64_t total = (int64_t)Cin * Cout * 4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ij = (int)(e & 3);
    const int64_t r = e >> 2;
    const int co = (int)(r % Cout), ci = (int)(r / Cout);
    const T v = ElemTraits<T>::from_f(w[e]);
    fwd[((size_t)ij * Cout + co) * Cin + ci] = v;
    bwd[(size_t)ci * 4 * Cout + ij * Cout + co] = v;
    if (ci == 0) bias4[ij * Cout + co] = bias[co];
  }
}

// ---------------------------------------------------------------- one-launch pack plan
// One workgroup per task; an entry owns tasks [start, start + count).  Entries are few (~150),
// tasks many, so the entry lookup is a binary search per workgroup.
__device__ __forceinline__ float load_as(const void* p, int64_t i, int dtype) {
  return dtype == DFCSA_DT_BF16 ? bf2f(((const bf16_t*)p)[i]) : ((const float*)p)[i];
}
__device__ __forceinline__ void store_as(void* out, int64_t i, int dtype, float v) {
  if (dtype == DFCSA_DT_BF16) ((bf16_t*)out)[i] = f2bf(v);
  else ((float*)out)[i] = v;
}

// LDS slot of staged element s in the ROWS case: one pad float after every q = 8*ntaps floats.
// A lane reads 8 consecutive ci of one tap (a stride of ntaps), the lanes of a group a stride of
// 8*ntaps apart: unpadded, 1x1-like and 2x2 (ConvTranspose) rows put 4-32 lanes on one bank; padded,
// rows of >= 128 channels are conflict-free (<= 2-way below).  s < 4096 and q <= 8*49, so the
// float quotient is exact.
__device__ __forceinline__ int rows_slot(int s, float rq) { return s + (int)(((float)s + 0.5f) * rq); }
// 64 x 64 transpose tile: row stride 69 (odd, >= 64 + 4) plus 4 words after 32 rows and after
// 32 columns, so the 8-wide row chunks written by a ds_write_b32 group (4 rows x 8 chunks) and the
// 8-row column chunks it reads (4 columns x 8 chunks) both fall on 32 distinct banks, and so do
// the scalar path's rows (32 columns) and columns (32 rows, stride 69 = 5 mod 32)
__device__ __forceinline__ int tile_at(int r, int c) { return r * 69 + c + 4 * ((r >> 5) + (c >> 5)); }

__global__ void __launch_bounds__(256) pack_plan_kernel(const dfcsa_pack_entry* __restrict__ tab, int n) {
  __shared__ float smem[4420];   // ROWS: 4096 staged floats + pads (q >= 16); TRANSPOSE: tile_at < 4420
  const int64_t task = blockIdx.x;
  // last entry with start <= task = (number of entries with start <= task) - 1 (starts ascend,
  // start[0] = 0): every lane tests four entries per 256, all loads in flight, counted by ballot
  // (a binary search was eight dependent L2 round trips per workgroup)
  int cnt = 0;
  const int lane64 = threadIdx.x & 63;
  for (int base = 0; base < n; base += 256) {
    int64_t st[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) st[u] = tab[min(base + u * 64 + lane64, n - 1)].start;
#pragma unroll
    for (int u = 0; u < 4; ++u) cnt += __popcll(__ballot(base + u * 64 + lane64 < n && st[u] <= task));
  }
  const int lo = cnt - 1;
  const dfcsa_pack_entry& t = tab[lo];
  const int64_t tl = task - t.start;
  if (tl >= t.count) return;
  const int* a = t.a;
  const int tid = threadIdx.x;
  switch (t.kind) {
    case DFCSA_PACK_ROWS: {
      // out[(row0 + co)*Kpad + tap*Cpad + ci] = w[co][ci][tap].  The task's rows (or, for rows
      // longer than 4096 floats, one row's input-channel chunk) are a contiguous source block of
      // <= 4096 floats: it is staged in LDS by sixteen unconditional loads per lane, all in flight
      // (clamped index past the end), and written in output order (consecutive ci: coalesced),
      // reading LDS at a stride of ntaps (padded, rows_slot).  A 1x1 conv (ntaps = 1) is a plain
      // row copy and skips the staging.
      const int Cout = a[0], Cin = a[1], ntaps = a[2], Cpad = a[3], Kpad = a[4], row0 = a[5], per = a[6];
      const int nrow = Cin * ntaps;
      const int co0 = (int)tl * per, nr = min(per, Cout - co0);
      const float* __restrict__ w = t.w0;
      const bool vec = t.dtype == DFCSA_DT_BF16 && Cin % 8 == 0 && Cpad % 8 == 0 && Kpad % 8 == 0 &&
                       ((uintptr_t)t.out & 15) == 0;
      if (ntaps == 1) {
        const float* __restrict__ src = w + (size_t)co0 * Cin;
        const int n1 = nr * Cin;
        if (vec && ((uintptr_t)w & 15) == 0) {
          for (int o = tid * 8; o < n1; o += 256 * 8) {
            const int r = o / Cin, ci = o - r * Cin;
            const float4 x0 = *(const float4*)(src + o), x1 = *(const float4*)(src + o + 4);
            const float v8[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            store8<bf16_t>((bf16_t*)t.out + (int64_t)(row0 + co0 + r) * Kpad + ci, v8);
          }
        } else {
          for (int o = tid; o < n1; o += 256) {
            const int r = o / Cin, ci = o - r * Cin;
            store_as(t.out, (int64_t)(row0 + co0 + r) * Kpad + ci, t.dtype, src[o]);
          }
        }
        break;
      }
      const int ccmax = nrow <= 4096 ? Cin : max(vec ? 8 : 1, (4096 / ntaps) & (vec ? ~7 : ~0));
      const float rq = 1.f / (float)(8 * ntaps);
      for (int c0 = 0; c0 < Cin; c0 += ccmax) {
        const int cc = min(ccmax, Cin - c0), rl = cc * ntaps, n = nr * rl;   // n <= 4096
        const float* __restrict__ src = w + (size_t)co0 * nrow + (size_t)c0 * ntaps;
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = src[min(tid + u * 256, n - 1)];
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (tid + u * 256 < n) smem[rows_slot(tid + u * 256, rq)] = v[u];
        __syncthreads();
        if (vec) {
          // 8 consecutive ci of one tap per lane: one 16-B store (cc % 8 == 0)
          for (int o = tid * 8; o < n; o += 256 * 8) {
            const int r = o / rl, rem = o - r * rl, tap = rem / cc, ci = rem - tap * cc;
            const int s0 = r * rl + ci * ntaps + tap;
            float v8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v8[j] = smem[rows_slot(s0 + j * ntaps, rq)];
            store8<bf16_t>((bf16_t*)t.out + (int64_t)(row0 + co0 + r) * Kpad + tap * Cpad + c0 + ci, v8);
          }
        } else {
          for (int o = tid; o < n; o += 256) {
            const int r = o / rl, rem = o - r * rl, tap = rem / cc, ci = rem - tap * cc;
            store_as(t.out, (int64_t)(row0 + co0 + r) * Kpad + tap * Cpad + c0 + ci, t.dtype,
                     smem[rows_slot(r * rl + ci * ntaps + tap, rq)]);
          }
        }
        __syncthreads();
      }
      break;
    }
    case DFCSA_PACK_TRANSPOSE: {
      // dst[c*ldd + r] = src[r*lds + c] for r < R, c < C (elements of `dtype`), 64x64 tiles
      const int R = a[0], C = a[1], lds = a[2], ldd = a[3], tc = a[4];
      const int r0 = (int)(tl / tc) * 64, c0 = (int)(tl % tc) * 64;
      const int lane = tid & 63, q = tid >> 6;
      if (t.dtype == DFCSA_DT_BF16 && lds % 8 == 0 && ldd % 8 == 0 && ((uintptr_t)t.w0 & 15) == 0 &&
          ((uintptr_t)t.out & 15) == 0) {
        // 16-B loads of 8 consecutive columns and 16-B stores of 8 consecutive rows (partial
        // chunks at the R / C edges element by element)
        for (int e = tid; e < 512; e += 256) {
          const int i = e >> 3, k = (e & 7) * 8, rr = r0 + i, cc = c0 + k;
          if (rr >= R) continue;
          const bf16_t* sp = (const bf16_t*)t.w0 + (int64_t)rr * lds + cc;
          if (cc + 8 <= C) {
            float v[8];
            load8<bf16_t>(sp, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) smem[tile_at(i, k + j)] = v[j];
          } else {
            for (int j = 0; j < 8 && cc + j < C; ++j) smem[tile_at(i, k + j)] = bf2f(sp[j]);
          }
        }
        __syncthreads();
        for (int e = tid; e < 512; e += 256) {
          const int ci = e >> 3, k = (e & 7) * 8, cc = c0 + ci, rr = r0 + k;
          if (cc >= C || rr >= R) continue;
          bf16_t* dp = (bf16_t*)t.out + (int64_t)cc * ldd + rr;
          if (rr + 8 <= R) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = smem[tile_at(k + j, ci)];
            store8<bf16_t>(dp, v);
          } else {
            for (int j = 0; j < 8 && rr + j < R; ++j) dp[j] = f2bf(smem[tile_at(k + j, ci)]);
          }
        }
        break;
      }
      for (int i = 0; i < 16; ++i) {
        const int rr = r0 + i * 4 + q, cc = c0 + lane;
        if (rr < R && cc < C) smem[tile_at(i * 4 + q, lane)] = load_as(t.w0, (int64_t)rr * lds + cc, t.dtype);
      }
      __syncthreads();
      for (int i = 0; i < 16; ++i) {
        const int cc = c0 + i * 4 + q, rr = r0 + lane;
        if (rr < R && cc < C) store_as(t.out, (int64_t)cc * ldd + rr, t.dtype, smem[tile_at(lane, i * 4 + q)]);
      }
      break;
    }
    case DFCSA_PACK_CONCAT: {
      const int n0 = a[0], n1 = a[1], n2 = a[2], total = a[3];
      for (int i = tid; i < total; i += 256) {
        float v = 0.f;
        if (i < n0) v = t.w0[i];
        else if (i < n0 + n1) v = t.w1[i - n0];
        else if (i < n0 + n1 + n2) v = t.w2[i - n0 - n1];
        ((float*)t.out)[i] = v;
      }
      break;
    }
    case DFCSA_PACK_BIAS4: {
      for (int i = tid; i < 4 * a[0]; i += 256) ((float*)t.out)[i] = t.w0[i % a[0]];
      break;
    }
    default:
      break;
  }
}

// ---------------------------------------------------------------- sigmoid / loss
__global__ void sigmoid_kernel(int64_t n, const float* __restrict__ x, float* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[i] = 1.f / (1.f + expf(-x[i]));
}
__global__ void sigmoid_bwd_kernel(int64_t n, const float* __restrict__ y, const float* __restrict__ dy,
                                   float* __restrict__ dx) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = y[i];
    dx[i] = dy[i] * (1.f - v) * v;
  }
}

constexpr int kLossBlocks = 512;

// partial[blk][6] = {sum bce, sum p*t, sum p, sum t, sum b*t, sum b}
__global__ void __launch_bounds__(256) bce_dice_partial_kernel(int64_t n, const float* __restrict__ p,
                                                               const float* __restrict__ t,
                                                               float* __restrict__ partial) {
  double acc[6] = {0, 0, 0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float pv = p[i], tv = t[i];
    const float lp = fmaxf(logf(pv), -100.f), l1p = fmaxf(log1pf(-pv), -100.f);
    const float bce = -(tv * lp + (1.f - tv) * l1p);
    const float b = pv > 0.5f ? 1.f : 0.f;
    acc[0] += bce; acc[1] += pv * tv; acc[2] += pv; acc[3] += tv; acc[4] += b * tv; acc[5] += b;
  }
  __shared__ double red[6][256];
  for (int k = 0; k < 6; ++k) red[k][threadIdx.x] = acc[k];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
      for (int k = 0; k < 6; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 6) partial[blockIdx.x * 6 + threadIdx.x] = (float)red[threadIdx.x][0];
}

__global__ void bce_dice_final_kernel(int64_t n, int nparts, const float* __restrict__ partial, float wbce,
                                      float wdice, float* __restrict__ stats) {
  __shared__ double red[6][64];
  double acc[6] = {0, 0, 0, 0, 0, 0};
  for (int i = threadIdx.x; i < nparts; i += 64)
    for (int k = 0; k < 6; ++k) acc[k] += partial[i * 6 + k];
  for (int k = 0; k < 6; ++k) red[k][threadIdx.x] = acc[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    double s[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 64; ++i)
      for (int k = 0; k < 6; ++k) s[k] += red[k][i];
    const float bce = (float)(s[0] / (double)n);
    const float inter = (float)s[1], ps = (float)s[2], ts = (float)s[3];
    const float dice = (2.f * inter + 1.f) / (ps + ts + 1.f);
    const float loss = wbce * bce + wdice * (1.f - dice);
    stats[0] = loss;
    stats[1] = (float)s[0];
    for (int k = 1; k < 6; ++k) stats[1 + k] = (float)s[k];
    stats[7] = isfinite(loss) ? 1.f : 0.f;
  }
}

// dp = dloss * (wbce * (p - t) / max((1 - p) p, 1e-12) / n + wdice * d(1 - dice)/dp)
__global__ void bce_dice_bwd_kernel(int64_t n, const float* __restrict__ p, const float* __restrict__ t,
                                    const float* __restrict__ stats, float wbce, float wdice,
                                    const float* __restrict__ dloss, float* __restrict__ dp) {
  const float g = dloss ? *dloss : 1.f;
  const float inter = stats[2], den = stats[3] + stats[4] + 1.f;
  const float num = 2.f * inter + 1.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float pv = p[i], tv = t[i];
    const float gb = (pv - tv) / fmaxf((1.f - pv) * pv, 1e-12f) / (float)n;
    // dice = num/den; d(1-dice)/dp = -(2 t den - num) / den^2
    const float gd = -(2.f * tv * den - num) / (den * den);
    dp[i] = g * (wbce * gb + wdice * gd);
  }
}

}  // namespace

extern "C" int dfcsa_maxpool2_fwd(int dtype, int B, int H, int W, int C, const void* x, void* out, void* stream) {
  if (C % 8) return DFCSA_EINVAL;
  int64_t n = (int64_t)B * (H / 2) * (W / 2) * (C / 8);
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(maxpool2_fwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, B, H, W, C,
                       (const bf16_t*)x, (bf16_t*)out);
  else
    hipLaunchKernelGGL(maxpool2_fwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, B, H, W, C, (const float*)x,
                       (float*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_maxpool2_bwd(int dtype, int B, int H, int W, int C, const void* x, const void* dout, void* dx,
                                  void* stream) {
  if (C % 8) return DFCSA_EINVAL;
  int64_t n = (int64_t)B * (H / 2) * (W / 2) * (C / 8);
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(maxpool2_bwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, B, H, W, C,
                       (const bf16_t*)x, (const bf16_t*)dout, (bf16_t*)dx);
  else
    hipLaunchKernelGGL(maxpool2_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, B, H, W, C, (const float*)x,
                       (const float*)dout, (float*)dx);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_pack_input(int dtype, int B, int Cin, int H, int W, const float* x, int Cpad, void* out,
                                void* stream) {
  if (Cpad % 8 || Cpad < Cin) return DFCSA_EINVAL;
  int64_t n = (int64_t)B * H * W;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(pack_input_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, B, Cin, H, W, x, Cpad,
                       (bf16_t*)out);
  else
    hipLaunchKernelGGL(pack_input_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, B, Cin, H, W, x, Cpad,
                       (float*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_resize_bilinear(int dtype, int B, int C, int Hi, int Wi, int Ho, int Wo, const void* x,
                                     void* out, void* stream) {
  if (C % 8) return DFCSA_EINVAL;
  int64_t n = (int64_t)B * Ho * Wo * (C / 8);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(resize_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, B, C, Hi, Wi, Ho, Wo,
                       (const bf16_t*)x, (bf16_t*)out);
  else
    hipLaunchKernelGGL(resize_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, B, C, Hi, Wi, Ho, Wo,
                       (const float*)x, (float*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_resize_bilinear_bwd(int dtype, int B, int C, int Hi, int Wi, int Ho, int Wo, const void* dout,
                                         float* dx32, void* stream) {
  if (C % 8) return DFCSA_EINVAL;
  int64_t n = (int64_t)B * Ho * Wo * (C / 8);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(resize_bwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, B, C, Hi, Wi, Ho, Wo,
                       (const bf16_t*)dout, dx32);
  else
    hipLaunchKernelGGL(resize_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, B, C, Hi, Wi, Ho, Wo,
                       (const float*)dout, dx32);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_cast_f32(int dtype, int64_t n, const float* x, void* out, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(cast_f32_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, n, x, (bf16_t*)out, accumulate);
  else
    hipLaunchKernelGGL(cast_f32_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, n, x, (float*)out, accumulate);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_head_fwd(int dtype, int B, int HW, int C, int Cout, const void* x, const float* w,
                              const float* b, float* logits, void* stream) {
  if (C % 8 || Cout < 1 || Cout > 8) return DFCSA_EINVAL;
  int64_t M = (int64_t)B * HW;
  hipStream_t st = (hipStream_t)stream;
  if (head_fast_ok(C, Cout)) {
    const int ppw = 64 / (C / 8);
    int blocks = (int)std::min<int64_t>(4096, (M / ppw + 3) / 4 + 1);
#define HF(NO)                                                                                             \
  if (Cout == NO) {                                                                                        \
    if (dtype == DFCSA_DT_BF16)                                                                            \
      hipLaunchKernelGGL((head_fwd_fast_kernel<bf16_t, NO>), dim3(blocks), dim3(256), 0, st, B, HW, C,       \
                         (const bf16_t*)x, w, b, logits);                                                  \
    else                                                                                                   \
      hipLaunchKernelGGL((head_fwd_fast_kernel<float, NO>), dim3(blocks), dim3(256), 0, st, B, HW, C,        \
                         (const float*)x, w, b, logits);                                                   \
  }
    HF(1) HF(2) HF(3) HF(4)
#undef HF
    DFCSA_CHECK_LAUNCH();
    return 0;
  }
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(head_fwd_kernel<bf16_t>, dim3(grid_for(M)), dim3(256), 0, st, B, HW, C, Cout,
                       (const bf16_t*)x, w, b, logits);
  else
    hipLaunchKernelGGL(head_fwd_kernel<float>, dim3(grid_for(M)), dim3(256), 0, st, B, HW, C, Cout, (const float*)x,
                       w, b, logits);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_head_bwd(int dtype, int B, int HW, int C, int Cout, const void* x, const float* w,
                              const float* dlogit, void* dx, float* partial_w, float* partial_b, int* ntiles,
                              void* stream) {
  if (C % 8 || Cout < 1 || Cout > 8) return DFCSA_EINVAL;
  int64_t M = (int64_t)B * HW;
  const bool fast = head_fast_ok(C, Cout);
  int blocks = fast ? kHeadBwdBlocks : (int)((M + 255) / 256);
  if (ntiles) *ntiles = blocks;
  if (!partial_w) return 0;  // size query
  hipStream_t st = (hipStream_t)stream;
  if (fast) {
#define HB(NO)                                                                                             \
  if (Cout == NO) {                                                                                        \
    if (dtype == DFCSA_DT_BF16)                                                                            \
      hipLaunchKernelGGL((head_bwd_fast_kernel<bf16_t, NO>), dim3(blocks), dim3(256), 0, st, B, HW, C,       \
                         (const bf16_t*)x, w, dlogit, (bf16_t*)dx, partial_w, partial_b);                  \
    else                                                                                                   \
      hipLaunchKernelGGL((head_bwd_fast_kernel<float, NO>), dim3(blocks), dim3(256), 0, st, B, HW, C,        \
                         (const float*)x, w, dlogit, (float*)dx, partial_w, partial_b);                    \
  }
    HB(1) HB(2) HB(3) HB(4)
#undef HB
    DFCSA_CHECK_LAUNCH();
    return 0;
  }
  size_t shm = (size_t)256 * Cout * sizeof(float);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(head_bwd_kernel<bf16_t>, dim3(blocks), dim3(256), shm, st, B, HW, C, Cout, (const bf16_t*)x,
                       w, dlogit, (bf16_t*)dx, partial_w, partial_b);
  else
    hipLaunchKernelGGL(head_bwd_kernel<float>, dim3(blocks), dim3(256), shm, st, B, HW, C, Cout, (const float*)x, w,
                       dlogit, (float*)dx, partial_w, partial_b);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_pack_conv_w(int dtype, const float* w, int Cout, int Cin, int ntaps, int Cpad, int Kpad,
                                 int row0, void* out, void* stream) {
  if (Cpad < Cin || Kpad < ntaps * Cpad) return DFCSA_EINVAL;
  int64_t n = (int64_t)Cout * Kpad;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(pack_conv_w_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, w, Cout, Cin, ntaps, Cpad,
                       Kpad, row0, (bf16_t*)out);
  else
    hipLaunchKernelGGL(pack_conv_w_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, w, Cout, Cin, ntaps, Cpad,
                       Kpad, row0, (float*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_pack_conv_w_t(int dtype, const float* w, int Cout, int Cin, int ntaps, int Kpad, int col0,
                                   void* out, void* stream) {
  if (col0 + ntaps * Cout > Kpad) return DFCSA_EINVAL;
  int64_t n = (int64_t)Cin * ntaps * Cout;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(pack_conv_w_t_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, w, Cout, Cin, ntaps, Kpad,
                       col0, (bf16_t*)out);
  else
    hipLaunchKernelGGL(pack_conv_w_t_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, w, Cout, Cin, ntaps, Kpad,
                       col0, (float*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_pack_t3(int dtype, int Cin, int Kpad, int wcin, const float* w0, int cout0, int ntaps0, const float* w1,
                             int cout1, int ntaps1, const float* w2, int cout2, int ntaps2, int identity2, void* out,
                             void* stream) {
  if (!w0) { cout0 = 0; ntaps0 = 1; }
  if (!w1) { cout1 = 0; ntaps1 = 1; }
  if (!w2 && !identity2) { cout2 = 0; ntaps2 = 1; }
  if (identity2) ntaps2 = 1;
  if (ntaps0 * cout0 + ntaps1 * cout1 + ntaps2 * cout2 > Kpad) return DFCSA_EINVAL;
  int64_t n = (int64_t)Cin * Kpad;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(pack_t3_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, Cin, Kpad, wcin, w0, cout0, ntaps0, w1,
                       cout1, ntaps1, w2, cout2, ntaps2, identity2, (bf16_t*)out);
  else
    hipLaunchKernelGGL(pack_t3_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, Cin, Kpad, wcin, w0, cout0, ntaps0, w1,
                       cout1, ntaps1, w2, cout2, ntaps2, identity2, (float*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_pack_convT_w(int dtype, const float* w, const float* bias, int Cin, int Cout, void* out_fwd,
                                  void* out_bwd, float* bias4, void* stream) {
  int64_t n = (int64_t)Cin * Cout * 4;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(pack_convT_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, w, bias, Cin, Cout,
                       (bf16_t*)out_fwd, (bf16_t*)out_bwd, bias4);
  else
    hipLaunchKernelGGL(pack_convT_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, w, bias, Cin, Cout,
                       (float*)out_fwd, (float*)out_bwd, bias4);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_pack_plan(const dfcsa_pack_entry* table_dev, int n, int64_t total, void* stream) {
  if (!table_dev || n <= 0 || total <= 0 || total > (1 << 30)) return DFCSA_EINVAL;
  hipLaunchKernelGGL(pack_plan_kernel, dim3((unsigned)total), dim3(256), 0, (hipStream_t)stream, table_dev, n);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_zero(void* p, int64_t bytes, void* stream) {
  hipError_t e = hipMemsetAsync(p, 0, (size_t)bytes, (hipStream_t)stream);
  return e == hipSuccess ? 0 : -(int)e;
}

extern "C" int dfcsa_sigmoid(int64_t n, const float* x, float* y, void* stream) {
  hipLaunchKernelGGL(sigmoid_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, n, x, y);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_sigmoid_bwd(int64_t n, const float* y, const float* dy, float* dx, void* stream) {
  hipLaunchKernelGGL(sigmoid_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, n, y, dy, dx);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_bce_dice_partial_count(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(kLossBlocks, (n + 255) / 256));
}

extern "C" int dfcsa_bce_dice_fwd(int64_t n, const float* p, const float* t, float* partial, float wbce, float wdice,
                                  float* stats, void* stream) {
  if (n <= 0) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  int nb = dfcsa_bce_dice_partial_count(n);
  hipLaunchKernelGGL(bce_dice_partial_kernel, dim3(nb), dim3(256), 0, st, n, p, t, partial);
  DFCSA_CHECK_LAUNCH();
  hipLaunchKernelGGL(bce_dice_final_kernel, dim3(1), dim3(64), 0, st, n, nb, partial, wbce, wdice, stats);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_bce_dice_bwd(int64_t n, const float* p, const float* t, const float* stats, float wbce,
                                  float wdice, const float* dloss, float* dp, void* stream) {
  hipLaunchKernelGGL(bce_dice_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, n, p, t, stats, wbce,
                     wdice, dloss, dp);
  DFCSA_CHECK_LAUNCH();
  return 0;
}
