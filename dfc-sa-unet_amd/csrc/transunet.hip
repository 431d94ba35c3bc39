// TransUNet (R50-ViT-B/16) kernels: BASELINE config 4, reference models/transformer_unet.py.
//
// The ResNetV2 hybrid stem, the ViT encoder and the DecoderCup reuse the implicit-GEMM conv
// engine (conv_gemm.hip / wgrad.hip) for every convolution and linear layer; this file holds the
// operations the DFC-SA-Res path does not have:
//   StdConv2d weight standardisation        transformer_unet.py:21-27   wstd_fwd / wstd_bwd
//   root 7x7/s2 conv input gather           :77                         im2col_input
//   GroupNorm (+ residual, ReLU)            :46-67, :78-79              gn_*
//   MaxPool2d(3, 2, padding=1)              :101                        maxpool3s2_*
//   strided-conv data gradient              :36, :55 (stride 2)         col2im
//   LayerNorm                               :206-207, :226              ln_*
//   Dropout / GELU / residual adds          :164-172, :198, :211-220    drop_add / gelu_drop
//   multi-head self-attention core          :137-157                    mha_fwd / mha_bwd
//   UpsamplingBilinear2d(2) (align_corners) :262                        upsample2_ac_*
//   skip concat with unequal widths         :267                        copy_cols
//   SegmentationHead 3x3 conv (+bias)       :272-276                    head3_*
// Layouts: NHWC activations ([M][C], M = B*H*W, C % 8 == 0); token activations are the NHWC
// tensors of the patch grid (so "tokens x hidden" needs no transpose).  The ViT residual stream
// is fp32 in every precision mode.  All reductions are deterministic (no float atomics).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "common.h"
#include "dfcsa_internal.h"

namespace {

inline int grid_for(int64_t n, int per = 256, int cap = 8192) {
  int64_t b = (n + per - 1) / per;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, cap));
}

__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8f(float* p, const float (&v)[8]) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
template <typename T>
__device__ __forceinline__ void load16(const T* p, float (&v)[16]) {
  load8<T>(p, *(float(*)[8])v);
  load8<T>(p + 8, *(float(*)[8])(v + 8));
}
template <typename T>
__device__ __forceinline__ void store16(T* p, const float (&v)[16]) {
  store8<T>(p, *(const float(*)[8])v);
  store8<T>(p + 8, *(const float(*)[8])(v + 8));
}

// ------------------------------------------------------------ StdConv2d weight standardisation
// what[r][k] = (w[r][k] - mean_r) * rstd_r, rstd_r = 1/sqrt(var_r + 1e-5) (biased variance over
// the Cin*kh*kw row, torch.var_mean(unbiased=False), transformer_unet.py:24-25).  One wave per row;
// one table covers every StdConv2d of the model.
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int find_entry(const dfcsa_wstd_entry* tab, int n, int r) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].row0 <= r) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ void __launch_bounds__(256) wstd_fwd_kernel(const dfcsa_wstd_entry* __restrict__ tab, int n, int total) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= total) return;
  const dfcsa_wstd_entry& e = tab[find_entry(tab, n, r)];
  const int row = r - e.row0, K = e.K;
  const float* w = e.w + (size_t)row * K;
  double s = 0.0;
  for (int k = lane; k < K; k += 64) s += (double)w[k];
  const double mean = wave_sum_d(s) / K;
  double q = 0.0;
  for (int k = lane; k < K; k += 64) {
    const double d = (double)w[k] - mean;
    q += d * d;
  }
  const double var = wave_sum_d(q) / K;
  const float rstd = (float)(1.0 / sqrt(var + 1e-5));
  const float mf = (float)mean;
  float* o = e.what + (size_t)row * K;
  for (int k = lane; k < K; k += 64) o[k] = (w[k] - mf) * rstd;
  if (lane == 0) e.rstd[row] = rstd;
}

// dw[r][k] += rstd_r * (g - mean(g) - what * mean(g * what))   (g = dL/dwhat)
__global__ void __launch_bounds__(256) wstd_bwd_kernel(const dfcsa_wstd_entry* __restrict__ tab, int n, int total) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= total) return;
  const dfcsa_wstd_entry& e = tab[find_entry(tab, n, r)];
  const int row = r - e.row0, K = e.K;
  const float* g = e.g + (size_t)row * K;
  const float* wh = e.what + (size_t)row * K;
  double s = 0.0, sw = 0.0;
  for (int k = lane; k < K; k += 64) {
    s += (double)g[k];
    sw += (double)g[k] * (double)wh[k];
  }
  const float mg = (float)(wave_sum_d(s) / K), mgw = (float)(wave_sum_d(sw) / K);
  const float rstd = e.rstd[row];
  float* dw = e.dw + (size_t)row * K;
  for (int k = lane; k < K; k += 64) dw[k] += rstd * (g[k] - mg - wh[k] * mgw);
}

// ------------------------------------------------------------ root conv input gather
// out[m][tap*Cin + ci] = x[b][ci % Csrc][oh*s - p + kh][ow*s - p + kw] (0 outside the image and for
// columns >= k*k*Cin); x NCHW fp32 (Csrc = 1 replicates the single channel, transformer_unet.py:363-364)
template <typename T>
__global__ void im2col_input_kernel(int B, int Csrc, int Cin, int H, int W, int k, int s, int p, int Ho, int Wo,
                                    const float* __restrict__ x, int Kpad, T* __restrict__ out) {
  const int cpr = Kpad >> 3;
  const int64_t total = (int64_t)B * Ho * Wo * cpr;
  const int kk = k * k * Cin;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ch = (int)(e % cpr);
    const int64_t m = e / cpr;
    const int ow = (int)(m % Wo);
    const int oh = (int)((m / Wo) % Ho);
    const int b = (int)(m / ((int64_t)Wo * Ho));
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int col = ch * 8 + q;
      float val = 0.f;
      if (col < kk) {
        const int tap = col / Cin, ci = col - tap * Cin;
        const int kh = tap / k, kw = tap - kh * k;
        const int ih = oh * s - p + kh, iw = ow * s - p + kw;
        if (ih >= 0 && ih < H && iw >= 0 && iw < W)
          val = x[(((size_t)b * Csrc + (ci % Csrc)) * H + ih) * W + iw];
      }
      v[q] = val;
    }
    store8<T>(out + (size_t)m * Kpad + ch * 8, v);
  }
}

// ------------------------------------------------------------ GroupNorm
// Channel sums over (pixel lanes x 8-channel chunks) through LDS, fixed order.
template <int NS>
__device__ __forceinline__ void lane_reduce_store(const float (&acc)[NS][8], int C, int cpp, int pl, int lane_px,
                                                  int ck, bool active, float* out /* [NS][C] */) {
  __shared__ __attribute__((aligned(16))) float red[256 * 8];
  for (int s = 0; s < NS; ++s) {
    if (active) lds_st8(red + (lane_px * cpp + ck) * 8, acc[s]);
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      const int kq = c >> 3, q = c & 7;
      float v = 0.f;
      for (int p = 0; p < pl; ++p) v += red[(p * cpp + kq) * 8 + q];
      out[s * C + c] = v;
    }
    __syncthreads();
  }
}

// partial[b][sl][0][c] = sum over the pixel slice sl of image b of y, [1][c] = sum of y^2
template <typename T>
__global__ void __launch_bounds__(256) gn_stats_kernel(int HW, int C, int S, const T* __restrict__ y,
                                                       float* __restrict__ partial) {
  const int sl = blockIdx.x, b = blockIdx.y;
  const int cpp = C >> 3, pl = 256 / cpp;
  const int lane_px = threadIdx.x / cpp, ck = threadIdx.x - lane_px * cpp;
  const bool active = lane_px < pl;
  const int per = (HW + S - 1) / S, p0 = sl * per, p1 = min(HW, p0 + per);
  float acc[2][8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[0][q] = acc[1][q] = 0.f;
  if (active) {
    const T* yb = y + (size_t)b * HW * C + ck * 8;
#pragma unroll 4
    for (int p = p0 + lane_px; p < p1; p += pl) {
      float v[8];
      load8<T>(yb + (size_t)p * C, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        acc[0][q] += v[q];
        acc[1][q] += v[q] * v[q];
      }
    }
  }
  lane_reduce_store<2>(acc, C, cpp, pl, lane_px, ck, active, partial + ((size_t)b * S + sl) * 2 * C);
}

// per (b, g): mean, rstd (fp64 over S slices x Cg channels) -> mr[b][0][g], mr[b][1][g];
// scsh[b][0][c] = gamma_c*rstd, scsh[b][1][c] = beta_c - mean*gamma_c*rstd
__global__ void __launch_bounds__(256) gn_finalize_kernel(int HW, int C, int G, int S, const float* __restrict__ partial,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps,
                                                          float* __restrict__ mr, float* __restrict__ scsh) {
  const int b = blockIdx.x, Cg = C / G;
  for (int g = threadIdx.x; g < G; g += 256) {
    double s = 0.0, q = 0.0;
    for (int sl = 0; sl < S; ++sl) {
      const float* p = partial + ((size_t)b * S + sl) * 2 * C + g * Cg;
      for (int c = 0; c < Cg; ++c) {
        s += (double)p[c];
        q += (double)p[C + c];
      }
    }
    const double n = (double)HW * Cg;
    const double mean = s / n;
    double var = q / n - mean * mean;
    if (var < 0.0) var = 0.0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    mr[(size_t)b * 2 * G + g] = (float)mean;
    mr[(size_t)b * 2 * G + G + g] = rstd;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
      const float sc = gamma[c] * rstd;
      scsh[(size_t)b * 2 * C + c] = sc;
      scsh[(size_t)b * 2 * C + C + c] = beta[c] - (float)mean * sc;
    }
  }
}

// out = act(y*sc + sh + r), r = res*sc2 + sh2 (scsh2 given) or res (or 0)
template <typename T>
__global__ void gn_apply_kernel(int HW, int C, int64_t total, const T* __restrict__ y, const float* __restrict__ scsh,
                                const T* __restrict__ res, const float* __restrict__ scsh2, int act,
                                T* __restrict__ out) {
  const int cpp = C >> 3;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t m = e / cpp;
    const int c0 = (int)(e - m * cpp) * 8;
    const int b = (int)(m / HW);
    float v[8], sc[8], sh[8];
    load8<T>(y + m * C + c0, v);
    ld8f(scsh + (size_t)b * 2 * C + c0, sc);
    ld8f(scsh + (size_t)b * 2 * C + C + c0, sh);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = v[q] * sc[q] + sh[q];
    if (res) {
      float r[8];
      load8<T>(res + m * C + c0, r);
      if (scsh2) {
        float s2[8], h2[8];
        ld8f(scsh2 + (size_t)b * 2 * C + c0, s2);
        ld8f(scsh2 + (size_t)b * 2 * C + C + c0, h2);
#pragma unroll
        for (int q = 0; q < 8; ++q) r[q] = r[q] * s2[q] + h2[q];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += r[q];
    }
    if (act)
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
    store8<T>(out + m * C + c0, v);
  }
}

// dz = dout * (mask > 0) (mask NULL: dz = dout); xh = (y - mean_bg) * rstd_bg
// partial[b][sl][0][c] = sum dz, [1][c] = sum dz*xh
template <typename T>
__global__ void __launch_bounds__(256) gn_bwd_reduce_kernel(int HW, int C, int G, int S, const T* __restrict__ dout,
                                                            const T* __restrict__ mask, const T* __restrict__ y,
                                                            const float* __restrict__ mr, float* __restrict__ partial) {
  const int sl = blockIdx.x, b = blockIdx.y;
  const int cpp = C >> 3, pl = 256 / cpp;
  const int lane_px = threadIdx.x / cpp, ck = threadIdx.x - lane_px * cpp;
  const bool active = lane_px < pl;
  const int per = (HW + S - 1) / S, p0 = sl * per, p1 = min(HW, p0 + per);
  const int Cg = C / G;
  float acc[2][8], mu[8], rs[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    acc[0][q] = acc[1][q] = 0.f;
    const int g = (ck * 8 + q) / Cg;
    mu[q] = active ? mr[(size_t)b * 2 * G + g] : 0.f;
    rs[q] = active ? mr[(size_t)b * 2 * G + G + g] : 0.f;
  }
  if (active) {
    const size_t base = (size_t)b * HW * C + ck * 8;
#pragma unroll 4
    for (int p = p0 + lane_px; p < p1; p += pl) {
      const size_t off = base + (size_t)p * C;
      float d[8], v[8];
      load8<T>(dout + off, d);
      load8<T>(y + off, v);
      if (mask) {
        float mk[8];
        load8<T>(mask + off, mk);
#pragma unroll
        for (int q = 0; q < 8; ++q) d[q] = mk[q] > 0.f ? d[q] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        acc[0][q] += d[q];
        acc[1][q] += d[q] * ((v[q] - mu[q]) * rs[q]);
      }
    }
  }
  lane_reduce_store<2>(acc, C, cpp, pl, lane_px, ck, active, partial + ((size_t)b * S + sl) * 2 * C);
}

// One thread per channel (256 channels per workgroup; a group never straddles workgroups since
// Cg is a power of two <= 256): coef[b][0][g] = mean over the group of gamma*dz, coef[b][1][g] =
// mean of gamma*dz*xh; dgamma[c] += sum_b sum dz*xh, dbeta[c] += sum_b sum dz.
__global__ void __launch_bounds__(256) gn_bwd_finalize_kernel(int B, int HW, int C, int G, int S,
                                                              const float* __restrict__ partial,
                                                              const float* __restrict__ gamma, float* __restrict__ coef,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ double u0[256], u1[256];
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int Cg = C / G;
  const bool valid = c < C;
  const double gm = valid ? (double)gamma[c] : 0.0;
  double tg = 0.0, tb = 0.0;
  for (int b = 0; b < B; ++b) {
    double s0 = 0.0, s1 = 0.0;
    if (valid)
      for (int sl = 0; sl < S; ++sl) {
        const float* p = partial + ((size_t)b * S + sl) * 2 * C;
        s0 += (double)p[c];
        s1 += (double)p[C + c];
      }
    tb += s0;
    tg += s1;
    u0[threadIdx.x] = gm * s0;
    u1[threadIdx.x] = gm * s1;
    __syncthreads();
    if (valid && (threadIdx.x % Cg) == 0) {
      double a0 = 0.0, a1 = 0.0;
      for (int j = 0; j < Cg; ++j) {
        a0 += u0[threadIdx.x + j];
        a1 += u1[threadIdx.x + j];
      }
      const double n = (double)HW * Cg;
      const int g = c / Cg;
      coef[(size_t)b * 2 * G + g] = (float)(a0 / n);
      coef[(size_t)b * 2 * G + G + g] = (float)(a1 / n);
    }
    __syncthreads();
  }
  if (valid) {
    if (dgamma) dgamma[c] += (float)tg;
    if (dbeta) dbeta[c] += (float)tb;
  }
}

// dy = rstd*(gamma*dz - coef0 - xh*coef1); dz_out (optional) = dz
template <typename T>
__global__ void gn_bwd_apply_kernel(int HW, int C, int G, int64_t total, const T* __restrict__ dout,
                                    const T* __restrict__ mask, const T* __restrict__ y, const float* __restrict__ mr,
                                    const float* __restrict__ gamma, const float* __restrict__ coef, T* __restrict__ dy,
                                    T* __restrict__ dz_out) {
  const int cpp = C >> 3, Cg = C / G;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t m = e / cpp;
    const int c0 = (int)(e - m * cpp) * 8;
    const int b = (int)(m / HW);
    float d[8], v[8], gm[8], o[8];
    load8<T>(dout + m * C + c0, d);
    load8<T>(y + m * C + c0, v);
    if (mask) {
      float mk[8];
      load8<T>(mask + m * C + c0, mk);
#pragma unroll
      for (int q = 0; q < 8; ++q) d[q] = mk[q] > 0.f ? d[q] : 0.f;
    }
    ld8f(gamma + c0, gm);
    const float* mb = mr + (size_t)b * 2 * G;
    const float* cb = coef + (size_t)b * 2 * G;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int g = (c0 + q) / Cg;
      const float rs = mb[G + g];
      const float xh = (v[q] - mb[g]) * rs;
      o[q] = rs * (gm[q] * d[q] - cb[g] - xh * cb[G + g]);
    }
    store8<T>(dy + m * C + c0, o);
    if (dz_out) store8<T>(dz_out + m * C + c0, d);
  }
}

// ---------------------------------------------------------------- GroupNorm, fused reductions
// The statistics pass and the backward reduction pass each finish their own reduction in the
// launch: every (slice, image) workgroup publishes its [2][C] row with write-through (sc1) stores
// and takes the image's ticket (wg_last_of); the image's last-arriving workgroup sums the image's S
// rows per channel in a fixed order (sc1 loads, eight in flight) and finalises the image.  This
// replaces the separate gn_finalize / gn_bwd_finalize launches (a one-workgroup-per-image serial
// loop over S x Cg partials: 9 / 16 us each, 52 of each per TransUNet step).  The backward also
// needs sum_b over the images (dgamma, dbeta): each image's finaliser publishes its channel sums
// (double) and takes a second ticket; the last image adds them in image order.  Deterministic.

// sum over the rows r in [0, S) of rows[r * 2C + k * C + c] (k = 0, 1) for every channel c into
// ch[k][c] (LDS, double): passes of NCH = min(C, 256) channels, P = 256 / NCH parts per pass, part
// p sums rows p, p + P, ... in order (4 rows x 2 sums = 8 sc1 loads in flight), parts combined in
// part order.  256 threads; tmp: LDS [2][256] doubles.
__device__ void gn_rows_colsum(const float* rows, int S, int C, double* ch, double* tmp) {
  const int t = threadIdx.x;
  const int NCH = C < 256 ? C : 256, P = 256 / NCH;
  for (int c0 = 0; c0 < C; c0 += NCH) {
    const int cl = t % NCH, part = t / NCH, c = c0 + cl;
    double s0 = 0.0, s1 = 0.0;
    if (part < P && c < C) {
      int r = part;
      for (; r + 3 * P < S; r += 4 * P) {
        const float* pp[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pp[2 * j] = rows + (size_t)(r + j * P) * 2 * C + c;
          pp[2 * j + 1] = pp[2 * j] + C;
        }
        float v[8];
        ld_sc1_f8(pp, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) { s0 += (double)v[2 * j]; s1 += (double)v[2 * j + 1]; }
      }
      for (; r < S; r += P) {
        s0 += (double)ld_sc1_f(rows + (size_t)r * 2 * C + c);
        s1 += (double)ld_sc1_f(rows + (size_t)r * 2 * C + C + c);
      }
    }
    tmp[t] = s0;
    tmp[256 + t] = s1;
    __syncthreads();
    if (t < NCH && c < C) {
      double a0 = 0.0, a1 = 0.0;
      for (int q = 0; q < P; ++q) { a0 += tmp[q * NCH + t]; a1 += tmp[256 + q * NCH + t]; }
      ch[c] = a0;
      ch[C + c] = a1;
    }
    __syncthreads();
  }
}

// this workgroup's [2][C] row (the lane accumulators of gn_stats / gn_bwd_reduce) -> rows, sc1
template <int NS>
__device__ __forceinline__ void gn_publish_row(const float (&acc)[NS][8], int C, int cpp, int pl, int lane_px,
                                               int ck, bool active, float* red, float* row) {
  for (int k = 0; k < NS; ++k) {
    if (active) lds_st8(red + (lane_px * cpp + ck) * 8, acc[k]);
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      const int kq = c >> 3, q = c & 7;
      float v = 0.f;
      for (int p = 0; p < pl; ++p) v += red[(p * cpp + kq) * 8 + q];
      st_sc1_dw(row + k * C + c, v);
    }
    __syncthreads();
  }
}

// statistics + finalize: mr[b][0][g] = mean, mr[b][1][g] = rstd; scsh[b][0][c] = gamma_c*rstd,
// scsh[b][1][c] = beta_c - mean*gamma_c*rstd (as gn_finalize_kernel)
// Channel chunks (grid.z, CW = gn_chunk(C, G) channels each, whole groups): the last-arriver sums
// S rows of 2 CW values instead of 2 C -- at C = 1024 its serial column sum was 24 rows x 2048 values
// of write-through loads per image, most of a 23 us launch.  Rows [B][nck][S][2][CW].
template <typename T>
__global__ void __launch_bounds__(256) gn_stats_fin_kernel(int HW, int C, int CW, int G, int S, const T* __restrict__ y,
                                                           float* rows, unsigned* cnt, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float eps, float* mr,
                                                           float* scsh) {
  __shared__ __attribute__((aligned(16))) float red[256 * 8];   // (also the colsum's [2][256] doubles)
  __shared__ double ch[2 * 1024];
  __shared__ float grp[2 * 256];
  __shared__ int flag;
  double* tmp = (double*)red;
  const int sl = blockIdx.x, b = blockIdx.y, kc = blockIdx.z, nck = gridDim.z, c0 = kc * CW;
  const int cpp = CW >> 3, pl = 256 / cpp;
  const int lane_px = threadIdx.x / cpp, ck = threadIdx.x - lane_px * cpp;
  const bool active = lane_px < pl;
  const int per = (HW + S - 1) / S, p0 = sl * per, p1 = min(HW, p0 + per);
  float acc[2][8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[0][q] = acc[1][q] = 0.f;
  if (active) {
    const T* yb = y + (size_t)b * HW * C + c0 + ck * 8;
#pragma unroll 4
    for (int p = p0 + lane_px; p < p1; p += pl) {
      float v[8];
      load8<T>(yb + (size_t)p * C, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        acc[0][q] += v[q];
        acc[1][q] += v[q] * v[q];
      }
    }
  }
  float* img = rows + ((size_t)b * nck + kc) * S * 2 * CW;
  gn_publish_row<2>(acc, CW, cpp, pl, lane_px, ck, active, red, img + (size_t)sl * 2 * CW);
  if (!wg_last_of(cnt + b * nck + kc, S, &flag)) return;
  gn_rows_colsum(img, S, CW, ch, tmp);   // ch[k * CW + (c - c0)]
  const int Cg = C / G, g0 = c0 / Cg, g1 = (c0 + CW) / Cg;
  const double n = (double)HW * Cg;
  for (int g = g0 + (int)threadIdx.x; g < g1; g += 256) {
    double s0 = 0.0, q0 = 0.0;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) { s0 += ch[c - c0]; q0 += ch[CW + c - c0]; }
    const double mean = s0 / n;
    double var = q0 / n - mean * mean;
    if (var < 0.0) var = 0.0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    mr[(size_t)b * 2 * G + g] = (float)mean;
    mr[(size_t)b * 2 * G + G + g] = rstd;
    grp[g] = (float)mean;
    grp[G + g] = rstd;
  }
  __syncthreads();
  for (int c = c0 + (int)threadIdx.x; c < c0 + CW; c += 256) {
    const int g = c / Cg;
    const float sc = gamma[c] * grp[G + g];
    scsh[(size_t)b * 2 * C + c] = sc;
    scsh[(size_t)b * 2 * C + C + c] = beta[c] - grp[g] * sc;
  }
}

// backward reduction + finalize: coef[b][0][g] = mean over the group of gamma*dz, coef[b][1][g] =
// mean of gamma*dz*xh (as gn_bwd_finalize_kernel); dgamma[c] += sum_b sum dz*xh, dbeta[c] +=
// sum_b sum dz (last image, image order).  work: [B][2][C] doubles (hand-off of the images' sums).
template <typename T>
__global__ void __launch_bounds__(256) gn_bwd_reduce_fin_kernel(
    int HW, int C, int CW, int G, int S, const T* __restrict__ dout, const T* __restrict__ mask, const T* __restrict__ y,
    const float* __restrict__ mr, const float* __restrict__ gamma, float* rows, double* work, unsigned* cnt,
    float* coef, float* dgamma, float* dbeta) {
  __shared__ __attribute__((aligned(16))) float red[256 * 8];   // (also the colsum's [2][256] doubles)
  __shared__ double ch[2 * 1024];
  __shared__ int flag;
  double* tmp = (double*)red;
  const int sl = blockIdx.x, b = blockIdx.y, B = gridDim.y, kc = blockIdx.z, nck = gridDim.z, c0 = kc * CW;
  const int cpp = CW >> 3, pl = 256 / cpp;
  const int lane_px = threadIdx.x / cpp, ck = threadIdx.x - lane_px * cpp;
  const bool active = lane_px < pl;
  const int per = (HW + S - 1) / S, p0 = sl * per, p1 = min(HW, p0 + per);
  const int Cg = C / G;
  float acc[2][8], mu[8], rs[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    acc[0][q] = acc[1][q] = 0.f;
    const int g = (c0 + ck * 8 + q) / Cg;
    mu[q] = active ? mr[(size_t)b * 2 * G + g] : 0.f;
    rs[q] = active ? mr[(size_t)b * 2 * G + G + g] : 0.f;
  }
  if (active) {
    const size_t base = (size_t)b * HW * C + c0 + ck * 8;
#pragma unroll 4
    for (int p = p0 + lane_px; p < p1; p += pl) {
      const size_t off = base + (size_t)p * C;
      float d[8], v[8];
      load8<T>(dout + off, d);
      load8<T>(y + off, v);
      if (mask) {
        float mk[8];
        load8<T>(mask + off, mk);
#pragma unroll
        for (int q = 0; q < 8; ++q) d[q] = mk[q] > 0.f ? d[q] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        acc[0][q] += d[q];
        acc[1][q] += d[q] * ((v[q] - mu[q]) * rs[q]);
      }
    }
  }
  float* img = rows + ((size_t)b * nck + kc) * S * 2 * CW;
  gn_publish_row<2>(acc, CW, cpp, pl, lane_px, ck, active, red, img + (size_t)sl * 2 * CW);
  if (!wg_last_of(cnt + b * nck + kc, S, &flag)) return;
  gn_rows_colsum(img, S, CW, ch, tmp);   // ch[k * CW + (c - c0)]
  // this image's channel sums (of the chunk) -> work[b] (hand-off to the last image); group coefficients
  double* wb = work + (size_t)b * 2 * C;
  for (int c = c0 + (int)threadIdx.x; c < c0 + CW; c += 256) {
    st_sc1_d(wb + c, ch[c - c0]);
    st_sc1_d(wb + C + c, ch[CW + c - c0]);
  }
  const double n = (double)HW * Cg;
  for (int g = c0 / Cg + (int)threadIdx.x; g < (c0 + CW) / Cg; g += 256) {
    double a0 = 0.0, a1 = 0.0;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
      const double gm = (double)gamma[c];
      a0 += gm * ch[c - c0];
      a1 += gm * ch[CW + c - c0];
    }
    coef[(size_t)b * 2 * G + g] = (float)(a0 / n);
    coef[(size_t)b * 2 * G + G + g] = (float)(a1 / n);
  }
  if (!dgamma && !dbeta) return;
  if (!wg_last_of(cnt + B * nck + kc, B, &flag)) return;
  for (int c = c0 + (int)threadIdx.x; c < c0 + CW; c += 256) {
    double tb = 0.0, tg = 0.0;
    for (int bb = 0; bb < B; ++bb) {
      double v0, v1, v2;
      const double* w = work + (size_t)bb * 2 * C;
      ld_sc1_d3(w + c, w + C + c, w + c, v0, v1, v2);
      tb += v0;
      tg += v1;
    }
    if (dgamma) dgamma[c] += (float)tg;
    if (dbeta) dbeta[c] += (float)tb;
  }
}

// ------------------------------------------------------------ MaxPool2d(3, 2, padding=1)
// out = max over the in-bounds taps of each window (first maximum in (kh, kw) order, NaN wins, as
// ATen); idx[b][oh][ow][c] = tap index (kh*3 + kw) of that maximum.
template <typename T>
__global__ void maxpool3s2_fwd_kernel(int B, int H, int W, int C, int Ho, int Wo, const T* __restrict__ x,
                                      T* __restrict__ y, uint8_t* __restrict__ idx) {
  const int cpp = C >> 3;
  const int64_t total = (int64_t)B * Ho * Wo * cpp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t p = e / cpp;
    const int ow = (int)(p % Wo);
    p /= Wo;
    const int oh = (int)(p % Ho);
    const int b = (int)(p / Ho);
    float best[8];
    int arg[8];
    bool first = true;
#pragma unroll
    for (int q = 0; q < 8; ++q) { best[q] = 0.f; arg[q] = 0; }
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - 1 + kw;
        if (iw < 0 || iw >= W) continue;
        float v[8];
        load8<T>(x + (((size_t)b * H + ih) * W + iw) * C + ck * 8, v);
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (first || v[q] > best[q] || isnan(v[q])) { best[q] = v[q]; arg[q] = kh * 3 + kw; }
        first = false;
      }
    }
    store8<T>(y + (size_t)e * 8, best);
    uint2 packed;
    packed.x = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) | ((uint32_t)arg[3] << 24);
    packed.y = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) | ((uint32_t)arg[7] << 24);
    *(uint2*)(idx + (size_t)e * 8) = packed;
  }
}

// dx[b][ih][iw][c] = sum over the windows containing (ih, iw) whose maximum sits there of dy
template <typename T>
__global__ void maxpool3s2_bwd_kernel(int B, int H, int W, int C, int Ho, int Wo, const uint8_t* __restrict__ idx,
                                      const T* __restrict__ dy, T* __restrict__ dx) {
  const int cpp = C >> 3;
  const int64_t total = (int64_t)B * H * W * cpp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t p = e / cpp;
    const int iw = (int)(p % W);
    p /= W;
    const int ih = (int)(p % H);
    const int b = (int)(p / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int oh0 = ih / 2, oh1 = min(Ho - 1, (ih + 1) / 2);
    const int ow0 = iw / 2, ow1 = min(Wo - 1, (iw + 1) / 2);
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int kh = ih - 2 * oh + 1;
      if (kh < 0 || kh > 2) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int kw = iw - 2 * ow + 1;
        if (kw < 0 || kw > 2) continue;
        const size_t o = (((size_t)b * Ho + oh) * Wo + ow) * C + ck * 8;
        const uint2 pk = *(const uint2*)(idx + o);
        float g[8];
        load8<T>(dy + o, g);
        const int tap = kh * 3 + kw;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint32_t word = q < 4 ? pk.x : pk.y;
          const int a = (int)((word >> (8 * (q & 3))) & 0xffu);
          if (a == tap) acc[q] += g[q];
        }
      }
    }
    store8<T>(dx + (size_t)e * 8, acc);
  }
}

// ------------------------------------------------------------ col2im (strided-conv dgrad)
// dx[b][ih][iw][c] (+)= sum over taps (kh, kw) with oh = (ih + p - kh)/s, ow = (iw + p - kw)/s
// integral and in range of dcols[b][oh][ow][(kh*k + kw)*C + c]
template <typename T>
__global__ void col2im_kernel(int B, int H, int W, int C, int Ho, int Wo, int k, int s, int p,
                              const T* __restrict__ dcols, T* __restrict__ dx, int accumulate) {
  const int cpp = C >> 3;
  const int64_t total = (int64_t)B * H * W * cpp;
  const int64_t ld = (int64_t)k * k * C;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t q = e / cpp;
    const int iw = (int)(q % W);
    q /= W;
    const int ih = (int)(q % H);
    const int b = (int)(q / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int kh = 0; kh < k; ++kh) {
      const int th = ih + p - kh;
      if (th < 0 || th % s) continue;
      const int oh = th / s;
      if (oh >= Ho) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int tw = iw + p - kw;
        if (tw < 0 || tw % s) continue;
        const int ow = tw / s;
        if (ow >= Wo) continue;
        float v[8];
        load8<T>(dcols + (((int64_t)b * Ho + oh) * Wo + ow) * ld + (kh * k + kw) * C + ck * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j];
      }
    }
    T* dst = dx + (size_t)e * 8;
    if (accumulate) {
      float o[8];
      load8<T>(dst, o);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += o[j];
    }
    store8<T>(dst, acc);
  }
}

// ------------------------------------------------------------ LayerNorm (one wave per row)
// x fp32 [rows][C]; y = (x - mean)*rstd*gamma + beta (dtype); mr[row] = {mean, rstd}
constexpr int LN_MAXCH = 4;   // 8-channel chunks per lane: C <= 64*8*4 = 2048

template <typename T>
__global__ void __launch_bounds__(256) ln_fwd_kernel(int rows, int C, const float* __restrict__ x,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float eps, T* __restrict__ y, float* __restrict__ mr) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nch = C >> 3;
  const float* xr = x + (size_t)row * C;
  float v[LN_MAXCH][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXCH; ++i) {
    const int ch = lane + 64 * i;
    if (ch < nch) {
      ld8f(xr + ch * 8, v[i]);
#pragma unroll
      for (int q = 0; q < 8; ++q) s += v[i][q];
    }
  }
  const float mean = wave_sum(s) / C;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXCH; ++i) {
    const int ch = lane + 64 * i;
    if (ch < nch)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float d = v[i][q] - mean;
        ss += d * d;
      }
  }
  const float rstd = 1.f / sqrtf(wave_sum(ss) / C + eps);
#pragma unroll
  for (int i = 0; i < LN_MAXCH; ++i) {
    const int ch = lane + 64 * i;
    if (ch < nch) {
      float g[8], bt[8], o[8];
      ld8f(gamma + ch * 8, g);
      ld8f(beta + ch * 8, bt);
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = (v[i][q] - mean) * rstd * g[q] + bt[q];
      store8<T>(y + (size_t)row * C + ch * 8, o);
    }
  }
  if (lane == 0) {
    mr[2 * row] = mean;
    mr[2 * row + 1] = rstd;
  }
}

// dx = rstd*(g - mean(g) - xh*mean(g*xh)) + dres, g = dy*gamma (dx, dres fp32; dres may alias dx);
// partial[(blk*4 + wave)][0][c] = sum dy*xh, [1][c] = sum dy over the wave's rows
constexpr int LN_ROWS_PER_WAVE = 4;

template <typename T>
__global__ void __launch_bounds__(256) ln_bwd_kernel(int rows, int C, const T* __restrict__ dy,
                                                     const float* __restrict__ x, const float* __restrict__ mr,
                                                     const float* __restrict__ gamma, const float* dres, float* dx,
                                                     float* __restrict__ partial) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + wave;
  const int nch = C >> 3;
  float pg[LN_MAXCH][8], pb[LN_MAXCH][8];
#pragma unroll
  for (int i = 0; i < LN_MAXCH; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) pg[i][q] = pb[i][q] = 0.f;
  for (int r = 0; r < LN_ROWS_PER_WAVE; ++r) {
    const int row = wid * LN_ROWS_PER_WAVE + r;
    if (row >= rows) break;
    const float mean = mr[2 * row], rstd = mr[2 * row + 1];
    float xh[LN_MAXCH][8], gg[LN_MAXCH][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXCH; ++i) {
      const int ch = lane + 64 * i;
      if (ch < nch) {
        float xv[8], d[8], gm[8];
        ld8f(x + (size_t)row * C + ch * 8, xv);
        load8<T>(dy + (size_t)row * C + ch * 8, d);
        ld8f(gamma + ch * 8, gm);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          xh[i][q] = (xv[q] - mean) * rstd;
          gg[i][q] = d[q] * gm[q];
          s1 += gg[i][q];
          s2 += gg[i][q] * xh[i][q];
          pg[i][q] += d[q] * xh[i][q];
          pb[i][q] += d[q];
        }
      }
    }
    const float m1 = wave_sum(s1) / C, m2 = wave_sum(s2) / C;
#pragma unroll
    for (int i = 0; i < LN_MAXCH; ++i) {
      const int ch = lane + 64 * i;
      if (ch < nch) {
        float o[8];
        if (dres) {
          ld8f(dres + (size_t)row * C + ch * 8, o);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = 0.f;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] += rstd * (gg[i][q] - m1 - xh[i][q] * m2);
        st8f(dx + (size_t)row * C + ch * 8, o);
      }
    }
  }
  float* pp = partial + (size_t)wid * 2 * C;
#pragma unroll
  for (int i = 0; i < LN_MAXCH; ++i) {
    const int ch = lane + 64 * i;
    if (ch < nch) {
      st8f(pp + ch * 8, pg[i]);
      st8f(pp + C + ch * 8, pb[i]);
    }
  }
}

// ------------------------------------------------------------ dropout, GELU, residual adds
// Counter-based dropout: keep(i) depends only on (device RNG state, call site, element index), so
// the backward regenerates the forward's mask with no mask tensor, and HIP-graph replays draw a
// new mask every step (the state advances on the device).  The masks are statistically, not
// bitwise, equivalent to nn.Dropout's Philox stream (transformer_unet.py:164-172, :198).
__device__ __forceinline__ uint32_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}
__device__ __forceinline__ uint64_t drop_key(const int64_t* rng, int site) {
  return ((uint64_t)rng[0] * 0x100000001B3ull) ^ ((uint64_t)rng[1] << 20) ^ ((uint64_t)site << 52);
}
__device__ __forceinline__ bool keep_elem(uint64_t key, int64_t i, float p) {
  const float u = (float)(mix64(key ^ ((uint64_t)i * 0xD6E8FEB86659FD93ull)) >> 8) * (1.0f / 16777216.0f);
  return u >= p;
}

// out[i] = drop(a[i] + pos[i % L]) + res[i]   (pos/res optional; out, pos, res fp32; a dtype)
template <typename T>
__global__ void drop_add_fwd_kernel(int64_t n, const T* __restrict__ a, const float* __restrict__ pos, int64_t L,
                                    const float* __restrict__ res, float p, const int64_t* __restrict__ rng, int site,
                                    float* __restrict__ out) {
  const uint64_t key = p > 0.f ? drop_key(rng, site) : 0;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e * 8 < n; e += (int64_t)gridDim.x * 256) {
    const int64_t i0 = e * 8;
    float v[8];
    load8<T>(a + i0, v);
    if (pos) {
      float ps[8];
      ld8f(pos + (i0 % L), ps);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += ps[q];
    }
    if (p > 0.f)
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = keep_elem(key, i0 + q, p) ? v[q] * scale : 0.f;
    if (res) {
      float r[8];
      ld8f(res + i0, r);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += r[q];
    }
    st8f(out + i0, v);
  }
}

// da[i] = dout[i] * keep(i) / (1 - p)   (dout fp32, da dtype)
template <typename T>
__global__ void drop_bwd_kernel(int64_t n, const float* __restrict__ dout, float p, const int64_t* __restrict__ rng,
                                int site, T* __restrict__ da) {
  const uint64_t key = p > 0.f ? drop_key(rng, site) : 0;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e * 8 < n; e += (int64_t)gridDim.x * 256) {
    const int64_t i0 = e * 8;
    float v[8];
    ld8f(dout + i0, v);
    if (p > 0.f)
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = keep_elem(key, i0 + q, p) ? v[q] * scale : 0.f;
    store8<T>(da + i0, v);
  }
}

__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.7071067811865476f)); }
__device__ __forceinline__ float gelu_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
  const float pdf = expf(-0.5f * x * x) * 0.3989422804014327f;
  return cdf + x * pdf;
}

// out = drop(gelu(x))  (F.gelu exact erf form, transformer_unet.py:114, :169-170)
template <typename T>
__global__ void gelu_drop_fwd_kernel(int64_t n, const T* __restrict__ x, float p, const int64_t* __restrict__ rng,
                                     int site, T* __restrict__ out) {
  const uint64_t key = p > 0.f ? drop_key(rng, site) : 0;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e * 8 < n; e += (int64_t)gridDim.x * 256) {
    const int64_t i0 = e * 8;
    float v[8];
    load8<T>(x + i0, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float g = gelu_f(v[q]);
      if (p > 0.f) g = keep_elem(key, i0 + q, p) ? g * scale : 0.f;
      v[q] = g;
    }
    store8<T>(out + i0, v);
  }
}

template <typename T>
__global__ void gelu_drop_bwd_kernel(int64_t n, const T* __restrict__ x, const T* __restrict__ dout, float p,
                                     const int64_t* __restrict__ rng, int site, T* __restrict__ dx) {
  const uint64_t key = p > 0.f ? drop_key(rng, site) : 0;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e * 8 < n; e += (int64_t)gridDim.x * 256) {
    const int64_t i0 = e * 8;
    float v[8], d[8];
    load8<T>(x + i0, v);
    load8<T>(dout + i0, d);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float g = d[q] * gelu_grad(v[q]);
      if (p > 0.f) g = keep_elem(key, i0 + q, p) ? g * scale : 0.f;
      v[q] = g;
    }
    store8<T>(dx + i0, v);
  }
}

constexpr int COLSUM_ROWS = 64;   // rows per column-sum tile of colsum_partial
constexpr int CS_ROWS = 16;       // rows per tile of the passes that also emit column partials (*_cs):
                                  // at the ViT's M = 1568 a 64-row tile left 25 row tiles, too few workgroups

// drop_bwd / gelu_drop_bwd over a [M][C] matrix with the column sums of their (stored) output per
// COLSUM_ROWS-row tile: partial[tile][C] for dfcsa_slab_colsum3 -- the Linear bias gradient of the
// GEMM whose dY this is (fc2 / out-projection: drop_bwd; fc1: gelu_drop_bwd), without the
// colsum_partial pass over dY.  The element index of the dropout mask is the flat one (r*C + c), as
// the flat kernels'; the sums add the values as stored (bf16-rounded), as colsum_partial reads them.
template <typename T, bool GELU>
__global__ void __launch_bounds__(256) drop_bwd_cs_kernel(int64_t M, int C, const T* __restrict__ x,
                                                          const void* __restrict__ dout, float p,
                                                          const int64_t* __restrict__ rng, int site,
                                                          T* __restrict__ out, float* __restrict__ partial) {
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c0 >= C) return;
  const uint64_t key = p > 0.f ? drop_key(rng, site) : 0;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int64_t r0 = (int64_t)blockIdx.y * CS_ROWS, r1 = min(M, r0 + CS_ROWS);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t r = r0; r < r1; r += 4) {
    const int nr = (int)min((int64_t)4, r1 - r);
    float d[4][8], v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t rr = r + min(u, nr - 1);   // rows past the tile re-load the last one (unused)
      if constexpr (GELU) {
        load8<T>((const T*)dout + rr * C + c0, d[u]);
        load8<T>(x + rr * C + c0, v[u]);
      } else {
        ld8f((const float*)dout + rr * C + c0, d[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u >= nr) break;
      const int64_t i0 = (r + u) * C + c0;
      float o[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float g = GELU ? d[u][q] * gelu_grad(v[u][q]) : d[u][q];
        if (p > 0.f) g = keep_elem(key, i0 + q, p) ? g * scale : 0.f;
        o[q] = g;
      }
      store8<T>(out + i0, o);
#pragma unroll
      for (int q = 0; q < 8; ++q) {   // the stored (rounded) value
        if constexpr (sizeof(T) == 2) acc[q] += bf2f(f2bf(o[q]));
        else acc[q] += o[q];
      }
    }
  }
  st8f(partial + (size_t)blockIdx.y * C + c0, acc);
}

// out[j] += sum_b x[b*L + j]  (position-embedding gradient; fp64 over the batch)
template <typename T>
__global__ void batch_sum_kernel(int B, int64_t L, const T* __restrict__ x, float* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < L; j += (int64_t)gridDim.x * 256) {
    double s = 0.0;
    for (int b = 0; b < B; ++b) s += (double)ElemTraits<T>::to_f(x[(int64_t)b * L + j]);
    out[j] += (float)s;
  }
}

// ------------------------------------------------------------ attention-probability dropout
// Attention.forward with attention_dropout_rate > 0 in training (transformer_unet.py:146-151):
// probs = softmax(q k^T * scale); ctx = attn_dropout(probs) @ v.  The score matrix of the ViT
// (N = 196 tokens) is small, so this path materialises the UNDROPPED probabilities (fp32
// [B*heads][N][N]) for the backward and regenerates the dropout mask from the counter-based key
// (keep(i), i = (bh*N + n)*N + m).  One workgroup per query row (forward, dq) or key row (dk, dv).
// Backward: dPd = dctx v^T; dP = dPd * keep / (1 - p); dS = P (dP - rowsum(P dP));
// dq = scale dS k; dk = scale dS^T q; dv = Pd^T dctx.
__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}
__device__ __forceinline__ float block_max256(float v, float* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

template <typename T>
__global__ void __launch_bounds__(256) mha_drop_fwd_kernel(int N, int heads, int dh, int ldq, float scale,
                                                           const T* __restrict__ qkv, float p,
                                                           const int64_t* __restrict__ rng, int site,
                                                           float* __restrict__ probs, T* __restrict__ ctx) {
  extern __shared__ float sm[];   // q [dh] | e [N] | red [4]
  float* q = sm;
  float* e = sm + dh;
  float* red = e + N;
  const int n = blockIdx.x, bh = blockIdx.y, b = bh / heads, h = bh - b * heads, D = heads * dh;
  const T* base = qkv + (size_t)b * N * ldq;
  for (int c = threadIdx.x; c < dh; c += 256) q[c] = ElemTraits<T>::to_f(base[(size_t)n * ldq + h * dh + c]);
  __syncthreads();
  float mx = -INFINITY;
  for (int m = threadIdx.x; m < N; m += 256) {
    const T* k = base + (size_t)m * ldq + D + h * dh;
    float s = 0.f;
    for (int c = 0; c < dh; ++c) s += q[c] * ElemTraits<T>::to_f(k[c]);
    s *= scale;
    e[m] = s;
    mx = fmaxf(mx, s);
  }
  mx = block_max256(mx, red);
  float sum = 0.f;
  for (int m = threadIdx.x; m < N; m += 256) {
    const float v = __expf(e[m] - mx);
    e[m] = v;
    sum += v;
  }
  sum = block_sum256(sum, red);
  const float inv = 1.f / sum, kscale = 1.f / (1.f - p);
  const uint64_t key = drop_key(rng, site);
  const int64_t row = ((int64_t)bh * N + n) * N;
  for (int m = threadIdx.x; m < N; m += 256) {
    const float pr = e[m] * inv;
    probs[row + m] = pr;
    e[m] = keep_elem(key, row + m, p) ? pr * kscale : 0.f;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < dh; c += 256) {
    float acc = 0.f;
    for (int m = 0; m < N; ++m) acc += e[m] * ElemTraits<T>::to_f(base[(size_t)m * ldq + 2 * D + h * dh + c]);
    ctx[((size_t)b * N + n) * D + h * dh + c] = ElemTraits<T>::from_f(acc);
  }
}

// query row n: dS row -> dscores, dq
template <typename T>
__global__ void __launch_bounds__(256) mha_drop_bwd_rows_kernel(int N, int heads, int dh, int ldq, float scale,
                                                                const T* __restrict__ qkv, const T* __restrict__ dctx,
                                                                const float* __restrict__ probs, float p,
                                                                const int64_t* __restrict__ rng, int site,
                                                                float* __restrict__ dscores, T* __restrict__ dqkv) {
  extern __shared__ float sm[];   // dctx row [dh] | dS [N] | red [4]
  float* dor = sm;
  float* ds = sm + dh;
  float* red = ds + N;
  const int n = blockIdx.x, bh = blockIdx.y, b = bh / heads, h = bh - b * heads, D = heads * dh;
  const T* base = qkv + (size_t)b * N * ldq;
  for (int c = threadIdx.x; c < dh; c += 256) dor[c] = ElemTraits<T>::to_f(dctx[((size_t)b * N + n) * D + h * dh + c]);
  __syncthreads();
  const float kscale = 1.f / (1.f - p);
  const uint64_t key = drop_key(rng, site);
  const int64_t row = ((int64_t)bh * N + n) * N;
  float dot = 0.f;
  for (int m = threadIdx.x; m < N; m += 256) {
    const T* v = base + (size_t)m * ldq + 2 * D + h * dh;
    float s = 0.f;
    for (int c = 0; c < dh; ++c) s += dor[c] * ElemTraits<T>::to_f(v[c]);
    const float dp = keep_elem(key, row + m, p) ? s * kscale : 0.f;
    ds[m] = dp;
    dot += probs[row + m] * dp;
  }
  dot = block_sum256(dot, red);
  for (int m = threadIdx.x; m < N; m += 256) {
    const float g = probs[row + m] * (ds[m] - dot);
    ds[m] = g;
    dscores[row + m] = g;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < dh; c += 256) {
    float acc = 0.f;
    for (int m = 0; m < N; ++m) acc += ds[m] * ElemTraits<T>::to_f(base[(size_t)m * ldq + D + h * dh + c]);
    dqkv[((size_t)b * N + n) * ldq + h * dh + c] = ElemTraits<T>::from_f(acc * scale);
  }
}

// key row m: dk, dv
template <typename T>
__global__ void __launch_bounds__(256) mha_drop_bwd_cols_kernel(int N, int heads, int dh, int ldq, float scale,
                                                                const T* __restrict__ qkv, const T* __restrict__ dctx,
                                                                const float* __restrict__ probs, float p,
                                                                const int64_t* __restrict__ rng, int site,
                                                                const float* __restrict__ dscores,
                                                                T* __restrict__ dqkv) {
  extern __shared__ float sm[];   // dS column [N] | Pd column [N]
  float* dsc = sm;
  float* pd = sm + N;
  const int m = blockIdx.x, bh = blockIdx.y, b = bh / heads, h = bh - b * heads, D = heads * dh;
  const float kscale = 1.f / (1.f - p);
  const uint64_t key = drop_key(rng, site);
  for (int n = threadIdx.x; n < N; n += 256) {
    const int64_t i = ((int64_t)bh * N + n) * N + m;
    dsc[n] = dscores[i];
    pd[n] = keep_elem(key, i, p) ? probs[i] * kscale : 0.f;
  }
  __syncthreads();
  const T* base = qkv + (size_t)b * N * ldq;
  for (int c = threadIdx.x; c < dh; c += 256) {
    float dk = 0.f, dv = 0.f;
    for (int n = 0; n < N; ++n) {
      dk += dsc[n] * ElemTraits<T>::to_f(base[(size_t)n * ldq + h * dh + c]);
      dv += pd[n] * ElemTraits<T>::to_f(dctx[((size_t)b * N + n) * D + h * dh + c]);
    }
    dqkv[((size_t)b * N + m) * ldq + D + h * dh + c] = ElemTraits<T>::from_f(dk * scale);
    dqkv[((size_t)b * N + m) * ldq + 2 * D + h * dh + c] = ElemTraits<T>::from_f(dv);
  }
}

__global__ void rng_advance_kernel(int64_t* rng) {
  if (threadIdx.x == 0 && blockIdx.x == 0) rng[1] += 1;
}

// ------------------------------------------------------------ multi-head attention core
// qkv [B*N][ldq] (dtype): head h reads q at column h*DH, k at D + h*DH, v at 2D + h*DH (D =
// heads*DH: the query/key/value Linear outputs side by side, one GEMM); ctx [B*N][D] (dtype) =
// softmax(q k^T * scale) v per head (transformer_unet.py:146-154); lse [B][heads][N] = row
// log-sum-exp of the scaled scores (saved for the backward, which recomputes P).
// Lane mapping: a query (or key) row owns SL = DH/16 consecutive lanes, 16 dims each; 64-row
// key/value (query/dout) tiles are staged in LDS as fp32; online softmax over the tiles.
constexpr int MHA_T = 64;

template <typename T, int DH>
__device__ __forceinline__ void stage_rows(float* dst, const T* src, int ldsrc, int r0, int N) {
  constexpr int CH = DH / 8;
  for (int e = threadIdx.x; e < MHA_T * CH; e += 256) {
    const int r = e / CH, c = (e - r * CH) * 8;
    float v[8];
    if (r0 + r < N) {
      load8<T>(src + (size_t)(r0 + r) * ldsrc + c, v);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = 0.f;
    }
    st8f(dst + r * DH + c, v);
  }
}

template <int SL>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = 1; o < SL; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T, int DH>
__global__ void __launch_bounds__(256) mha_fwd_kernel(int N, int heads, int ldq, float scale,
                                                      const T* __restrict__ qkv, T* __restrict__ ctx,
                                                      float* __restrict__ lse) {
  constexpr int SL = DH / 16, RPW = 64 / SL, RPB = 4 * RPW;
  __shared__ float Ks[MHA_T * DH], Vs[MHA_T * DH];
  const int b = blockIdx.z, h = blockIdx.y;
  const int D = heads * DH;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sl = lane % SL;
  const int row = blockIdx.x * RPB + wave * RPW + lane / SL;
  const T* base = qkv + (size_t)b * N * ldq;
  float q[16], o[16];
  if (row < N) {
    load16<T>(base + (size_t)row * ldq + h * DH + sl * 16, q);
  } else {
#pragma unroll
    for (int d = 0; d < 16; ++d) q[d] = 0.f;
  }
#pragma unroll
  for (int d = 0; d < 16; ++d) o[d] = 0.f;
  float m = -INFINITY, l = 0.f;
  for (int t0 = 0; t0 < N; t0 += MHA_T) {
    __syncthreads();
    stage_rows<T, DH>(Ks, base + D + h * DH, ldq, t0, N);
    stage_rows<T, DH>(Vs, base + 2 * D + h * DH, ldq, t0, N);
    __syncthreads();
    const int jn = min(MHA_T, N - t0);
    float s[MHA_T];
    float mt = -INFINITY;
#pragma unroll
    for (int j = 0; j < MHA_T; ++j) {
      float a = 0.f;
      const float* kr = Ks + j * DH + sl * 16;
#pragma unroll
      for (int d = 0; d < 16; ++d) a += q[d] * kr[d];
      a = group_sum<SL>(a) * scale;
      if (j < jn) mt = fmaxf(mt, a);
      s[j] = a;
    }
    const float mn = fmaxf(m, mt);
    const float corr = expf(m - mn);
    l *= corr;
#pragma unroll
    for (int d = 0; d < 16; ++d) o[d] *= corr;
#pragma unroll
    for (int j = 0; j < MHA_T; ++j) {
      const float pj = j < jn ? expf(s[j] - mn) : 0.f;
      l += pj;
      const float* vr = Vs + j * DH + sl * 16;
#pragma unroll
      for (int d = 0; d < 16; ++d) o[d] += pj * vr[d];
    }
    m = mn;
  }
  if (row < N) {
    const float inv = 1.f / l;
#pragma unroll
    for (int d = 0; d < 16; ++d) o[d] *= inv;
    store16<T>(ctx + ((size_t)b * N + row) * D + h * DH + sl * 16, o);
    if (sl == 0) lse[((size_t)b * heads + h) * N + row] = m + logf(l);
  }
}

// dQ (and dvec[row] = sum dctx*ctx, used by the key-side kernel): rows are queries
template <typename T, int DH>
__global__ void __launch_bounds__(256) mha_bwd_q_kernel(int N, int heads, int ldq, float scale,
                                                        const T* __restrict__ qkv, const T* __restrict__ ctx,
                                                        const T* __restrict__ dctx, const float* __restrict__ lse,
                                                        float* __restrict__ dvec, T* __restrict__ dqkv) {
  constexpr int SL = DH / 16, RPW = 64 / SL, RPB = 4 * RPW;
  __shared__ float Ks[MHA_T * DH], Vs[MHA_T * DH];
  const int b = blockIdx.z, h = blockIdx.y;
  const int D = heads * DH;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sl = lane % SL;
  const int row = blockIdx.x * RPB + wave * RPW + lane / SL;
  const bool valid = row < N;
  const T* base = qkv + (size_t)b * N * ldq;
  float q[16], dO[16], dq[16];
  float Di = 0.f, L = 0.f;
  if (valid) {
    const size_t off = ((size_t)b * N + row) * D + h * DH + sl * 16;
    float oo[16];
    load16<T>(base + (size_t)row * ldq + h * DH + sl * 16, q);
    load16<T>(dctx + off, dO);
    load16<T>(ctx + off, oo);
#pragma unroll
    for (int d = 0; d < 16; ++d) Di += dO[d] * oo[d];
    L = lse[((size_t)b * heads + h) * N + row];
  } else {
#pragma unroll
    for (int d = 0; d < 16; ++d) q[d] = dO[d] = 0.f;
  }
  Di = group_sum<SL>(Di);
  if (valid && sl == 0) dvec[((size_t)b * heads + h) * N + row] = Di;
#pragma unroll
  for (int d = 0; d < 16; ++d) dq[d] = 0.f;
  for (int t0 = 0; t0 < N; t0 += MHA_T) {
    __syncthreads();
    stage_rows<T, DH>(Ks, base + D + h * DH, ldq, t0, N);
    stage_rows<T, DH>(Vs, base + 2 * D + h * DH, ldq, t0, N);
    __syncthreads();
    const int jn = min(MHA_T, N - t0);
    for (int j = 0; j < jn; ++j) {
      const float* kr = Ks + j * DH + sl * 16;
      const float* vr = Vs + j * DH + sl * 16;
      float a = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        a += q[d] * kr[d];
        dp += dO[d] * vr[d];
      }
      a = group_sum<SL>(a) * scale;
      dp = group_sum<SL>(dp);
      const float p = valid ? expf(a - L) : 0.f;
      const float ds = p * (dp - Di);
#pragma unroll
      for (int d = 0; d < 16; ++d) dq[d] += ds * kr[d];
    }
  }
  if (valid) {
#pragma unroll
    for (int d = 0; d < 16; ++d) dq[d] *= scale;
    store16<T>(dqkv + ((size_t)b * N + row) * ldq + h * DH + sl * 16, dq);
  }
}

// dK, dV: rows are keys; query rows (q, dctx, lse, dvec) are staged in LDS
template <typename T, int DH>
__global__ void __launch_bounds__(256) mha_bwd_kv_kernel(int N, int heads, int ldq, float scale,
                                                         const T* __restrict__ qkv, const T* __restrict__ dctx,
                                                         const float* __restrict__ lse, const float* __restrict__ dvec,
                                                         T* __restrict__ dqkv) {
  constexpr int SL = DH / 16, RPW = 64 / SL, RPB = 4 * RPW;
  __shared__ float Qs[MHA_T * DH], Gs[MHA_T * DH], Ls[MHA_T], Ds[MHA_T];
  const int b = blockIdx.z, h = blockIdx.y;
  const int D = heads * DH;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sl = lane % SL;
  const int row = blockIdx.x * RPB + wave * RPW + lane / SL;   // key index
  const bool valid = row < N;
  const T* base = qkv + (size_t)b * N * ldq;
  float k[16], v[16], dk[16], dv[16];
  if (valid) {
    load16<T>(base + (size_t)row * ldq + D + h * DH + sl * 16, k);
    load16<T>(base + (size_t)row * ldq + 2 * D + h * DH + sl * 16, v);
  } else {
#pragma unroll
    for (int d = 0; d < 16; ++d) k[d] = v[d] = 0.f;
  }
#pragma unroll
  for (int d = 0; d < 16; ++d) dk[d] = dv[d] = 0.f;
  const float* lb = lse + ((size_t)b * heads + h) * N;
  const float* db = dvec + ((size_t)b * heads + h) * N;
  for (int t0 = 0; t0 < N; t0 += MHA_T) {
    __syncthreads();
    stage_rows<T, DH>(Qs, base + h * DH, ldq, t0, N);
    stage_rows<T, DH>(Gs, dctx + (size_t)b * N * D + h * DH, D, t0, N);
    for (int e = threadIdx.x; e < MHA_T; e += 256) {
      Ls[e] = t0 + e < N ? lb[t0 + e] : 0.f;
      Ds[e] = t0 + e < N ? db[t0 + e] : 0.f;
    }
    __syncthreads();
    const int in = min(MHA_T, N - t0);
    for (int i = 0; i < in; ++i) {
      const float* qr = Qs + i * DH + sl * 16;
      const float* gr = Gs + i * DH + sl * 16;
      float a = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        a += qr[d] * k[d];
        dp += gr[d] * v[d];
      }
      a = group_sum<SL>(a) * scale;
      dp = group_sum<SL>(dp);
      const float p = valid ? expf(a - Ls[i]) : 0.f;
      const float ds = p * (dp - Ds[i]);
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        dv[d] += p * gr[d];
        dk[d] += ds * qr[d];
      }
    }
  }
  if (valid) {
#pragma unroll
    for (int d = 0; d < 16; ++d) dk[d] *= scale;
    T* dst = dqkv + ((size_t)b * N + row) * ldq + D + h * DH + sl * 16;
    store16<T>(dst, dk);
    store16<T>(dst + D, dv);
  }
}

// ------------------------------------------------------------ UpsamplingBilinear2d(scale 2)
// nn.UpsamplingBilinear2d = F.interpolate(bilinear, align_corners=True): src = dst*(in-1)/(out-1).
__device__ __forceinline__ void ac_axis(int dst, int in, float sc, int& i0, int& i1, float& l0, float& l1) {
  const float src = sc * (float)dst;
  i0 = (int)src;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = src - (float)i0;
  l0 = 1.f - l1;
}
inline float ac_scale(int in, int out) { return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f; }

template <typename T>
__global__ void upsample2_ac_kernel(int B, int C, int Hi, int Wi, float sh, float sw, const T* __restrict__ x,
                                    T* __restrict__ y) {
  const int Ho = 2 * Hi, Wo = 2 * Wi, cpp = C >> 3;
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
    ac_axis(oh, Hi, sh, h0, h1, lh0, lh1);
    ac_axis(ow, Wi, sw, w0, w1, lw0, lw1);
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

// weight of output index o on input index i along one axis (the forward's own arithmetic)
__device__ __forceinline__ float ac_weight(int o, int i, int in, float sc) {
  int i0, i1;
  float l0, l1;
  ac_axis(o, in, sc, i0, i1, l0, l1);
  return (i0 == i ? l0 : 0.f) + (i1 == i ? l1 : 0.f);
}
__device__ __forceinline__ void ac_range(int i, int out, float sc, int& o0, int& o1) {
  if (sc <= 0.f) { o0 = 0; o1 = out - 1; return; }
  o0 = max(0, (int)floorf((float)(i - 1) / sc) - 1);
  o1 = min(out - 1, (int)ceilf((float)(i + 1) / sc) + 1);
}

// dx[b][ih][iw] = sum_{oh, ow} wh(oh, ih) * ww(ow, iw) * dy[b][oh][ow]  (gather: deterministic)
template <typename T>
__global__ void upsample2_ac_bwd_kernel(int B, int C, int Hi, int Wi, float sh, float sw, const T* __restrict__ dy,
                                        T* __restrict__ dx) {
  const int Ho = 2 * Hi, Wo = 2 * Wi, cpp = C >> 3;
  const int64_t total = (int64_t)B * Hi * Wi * cpp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t p = e / cpp;
    const int iw = (int)(p % Wi);
    p /= Wi;
    const int ih = (int)(p % Hi);
    const int b = (int)(p / Hi);
    int oh0, oh1, ow0, ow1;
    ac_range(ih, Ho, sh, oh0, oh1);
    ac_range(iw, Wo, sw, ow0, ow1);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int oh = oh0; oh <= oh1; ++oh) {
      const float wh = ac_weight(oh, ih, Hi, sh);
      if (wh == 0.f) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const float ww = ac_weight(ow, iw, Wi, sw);
        if (ww == 0.f) continue;
        float g[8];
        load8<T>(dy + (((size_t)b * Ho + oh) * Wo + ow) * C + ck * 8, g);
        const float wgt = wh * ww;
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += wgt * g[q];
      }
    }
    store8<T>(dx + (size_t)e * 8, acc);
  }
}

// UpsamplingBilinear2d(scale_factor = s) (align_corners) on fp32 NCHW planes, any output size:
// SegmentationHead(upsampling > 1) (:272-276) after the head conv's logits.  The backward is the
// same gather as upsample2_ac_bwd_kernel (deterministic).
__global__ void upsample_ac_planes_kernel(int64_t planes, int Hi, int Wi, int Ho, int Wo, float sh, float sw,
                                          const float* __restrict__ x, float* __restrict__ y) {
  const int64_t total = planes * Ho * Wo;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ow = (int)(e % Wo);
    int64_t p = e / Wo;
    const int oh = (int)(p % Ho);
    p /= Ho;
    int h0, h1, w0, w1;
    float lh0, lh1, lw0, lw1;
    ac_axis(oh, Hi, sh, h0, h1, lh0, lh1);
    ac_axis(ow, Wi, sw, w0, w1, lw0, lw1);
    const float* xp = x + (size_t)p * Hi * Wi;
    y[e] = lh0 * (lw0 * xp[h0 * Wi + w0] + lw1 * xp[h0 * Wi + w1]) + lh1 * (lw0 * xp[h1 * Wi + w0] + lw1 * xp[h1 * Wi + w1]);
  }
}

__global__ void upsample_ac_planes_bwd_kernel(int64_t planes, int Hi, int Wi, int Ho, int Wo, float sh, float sw,
                                              const float* __restrict__ dy, float* __restrict__ dx) {
  const int64_t total = planes * Hi * Wi;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int iw = (int)(e % Wi);
    int64_t p = e / Wi;
    const int ih = (int)(p % Hi);
    p /= Hi;
    int oh0, oh1, ow0, ow1;
    ac_range(ih, Ho, sh, oh0, oh1);
    ac_range(iw, Wo, sw, ow0, ow1);
    const float* g = dy + (size_t)p * Ho * Wo;
    float acc = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
      const float wh = ac_weight(oh, ih, Hi, sh);
      if (wh == 0.f) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const float ww = ac_weight(ow, iw, Wi, sw);
        if (ww != 0.f) acc += wh * ww * g[oh * Wo + ow];
      }
    }
    dx[e] = acc;
  }
}

// ------------------------------------------------------------ column copy (concat / split)
template <typename T>
__global__ void copy_cols_kernel(int64_t M, int ncols, const T* __restrict__ src, int lds, T* __restrict__ dst,
                                 int ldd, int accumulate) {
  const int cpr = ncols >> 3;
  const int64_t total = M * cpr;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t m = e / cpr;
    const int c = (int)(e - m * cpr) * 8;
    float v[8];
    load8<T>(src + m * lds + c, v);
    if (accumulate) {
      float o[8];
      load8<T>(dst + m * ldd + c, o);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += o[q];
    }
    store8<T>(dst + m * ldd + c, v);
  }
}

// ------------------------------------------------------------ 3x3 segmentation head (+bias)
// logits NCHW fp32 [B][Cout][H][W] = bias + conv3x3(x) (x NHWC dtype [B][H][W][C], C <= 64, Cout <= 4)
constexpr int HEAD3_MAXW = 4 * 64 * 9;
constexpr int HEAD3_XS = 12288;  // staged halo floats of head3_bwd (48 KB: 16 channels x 768 pixels, W <= 255)

template <typename T>
__global__ void __launch_bounds__(256) head3_fwd_kernel(int B, int H, int W, int C, int Cout,
                                                        const T* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, float* __restrict__ out) {
  __shared__ float ws[HEAD3_MAXW];   // [o][tap][c]
  for (int e = threadIdx.x; e < Cout * C * 9; e += 256) {
    const int o = e / (C * 9), r = e - o * C * 9, c = r / 9, tap = r - c * 9;
    ws[(o * 9 + tap) * C + c] = w[e];
  }
  __syncthreads();
  const int64_t M = (int64_t)B * H * W;
  for (int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x; m < M; m += (int64_t)gridDim.x * 256) {
    const int wq = (int)(m % W), hq = (int)((m / W) % H), b = (int)(m / ((int64_t)H * W));
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int tap = 0; tap < 9; ++tap) {
      const int ih = hq + tap / 3 - 1, iw = wq + tap % 3 - 1;
      if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
      const T* xp = x + (((size_t)b * H + ih) * W + iw) * C;
      for (int c0 = 0; c0 < C; c0 += 8) {
        float v[8];
        load8<T>(xp + c0, v);
        for (int o = 0; o < Cout; ++o) {
          const float* wr = ws + (o * 9 + tap) * C + c0;
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[o] += v[q] * wr[q];
        }
      }
    }
    for (int o = 0; o < Cout; ++o) out[((size_t)b * Cout + o) * H * W + (size_t)hq * W + wq] = acc[o] + bias[o];
  }
}

// dx[b][h][w][c] = sum_{o, tap} w[o][c][tap] * dl[b][o][h - kh + 1][w - kw + 1];
// partial_w[tile][o][c][tap] = sum over the tile's 256 pixels of dl[o][pix] * x[pix + shift][c];
// partial_b[tile][o] = sum of dl[o][pix]
template <typename T>
__global__ void __launch_bounds__(256) head3_bwd_kernel(int B, int H, int W, int C, int Cout,
                                                        const T* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ dl, T* __restrict__ dx,
                                                        float* __restrict__ pw, float* __restrict__ pb) {
  __shared__ float ws[HEAD3_MAXW];
  __shared__ float gs[4][256];
  for (int e = threadIdx.x; e < Cout * C * 9; e += 256) {
    const int o = e / (C * 9), r = e - o * C * 9, c = r / 9, tap = r - c * 9;
    ws[(o * 9 + tap) * C + c] = w[e];
  }
  const int64_t M = (int64_t)B * H * W;
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int HWn = H * W;
  for (int o = 0; o < 4; ++o) {
    float g = 0.f;
    if (o < Cout && m < M) {
      const int b = (int)(m / HWn), hw = (int)(m % HWn);
      g = dl[((size_t)b * Cout + o) * HWn + hw];
    }
    gs[o][threadIdx.x] = g;
  }
  __syncthreads();
  if (m < M) {
    const int wq = (int)(m % W), hq = (int)((m / W) % H), b = (int)(m / HWn);
    // the pixel's 9 x Cout logit gradients, loaded together (independent loads in flight) and kept in
    // registers across the channel chunks
    float gv[4][9];
#pragma unroll
    for (int o = 0; o < 4; ++o)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int oh = hq - (tap / 3 - 1), ow = wq - (tap % 3 - 1);
        const bool in = o < Cout && oh >= 0 && oh < H && ow >= 0 && ow < W;
        gv[o][tap] = in ? dl[((size_t)b * Cout + o) * HWn + (size_t)oh * W + ow] : 0.f;
      }
    for (int c0 = 0; c0 < C; c0 += 8) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          if (o >= Cout) break;
          const float g = gv[o][tap];
          const float* wr = ws + (o * 9 + tap) * C + c0;
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] += g * wr[q];
        }
      store8<T>(dx + (size_t)m * C + c0, acc);
    }
  }
  // weight / bias partials for this tile.  The tile's pixels with their +-(W+1) halo (one linear
  // range of NHWC rows: an in-image 3x3 neighbour of linear pixel m is m + dh*W + dw) are staged in
  // LDS as fp32, with each pixel's 9-bit in-image tap mask, so the (o, c, tap) threads walk the 256
  // pixels from LDS (a strided global load per pixel made this loop the whole kernel's time).
  const int64_t m0 = (int64_t)blockIdx.x * 256;
  const int np = (int)std::min<int64_t>(256, M - m0);
  const int nw = Cout * C * 9;
  __shared__ float xs[HEAD3_XS];
  __shared__ unsigned short tmask[256];
  const int64_t L0 = std::max<int64_t>(0, m0 - W - 1), L1 = std::min<int64_t>(M, m0 + np + W + 1);
  const bool staged = (L1 - L0) * C <= HEAD3_XS;
  if (staged) {
    const int cpp = C >> 3;
    for (int64_t e = threadIdx.x; e < (L1 - L0) * cpp; e += 256) {
      float v[8];
      load8<T>(x + (L0 + e / cpp) * C + (e % cpp) * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) xs[e * 8 + q] = v[q];
    }
    if ((int)threadIdx.x < np) {
      const int64_t mm = m0 + threadIdx.x;
      const int wq = (int)(mm % W), hq = (int)((mm / W) % H);
      unsigned t = 0;
      for (int tap = 0; tap < 9; ++tap) {
        const int ih = hq + tap / 3 - 1, iw = wq + tap % 3 - 1;
        t |= (unsigned)(ih >= 0 && ih < H && iw >= 0 && iw < W) << tap;
      }
      tmask[threadIdx.x] = (unsigned short)t;
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < nw; e += 256) {
    const int o = e / (C * 9), r = e - o * C * 9, c = r / 9, tap = r - c * 9;
    const int dh = tap / 3 - 1, dw = tap % 3 - 1;
    float s = 0.f;
    if (staged) {
      const float* xb = xs + (m0 + dh * W + dw - L0) * C + c;   // in range wherever the tap is in-image
      float s4[4] = {0.f, 0.f, 0.f, 0.f};
      int pq = 0;
      for (; pq + 4 <= np; pq += 4)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if ((tmask[pq + u] >> tap) & 1) s4[u] += gs[o][pq + u] * xb[(pq + u) * C];
      for (; pq < np; ++pq)
        if ((tmask[pq] >> tap) & 1) s4[0] += gs[o][pq] * xb[pq * C];
      s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    } else {
      for (int pq = 0; pq < np; ++pq) {
        const int64_t mm = m0 + pq;
        const int wq = (int)(mm % W), hq = (int)((mm / W) % H), b = (int)(mm / HWn);
        const int ih = hq + dh, iw = wq + dw;
        if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
        s += gs[o][pq] * ElemTraits<T>::to_f(x[(((size_t)b * H + ih) * W + iw) * C + c]);
      }
    }
    pw[(size_t)blockIdx.x * nw + e] = s;
  }
  for (int o = threadIdx.x; o < Cout; o += 256) {
    float s = 0.f;
    for (int pq = 0; pq < np; ++pq) s += gs[o][pq];
    pb[(size_t)blockIdx.x * Cout + o] = s;
  }
}


// ------------------------------------------------------------ wide column sums (bias gradients)
// partial[t][c] = sum over rows [t*64, min(M, t*64 + 64)) of x[row][c]; any C % 8 == 0 (the Linear
// layers of the ViT reach C = 3072, beyond the 2048-channel elementwise reductions)

template <typename T>
__global__ void __launch_bounds__(256) colsum_partial_kernel(int64_t M, int C, const T* __restrict__ x,
                                                             float* __restrict__ partial) {
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c0 >= C) return;
  const int64_t r0 = (int64_t)blockIdx.y * COLSUM_ROWS, r1 = min(M, r0 + COLSUM_ROWS);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t r = r0;
  // 8 rows' loads in flight per thread; the adds keep the sequential row order (same result)
  for (; r + 7 < r1; r += 8) {
    float v[8][8];
#pragma unroll
    for (int u = 0; u < 8; ++u) load8<T>(x + (r + u) * C + c0, v[u]);
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += v[u][q];
  }
  for (; r < r1; ++r) {
    float v[8];
    load8<T>(x + r * C + c0, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += v[q];
  }
  st8f(partial + (size_t)blockIdx.y * C + c0, acc);
}

// Column sums of x [M][C] added into d0 [0, n0), d1 [n0, n0 + n1), d2 [n0 + n1, C), one launch:
// the colsum_partial rows are published with write-through (sc1) stores, and the last-arriving
// workgroup of each 2048-column block sums the block's T rows in row order (eight sc1 loads in
// flight per column) and adds them -- the result of colsum_partial + slab_colsum3 without the
// second launch (the Linear bias gradients of the ViT, 49 per TransUNet step).
template <typename T>
__global__ void __launch_bounds__(256) colsum_fused_kernel(int64_t M, int C, const T* __restrict__ x, float* partial,
                                                           unsigned* cnt, int n0, int n1, float* d0, float* d1,
                                                           float* d2) {
  __shared__ int flag;
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 8;
  const int T_ = gridDim.y;
  if (c0 < C) {
    const int64_t r0 = (int64_t)blockIdx.y * COLSUM_ROWS, r1 = min(M, r0 + COLSUM_ROWS);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int64_t r = r0;
    for (; r + 7 < r1; r += 8) {
      float v[8][8];
#pragma unroll
      for (int u = 0; u < 8; ++u) load8<T>(x + (r + u) * C + c0, v[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += v[u][q];
    }
    for (; r < r1; ++r) {
      float v[8];
      load8<T>(x + r * C + c0, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += v[q];
    }
    float* row = partial + (size_t)blockIdx.y * C + c0;
#pragma unroll
    for (int q = 0; q < 8; ++q) st_sc1_dw(row + q, acc[q]);
  }
  if (!wg_last_of(cnt + blockIdx.x, T_, &flag)) return;
  // each thread sums its own 8-column chunk over the T rows in row order: two 16-B sc1 loads per
  // row, eight rows (16 loads) in flight
  if (c0 >= C) return;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int t = 0;
  for (; t + 7 < T_; t += 8) {
    f4v_t v[16];
    ld_sc1_f4x16(partial + (size_t)t * C + c0, C, v);
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) { s[q] += v[2 * u][q]; s[4 + q] += v[2 * u + 1][q]; }
  }
  for (; t < T_; ++t)
#pragma unroll
    for (int q = 0; q < 8; ++q) s[q] += ld_sc1_f(partial + (size_t)t * C + c0 + q);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = c0 + q;
    if (c < n0) d0[c] += s[q];
    else if (c < n0 + n1) d1[c - n0] += s[q];
    else d2[c - n0 - n1] += s[q];
  }
}

// ------------------------------------------------------------ head-major relayout (bf16)
// Token-major [B*N][ld] (ld = nparts * heads * dh; part p of head h at columns p*D + h*dh) <->
// head-major [heads*B][N][nparts*dh] (the layout of the flash-attention kernels of fra.hip, one
// "image" per (head, batch)).  Part 0 is multiplied by scale0 (the 1/sqrt(dh) of the scores folded
// into q; a power of two for dh = 4^k, so exact).  One thread per 8-element chunk.
__global__ void __launch_bounds__(256) heads_relayout_kernel(int unpack, int B, int N, int heads, int dh, int nparts,
                                                             float scale0, const bf16_t* __restrict__ src,
                                                             bf16_t* __restrict__ dst) {
  const int D = heads * dh, ld = nparts * D, cpr = ld / 8;   // 8-element chunks per token row
  const int64_t total = (int64_t)B * N * cpr;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = e / cpr;
    const int col = (int)(e - m * cpr) * 8;
    const int p = col / D, rem = col - p * D, h = rem / dh, j = rem - h * dh;
    const int b = (int)(m / N), n = (int)(m - (int64_t)b * N);
    const int64_t tok = m * ld + col;
    const int64_t hm = ((int64_t)(h * B + b) * N + n) * (nparts * dh) + p * dh + j;
    const bf16_t* s8 = src + (unpack ? hm : tok);
    bf16_t* d8 = dst + (unpack ? tok : hm);
    if (p == 0 && scale0 != 1.0f) {
      float v[8];
      load8<bf16_t>(s8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] *= scale0;
      store8<bf16_t>(d8, v);
    } else {
      *(uint4*)d8 = *(const uint4*)s8;
    }
  }
}

// unpack (head-major -> token-major) of dfcsa_heads_relayout with the column sums of the token-major
// output per COLSUM_ROWS-row tile (partial [tile][ld]): the q / k / v bias gradients of the
// attention backward without a colsum pass over dqkv.  Thread = one 8-element chunk column of a
// row tile; the sums add the stored (bf16) values in row order, as colsum_partial does.
__global__ void __launch_bounds__(256) heads_unpack_cs_kernel(int B, int N, int heads, int dh, int nparts,
                                                              float scale0, const bf16_t* __restrict__ src,
                                                              bf16_t* __restrict__ dst, float* __restrict__ partial) {
  const int D = heads * dh, ld = nparts * D, cpr = ld / 8;
  const int ck = blockIdx.x * 256 + threadIdx.x;
  if (ck >= cpr) return;
  const int col = ck * 8;
  const int p = col / D, rem = col - p * D, h = rem / dh, j = rem - h * dh;
  const int64_t M = (int64_t)B * N;
  const int64_t r0 = (int64_t)blockIdx.y * CS_ROWS, r1 = min(M, r0 + CS_ROWS);
  const float sc = p == 0 ? scale0 : 1.f;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t m0 = r0; m0 < r1; m0 += 4) {
    const int nr = (int)min((int64_t)4, r1 - m0);
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {   // 4 rows' loads in flight (rows past the tile re-load the last)
      const int64_t m = m0 + min(u, nr - 1);
      const int b = (int)(m / N), n = (int)(m - (int64_t)b * N);
      load8<bf16_t>(src + ((int64_t)(h * B + b) * N + n) * (nparts * dh) + p * dh + j, v[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u >= nr) break;
      if (sc != 1.f)
#pragma unroll
        for (int q = 0; q < 8; ++q) v[u][q] *= sc;
      store8<bf16_t>(dst + (m0 + u) * ld + col, v[u]);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += bf2f(f2bf(v[u][q]));
    }
  }
  st8f(partial + (size_t)blockIdx.y * ld + col, acc);
}

// ------------------------------------------------------------ attention launch helpers
template <typename T, int DH>
int mha_launch(int B, int N, int heads, int ldq, float scale, const void* qkv, const void* ctx, const void* dctx,
               const float* lse_in, float* lse_out, float* dvec, void* out, int which, hipStream_t st) {
  constexpr int RPB = 4 * (64 / (DH / 16));
  dim3 grid((N + RPB - 1) / RPB, heads, B);
  if (which == 0)
    hipLaunchKernelGGL((mha_fwd_kernel<T, DH>), grid, dim3(256), 0, st, N, heads, ldq, scale, (const T*)qkv, (T*)out,
                       lse_out);
  else if (which == 1)
    hipLaunchKernelGGL((mha_bwd_q_kernel<T, DH>), grid, dim3(256), 0, st, N, heads, ldq, scale, (const T*)qkv,
                       (const T*)ctx, (const T*)dctx, lse_in, dvec, (T*)out);
  else
    hipLaunchKernelGGL((mha_bwd_kv_kernel<T, DH>), grid, dim3(256), 0, st, N, heads, ldq, scale, (const T*)qkv,
                       (const T*)dctx, lse_in, dvec, (T*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

template <typename T>
int mha_dispatch(int dh, int B, int N, int heads, int ldq, float scale, const void* qkv, const void* ctx,
                 const void* dctx, const float* lse_in, float* lse_out, float* dvec, void* out, int which,
                 hipStream_t st) {
  switch (dh) {
    case 16: return mha_launch<T, 16>(B, N, heads, ldq, scale, qkv, ctx, dctx, lse_in, lse_out, dvec, out, which, st);
    case 32: return mha_launch<T, 32>(B, N, heads, ldq, scale, qkv, ctx, dctx, lse_in, lse_out, dvec, out, which, st);
    case 64: return mha_launch<T, 64>(B, N, heads, ldq, scale, qkv, ctx, dctx, lse_in, lse_out, dvec, out, which, st);
    default: return DFCSA_EINVAL;
  }
}

}  // namespace

// =================================================================== C ABI
extern "C" int dfcsa_wstd_fwd(const dfcsa_wstd_entry* tab, int n, int total_rows, void* stream) {
  if (!tab || n <= 0 || total_rows <= 0) return DFCSA_EINVAL;
  hipLaunchKernelGGL(wstd_fwd_kernel, dim3((total_rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, tab, n,
                     total_rows);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_wstd_bwd(const dfcsa_wstd_entry* tab, int n, int total_rows, void* stream) {
  if (!tab || n <= 0 || total_rows <= 0) return DFCSA_EINVAL;
  hipLaunchKernelGGL(wstd_bwd_kernel, dim3((total_rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, tab, n,
                     total_rows);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_im2col_input(int dtype, int B, int Csrc, int Cin, int H, int W, int k, int s, int p,
                                  const float* x, int Kpad, void* out, void* stream) {
  if (B <= 0 || Csrc <= 0 || Cin <= 0 || k <= 0 || s <= 0 || p < 0 || Kpad % 8 || Kpad < k * k * Cin)
    return DFCSA_EINVAL;
  const int Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  if (Ho <= 0 || Wo <= 0) return DFCSA_EINVAL;
  const int64_t total = (int64_t)B * Ho * Wo * (Kpad / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(im2col_input_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, Csrc,
                       Cin, H, W, k, s, p, Ho, Wo, x, Kpad, (bf16_t*)out);
  else
    hipLaunchKernelGGL(im2col_input_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, Csrc,
                       Cin, H, W, k, s, p, Ho, Wo, x, Kpad, (float*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_gn_nslices(int HW, int C) {
  // about 32 pixels per pixel-lane per slice, at most 64 slices
  const int cpp = C / 8 > 0 ? C / 8 : 1, pl = std::max(1, 256 / cpp);
  const int s = (HW + 32 * pl - 1) / (32 * pl);
  return std::max(1, std::min(64, s));
}

extern "C" int dfcsa_gn_stats(int dtype, int B, int HW, int C, int S, const void* y, float* partial, void* stream) {
  if (B <= 0 || HW <= 0 || C % 8 || C > 2048 || S <= 0) return DFCSA_EINVAL;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(gn_stats_kernel<bf16_t>, dim3(S, B), dim3(256), 0, (hipStream_t)stream, HW, C, S,
                       (const bf16_t*)y, partial);
  else
    hipLaunchKernelGGL(gn_stats_kernel<float>, dim3(S, B), dim3(256), 0, (hipStream_t)stream, HW, C, S,
                       (const float*)y, partial);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_gn_finalize(int B, int HW, int C, int G, int S, const float* partial, const float* gamma,
                                 const float* beta, float eps, float* mean_rstd, float* scale_shift, void* stream) {
  if (B <= 0 || G <= 0 || C % G || S <= 0) return DFCSA_EINVAL;
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, HW, C, G, S, partial, gamma,
                     beta, eps, mean_rstd, scale_shift);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_gn_apply(int dtype, int B, int HW, int C, const void* y, const float* scale_shift,
                              const void* res, const float* res_scale_shift, int act, void* out, void* stream) {
  if (B <= 0 || HW <= 0 || C % 8) return DFCSA_EINVAL;
  const int64_t total = (int64_t)B * HW * (C / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(gn_apply_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, HW, C,
                       total, (const bf16_t*)y, scale_shift, (const bf16_t*)res, res_scale_shift, act, (bf16_t*)out);
  else
    hipLaunchKernelGGL(gn_apply_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, HW, C,
                       total, (const float*)y, scale_shift, (const float*)res, res_scale_shift, act, (float*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_gn_bwd_reduce(int dtype, int B, int HW, int C, int G, int S, const void* dout,
                                   const void* mask, const void* y, const float* mean_rstd, float* partial,
                                   void* stream) {
  if (B <= 0 || HW <= 0 || C % 8 || C > 2048 || G <= 0 || C % G || S <= 0) return DFCSA_EINVAL;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(gn_bwd_reduce_kernel<bf16_t>, dim3(S, B), dim3(256), 0, (hipStream_t)stream, HW, C, G, S,
                       (const bf16_t*)dout, (const bf16_t*)mask, (const bf16_t*)y, mean_rstd, partial);
  else
    hipLaunchKernelGGL(gn_bwd_reduce_kernel<float>, dim3(S, B), dim3(256), 0, (hipStream_t)stream, HW, C, G, S,
                       (const float*)dout, (const float*)mask, (const float*)y, mean_rstd, partial);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_gn_bwd_finalize(int B, int HW, int C, int G, int S, const float* partial, const float* gamma,
                                     float* coef, float* dgamma, float* dbeta, void* stream) {
  if (B <= 0 || G <= 0 || C % G) return DFCSA_EINVAL;
  const int Cg = C / G;
  if (Cg > 256 || (Cg & (Cg - 1))) return DFCSA_EINVAL;
  hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, B, HW, C, G,
                     S, partial, gamma, coef, dgamma, dbeta);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_gn_bwd_apply(int dtype, int B, int HW, int C, int G, const void* dout, const void* mask,
                                  const void* y, const float* mean_rstd, const float* gamma, const float* coef,
                                  void* dy, void* dz_out, void* stream) {
  if (B <= 0 || HW <= 0 || C % 8 || G <= 0 || C % G) return DFCSA_EINVAL;
  const int64_t total = (int64_t)B * HW * (C / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(gn_bwd_apply_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, HW, C,
                       G, total, (const bf16_t*)dout, (const bf16_t*)mask, (const bf16_t*)y, mean_rstd, gamma, coef,
                       (bf16_t*)dy, (bf16_t*)dz_out);
  else
    hipLaunchKernelGGL(gn_bwd_apply_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, HW, C,
                       G, total, (const float*)dout, (const float*)mask, (const float*)y, mean_rstd, gamma, coef,
                       (float*)dy, (float*)dz_out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// channel chunk of the fused GroupNorm reductions: 128 channels (whole groups) when C > 128 splits so
// (knob 50 = 0: one chunk, the round-5 layout), else all C
int g_gn_chunk = 1;
static int gn_chunk_w(int C) { return (g_gn_chunk && C > 128 && C % 128 == 0) ? 128 : C; }
static int gn_chunk(int C, int G) {
  const int Cg = (G > 0 && C % G == 0) ? C / G : 0;
  const int cw = gn_chunk_w(C);
  return (Cg > 0 && cw % Cg == 0) ? cw : C;
}

extern "C" int dfcsa_gn_nslices_fused(int B, int HW, int C) {
  // about 512 workgroups over the batch and the channel chunks, at least 4 pixels per pixel-lane, at
  // most 64 slices (any S is valid for the launch: the rows buffer is B * S * 2C floats either way)
  const int CW = gn_chunk_w(C), nck = C / CW;
  const int cpp = CW / 8 > 0 ? CW / 8 : 1, pl = std::max(1, 256 / cpp);
  int s = (512 + std::max(1, B * nck) - 1) / std::max(1, B * nck);
  s = std::min(s, 64);
  s = std::min(s, std::max(1, HW / (4 * pl)));
  return std::max(1, s);
}

static bool gn_fused_ok(int B, int HW, int C, int G, int S) {
  return B > 0 && HW > 0 && C % 8 == 0 && C <= 1024 && G > 0 && G <= 256 && C % G == 0 && S > 0 && S <= HW;
}

extern "C" int dfcsa_gn_stats_fused(int dtype, int B, int HW, int C, int G, int S, const void* y, float* rows,
                                    const float* gamma, const float* beta, float eps, float* mean_rstd,
                                    float* scale_shift, void* stream) {
  if (!gn_fused_ok(B, HW, C, G, S) || !rows) return DFCSA_EINVAL;
  const int CW = gn_chunk(C, G), nck = C / CW;
  unsigned* cnt = dfcsa_ticket_alloc(B * nck);
  if (!cnt) return DFCSA_EINVAL;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(gn_stats_fin_kernel<bf16_t>, dim3(S, B, nck), dim3(256), 0, (hipStream_t)stream, HW, C, CW, G,
                       S, (const bf16_t*)y, rows, cnt, gamma, beta, eps, mean_rstd, scale_shift);
  else
    hipLaunchKernelGGL(gn_stats_fin_kernel<float>, dim3(S, B, nck), dim3(256), 0, (hipStream_t)stream, HW, C, CW, G,
                       S, (const float*)y, rows, cnt, gamma, beta, eps, mean_rstd, scale_shift);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_gn_bwd_reduce_fused(int dtype, int B, int HW, int C, int G, int S, const void* dout,
                                         const void* mask, const void* y, const float* mean_rstd, const float* gamma,
                                         float* rows, double* work, float* coef, float* dgamma, float* dbeta,
                                         void* stream) {
  if (!gn_fused_ok(B, HW, C, G, S) || !rows || !work) return DFCSA_EINVAL;
  const int CW = gn_chunk(C, G), nck = C / CW;
  unsigned* cnt = dfcsa_ticket_alloc((B + 1) * nck);
  if (!cnt) return DFCSA_EINVAL;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(gn_bwd_reduce_fin_kernel<bf16_t>, dim3(S, B, nck), dim3(256), 0, (hipStream_t)stream, HW, C,
                       CW, G, S,
                       (const bf16_t*)dout, (const bf16_t*)mask, (const bf16_t*)y, mean_rstd, gamma, rows, work, cnt,
                       coef, dgamma, dbeta);
  else
    hipLaunchKernelGGL(gn_bwd_reduce_fin_kernel<float>, dim3(S, B, nck), dim3(256), 0, (hipStream_t)stream, HW, C,
                       CW, G, S,
                       (const float*)dout, (const float*)mask, (const float*)y, mean_rstd, gamma, rows, work, cnt,
                       coef, dgamma, dbeta);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_maxpool3s2_fwd(int dtype, int B, int H, int W, int C, const void* x, void* out, void* idx,
                                    void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || C % 8) return DFCSA_EINVAL;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int64_t total = (int64_t)B * Ho * Wo * (C / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(maxpool3s2_fwd_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, H,
                       W, C, Ho, Wo, (const bf16_t*)x, (bf16_t*)out, (uint8_t*)idx);
  else
    hipLaunchKernelGGL(maxpool3s2_fwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, H,
                       W, C, Ho, Wo, (const float*)x, (float*)out, (uint8_t*)idx);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_maxpool3s2_bwd(int dtype, int B, int H, int W, int C, const void* idx, const void* dout,
                                    void* dx, void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || C % 8) return DFCSA_EINVAL;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int64_t total = (int64_t)B * H * W * (C / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, H,
                       W, C, Ho, Wo, (const uint8_t*)idx, (const bf16_t*)dout, (bf16_t*)dx);
  else
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, H,
                       W, C, Ho, Wo, (const uint8_t*)idx, (const float*)dout, (float*)dx);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_col2im(int dtype, int B, int H, int W, int C, int Ho, int Wo, int k, int s, int p,
                            const void* dcols, void* dx, int accumulate, void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || C % 8 || k <= 0 || s <= 0 || p < 0) return DFCSA_EINVAL;
  if (Ho != (H + 2 * p - k) / s + 1 || Wo != (W + 2 * p - k) / s + 1) return DFCSA_EINVAL;
  const int64_t total = (int64_t)B * H * W * (C / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(col2im_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, H, W, C,
                       Ho, Wo, k, s, p, (const bf16_t*)dcols, (bf16_t*)dx, accumulate);
  else
    hipLaunchKernelGGL(col2im_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, H, W, C,
                       Ho, Wo, k, s, p, (const float*)dcols, (float*)dx, accumulate);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_ln_fwd(int dtype, int rows, int C, const float* x, const float* gamma, const float* beta,
                            float eps, void* y, float* mean_rstd, void* stream) {
  if (rows <= 0 || C % 8 || C > 64 * 8 * LN_MAXCH) return DFCSA_EINVAL;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(ln_fwd_kernel<bf16_t>, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, rows, C, x,
                       gamma, beta, eps, (bf16_t*)y, mean_rstd);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<float>, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, rows, C, x,
                       gamma, beta, eps, (float*)y, mean_rstd);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_ln_bwd_ntiles(int rows) {
  const int per_block = 4 * LN_ROWS_PER_WAVE;
  return ((rows + per_block - 1) / per_block) * 4;
}

extern "C" int dfcsa_ln_bwd(int dtype, int rows, int C, const void* dy, const float* x, const float* mean_rstd,
                            const float* gamma, const float* dres, float* dx, float* partial, void* stream) {
  if (rows <= 0 || C % 8 || C > 64 * 8 * LN_MAXCH) return DFCSA_EINVAL;
  const int blocks = dfcsa_ln_bwd_ntiles(rows) / 4;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(ln_bwd_kernel<bf16_t>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, rows, C,
                       (const bf16_t*)dy, x, mean_rstd, gamma, dres, dx, partial);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, rows, C,
                       (const float*)dy, x, mean_rstd, gamma, dres, dx, partial);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_drop_add_fwd(int dtype, int64_t n, const void* a, const float* pos, int64_t L, const float* res,
                                  float p, const int64_t* rng, int site, float* out, void* stream) {
  if (n <= 0 || n % 8 || (pos && (L <= 0 || L % 8)) || p < 0.f || p >= 1.f || (p > 0.f && !rng))
    return DFCSA_EINVAL;
  const int g = grid_for(n / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(drop_add_fwd_kernel<bf16_t>, dim3(g), dim3(256), 0, (hipStream_t)stream, n, (const bf16_t*)a,
                       pos, L, res, p, rng, site, out);
  else
    hipLaunchKernelGGL(drop_add_fwd_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, n, (const float*)a,
                       pos, L, res, p, rng, site, out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_drop_bwd(int dtype, int64_t n, const float* dout, float p, const int64_t* rng, int site, void* da,
                              void* stream) {
  if (n <= 0 || n % 8 || p < 0.f || p >= 1.f || (p > 0.f && !rng)) return DFCSA_EINVAL;
  const int g = grid_for(n / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(drop_bwd_kernel<bf16_t>, dim3(g), dim3(256), 0, (hipStream_t)stream, n, dout, p, rng, site,
                       (bf16_t*)da);
  else
    hipLaunchKernelGGL(drop_bwd_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, n, dout, p, rng, site,
                       (float*)da);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_gelu_drop_fwd(int dtype, int64_t n, const void* x, float p, const int64_t* rng, int site,
                                   void* out, void* stream) {
  if (n <= 0 || n % 8 || p < 0.f || p >= 1.f || (p > 0.f && !rng)) return DFCSA_EINVAL;
  const int g = grid_for(n / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(gelu_drop_fwd_kernel<bf16_t>, dim3(g), dim3(256), 0, (hipStream_t)stream, n, (const bf16_t*)x,
                       p, rng, site, (bf16_t*)out);
  else
    hipLaunchKernelGGL(gelu_drop_fwd_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, n, (const float*)x, p,
                       rng, site, (float*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_gelu_drop_bwd(int dtype, int64_t n, const void* x, const void* dout, float p, const int64_t* rng,
                                   int site, void* dx, void* stream) {
  if (n <= 0 || n % 8 || p < 0.f || p >= 1.f || (p > 0.f && !rng)) return DFCSA_EINVAL;
  const int g = grid_for(n / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(gelu_drop_bwd_kernel<bf16_t>, dim3(g), dim3(256), 0, (hipStream_t)stream, n, (const bf16_t*)x,
                       (const bf16_t*)dout, p, rng, site, (bf16_t*)dx);
  else
    hipLaunchKernelGGL(gelu_drop_bwd_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, n, (const float*)x,
                       (const float*)dout, p, rng, site, (float*)dx);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

template <bool GELU>
static int launch_drop_cs(int dtype, int64_t M, int C, const void* x, const void* dout, float p, const int64_t* rng,
                          int site, void* out, float* partial, int64_t partial_floats, hipStream_t st) {
  if (M <= 0 || C <= 0 || C % 8 || p < 0.f || p >= 1.f || (p > 0.f && !rng) || !dout || !out || !partial ||
      (GELU && !x))
    return DFCSA_EINVAL;
  const int64_t nt = (M + CS_ROWS - 1) / CS_ROWS;
  if (nt * C > partial_floats) return DFCSA_EINVAL;
  dim3 grid((C / 8 + 255) / 256, (unsigned)nt);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL((drop_bwd_cs_kernel<bf16_t, GELU>), grid, dim3(256), 0, st, M, C, (const bf16_t*)x, dout, p,
                       rng, site, (bf16_t*)out, partial);
  else
    hipLaunchKernelGGL((drop_bwd_cs_kernel<float, GELU>), grid, dim3(256), 0, st, M, C, (const float*)x, dout, p, rng,
                       site, (float*)out, partial);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_cs_ntiles(int64_t M) { return (int)((M + CS_ROWS - 1) / CS_ROWS); }

extern "C" int dfcsa_drop_bwd_cs(int dtype, int64_t M, int C, const float* dout, float p, const int64_t* rng, int site,
                                 void* da, float* partial, int64_t partial_floats, void* stream) {
  return launch_drop_cs<false>(dtype, M, C, nullptr, dout, p, rng, site, da, partial, partial_floats,
                               (hipStream_t)stream);
}

extern "C" int dfcsa_gelu_drop_bwd_cs(int dtype, int64_t M, int C, const void* x, const void* dout, float p,
                                      const int64_t* rng, int site, void* dx, float* partial, int64_t partial_floats,
                                      void* stream) {
  return launch_drop_cs<true>(dtype, M, C, x, dout, p, rng, site, dx, partial, partial_floats, (hipStream_t)stream);
}

extern "C" int dfcsa_batch_sum(int dtype, int B, int64_t L, const void* x, float* out, void* stream) {
  if (B <= 0 || L <= 0) return DFCSA_EINVAL;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(batch_sum_kernel<bf16_t>, dim3(grid_for(L)), dim3(256), 0, (hipStream_t)stream, B, L,
                       (const bf16_t*)x, out);
  else
    hipLaunchKernelGGL(batch_sum_kernel<float>, dim3(grid_for(L)), dim3(256), 0, (hipStream_t)stream, B, L,
                       (const float*)x, out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_rng_advance(int64_t* state, void* stream) {
  if (!state) return DFCSA_EINVAL;
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, state);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_heads_relayout(int unpack, int B, int N, int heads, int dh, int nparts, float scale0,
                                    const void* src, void* dst, void* stream) {
  if (B <= 0 || N <= 0 || heads <= 0 || dh <= 0 || dh % 8 || nparts <= 0 || !src || !dst) return DFCSA_EINVAL;
  const int64_t chunks = (int64_t)B * N * nparts * heads * dh / 8;
  hipLaunchKernelGGL(heads_relayout_kernel, dim3(grid_for(chunks)), dim3(256), 0, (hipStream_t)stream, unpack, B, N,
                     heads, dh, nparts, scale0, (const bf16_t*)src, (bf16_t*)dst);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_heads_unpack_cs(int B, int N, int heads, int dh, int nparts, float scale0, const void* src,
                                     void* dst, float* partial, int64_t partial_floats, void* stream) {
  if (B <= 0 || N <= 0 || heads <= 0 || dh <= 0 || dh % 8 || nparts <= 0 || !src || !dst || !partial)
    return DFCSA_EINVAL;
  const int64_t M = (int64_t)B * N, ld = (int64_t)nparts * heads * dh;
  const int64_t nt = (M + CS_ROWS - 1) / CS_ROWS;
  if (nt * ld > partial_floats) return DFCSA_EINVAL;
  dim3 grid((unsigned)((ld / 8 + 255) / 256), (unsigned)nt);
  hipLaunchKernelGGL(heads_unpack_cs_kernel, grid, dim3(256), 0, (hipStream_t)stream, B, N, heads, dh, nparts, scale0,
                     (const bf16_t*)src, (bf16_t*)dst, partial);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_mha_fwd(int dtype, int B, int N, int heads, int dh, int ldq, float scale, const void* qkv,
                             void* ctx, float* lse, void* stream) {
  if (B <= 0 || N <= 0 || heads <= 0 || ldq < 3 * heads * dh || ldq % 8) return DFCSA_EINVAL;
  if (dtype == DFCSA_DT_BF16)
    return mha_dispatch<bf16_t>(dh, B, N, heads, ldq, scale, qkv, nullptr, nullptr, nullptr, lse, nullptr, ctx, 0,
                                (hipStream_t)stream);
  return mha_dispatch<float>(dh, B, N, heads, ldq, scale, qkv, nullptr, nullptr, nullptr, lse, nullptr, ctx, 0,
                             (hipStream_t)stream);
}

extern "C" int dfcsa_mha_drop_fwd(int dtype, int B, int N, int heads, int dh, int ldq, float scale, const void* qkv,
                                  float p, const int64_t* rng, int site, float* probs, void* ctx, void* stream) {
  if (B <= 0 || N <= 0 || N > 8192 || heads <= 0 || dh <= 0 || ldq < 3 * heads * dh || p < 0.f || p >= 1.f || !rng ||
      !probs)
    return DFCSA_EINVAL;
  const dim3 grid(N, B * heads);
  const size_t sm = (size_t)(dh + N + 4) * sizeof(float);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(mha_drop_fwd_kernel<bf16_t>, grid, dim3(256), sm, (hipStream_t)stream, N, heads, dh, ldq, scale,
                       (const bf16_t*)qkv, p, rng, site, probs, (bf16_t*)ctx);
  else
    hipLaunchKernelGGL(mha_drop_fwd_kernel<float>, grid, dim3(256), sm, (hipStream_t)stream, N, heads, dh, ldq, scale,
                       (const float*)qkv, p, rng, site, probs, (float*)ctx);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_mha_drop_bwd(int dtype, int B, int N, int heads, int dh, int ldq, float scale, const void* qkv,
                                  const void* dctx, const float* probs, float p, const int64_t* rng, int site,
                                  float* dscores, void* dqkv, void* stream) {
  if (B <= 0 || N <= 0 || N > 8192 || heads <= 0 || dh <= 0 || ldq < 3 * heads * dh || p < 0.f || p >= 1.f || !rng ||
      !probs || !dscores)
    return DFCSA_EINVAL;
  const dim3 grid(N, B * heads);
  hipStream_t st = (hipStream_t)stream;
  const size_t sm1 = (size_t)(dh + N + 4) * sizeof(float), sm2 = (size_t)2 * N * sizeof(float);
  if (dtype == DFCSA_DT_BF16) {
    hipLaunchKernelGGL(mha_drop_bwd_rows_kernel<bf16_t>, grid, dim3(256), sm1, st, N, heads, dh, ldq, scale,
                       (const bf16_t*)qkv, (const bf16_t*)dctx, probs, p, rng, site, dscores, (bf16_t*)dqkv);
    DFCSA_CHECK_LAUNCH();
    hipLaunchKernelGGL(mha_drop_bwd_cols_kernel<bf16_t>, grid, dim3(256), sm2, st, N, heads, dh, ldq, scale,
                       (const bf16_t*)qkv, (const bf16_t*)dctx, probs, p, rng, site, dscores, (bf16_t*)dqkv);
  } else {
    hipLaunchKernelGGL(mha_drop_bwd_rows_kernel<float>, grid, dim3(256), sm1, st, N, heads, dh, ldq, scale,
                       (const float*)qkv, (const float*)dctx, probs, p, rng, site, dscores, (float*)dqkv);
    DFCSA_CHECK_LAUNCH();
    hipLaunchKernelGGL(mha_drop_bwd_cols_kernel<float>, grid, dim3(256), sm2, st, N, heads, dh, ldq, scale,
                       (const float*)qkv, (const float*)dctx, probs, p, rng, site, dscores, (float*)dqkv);
  }
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_mha_bwd(int dtype, int B, int N, int heads, int dh, int ldq, float scale, const void* qkv,
                             const void* ctx, const void* dctx, const float* lse, float* dvec, void* dqkv,
                             void* stream) {
  if (B <= 0 || N <= 0 || heads <= 0 || ldq < 3 * heads * dh || ldq % 8 || !dvec) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  int rc;
  if (dtype == DFCSA_DT_BF16) {
    rc = mha_dispatch<bf16_t>(dh, B, N, heads, ldq, scale, qkv, ctx, dctx, lse, nullptr, dvec, dqkv, 1, st);
    if (rc == 0)
      rc = mha_dispatch<bf16_t>(dh, B, N, heads, ldq, scale, qkv, ctx, dctx, lse, nullptr, dvec, dqkv, 2, st);
  } else {
    rc = mha_dispatch<float>(dh, B, N, heads, ldq, scale, qkv, ctx, dctx, lse, nullptr, dvec, dqkv, 1, st);
    if (rc == 0)
      rc = mha_dispatch<float>(dh, B, N, heads, ldq, scale, qkv, ctx, dctx, lse, nullptr, dvec, dqkv, 2, st);
  }
  return rc;
}

extern "C" int dfcsa_upsample2_ac(int dtype, int B, int C, int Hi, int Wi, const void* x, void* out, void* stream) {
  if (B <= 0 || Hi <= 0 || Wi <= 0 || C % 8) return DFCSA_EINVAL;
  const float sh = ac_scale(Hi, 2 * Hi), sw = ac_scale(Wi, 2 * Wi);
  const int64_t total = (int64_t)B * 4 * Hi * Wi * (C / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(upsample2_ac_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, C, Hi,
                       Wi, sh, sw, (const bf16_t*)x, (bf16_t*)out);
  else
    hipLaunchKernelGGL(upsample2_ac_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, C, Hi,
                       Wi, sh, sw, (const float*)x, (float*)out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_upsample2_ac_bwd(int dtype, int B, int C, int Hi, int Wi, const void* dout, void* dx,
                                      void* stream) {
  if (B <= 0 || Hi <= 0 || Wi <= 0 || C % 8) return DFCSA_EINVAL;
  const float sh = ac_scale(Hi, 2 * Hi), sw = ac_scale(Wi, 2 * Wi);
  const int64_t total = (int64_t)B * Hi * Wi * (C / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(upsample2_ac_bwd_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, C,
                       Hi, Wi, sh, sw, (const bf16_t*)dout, (bf16_t*)dx);
  else
    hipLaunchKernelGGL(upsample2_ac_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, C,
                       Hi, Wi, sh, sw, (const float*)dout, (float*)dx);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_upsample_ac_f32(int64_t planes, int Hi, int Wi, int Ho, int Wo, const float* x, float* out,
                                     void* stream) {
  if (planes <= 0 || Hi <= 0 || Wi <= 0 || Ho <= 0 || Wo <= 0) return DFCSA_EINVAL;
  const int64_t total = planes * Ho * Wo;
  hipLaunchKernelGGL(upsample_ac_planes_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, planes, Hi,
                     Wi, Ho, Wo, ac_scale(Hi, Ho), ac_scale(Wi, Wo), x, out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_upsample_ac_f32_bwd(int64_t planes, int Hi, int Wi, int Ho, int Wo, const float* dout, float* dx,
                                         void* stream) {
  if (planes <= 0 || Hi <= 0 || Wi <= 0 || Ho <= 0 || Wo <= 0) return DFCSA_EINVAL;
  const int64_t total = planes * Hi * Wi;
  hipLaunchKernelGGL(upsample_ac_planes_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, planes,
                     Hi, Wi, Ho, Wo, ac_scale(Hi, Ho), ac_scale(Wi, Wo), dout, dx);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_copy_cols(int dtype, int64_t M, int ncols, const void* src, int ld_src, void* dst, int ld_dst,
                               int accumulate, void* stream) {
  if (M <= 0 || ncols <= 0 || ncols % 8 || ld_src % 8 || ld_dst % 8) return DFCSA_EINVAL;
  const int64_t total = M * (ncols / 8);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(copy_cols_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, M, ncols,
                       (const bf16_t*)src, ld_src, (bf16_t*)dst, ld_dst, accumulate);
  else
    hipLaunchKernelGGL(copy_cols_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, M, ncols,
                       (const float*)src, ld_src, (float*)dst, ld_dst, accumulate);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_head3_fwd(int dtype, int B, int H, int W, int C, int Cout, const void* x, const float* w,
                               const float* bias, float* logits, void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || C % 8 || C > 64 || Cout <= 0 || Cout > 4 || !bias) return DFCSA_EINVAL;
  const int64_t M = (int64_t)B * H * W;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(head3_fwd_kernel<bf16_t>, dim3(grid_for(M)), dim3(256), 0, (hipStream_t)stream, B, H, W, C,
                       Cout, (const bf16_t*)x, w, bias, logits);
  else
    hipLaunchKernelGGL(head3_fwd_kernel<float>, dim3(grid_for(M)), dim3(256), 0, (hipStream_t)stream, B, H, W, C, Cout,
                       (const float*)x, w, bias, logits);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_head3_ntiles(int B, int H, int W) { return (int)(((int64_t)B * H * W + 255) / 256); }

extern "C" int dfcsa_head3_bwd(int dtype, int B, int H, int W, int C, int Cout, const void* x, const float* w,
                               const float* dlogits, void* dx, float* partial_w, float* partial_b, void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || C % 8 || C > 64 || Cout <= 0 || Cout > 4) return DFCSA_EINVAL;
  const int nt = dfcsa_head3_ntiles(B, H, W);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(head3_bwd_kernel<bf16_t>, dim3(nt), dim3(256), 0, (hipStream_t)stream, B, H, W, C, Cout,
                       (const bf16_t*)x, w, dlogits, (bf16_t*)dx, partial_w, partial_b);
  else
    hipLaunchKernelGGL(head3_bwd_kernel<float>, dim3(nt), dim3(256), 0, (hipStream_t)stream, B, H, W, C, Cout,
                       (const float*)x, w, dlogits, (float*)dx, partial_w, partial_b);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_colsum_ntiles(int64_t M) { return (int)((M + COLSUM_ROWS - 1) / COLSUM_ROWS); }

extern "C" int dfcsa_colsum_fused(int dtype, int64_t M, int C, const void* x, float* partial, int n0, int n1,
                                  float* d0, float* d1, float* d2, void* stream) {
  if (M <= 0 || C <= 0 || C % 8 || !partial || !d0 || n0 < 0 || n1 < 0 || n0 + n1 > C) return DFCSA_EINVAL;
  if ((n1 > 0 && !d1) || (n0 + n1 < C && !d2)) return DFCSA_EINVAL;
  dim3 grid((C / 8 + 255) / 256, dfcsa_colsum_ntiles(M));
  unsigned* cnt = dfcsa_ticket_alloc(grid.x);
  if (!cnt) return DFCSA_EINVAL;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(colsum_fused_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, M, C, (const bf16_t*)x,
                       partial, cnt, n0, n1, d0, d1, d2);
  else
    hipLaunchKernelGGL(colsum_fused_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, M, C, (const float*)x,
                       partial, cnt, n0, n1, d0, d1, d2);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_colsum_partial(int dtype, int64_t M, int C, const void* x, float* partial, void* stream) {
  if (M <= 0 || C <= 0 || C % 8) return DFCSA_EINVAL;
  dim3 grid((C / 8 + 255) / 256, dfcsa_colsum_ntiles(M));
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(colsum_partial_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, M, C, (const bf16_t*)x,
                       partial);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, M, C, (const float*)x,
                       partial);
  DFCSA_CHECK_LAUNCH();
  return 0;
}
