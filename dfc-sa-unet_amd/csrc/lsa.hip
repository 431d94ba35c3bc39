// LightSelfAttention (reference models/unet_dfc_sa_res.py:5-39) forward and backward.
//
// The attention itself runs on the P x P pooled map (N = P*P <= 1024 tokens), so it is tiny;
// what costs HBM bandwidth is the full-resolution traffic around it: the adaptive average pool
// (read once, BN+ReLU of the producing conv applied on the fly) and, in backward, the
// transposed bilinear upsample (a weighted reduction of the full-resolution gradient onto the
// P x P grid, done separably: first along W per image row, then along H).
//
// Semantics kept exactly: adaptive_avg_pool2d windows [floor(i*H/P), ceil((i+1)*H/P)) (they
// overlap when P does not divide H, and repeat pixels when P > H); no 1/sqrt(d) scale on
// q.k; softmax over keys; o = v @ A^T; F.interpolate(bilinear, align_corners=False) with the
// source index clamped at 0; out = gamma * o + x (x added by the caller's fused stage).
// Everything here is fp32 and deterministic (fixed-order reductions, no atomics).
#include <algorithm>

#include "common.h"
#include "dfcsa_internal.h"

int g_lsa_rows_old = 0;
int g_lsa_cols_nt = 256;    // knob 35: threads of the upsample-backward column kernel at C <= 128 (256 = old)
int g_lsa_key_centre = 1;    // knob 48: 0 = uncentred dQ in the bf16 pooled-attention backward (old)
int g_lsa_pool_direct = 1;   // knob 47: 0 = large pools on the sliced pool + pooled launches (old)
int g_lsa_cols_flash = 1;    // knob 49: 0 = the bf16 flash layers' column pass + separate prep (old)
int g_lsa_pool_one_slice = 1;   // knob 46: 0 = split the <= 8-row windows of P >= 16 pools into row slices (old)

namespace {

__device__ __forceinline__ int win_lo(int i, int H, int P) { return (i * H) / P; }
__device__ __forceinline__ int win_hi(int i, int H, int P) { return ((i + 1) * H + P - 1) / P; }

// scale = (float)in / (float)out (a loop computes it once: the same correctly rounded quotient)
__device__ __forceinline__ void bilin_axis_s(int dst, int in, float scale, int& i0, int& i1, float& l0, float& l1) {
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  l0 = 1.f - l1;
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

// weight of source index `p` for destination `dst` along one axis
__device__ __forceinline__ float bilin_w(int dst, int p, int in, int out) {
  int i0, i1;
  float l0, l1;
  bilin_axis(dst, in, out, i0, i1, l0, l1);
  return (i0 == p ? l0 : 0.f) + (i1 == p ? l1 : 0.f);
}

__device__ __forceinline__ float block_reduce_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = 0.f;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) r += sh[i];
  return r;
}
__device__ __forceinline__ float block_reduce_max(float v, float* sh) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = -INFINITY;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, sh[i]);
  return r;
}

int pool_splits(int H, int P) {
  int maxwh = (H + P - 1) / P + 1;
  // large pools' small windows (P >= 16, <= 8 rows: P = 32 on 224^2 is 7 x 7) in one slice: 3 slices of
  // ~16 pixels per workgroup left the launch to workgroup overheads (114 us per launch at P = 32 with
  // the window sums); P * P windows per image are plenty of workgroups without the split
  if (P >= 16 && maxwh <= 8 && g_lsa_pool_one_slice) return 1;
  int s = (maxwh + 3) / 4;
  return s < 1 ? 1 : s;
}

// grid (S, N, B): row slice s of window n of image b.  One load in flight per lane at 45 VGPRs:
// occupancy hides the latency (an eight-loads-in-flight variant at 108 VGPRs measured slower,
// profiles/r03c_lsa_bench.jsonl).  Large pools' small windows take dfcsa_lsa_pool_direct (one wave per
// window); batching several windows per workgroup here measured slower (614 -> 690 us per step at
// P = 32, round 6) and was removed.
template <typename T, bool WS = false>
__global__ void __launch_bounds__(256) lsa_pool_kernel(int H, int W, int C, const T* __restrict__ y2,
                                                       const float* __restrict__ sc, const float* __restrict__ sh,
                                                       int P, int S, int relu, float* __restrict__ partial,
                                                       float* __restrict__ wpart) {
  const int s = blockIdx.x, n = blockIdx.y, b = blockIdx.z;
  const int pi = n / P, pj = n - pi * P;
  const int hs = win_lo(pi, H, P), he = win_hi(pi, H, P);
  const int ws = win_lo(pj, W, P), we = win_hi(pj, W, P);
  const int wh = he - hs, ww = we - ws;
  const int R = (wh + S - 1) / S;
  const int r0 = hs + s * R, r1 = min(he, r0 + R);
  const int cpp = C >> 3, pl = 256 / cpp;
  const int tid = threadIdx.x, lp = tid / cpp, ck = tid - lp * cpp, c0 = ck * 8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // WS: the window sums the attention-entry backward needs (relu mask r = [bn(y) > 0]):
  // sum r and sum r*y, so that backward's pool term is a [B][N][C] contraction
  float accr[WS ? 8 : 1], accy[WS ? 8 : 1];
  if constexpr (WS)
#pragma unroll
    for (int q = 0; q < 8; ++q) { accr[q] = 0.f; accy[q] = 0.f; }
  if (lp < pl) {
    float a[8], bb[8];
    for (int q = 0; q < 8; ++q) { a[q] = sc[c0 + q]; bb[q] = sh[c0 + q]; }
    const int npx = (r1 > r0 ? (r1 - r0) : 0) * ww;
    for (int i = lp; i < npx; i += pl) {
      const int h = r0 + i / ww, w = ws + i % ww;
      float v[8];
      load8<T>(y2 + ((size_t)(b * H + h) * W + w) * C + c0, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float t = v[q] * a[q] + bb[q];
        acc[q] += relu ? fmaxf(t, 0.f) : t;
        if constexpr (WS) {
          const float r = (!relu || t > 0.f) ? 1.f : 0.f;
          accr[q] += r;
          accy[q] += r * v[q];
        }
      }
    }
  }
  // lane partials staged element-major, red[q][stride] with stride = 256 + min(cpp, 64): the stores
  // (lanes consecutive) and the combine's reads (a wave covers chunks kk < cpp of up to 64 / cpp
  // elements q: banks 8q + kk ... distinct) are free of LDS bank conflicts (the chunk-major
  // lds_st8 staging measured 33 % conflict cycles)
  __shared__ float red[8 * (256 + 64)];
  const int stride = 256 + min(cpp, 64);
  for (int k = 0; k < (WS ? 3 : 1); ++k) {
    if (k) __syncthreads();
    if (lp < pl) {
      auto stage = [&](const float (&v)[8]) {
#pragma unroll
        for (int q = 0; q < 8; ++q) red[q * stride + tid] = v[q];
      };
      if constexpr (WS) {
        if (k == 1) stage(accr);
        else if (k == 2) stage(accy);
        else stage(acc);
      } else {
        stage(acc);
      }
    }
    __syncthreads();
    // k = 0: partial [B][N][S][C]; k = 1, 2: wpart [B][N][S][2][C]
    float* out = k == 0 ? partial + (((size_t)b * P * P + n) * S + s) * C
                        : wpart + ((((size_t)b * P * P + n) * S + s) * 2 + (k - 1)) * C;
    for (int e = tid; e < C; e += 256) {
      const int kk = e % cpp, q = e / cpp;   // element q of chunk kk: channel kk * 8 + q
      float v = 0.f;
      for (int p = 0; p < pl; ++p) v += red[q * stride + p * cpp + kk];
      out[kk * 8 + q] = v;
    }
  }
}

// Large pools (P >= 16: 7 x 7 / 14 x 14 windows at 224^2): ONE WAVE per window, 4 windows (consecutive
// pj of one pooled row) per workgroup, and the pooled values / window sums written directly -- no
// partial slices, no block barrier, no separate dfcsa_lsa_pooled_ws launch (which at P = 32 was one
// ~34 us launch of 16 k single-token workgroups per layer).  Lanes: cw = min(C / 8, 64) channel chunks
// x 64 / cw pixel lanes (C / 8 a power of two or a multiple of 64, host-checked); the pixel lanes are
// combined by xor shuffles.  Writes pooled [B][N][C] = window mean (fp32, optional), pooled16 (bf16
// copy, the projection GEMM's operand) and optional wsum [B][N][2][C] (sum r, sum r*y; see
// lsa_pool_kernel).
template <typename T, bool WS>
__global__ void __launch_bounds__(256) lsa_pool_direct_kernel(int H, int W, int C, int P, const T* __restrict__ y2,
                                                              const float* __restrict__ sc,
                                                              const float* __restrict__ sh, int relu,
                                                              float* __restrict__ pooled, bf16_t* __restrict__ pooled16,
                                                              float* __restrict__ wsum) {
  const int lane = threadIdx.x & 63, b = blockIdx.y, N = P * P;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const int pi = n / P, pj = n - pi * P;
  const int hs = win_lo(pi, H, P), he = win_hi(pi, H, P);
  const int ws = win_lo(pj, W, P), we = win_hi(pj, W, P);
  const int ww = we - ws, npx = (he - hs) * ww;
  const float inv = 1.f / (float)npx;
  const int cpp = C >> 3, cw = cpp < 64 ? cpp : 64, plw = 64 / cw;
  const int pl = lane / cw, kl = lane - pl * cw;
  const size_t orow = (size_t)b * N + n;
  for (int cb = 0; cb < cpp; cb += cw) {
    const int c0 = (cb + kl) * 8;
    float a[8], bb[8], acc[8], accr[WS ? 8 : 1], accy[WS ? 8 : 1];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      a[q] = sc[c0 + q]; bb[q] = sh[c0 + q]; acc[q] = 0.f;
      if constexpr (WS) { accr[q] = 0.f; accy[q] = 0.f; }
    }
#pragma unroll 4
    for (int i = pl; i < npx; i += plw) {
      const int h = hs + i / ww, w = ws + i % ww;
      float v[8];
      load8<T>(y2 + ((size_t)(b * H + h) * W + w) * C + c0, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float t = v[q] * a[q] + bb[q];
        acc[q] += relu ? fmaxf(t, 0.f) : t;
        if constexpr (WS) {
          const float r = (!relu || t > 0.f) ? 1.f : 0.f;
          accr[q] += r;
          accy[q] += r * v[q];
        }
      }
    }
    for (int off = cw; off < 64; off <<= 1) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        acc[q] += __shfl_xor(acc[q], off, 64);
        if constexpr (WS) {
          accr[q] += __shfl_xor(accr[q], off, 64);
          accy[q] += __shfl_xor(accy[q], off, 64);
        }
      }
    }
    if (pl == 0) {
      float m[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) m[q] = acc[q] * inv;
      if (pooled) {
        float* po = pooled + orow * C + c0;
        *(float4*)po = make_float4(m[0], m[1], m[2], m[3]);
        *(float4*)(po + 4) = make_float4(m[4], m[5], m[6], m[7]);
      }
      if (pooled16)
        *(uint4*)(pooled16 + orow * C + c0) =
            make_uint4(pack2bf(m[0], m[1]), pack2bf(m[2], m[3]), pack2bf(m[4], m[5]), pack2bf(m[6], m[7]));
      if constexpr (WS) {
        float* wr = wsum + orow * 2 * C + c0;
        *(float4*)wr = make_float4(accr[0], accr[1], accr[2], accr[3]);
        *(float4*)(wr + 4) = make_float4(accr[4], accr[5], accr[6], accr[7]);
        *(float4*)(wr + C) = make_float4(accy[0], accy[1], accy[2], accy[3]);
        *(float4*)(wr + C + 4) = make_float4(accy[4], accy[5], accy[6], accy[7]);
      }
    }
  }
}

// grid (N, B): pooled[b][n][c] = sum of the S partial slices / window area; with wpart, also the
// window sums wsum[b][n][2][c] (sum r, sum r*y over the window, summed over the S slices)
__global__ void __launch_bounds__(256) lsa_pooled_kernel(int H, int W, int C, int P, int S,
                                                         const float* __restrict__ partial, float* __restrict__ pooled,
                                                         const float* __restrict__ wpart, float* __restrict__ wsum) {
  const int n = blockIdx.x, b = blockIdx.y, N = P * P;
  const int pi = n / P, pj = n - pi * P;
  const float inv = 1.f / (float)((win_hi(pi, H, P) - win_lo(pi, H, P)) * (win_hi(pj, W, P) - win_lo(pj, W, P)));
  const float* p = partial + (((size_t)b * N + n) * S) * C;
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int k = 0; k < S; ++k) s += p[(size_t)k * C + c];
    pooled[((size_t)b * N + n) * C + c] = s * inv;
  }
  if (!wpart) return;
  const float* q = wpart + (((size_t)b * N + n) * S) * 2 * C;
  for (int e = threadIdx.x; e < 2 * C; e += 256) {
    float s = 0.f;
    for (int k = 0; k < S; ++k) s += q[(size_t)k * 2 * C + e];
    wsum[((size_t)b * N + n) * 2 * C + e] = s;
  }
}

// grid (ceil(J/256), ceil(N/16), B); J = 2Cq + C
__global__ void __launch_bounds__(256) lsa_qkv_kernel(int H, int W, int C, int Cq, int P, int S,
                                                      const float* __restrict__ partial,
                                                      const float* __restrict__ wT, const float* __restrict__ bias,
                                                      float* __restrict__ pooled, float* __restrict__ qkv) {
  extern __shared__ float prow[];  // [16][C]
  const int N = P * P, J = 2 * Cq + C;
  const int b = blockIdx.z, n0 = blockIdx.y * 16, j = blockIdx.x * 256 + threadIdx.x;
  const int nr = min(16, N - n0);
  for (int e = threadIdx.x; e < nr * C; e += 256) {
    const int r = e / C, c = e - r * C, n = n0 + r;
    const int pi = n / P, pj = n - pi * P;
    const float area = (float)((win_hi(pi, H, P) - win_lo(pi, H, P)) * (win_hi(pj, W, P) - win_lo(pj, W, P)));
    const float* p = partial + (((size_t)b * N + n) * S) * C + c;
    float s = 0.f;
    for (int k = 0; k < S; ++k) s += p[(size_t)k * C];
    const float v = s / area;
    prow[r * C + c] = v;
    if (blockIdx.x == 0) pooled[((size_t)b * N + n) * C + c] = v;
  }
  __syncthreads();
  if (j >= J) return;
  float acc[16];
  const float bj = bias[j];
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = bj;
  for (int c = 0; c < C; ++c) {
    const float w = wT[(size_t)c * J + j];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += prow[r * C + c] * w;
  }
  for (int r = 0; r < nr; ++r) qkv[((size_t)b * N + n0 + r) * J + j] = acc[r];
}

// grid (N, B): one query row per workgroup
__global__ void __launch_bounds__(256) lsa_attn_kernel(int N, int C, int Cq, const float* __restrict__ qkv,
                                                       float* __restrict__ A, float* __restrict__ o) {
  extern __shared__ float sm[];  // q [Cq] | e [N] | red [8]
  float* q = sm;
  float* e = sm + Cq;
  float* red = e + N;
  const int n = blockIdx.x, b = blockIdx.y, J = 2 * Cq + C;
  const float* base = qkv + (size_t)b * N * J;
  for (int c = threadIdx.x; c < Cq; c += 256) q[c] = base[(size_t)n * J + c];
  __syncthreads();
  float mx = -INFINITY;
  for (int m = threadIdx.x; m < N; m += 256) {
    const float* k = base + (size_t)m * J + Cq;
    float s = 0.f;
    for (int c = 0; c < Cq; ++c) s += q[c] * k[c];
    e[m] = s;
    mx = fmaxf(mx, s);
  }
  mx = block_reduce_max(mx, red);
  float sum = 0.f;
  for (int m = threadIdx.x; m < N; m += 256) {
    const float v = __expf(e[m] - mx);
    e[m] = v;
    sum += v;
  }
  sum = block_reduce_sum(sum, red);
  const float inv = 1.f / sum;
  for (int m = threadIdx.x; m < N; m += 256) {
    const float v = e[m] * inv;
    e[m] = v;
    A[((size_t)b * N + n) * N + m] = v;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int m = 0; m < N; ++m) s += e[m] * base[(size_t)m * J + 2 * Cq + c];
    o[((size_t)b * N + n) * C + c] = s;
  }
}

// Source positions of the bilinear upsample increase with the destination index, so the
// destinations that read source cell p along an axis (in -> out) form one range [lo, hi): lo a
// little before the first contributor, hi past the last (i0 > p beyond it).  The ranges are
// over-estimates; positions inside them with a zero weight are skipped, so only the summation
// split (fixed) depends on them.
__device__ __forceinline__ void contrib_range(int p, int in, int out, int& lo, int& hi) {
  lo = (int)(((float)(p - 1) + 0.5f) * (float)out / (float)in - 0.5f) - 2;
  if (lo < 0) lo = 0;
  hi = (int)(((float)p + 1.5f) * (float)out / (float)in - 0.5f) + 3;
  if (hi > out) hi = out;
}

// P <= PM: the same row reduction with every source column read once.  Lanes (column slice sl,
// 8-channel chunk ck) walk the row's columns w = sl, sl + nsl, ... eight loads in flight
// (unconditional: a load under a branch is waited for before the branch joins), each column
// adding its two bilinear weights into acc[pj] (the other pj get weight 0).  The slices are
// reduced by a butterfly inside the wave (power-of-two cpp < 64), then <= 4 partials per output
// through LDS.
template <typename T, int PM>
__global__ void __launch_bounds__(256) lsa_up_bwd_rows_pix_kernel(int H, int W, int C, const T* __restrict__ d, int P,
                                                                  float* __restrict__ rows) {
  __shared__ __attribute__((aligned(16))) float red[4 * PM * 512];
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int cpp = C >> 3, nsl = 256 / cpp;
  const int sl = tid / cpp, ck = tid - sl * cpp, c0 = ck * 8;
  const T* row = d + ((size_t)b * H + h) * W * C;   // 32-bit element offsets below
  const float bsc = (float)P / (float)W;
  float acc[PM][8];
#pragma unroll
  for (int j = 0; j < PM; ++j)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[j][q] = 0.f;
  if (sl < nsl) {
    constexpr int U = 8;
    for (int w0 = sl; w0 < W; w0 += U * nsl) {
      Raw8<T> r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) ld_raw8(at_bytes(row, (unsigned)((min(w0 + u * nsl, W - 1) * C + c0) * (int)sizeof(T))), r[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int w = w0 + u * nsl;
        float v[8];
        cvt8(r[u], v);
        int i0, i1;
        float l0, l1;
        bilin_axis_s(min(w, W - 1), P, bsc, i0, i1, l0, l1);
        if (w >= W) l0 = l1 = 0.f;
#pragma unroll
        for (int j = 0; j < PM; ++j) {
          const float wt = (i0 == j ? l0 : 0.f) + (i1 == j ? l1 : 0.f);
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[j][q] += wt * v[q];
        }
      }
    }
  }
  const bool bfly = cpp < 64 && (cpp & (cpp - 1)) == 0;
  if (bfly) {
    for (int off = cpp; off < 64; off <<= 1)
#pragma unroll
      for (int j = 0; j < PM; ++j)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[j][q] += __shfl_xor(acc[j][q], off);
  }
  const int nslot = bfly ? 4 : nsl;
  const int slot = bfly ? (tid >> 6) : sl;
  if (sl < nsl && (!bfly || (tid & 63) < cpp))
#pragma unroll
    for (int j = 0; j < PM; ++j)
      if (j < P) lds_st8(red + ((size_t)(slot * P + j) * C + c0), acc[j]);
  __syncthreads();
  float* out = rows + ((size_t)b * H + h) * P * C;
  for (int k = tid; k < P * C; k += 256) {
    float v = 0.f;
    for (int s2 = 0; s2 < nslot; ++s2) v += red[(size_t)s2 * P * C + k];
    out[k] = v;
  }
}

// grid (H, B): rows[b][h][pj][c] = sum_w wx(pj, w) * dattn[b][h][w][c].  Work items (pj, 8
// channels) x NSL slices of the w range, so all 256 threads stream the row (P * C / 8 items alone
// leave most of the workgroup idle at C = 64); slices are combined in a fixed order through LDS.
template <typename T>
__global__ void __launch_bounds__(256) lsa_up_bwd_rows_kernel(int H, int W, int C, const T* __restrict__ d, int P,
                                                              float* __restrict__ rows) {
  __shared__ __attribute__((aligned(16))) float red[256 * 8];
  const int h = blockIdx.x, b = blockIdx.y;
  const int cpp = C >> 3, items = P * cpp;
  const int nsl = items >= 256 ? 1 : 256 / items;
  const T* row = d + ((size_t)b * H + h) * W * C;
  const float bsc = (float)P / (float)W;   // bilinear source scale along W
  for (int base = 0; base < items; base += 256) {
    const int e = base + threadIdx.x % (nsl == 1 ? 256 : items), sl = nsl == 1 ? 0 : threadIdx.x / items;
    const bool on = e < items && sl < nsl;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int pj = 0, c0 = 0;
    if (on) {
      pj = e / cpp;
      c0 = (e - pj * cpp) * 8;
      int lo, hi;
      contrib_range(pj, P, W, lo, hi);
      // 4 source columns per step, loaded unconditionally (columns past the range clamped, weight 0):
      // a load under a (lane-divergent) zero-weight branch was waited for before the branch joined,
      // which serialised the four loads (the clamped / zero-weight columns are the row this workgroup
      // reads anyway: L1 / L2 hits)
      for (int w0 = lo + sl; w0 < hi; w0 += 4 * nsl) {
        float wt[4], v[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int w = w0 + u * nsl;
          const int wc = w < hi ? w : hi - 1;
          int i0, i1;
          float l0, l1;
          bilin_axis_s(wc, P, bsc, i0, i1, l0, l1);
          wt[u] = w < hi ? (i0 == pj ? l0 : 0.f) + (i1 == pj ? l1 : 0.f) : 0.f;
          load8<T>(row + (size_t)wc * C + c0, v[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] += wt[u] * v[u][q];
      }
    }
    if (nsl == 1) {
      if (on) {
        float* out = rows + (((size_t)b * H + h) * P + pj) * C + c0;
#pragma unroll
        for (int q = 0; q < 8; ++q) out[q] = acc[q];
      }
      continue;
    }
    if (on) lds_st8(red + (sl * items + e) * 8, acc);
    __syncthreads();
    for (int k = threadIdx.x; k < items * 8; k += 256) {
      const int it = k >> 3, q = k & 7;
      float v = 0.f;
      for (int s2 = 0; s2 < nsl; ++s2) v += red[(s2 * items + it) * 8 + q];
      const int pj2 = it / cpp, cc = (it - pj2 * cpp) * 8 + q;
      rows[(((size_t)b * H + h) * P + pj2) * C + cc] = v;
    }
    __syncthreads();
  }
}

// grid (ceil(N / npw), B): tokens n = blockIdx.x * npw + t, t < npw, each:
// du = sum_h wy(pi, h) rows[b][h][pj]; dO = gamma * du; gpart = sum_c o * du.
// Channels x NSL slices of the h range (all 256 threads busy at C = 64), combined in LDS.
// NT = 1024 for C <= 128: four times the row slices per output (the 224^2 level's ~84 source rows
// per pooled row were ~21 dependent loads per lane with 256 threads)
// npw > 1 (fused dgamma only: gpart then holds one partial per workgroup): large pools (P = 32: 16 k
// one-token workgroups) spent most of the launch in the dgamma ticket, one atomic per workgroup
template <int NT>
__global__ void __launch_bounds__(NT) lsa_up_bwd_cols_kernel(int H, int C, int P, int npw, const float* __restrict__ rows,
                                                             const float* __restrict__ o, const float* gamma,
                                                             float* __restrict__ dO, float* __restrict__ gpart,
                                                             unsigned* cnt, float* gamma_grad) {
  __shared__ float red[NT + 32];
  __shared__ double rd[NT];
  __shared__ int flag;
  const int b = blockIdx.y, N = P * P;
  const float gm = *gamma;
  const float bsc = (float)P / (float)H;   // bilinear source scale along H
  const int nsl = C >= NT ? 1 : NT / C;
  const int cw = nsl == 1 ? NT : C;
  const int sl = threadIdx.x / cw, cl = threadIdx.x - sl * cw;
  float gsum = 0.f;
  for (int t = 0; t < npw; ++t) {
  const int n = blockIdx.x * npw + t;
  if (n >= N) break;
  const int pi = n / P, pj = n - pi * P;
  int lo, hi;
  contrib_range(pi, P, H, lo, hi);
  for (int cb = 0; cb < C; cb += cw) {
    const int c = cb + cl;
    float s = 0.f;
    if (c < C && sl < nsl) {
      // 8 independent loads in flight, unconditional (rows past the range clamped, weight 0): a
      // load under a branch is waited for before the branch joins
      for (int h0 = lo + sl; h0 < hi; h0 += 8 * nsl) {
        float wt[8], v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int h = min(h0 + u * nsl, hi - 1);
          int i0, i1;
          float l0, l1;
          bilin_axis_s(h, P, bsc, i0, i1, l0, l1);
          wt[u] = h0 + u * nsl < hi ? (i0 == pi ? l0 : 0.f) + (i1 == pi ? l1 : 0.f) : 0.f;
          v[u] = rows[(((size_t)b * H + h) * P + pj) * C + c];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) s += wt[u] * v[u];
      }
    }
    if (nsl > 1) {
      if (sl < nsl) red[threadIdx.x] = s;
      __syncthreads();
      s = 0.f;
      if (sl == 0)
        for (int s2 = 0; s2 < nsl; ++s2) s += red[s2 * cw + cl];
      __syncthreads();
    }
    if (sl == 0 && c < C) {
      const size_t idx = ((size_t)b * N + n) * C + c;
      gsum += o[idx] * s;
      dO[idx] = gm * s;
    }
  }
  }
  gsum = block_reduce_sum(gsum, red + NT);
  const size_t gi = (size_t)b * gridDim.x + blockIdx.x;   // = b * N + n when npw == 1
  if (!gamma_grad) {
    if (threadIdx.x == 0) gpart[gi] = gsum;
    return;
  }
  // fused dgamma: the last workgroup sums gpart in index order (per thread), then a fixed tree
  if (threadIdx.x == 0) st_sc1_dw(gpart + gi, gsum);
  if (!wg_last_of(cnt, gridDim.x * gridDim.y, &flag)) return;
  double v = 0.0;
  const int total = gridDim.x * gridDim.y;
  for (int i = threadIdx.x; i < total; i += NT) v += (double)ld_sc1_f(gpart + i);
  rd[threadIdx.x] = v;
  __syncthreads();
  for (int k = NT / 2; k > 0; k >>= 1) {
    if (threadIdx.x < k) rd[threadIdx.x] += rd[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) *gamma_grad += (float)rd[0];
}

// bf16 flash layers (dfcsa_lsa_flash_bwd_up): the upsample-backward column pass fused with the flash
// backward's prep.  ONE WAVE per token n = (pi, pj) of image b, lanes over channels (64 per step):
//   du[c] = sum_h wy(pi, h) rows[b][h][pj][c]   (the source rows with a non-zero weight, found once per
//           wave by a ballot over h = lo + lane; weights fetched by readlane),
//   dO16 = bf16(gamma du), r = sum_c dO16 * o (per 128-column share when nch > 1, as the prep kernel's),
//   gpart[b N + n] = sum_c o du (the dgamma partial).
// The fp32 dO never exists: the separate pass (dfcsa_lsa_up_bwd_cols + the prep kernel) wrote it and
// read it back with o.  hi - lo <= 64 is host-checked (H <= 29 P).
__global__ void __launch_bounds__(256) lsa_up_bwd_cols_flash_kernel(int H, int C, int P, int nch,
                                                                    const float* __restrict__ rows,
                                                                    const float* __restrict__ o, const float* gamma,
                                                                    bf16_t* __restrict__ dO16, float* __restrict__ r,
                                                                    float* __restrict__ gpart) {
  const int lane = threadIdx.x & 63, b = blockIdx.y, N = P * P;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const int pi = n / P, pj = n - pi * P;
  int lo, hi;
  contrib_range(pi, P, H, lo, hi);
  const float bsc = (float)P / (float)H;
  float wl = 0.f;
  {
    const int h = lo + lane;
    if (h < hi) {
      int i0, i1;
      float l0, l1;
      bilin_axis_s(h, P, bsc, i0, i1, l0, l1);
      wl = (i0 == pi ? l0 : 0.f) + (i1 == pi ? l1 : 0.f);
    }
  }
  const unsigned long long hm = __ballot(wl != 0.f);
  const int wli = __float_as_int(wl);
  const float gm = *gamma;
  const int PC = P * C;
  const float* rb = rows + ((size_t)b * H * P + pj) * C;   // rows[b][h][pj][c] = rb[h * PC + c]
  const size_t row = (size_t)b * N + n, rows_tot = (size_t)gridDim.y * N;
  float g = 0.f, rs = 0.f;
  for (int c0 = 0; c0 < C; c0 += 64) {
    const int c = c0 + lane;
    const int cc = c < C ? c : C - 1;
    float s = 0.f;
    unsigned long long m = hm;
    while (m) {   // 4 source rows in flight (the tail repeats the last row at weight 0)
      int hh[4];
      float wv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (m) {
          const int j = __builtin_ctzll(m);
          m &= m - 1;
          hh[u] = lo + j;
          wv[u] = __int_as_float(__builtin_amdgcn_readlane(wli, j));
        } else {
          hh[u] = hh[0];
          wv[u] = 0.f;
        }
      }
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = rb[(size_t)hh[u] * PC + cc];
#pragma unroll
      for (int u = 0; u < 4; ++u) s += wv[u] * v[u];
    }
    if (c < C) {
      const float ov = o[row * C + c];
      g += ov * s;
      const bf16_t d16 = f2bf(gm * s);
      dO16[row * C + c] = d16;
      rs += bf2f(d16) * ov;
    }
    if (nch > 1 && ((c0 + 64) % 128 == 0 || c0 + 64 >= C)) {   // end of a 128-column share
      const float t = wave_sum(rs);
      if (lane == 0) r[(size_t)(c0 / 128) * rows_tot + row] = t;
      rs = 0.f;
    }
  }
  if (nch <= 1) {
    const float t = wave_sum(rs);
    if (lane == 0) r[row] = t;
  }
  g = wave_sum(g);
  if (lane == 0) gpart[row] = g;
}

// grid (N, B): query row n -> dE[b][n][:], dq[b][n][:]
__global__ void __launch_bounds__(256) lsa_attn_bwd_rows_kernel(int N, int C, int Cq, const float* __restrict__ qkv,
                                                                const float* __restrict__ A,
                                                                const float* __restrict__ dO, float* __restrict__ dE,
                                                                float* __restrict__ dqkv) {
  extern __shared__ float sm[];  // dO row [C] | dA [N] | red [8]
  float* dor = sm;
  float* da = sm + C;
  float* red = da + N;
  const int n = blockIdx.x, b = blockIdx.y, J = 2 * Cq + C;
  const float* base = qkv + (size_t)b * N * J;
  const float* arow = A + ((size_t)b * N + n) * N;
  for (int c = threadIdx.x; c < C; c += 256) dor[c] = dO[((size_t)b * N + n) * C + c];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int m = wave; m < N; m += 4) {
    const float* v = base + (size_t)m * J + 2 * Cq;
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += dor[c] * v[c];
    s = wave_sum(s);
    if (lane == 0) da[m] = s;
  }
  __syncthreads();
  float dot = 0.f;
  for (int m = threadIdx.x; m < N; m += 256) dot += arow[m] * da[m];
  dot = block_reduce_sum(dot, red);
  for (int m = threadIdx.x; m < N; m += 256) {
    const float g = arow[m] * (da[m] - dot);
    da[m] = g;
    dE[((size_t)b * N + n) * N + m] = g;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < Cq; c += 256) {
    float s = 0.f;
    for (int m = 0; m < N; ++m) s += da[m] * base[(size_t)m * J + Cq + c];
    dqkv[((size_t)b * N + n) * J + c] = s;
  }
}

// N <= 16: the same query-row backward with the value rows staged in LDS 256 channels at a time
// (every lane's loads of a chunk in flight at once; the generic kernel above walks the keys one
// wave at a time, a dependent L2 round trip per key), the 16 dots accumulated by 16-lane groups
// and reduced with a butterfly; the key rows for dq staged the same way.
__global__ void __launch_bounds__(256) lsa_attn_bwd_rows16_kernel(int N, int C, int Cq, const float* __restrict__ qkv,
                                                                  const float* __restrict__ A,
                                                                  const float* __restrict__ dO, float* __restrict__ dE,
                                                                  float* __restrict__ dqkv) {
  constexpr int CH = 256;
  __shared__ __attribute__((aligned(16))) float vs[16][CH + 4];
  __shared__ __attribute__((aligned(16))) float ds[CH];
  __shared__ float dEs[16];
  const int n = blockIdx.x, b = blockIdx.y, J = 2 * Cq + C, t = threadIdx.x;
  const float* base = qkv + (size_t)b * N * J;
  const float* dOn = dO + ((size_t)b * N + n) * C;
  const int m = t >> 4, seg = t & 15;    // dot (n, m): lanes seg of group m
  const float a = A[((size_t)b * N + n) * N + min(m, N - 1)];   // used for m < N only
  float part = 0.f;
  for (int c0 = 0; c0 < C; c0 += CH) {
    const int cw = min(CH, C - c0);
    __syncthreads();
{   // unconditional (clamped) loads, all four in flight before the LDS stores
      float4 r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = t + 256 * k, mm = e / (CH / 4), c4 = (e % (CH / 4)) * 4;
        r[k] = *(const float4*)(base + (size_t)min(mm, N - 1) * J + 2 * Cq + c0 + min(c4, cw - 4));
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = t + 256 * k;
        *(float4*)&vs[e / (CH / 4)][(e % (CH / 4)) * 4] = r[k];
      }
    }
    if (t * 4 < cw) *(float4*)&ds[t * 4] = *(const float4*)(dOn + c0 + t * 4);
    __syncthreads();
    if (m < N)
      for (int c = seg; c < cw; c += 16) part += ds[c] * vs[m][c];
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) part += __shfl_xor(part, off, 16);
  // part (every lane of group m) = dA[n][m]; dot = sum_m A[n][m] dA[n][m] over the 16 group leaders
  float w = (seg == 0 && m < N) ? a * part : 0.f;
  w = wave_sum(w);
  __shared__ float wred[4];
  if ((t & 63) == 0) wred[t >> 6] = w;
  __syncthreads();
  const float dot = (wred[0] + wred[1]) + (wred[2] + wred[3]);
  if (seg == 0 && m < N) {
    const float g = a * (part - dot);
    dEs[m] = g;
    dE[((size_t)b * N + n) * N + m] = g;
  }
  __syncthreads();
  // dq[n][c] = sum_m dE[n][m] k[m][c] (Cq <= 256: one staged chunk of the key rows)
  for (int c0 = 0; c0 < Cq; c0 += CH) {
    const int cw = min(CH, Cq - c0);
    __syncthreads();
{   // unconditional (clamped) loads, all four in flight before the LDS stores
      float4 r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = t + 256 * k, mm = e / (CH / 4), c4 = (e % (CH / 4)) * 4;
        r[k] = *(const float4*)(base + (size_t)min(mm, N - 1) * J + Cq + c0 + min(c4, cw - 4));
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = t + 256 * k;
        *(float4*)&vs[e / (CH / 4)][(e % (CH / 4)) * 4] = r[k];
      }
    }
    __syncthreads();
    for (int c = t; c < cw; c += 256) {
      float sq = 0.f;
      for (int mm = 0; mm < N; ++mm) sq += dEs[mm] * vs[mm][c];
      dqkv[((size_t)b * N + n) * J + c0 + c] = sq;
    }
  }
}

// grid (N, B): key/value row m -> dk[b][m][:], dv[b][m][:]
// N <= 16: the same key-column backward with the n loop unrolled to 16 unconditional loads in
// flight per output (rows past N clamped, weight 0 -- the same products summed in the same order;
// the generic loop issued them four at a time)
__global__ void __launch_bounds__(256) lsa_attn_bwd_cols16_kernel(int N, int C, int Cq, const float* __restrict__ qkv,
                                                                  const float* __restrict__ A,
                                                                  const float* __restrict__ dO,
                                                                  const float* __restrict__ dE,
                                                                  float* __restrict__ dqkv) {
  __shared__ float de[16], ac[16];
  const int m = blockIdx.x, b = blockIdx.y, J = 2 * Cq + C;
  if (threadIdx.x < 16) {
    const int n = threadIdx.x, nc = min(n, N - 1);
    const float dv = dE[((size_t)b * N + nc) * N + m], av = A[((size_t)b * N + nc) * N + m];
    de[n] = n < N ? dv : 0.f;
    ac[n] = n < N ? av : 0.f;
  }
  __syncthreads();
  const float* base = qkv + (size_t)b * N * J;
  const float* dOb = dO + (size_t)b * N * C;
  float* out = dqkv + ((size_t)b * N + m) * J;
  for (int c = threadIdx.x; c < Cq; c += 256) {
    float v[16];
#pragma unroll
    for (int n = 0; n < 16; ++n) v[n] = base[(size_t)min(n, N - 1) * J + c];
    float s = 0.f;
#pragma unroll
    for (int n = 0; n < 16; ++n) s += de[n] * v[n];
    out[Cq + c] = s;
  }
  for (int c = threadIdx.x; c < C; c += 256) {
    float v[16];
#pragma unroll
    for (int n = 0; n < 16; ++n) v[n] = dOb[(size_t)min(n, N - 1) * C + c];
    float s = 0.f;
#pragma unroll
    for (int n = 0; n < 16; ++n) s += ac[n] * v[n];
    out[2 * Cq + c] = s;
  }
}

__global__ void __launch_bounds__(256) lsa_attn_bwd_cols_kernel(int N, int C, int Cq, const float* __restrict__ qkv,
                                                                const float* __restrict__ A,
                                                                const float* __restrict__ dO,
                                                                const float* __restrict__ dE, float* __restrict__ dqkv) {
  extern __shared__ float sm[];  // dE col [N] | A col [N]
  float* de = sm;
  float* ac = sm + N;
  const int m = blockIdx.x, b = blockIdx.y, J = 2 * Cq + C;
  for (int n = threadIdx.x; n < N; n += 256) {
    de[n] = dE[((size_t)b * N + n) * N + m];
    ac[n] = A[((size_t)b * N + n) * N + m];
  }
  __syncthreads();
  const float* base = qkv + (size_t)b * N * J;
  float* out = dqkv + ((size_t)b * N + m) * J;
  for (int c = threadIdx.x; c < Cq; c += 256) {
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += de[n] * base[(size_t)n * J + c];
    out[Cq + c] = s;
  }
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += ac[n] * dO[((size_t)b * N + n) * C + c];
    out[2 * Cq + c] = s;
  }
}

// dW[j][c] += sum_bn dqkv[bn][j] * pooled[bn][c]; grid (ceil(C/256), J)
__global__ void __launch_bounds__(256) lsa_proj_dw_kernel(int BN, int C, int Cq, const float* __restrict__ dqkv,
                                                          const float* __restrict__ pooled, float* dWq, float* dWk,
                                                          float* dWv) {
  const int J = 2 * Cq + C;
  const int j = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int r = 0; r < BN; ++r) s += dqkv[(size_t)r * J + j] * pooled[(size_t)r * C + c];
  if (j < Cq) dWq[(size_t)j * C + c] += s;
  else if (j < 2 * Cq) dWk[(size_t)(j - Cq) * C + c] += s;
  else dWv[(size_t)(j - 2 * Cq) * C + c] += s;
}

__global__ void __launch_bounds__(256) lsa_proj_db_kernel(int BN, int C, int Cq, const float* __restrict__ dqkv,
                                                          float* dbq, float* dbk, float* dbv) {
  const int J = 2 * Cq + C;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= J) return;
  float s = 0.f;
  for (int r = 0; r < BN; ++r) s += dqkv[(size_t)r * J + j];
  if (j < Cq) dbq[j] += s;
  else if (j < 2 * Cq) dbk[j - Cq] += s;
  else dbv[j - 2 * Cq] += s;
}

// dpooled[bn][c] = sum_j dqkv[bn][j] * w[j][c]; grid (ceil(C/256), BN)
__global__ void __launch_bounds__(256) lsa_proj_dx_kernel(int C, int Cq, const float* __restrict__ dqkv,
                                                          const float* __restrict__ w, float* __restrict__ dpooled) {
  extern __shared__ float drow[];
  const int J = 2 * Cq + C;
  const int r = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  for (int j = threadIdx.x; j < J; j += 256) drow[j] = dqkv[(size_t)r * J + j];
  __syncthreads();
  if (c >= C) return;
  float s = 0.f;
  for (int j = 0; j < J; ++j) s += drow[j] * w[(size_t)j * C + c];
  dpooled[(size_t)r * C + c] = s;
}

}  // namespace

extern "C" int dfcsa_lsa_pool_splits(int H, int P) { return pool_splits(H, P); }

extern "C" int dfcsa_lsa_pool_ws(int dtype, int B, int H, int W, int C, const void* y2, const float* sc2,
                                 const float* sh2, int P, int relu, float* partial, float* wpart, void* stream) {
  if (C % 8 || C > 2048 || P <= 0) return DFCSA_EINVAL;
  const int S = pool_splits(H, P);
  dim3 grid(S, P * P, B);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16) {
    if (wpart)
      hipLaunchKernelGGL((lsa_pool_kernel<bf16_t, true>), grid, dim3(256), 0, st, H, W, C, (const bf16_t*)y2, sc2,
                         sh2, P, S, relu, partial, wpart);
    else
      hipLaunchKernelGGL((lsa_pool_kernel<bf16_t, false>), grid, dim3(256), 0, st, H, W, C, (const bf16_t*)y2, sc2,
                         sh2, P, S, relu, partial, wpart);
  } else {
    if (wpart)
      hipLaunchKernelGGL((lsa_pool_kernel<float, true>), grid, dim3(256), 0, st, H, W, C, (const float*)y2, sc2, sh2,
                         P, S, relu, partial, wpart);
    else
      hipLaunchKernelGGL((lsa_pool_kernel<float, false>), grid, dim3(256), 0, st, H, W, C, (const float*)y2, sc2, sh2,
                         P, S, relu, partial, wpart);
  }
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_lsa_pool_direct_ok(int C, int P, int H, int W) {
  const int cpp = C / 8;
  // large pools, or P = 8 windows of at most 8 x 8 pixels (below 224^2): a wave per window has the
  // whole window in a few loads per lane; larger windows keep the row-sliced launches.  (P = 4's deep
  // levels measured 0.6 % slower on it, profiles/r06z_ab.txt: P = 4 keeps the sliced launches.)
  const bool small = P >= 16 || (P >= 8 && (H + P - 1) / P <= 8 && (W + P - 1) / P <= 8);
  return (g_lsa_pool_direct && small && P > 0 && C % 8 == 0 && C <= 2048 && cpp > 0 &&
          ((cpp & (cpp - 1)) == 0 || cpp % 64 == 0)) ? 1 : 0;
}

extern "C" int dfcsa_lsa_pool_direct(int dtype, int B, int H, int W, int C, const void* y2, const float* sc2,
                                     const float* sh2, int P, int relu, float* pooled, void* pooled16, float* wsum,
                                     void* stream) {
  if (!dfcsa_lsa_pool_direct_ok(C, P, H, W) || B <= 0 || H <= 0 || W <= 0 || !y2 || !sc2 || !sh2 || (!pooled && !pooled16) ||
      ((uintptr_t)pooled & 15) || ((uintptr_t)pooled16 & 15) || ((uintptr_t)wsum & 15))
    return DFCSA_EINVAL;
  if (pooled16 && dtype != DFCSA_DT_BF16 && dtype != DFCSA_DT_F32) return DFCSA_EINVAL;
  dim3 grid((P * P + 3) / 4, B);
  hipStream_t st = (hipStream_t)stream;
  bf16_t* p16 = (bf16_t*)pooled16;
#define DFCSA_POOL_DIRECT(TT, WSV)                                                                              \
  hipLaunchKernelGGL((lsa_pool_direct_kernel<TT, WSV>), grid, dim3(256), 0, st, H, W, C, P, (const TT*)y2, sc2, \
                     sh2, relu, pooled, p16, wsum)
  if (dtype == DFCSA_DT_BF16) {
    if (wsum) DFCSA_POOL_DIRECT(bf16_t, true);
    else DFCSA_POOL_DIRECT(bf16_t, false);
  } else {
    if (wsum) DFCSA_POOL_DIRECT(float, true);
    else DFCSA_POOL_DIRECT(float, false);
  }
#undef DFCSA_POOL_DIRECT
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_lsa_pool(int dtype, int B, int H, int W, int C, const void* y2, const float* sc2,
                              const float* sh2, int P, int relu, float* partial, void* stream) {
  return dfcsa_lsa_pool_ws(dtype, B, H, W, C, y2, sc2, sh2, P, relu, partial, nullptr, stream);
}

extern "C" int dfcsa_lsa_pooled_ws(int B, int H, int W, int C, int P, const float* partial, float* pooled,
                                   const float* wpart, float* wsum, void* stream) {
  if ((wpart == nullptr) != (wsum == nullptr)) return DFCSA_EINVAL;
  hipLaunchKernelGGL(lsa_pooled_kernel, dim3(P * P, B), dim3(256), 0, (hipStream_t)stream, H, W, C, P,
                     pool_splits(H, P), partial, pooled, wpart, wsum);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_lsa_pooled(int B, int H, int W, int C, int P, const float* partial, float* pooled,
                                void* stream) {
  return dfcsa_lsa_pooled_ws(B, H, W, C, P, partial, pooled, nullptr, nullptr, stream);
}

extern "C" int dfcsa_lsa_qkv(int B, int H, int W, int C, int Cq, int P, const float* partial, const float* wT,
                             const float* bias, float* pooled, float* qkv, void* stream) {
  const int N = P * P, J = 2 * Cq + C;
  size_t shm = (size_t)16 * C * sizeof(float);
  if (shm > 64 * 1024) return DFCSA_EINVAL;
  dim3 grid((J + 255) / 256, (N + 15) / 16, B);
  hipLaunchKernelGGL(lsa_qkv_kernel, grid, dim3(256), shm, (hipStream_t)stream, H, W, C, Cq, P, pool_splits(H, P),
                     partial, wT, bias, pooled, qkv);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_lsa_attn(int B, int N, int C, int Cq, const float* qkv, float* A, float* o, void* stream) {
  size_t shm = (size_t)(Cq + N + 8) * sizeof(float);
  hipLaunchKernelGGL(lsa_attn_kernel, dim3(N, B), dim3(256), shm, (hipStream_t)stream, N, C, Cq, qkv, A, o);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_lsa_up_bwd_rows(int dtype, int B, int H, int W, int C, const void* dattn, int P, float* rows,
                                     void* stream) {
  if (C % 8) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  // the column-owner kernel: P <= 4 and nslot * P * C <= 4 * 4 * 512 LDS floats
  const int cpp = C / 8, nsl = cpp <= 256 ? 256 / cpp : 0;
  const bool bfly = cpp < 64 && (cpp & (cpp - 1)) == 0;
  if (P <= 4 && nsl > 0 && (size_t)(bfly ? 4 : nsl) * P * C <= 4 * 4 * 512 && !g_lsa_rows_old) {
    if (dtype == DFCSA_DT_BF16)
      hipLaunchKernelGGL((lsa_up_bwd_rows_pix_kernel<bf16_t, 4>), dim3(H, B), dim3(256), 0, st, H, W, C,
                         (const bf16_t*)dattn, P, rows);
    else
      hipLaunchKernelGGL((lsa_up_bwd_rows_pix_kernel<float, 4>), dim3(H, B), dim3(256), 0, st, H, W, C,
                         (const float*)dattn, P, rows);
  } else if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(lsa_up_bwd_rows_kernel<bf16_t>, dim3(H, B), dim3(256), 0, st, H, W, C, (const bf16_t*)dattn,
                       P, rows);
  else
    hipLaunchKernelGGL(lsa_up_bwd_rows_kernel<float>, dim3(H, B), dim3(256), 0, st, H, W, C, (const float*)dattn, P,
                       rows);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// Fused pooled-attention backward, token-parallel: grid (N, B), one workgroup per (token, image)
// as lsa_up_bwd_cols, so the column pass keeps its 256-workgroup memory parallelism.  Each
// workgroup forms dO[n] (column pass of the upsample backward, kept in LDS and published with
// write-through stores), runs query row n of the softmax backward (dA[n][m] = dO[n] . v[m],
// dE[n][m] = A (dA - rowsum(A dA)), dq[n] = dE[n] k) and publishes dE[n]; the LAST workgroup of the
// image (ticket) forms dk = dE^T q and dv = A^T dO for the image's tokens from the published rows;
// the last of all adds dgamma (partials in token order).  Replaces lsa_up_bwd_cols +
// lsa_attn_bwd_rows + lsa_attn_bwd_cols (three dependent launches on the backward's critical path).
__global__ void __launch_bounds__(256) lsa_core_bwd_kernel(int H, int C, int Cq, int P, const float* __restrict__ rows,
                                                           const float* __restrict__ o, const float* gamma,
                                                           const float* __restrict__ qkv, const float* __restrict__ A,
                                                           float* __restrict__ dqkv, float* dOg, float* dEg,
                                                           float* gpart, unsigned* cnt, float* gamma_grad) {
  __shared__ float red[256 + 8];
  __shared__ double rd[256];
  __shared__ float dor[1024];
  __shared__ float da[16];
  __shared__ float dEs[16][17];
  __shared__ int flag;
  const int n = blockIdx.x, b = blockIdx.y, N = P * P, J = 2 * Cq + C, t = threadIdx.x;
  const int pi = n / P, pj = n - pi * P;
  const float gm = *gamma;
  const float bsc = (float)P / (float)H;
  const float* qb = qkv + (size_t)b * N * J;
  // ---- column pass of the upsample backward for token n (lsa_up_bwd_cols' slicing) ----
  const int nsl = C >= 256 ? 1 : 256 / C;
  const int cw = nsl == 1 ? 256 : C;
  const int sl = t / cw, cl = t - sl * cw;
  int lo, hi;
  contrib_range(pi, P, H, lo, hi);
  float gsum = 0.f;
  for (int cb = 0; cb < C; cb += cw) {
    const int c = cb + cl;
    float sacc = 0.f;
    if (c < C && sl < nsl) {
      for (int h0 = lo + sl; h0 < hi; h0 += 4 * nsl) {
        float wt[4], v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int h = h0 + u * nsl;
          wt[u] = 0.f;
          if (h < hi) {
            int i0, i1;
            float l0, l1;
            bilin_axis_s(h, P, bsc, i0, i1, l0, l1);
            wt[u] = (i0 == pi ? l0 : 0.f) + (i1 == pi ? l1 : 0.f);
          }
          v[u] = wt[u] != 0.f ? rows[(((size_t)b * H + h) * P + pj) * C + c] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (wt[u] != 0.f) sacc += wt[u] * v[u];
      }
    }
    if (nsl > 1) {
      if (sl < nsl) red[t] = sacc;
      __syncthreads();
      sacc = 0.f;
      if (sl == 0)
        for (int s2 = 0; s2 < nsl; ++s2) sacc += red[s2 * cw + cl];
      __syncthreads();
    }
    if (sl == 0 && c < C) {
      gsum += o[((size_t)b * N + n) * C + c] * sacc;
      dor[c] = gm * sacc;
    }
  }
  __syncthreads();
  // publish dO[n] (write-through: read back by the image's last workgroup)
  float* dOn = dOg + ((size_t)b * N + n) * C;
  for (int c4 = t * 4; c4 < C; c4 += 1024) st_sc1_f4(dOn + c4, dor[c4], dor[c4 + 1], dor[c4 + 2], dor[c4 + 3]);
  // ---- query row n: dA[m] = dO[n] . v[m] (wave per key, lanes over channels) ----
  const int wave = t >> 6, lane = t & 63;
  for (int m = wave; m < N; m += 4) {
    const float* v = qb + (size_t)m * J + 2 * Cq;
    float sv = 0.f;
    for (int c = lane; c < C; c += 64) sv += dor[c] * v[c];
    sv = wave_sum(sv);
    if (lane == 0) da[m] = sv;
  }
  __syncthreads();
  const float* An = A + ((size_t)b * N + n) * N;
  if (t < 64) {
    float w = t < N ? An[t] * da[t] : 0.f;
    w = wave_sum(w);
    if (t < N) {
      const float g = An[t] * (da[t] - w);
      dEs[0][t] = g;
      st_sc1_dw(dEg + ((size_t)b * N + n) * N + t, g);
    }
  }
  __syncthreads();
  for (int c = t; c < Cq; c += 256) {
    float sq = 0.f;
    for (int m = 0; m < N; ++m) sq += dEs[0][m] * qb[(size_t)m * J + Cq + c];
    dqkv[((size_t)b * N + n) * J + c] = sq;
  }
  gsum = block_reduce_sum(gsum, red);
  if (t == 0) st_sc1_dw(gpart + (size_t)b * N + n, gsum);
  // ---- the image's last workgroup: dk = dE^T q, dv = A^T dO over its N tokens ----
  if (wg_last_of(cnt + 1 + b, N, &flag)) {
    if (t < N * N) dEs[t / N][t % N] = ld_sc1_f(dEg + (size_t)b * N * N + t);
    __syncthreads();
    for (int e = t; e < N * Cq; e += 256) {
      const int m = e / Cq, c = e - m * Cq;
      float sk = 0.f;
      for (int nn = 0; nn < N; ++nn) sk += dEs[nn][m] * qb[(size_t)nn * J + c];
      dqkv[((size_t)b * N + m) * J + Cq + c] = sk;
    }
    const float* Ab = A + (size_t)b * N * N;
    for (int c4 = t * 4; c4 < C; c4 += 1024) {
      float4 dv[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) dv[m] = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int nn = 0; nn < N; ++nn) {
        const float4 d = ld_sc1_f4(dOg + ((size_t)b * N + nn) * C + c4);
#pragma unroll
        for (int m = 0; m < 16; ++m)
          if (m < N) {
            const float a = Ab[nn * N + m];
            dv[m].x += a * d.x; dv[m].y += a * d.y; dv[m].z += a * d.z; dv[m].w += a * d.w;
          }
      }
#pragma unroll
      for (int m = 0; m < 16; ++m)
        if (m < N) *(float4*)(dqkv + ((size_t)b * N + m) * J + 2 * Cq + c4) = dv[m];
    }
  }
  if (!gamma_grad) return;
  // ---- dgamma: the last workgroup of all sums the token partials in order ----
  if (!wg_last_of(cnt, gridDim.x * gridDim.y, &flag)) return;
  double v = 0.0;
  const int total = gridDim.x * gridDim.y;
  for (int i = t; i < total; i += 256) v += (double)ld_sc1_f(gpart + i);
  rd[t] = v;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (t < k) rd[t] += rd[t + k];
    __syncthreads();
  }
  if (t == 0) *gamma_grad += (float)rd[0];
}

extern "C" int dfcsa_lsa_core_bwd(int B, int H, int C, int Cq, int P, const float* rows, const float* o,
                                  const float* gamma, const float* qkv, const float* A, float* dqkv, float* dO,
                                  float* dE, float* gpart, float* gamma_grad, void* stream) {
  if (B <= 0 || H <= 0 || P < 1 || P > 4 || C % 8 || C > 1024 || Cq <= 0 || Cq % 2 || !gpart || !dO || !dE)
    return DFCSA_EINVAL;
  unsigned* cnt = dfcsa_ticket_alloc(1 + B);
  if (!cnt) return DFCSA_EINVAL;
  hipLaunchKernelGGL(lsa_core_bwd_kernel, dim3(P * P, B), dim3(256), 0, (hipStream_t)stream, H, C, Cq, P, rows, o,
                     gamma, qkv, A, dqkv, dO, dE, gpart, cnt, gamma_grad);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_lsa_up_bwd_cols(int B, int H, int C, int P, const float* rows, const float* o,
                                     const float* gamma, float* dO, float* gpart, int* ngpart, float* gamma_grad,
                                     void* stream) {
  unsigned* cnt = nullptr;
  if (gamma_grad && !(cnt = dfcsa_ticket_alloc(1))) return DFCSA_EINVAL;
  // fused dgamma: at most ~64 workgroups per image (one ticket atomic each)
  const int N = P * P, npw = gamma_grad ? (N + 63) / 64 : 1, gx = (N + npw - 1) / npw;
  if (C <= 128 && g_lsa_cols_nt > 256)
    hipLaunchKernelGGL(lsa_up_bwd_cols_kernel<1024>, dim3(gx, B), dim3(1024), 0, (hipStream_t)stream, H, C, P, npw, rows,
                       o, gamma, dO, gpart, cnt, gamma_grad);
  else
    hipLaunchKernelGGL(lsa_up_bwd_cols_kernel<256>, dim3(gx, B), dim3(256), 0, (hipStream_t)stream, H, C, P, npw, rows,
                       o, gamma, dO, gpart, cnt, gamma_grad);
  DFCSA_CHECK_LAUNCH();
  if (ngpart) *ngpart = B * P * P;
  return 0;
}

extern "C" int dfcsa_lsa_flash_bwd_up(int B, int H, int C, int Cq, int P, const float* rows, const float* o,
                                      const float* gamma, const void* qkv16, const float* lse, void* dqkv16,
                                      float* gpart, void* work, int64_t work_bytes, void* stream) {
  const int N = P * P, ldq = 2 * Cq + C;
  if (!g_lsa_cols_flash || B <= 0 || H <= 0 || P <= 0 || H > 29 * P || !rows || !o || !gamma || !qkv16 || !lse ||
      !dqkv16 || !gpart)
    return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  bf16_t* dO16 = nullptr;
  float* r = nullptr;
  int nch = 1;
  const float* kb = nullptr;
  if (lsa_flash_prepare_ext(B, N, C, Cq, ldq, qkv16, work, work_bytes, &dO16, &r, &nch, &kb, st)) return DFCSA_EINVAL;
  hipLaunchKernelGGL(lsa_up_bwd_cols_flash_kernel, dim3((N + 3) / 4, B), dim3(256), 0, st, H, C, P, nch, rows, o,
                     gamma, dO16, r, gpart);
  DFCSA_CHECK_LAUNCH();
  lsa_flash_bwd_core(B, N, C, Cq, ldq, qkv16, lse, dqkv16, work, kb, st);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_lsa_attn_bwd(int B, int N, int C, int Cq, const float* qkv, const float* A, const float* dO,
                                  float* dE, float* dqkv, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  size_t shm1 = (size_t)(C + N + 8) * sizeof(float);
  if (N <= 16 && C % 4 == 0 && Cq % 4 == 0)
    hipLaunchKernelGGL(lsa_attn_bwd_rows16_kernel, dim3(N, B), dim3(256), 0, st, N, C, Cq, qkv, A, dO, dE, dqkv);
  else
    hipLaunchKernelGGL(lsa_attn_bwd_rows_kernel, dim3(N, B), dim3(256), shm1, st, N, C, Cq, qkv, A, dO, dE, dqkv);
  DFCSA_CHECK_LAUNCH();
  size_t shm2 = (size_t)(2 * N) * sizeof(float);
  if (N <= 16)
    hipLaunchKernelGGL(lsa_attn_bwd_cols16_kernel, dim3(N, B), dim3(256), 0, st, N, C, Cq, qkv, A, dO, dE, dqkv);
  else
    hipLaunchKernelGGL(lsa_attn_bwd_cols_kernel, dim3(N, B), dim3(256), shm2, st, N, C, Cq, qkv, A, dO, dE, dqkv);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_lsa_proj_bwd(int B, int N, int C, int Cq, const float* dqkv, const float* pooled,
                                  const float* w, float* dWq, float* dWk, float* dWv, float* dbq, float* dbk,
                                  float* dbv, float* dpooled, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int J = 2 * Cq + C, BN = B * N;
  hipLaunchKernelGGL(lsa_proj_dw_kernel, dim3((C + 255) / 256, J), dim3(256), 0, st, BN, C, Cq, dqkv, pooled, dWq,
                     dWk, dWv);
  DFCSA_CHECK_LAUNCH();
  hipLaunchKernelGGL(lsa_proj_db_kernel, dim3((J + 255) / 256), dim3(256), 0, st, BN, C, Cq, dqkv, dbq, dbk, dbv);
  DFCSA_CHECK_LAUNCH();
  hipLaunchKernelGGL(lsa_proj_dx_kernel, dim3((C + 255) / 256, BN), dim3(256), (size_t)J * sizeof(float), st, C, Cq,
                     dqkv, w, dpooled);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// The attention entry's pool-backward BatchNorm sums as partial rows (the pool term of
// dfcsa_bwd_attn_entry's statistics, as dfcsa_conv_wgrad_dgrad1x1_pool's epilogue forms them for the
// fp32 projections): for the 16 tokens m of row block bx and channel c,
//   rows[bx][0][c] = sum_m dpooled[m][c] / area(m) * wsum[m][0][c]
//   rows[bx][1][c] = sum_m dpooled[m][c] / area(m) * invstd[c] * (wsum[m][1][c] - mean[c] * wsum[m][0][c])
// grid (ceil(BN / 16), ceil(C / 64)), 256 threads: 4 token phases x 64 channels, fixed-order combine.
namespace {
template <typename T>
__global__ void __launch_bounds__(256) lsa_pool_rows_kernel(int BN, int C, int P, int H, int W,
                                                            const T* __restrict__ dpooled,
                                                            const float* __restrict__ wsum,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd,
                                                            float* __restrict__ rows) {
  __shared__ float red[2][4][64];
  const int bx = blockIdx.x, cl = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl, NP = P * P;
  float s0 = 0.f, s1 = 0.f;
  if (c < C) {
    const float mu = mean[c], is = invstd[c];
    for (int k = 0; k < 4; ++k) {
      const int m = bx * 16 + ph + 4 * k;
      if (m >= BN) break;
      const int n = m % NP, pi = n / P, pj = n - pi * P;
      const float area = (float)(((pi + 1) * H + P - 1) / P - (pi * H) / P) *
                         (float)(((pj + 1) * W + P - 1) / P - (pj * W) / P);
      const float dd = ElemTraits<T>::to_f(dpooled[(size_t)m * C + c]) / area;
      const float R = wsum[((size_t)m * 2) * C + c], Y = wsum[((size_t)m * 2 + 1) * C + c];
      s0 += dd * R;
      s1 += dd * is * (Y - mu * R);
    }
  }
  red[0][ph][cl] = s0;
  red[1][ph][cl] = s1;
  __syncthreads();
  if (ph < 2 && c < C) {
    const float v = (red[ph][0][cl] + red[ph][1][cl]) + (red[ph][2][cl] + red[ph][3][cl]);
    rows[((size_t)bx * 2 + ph) * C + c] = v;
  }
}
}  // namespace

extern "C" int dfcsa_lsa_pool_rows(int dtype, int BN, int C, int P, int H, int W, const void* dpooled,
                                   const float* wsum, const float* mean, const float* invstd, float* rows,
                                   int64_t rows_floats, void* stream) {
  if (BN <= 0 || C <= 0 || P <= 0 || H <= 0 || W <= 0 || BN % (P * P) || !dpooled || !wsum || !mean || !invstd ||
      !rows)
    return DFCSA_EINVAL;
  const int nb = (BN + 15) / 16;
  if (rows_floats < (int64_t)nb * 2 * C) return DFCSA_EINVAL;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(lsa_pool_rows_kernel<bf16_t>, dim3(nb, (C + 63) / 64), dim3(256), 0, (hipStream_t)stream, BN, C,
                       P, H, W, (const bf16_t*)dpooled, wsum, mean, invstd, rows);
  else
    hipLaunchKernelGGL(lsa_pool_rows_kernel<float>, dim3(nb, (C + 63) / 64), dim3(256), 0, (hipStream_t)stream, BN, C,
                       P, H, W, (const float*)dpooled, wsum, mean, invstd, rows);
  DFCSA_CHECK_LAUNCH();
  return 0;
}
