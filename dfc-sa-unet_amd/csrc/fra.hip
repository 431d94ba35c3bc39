// Full-resolution self-attention (reference models/unet_dfc_sa_ablation_attention.py:7-26,
// FullResolutionAttention, used by FullResAttnDFCBlock :29-92 / UNet_FullResAttention :95-97 and
// config_ablation3_full_res_attn.yaml) forward and backward, flash-style.
//
// Per image (N = H*W tokens; the q/k/v projections are done by the implicit GEMM beforehand):
//   q = a Wq^T + bq, k = a Wk^T + bk   (Cq = C/8 channels),   v = a Wv^T + bv   (C channels)
//   A = softmax_rows(q k^T)            (no 1/sqrt(d) scale, :19-21)
//   O = A v                            (:22-24, out[c][n] = sum_m v[c][m] A[n][m])
//   out = gamma * O + a                (:25)
// qkv is one NHWC tensor [B][N][ldq] with q at columns [0,Cq), k at [Cq,2Cq), v at [2Cq,2Cq+C).
//
// The N x N score matrix is never materialised (N^2 * 4 B = 275 GB per image at 512^2): the
// forward keeps a running max and sum per query (online softmax) and stores the log-sum-exp;
// the backward recomputes P from it twice (a key-major pass that owns dK/dV and a query-major
// pass that owns dQ), so no N^2-sized tensor and no float atomics touch HBM.  With d_qk = C/8 = 8
// at the 512^2 levels the work is exp/VALU-bound, not MFMA-bound.
//
// Two implementations of the same semantics:
//  * MFMA (bf16): 16x16x32 / 16x16x16 bf16 MFMAs.  Scores are computed with the contraction
//    partner's index on the lanes and the softmax row index... arranged so that a score tile's
//    accumulator registers ARE the B operand of the next MFMA (P*V, dS*K, ...) after a bf16 pack,
//    with no lane movement; the matching A operand (V^T, K^T, Q^T, dO^T) comes from the
//    row-major LDS tile through the gfx950 transposing read ds_read_b64_tr_b16.  exp2 with
//    log2(e) folded into one FMA; the output accumulators are rescaled lazily (only when a row
//    max grows by more than 2^8).
//  * generic (fp32 or bf16 storage, any C/Cq): one wave per row, fp32 VALU, exact online
//    softmax; the fp32 parity path and the path for narrow or unaligned shapes.
#include <algorithm>

#include "common.h"
#include "dfcsa_internal.h"

int g_fra_generic = 0;  // tuning knob 9: force the generic kernels (coverage tests)
int g_fra_occ = 15;     // tuning knob 10: waves-per-SIMD budgets of the narrow MFMA kernels

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4;

constexpr float kL2E = 1.4426950408889634f;
constexpr float kRescale = 8.0f;  // lazy-rescale threshold (log2 units)

// ============================================================================ generic kernels
// one wave per query row; grid (ceil(N/4), B); dynamic LDS: 4 x Cq floats
template <typename T>
__global__ void __launch_bounds__(256) fra_fwd_generic(int N, int C, int Cq, int ldq, const T* __restrict__ qkv,
                                                       const T* __restrict__ x, const float* __restrict__ gamma,
                                                       T* __restrict__ o, T* __restrict__ y, float* __restrict__ lse) {
  using E = ElemTraits<T>;
  extern __shared__ float sm[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, b = blockIdx.y;
  const int n = blockIdx.x * 4 + w;
  float* qs = sm + w * Cq;
  const T* base = qkv + (size_t)b * N * ldq;
  if (n < N)
    for (int d = lane; d < Cq; d += 64) qs[d] = E::to_f(base[(size_t)n * ldq + d]);
  __syncthreads();
  if (n >= N) return;
  constexpr int MAXR = 16;  // C <= 1024
  float acc[MAXR];
#pragma unroll
  for (int i = 0; i < MAXR; ++i) acc[i] = 0.f;
  float m = -INFINITY, l = 0.f;
  for (int kb = 0; kb < N; kb += 64) {
    const int key = kb + lane;
    float s = -INFINITY;
    if (key < N) {
      const T* kr = base + (size_t)key * ldq + Cq;
      float t = 0.f;
      for (int d = 0; d < Cq; ++d) t += qs[d] * E::to_f(kr[d]);
      s = t;
    }
    const float mn = fmaxf(m, wave_max(s));
    const float alpha = (m == -INFINITY) ? 0.f : __expf(m - mn);
    const float p = (key < N) ? __expf(s - mn) : 0.f;
    l = l * alpha + wave_sum(p);
    m = mn;
#pragma unroll
    for (int i = 0; i < MAXR; ++i) acc[i] *= alpha;
    const int nk = min(64, N - kb);
    for (int j = 0; j < nk; ++j) {
      const float pj = __shfl(p, j, 64);
      const T* vr = base + (size_t)(kb + j) * ldq + 2 * Cq;
#pragma unroll
      for (int i = 0; i < MAXR; ++i) {
        const int c = lane + 64 * i;
        if (c < C) acc[i] += pj * E::to_f(vr[c]);
      }
    }
  }
  const float inv = 1.f / l, gm = y ? *gamma : 0.f;
  const size_t row = (size_t)b * N + n;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int c = lane + 64 * i;
    if (c < C) {
      const float ov = acc[i] * inv;
      o[row * C + c] = E::from_f(ov);
      if (y) y[row * C + c] = E::from_f(gm * ov + E::to_f(x[row * C + c]));
    }
  }
  if (lane == 0) lse[row] = m + __logf(l);
}

// r[row] = sum_c dy[row][c] * o[row][c]   (delta = gamma * r; dgamma = sum r); wave per row
template <typename T>
__global__ void __launch_bounds__(256) fra_bwd_prep_kernel(int rows, int C, const T* __restrict__ dy,
                                                           const T* __restrict__ o, float* __restrict__ r) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float s = 0.f;
  if ((C & 7) == 0) {
    for (int c = lane * 8; c < C; c += 512) {
      float a[8], v[8];
      load8<T>(dy + (size_t)row * C + c, a);
      load8<T>(o + (size_t)row * C + c, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) s += a[k] * v[k];
    }
  } else {
    for (int c = lane; c < C; c += 64)
      s += ElemTraits<T>::to_f(dy[(size_t)row * C + c]) * ElemTraits<T>::to_f(o[(size_t)row * C + c]);
  }
  s = wave_sum(s);
  if (lane == 0) r[row] = s;
}

// dQ (query-major): wave per query; LDS per wave: q [Cq] | dy [C]; grid (ceil(N/4), B).
// Also zeroes the GEMM padding columns [2Cq + C, ldq) of its dqkv row.
template <typename T>
__global__ void __launch_bounds__(256) fra_bwd_dq_generic(int N, int C, int Cq, int ldq, const T* __restrict__ qkv,
                                                          const T* __restrict__ dy, const float* __restrict__ gamma,
                                                          const float* __restrict__ lse, const float* __restrict__ rr,
                                                          T* __restrict__ dqkv) {
  using E = ElemTraits<T>;
  extern __shared__ float sm[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, b = blockIdx.y;
  const int n = blockIdx.x * 4 + w;
  float* qs = sm + w * (Cq + C);
  float* dys = qs + Cq;
  const T* base = qkv + (size_t)b * N * ldq;
  const size_t row = (size_t)b * N + n;
  if (n < N) {
    for (int d = lane; d < Cq; d += 64) qs[d] = E::to_f(base[(size_t)n * ldq + d]);
    for (int c = lane; c < C; c += 64) dys[c] = E::to_f(dy[row * C + c]);
  }
  __syncthreads();
  if (n >= N) return;
  const float gm = *gamma, L = lse[row], R = rr[row];
  float dq0 = 0.f, dq1 = 0.f;  // d = lane, lane + 64 (Cq <= 128)
  for (int kb = 0; kb < N; kb += 64) {
    const int key = kb + lane;
    float dsv = 0.f;
    if (key < N) {
      const T* kr = base + (size_t)key * ldq;
      float s = 0.f, dp = 0.f;
      for (int d = 0; d < Cq; ++d) s += qs[d] * E::to_f(kr[Cq + d]);
      for (int c = 0; c < C; ++c) dp += dys[c] * E::to_f(kr[2 * Cq + c]);
      dsv = gm * __expf(s - L) * (dp - R);
    }
    const int nk = min(64, N - kb);
    for (int j = 0; j < nk; ++j) {
      const float sj = __shfl(dsv, j, 64);
      const T* kr = base + (size_t)(kb + j) * ldq + Cq;
      if (lane < Cq) dq0 += sj * E::to_f(kr[lane]);
      if (lane + 64 < Cq) dq1 += sj * E::to_f(kr[lane + 64]);
    }
  }
  T* out = dqkv + row * ldq;
  if (lane < Cq) out[lane] = E::from_f(dq0);
  if (lane + 64 < Cq) out[lane + 64] = E::from_f(dq1);
  for (int j = 2 * Cq + C + lane; j < ldq; j += 64) out[j] = E::from_f(0.f);
}

// dK, dV (key-major): wave per key; LDS per wave: k [Cq] | v [C]; grid (ceil(N/4), B)
template <typename T>
__global__ void __launch_bounds__(256) fra_bwd_dkv_generic(int N, int C, int Cq, int ldq, const T* __restrict__ qkv,
                                                           const T* __restrict__ dy, const float* __restrict__ gamma,
                                                           const float* __restrict__ lse, const float* __restrict__ rr,
                                                           T* __restrict__ dqkv) {
  using E = ElemTraits<T>;
  extern __shared__ float sm[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, b = blockIdx.y;
  const int m = blockIdx.x * 4 + w;
  float* ks = sm + w * (Cq + C);
  float* vs = ks + Cq;
  const T* base = qkv + (size_t)b * N * ldq;
  if (m < N) {
    for (int d = lane; d < Cq; d += 64) ks[d] = E::to_f(base[(size_t)m * ldq + Cq + d]);
    for (int c = lane; c < C; c += 64) vs[c] = E::to_f(base[(size_t)m * ldq + 2 * Cq + c]);
  }
  __syncthreads();
  if (m >= N) return;
  const float gm = *gamma;
  constexpr int MAXR = 16;
  float dv[MAXR];
#pragma unroll
  for (int i = 0; i < MAXR; ++i) dv[i] = 0.f;
  float dk0 = 0.f, dk1 = 0.f;
  const T* dyb = dy + (size_t)b * N * C;
  for (int qb = 0; qb < N; qb += 64) {
    const int n = qb + lane;
    float pv = 0.f, dsv = 0.f;
    if (n < N) {
      const T* qr = base + (size_t)n * ldq;
      const T* dr = dyb + (size_t)n * C;
      float s = 0.f, dp = 0.f;
      for (int d = 0; d < Cq; ++d) s += ks[d] * E::to_f(qr[d]);
      for (int c = 0; c < C; ++c) dp += vs[c] * E::to_f(dr[c]);
      const size_t nr = (size_t)b * N + n;
      const float p = __expf(s - lse[nr]);
      pv = gm * p;
      dsv = pv * (dp - rr[nr]);
    }
    const int nn = min(64, N - qb);
    for (int j = 0; j < nn; ++j) {
      const float pj = __shfl(pv, j, 64), sj = __shfl(dsv, j, 64);
      const T* dr = dyb + (size_t)(qb + j) * C;
      const T* qr = base + (size_t)(qb + j) * ldq;
#pragma unroll
      for (int i = 0; i < MAXR; ++i) {
        const int c = lane + 64 * i;
        if (c < C) dv[i] += pj * E::to_f(dr[c]);
      }
      if (lane < Cq) dk0 += sj * E::to_f(qr[lane]);
      if (lane + 64 < Cq) dk1 += sj * E::to_f(qr[lane + 64]);
    }
  }
  T* out = dqkv + ((size_t)b * N + m) * ldq;
  if (lane < Cq) out[Cq + lane] = E::from_f(dk0);
  if (lane + 64 < Cq) out[Cq + lane + 64] = E::from_f(dk1);
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int c = lane + 64 * i;
    if (c < C) out[2 * Cq + c] = E::from_f(dv[i]);
  }
}

// ============================================================================ MFMA kernels (bf16)
// LDS tile images are row-major [row][W] bf16.  32-byte blocks are XOR-swizzled by row so that
// the transposing reads (per 32-lane half: 8 rows x 32 B) hit 8 distinct 32-B bank slots.
template <int W>
__device__ __forceinline__ int swz(int row) {  // in 16-B chunk units (always even)
  if constexpr (W <= 16) return 0;
  else if constexpr (W == 32) return ((row >> 2) & 1) << 1;
  else if constexpr (W == 64) return ((row >> 1) & 3) << 1;
  else return (row & 7) << 1;
}
template <int W>
__device__ __forceinline__ int lds_off(int row, int col) {  // byte offset of element (row, col)
  return row * (W * 2) + (((col >> 3) ^ swz<W>(row)) << 4) + (col & 7) * 2;
}
template <int W>
__device__ __forceinline__ bf16x8_t lds_row8(const char* img, int row, int col) {
  return *(const bf16x8_t*)(img + lds_off<W>(row, col));
}
template <int W>
__device__ __forceinline__ bf16x4_t lds_row4(const char* img, int row, int col) {
  return *(const bf16x4_t*)(img + lds_off<W>(row, col));
}

// Transposed fragment: lane (g = lane>>4, i = lane&15) receives column cb*16 + i of rows
// r0 + 4g + t (element t) and r0 + 16 + 4g + t (element 4 + t), t = 0..3 -- the contraction
// order in which two stacked 16-row accumulator tiles hold their rows (row 4g + reg).
template <int W>
__device__ __forceinline__ bf16x8_t lds_tr8(const char* img, int r0, int cb, int lane) {
  const int g = lane >> 4, i = lane & 15, q4 = i >> 2, p4 = i & 3;
  const int ra = r0 + 4 * g + q4, rb = ra + 16, col = cb * 16 + 4 * p4;
  bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + lds_off<W>(ra, col)));
  bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(img + lds_off<W>(rb, col)));
  bf16x8_t f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

__device__ __forceinline__ short bfbits(float v) { return (short)f2bf(v); }

// two stacked 16x16 accumulator tiles (rows 16t + 4g + r) -> a B fragment over 32 contraction rows
__device__ __forceinline__ bf16x8_t pack_b(const f32x4_t& a, const f32x4_t& b) {
  bf16x8_t f;
  f[0] = bfbits(a[0]); f[1] = bfbits(a[1]); f[2] = bfbits(a[2]); f[3] = bfbits(a[3]);
  f[4] = bfbits(b[0]); f[5] = bfbits(b[1]); f[6] = bfbits(b[2]); f[7] = bfbits(b[3]);
  return f;
}

__device__ __forceinline__ f32x4_t mfma32(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4_t mfma16(const bf16x4_t& a, const bf16x4_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4_t zero4() { return f32x4_t{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ float exp2_(float x) { return __builtin_amdgcn_exp2f(x); }

// Score-operand fragments over the qk width CQ:
//   CQ >= 32: CQ/32 steps of 16x16x32 (lane holds elements 32s + 8g + j);
//   CQ <= 16: one 16x16x16 step (lane holds elements 4g + j; zero past CQ).
template <int CQ>
struct QKFrag {
  static constexpr bool kWide = CQ >= 32;
  static constexpr int kSteps = kWide ? CQ / 32 : 1;
  bf16x8_t w[kSteps];
  bf16x4_t n;
};

template <int CQ>
__device__ __forceinline__ void qk_load_global(QKFrag<CQ>& f, const bf16_t* row, bool ok, int g) {
  if constexpr (QKFrag<CQ>::kWide) {
#pragma unroll
    for (int s = 0; s < QKFrag<CQ>::kSteps; ++s)
      f.w[s] = ok ? *(const bf16x8_t*)(row + 32 * s + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  } else {
    f.n = (ok && 4 * g < CQ) ? *(const bf16x4_t*)(row + 4 * g) : bf16x4_t{0, 0, 0, 0};
  }
}

template <int CQ, int KC>
__device__ __forceinline__ void qk_load_lds(QKFrag<CQ>& f, const char* img, int row, int g) {
  if constexpr (QKFrag<CQ>::kWide) {
#pragma unroll
    for (int s = 0; s < QKFrag<CQ>::kSteps; ++s) f.w[s] = lds_row8<KC>(img, row, 32 * s + 8 * g);
  } else {
    f.n = lds_row4<KC>(img, row, 4 * g);  // image columns >= CQ are zero
  }
}

template <int CQ>
__device__ __forceinline__ f32x4_t qk_mfma(const QKFrag<CQ>& a, const QKFrag<CQ>& b, f32x4_t acc) {
  if constexpr (QKFrag<CQ>::kWide) {
#pragma unroll
    for (int s = 0; s < QKFrag<CQ>::kSteps; ++s) acc = mfma32(a.w[s], b.w[s], acc);
  } else {
    acc = mfma16(a.n, b.n, acc);
  }
  return acc;
}

// Register staging of ROWS x WCH 16-B chunks (source row stride ld elements): chunk e = tid + 256 i.
// Rows >= nvalid load as zero.
template <int ROWS, int WCH>
struct Stage {
  static constexpr int kTotal = ROWS * WCH;
  static constexpr int kPer = (kTotal + 255) / 256;
  uint4 r[kPer];
  __device__ __forceinline__ void load(const bf16_t* base, size_t ld, int row0, int nvalid, int tid) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + 256 * i;
      const int rr = e / WCH, ch = e - rr * WCH;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (e < kTotal && row0 + rr < nvalid) v = *(const uint4*)(base + (size_t)(row0 + rr) * ld + ch * 8);
      r[i] = v;
    }
  }
  template <int W>
  __device__ __forceinline__ void store(char* img, int tid) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + 256 * i;
      const int rr = e / WCH, ch = e - rr * WCH;
      if (e < kTotal) *(uint4*)(img + lds_off<W>(rr, ch * 8)) = r[i];
    }
  }
};

// zero the image columns [8, 16) of a KC = 16 image holding CQ = 8 (kept zero for the whole kernel)
template <int CQ, int KC>
__device__ __forceinline__ void zero_pad_cols(char* smem, int tile_bytes, int rows, int tid) {
  if constexpr (CQ < KC) {
    for (int e = tid; e < 2 * rows; e += 256) {
      char* img = smem + (e / rows) * tile_bytes;
      *(uint4*)(img + lds_off<KC>(e % rows, 8)) = make_uint4(0, 0, 0, 0);
    }
  }
}

// ---------------------------------------------------------------------------- forward
// Workgroup: 4 waves x QB 16-query blocks; value columns [c0, c0 + DV) of grid.y; KT = 64 keys
// per LDS tile (double-buffered, register-staged).  grid (ceil(N / (64 QB)), C/DV, B).
// OT: the type of o (bf16_t; float for the pooled attention, dfcsa_lsa_flash_fwd).  y == nullptr:
// only o and lse are written (x and gamma are not read).
template <int CQ, int DV, int QB, int WPE, typename OT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
fra_fwd_mfma(int N, int C, int ldq, const bf16_t* __restrict__ qkv,
                                                    const bf16_t* __restrict__ x, const float* __restrict__ gamma,
                                                    OT* __restrict__ o, bf16_t* __restrict__ y,
                                                    float* __restrict__ lse) {
  constexpr int KT = 64;
  constexpr int KC = CQ < 16 ? 16 : CQ;
  constexpr int KB = KT * KC * 2, VB = KT * DV * 2;
  constexpr int NCB = DV / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * (KB + VB)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int b = blockIdx.z, c0 = blockIdx.y * DV;
  const int qw0 = (blockIdx.x * 4 + wave) * (16 * QB);
  const bf16_t* base = qkv + (size_t)b * N * ldq;

  zero_pad_cols<CQ, KC>(smem, KB + VB, KT, tid);

  QKFrag<CQ> qf[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const int q = qw0 + 16 * qb + li;
    qk_load_global<CQ>(qf[qb], base + (size_t)q * ldq, q < N, g);
  }
  // acc[qb][NCB] is the softmax denominator: a block of all-ones value columns, so the MFMA forms
  // the row sum of the (bf16) P it multiplies, already reduced over the query's 4 lane groups
  f32x4_t acc[QB][NCB + 1];
  float m[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    m[qb] = -INFINITY;
#pragma unroll
    for (int cb = 0; cb <= NCB; ++cb) acc[qb][cb] = zero4();
  }
  const short one = (short)0x3f80;  // bf16 1.0
  const bf16x8_t ones = {one, one, one, one, one, one, one, one};

  Stage<KT, CQ / 8> sk;
  Stage<KT, DV / 8> sv;
  const int ntiles = (N + KT - 1) / KT;
  sk.load(base + CQ, ldq, 0, N, tid);
  sv.load(base + 2 * CQ + c0, ldq, 0, N, tid);
  sk.template store<KC>(smem, tid);
  sv.template store<DV>(smem + KB, tid);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int kt0 = t * KT;
    if (t + 1 < ntiles) {
      sk.load(base + CQ, ldq, kt0 + KT, N, tid);
      sv.load(base + 2 * CQ + c0, ldq, kt0 + KT, N, tid);
    }
    const char* Ki = smem + (t & 1) * (KB + VB);
    const char* Vi = Ki + KB;

    // scores S^T[key][query] (keys on registers: row 16 ks + 4g + r; query on the lane)
    f32x4_t st[4][QB];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      QKFrag<CQ> kf;
      qk_load_lds<CQ, KC>(kf, Ki, ks * 16 + li, g);
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) st[ks][qb] = qk_mfma<CQ>(kf, qf[qb], zero4());
    }
    if (kt0 + KT > N) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kt0 + ks * 16 + 4 * g + r >= N)
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) st[ks][qb][r] = -INFINITY;
    }
    // online softmax: a query's keys are spread over its 4 lane groups and the registers
    bool need = false;
    float mx[QB];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      float v = st[0][qb][0];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int r = 0; r < 4; ++r) v = fmaxf(v, st[ks][qb][r]);
      v = fmaxf(v, __shfl_xor(v, 16, 64));
      v = fmaxf(v, __shfl_xor(v, 32, 64));
      mx[qb] = v;
      need |= (m[qb] == -INFINITY) || (v * kL2E > m[qb] * kL2E + kRescale);
    }
    if (__any(need)) {
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        const float mn = fmaxf(m[qb], mx[qb]);
        const float alpha = (m[qb] == -INFINITY) ? 0.f : exp2_((m[qb] - mn) * kL2E);
#pragma unroll
        for (int cb = 0; cb <= NCB; ++cb) acc[qb][cb] *= alpha;
        m[qb] = mn;
      }
    }
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      const float nm = -m[qb] * kL2E;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int r = 0; r < 4; ++r) st[ks][qb][r] = exp2_(fmaf(st[ks][qb][r], kL2E, nm));
    }
    // O^T[c][q] += V^T[c][key] P^T[key][q], 32 keys per MFMA
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8_t pb[QB];
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) pb[qb] = pack_b(st[2 * h][qb], st[2 * h + 1][qb]);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const bf16x8_t vf = lds_tr8<DV>(Vi, 32 * h, cb, lane);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) acc[qb][cb] = mfma32(vf, pb[qb], acc[qb][cb]);
      }
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) acc[qb][NCB] = mfma32(ones, pb[qb], acc[qb][NCB]);
    }
    if (t + 1 < ntiles) {
      char* nk = smem + ((t + 1) & 1) * (KB + VB);
      sk.template store<KC>(nk, tid);
      sv.template store<DV>(nk + KB, tid);
    }
    __syncthreads();
  }

  const float gm = y ? *gamma : 0.f;
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const float lt = acc[qb][NCB][0];
    const int q = qw0 + 16 * qb + li;
    if (q >= N) continue;
    const float inv = 1.f / lt;
    const size_t row = (size_t)b * N + q;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      const size_t off = row * C + c0 + cb * 16 + 4 * g;
      const float ov0 = acc[qb][cb][0] * inv, ov1 = acc[qb][cb][1] * inv;
      const float ov2 = acc[qb][cb][2] * inv, ov3 = acc[qb][cb][3] * inv;
      if constexpr (sizeof(OT) == 4)
        *(float4*)(o + off) = make_float4(ov0, ov1, ov2, ov3);
      else
        *(uint2*)(o + off) = make_uint2(pack2bf(ov0, ov1), pack2bf(ov2, ov3));
      if (!y) continue;
      const uint2 xv = *(const uint2*)(x + off);
      const float x0 = __uint_as_float(xv.x << 16), x1 = __uint_as_float(xv.x & 0xffff0000u);
      const float x2 = __uint_as_float(xv.y << 16), x3 = __uint_as_float(xv.y & 0xffff0000u);
      *(uint2*)(y + off) = make_uint2(pack2bf(fmaf(gm, ov0, x0), fmaf(gm, ov1, x1)),
                                      pack2bf(fmaf(gm, ov2, x2), fmaf(gm, ov3, x3)));
    }
    if (g == 0 && blockIdx.y == 0) lse[row] = m[qb] + __logf(lt);
  }
}

// ---------------------------------------------------------------------------- backward, dK/dV
// Workgroup: 4 waves x 32 keys (two 16-key blocks per wave, K and V rows held in registers);
// sweeps all queries in LDS tiles of QT = 64 (Q rows, dy rows, lse, r).  grid (ceil(N/128), 1, B).
//   S[q][k] = Q K^T, dPy'[q][k] = dy V^T - r_q (the MFMA chain starts from -r_q), P = exp(S - lse_q),
//   dS/gamma = P dPy';  dV^T[c][k] += dy^T[c][q] P[q][k], dK^T[d][k] += Q^T[d][q] (dS/gamma)[q][k],
//   both scaled by gamma at the end.  Query rows past N stage Q = dy = 0 and lse = r = 0, so their
//   P = 1 and dPy' = 0 contribute exactly nothing: no per-score masking.
template <int CQ, int C, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
fra_bwd_dkv_mfma(int N, int ldq, int ldd, const bf16_t* __restrict__ qkv,
                                                        const bf16_t* __restrict__ dy, const float* __restrict__ gamma,
                                                        const float* __restrict__ lse, const float* __restrict__ rr,
                                                        bf16_t* __restrict__ dqkv, float* __restrict__ part,
                                                        int64_t rstride) {
  constexpr int QT = 64;
  constexpr int KC = CQ < 16 ? 16 : CQ;
  constexpr int QBy = QT * KC * 2, DBy = QT * C * 2, LBy = QT * 4 * 2;
  constexpr int TB = QBy + DBy + LBy;
  constexpr int NDC = C / 32, NCB = C / 16, NDB = KC / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * TB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int b = blockIdx.z, ch = blockIdx.y, c0 = ch * C;   // value-column chunk (wide layers)
  const int kw0 = (blockIdx.x * 4 + wave) * 32;
  const bf16_t* base = qkv + (size_t)b * N * ldq;
  const bf16_t* dyb = dy + (size_t)b * N * ldd + c0;
  const float* lseb = lse + (size_t)b * N;
  const float* rrb = rr + (size_t)b * N;

  zero_pad_cols<CQ, KC>(smem, TB, QT, tid);
  // the wave's keys: K rows (B operand of S = Q K^T) and V rows (B operand of dPy = dy V^T)
  QKFrag<CQ> kf[2];
  bf16x8_t vf[2][NDC];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int key = kw0 + 16 * kb + li;
    const bool ok = key < N;
    qk_load_global<CQ>(kf[kb], base + (size_t)key * ldq + CQ, ok, g);
#pragma unroll
    for (int dc = 0; dc < NDC; ++dc)
      vf[kb][dc] = ok ? *(const bf16x8_t*)(base + (size_t)key * ldq + 2 * CQ + c0 + 32 * dc + 8 * g)
                      : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  f32x4_t dva[2][NCB], dka[2][NDB];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) dva[kb][cb] = zero4();
#pragma unroll
    for (int db = 0; db < NDB; ++db) dka[kb][db] = zero4();
  }
  const float gm = *gamma;

  Stage<QT, CQ / 8> sq;
  Stage<QT, C / 8> sd;
  auto stage_scalars = [&](char* img, int qt0) {
    float* ls = (float*)(img + QBy + DBy);
    if (tid < QT) {
      const int q = qt0 + tid;
      ls[tid] = q < N ? lseb[q] * kL2E : 0.f;
      // -r enters dP once, in chunk 0; rstride > 0: each chunk subtracts its own share r_ch (the
      // chunk's columns of rowsum(dy * o), dfcsa_lsa_flash_bwd), so every chunk's dS stays centred
      ls[QT + tid] = (q < N && (ch == 0 || rstride)) ? -rrb[q + ch * rstride] : 0.f;
    }
  };
  const int ntiles = (N + QT - 1) / QT;
  sq.load(base, ldq, 0, N, tid);
  sd.load(dyb, ldd, 0, N, tid);
  sq.template store<KC>(smem, tid);
  sd.template store<C>(smem + QBy, tid);
  stage_scalars(smem, 0);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int qt0 = t * QT;
    if (t + 1 < ntiles) {
      sq.load(base, ldq, qt0 + QT, N, tid);
      sd.load(dyb, ldd, qt0 + QT, N, tid);
    }
    const char* Qi = smem + (t & 1) * TB;
    const char* Di = Qi + QBy;
    const float* Ls = (const float*)(Di + DBy);

    // two halves of 32 queries: scores of one half are consumed by the dV/dK MFMAs before the next
    // half is formed (half the live score registers)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x4_t sp[2][2], dp[2][2];
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        const int qs = 2 * h + hs;
        QKFrag<CQ> qa;
        qk_load_lds<CQ, KC>(qa, Qi, qs * 16 + li, g);
        bf16x8_t da[NDC];
#pragma unroll
        for (int dc = 0; dc < NDC; ++dc) da[dc] = lds_row8<C>(Di, qs * 16 + li, 32 * dc + 8 * g);
        const float4 R4 = *(const float4*)(Ls + QT + qs * 16 + 4 * g);  // -r of rows 16 qs + 4g + r
        const f32x4_t nr = {R4.x, R4.y, R4.z, R4.w};
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          sp[hs][kb] = qk_mfma<CQ>(qa, kf[kb], zero4());
          f32x4_t a = nr;
#pragma unroll
          for (int dc = 0; dc < NDC; ++dc) a = mfma32(da[dc], vf[kb][dc], a);
          dp[hs][kb] = a;
        }
        // P and dS / gamma (rows = queries 16 qs + 4g + r)
        const float4 L4 = *(const float4*)(Ls + qs * 16 + 4 * g);  // lse * log2(e)
        const float Lr[4] = {L4.x, L4.y, L4.z, L4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) {
            const float p = exp2_(fmaf(sp[hs][kb][r], kL2E, -Lr[r]));
            sp[hs][kb][r] = p;
            dp[hs][kb][r] *= p;
          }
        }
      }
      bf16x8_t pb[2], sb[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        pb[kb] = pack_b(sp[0][kb], sp[1][kb]);
        sb[kb] = pack_b(dp[0][kb], dp[1][kb]);
      }
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const bf16x8_t a = lds_tr8<C>(Di, 32 * h, cb, lane);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) dva[kb][cb] = mfma32(a, pb[kb], dva[kb][cb]);
      }
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        const bf16x8_t a = lds_tr8<KC>(Qi, 32 * h, db, lane);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) dka[kb][db] = mfma32(a, sb[kb], dka[kb][db]);
      }
    }
    if (t + 1 < ntiles) {
      char* nx = smem + ((t + 1) & 1) * TB;
      sq.template store<KC>(nx, tid);
      sd.template store<C>(nx + QBy, tid);
      stage_scalars(nx, qt0 + QT);
    }
    __syncthreads();
  }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int key = kw0 + 16 * kb + li;
    if (key >= N) continue;
    bf16_t* out = dqkv + ((size_t)b * N + key) * ldq;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      const f32x4_t v = dva[kb][cb] * gm;
      *(uint2*)(out + 2 * CQ + c0 + cb * 16 + 4 * g) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
    }
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      const int d = db * 16 + 4 * g;
      if (d < CQ) {
        if (part) {  // wide layers: this chunk's share of dK (fp32, unscaled), summed by fra_wide_finish
          float* pp = part + (((size_t)ch * gridDim.z + b) * N + key) * CQ + d;
          *(float4*)pp = make_float4(dka[kb][db][0], dka[kb][db][1], dka[kb][db][2], dka[kb][db][3]);
        } else {
          const f32x4_t v = dka[kb][db] * gm;
          *(uint2*)(out + CQ + d) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------- backward, dQ
// Workgroup: 4 waves x 32 queries (Q and dy rows in registers); sweeps all keys in LDS tiles of
// KT = 64 (K rows, V rows).  grid (ceil(N/128), 1, B).
//   S^T = K Q^T, dPy'^T = V dy^T - r_q (the MFMA chain starts from -r_q), dS^T / gamma = P^T dPy'^T,
//   dQ^T[d][q] += K^T[d][k] (dS / gamma)^T[k][q], scaled by gamma at the end.  Keys past N are
//   masked on the last tile only (tile-uniform branch).
// kbar != nullptr ([B][kKeySlices][CQ] fp32: partial key sums, the image's mean key is their sum / N):
//   dQ = sum_k dS16 (K_k - mean key).  Exact dS rows
//   sum to zero (softmax), so subtracting any fixed key changes nothing -- but the bf16-ROUNDED dS16 rows
//   do not, and their rounding residue times the mean key is a coherent error that dominates dQ (and
//   the query bias gradient, sum over queries) when the keys are alike, as pooled features are.  The
//   row sums come from one more MFMA against a ones fragment, so the subtraction is exact in fp32.
constexpr int kKeySlices = 8;   // key-sum partials per image (lsa_flash_prep_kernel)
// KCEN: the centred variant (kbar non-null); the other keeps the row-sum registers out of the
// full-resolution attention's dQ kernel (config 5: 12 -> 40 spilled bytes per lane with them)
template <int CQ, int C, int WPE, bool KCEN>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
fra_bwd_dq_mfma(int N, int ldq, int ldd, const bf16_t* __restrict__ qkv,
                                                       const bf16_t* __restrict__ dy, const float* __restrict__ gamma,
                                                       const float* __restrict__ lse, const float* __restrict__ rr,
                                                       bf16_t* __restrict__ dqkv, float* __restrict__ part,
                                                       int64_t rstride, const float* __restrict__ kbar) {
  constexpr int KT = 64;
  constexpr int KC = CQ < 16 ? 16 : CQ;
  constexpr int KBy = KT * KC * 2, VBy = KT * C * 2, TB = KBy + VBy;
  constexpr int NDC = C / 32, NDB = KC / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * TB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int b = blockIdx.z, ch = blockIdx.y, c0 = ch * C;   // value-column chunk (wide layers)
  const int qw0 = (blockIdx.x * 4 + wave) * 32;
  const bf16_t* base = qkv + (size_t)b * N * ldq;
  const bf16_t* dyb = dy + (size_t)b * N * ldd + c0;

  zero_pad_cols<CQ, KC>(smem, TB, KT, tid);
  QKFrag<CQ> qf[2];
  bf16x8_t df[2][NDC];
  float Lq[2];
  f32x4_t nR[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = qw0 + 16 * qb + li;
    const bool ok = q < N;
    qk_load_global<CQ>(qf[qb], base + (size_t)q * ldq, ok, g);
#pragma unroll
    for (int dc = 0; dc < NDC; ++dc)
      df[qb][dc] = ok ? *(const bf16x8_t*)(dyb + (size_t)q * ldd + 32 * dc + 8 * g) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    Lq[qb] = ok ? -lse[(size_t)b * N + q] * kL2E : 0.f;
    const float nr = (ok && (ch == 0 || rstride)) ? -rr[(size_t)b * N + q + ch * rstride] : 0.f;  // (see dK/dV)
    nR[qb] = f32x4_t{nr, nr, nr, nr};
  }
  f32x4_t dqa[2][NDB], rsum[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    rsum[qb] = zero4();
#pragma unroll
    for (int db = 0; db < NDB; ++db) dqa[qb][db] = zero4();
  }
  const short b1 = 0x3F80;   // bf16 1.0
  const bf16x8_t ones = {b1, b1, b1, b1, b1, b1, b1, b1};
  const float gm = *gamma;

  Stage<KT, CQ / 8> sk;
  Stage<KT, C / 8> sv;
  const int ntiles = (N + KT - 1) / KT;
  sk.load(base + CQ, ldq, 0, N, tid);
  sv.load(base + 2 * CQ + c0, ldq, 0, N, tid);
  sk.template store<KC>(smem, tid);
  sv.template store<C>(smem + KBy, tid);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int kt0 = t * KT;
    if (t + 1 < ntiles) {
      sk.load(base + CQ, ldq, kt0 + KT, N, tid);
      sv.load(base + 2 * CQ + c0, ldq, kt0 + KT, N, tid);
    }
    const char* Ki = smem + (t & 1) * TB;
    const char* Vi = Ki + KBy;
    f32x4_t ds[4][2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      QKFrag<CQ> ka;
      qk_load_lds<CQ, KC>(ka, Ki, ks * 16 + li, g);
      bf16x8_t va[NDC];
#pragma unroll
      for (int dc = 0; dc < NDC; ++dc) va[dc] = lds_row8<C>(Vi, ks * 16 + li, 32 * dc + 8 * g);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const f32x4_t s = qk_mfma<CQ>(ka, qf[qb], zero4());
        f32x4_t d = nR[qb];
#pragma unroll
        for (int dc = 0; dc < NDC; ++dc) d = mfma32(va[dc], df[qb][dc], d);
#pragma unroll
        for (int r = 0; r < 4; ++r) d[r] *= exp2_(fmaf(s[r], kL2E, Lq[qb]));
        ds[ks][qb] = d;
      }
    }
    if (kt0 + KT > N) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kt0 + ks * 16 + 4 * g + r >= N)
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) ds[ks][qb][r] = 0.f;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8_t sb[2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) sb[qb] = pack_b(ds[2 * h][qb], ds[2 * h + 1][qb]);
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        const bf16x8_t a = lds_tr8<KC>(Ki, 32 * h, db, lane);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) dqa[qb][db] = mfma32(a, sb[qb], dqa[qb][db]);
      }
      if (KCEN) {   // column sums of the rounded dS^T tile (every row of rsum holds them)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) rsum[qb] = mfma32(ones, sb[qb], rsum[qb]);
      }
    }
    if (t + 1 < ntiles) {
      char* nx = smem + ((t + 1) & 1) * TB;
      sk.template store<KC>(nx, tid);
      sv.template store<C>(nx + KBy, tid);
    }
    __syncthreads();
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = qw0 + 16 * qb + li;
    if (q >= N) continue;
    bf16_t* out = dqkv + ((size_t)b * N + q) * ldq;
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      const int d = db * 16 + 4 * g;
      if (d < CQ) {
        if (KCEN) {   // kbar: kKeySlices partial key sums per image, [B][kKeySlices][CQ]
          float4 kb = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int ks = 0; ks < kKeySlices; ++ks) {
            const float4 v = *(const float4*)(kbar + ((size_t)b * kKeySlices + ks) * CQ + d);
            kb.x += v.x; kb.y += v.y; kb.z += v.z; kb.w += v.w;
          }
          const float invn = 1.f / (float)N;
          kb.x *= invn; kb.y *= invn; kb.z *= invn; kb.w *= invn;
          const float rs = rsum[qb][0];
          dqa[qb][db][0] -= rs * kb.x; dqa[qb][db][1] -= rs * kb.y;
          dqa[qb][db][2] -= rs * kb.z; dqa[qb][db][3] -= rs * kb.w;
        }
        if (part) {  // wide layers: this chunk's share of dQ (fp32, unscaled)
          float* pp = part + (((size_t)ch * gridDim.z + b) * N + q) * CQ + d;
          *(float4*)pp = make_float4(dqa[qb][db][0], dqa[qb][db][1], dqa[qb][db][2], dqa[qb][db][3]);
        } else {
          const f32x4_t v = dqa[qb][db] * gm;
          *(uint2*)(out + d) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------- dispatch
// Waves-per-SIMD budgets of the C = 64 / 128 MFMA kernels (tuning knob 10): bit 0 forward (3 / 2
// waves), bit 1 dK/dV (3 / 2), bit 2 dQ (4 / 3), bit 3 forward at 4 waves for C = 64; 0 leaves the
// compiler's default budget (kept for A/B measurements).  Default 15: all on.
int fra_occ_tuned() { return g_fra_occ; }

int fwd_dv(int C) {
  if (C == 64 || C == 128 || C == 256) return C;
  if (C % 256 == 0) return 256;
  if (C % 128 == 0) return 128;
  return 64;
}

bool mfma_fwd_ok(int dtype, int C, int Cq, int ldq) {
  return dtype == DFCSA_DT_BF16 && C % 64 == 0 && ldq % 8 == 0 &&
         (Cq == 8 || Cq == 16 || Cq == 32 || Cq == 64 || Cq == 128);
}
bool mfma_bwd_ok(int dtype, int C, int Cq, int ldq) {
  return dtype == DFCSA_DT_BF16 && (C == 64 || C == 128 || C == 256) && ldq % 8 == 0 &&
         (Cq == 8 || Cq == 16 || Cq == 32 || (Cq == 64 && C == 64));
}

template <int CQ, int DV, int QB, int WPE, typename OT>
void launch_fwd_w(dim3 grid, int N, int C, int ldq, const void* qkv, const void* x, const float* gamma, void* o,
                  void* y, float* lse, hipStream_t st) {
  hipLaunchKernelGGL((fra_fwd_mfma<CQ, DV, QB, WPE, OT>), grid, dim3(256), 0, st, N, C, ldq, (const bf16_t*)qkv,
                     (const bf16_t*)x, gamma, (OT*)o, (bf16_t*)y, lse);
}

template <int CQ, int DV, typename OT>
void launch_fwd(int B, int N, int C, int ldq, const void* qkv, const void* x, const float* gamma, void* o, void* y,
                float* lse, hipStream_t st) {
  constexpr int QB = DV <= 128 ? 2 : 1;
  dim3 grid((N + 64 * QB - 1) / (64 * QB), C / DV, B);
  // waves-per-SIMD budgets (knob 10): without one the compiler sizes these kernels for 1-2 waves
  const int occ = fra_occ_tuned();
  if constexpr (DV == 64 && CQ <= 16) {
    if (occ & 8) return launch_fwd_w<CQ, DV, QB, 4, OT>(grid, N, C, ldq, qkv, x, gamma, o, y, lse, st);
    if (occ & 1) return launch_fwd_w<CQ, DV, QB, 3, OT>(grid, N, C, ldq, qkv, x, gamma, o, y, lse, st);
  }
  if constexpr (DV == 128 && CQ <= 16) {
    if (occ & 1) return launch_fwd_w<CQ, DV, QB, 2, OT>(grid, N, C, ldq, qkv, x, gamma, o, y, lse, st);
  }
  launch_fwd_w<CQ, DV, QB, 1, OT>(grid, N, C, ldq, qkv, x, gamma, o, y, lse, st);
}

template <int CQ, typename OT = bf16_t>
void launch_fwd_cq(int B, int N, int C, int ldq, const void* qkv, const void* x, const float* gamma, void* o,
                   void* y, float* lse, hipStream_t st) {
  switch (fwd_dv(C)) {
    case 64: launch_fwd<CQ, 64, OT>(B, N, C, ldq, qkv, x, gamma, o, y, lse, st); break;
    case 128: launch_fwd<CQ, 128, OT>(B, N, C, ldq, qkv, x, gamma, o, y, lse, st); break;
    default: launch_fwd<CQ, 256, OT>(B, N, C, ldq, qkv, x, gamma, o, y, lse, st); break;
  }
}

// C = the value-column width one workgroup owns; Ctot = C except on wide layers, where grid.y runs
// over the Ctot / C chunks and dQ / dK leave as per-chunk fp32 partials (part: dK shares, then dQ
// shares) for fra_wide_finish.
template <int CQ, int C>
void launch_bwd(int B, int N, int ldq, int Ctot, const void* qkv, const void* dy, const float* gamma,
                const float* lse, const float* rr, void* dqkv, float* part, hipStream_t st, int64_t rstride = 0,
                const float* kbar = nullptr) {
  dim3 grid((N + 127) / 128, Ctot / C, B);
  float* pk = part;
  float* pq = part ? part + (size_t)(Ctot / C) * B * N * CQ : nullptr;
  const int occ = fra_occ_tuned();
  constexpr bool narrow = CQ <= 16 && (C == 64 || C == 128);
  constexpr int WKV = C == 64 ? 3 : 2, WQ = C == 64 ? 4 : 3;
  if (narrow && (occ & 2))
    hipLaunchKernelGGL((fra_bwd_dkv_mfma<CQ, C, narrow ? WKV : 1>), grid, dim3(256), 0, st, N, ldq, Ctot,
                       (const bf16_t*)qkv, (const bf16_t*)dy, gamma, lse, rr, (bf16_t*)dqkv, pk, rstride);
  else
    hipLaunchKernelGGL((fra_bwd_dkv_mfma<CQ, C, 1>), grid, dim3(256), 0, st, N, ldq, Ctot, (const bf16_t*)qkv,
                       (const bf16_t*)dy, gamma, lse, rr, (bf16_t*)dqkv, pk, rstride);
  if (narrow && (occ & 4)) {
    if (kbar)
      hipLaunchKernelGGL((fra_bwd_dq_mfma<CQ, C, narrow ? WQ : 1, true>), grid, dim3(256), 0, st, N, ldq, Ctot,
                         (const bf16_t*)qkv, (const bf16_t*)dy, gamma, lse, rr, (bf16_t*)dqkv, pq, rstride, kbar);
    else
      hipLaunchKernelGGL((fra_bwd_dq_mfma<CQ, C, narrow ? WQ : 1, false>), grid, dim3(256), 0, st, N, ldq, Ctot,
                         (const bf16_t*)qkv, (const bf16_t*)dy, gamma, lse, rr, (bf16_t*)dqkv, pq, rstride, kbar);
  } else {
    if (kbar)
      hipLaunchKernelGGL((fra_bwd_dq_mfma<CQ, C, 1, true>), grid, dim3(256), 0, st, N, ldq, Ctot, (const bf16_t*)qkv,
                         (const bf16_t*)dy, gamma, lse, rr, (bf16_t*)dqkv, pq, rstride, kbar);
    else
      hipLaunchKernelGGL((fra_bwd_dq_mfma<CQ, C, 1, false>), grid, dim3(256), 0, st, N, ldq, Ctot, (const bf16_t*)qkv,
                         (const bf16_t*)dy, gamma, lse, rr, (bf16_t*)dqkv, pq, rstride, kbar);
  }
}

template <int CQ>
void launch_bwd_cq(int B, int N, int C, int ldq, const void* qkv, const void* dy, const float* gamma,
                   const float* lse, const float* rr, void* dqkv, hipStream_t st, const float* kbar = nullptr) {
  if (C == 64) launch_bwd<CQ, 64>(B, N, ldq, C, qkv, dy, gamma, lse, rr, dqkv, nullptr, st, 0, kbar);
  else if (C == 128) launch_bwd<CQ, 128>(B, N, ldq, C, qkv, dy, gamma, lse, rr, dqkv, nullptr, st, 0, kbar);
  else launch_bwd<CQ, 256>(B, N, ldq, C, qkv, dy, gamma, lse, rr, dqkv, nullptr, st, 0, kbar);
}

// Wide layers (C > 256: the 64^2 / 32^2 levels of config 5): value columns in chunks of kWideChunk.
// dP = dy V^T is a sum over value columns and dS = gamma P (dP - r) is linear in dP, so each chunk's
// kernels compute dS_chunk = gamma P dP_chunk (-r added by chunk 0 only) and dQ = sum_chunks dS_chunk K,
// dK = sum_chunks dS_chunk^T Q exactly; dV columns belong to one chunk and are written directly.
// The score tile is recomputed per chunk (d_qk = C/8 << kWideChunk, a small share of the MFMAs).
constexpr int kWideChunk = 128;

bool wide_bwd_ok(int dtype, int C, int Cq, int ldq) {
  return dtype == DFCSA_DT_BF16 && C > 256 && C % kWideChunk == 0 && C <= 4096 && ldq % 8 == 0 &&
         (Cq == 8 || Cq == 16 || Cq == 32 || Cq == 64 || Cq == 128);
}

// dqkv[row][0, CQ) = gamma * sum_chunks dQ share, dqkv[row][CQ, 2CQ) = gamma * sum_chunks dK share;
// one thread per (row, 4 columns), chunk order fixed (deterministic)
__global__ void __launch_bounds__(256) fra_wide_finish(int64_t rows, int CQ, int nch, int ldq,
                                                       const float* __restrict__ part,
                                                       const float* __restrict__ gamma, bf16_t* __restrict__ dqkv) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int q4 = CQ / 4;
  if (e >= 2 * rows * q4) return;
  const int which = (int)(e / (rows * q4));  // 0 = dK, 1 = dQ
  const int64_t rem = e - (int64_t)which * rows * q4;
  const int64_t row = rem / q4;
  const int d = (int)(rem - row * q4) * 4;
  const float* p = part + ((size_t)which * nch * rows + row) * CQ + d;
  float4 s = *(const float4*)p;
  for (int c = 1; c < nch; ++c) {
    const float4 v = *(const float4*)(p + (size_t)c * rows * CQ);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const float gm = *gamma;
  bf16_t* out = dqkv + row * ldq + (which == 0 ? CQ : 0) + d;
  *(uint2*)out = make_uint2(pack2bf(gm * s.x, gm * s.y), pack2bf(gm * s.z, gm * s.w));
}

}  // namespace

extern "C" int dfcsa_fra_path(int dtype, int C, int Cq, int ldq, int backward) {
  if (g_fra_generic) return 0;
  if (!backward) return mfma_fwd_ok(dtype, C, Cq, ldq) ? 1 : 0;
  if (mfma_bwd_ok(dtype, C, Cq, ldq)) return 1;
  return wide_bwd_ok(dtype, C, Cq, ldq) ? 2 : 0;  // value-chunked MFMA kernels + dfcsa_fra_bwd_wide
}

extern "C" int dfcsa_fra_bwd_wide_bytes(int B, int N, int C, int Cq, int64_t* bytes) {
  if (B <= 0 || N <= 0 || C <= 0 || Cq <= 0 || !bytes) return DFCSA_EINVAL;
  *bytes = (int64_t)2 * (C / kWideChunk) * B * N * Cq * (int64_t)sizeof(float);
  return 0;
}

extern "C" int dfcsa_fra_bwd_wide(int dtype, int B, int N, int C, int Cq, int ldq, const void* qkv, const void* dy,
                                  const float* gamma, const float* lse, const float* r, void* dqkv, float* work,
                                  void* stream) {
  if (B <= 0 || N <= 0 || !work || !wide_bwd_ok(dtype, C, Cq, ldq) || g_fra_generic) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  ProfScope prof(DFCSA_PROF_ATTN, st, 4.0 * B * (double)N * N * (Cq + C));
  if (ldq != 2 * Cq + C) {
    hipError_t e = hipMemsetAsync(dqkv, 0, (size_t)B * N * ldq * 2, st);
    if (e != hipSuccess) return -(int)e;
  }
  switch (Cq) {
    case 8: launch_bwd<8, kWideChunk>(B, N, ldq, C, qkv, dy, gamma, lse, r, dqkv, work, st); break;
    case 16: launch_bwd<16, kWideChunk>(B, N, ldq, C, qkv, dy, gamma, lse, r, dqkv, work, st); break;
    case 32: launch_bwd<32, kWideChunk>(B, N, ldq, C, qkv, dy, gamma, lse, r, dqkv, work, st); break;
    case 64: launch_bwd<64, kWideChunk>(B, N, ldq, C, qkv, dy, gamma, lse, r, dqkv, work, st); break;
    default: launch_bwd<128, kWideChunk>(B, N, ldq, C, qkv, dy, gamma, lse, r, dqkv, work, st); break;
  }
  const int64_t rows = (int64_t)B * N, threads = 2 * rows * (Cq / 4);
  hipLaunchKernelGGL(fra_wide_finish, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, rows, Cq,
                     C / kWideChunk, ldq, work, gamma, (bf16_t*)dqkv);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_fra_fwd(int dtype, int B, int N, int C, int Cq, int ldq, const void* qkv, const void* x,
                             const float* gamma, void* o, void* y, float* lse, void* stream) {
  if (B <= 0 || N <= 0 || C <= 0 || C > 4096 || Cq <= 0 || Cq > 128 || ldq < 2 * Cq + C) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const bool fast = !g_fra_generic && mfma_fwd_ok(dtype, C, Cq, ldq);
  if (!fast && C > 1024) return DFCSA_EINVAL;
  ProfScope prof(DFCSA_PROF_ATTN, st, 2.0 * B * (double)N * N * (Cq + C));
  if (fast) {
    switch (Cq) {
      case 8: launch_fwd_cq<8>(B, N, C, ldq, qkv, x, gamma, o, y, lse, st); break;
      case 16: launch_fwd_cq<16>(B, N, C, ldq, qkv, x, gamma, o, y, lse, st); break;
      case 32: launch_fwd_cq<32>(B, N, C, ldq, qkv, x, gamma, o, y, lse, st); break;
      case 64: launch_fwd_cq<64>(B, N, C, ldq, qkv, x, gamma, o, y, lse, st); break;
      default: launch_fwd_cq<128>(B, N, C, ldq, qkv, x, gamma, o, y, lse, st); break;
    }
  } else {
    dim3 grid((N + 3) / 4, B);
    const size_t shm = (size_t)4 * Cq * sizeof(float);
    if (dtype == DFCSA_DT_BF16)
      hipLaunchKernelGGL(fra_fwd_generic<bf16_t>, grid, dim3(256), shm, st, N, C, Cq, ldq, (const bf16_t*)qkv,
                         (const bf16_t*)x, gamma, (bf16_t*)o, (bf16_t*)y, lse);
    else
      hipLaunchKernelGGL(fra_fwd_generic<float>, grid, dim3(256), shm, st, N, C, Cq, ldq, (const float*)qkv,
                         (const float*)x, gamma, (float*)o, (float*)y, lse);
  }
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_fra_bwd_prep(int dtype, int rows, int C, const void* dy, const void* o, float* r, void* stream) {
  if (rows <= 0 || C <= 0) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((rows + 3) / 4);
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(fra_bwd_prep_kernel<bf16_t>, grid, dim3(256), 0, st, rows, C, (const bf16_t*)dy,
                       (const bf16_t*)o, r);
  else
    hipLaunchKernelGGL(fra_bwd_prep_kernel<float>, grid, dim3(256), 0, st, rows, C, (const float*)dy,
                       (const float*)o, r);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_fra_bwd(int dtype, int B, int N, int C, int Cq, int ldq, const void* qkv, const void* dy,
                             const float* gamma, const float* lse, const float* r, void* dqkv, void* stream) {
  if (B <= 0 || N <= 0 || C <= 0 || C > 1024 || Cq <= 0 || Cq > 128 || ldq < 2 * Cq + C) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  ProfScope prof(DFCSA_PROF_ATTN, st, 4.0 * B * (double)N * N * (Cq + C));
  if (!g_fra_generic && mfma_bwd_ok(dtype, C, Cq, ldq)) {
    if (ldq != 2 * Cq + C) {  // padding columns are not written by the MFMA kernels
      hipError_t e = hipMemsetAsync(dqkv, 0, (size_t)B * N * ldq * 2, st);
      if (e != hipSuccess) return -(int)e;
    }
    switch (Cq) {
      case 8: launch_bwd_cq<8>(B, N, C, ldq, qkv, dy, gamma, lse, r, dqkv, st); break;
      case 16: launch_bwd_cq<16>(B, N, C, ldq, qkv, dy, gamma, lse, r, dqkv, st); break;
      case 32: launch_bwd_cq<32>(B, N, C, ldq, qkv, dy, gamma, lse, r, dqkv, st); break;
      default: launch_bwd<64, 64>(B, N, ldq, C, qkv, dy, gamma, lse, r, dqkv, nullptr, st); break;   // ViT heads
    }
  } else {
    dim3 grid((N + 3) / 4, B);
    const size_t shm = (size_t)4 * (Cq + C) * sizeof(float);
    if (dtype == DFCSA_DT_BF16) {
      hipLaunchKernelGGL(fra_bwd_dq_generic<bf16_t>, grid, dim3(256), shm, st, N, C, Cq, ldq, (const bf16_t*)qkv,
                         (const bf16_t*)dy, gamma, lse, r, (bf16_t*)dqkv);
      hipLaunchKernelGGL(fra_bwd_dkv_generic<bf16_t>, grid, dim3(256), shm, st, N, C, Cq, ldq, (const bf16_t*)qkv,
                         (const bf16_t*)dy, gamma, lse, r, (bf16_t*)dqkv);
    } else {
      hipLaunchKernelGGL(fra_bwd_dq_generic<float>, grid, dim3(256), shm, st, N, C, Cq, ldq, (const float*)qkv,
                         (const float*)dy, gamma, lse, r, (float*)dqkv);
      hipLaunchKernelGGL(fra_bwd_dkv_generic<float>, grid, dim3(256), shm, st, N, C, Cq, ldq, (const float*)qkv,
                         (const float*)dy, gamma, lse, r, (float*)dqkv);
    }
  }
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// ============================================================================ pooled attention
// LightSelfAttention's core at P >= 8 (reference models/unet_dfc_sa_res.py:28-33, the
// config_dfc-sa-res-block-p16 / -p32 pool sizes: N = P*P = 256 / 1024 pooled tokens) on the flash
// kernels above, with gamma = 1: the LSA applies gamma after the bilinear upsample (:36-38), and its
// backward hands over dO = gamma * U^T dattn (dfcsa_lsa_up_bwd_cols).  qkv [B][N][ldq], ldq = 2Cq + C,
// is the fp32 projection output (fp32 mode: the generic fp32 kernels read it directly) or its bf16
// copy (bf16 mode: the bf16 MFMA kernels).  o, dO and dqkv are fp32 in both modes (what the pooled
// path's other kernels consume).
namespace {

constexpr size_t kLsaAlign = 256;
size_t lsa_al(size_t b) { return (b + kLsaAlign - 1) / kLsaAlign * kLsaAlign; }

bool lsa_mfma_ok(int C, int Cq, int ldq) {
  return mfma_fwd_ok(DFCSA_DT_BF16, C, Cq, ldq) &&
         (mfma_bwd_ok(DFCSA_DT_BF16, C, Cq, ldq) || wide_bwd_ok(DFCSA_DT_BF16, C, Cq, ldq));
}

// wave per row: r[row] = sum_c dO * o (fp32); bf16 mode also writes dO16 = bf16(dO) and forms r from
// the ROUNDED dO16, the same operand the MFMA dP = dO16 V^T uses: dS = P (dP - r) then holds
// sum_c dO16_c (V_jc - o_c), in which the rounding error of dO (nearly the same for every key when the
// value rows are alike, as pooled features after BatchNorm + ReLU are) cancels instead of entering
// dS as P * sum_c (dO16 - dO)_c V_c -- a coherent error along P that swamped dq / dk at the model's
// P = 8 layers (cos 0.44 against float64 on down1's query weight gradient with fp32 r).  Block 0
// writes one[0] = 1 (the gamma the flash kernels read).
// nch > 1 (value-chunked backward): r holds one share per 128-column chunk, r[ch * rows + row]
// kpart != nullptr: the workgroups past the row blocks (B * kKeySlices of them) also form the key sums
// the centred dQ needs, kpart[b][s][c] = sum of the bf16 key column c over tokens [s N/8, (s+1) N/8) of
// image b (fixed order: thread (row lane, c) strided sums, then the row lanes in order)
__global__ void __launch_bounds__(256) lsa_flash_prep_kernel(int rows, int C, int nch, const float* __restrict__ dO,
                                                             const float* __restrict__ o, float* __restrict__ r,
                                                             bf16_t* __restrict__ dO16, float* __restrict__ one,
                                                             int N, int Cq, int ldq, const bf16_t* __restrict__ qkv,
                                                             float* __restrict__ kpart) {
  const int rblocks = (rows + 3) / 4;
  if (blockIdx.x == 0 && threadIdx.x == 0) *one = 1.f;
  if ((int)blockIdx.x >= rblocks) {
    __shared__ float red[256];
    const int kb = blockIdx.x - rblocks, b = kb / kKeySlices, sl = kb - b * kKeySlices;
    const int t0 = (int)(((int64_t)sl * N) / kKeySlices), t1 = (int)(((int64_t)(sl + 1) * N) / kKeySlices);
    const int c = threadIdx.x % Cq, rl = threadIdx.x / Cq, nrl = 256 / Cq;   // Cq divides 256 (host-checked)
    const bf16_t* k = qkv + (size_t)b * N * ldq + Cq + c;
    float a0 = 0.f, a1 = 0.f;
    int t = t0 + rl;
    for (; t + nrl < t1; t += 2 * nrl) {
      a0 += bf2f(k[(size_t)t * ldq]);
      a1 += bf2f(k[(size_t)(t + nrl) * ldq]);
    }
    if (t < t1) a0 += bf2f(k[(size_t)t * ldq]);
    red[threadIdx.x] = a0 + a1;
    __syncthreads();
    if ((int)threadIdx.x < Cq) {
      float v = 0.f;
      for (int i = 0; i < nrl; ++i) v += red[i * Cq + threadIdx.x];
      kpart[((size_t)b * kKeySlices + sl) * Cq + threadIdx.x] = v;
    }
    return;
  }
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* a = dO + (size_t)row * C;
  const float* v = o + (size_t)row * C;
  if (nch > 1) {   // C = 128 nch: lanes 0-31 cover the first 128 columns of each 256, lanes 32-63 the next
    for (int c0 = 0; c0 < C; c0 += 256) {
      const int c = c0 + lane * 4;
      float s = 0.f;
      if (c < C) {   // (C = 384: the last 256-column step is half full)
        float4 x = *(const float4*)(a + c);
        const float4 y = *(const float4*)(v + c);
        const uint2 u = make_uint2(pack2bf(x.x, x.y), pack2bf(x.z, x.w));
        *(uint2*)(dO16 + (size_t)row * C + c) = u;
        x.x = __uint_as_float(u.x << 16); x.y = __uint_as_float(u.x & 0xffff0000u);
        x.z = __uint_as_float(u.y << 16); x.w = __uint_as_float(u.y & 0xffff0000u);
        s = x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
      }
#pragma unroll
      for (int off = 1; off < 32; off <<= 1) s += __shfl_xor(s, off, 64);   // within each 32-lane half
      const int ch = c0 / 128 + (lane >> 5);
      if ((lane & 31) == 0 && ch < nch) r[(size_t)ch * rows + row] = s;
    }
    return;
  }
  float s = 0.f;
  for (int c = lane * 4; c < C; c += 256) {
    float4 x = *(const float4*)(a + c);
    const float4 y = *(const float4*)(v + c);
    if (dO16) {
      const uint2 u = make_uint2(pack2bf(x.x, x.y), pack2bf(x.z, x.w));
      *(uint2*)(dO16 + (size_t)row * C + c) = u;
      x.x = __uint_as_float(u.x << 16); x.y = __uint_as_float(u.x & 0xffff0000u);
      x.z = __uint_as_float(u.y << 16); x.w = __uint_as_float(u.y & 0xffff0000u);
    }
    s += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
  }
  s = wave_sum(s);
  if (lane == 0) r[row] = s;
}

// dst (fp32) = src (bf16), 8 elements per thread (dfcsa_bf16_to_f32)
__global__ void __launch_bounds__(256) lsa_flash_widen_kernel(int64_t n8, const bf16_t* __restrict__ src,
                                                              float* __restrict__ dst) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n8) return;
  const uint4 u = *(const uint4*)(src + 8 * e);
  float4 lo, hi;
  lo.x = __uint_as_float(u.x << 16); lo.y = __uint_as_float(u.x & 0xffff0000u);
  lo.z = __uint_as_float(u.y << 16); lo.w = __uint_as_float(u.y & 0xffff0000u);
  hi.x = __uint_as_float(u.z << 16); hi.y = __uint_as_float(u.z & 0xffff0000u);
  hi.z = __uint_as_float(u.w << 16); hi.w = __uint_as_float(u.w & 0xffff0000u);
  *(float4*)(dst + 8 * e) = lo;
  *(float4*)(dst + 8 * e + 4) = hi;
}

// work layout: one (1 float) | r [B*N] | bf16 mode: dO16 [B*N][C] | key sums [B][kKeySlices][Cq] | wide partials
struct LsaWork {
  size_t one, r, dO16, kbar, part, total;
};
LsaWork lsa_work(int dtype, int B, int N, int C, int Cq, int ldq) {
  LsaWork w{};
  const size_t rows = (size_t)B * N;
  const bool wide = dtype == DFCSA_DT_BF16 && !mfma_bwd_ok(dtype, C, Cq, ldq);
  const int nch = wide ? C / kWideChunk : 1;   // r: one share per 128-column chunk on wide layers
  w.one = 0;
  w.r = lsa_al(sizeof(float));
  size_t e = w.r + lsa_al((size_t)nch * rows * sizeof(float));
  if (dtype == DFCSA_DT_BF16) {
    w.dO16 = e;
    e += lsa_al(rows * C * 2);
    w.kbar = e;
    e += lsa_al((size_t)B * kKeySlices * Cq * sizeof(float));
    if (wide) {
      w.part = e;
      e += lsa_al((size_t)2 * nch * rows * Cq * sizeof(float));
    }
  }
  w.total = e;
  return w;
}

bool lsa_shape_ok(int dtype, int B, int N, int C, int Cq, int ldq) {
  if (B <= 0 || N <= 0 || C <= 0 || C % 4 || C > 1024 || Cq <= 0 || Cq > 128 || ldq != 2 * Cq + C) return false;
  if (dtype == DFCSA_DT_BF16) return !g_fra_generic && lsa_mfma_ok(C, Cq, ldq);
  return dtype == DFCSA_DT_F32;
}

}  // namespace

extern "C" int dfcsa_lsa_flash_path(int C, int Cq, int ldq) {
  return (!g_fra_generic && ldq == 2 * Cq + C && C <= 1024 && lsa_mfma_ok(C, Cq, ldq)) ? 1 : 0;
}

extern "C" int dfcsa_lsa_flash_fwd(int dtype, int B, int N, int C, int Cq, int ldq, const void* qkv, float* o,
                                   float* lse, void* stream) {
  if (!lsa_shape_ok(dtype, B, N, C, Cq, ldq) || !qkv || !o || !lse) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  ProfScope prof(DFCSA_PROF_ATTN, st, 2.0 * B * (double)N * N * (Cq + C));
  if (dtype == DFCSA_DT_BF16) {
    switch (Cq) {
      case 8: launch_fwd_cq<8, float>(B, N, C, ldq, qkv, nullptr, nullptr, o, nullptr, lse, st); break;
      case 16: launch_fwd_cq<16, float>(B, N, C, ldq, qkv, nullptr, nullptr, o, nullptr, lse, st); break;
      case 32: launch_fwd_cq<32, float>(B, N, C, ldq, qkv, nullptr, nullptr, o, nullptr, lse, st); break;
      case 64: launch_fwd_cq<64, float>(B, N, C, ldq, qkv, nullptr, nullptr, o, nullptr, lse, st); break;
      default: launch_fwd_cq<128, float>(B, N, C, ldq, qkv, nullptr, nullptr, o, nullptr, lse, st); break;
    }
  } else {
    hipLaunchKernelGGL(fra_fwd_generic<float>, dim3((N + 3) / 4, B), dim3(256), (size_t)4 * Cq * sizeof(float), st,
                       N, C, Cq, ldq, (const float*)qkv, nullptr, nullptr, o, nullptr, lse);
  }
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// The bf16 flash backward's kernels after the prep step (dO16, r and one already in `work`; kb: the key
// sums of the centred dQ, or nullptr): dfcsa_lsa_flash_bwd and the fused column pass of lsa.hip
// (dfcsa_lsa_flash_bwd_up) share it.
void lsa_flash_bwd_core(int B, int N, int C, int Cq, int ldq, const void* qkv, const float* lse, void* dqkv, void* work,
                        const float* kb, hipStream_t st) {
  const int dtype = DFCSA_DT_BF16;
  const LsaWork w = lsa_work(dtype, B, N, C, Cq, ldq);
  char* wb = (char*)work;
  const float* one = (const float*)(wb + w.one);
  const float* r = (const float*)(wb + w.r);
  const bf16_t* dO16 = (const bf16_t*)(wb + w.dO16);
  const int rows = B * N;
  bf16_t* dq16 = (bf16_t*)dqkv;
  if (mfma_bwd_ok(dtype, C, Cq, ldq)) {
    switch (Cq) {
      case 8: launch_bwd_cq<8>(B, N, C, ldq, qkv, dO16, one, lse, r, dq16, st, kb); break;
      case 16: launch_bwd_cq<16>(B, N, C, ldq, qkv, dO16, one, lse, r, dq16, st, kb); break;
      case 32: launch_bwd_cq<32>(B, N, C, ldq, qkv, dO16, one, lse, r, dq16, st, kb); break;
      default: launch_bwd<64, 64>(B, N, ldq, C, qkv, dO16, one, lse, r, dq16, nullptr, st, 0, kb); break;
    }
  } else {
    float* part = (float*)(wb + w.part);
    switch (Cq) {
      case 8: launch_bwd<8, kWideChunk>(B, N, ldq, C, qkv, dO16, one, lse, r, dq16, part, st, rows, kb); break;
      case 16: launch_bwd<16, kWideChunk>(B, N, ldq, C, qkv, dO16, one, lse, r, dq16, part, st, rows, kb); break;
      case 32: launch_bwd<32, kWideChunk>(B, N, ldq, C, qkv, dO16, one, lse, r, dq16, part, st, rows, kb); break;
      case 64: launch_bwd<64, kWideChunk>(B, N, ldq, C, qkv, dO16, one, lse, r, dq16, part, st, rows, kb); break;
      default: launch_bwd<128, kWideChunk>(B, N, ldq, C, qkv, dO16, one, lse, r, dq16, part, st, rows, kb); break;
    }
    const int64_t threads = 2 * (int64_t)rows * (Cq / 4);
    hipLaunchKernelGGL(fra_wide_finish, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, (int64_t)rows, Cq,
                       C / kWideChunk, ldq, part, one, dq16);
  }
}


// work pointers of the bf16 flash backward for a caller that forms dO16 / r itself (r: nch shares of
// 128 value columns on wide layers, else 1) and the key-sum / one launch; 0 or DFCSA_EINVAL
int lsa_flash_prepare_ext(int B, int N, int C, int Cq, int ldq, const void* qkv, void* work, int64_t work_bytes,
                          bf16_t** dO16, float** r, int* nch, const float** kb, hipStream_t st) {
  const int dtype = DFCSA_DT_BF16;
  if (!lsa_shape_ok(dtype, B, N, C, Cq, ldq) || !qkv || !work) return DFCSA_EINVAL;
  const LsaWork w = lsa_work(dtype, B, N, C, Cq, ldq);
  if (work_bytes < (int64_t)w.total || ((uintptr_t)work & 15)) return DFCSA_EINVAL;
  char* wb = (char*)work;
  *dO16 = (bf16_t*)(wb + w.dO16);
  *r = (float*)(wb + w.r);
  *nch = mfma_bwd_ok(dtype, C, Cq, ldq) ? 1 : C / kWideChunk;
  float* k = (g_lsa_key_centre && 256 % Cq == 0) ? (float*)(wb + w.kbar) : nullptr;
  *kb = k;
  // one = 1 (the gamma the kernels read) and the key sums: the prep kernel with no dO rows
  hipLaunchKernelGGL(lsa_flash_prep_kernel, dim3(k ? B * kKeySlices : 1), dim3(256), 0, st, 0, C, *nch, nullptr,
                     nullptr, nullptr, nullptr, (float*)(wb + w.one), N, Cq, ldq, (const bf16_t*)qkv, k);
  return 0;
}

extern "C" int dfcsa_lsa_flash_bwd_bytes(int dtype, int B, int N, int C, int Cq, int ldq, int64_t* bytes) {
  if (!lsa_shape_ok(dtype, B, N, C, Cq, ldq) || !bytes) return DFCSA_EINVAL;
  *bytes = (int64_t)lsa_work(dtype, B, N, C, Cq, ldq).total;
  return 0;
}

extern "C" int dfcsa_lsa_flash_bwd(int dtype, int B, int N, int C, int Cq, int ldq, const void* qkv, const float* dO,
                                   const float* o, const float* lse, void* dqkv, void* work, int64_t work_bytes,
                                   void* stream) {
  if (!lsa_shape_ok(dtype, B, N, C, Cq, ldq) || !qkv || !dO || !o || !lse || !dqkv || !work) return DFCSA_EINVAL;
  const LsaWork w = lsa_work(dtype, B, N, C, Cq, ldq);
  if (work_bytes < (int64_t)w.total || ((uintptr_t)work & 15)) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  ProfScope prof(DFCSA_PROF_ATTN, st, 4.0 * B * (double)N * N * (Cq + C));
  char* wb = (char*)work;
  float* one = (float*)(wb + w.one);
  float* r = (float*)(wb + w.r);
  const int rows = B * N;
  const bool bf = dtype == DFCSA_DT_BF16;
  bf16_t* dO16 = bf ? (bf16_t*)(wb + w.dO16) : nullptr;
  const int nch = (bf && !mfma_bwd_ok(dtype, C, Cq, ldq)) ? C / kWideChunk : 1;
  // the key sums of the centred dQ (bf16, knob 48; knob 0 leaves dQ uncentred) ride on the prep launch
  float* kb = (bf && g_lsa_key_centre && 256 % Cq == 0) ? (float*)(wb + w.kbar) : nullptr;
  hipLaunchKernelGGL(lsa_flash_prep_kernel, dim3((rows + 3) / 4 + (kb ? B * kKeySlices : 0)), dim3(256), 0, st, rows,
                     C, nch, dO, o, r, dO16, one, N, Cq, ldq, (const bf16_t*)qkv, kb);
  DFCSA_CHECK_LAUNCH();
  if (!bf) {
    dim3 grid((N + 3) / 4, B);
    const size_t shm = (size_t)4 * (Cq + C) * sizeof(float);
    hipLaunchKernelGGL(fra_bwd_dq_generic<float>, grid, dim3(256), shm, st, N, C, Cq, ldq, (const float*)qkv, dO, one,
                       lse, r, (float*)dqkv);
    hipLaunchKernelGGL(fra_bwd_dkv_generic<float>, grid, dim3(256), shm, st, N, C, Cq, ldq, (const float*)qkv, dO,
                       one, lse, r, (float*)dqkv);
    DFCSA_CHECK_LAUNCH();
    return 0;
  }
  lsa_flash_bwd_core(B, N, C, Cq, ldq, qkv, lse, dqkv, work, kb, st);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_bf16_to_f32(int64_t n, const void* src, float* dst, void* stream) {
  if (n <= 0 || n % 8 || !src || !dst || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15)) return DFCSA_EINVAL;
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(lsa_flash_widen_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n8,
                     (const bf16_t*)src, dst);
  DFCSA_CHECK_LAUNCH();
  return 0;
}
