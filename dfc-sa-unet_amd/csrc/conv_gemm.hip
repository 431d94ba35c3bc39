// Implicit-GEMM convolution on MFMA, NHWC, for gfx950.
//
//   C[m][n] = sum_k A[m][k] * Bw[n][k]   (+ bias[n]),  fp32 accumulation
//
// m enumerates output pixels (b, oh, ow) of an Ho x Wo grid; k enumerates (segment, channel)
// with segment s = (source tensor, spatial shift dh/dw) and channel c in [0, Cseg):
//   A[m][s*Cseg + c] = src_s[b, oh*stride + dh_s, ow*stride + dw_s, c]   (0 outside the image)
// This one formulation covers every convolution of the training step:
//   * 3x3 conv forward: 9 taps x (1 or 2 concatenated sources)  -> the skip concat is never
//     materialised (reference models/unet_dfc_sa_res.py:182/188/194/200 torch.cat);
//   * 1x1 convs over [local, attn] and [fused, local, attn] (reference :102, :109 cat);
//   * 3x3 dgrad (shifts 1-kh, 1-kw) plus the 1x1 dgrads of the same input in ONE GEMM;
//   * ConvTranspose2d(k2,s2) forward (epilogue pixel-shuffle) and its dgrad (stride-2 gather).
// Epilogue: bias, optional accumulate into the destination, split of the N columns over up to
// three destination tensors, and per-column partial sums (sum, sum of squares) of the fp32
// accumulator for the following train-mode BatchNorm (one slab row per M tile: deterministic).
//
// Tiling: BM x BN workgroup tile, WM x WN waves (wave64), 128-byte K-stage (64 bf16 / 32 f32),
// register-staged double-buffered LDS with an XOR swizzle that makes the ds_read_b128 fragment
// reads conflict-free; mfma_f32_16x16x32_bf16 (bf16) or 8 x mfma_f32_16x16x4f32 (f32 parity
// mode; exact f32 FMA chain).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "dfcsa_internal.h"
#include "small_gemm.h"

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <typename T> struct Frag;
template <> struct Frag<bf16_t> { bf16x8_t v; };
template <> struct Frag<float> { float v[8]; };

__device__ __forceinline__ int swz(int r, int c) { return (c ^ ((r >> 1) & 7)); }

template <typename T>
__device__ __forceinline__ void read_frag(const char* lds_tile, int row, int g, int lane, Frag<T>& f);

// 8 consecutive k at element offset 32*g + 8*(lane>>4) of row `row` (128-byte swizzled rows).
template <>
__device__ __forceinline__ void read_frag<bf16_t>(const char* t, int row, int g, int lane, Frag<bf16_t>& f) {
  int chunk = 4 * g + (lane >> 4);
  f.v = *(const bf16x8_t*)(t + row * 128 + swz(row, chunk) * 16);
}
template <>
__device__ __forceinline__ void read_frag<float>(const char* t, int row, int g, int lane, Frag<float>& f) {
  int chunk = 8 * g + 2 * (lane >> 4);
  float4 a = *(const float4*)(t + row * 128 + swz(row, chunk) * 16);
  float4 b = *(const float4*)(t + row * 128 + swz(row, chunk + 1) * 16);
  f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w;
  f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
}

__device__ __forceinline__ void mma(f32x4_t& acc, const Frag<bf16_t>& a, const Frag<bf16_t>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
}
__device__ __forceinline__ void mma(f32x4_t& acc, const Frag<float>& a, const Frag<float>& b) {
#pragma unroll
  for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[s], b.v[s], acc, 0, 0, 0);
}

// BatchNorm finalisation in a producer's tail (dfcsa_conv_gemm_bn).  Every workgroup has just written
// (write-through) its statistics row `row` of [T][2][N] for the columns of its column block cb (the
// launch's N tile, cw columns).  Level 1: the workgroups of row group g (GS consecutive rows) take
// ticket (cb, g); the last one sums the group's rows per column in a fixed order (P = NT / cw parts of
// rows p, p + P, ..., combined in part order; fp64) and hands the two sums over (write-through).
// Level 2: the level-1 finishers take ticket cb; the last one sums the ng group sums in the same
// fixed order and finalises the block's channels (< f.C) exactly as bn_finalize_kernel (training):
// scale / shift / mean / invstd, running statistics with the unbiased variance, num_batches_tracked
// (block 0).  Deterministic; no separate finalize launch.
template <int NT, int CW>
__device__ void bn_fold_tail(const BnFold& f, const float* stats, int N, int row, int T, int n0, char* smem) {
  static_assert(CW <= NT, "fold: at most one column per thread");
  constexpr int P = NT / CW;   // parts (threads past P * CW idle)
  const int cb = n0 / CW;
  if (n0 >= f.C) return;   // columns past the BatchNorm's channels (e.g. a fused residual conv)
  double* red = (double*)smem;            // [2][NT]
  int* flag = (int*)(red + 2 * NT);
  __syncthreads();                        // smem is reused (the output tile staging is done)
  const int g = row / f.GS, g0 = g * f.GS, g1 = min(T, g0 + f.GS);
  if (!wg_last_of(f.cnt + cb * f.ng + g, (unsigned)(g1 - g0), flag)) return;
  const int cl = threadIdx.x % CW, part = threadIdx.x / CW, c = n0 + cl;
  const bool live = c < f.C && part < P;
  double s0 = 0.0, s1 = 0.0;
  if (live) {
    int r = g0 + part;
    for (; r + 3 * P < g1; r += 4 * P) {
      const float* pp[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pp[2 * j] = stats + (size_t)(r + j * P) * 2 * N + c;
        pp[2 * j + 1] = pp[2 * j] + N;
      }
      float v[8];
      ld_sc1_f8(pp, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) { s0 += (double)v[2 * j]; s1 += (double)v[2 * j + 1]; }
    }
    for (; r < g1; r += P) {
      s0 += (double)ld_sc1_f(stats + (size_t)r * 2 * N + c);
      s1 += (double)ld_sc1_f(stats + (size_t)r * 2 * N + N + c);
    }
  }
  red[threadIdx.x] = s0;
  red[NT + threadIdx.x] = s1;
  __syncthreads();
  double* slot = f.scr + ((size_t)(cb * f.ng + g) * 2) * CW;
  if (part == 0 && live) {
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int q = 0; q < P; ++q) { a0 += red[q * CW + cl]; a1 += red[NT + q * CW + cl]; }
    st_sc1_d(slot + cl, a0);
    st_sc1_d(slot + CW + cl, a1);
  }
  if (!wg_last_of(f.cnt + f.ncb * f.ng + cb, (unsigned)f.ng, flag)) return;
  s0 = s1 = 0.0;
  if (live) {
    const double* base = f.scr + (size_t)cb * f.ng * 2 * CW + cl;
    int gg = part;
    for (; gg + 3 * P < f.ng; gg += 4 * P) {
      const double* pp[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pp[2 * j] = base + (size_t)(gg + j * P) * 2 * CW;
        pp[2 * j + 1] = pp[2 * j] + CW;
      }
      double v[8];
      ld_sc1_d8(pp, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) { s0 += v[2 * j]; s1 += v[2 * j + 1]; }
    }
    for (; gg < f.ng; gg += P) {
      double v0, v1, v2;
      const double* q = base + (size_t)gg * 2 * CW;
      ld_sc1_d3(q, q + CW, q, v0, v1, v2);
      s0 += v0;
      s1 += v1;
    }
  }
  __syncthreads();
  red[threadIdx.x] = s0;
  red[NT + threadIdx.x] = s1;
  __syncthreads();
  if (part == 0 && live) {
    double t0 = 0.0, t1 = 0.0;
#pragma unroll
    for (int q = 0; q < P; ++q) { t0 += red[q * CW + cl]; t1 += red[NT + q * CW + cl]; }
    const double n = (double)f.count;
    const double ma = t0 / n;
    double v = t1 / n - ma * ma;
    if (v < 0.0) v = 0.0;
    const double b = f.bias ? (double)f.bias[c] : 0.0;
    const float mu = (float)(ma + b), istd = (float)(1.0 / sqrt(v + (double)f.eps));
    const double unb = f.count > 1 ? v * n / (n - 1.0) : v;
    f.rmean[c] = (1.f - f.momentum) * f.rmean[c] + f.momentum * mu;
    f.rvar[c] = (float)((1.0 - f.momentum) * (double)f.rvar[c] + f.momentum * unb);
    const float sc = f.gamma[c] * istd;
    f.scale[c] = sc;
    f.shift[c] = f.beta[c] - mu * sc;
    f.mean[c] = mu;
    f.invstd[c] = istd;
  }
  if (cb == 0 && threadIdx.x == 0 && f.nbt) *f.nbt += 1;
}

// Shared epilogue: BN partial statistics of the fp32 accumulator, bias, conversion, LDS-staged
// coalesced 16-byte stores (plain / 3-way column split / ConvTranspose pixel shuffle), optional
// accumulate into the destination.  smem must hold max(2*WM*BN floats, BM*(BN*sizeof(T)+16)) B.
template <typename T, int BM, int BN, int WM, int WN>
__device__ __forceinline__ void conv_epilogue(const ConvGemmArgs& args, f32x4_t (&acc)[BM / WM / 16][BN / WN / 16],
                                              char* smem, int m0, int n0, int m_tile, int tid, int lane, int wm,
                                              int wn) {
  constexpr int NT = WM * WN * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int OSTR = BN * (int)sizeof(T) + 16;
  const int M = args.M, N = args.N;
  // (1) BatchNorm partial statistics of the raw accumulator, per column, rows m < M only, ONE
  //     slab row per M tile (dfcsa_conv_stats_rows = ceil(M / BM)): the finalize reads BM/64 x
  //     fewer rows.
  constexpr int SUBW = WTM >= 64 ? WTM / 64 : 1;   // sub-tiles covered by one wave
  constexpr int SUBS = BM / 64;                    // sub-tiles of the workgroup tile
  float* red = (float*)smem;                       // [WM][SUBW][2][BN] after the main loop
  if (args.stats) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float s[SUBW], q[SUBW];
#pragma unroll
      for (int u = 0; u < SUBW; ++u) { s[u] = 0.f; q[u] = 0.f; }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
          const float v = (m < M) ? acc[i][j][r] : 0.f;
          constexpr int dummy = 0;
          const int u = SUBW > 1 ? (i * 16) / 64 : dummy;
          s[u] += v;
          q[u] += v * v;
        }
#pragma unroll
      for (int u = 0; u < SUBW; ++u) {
        float a = s[u], b = q[u];
        a += __shfl_xor(a, 16, 64); a += __shfl_xor(a, 32, 64);
        b += __shfl_xor(b, 16, 64); b += __shfl_xor(b, 32, 64);
        if (lane < 16) {
          const int col = wn * WTN + j * 16 + lane;
          red[((wm * SUBW + u) * 2 + 0) * BN + col] = a;
          red[((wm * SUBW + u) * 2 + 1) * BN + col] = b;
        }
      }
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      const int n = n0 + c;
      if (n >= N) continue;
      float sm = 0.f, q = 0.f;
      for (int st = 0; st < SUBS; ++st) {    // sub-tiles in order (fixed summation order)
        if (WTM >= 64) {
          const int w = (st * 64) / WTM, u = st - w * SUBW;
          sm += red[((w * SUBW + u) * 2) * BN + c];
          q += red[((w * SUBW + u) * 2 + 1) * BN + c];
        } else {
          for (int w = 0; w < WM; ++w)
            if ((w * WTM) / 64 == st) { sm += red[(w * 2) * BN + c]; q += red[(w * 2 + 1) * BN + c]; }
        }
      }
      if (args.fold.on) {   // the fold's last workgroups read these rows (write-through)
        st_sc1_dw(args.stats + (size_t)m_tile * 2 * N + n, sm);
        st_sc1_dw(args.stats + (size_t)m_tile * 2 * N + N + n, q);
      } else {
        args.stats[(size_t)m_tile * 2 * N + n] = sm;
        args.stats[(size_t)m_tile * 2 * N + N + n] = q;
      }
    }
    __syncthreads();
  }

  // (2) bias, convert, stage the tile through LDS, coalesced 16-B stores.
  T* otile = (T*)smem;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    int col = wn * WTN + j * 16 + (lane & 15);
    int n = n0 + col;
    float bv = (args.bias && n < N) ? args.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = wm * WTM + i * 16 + (lane >> 4) * 4 + r;
        *(T*)((char*)otile + row * OSTR + col * sizeof(T)) = ElemTraits<T>::from_f(acc[i][j][r] + bv);
      }
  }
  __syncthreads();
  constexpr int OCH = BN / 8;                      // 8-element chunks per tile row
  for (int e = tid; e < BM * OCH; e += NT) {
    int row = e / OCH, cc = e % OCH;
    int m = m0 + row, n = n0 + cc * 8;
    if (m >= M || n >= N) continue;
    const T* src = (const T*)((const char*)otile + row * OSTR + cc * 8 * sizeof(T));
    if (sizeof(T) == 2 && !args.accumulate && args.mode == CONV_STORE_PLAIN) {
      // the staged bf16 values are the output: a 16-B copy (no unpack / repack)
      const int d = n / args.Nd, col = n - d * args.Nd;
      *(uint4*)((T*)args.dest[d] + ((size_t)m * args.Nd + col)) = *(const uint4*)src;
      continue;
    }
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = ElemTraits<T>::to_f(src[q]);
    T* dst;
    if (args.mode == CONV_STORE_SHUFFLE2) {
      // ConvTranspose2d(k=2, s=2): column n = (i*2 + j) * Cout + co  ->  pixel (2oh+i, 2ow+j)
      int ij = n / args.Nd, co = n - ij * args.Nd;
      int b = dm_div(args.dm_hw, m);
      int rem = m - b * args.dm_hw.d;
      int oh = dm_div(args.dm_w, rem);
      int ow = rem - oh * args.dm_w.d;
      int y = 2 * oh + (ij >> 1), x = 2 * ow + (ij & 1);
      dst = (T*)args.dest[0] + ((size_t)((b * args.Hout + y) * args.Wout + x) * args.Nd + co);
    } else {
      int d = n / args.Nd, col = n - d * args.Nd;
      dst = (T*)args.dest[d] + ((size_t)m * args.Nd + col);
    }
    if (args.accumulate) {
      float o[8];
      load8<T>(dst, o);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += o[q];
    }
    store8<T>(dst, v);
  }
  static_assert(BN <= NT, "the BatchNorm fold gives each column of the tile a thread");
  if (args.fold.on && args.stats) bn_fold_tail<NT, BN>(args.fold, args.stats, N, m_tile, (M + BM - 1) / BM, n0, smem);
}

template <typename T, int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(WM* WN * 64)
conv_gemm_kernel(const ConvGemmArgs args) {
  constexpr int NT = WM * WN * 64;
  constexpr int EPC = ElemTraits<T>::kChunk;     // elements per 16-B chunk
  constexpr int KST = 128 / sizeof(T);           // elements per K stage
  constexpr int NG = KST / 32;                   // 32-wide k groups per stage
  constexpr int A_CH = BM * 8 / NT;              // A chunks per thread per stage
  constexpr int B_CH = BN * 8 / NT;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  static_assert(A_CH >= 1 && B_CH >= 1, "tile too small for thread count");

  constexpr int OSTR = BN * (int)sizeof(T) + 16;  // padded output-tile row stride (bytes)
  constexpr int SMEM_MAIN = 2 * (BM + BN) * 128, SMEM_OUT = BM * OSTR;
  __shared__ __attribute__((aligned(16))) char smem[SMEM_MAIN > SMEM_OUT ? SMEM_MAIN : SMEM_OUT];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int n_tile = blockIdx.x, m_tile = blockIdx.y;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int M = args.M, N = args.N;

  // ---- per-thread A row info (rows fixed over the K loop) ----
  const int cchunk = tid & 7;                  // chunk column handled by this thread
  int a_b[A_CH], a_oh[A_CH], a_ow[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    int r = (tid >> 3) + i * (NT / 8);
    int m = m0 + r;
    if (m < M) {
      int b = dm_div(args.dm_hw, m);
      int rem = m - b * args.dm_hw.d;
      int oh = dm_div(args.dm_w, rem);
      a_b[i] = b;
      a_oh[i] = oh * args.stride;
      a_ow[i] = (rem - oh * args.dm_w.d) * args.stride;
    } else {
      a_b[i] = -1; a_oh[i] = 0; a_ow[i] = 0;
    }
  }

  const int nk = args.Kpad / KST;
  uint4 ra[A_CH], rb[B_CH];

  auto load_stage = [&](int kt) {
    const int kbase = kt * KST + cchunk * EPC;
    // A: implicit im2col gather
    int seg = dm_div(args.dm_cseg, kbase);
    int ch = kbase - seg * args.Cseg;
    bool kvalid = kbase < args.K;
    const ConvSeg sg = args.seg[kvalid ? seg : 0];
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      int ih = a_oh[i] + sg.dh, iw = a_ow[i] + sg.dw;
      bool ok = kvalid && a_b[i] >= 0 && ih >= 0 && ih < args.Hi && iw >= 0 && iw < args.Wi;
      if (ok) {
        const T* p = (const T*)sg.ptr + ((size_t)((a_b[i] * args.Hi + ih) * args.Wi + iw) * args.Cseg + ch);
        ra[i] = *(const uint4*)p;
      } else {
        ra[i] = make_uint4(0, 0, 0, 0);
      }
    }
    // B: packed weights [N][Kpad]
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      int r = (tid >> 3) + i * (NT / 8);
      int n = n0 + r;
      if (n < N) {
        const T* p = (const T*)args.Bw + ((size_t)n * args.Kpad + kbase);
        rb[i] = *(const uint4*)p;
      } else {
        rb[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_stage = [&](int s) {
    char* A = smem + s * (BM + BN) * 128;
    char* B = A + BM * 128;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      int r = (tid >> 3) + i * (NT / 8);
      *(uint4*)(A + r * 128 + swz(r, cchunk) * 16) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      int r = (tid >> 3) + i * (NT / 8);
      *(uint4*)(B + r * 128 + swz(r, cchunk) * 16) = rb[i];
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};

  load_stage(0);
  store_stage(0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) load_stage(kt + 1);
    const char* A = smem + (kt & 1) * (BM + BN) * 128;
    const char* B = A + BM * 128;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      Frag<T> fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) read_frag<T>(A, wm * WTM + i * 16 + (lane & 15), g, lane, fa[i]);
#pragma unroll
      for (int j = 0; j < FN; ++j) read_frag<T>(B, wn * WTN + j * 16 + (lane & 15), g, lane, fb[j]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) mma(acc[i][j], fa[i], fb[j]);
    }
    if (more) store_stage((kt + 1) & 1);
    __syncthreads();
  }

  conv_epilogue<T, BM, BN, WM, WN>(args, acc, smem, m0, n0, m_tile, tid, lane, wm, wn);
}


// --------------------------------------------------------------------------------------------
// bf16 hot path: operands staged by LDS-DMA (buffer_load_dwordx4 ... lds through a raw buffer
// descriptor, blds16 below).  Each wave-instruction fills one 8-row x 128-B block of the K-stage
// image; the XOR swizzle is applied on the SOURCE side (lane -> which 16-B chunk of its row it
// fetches), so the fragment reads are the same conflict-free ds_read_b128 as the register-staged
// kernel.  Zero padding (image border, N tail) is an out-of-range lane offset, which reads zeros,
// so every LDS slot is written each stage; the stage's tap shift and K offset are scalar (the
// descriptor base / soffset), leaving ~2 VALU per DMA (round 2's 64-bit addresses and zero-page
// selects cost ~8).  Two LDS buffers; one vmcnt(0) + barrier per 64-deep K stage.
// --------------------------------------------------------------------------------------------
__device__ __attribute__((aligned(16))) uint4 g_zero_page[64];
// dfcsa_conv_stats_rows: the launch functions report the statistics rows of the kernel they would
// launch instead of launching (one row per M tile / per persistent workgroup)
thread_local int* t_dry_rows = nullptr;
// dry run (desc_args): the column-block width of the picked kernel when its epilogue can fold the
// BatchNorm finalisation (conv_epilogue kernels), 0 otherwise
thread_local int* t_dry_bn = nullptr;
__device__ __attribute__((aligned(16))) float g_store_sink[4 * 64];   // write-only target of masked stores

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void glb_void;

__device__ __forceinline__ void glds16(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)lds_base, 16, 0, 0);
}

// LDS-DMA through a raw buffer descriptor (buffer_load_dwordx4 ... offen lds): the base is scalar
// (SGPRs), the lane supplies a 32-bit byte offset, and an offset >= num_records reads zeros -- the
// zero padding of image borders and N tails costs one bit-select per lane instead of a 64-bit
// address and two selects against a zero page.  Sources must stay below 2 GiB (host-checked).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr unsigned kBufOOB = 0x80000000u;        // any offset >= 2^31 is out of range
__device__ __forceinline__ rsrc_t buf_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void blds16(rsrc_t r, unsigned voff, unsigned soff, char* lds_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds_base, 16, (int)voff, (int)soff, 0, 0);
}
// voff if bit `bit` of mask is set, else out of range (v_bfe_i32 + v_bfi_b32)
__device__ __forceinline__ unsigned sel_oob(unsigned mask, int bit, unsigned voff) {
  const unsigned m = (unsigned)__builtin_amdgcn_sbfe((int)mask, bit, 1);
  return (voff & m) | (kBufOOB & ~m);
}

template <int BM, int BN, int WM, int WN, int NST, bool SPLIT = false>
__global__ void __launch_bounds__(WM* WN * 64)
conv_gemm_glds_kernel(const ConvGemmArgs args) {
  using T = bf16_t;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int A_IN = BM / (8 * NW), B_IN = BN / (8 * NW);
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int OSTR = BN * (int)sizeof(T) + 16;
  constexpr int SMEM = (NST * STAGE > BM * OSTR) ? NST * STAGE : BM * OSTR;
  constexpr int OPS = A_IN + B_IN;  // LDS-DMA instructions per wave per stage
  static_assert(NW % 2 == 0 && A_IN >= 1 && B_IN >= 1, "glds tiling");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nN = (args.N + BN - 1) / BN;
  const int ntiles = nN * ((args.M + BM - 1) / BM);
  const int L0 = xcd_remap(blockIdx.x, SPLIT ? ntiles * args.ksplit : ntiles);
  if (L0 < 0) return;
  // split-K: consecutive workgroups take the splits of one tile (the same XCD's L2 holds its A rows)
  const int split = SPLIT ? L0 % args.ksplit : 0;
  const int L = SPLIT ? L0 / args.ksplit : L0;
  const int n_tile = L % nN, m_tile = L / nN;  // the N tiles of one M tile share an XCD
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int M = args.M, N = args.N;
  // 16-B chunk this lane fetches within its 128-B row (source-side swizzle)
  const int cchunk = (lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7);
  const int rsub = lane >> 3;

  // Address generation is kept scalar wherever it can be: Cseg % 64 == 0 (host-checked), so a
  // 64-wide K stage lies inside ONE segment -> segment pointer, shift and channel base are
  // wave-uniform (SGPR, loaded from the kernel arguments); per lane only the row offset, the
  // chunk and a 9-bit "tap in bounds" mask (bit (dh+1)*3 + dw+1) remain.
  const int wv = __builtin_amdgcn_readfirstlane(wave);  // wave index as a scalar (M0 bases)
  const int lane_ch = cchunk * 8;
  // per lane: byte offset of its pixel row (+ chunk) in a source, and the 9-bit tap mask; the
  // stage's shift and channel base go into the (scalar) buffer base
  unsigned a_off[A_IN], a_tap[A_IN];
#pragma unroll
  for (int i = 0; i < A_IN; ++i) {
    const int m = m0 + (i * NW + wave) * 8 + rsub;
    a_off[i] = 0;
    a_tap[i] = 0;
    if (m < M) {
      const int b = dm_div(args.dm_hw, m);
      const int rem = m - b * args.dm_hw.d;
      const int oh = dm_div(args.dm_w, rem);
      const int ow = rem - oh * args.dm_w.d;
      const int ih = oh * args.stride, iw = ow * args.stride;
      a_off[i] = 2u * (unsigned)(((b * args.Hi + ih) * args.Wi + iw) * args.Cseg + lane_ch);
      unsigned t = 0;
#pragma unroll
      for (int dh = -1; dh <= 1; ++dh)
#pragma unroll
        for (int dw = -1; dw <= 1; ++dw)
          t |= (unsigned)(ih + dh >= 0 && ih + dh < args.Hi && iw + dw >= 0 && iw + dw < args.Wi) << ((dh + 1) * 3 + dw + 1);
      a_tap[i] = t;
    }
  }
  // B rows: byte offset of the lane's row + chunk at K = 0 (out of range for rows >= N); the
  // stage's K offset is the scalar soffset
  unsigned b_off[B_IN];
#pragma unroll
  for (int i = 0; i < B_IN; ++i) {
    const int n = n0 + (i * NW + wave) * 8 + rsub;
    b_off[i] = n < N ? 2u * (unsigned)(n * args.Kpad + lane_ch) : kBufOOB;
  }
  const rsrc_t rb = buf_rsrc(args.Bw);

  auto issue = [&](int kt, int buf) {
    char* A = smem + buf * STAGE;
    char* B = A + BM * 128;
    const int k0 = kt * 64;                               // uniform
    const int seg = dm_div(args.dm_cseg, k0);
    const int ch0 = k0 - seg * args.Cseg;
    const ConvSeg sg = args.seg[seg];                     // uniform index: scalar load
    const int delta = (sg.dh * args.Wi + sg.dw) * args.Cseg + ch0;
    const int tb = (sg.dh + 1) * 3 + sg.dw + 1;
    const rsrc_t ra = buf_rsrc((const T*)sg.ptr + delta);
#pragma unroll
    for (int i = 0; i < A_IN; ++i) blds16(ra, sel_oob(a_tap[i], tb, a_off[i]), 0, A + (i * NW + wv) * 8 * 128);
#pragma unroll
    for (int i = 0; i < B_IN; ++i) blds16(rb, b_off[i], (unsigned)kt * 128u, B + (i * NW + wv) * 8 * 128);
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};

  // NST-deep ring: stages kt+1 .. kt+NST-2 stay in flight while stage kt is multiplied; the
  // only vector-memory ops in the loop are the DMAs, so a counted vmcnt isolates stage kt.
  // (split-K: this workgroup's stages kb .. kb + nk - 1 of the K range; ring slots by local index)
  const int kb = SPLIT ? split * args.kper : 0;
  const int nk = SPLIT ? min(args.kper, args.Kpad / 64 - kb) : args.Kpad / 64;
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(kb + s, s);
  for (int kt = 0; kt < nk; ++kt) {
    const int after = min(NST - 2, nk - 1 - kt);
    if constexpr (NST >= 4) {
      if (after >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * OPS) : "memory");
      else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (NST == 3) {
      if (after >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();   // the DMA ring stays in flight (a __syncthreads fence would drain it)
    if (kt + NST - 1 < nk) issue(kb + kt + NST - 1, (kt + NST - 1) % NST);
    const char* A = smem + (kt % NST) * STAGE;
    const char* B = A + BM * 128;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      Frag<T> fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) read_frag<T>(A, wm * WTM + i * 16 + (lane & 15), g, lane, fa[i]);
#pragma unroll
      for (int j = 0; j < FN; ++j) read_frag<T>(B, wn * WTN + j * 16 + (lane & 15), g, lane, fb[j]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) mma(acc[i][j], fa[i], fb[j]);
    }
  }
  if constexpr (SPLIT) {
    // partial tile in the accumulator's own layout: [tile][split][wave][fragment][lane][4]
    float* out = args.kwork + (((size_t)L * args.ksplit + split) * NW + wave) * (FM * FN * 256) + lane * 4;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) *(f32x4_t*)(out + (i * FN + j) * 256) = acc[i][j];
    return;
  }
  __syncthreads();
  conv_epilogue<T, BM, BN, WM, WN>(args, acc, smem, m0, n0, m_tile, tid, lane, wm, wn);
}

// split-K epilogue launch: one workgroup per output tile sums the tile's ksplit partials in split
// order (each lane its own accumulator fragments: 16-B loads, coalesced per wave) and runs the
// tile kernel's epilogue (BN statistics row, bias, bf16 store) on the sum
template <int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(WM* WN * 64) conv_splitk_epi_kernel(const ConvGemmArgs args) {
  using T = bf16_t;
  constexpr int NW = WM * WN;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  constexpr int OSTR = BN * (int)sizeof(T) + 16;
  __shared__ __attribute__((aligned(16))) char smem[BM * OSTR > 2 * WM * BN * 4 ? BM * OSTR : 2 * WM * BN * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nN = (args.N + BN - 1) / BN;
  const int L = xcd_remap(blockIdx.x, nN * ((args.M + BM - 1) / BM));
  if (L < 0) return;
  const int n_tile = L % nN, m_tile = L / nN;
  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};
  const float* base = args.kwork + ((size_t)L * args.ksplit * NW + wave) * (FM * FN * 256) + lane * 4;
  for (int s = 0; s < args.ksplit; ++s) {
    const float* p = base + (size_t)s * NW * (FM * FN * 256);
    f32x4_t v[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) v[i][j] = *(const f32x4_t*)(p + (i * FN + j) * 256);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] += v[i][j];
  }
  conv_epilogue<T, BM, BN, WM, WN>(args, acc, smem, m_tile * BM, n_tile * BN, m_tile, tid, lane, wm, wn);
}

// --------------------------------------------------------------------------------------------
// Same tile kernel with 32-deep K slots in a deeper ring (NST slots of (BM + BN) x 64 B): at
// 128x128 four slots take the LDS of two 64-deep stages, so two workgroups still share a CU, but
// each slot's DMA is issued NST - 1 slots (not one stage) ahead of its use -- the round-3
// counters put the 64-deep kernel's waves 52 % in waits with one stage of MFMAs (~210 ns) to
// cover an L2 fetch.  Slot image: 64-B rows (4 chunks of 16 B), 16 rows per 1-KB DMA; physical
// chunk = logical ^ f(row) with f = {0, 2, 3, 1}[(row >> 2) & 3], which makes the fragment
// reads (lane -> row lane & 15, logical chunk lane >> 4) conflict-free in every ds_read_b128
// lane group; the DMA applies it on the source side as the 64-deep kernel does.
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ int swz32(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

template <int BM, int BN, int WM, int WN, int NST>
__global__ void __launch_bounds__(WM* WN * 64)
conv_gemm_glds32_kernel(const ConvGemmArgs args) {
  using T = bf16_t;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int A_IN = BM / (16 * NW), B_IN = BN / (16 * NW);
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int STAGE = (BM + BN) * 64;
  constexpr int OSTR = BN * (int)sizeof(T) + 16;
  constexpr int SMEM = (NST * STAGE > BM * OSTR) ? NST * STAGE : BM * OSTR;
  constexpr int OPS = A_IN + B_IN;
  static_assert(A_IN >= 1 && B_IN >= 1 && NST >= 2 && NST <= 6, "glds32 tiling");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nN = (args.N + BN - 1) / BN;
  const int L = xcd_remap(blockIdx.x, nN * ((args.M + BM - 1) / BM));
  if (L < 0) return;
  const int n_tile = L % nN, m_tile = L / nN;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int M = args.M, N = args.N;
  // DMA: lane -> row (lane >> 2) of a 16-row block, physical chunk lane & 3
  const int rsub = lane >> 2;
  const int cchunk = (lane & 3) ^ swz32(rsub);
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int lane_ch = cchunk * 8;
  unsigned a_off[A_IN], a_tap[A_IN];
#pragma unroll
  for (int i = 0; i < A_IN; ++i) {
    const int m = m0 + (i * NW + wave) * 16 + rsub;
    a_off[i] = 0;
    a_tap[i] = 0;
    if (m < M) {
      const int b = dm_div(args.dm_hw, m);
      const int rem = m - b * args.dm_hw.d;
      const int oh = dm_div(args.dm_w, rem);
      const int ow = rem - oh * args.dm_w.d;
      const int ih = oh * args.stride, iw = ow * args.stride;
      a_off[i] = 2u * (unsigned)(((b * args.Hi + ih) * args.Wi + iw) * args.Cseg + lane_ch);
      unsigned t = 0;
#pragma unroll
      for (int dh = -1; dh <= 1; ++dh)
#pragma unroll
        for (int dw = -1; dw <= 1; ++dw)
          t |= (unsigned)(ih + dh >= 0 && ih + dh < args.Hi && iw + dw >= 0 && iw + dw < args.Wi) << ((dh + 1) * 3 + dw + 1);
      a_tap[i] = t;
    }
  }
  unsigned b_off[B_IN];
#pragma unroll
  for (int i = 0; i < B_IN; ++i) {
    const int n = n0 + (i * NW + wave) * 16 + rsub;
    b_off[i] = n < N ? 2u * (unsigned)(n * args.Kpad + lane_ch) : kBufOOB;
  }
  const rsrc_t rb = buf_rsrc(args.Bw);

  auto issue = [&](int kt, int buf) {
    char* A = smem + buf * STAGE;
    char* B = A + BM * 64;
    const int k0 = kt * 32;
    const int seg = dm_div(args.dm_cseg, k0);
    const int ch0 = k0 - seg * args.Cseg;
    const ConvSeg sg = args.seg[seg];
    const int delta = (sg.dh * args.Wi + sg.dw) * args.Cseg + ch0;
    const int tb = (sg.dh + 1) * 3 + sg.dw + 1;
    const rsrc_t ra = buf_rsrc((const T*)sg.ptr + delta);
#pragma unroll
    for (int i = 0; i < A_IN; ++i) blds16(ra, sel_oob(a_tap[i], tb, a_off[i]), 0, A + (i * NW + wv) * 1024);
#pragma unroll
    for (int i = 0; i < B_IN; ++i) blds16(rb, b_off[i], (unsigned)kt * 64u, B + (i * NW + wv) * 1024);
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (bytes within a slot image): row (lane & 15) + 16 i, logical chunk lane >> 4
  const int frow = lane & 15;
  const int fch = ((lane >> 4) ^ swz32(frow)) * 16;
  const int nk = args.Kpad / 32;
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    const int after = min(NST - 2, nk - 1 - kt);   // slots still allowed in flight
    switch (after) {
      case 4: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * OPS) : "memory"); break;
      case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * OPS) : "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * OPS) : "memory"); break;
      case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS) : "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
    lds_barrier();
    if (kt + NST - 1 < nk) issue(kt + NST - 1, (kt + NST - 1) % NST);
    const char* A = smem + (kt % NST) * STAGE;
    const char* B = A + BM * 64;
    Frag<T> fa[FM], fb[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i].v = *(const bf16x8_t*)(A + (wm * WTM + i * 16 + frow) * 64 + fch);
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j].v = *(const bf16x8_t*)(B + (wn * WTN + j * 16 + frow) * 64 + fch);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) mma(acc[i][j], fa[i], fb[j]);
  }
  __syncthreads();
  conv_epilogue<T, BM, BN, WM, WN>(args, acc, smem, m0, n0, m_tile, tid, lane, wm, wn);
}

template <int BM, int BN, int WM, int WN, int NST>
int launch_glds32(const ConvGemmArgs& a, hipStream_t st) {
  if (t_dry_rows) { *t_dry_rows = (a.M + BM - 1) / BM; if (t_dry_bn) *t_dry_bn = BN; return 0; }
  dim3 grid(xcd_pad(((a.N + BN - 1) / BN) * ((a.M + BM - 1) / BM)));
  hipLaunchKernelGGL((conv_gemm_glds32_kernel<BM, BN, WM, WN, NST>), grid, dim3(WM * WN * 64), 0, st, a);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

thread_local int64_t* t_dry_work = nullptr;   // dfcsa_conv_work_floats: the split-K workspace

// split-K plan of a 128x128 tile launch: ksplit, kper (64-deep stages per split); 1 = no split.
// Few tiles (< 150: the 14^2 bottleneck dgrad) with a long K (>= 64 stages) get ~600 workgroups of
// >= 12 stages each.
int g_splitk = 1;   // knob 25: 0 = never split
int g_splitk_min_nk = 24;     // knob 37: fewest 64-deep K stages a split launch may have (ViT GEMMs, tools/vit_gemm_bench.py)
int g_splitk_target = 600;    // knob 38: workgroups a split launch aims for
void splitk_plan(const ConvGemmArgs& a, int* ksplit, int* kper) {
  *ksplit = 1;
  *kper = a.Kpad / 64;
  const int tiles = ((a.N + 127) / 128) * ((a.M + 127) / 128);
  const int nk = a.Kpad / 64;
  // measured (profiles/r03b_splitk.jsonl): the 14^2 3x3 dgrad (100 tiles, 176 stages) 93 -> 63 us;
  // at 200 tiles / 72 stages (the 14^2 forward) the 64x64 tile stays faster (50 vs 57 us)
  if (!g_splitk || tiles >= 150 || nk < g_splitk_min_nk) return;
  int s = (g_splitk_target + tiles - 1) / tiles;
  s = std::min(s, nk / 12);
  if (s < 2) return;
  int per = (nk + s - 1) / s;
  s = (nk + per - 1) / per;
  *ksplit = s;
  *kper = per;
}

int launch_splitk(ConvGemmArgs a, int ksplit, int kper, hipStream_t st) {
  const int tiles = ((a.N + 127) / 128) * ((a.M + 127) / 128);
  const int64_t need = (int64_t)tiles * ksplit * 128 * 128;
  if (t_dry_rows) { *t_dry_rows = (a.M + 127) / 128; if (t_dry_work) *t_dry_work = need; if (t_dry_bn) *t_dry_bn = 128; return 0; }
  if (!a.kwork || a.kwork_floats < need) return DFCSA_EINVAL;
  a.ksplit = ksplit;
  a.kper = kper;
  hipLaunchKernelGGL((conv_gemm_glds_kernel<128, 128, 4, 2, 2, true>), dim3(xcd_pad(tiles * ksplit)), dim3(512), 0,
                     st, a);
  DFCSA_CHECK_LAUNCH();
  hipLaunchKernelGGL((conv_splitk_epi_kernel<128, 128, 4, 2>), dim3(xcd_pad(tiles)), dim3(512), 0, st, a);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

template <int BM, int BN, int WM, int WN, int NST = 2>
int launch_glds(const ConvGemmArgs& a, hipStream_t st) {
  if (t_dry_rows) { *t_dry_rows = (a.M + BM - 1) / BM; if (t_dry_bn) *t_dry_bn = BN; return 0; }
  dim3 grid(xcd_pad(((a.N + BN - 1) / BN) * ((a.M + BM - 1) / BM)));
  hipLaunchKernelGGL((conv_gemm_glds_kernel<BM, BN, WM, WN, NST>), grid, dim3(WM * WN * 64), 0, st, a);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// --------------------------------------------------------------------------------------------
// 256x256 ping-pong kernel (deep 3x3 convs and dgrads with N % 256 == 0): ONE workgroup per CU,
// 8 waves as 2 (M) x 4 (N), each wave owning a 128x64 output (acc[8][4] of 16x16 fragments).
// The two wave rows (groups G0 = waves 0-3, G1 = waves 4-7; one wave of each per SIMD) run one
// barrier apart: while one group issues its fragment reads and LDS-DMA for a phase, the other
// runs that phase's 16 MFMAs at raised priority, so each SIMD's matrix pipe alternates between
// its two waves instead of draining at a shared barrier.
//
// A K-tile (64 deep) is staged as four 16-KB half-tiles, A0 A1 B0 B1: A half h holds, for both
// wave rows, the 64 output rows of M-quadrant h (tile rows wr*128 + h*64 + r); B half h the 32
// columns of N-quadrant h of every wave column (tile columns wc*64 + h*32 + c).  Four phases per
// K-tile compute the quadrants (0,0) (0,1) (1,1) (1,0) and read A0+B0, B1, A1 and nothing; each
// phase also prefetches one half-tile into a slot whose previous contents both groups have
// finished reading: B1 and A1 of K-tile t+1 in phases 1-2, A0 and B0 of K-tile t+2 in phases 3-4
// (A0/B0 of this buffer were read in phase 1), so every half is issued 5-6 phases before it is
// read.  Each half = 2 DMA instructions per wave; the counted vmcnt of each phase retires the
// half read in the next phase, and precedes a barrier that both groups pass before that read
// (G0 reads after its second barrier of the phase, G1 one barrier later).
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Stream-K work decomposition (SK = true; round 5): the launch has G <= 256 workgroups (one per CU)
// and workgroup g walks iterations [g I / G, (g + 1) I / G) of the tile-major space of I = tiles x nk
// 64-deep K-tiles, so every CU does the same number of K-tiles whatever the tile count (the 28^2 /
// 56^2 grids of 98 / 196 / 392 tiles leave a quarter or more of a wave idle as whole tiles).  A
// segment that covers a whole tile runs the epilogue directly.  Otherwise the workgroup publishes
// its fp32 partial tile (write-through, accumulator fragment order) into its slot (two per
// workgroup: the first and the last tile it touches), takes the tile's ticket, and the tile's last
// arriving segment sums the tile's partials in SEGMENT order -- its own from registers -- and runs
// the epilogue (deterministic: the order does not depend on which segment arrives last).
__device__ __forceinline__ int sk_lo(int g, int I, int G) { return (int)(((int64_t)g * I) / G); }
// logical workgroup whose iteration range contains iteration i
__device__ __forceinline__ int sk_owner(int i, int I, int G) {
  int g = (int)(((int64_t)i * G) / I);
  while (g + 1 < G && sk_lo(g + 1, I, G) <= i) ++g;
  while (g > 0 && sk_lo(g, I, G) > i) --g;
  return g;
}

template <int DEPTH, bool RF, bool BAL>
__global__ void __launch_bounds__(512, 1) conv_gemm_pp_kernel(const ConvGemmArgs args) {
  using T = bf16_t;
  constexpr int BM = 256, BN = 256, WM = 2, WN = 4;
  constexpr int HALF = 128 * 128, BUF = 4 * HALF;
  constexpr int OSTR = BN * (int)sizeof(T) + 16;
  constexpr int SMEM = (2 * BUF > BM * OSTR) ? 2 * BUF : BM * OSTR;
  constexpr int LEAD = DEPTH == 1 ? 4 : 6;   // issue slot of half-tile s = s - LEAD
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int nN = args.N / BN;
  const int L = xcd_remap(blockIdx.x, nN * ((args.M + BM - 1) / BM));
  if (L < 0) return;  // whole workgroup: no barrier is left unmatched
  const int n_tile = L % nN, m_tile = L / nN;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int M = args.M;
  const int cchunk = (lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7);
  const int rsub = lane >> 3;
  const int lane_ch = cchunk * 8;
  const int wv = __builtin_amdgcn_readfirstlane(wave);

  // the 4 A rows and 4 B rows this lane fetches: index q = half*2 + instruction; byte offsets for
  // the buffer-descriptor LDS-DMA (blds16: the stage's shift goes into the scalar base)
  unsigned a_off[4], a_tap[4], b_off[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int h = q >> 1, j = q & 1;
    const int hr = (j * 8 + wave) * 8 + rsub;            // row of the half-tile image
    const int m = m0 + (hr >> 6) * 128 + h * 64 + (hr & 63);
    a_off[q] = 0;
    a_tap[q] = 0;
    if (m < M) {
      const int b = dm_div(args.dm_hw, m);
      const int rem = m - b * args.dm_hw.d;
      const int oh = dm_div(args.dm_w, rem);
      const int ow = rem - oh * args.dm_w.d;
      const int ih = oh * args.stride, iw = ow * args.stride;
      a_off[q] = 2u * (unsigned)(((b * args.Hi + ih) * args.Wi + iw) * args.Cseg + lane_ch);
      unsigned t = 0;
#pragma unroll
      for (int dh = -1; dh <= 1; ++dh)
#pragma unroll
        for (int dw = -1; dw <= 1; ++dw)
          t |= (unsigned)(ih + dh >= 0 && ih + dh < args.Hi && iw + dw >= 0 && iw + dw < args.Wi) << ((dh + 1) * 3 + dw + 1);
      a_tap[q] = t;
    }
    const int n = n0 + (hr >> 5) * 64 + h * 32 + (hr & 31);
    b_off[q] = 2u * (unsigned)(n * args.Kpad + lane_ch);
  }
  const rsrc_t rb = buf_rsrc(args.Bw);
  const int nk = args.Kpad / 64;
  const int slast = 4 * nk - 1;

  // half-tile s = 4 * K-tile + {0: A0, 1: B0, 2: B1, 3: A1} into buffer (K-tile & 1)
  auto issue = [&](int sq) {
    if (sq > slast) return;
    const int kt = sq >> 2, i = sq & 3;
    char* bufp = smem + (kt & 1) * BUF;
    if (i == 0 || i == 3) {
      const int h = i == 0 ? 0 : 1;
      char* dst = bufp + h * HALF;
      const int k0 = kt * 64;
      const int seg = dm_div(args.dm_cseg, k0);
      const int ch0 = k0 - seg * args.Cseg;
      const ConvSeg sg = args.seg[seg];
      const int delta = (sg.dh * args.Wi + sg.dw) * args.Cseg + ch0;
      const int tb = (sg.dh + 1) * 3 + sg.dw + 1;
      const rsrc_t ra = buf_rsrc((const T*)sg.ptr + delta);
#pragma unroll
      for (int j = 0; j < 2; ++j) blds16(ra, sel_oob(a_tap[h * 2 + j], tb, a_off[h * 2 + j]), 0, dst + (j * 8 + wv) * 1024);
    } else {
      const int h = i == 1 ? 0 : 1;
      char* dst = bufp + (2 + h) * HALF;
#pragma unroll
      for (int j = 0; j < 2; ++j) blds16(rb, b_off[h * 2 + j], (unsigned)kt * 128u, dst + (j * 8 + wv) * 1024);
    }
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};
  Frag<T> fa[4][2], fb0[2][2], fb1[2][2];

  auto read_a = [&](const char* img) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int g = 0; g < 2; ++g) read_frag<T>(img, wr * 64 + i * 16 + (lane & 15), g, lane, fa[i][g]);
  };
  auto read_b = [&](const char* img, Frag<T> (&fb)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 2; ++g) read_frag<T>(img, wc * 32 + j * 16 + (lane & 15), g, lane, fb[j][g]);
  };
  auto quad = [&](int ms, int ns, const Frag<T> (&fb)[2][2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mma(acc[ms * 4 + i][ns * 2 + j], fa[i][g], fb[j][g]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
  // The wait of slot q (= 4 * K-tile + phase) must retire every half read in slot q + 1:
  // A0 (q+1) and -- unless pre-read in phase 4 -- B0 (q+2) before phase 1; B1 (q+2) before
  // phase 2; A1 (q+2) before phase 3; with BAL the next B0 (q+3) before phase 4.
  auto vwait = [&](int q) {
    const int p = q & 3;
    const int need = p == 2 ? (BAL ? q + 3 : q + 1) : (p == 3 ? (BAL ? q + 1 : q + 2) : q + 2);
    const int r = min(q + LEAD, slast) - min(need, slast);
    if (r >= 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (r == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (r == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (r == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  for (int sq = 0; sq < LEAD; ++sq) issue(sq);
  {
    const int r = min(LEAD - 1, slast) - (BAL ? 1 : 1);   // halves 0 and 1 needed first
    if (r >= 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (r == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (r == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (r == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  raw_barrier();
  if (BAL) read_b(smem + 2 * HALF, fb0);   // B0 of K-tile 0 (later ones: pre-read in phase 4)
  if (wr == 1) raw_barrier();   // G1 runs one barrier behind G0

  // one K-tile; fbp holds (BAL) or receives its B0, fbq receives B1 (and with BAL the next B0)
  auto ktile = [&](int kt, Frag<T> (&fbp)[2][2], Frag<T> (&fbq)[2][2]) {
    const char* buf = smem + (kt & 1) * BUF;
    const char* nbuf = smem + ((kt + 1) & 1) * BUF;
    const int q = 4 * kt;
    // phase 1: quadrant (0,0) [A0 + B0]
    if (!RF) issue(q + LEAD);
    read_a(buf);
    if (!BAL) read_b(buf + 2 * HALF, fbp);
    if (RF) issue(q + LEAD);
    vwait(q);
    raw_barrier();
    quad(0, 0, fbp);
    raw_barrier();
    // phase 2: quadrant (0,1) [A0 + B1]
    if (!RF) issue(q + 1 + LEAD);
    read_b(buf + 3 * HALF, fbq);
    if (RF) issue(q + 1 + LEAD);
    vwait(q + 1);
    raw_barrier();
    quad(0, 1, fbq);
    raw_barrier();
    // phase 3: quadrant (1,1) [A1 + B1]
    if (!RF) issue(q + 2 + LEAD);
    read_a(buf + HALF);
    if (RF) issue(q + 2 + LEAD);
    vwait(q + 2);
    raw_barrier();
    quad(1, 1, fbq);
    raw_barrier();
    // phase 4: quadrant (1,0) [A1 + B0]
    if (!RF) issue(q + 3 + LEAD);
    if (BAL && kt + 1 < nk) read_b(nbuf + 2 * HALF, fbq);
    if (RF) issue(q + 3 + LEAD);
    vwait(q + 3);
    raw_barrier();
    quad(1, 0, fbp);
    raw_barrier();
  };
  if (BAL) {
    for (int kt = 0; kt < nk; kt += 2) {
      ktile(kt, fb0, fb1);
      if (kt + 1 < nk) ktile(kt + 1, fb1, fb0);
    }
  } else {
    for (int kt = 0; kt < nk; ++kt) ktile(kt, fb0, fb1);
  }
  if (wr == 0) raw_barrier();   // re-align the groups before the epilogue reuses the LDS
  __syncthreads();
  conv_epilogue<T, BM, BN, WM, WN>(args, acc, smem, m0, n0, m_tile, tid, lane, wr, wc);
}

template <int DEPTH, bool RF, bool BAL>
__global__ void __launch_bounds__(512, 1) conv_gemm_ppsk_kernel(const ConvGemmArgs args) {
  constexpr bool SK = true;
  using T = bf16_t;
  constexpr int BM = 256, BN = 256, WM = 2, WN = 4;
  constexpr int HALF = 128 * 128, BUF = 4 * HALF;
  constexpr int OSTR = BN * (int)sizeof(T) + 16;
  constexpr int SMEM = (2 * BUF > BM * OSTR) ? 2 * BUF : BM * OSTR;
  constexpr int LEAD = DEPTH == 1 ? 4 : 6;   // issue slot of half-tile s = s - LEAD
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int nN = args.N / BN;
  const int ntiles = nN * ((args.M + BM - 1) / BM);
  const int nk = args.Kpad / 64;
  const int M = args.M;
  const int cchunk = (lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7);
  const int rsub = lane >> 3;
  const int lane_ch = cchunk * 8;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const rsrc_t rb = buf_rsrc(args.Bw);

  // this workgroup's iterations: SK, a contiguous range of the (tile, K-tile) space (logical index
  // g: consecutive g share an XCD); else one whole tile
  int it, it_end, g = 0, G = 1, I = 0;
  if constexpr (SK) {
    G = gridDim.x;
    I = ntiles * nk;
    g = xcd_remap(blockIdx.x, G);
    if (g < 0) return;
    it = sk_lo(g, I, G);
    it_end = sk_lo(g + 1, I, G);
  } else {
    const int L = xcd_remap(blockIdx.x, ntiles);
    if (L < 0) return;  // whole workgroup: no barrier is left unmatched
    it = L * nk;
    it_end = it + nk;
  }
  const int first_tile = it / nk;

  f32x4_t acc[8][4];
  Frag<T> fa[4][2], fb0[2][2], fb1[2][2];

  while (it < it_end) {
    const int L = it / nk, k0 = it - L * nk, k1 = min(nk, k0 + (it_end - it));
    it += k1 - k0;
    const int n_tile = L % nN, m_tile = L / nN;
    const int m0 = m_tile * BM, n0 = n_tile * BN;

    // the 4 A rows and 4 B rows this lane fetches: index q = half*2 + instruction; byte offsets for
    // the buffer-descriptor LDS-DMA (blds16: the stage's shift goes into the scalar base)
    unsigned a_off[4], a_tap[4], b_off[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int h = q >> 1, j = q & 1;
      const int hr = (j * 8 + wave) * 8 + rsub;            // row of the half-tile image
      const int m = m0 + (hr >> 6) * 128 + h * 64 + (hr & 63);
      a_off[q] = 0;
      a_tap[q] = 0;
      if (m < M) {
        const int b = dm_div(args.dm_hw, m);
        const int rem = m - b * args.dm_hw.d;
        const int oh = dm_div(args.dm_w, rem);
        const int ow = rem - oh * args.dm_w.d;
        const int ih = oh * args.stride, iw = ow * args.stride;
        a_off[q] = 2u * (unsigned)(((b * args.Hi + ih) * args.Wi + iw) * args.Cseg + lane_ch);
        unsigned t = 0;
#pragma unroll
        for (int dh = -1; dh <= 1; ++dh)
#pragma unroll
          for (int dw = -1; dw <= 1; ++dw)
            t |= (unsigned)(ih + dh >= 0 && ih + dh < args.Hi && iw + dw >= 0 && iw + dw < args.Wi) << ((dh + 1) * 3 + dw + 1);
        a_tap[q] = t;
      }
      const int n = n0 + (hr >> 5) * 64 + h * 32 + (hr & 31);
      b_off[q] = 2u * (unsigned)(n * args.Kpad + lane_ch);
    }
    const int nks = k1 - k0;
    const int slast = 4 * nks - 1;

    // half-tile s = 4 * (local K-tile) + {0: A0, 1: B0, 2: B1, 3: A1} into buffer (local K-tile & 1)
    auto issue = [&](int sq) {
      if (sq > slast) return;
      const int lkt = sq >> 2, i = sq & 3, kt = k0 + lkt;
      char* bufp = smem + (lkt & 1) * BUF;
      if (i == 0 || i == 3) {
        const int h = i == 0 ? 0 : 1;
        char* dst = bufp + h * HALF;
        const int kk = kt * 64;
        const int seg = dm_div(args.dm_cseg, kk);
        const int ch0 = kk - seg * args.Cseg;
        const ConvSeg sg = args.seg[seg];
        const int delta = (sg.dh * args.Wi + sg.dw) * args.Cseg + ch0;
        const int tb = (sg.dh + 1) * 3 + sg.dw + 1;
        const rsrc_t ra = buf_rsrc((const T*)sg.ptr + delta);
#pragma unroll
        for (int j = 0; j < 2; ++j) blds16(ra, sel_oob(a_tap[h * 2 + j], tb, a_off[h * 2 + j]), 0, dst + (j * 8 + wv) * 1024);
      } else {
        const int h = i == 1 ? 0 : 1;
        char* dst = bufp + (2 + h) * HALF;
#pragma unroll
        for (int j = 0; j < 2; ++j) blds16(rb, b_off[h * 2 + j], (unsigned)kt * 128u, dst + (j * 8 + wv) * 1024);
      }
    };

#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};

    auto read_a = [&](const char* img) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int gq = 0; gq < 2; ++gq) read_frag<T>(img, wr * 64 + i * 16 + (lane & 15), gq, lane, fa[i][gq]);
    };
    auto read_b = [&](const char* img, Frag<T> (&fb)[2][2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int gq = 0; gq < 2; ++gq) read_frag<T>(img, wc * 32 + j * 16 + (lane & 15), gq, lane, fb[j][gq]);
    };
    auto quad = [&](int ms, int ns, const Frag<T> (&fb)[2][2]) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int gq = 0; gq < 2; ++gq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) mma(acc[ms * 4 + i][ns * 2 + j], fa[i][gq], fb[j][gq]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    };
    // The wait of slot q (= 4 * K-tile + phase) must retire every half read in slot q + 1:
    // A0 (q+1) and -- unless pre-read in phase 4 -- B0 (q+2) before phase 1; B1 (q+2) before
    // phase 2; A1 (q+2) before phase 3; with BAL the next B0 (q+3) before phase 4.
    auto vwait = [&](int q) {
      const int p = q & 3;
      const int need = p == 2 ? (BAL ? q + 3 : q + 1) : (p == 3 ? (BAL ? q + 1 : q + 2) : q + 2);
      const int r = min(q + LEAD, slast) - min(need, slast);
      if (r >= 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (r == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (r == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (r == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };

    for (int sq = 0; sq < LEAD; ++sq) issue(sq);
    {
      const int r = min(LEAD - 1, slast) - 1;   // halves 0 and 1 needed first
      if (r >= 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (r == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (r == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (r == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    raw_barrier();
    if (BAL) read_b(smem + 2 * HALF, fb0);   // B0 of K-tile 0 (later ones: pre-read in phase 4)
    if (wr == 1) raw_barrier();   // G1 runs one barrier behind G0

    // one K-tile; fbp holds (BAL) or receives its B0, fbq receives B1 (and with BAL the next B0)
    auto ktile = [&](int lkt, Frag<T> (&fbp)[2][2], Frag<T> (&fbq)[2][2]) {
      const char* buf = smem + (lkt & 1) * BUF;
      const char* nbuf = smem + ((lkt + 1) & 1) * BUF;
      const int q = 4 * lkt;
      // phase 1: quadrant (0,0) [A0 + B0]
      if (!RF) issue(q + LEAD);
      read_a(buf);
      if (!BAL) read_b(buf + 2 * HALF, fbp);
      if (RF) issue(q + LEAD);
      vwait(q);
      raw_barrier();
      quad(0, 0, fbp);
      raw_barrier();
      // phase 2: quadrant (0,1) [A0 + B1]
      if (!RF) issue(q + 1 + LEAD);
      read_b(buf + 3 * HALF, fbq);
      if (RF) issue(q + 1 + LEAD);
      vwait(q + 1);
      raw_barrier();
      quad(0, 1, fbq);
      raw_barrier();
      // phase 3: quadrant (1,1) [A1 + B1]
      if (!RF) issue(q + 2 + LEAD);
      read_a(buf + HALF);
      if (RF) issue(q + 2 + LEAD);
      vwait(q + 2);
      raw_barrier();
      quad(1, 1, fbq);
      raw_barrier();
      // phase 4: quadrant (1,0) [A1 + B0]
      if (!RF) issue(q + 3 + LEAD);
      if (BAL && lkt + 1 < nks) read_b(nbuf + 2 * HALF, fbq);
      if (RF) issue(q + 3 + LEAD);
      vwait(q + 3);
      raw_barrier();
      quad(1, 0, fbp);
      raw_barrier();
    };
    if (BAL) {
      for (int kt = 0; kt < nks; kt += 2) {
        ktile(kt, fb0, fb1);
        if (kt + 1 < nks) ktile(kt + 1, fb1, fb0);
      }
    } else {
      for (int kt = 0; kt < nks; ++kt) ktile(kt, fb0, fb1);
    }
    if (wr == 0) raw_barrier();   // re-align the groups before the epilogue reuses the LDS
    __syncthreads();
    if constexpr (SK) {
      if (k0 != 0 || k1 != nk) {
        // partial tile: publish, take the tile's ticket; the last segment combines and stores
        const int gf = sk_owner(L * nk, I, G), gl = sk_owner(L * nk + nk - 1, I, G);
        const int mine = g - gf;
        auto slot_of = [&](int gg) {   // the partial slot of the segment of tile L done by gg
          return 2 * gg + (L == sk_lo(gg, I, G) / nk ? 0 : 1);
        };
        constexpr int PT = 8 * 64 * 32 * 4;   // floats per partial tile (8 waves x 32 fragments x 64 lanes x 4)
        float* own = args.kwork + (size_t)slot_of(g) * PT + (wave * 32) * 256 + lane * 4;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4_t v = acc[i][j];
            st_sc1_f4(own + (i * 4 + j) * 256, v[0], v[1], v[2], v[3]);
          }
        int* flag = (int*)smem;
        if (!wg_last_of(args.kcnt + L, (unsigned)(gl - gf + 1), flag)) continue;
        // sum the tile's segments in segment order, every one (this workgroup's too) read back from
        // its slot: no second accumulator set in registers
        (void)mine;
        for (int sgm = 0; sgm <= gl - gf; ++sgm) {
          const float* src = args.kwork + (size_t)slot_of(gf + sgm) * PT + (wave * 32) * 256 + lane * 4;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            f4v_t v[4];
            ld_sc1_f4x4(src + (i * 4) * 256, 256, v);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const f32x4_t w = {v[j][0], v[j][1], v[j][2], v[j][3]};
              acc[i][j] = sgm == 0 ? w : acc[i][j] + w;
            }
          }
        }
      }
    }
    conv_epilogue<T, BM, BN, WM, WN>(args, acc, smem, m0, n0, m_tile, tid, lane, wr, wc);
    if constexpr (SK) __syncthreads();   // the next segment's DMA must not overwrite the staging tile
  }
  (void)first_tile;
}

template <int DEPTH, bool RF, bool BAL>
int launch_pp(const ConvGemmArgs& a, hipStream_t st) {
  if (t_dry_rows) { *t_dry_rows = (a.M + 255) / 256; if (t_dry_bn) *t_dry_bn = 256; return 0; }
  dim3 grid(xcd_pad((a.N / 256) * ((a.M + 255) / 256)));
  hipLaunchKernelGGL((conv_gemm_pp_kernel<DEPTH, RF, BAL>), grid, dim3(512), 0, st, a);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// stream-K ping-pong launch (see conv_gemm_pp_kernel): G = 256 persistent workgroups (one per CU);
// workspace: 2 partial tiles (256 KB each) per workgroup; tickets: one per tile
int g_ppsk = 0;   // knob 40: 1 = the stream-K ping-pong decomposition where it applies (measured slower: opt-in)
constexpr int kPpskG = 256;
int64_t ppsk_work_floats() { return (int64_t)2 * kPpskG * 256 * 256; }
bool ppsk_applies(const ConvGemmArgs& a) {
  if (!g_ppsk || a.N % 256 || a.K < 2048) return false;
  const int tiles = (a.N / 256) * ((a.M + 255) / 256);
  const int nk = a.Kpad / 64;
  const int64_t I = (int64_t)tiles * nk;
  if (tiles >= 2 * kPpskG || I < 8 * kPpskG) return false;
  // whole waves of tiles fill the chip already (>= 90 %)
  const int waves = (tiles + kPpskG - 1) / kPpskG;
  if (tiles * 10 >= waves * kPpskG * 9) return false;
  // at most ~3 segments per tile (the last arriver reads the others' 256 KB partials serially)
  return I / kPpskG >= nk / 3;
}
int launch_ppsk(ConvGemmArgs a, hipStream_t st) {
  if (t_dry_rows) {
    *t_dry_rows = (a.M + 255) / 256;
    if (t_dry_bn) *t_dry_bn = 256;
    if (t_dry_work) *t_dry_work = ppsk_work_floats();
    return 0;
  }
  if (!a.kwork || a.kwork_floats < ppsk_work_floats()) return DFCSA_EINVAL;
  const int tiles = (a.N / 256) * ((a.M + 255) / 256);
  a.kcnt = dfcsa_ticket_alloc(tiles);
  if (!a.kcnt) return DFCSA_EINVAL;
  hipLaunchKernelGGL((conv_gemm_ppsk_kernel<2, true, false>), dim3(kPpskG), dim3(512), 0, st, a);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// --------------------------------------------------------------------------------------------
// 3x3 convolutions (forward and the fused 3x3 + 1x1 data gradient) on 2-D halo tiles.
//
// The row-tile kernels above fetch, for every one of the 9 taps, the tile's rows shifted by
// (dh, dw): 9x the unique input per K chunk crosses L2 -> LDS.  Here a workgroup owns a TW x TR
// block of output pixels of ONE image (TW | W, TR | H: a tap never needs a per-pixel border
// mask, the halo pixels outside the image are zero) and, per 64-channel chunk of a source, stages
// its (TW+2) x (TR+2) halo in LDS once; the tap steps read their shifted windows from it.  Only
// the weight panel (BN x 64 of one tap) streams per step.
//
// Instruction economy (round-3 counters: the row-tile kernels issue ~5 VALU per MFMA, the
// round-3 v1/v2 halo kernels 10-13, and the wave time goes to issue, not to the MFMA pipe):
//  * halo pixels sit at a 160-B pitch (128 B of channels + 32 B pad): the 16 rows of a ds_read_b128
//    fragment read are then spread over all 64 banks whatever pixel they start at (the b128 lane
//    groups {0-3,12-15,20-27}... map rows to 40r + 4c words: distinct 4-bank spans), so the A
//    operand of tap (dh, dw) is one b128 per fragment at (lane base + tap offset): one v_add per
//    fragment per step, no swizzle arithmetic and no masks;
//  * the halo is register-staged (buffer_load_dwordx4 with a raw buffer descriptor: pixels outside
//    the image are out-of-range offsets and read as zeros), issued at the first tap of a chunk
//    and written at its last;
//  * the weight panel arrives by LDS-DMA through a buffer descriptor (scalar K offset per step, an
//    out-of-range row offset for the N tail) into a 3-slot ring, two steps ahead, XOR-swizzled on
//    the source side for conflict-free b128 reads;
//  * the step list (K column, tap offset, chunk boundaries) is precomputed on the host.
// 8 waves (4 x 2, wave tile 64 x BN/2), one workgroup per CU; one barrier per step.
// Epilogue: bias, bf16 store of the valid pixels (1-3 destinations, optional accumulate), BN
// partial statistics as ONE row per tile (dfcsa_conv_stats_rows gives the row count).
// --------------------------------------------------------------------------------------------
constexpr int HALO_PITCH = 160;                 // LDS bytes per halo pixel (64 channels + pad)
constexpr int HALO_MAXSTEP = 192;               // steps (source x chunk x tap) per launch

struct HaloArgs {
  int M, N, Kpad, Cseg, H, W;
  int tiles_x, tiles_y, tiles_m;    // W / TW, H / TR, all tiles
  int nsteps;
  const void* gptr[4];              // source tensors ([B][H][W][Cseg])
  const void* Bw;
  const float* bias;
  void* dest[3];
  int Nd, accumulate;
  float* stats;
  // step s: bits 0-15 K column of the weight panel, 16-23 tap offset (dh+1)*(TW+2) + dw+1 in halo
  // pixels, 24-25 source, 26 first tap of a chunk, 27 last tap of a chunk, 28-31 chunk index
  unsigned step[HALO_MAXSTEP];
};

// NBUF = 2: two halo buffers (the next chunk's halo is written while the current one is read),
// one workgroup per CU.  NBUF = 1 (BN = 64): one halo buffer, ~76 KB of LDS and <= 128 VGPRs, so
// two workgroups share a CU and one's prologue / barrier waits overlap the other's MFMAs; the next
// chunk's halo (already in registers) is written after the first barrier of that chunk, and a
// second barrier publishes it.
template <int TW, int TR, int BN, int NBUF>
__global__ void __launch_bounds__(512, NBUF == 1 ? 2 : 1) conv_halo_kernel(const HaloArgs args) {
  using T = bf16_t;
  constexpr int WM = 4, WN = 2, NT = 512;
  constexpr int WTN = BN / WN, FM = 4, FN = WTN / 16;
  constexpr int HW2 = TW + 2, HPX = (TW + 2) * (TR + 2);
  constexpr int HBUF = (HPX * HALO_PITCH + 255) / 256 * 256;
  constexpr int BSLOT = BN * 128, NBS = 3;
  constexpr int KB = BN / 64;                    // weight DMA pieces per wave per step (1 KB each)
  constexpr int HCH = HPX * 8;                   // 16-B chunks of one halo
  constexpr int HL = (HCH + NT - 1) / NT;        // halo chunks per thread
  constexpr int OSTR = BN * 2 + 16;
  constexpr int SMEM_MAIN = NBUF * HBUF + NBS * BSLOT;
  constexpr int SMEM_EPI = 256 * OSTR + WM * 2 * BN * 4;
  constexpr int SMEM = SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI;
  static_assert(TW * TR <= 256 && SMEM <= 160 * 1024 && FN >= 1, "halo tiling");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  char* const bbuf = smem + NBUF * HBUF;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int nN = (args.N + BN - 1) / BN;
  const int L = xcd_remap(blockIdx.x, nN * args.tiles_m);
  if (L < 0) return;
  const int tn = L % nN, tm = L / nN;            // the N tiles of one pixel tile share an XCD
  const int tx = tm % args.tiles_x, rest = tm / args.tiles_x;
  const int ty = rest % args.tiles_y, img = rest / args.tiles_y;
  const int y0 = ty * TR, x0 = tx * TW, n0 = tn * BN;
  const int H = args.H, W = args.W;

  // halo staging: thread chunk e = tid + k*NT -> halo pixel e/8, 16-B chunk e%8
  unsigned hoff[HL];
  int hlds[HL];
#pragma unroll
  for (int k = 0; k < HL; ++k) {
    const int e = tid + k * NT;
    const int q = e >> 3, c = e & 7;
    const int hy = q / HW2, hx = q - hy * HW2;
    const int y = y0 - 1 + hy, x = x0 - 1 + hx;
    const bool ok = e < HCH && y >= 0 && y < H && x >= 0 && x < W;
    hoff[k] = ok ? 2u * (unsigned)((((img * H + y) * W + x) * args.Cseg) + c * 8) : kBufOOB;
    hlds[k] = e < HCH ? q * HALO_PITCH + c * 16 : -1;
  }
  // weight panel DMA: piece p = wave + 8k holds panel rows 8p..8p+7; the lane fetches the logical
  // chunk that read_frag's swizzle expects in its LDS slot
  unsigned boff[KB];
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int nl = (wave + 8 * k) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((nl >> 1) & 7);
    const int n = n0 + nl;
    boff[k] = n < args.N ? 2u * (unsigned)(n * args.Kpad + c * 8) : kBufOOB;
  }
  const rsrc_t rb = buf_rsrc(args.Bw);
  auto issue_b = [&](int s) {
    const unsigned w = args.step[s];
    char* dst = bbuf + (s % NBS) * BSLOT;
#pragma unroll
    for (int k = 0; k < KB; ++k) blds16(rb, boff[k], 2u * (w & 0xffffu), dst + (wv + 8 * k) * 1024);
  };
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  u32x4_t hreg[HL];
  auto load_halo = [&](unsigned w) {
    const rsrc_t rs = buf_rsrc(args.gptr[(w >> 24) & 3]);
    const unsigned soff = (w >> 28) * 128u;      // chunk cc: channels 64cc..64cc+63
#pragma unroll
    for (int k = 0; k < HL; ++k) hreg[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)hoff[k], (int)soff, 0);
  };
  auto store_halo = [&](int buf) {
#pragma unroll
    for (int k = 0; k < HL; ++k)
      if (hlds[k] >= 0) *(u32x4_t*)(smem + buf * HBUF + hlds[k]) = hreg[k];
  };

  // A fragment bases: tile pixel m = wm*64 + 16i + lane%16 -> halo pixel of tap (-1, -1)
  int abase[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = wm * 64 + i * 16 + (lane & 15);
    const int r = m / TW, c = m - r * TW;
    abase[i] = (m < TW * TR ? (r * HW2 + c) * HALO_PITCH : 0) + (lane >> 4) * 16;
  }
  // B fragment offsets in a ring slot: row wn*WTN + 16jj + lane%16, logical chunk 4g2 + lane/16
  int bofs[FN][2];
#pragma unroll
  for (int jj = 0; jj < FN; ++jj)
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2) {
      const int row = wn * WTN + jj * 16 + (lane & 15);
      bofs[jj][g2] = row * 128 + swz(row, 4 * g2 + (lane >> 4)) * 16;
    }

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) acc[i][jj] = {0.f, 0.f, 0.f, 0.f};

  const int S = args.nsteps;
  load_halo(args.step[0]);
  store_halo(0);                                 // (the compiler waits for the loads)
  issue_b(0);
  if (S > 1) issue_b(1);
  int hb = 0;                                    // halo buffer of the current chunk
  int hs = -8;                                   // step that issued the halo loads in flight
  bool pending = false;                          // NBUF = 1: a loaded halo waits for the next chunk
  for (int s = 0; s < S; ++s) {
    const unsigned w = args.step[s];
    // this step's weight panel: vmcnt is in order, so the panel issued two steps ago is complete
    // once at most the later ones are in flight -- the next step's panel, plus, for the two steps
    // after a halo issue, that halo's HL loads (issued after panel s+2; the wait of step hs+3
    // retires them)
    if (s + 1 >= S) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (s - hs <= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KB + HL) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KB) : "memory");
    lds_barrier();   // publishes this step's weight panel (and, at a chunk's first tap, its halo)
    if constexpr (NBUF == 1) {
      if (pending) {   // every wave is past the previous chunk's reads: overwrite, then publish
        store_halo(0);
        lds_barrier();
        pending = false;
      }
    }
    if (s + 2 < S) issue_b(s + 2);
    const bool more = s + 1 < S;
    if (((w >> 26) & 1) && !((w >> 27) & 1 && !more)) {
      // first tap of a chunk: fetch the next chunk's halo (the step after this chunk's last tap)
      int u = s;
      while (u < S && !((args.step[u] >> 27) & 1)) ++u;
      if (u + 1 < S) {
        load_halo(args.step[u + 1]);
        hs = s;
      }
    }
    const int toff = hb * HBUF + (int)((w >> 16) & 0xffu) * HALO_PITCH;
    const char* bs = bbuf + (s % NBS) * BSLOT;
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2) {
      bf16x8_t fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = *(const bf16x8_t*)(smem + abase[i] + toff + 64 * g2);
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) fb[jj] = *(const bf16x8_t*)(bs + bofs[jj][g2]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jj = 0; jj < FN; ++jj)
          acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[jj], acc[i][jj], 0, 0, 0);
    }
    if (((w >> 27) & 1) && more) {
      if constexpr (NBUF == 2) {
        // last tap of a chunk: the next chunk's halo goes to the other buffer (read from the next
        // step on, after its barrier; that buffer's last reader was the previous chunk)
        hb ^= 1;
        store_halo(hb);
      } else {
        pending = true;
      }
      hs = -8;
    }
  }
  __syncthreads();

  // ---- epilogue: accumulator element (i, jj, r) = tile pixel wm*64 + 16i + 4(lane/16) + r ----
  constexpr int NPX = TW * TR;
  float* red = (float*)(smem + 256 * OSTR);      // [WM][2][BN]
  if (args.stats) {
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) {
      float sm = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
          const float v = m < NPX ? acc[i][jj][r] : 0.f;
          sm += v;
          q += v * v;
        }
      sm += __shfl_xor(sm, 16, 64); sm += __shfl_xor(sm, 32, 64);
      q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
      if (lane < 16) {
        const int col = wn * WTN + jj * 16 + lane;
        red[(wm * 2 + 0) * BN + col] = sm;
        red[(wm * 2 + 1) * BN + col] = q;
      }
    }
  }
  T* otile = (T*)smem;
#pragma unroll
  for (int jj = 0; jj < FN; ++jj) {
    const int col = wn * WTN + jj * 16 + (lane & 15);
    const int n = n0 + col;
    const float bv = (args.bias && n < args.N) ? args.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        *(T*)((char*)otile + row * OSTR + col * 2) = f2bf(acc[i][jj][r] + bv);
      }
  }
  __syncthreads();
  if (args.stats && tid < BN) {
    const int n = n0 + tid;
    if (n < args.N) {
      float sm = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) { sm += red[(w * 2) * BN + tid]; q += red[(w * 2 + 1) * BN + tid]; }
      args.stats[(size_t)tm * 2 * args.N + n] = sm;
      args.stats[(size_t)tm * 2 * args.N + args.N + n] = q;
    }
  }
  constexpr int OCH = BN / 8;
  for (int e = tid; e < NPX * OCH; e += NT) {
    const int row = e / OCH, ck = e - row * OCH;
    const int r = row / TW, c = row - r * TW;
    const int n = n0 + ck * 8;
    if (n >= args.N) continue;
    const size_t mg = (size_t)(img * H + y0 + r) * W + x0 + c;
    const int d = n / args.Nd, col = n - d * args.Nd;
    T* dst = (T*)args.dest[d] + (mg * args.Nd + col);
    if (!args.accumulate) {
      *(uint4*)dst = *(const uint4*)((const char*)otile + row * OSTR + ck * 16);
      continue;
    }
    float v[8];
    load8<T>((const T*)((const char*)otile + row * OSTR + ck * 16), v);
    if (args.accumulate) {
      float o[8];
      load8<T>(dst, o);
#pragma unroll
      for (int qq = 0; qq < 8; ++qq) v[qq] += o[qq];
    }
    store8<T>(dst, v);
  }
}

int g_halo_min_m = 0;   // knob 19: smallest M routed to the halo kernel (0: never)

// Build the halo launch for a bf16 3x3 (or fused 3x3 + 1x1) GEMM; false if it does not apply.
// Tile shapes: 16 x 16 (W, H multiples of 16: the 224^2 / 112^2 levels), 8 x 28 (56^2),
// 14 x 14 (28^2).  *tw / *tr return the shape.
bool halo_plan(const ConvGemmArgs& a, HaloArgs* h, int* tw, int* tr) {
  if (g_halo_min_m <= 0 || a.M < g_halo_min_m) return false;
  if (a.mode != CONV_STORE_PLAIN || a.stride != 1 || a.Ho != a.Hi || a.Wo != a.Wi || a.Cseg % 64) return false;
  const int H = a.Ho, W = a.Wo;
  if ((int64_t)a.M * a.Cseg * 2 >= (1ll << 31) || (int64_t)a.N * a.Kpad * 2 >= (1ll << 31) || a.Kpad > 65535)
    return false;
  int TW, TR;
  if (W % 16 == 0 && H % 16 == 0) { TW = 16; TR = 16; }
  else if (W % 8 == 0 && H % 28 == 0) { TW = 8; TR = 28; }
  else if (W % 14 == 0 && H % 14 == 0) { TW = 14; TR = 14; }
  else return false;
  std::memset(h, 0, sizeof(*h));
  // sources: segments grouped by tensor, in first-appearance order; each segment = one tap
  const void* src[4];
  int nsrc = 0, gseg[DFCSA_MAX_SEG];
  bool shifted = false;
  for (int i = 0; i < a.nseg; ++i) {
    const ConvSeg& s = a.seg[i];
    if (s.dh < -1 || s.dh > 1 || s.dw < -1 || s.dw > 1) return false;
    shifted |= (s.dh || s.dw);
    int g = 0;
    while (g < nsrc && src[g] != s.ptr) ++g;
    if (g == nsrc) {
      if (nsrc == 4) return false;
      src[nsrc++] = s.ptr;
    }
    gseg[i] = g;
  }
  if (!shifted) return false;
  const int nchunk = a.Cseg / 64;
  if (nchunk > 15) return false;
  int ns = 0;
  for (int g = 0; g < nsrc; ++g)
    for (int cc = 0; cc < nchunk; ++cc) {
      int first = ns, cnt = 0;
      for (int i = 0; i < a.nseg; ++i) {
        if (gseg[i] != g) continue;
        if (ns == HALO_MAXSTEP) return false;
        const unsigned kcol = (unsigned)(i * a.Cseg + cc * 64);
        const unsigned toff = (unsigned)((a.seg[i].dh + 1) * (TW + 2) + a.seg[i].dw + 1);
        h->step[ns++] = kcol | (toff << 16) | ((unsigned)g << 24) | ((unsigned)cc << 28);
        ++cnt;
      }
      h->step[first] |= 1u << 26;
      h->step[first + cnt - 1] |= 1u << 27;
    }
  h->nsteps = ns;
  for (int g = 0; g < nsrc; ++g) h->gptr[g] = src[g];
  h->M = a.M; h->N = a.N; h->Kpad = a.Kpad; h->Cseg = a.Cseg; h->H = H; h->W = W;
  h->tiles_x = W / TW; h->tiles_y = H / TR;
  h->tiles_m = (a.M / (H * W)) * h->tiles_x * h->tiles_y;
  h->Bw = a.Bw; h->bias = a.bias;
  for (int i = 0; i < 3; ++i) h->dest[i] = a.dest[i];
  h->Nd = a.Nd; h->accumulate = a.accumulate; h->stats = a.stats;
  *tw = TW; *tr = TR;
  return true;
}

int g_halo_variant = 0;   // knob 22: 0 = BN 64 single-buffer for N <= 64, BN 128 double-buffer above; 1 = BN 64 always;
                          // 2 = the double-buffered one-workgroup-per-CU kernel always

template <int TW, int TR>
void launch_halo_t(const HaloArgs& h, hipStream_t st) {
  if (g_halo_variant == 2) {
    if (h.N <= 64)
      hipLaunchKernelGGL((conv_halo_kernel<TW, TR, 64, 2>), dim3(xcd_pad(h.tiles_m)), dim3(512), 0, st, h);
    else
      hipLaunchKernelGGL((conv_halo_kernel<TW, TR, 128, 2>), dim3(xcd_pad(((h.N + 127) / 128) * h.tiles_m)), dim3(512),
                         0, st, h);
  } else if (h.N <= 64 || g_halo_variant == 1) {
    hipLaunchKernelGGL((conv_halo_kernel<TW, TR, 64, 1>), dim3(xcd_pad(((h.N + 63) / 64) * h.tiles_m)), dim3(512), 0,
                       st, h);
  } else {
    hipLaunchKernelGGL((conv_halo_kernel<TW, TR, 128, 2>), dim3(xcd_pad(((h.N + 127) / 128) * h.tiles_m)), dim3(512), 0,
                       st, h);
  }
}

int launch_halo(const HaloArgs& h, int tw, hipStream_t st) {
  if (t_dry_rows) { *t_dry_rows = h.tiles_m; return 0; }
  if (tw == 16) launch_halo_t<16, 16>(h, st);
  else if (tw == 8) launch_halo_t<8, 28>(h, st);
  else launch_halo_t<14, 14>(h, st);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// fp32 GEMMs with few rows (the LightSelfAttention q/k/v projections and their dgrad, M = B*P*P):
// split-reduction 16x64 tiles (small_gemm.h), plain 1x1 store with bias and column split
// K >= 256: 8 waves, 4 blocks of 16 in flight per wave (the 14^2 / 28^2 projections, K = 512-1280,
// were latency-bound at 11-25 us with 4 waves and 2 blocks in flight)
template <int NWV, int UNR>
__global__ void __launch_bounds__(NWV * 64) small_conv_f32_kernel(const ConvGemmArgs args) {
  __shared__ float lds[NWV * 16 * 64];
  const float* A = (const float*)args.seg[0].ptr;
  const float* Bw = (const float*)args.Bw;
  auto st = [&](int m, int n, float v) {
    if (args.bias) v += args.bias[n];
    const int d = n / args.Nd, col = n - d * args.Nd;
    ((float*)args.dest[d])[(size_t)m * args.Nd + col] = v;
  };
  small_gemm_tile<false, decltype(st), NWV, UNR>(A, args.Cseg, Bw, args.Kpad, args.M, args.N, args.K, blockIdx.x * 16,
                                                 blockIdx.y * 64, lds, st);
}

bool small_conv_applies(const ConvGemmArgs& a) {
  return a.M <= 4096 && a.nseg == 1 && a.seg[0].dh == 0 && a.seg[0].dw == 0 && a.stride == 1 &&
         a.mode == CONV_STORE_PLAIN && !a.stats && !a.accumulate && a.Ho == a.Hi && a.Wo == a.Wi &&
         a.Cseg % 4 == 0 && a.K % 4 == 0;
}

template <typename T, int BM, int BN, int WM, int WN>
int launch_cfg(const ConvGemmArgs& a, hipStream_t st) {
  if (t_dry_rows) { *t_dry_rows = (a.M + BM - 1) / BM; if (t_dry_bn) *t_dry_bn = BN; return 0; }
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM);
  hipLaunchKernelGGL((conv_gemm_kernel<T, BM, BN, WM, WN>), grid, dim3(WM * WN * 64), 0, st, a);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// --------------------------------------------------------------------------------------------
// Memory-bound 1x1 GEMMs (K <= 256, large M): persistent streaming kernel.
// A workgroup keeps its slice of the weights (N_wg = 4*NWC columns x KP) in REGISTERS (each wave
// owns NWC columns and holds their MFMA B fragments for the whole K), and walks 64-row M tiles
// grid-stride.  The next tile's A image is fetched by LDS-DMA while the current tile is
// multiplied and written, so loads, MFMA and the epilogue of different tiles overlap inside one
// workgroup, and the small LDS footprint lets several workgroups share a CU.  Waves split the
// columns, so per-column BatchNorm partial sums of a 64-row tile need no cross-wave reduction.
// --------------------------------------------------------------------------------------------
// SH: segments with (dh, dw) pixel shifts (a 3x3 conv whose 9 * Cin fits K <= 256, i.e. the
// first layer: Cin = 8, K = 72): each 8-channel chunk's row is the shifted pixel of its segment,
// the zero page outside the image; Ho = Hi, Wo = Wi, stride 1.
// SHUF: ConvTranspose2d(k=2, s=2) store (CONV_STORE_SHUFFLE2): column n = (i*2 + j)*Nd + co of
// input pixel (b, oh, ow) goes to output pixel (b, 2oh+i, 2ow+j), channel co -- 16-B chunks of 8
// consecutive co stay contiguous, so the stores are the plain kernel's with a per-row base.
// register budget for two waves per SIMD (two resident workgroups) on the wide-column variants,
// whose default allocation (264-440 VGPR+AGPR) leaves one (not the accumulating 64 x 128 one: it
// spills at 256)
template <int NWC, int KP, bool ACC>
constexpr int stream_wpe() { return NWC >= 48 && !(ACC && NWC * KP >= 64 * 128) ? 2 : 1; }

__device__ __forceinline__ int osw(int row) { return ((row >> 2) & 3) << 1; }

template <int NWC, int KP, bool ACC, bool SH = false, bool SHUF = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(stream_wpe<NWC, KP, ACC>())))
conv1x1_stream_kernel(const ConvGemmArgs args, int mtiles) {
  static_assert(!(SHUF && (ACC || SH)), "shuffle store: plain, unshifted");
  using T = bf16_t;
  constexpr int KS = KP / 64;               // 64-wide K stages (one 64x128B LDS image each)
  constexpr int KG = KP / 32;               // 32-wide MFMA k groups
  constexpr int FN = NWC / 16;              // column fragments per wave
  constexpr int NWG = 4 * NWC;              // columns per workgroup
  constexpr int IMG = 64 * 128;             // bytes of one stage image
  constexpr int SLOT = KS * IMG;
  // output staging tile: unpadded rows (NWG * 2 bytes), 16-B chunk c of row r stored at chunk
  // c ^ osw(r); the 1 KB the padding took lets the K = 256 variants keep two workgroups per CU
  // (80 KiB each): the bf16 stores of rows r, r + 4, r + 8, r + 12 (one instruction) land in four
  // different chunk pairs, the 16-B row reads stay whole rows
  constexpr int OSTR = NWG * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * SLOT];
  // separate LDS object: the waitcnt pass then knows the output staging reads cannot alias the
  // in-flight LDS-DMA images (one shared array makes it drain vmcnt before every staging read)
  __shared__ __attribute__((aligned(16))) char otile[64 * OSTR];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = args.M, N = args.N, K = args.K;
  const int n0 = blockIdx.y * NWG;
  const int rsub = lane >> 3;
  const int cchunk = (lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7);

  // B fragments of this wave's columns, whole K (zero beyond N / Kpad)
  bf16x8_t bfr[FN][KG];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wave * NWC + j * 16 + (lane & 15);
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      const int k = g * 32 + 8 * (lane >> 4);
      if (n < N && k < args.Kpad) bfr[j][g] = *(const bf16x8_t*)((const T*)args.Bw + (size_t)n * args.Kpad + k);
      else bfr[j][g] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  float bias[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wave * NWC + j * 16 + (lane & 15);
    bias[j] = (args.bias && n < N) ? args.bias[n] : 0.f;
  }
  const void* zero = (const void*)g_zero_page;

  // A image of tile t into slot s: instruction i covers stage i/2, rows ((i&1)*4 + wave)*8 + rsub.
  // The (segment, channel) of each of this lane's K chunks is tile-invariant: resolve the source
  // pointers once (a per-lane index into the kernel-argument segment table is a vector load that
  // the compiler follows with a full vmcnt drain -- not inside the streaming loop).
  const T* a_src[2 * KS];
  int a_dh[SH ? 2 * KS : 1], a_dw[SH ? 2 * KS : 1];
#pragma unroll
  for (int i = 0; i < 2 * KS; ++i) {
    const int k = (i >> 1) * 64 + cchunk * 8;
    a_src[i] = nullptr;
    if constexpr (SH) { a_dh[i] = 0; a_dw[i] = 0; }
    if (k < K) {
      const int seg = dm_div(args.dm_cseg, k);
      a_src[i] = (const T*)args.seg[seg].ptr + (k - seg * args.Cseg);
      if constexpr (SH) { a_dh[i] = args.seg[seg].dh; a_dw[i] = args.seg[seg].dw; }
    }
  }
  auto issue = [&](int t, int slot) {
    char* base = smem + slot * SLOT;
    // SH: (image, row, column) of this lane's two A rows of the tile
    int pb[2] = {0, 0}, ph[2] = {0, 0}, pw[2] = {0, 0};
    if constexpr (SH) {
#pragma unroll
      for (int r2 = 0; r2 < 2; ++r2) {
        const int m = t * 64 + (r2 * 4 + wave) * 8 + rsub;
        pb[r2] = dm_div(args.dm_hw, m);
        const int rem = m - pb[r2] * args.dm_hw.d;
        ph[r2] = dm_div(args.dm_w, rem);
        pw[r2] = rem - ph[r2] * args.dm_w.d;
      }
    }
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i) {
      const int st = i >> 1, rb = (i & 1) * 4 + wave;
      const int m = t * 64 + rb * 8 + rsub;
      const void* src = zero;
      if constexpr (SH) {
        const int ih = ph[i & 1] + a_dh[i], iw = pw[i & 1] + a_dw[i];
        if (m < M && a_src[i] && ih >= 0 && ih < args.Hi && iw >= 0 && iw < args.Wi)
          src = (const void*)(a_src[i] + ((size_t)(pb[i & 1] * args.Hi + ih) * args.Wi + iw) * args.Cseg);
      } else {
        if (m < M && a_src[i]) src = (const void*)(a_src[i] + (size_t)m * args.Cseg);
      }
      glds16(src, base + st * IMG + rb * 8 * 128);
    }
  };

  // vmcnt counts stores too and retires in order.  Every lane therefore issues a FIXED number of
  // global stores per tile (FN stats stores when stats are on, NSTORE output stores; out-of-range
  // ones go to a sink), so the wait for tile t's A image can leave the previous tile's stores in
  // flight instead of draining them every iteration (accumulate mode, whose epilogue loads the
  // destination, keeps the full drain).
  constexpr int NSTORE = (64 * (NWG / 8)) / 256;
  static_assert((64 * (NWG / 8)) % 256 == 0, "uniform store count per lane");
  constexpr int OCH = NWG / 8;
  // output chunk e = tid + it*256 of a tile: (row, column chunk) and the destination column base
  // are tile-invariant (resolved once; no per-store kernel-argument loads)
  T* o_base[NSTORE];
  int o_row[NSTORE], o_ld[NSTORE];
#pragma unroll
  for (int it = 0; it < NSTORE; ++it) {
    const int e = tid + it * 256;
    const int row = e / OCH, cc = e - row * OCH, n = n0 + cc * 8;
    o_row[it] = row;
    o_base[it] = nullptr;
    o_ld[it] = args.Nd;
    if (n < N) {
      const int d = n / args.Nd;
      if constexpr (SHUF)   // d = i*2 + j: output row offset i, column offset j
        o_base[it] = (T*)args.dest[0] + ((size_t)((d >> 1) * args.Wout + (d & 1)) * args.Nd + (n - d * args.Nd));
      else
        o_base[it] = (T*)args.dest[d] + (n - d * args.Nd);
    }
  }
  constexpr bool lean = !ACC;
  const bool with_stats = args.stats != nullptr;
  float st_s[FN], st_q[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) { st_s[j] = 0.f; st_q[j] = 0.f; }
  int t = blockIdx.x;
  if (t >= mtiles) return;
  issue(t, 0);
  int slot = 0;
  bool first_iter = true;
  for (; t < mtiles; t += gridDim.x, slot ^= 1) {
    const int tn = t + gridDim.x;
    // accumulate mode: fetch this tile's destination values now, ahead of the next A image, so
    // their latency overlaps the wait for this tile's A image instead of following the MFMAs
    uint4 dpre[ACC ? NSTORE : 1];
    if constexpr (ACC) {
#pragma unroll
      for (int it = 0; it < NSTORE; ++it) {
        const int m = t * 64 + o_row[it];
        dpre[it] = (m < M && o_base[it]) ? *(const uint4*)(o_base[it] + (size_t)m * o_ld[it]) : uint4{0, 0, 0, 0};
      }
    }
    if (tn < mtiles) {
      issue(tn, slot ^ 1);
      if (ACC || first_iter) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * KS) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * KS + NSTORE) : "memory");
    } else {
      if (ACC || first_iter) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NSTORE) : "memory");
    }
    first_iter = false;
    lds_barrier();
    const char* img = smem + slot * SLOT;
    f32x4_t acc[4][FN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      Frag<T> fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) read_frag<T>(img + (g >> 1) * IMG, i * 16 + (lane & 15), g & 1, lane, fa[i]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].v, bfr[j][g], acc[i][j], 0, 0, 0);
    }
    const int m0 = t * 64;
    // BatchNorm partial sums of the raw accumulator over this 64-row tile (valid rows only), kept
    // in registers across the workgroup's tiles: ONE statistics row per workgroup (row blockIdx.x)
    if (with_stats) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + i * 16 + (lane >> 4) * 4 + r;
            const float v = m < M ? acc[i][j][r] : 0.f;
            s += v;
            q += v * v;
          }
        s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
        q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
        st_s[j] += s;
        st_q[j] += q;
      }
    }
    // bias + convert into the staging tile (previous tile's stores have drained: barrier above)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wave * NWC + j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + (lane >> 4) * 4 + r;
          *(T*)(otile + row * OSTR + (((col >> 3) ^ osw(row)) << 4) + (col & 7) * 2) = f2bf(acc[i][j][r] + bias[j]);
        }
    }
    lds_barrier();
#pragma unroll
    for (int it = 0; it < NSTORE; ++it) {
      const int e = tid + it * 256;
      const int row = o_row[it], cc = e - row * OCH;
      const int m = m0 + row;
      uint4 v = *(const uint4*)(otile + row * OSTR + ((cc ^ osw(row)) << 4));
      const bool ok = m < M && o_base[it];
      size_t moff;
      if constexpr (SHUF) {   // input pixel m = (b, oh, ow) -> output pixel (b, 2oh, 2ow)
        const int b = dm_div(args.dm_hw, m), rem = m - b * args.dm_hw.d;
        const int oh = dm_div(args.dm_w, rem), ow = rem - oh * args.dm_w.d;
        moff = (size_t)((b * args.Hout + 2 * oh) * args.Wout + 2 * ow) * args.Nd;
      } else {
        moff = (size_t)m * o_ld[it];
      }
      T* dst = ok ? o_base[it] + moff : (T*)(g_store_sink + 4 * (tid & 63));
      if constexpr (lean) {   // branch-free: exactly one store instruction per iteration
        *(uint4*)dst = v;
        continue;
      }
      if (!ok) continue;
      if constexpr (ACC) {
        float a[8], o[8];
        load8<T>((const T*)&v, a);
        load8<T>((const T*)&dpre[it], o);
#pragma unroll
        for (int q = 0; q < 8; ++q) a[q] += o[q];
        store8<T>(dst, a);
      } else {
        *(uint4*)dst = v;
      }
    }
  }
  if (with_stats) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wave * NWC + j * 16 + (lane & 15);
      if (lane < 32 && n < N) {
        float* p = args.stats + (size_t)blockIdx.x * 2 * N + (lane < 16 ? 0 : N) + n;
        if (args.fold.on) st_sc1_dw(p, lane < 16 ? st_s[j] : st_q[j]);   // read by the fold's last workgroups
        else *p = lane < 16 ? st_s[j] : st_q[j];
      }
    }
    // BatchNorm finalisation in the launch's tail: one statistics row per workgroup (blockIdx.x) of
    // column block blockIdx.y
    if (args.fold.on) bn_fold_tail<256, NWG>(args.fold, args.stats, N, blockIdx.x, gridDim.x, n0, smem);
  }
}

// --------------------------------------------------------------------------------------------
// Fusion-conv input gradient with the gate backward in its epilogue (dfcsa_dgrad_gate):
//   [dfused | dlocal | dattn] = dy4 . W4t, each bf16-rounded as the unfused GEMM stores them;
//   g = sigmoid(bn3 y3); dlocal += dfused*g; dattn += dfused*(1-g); dz3 = dfused*(local-attn)*g*(1-g)
// plus the BN3-backward sums (sum dz3, sum dz3*xhat3), one partial row per workgroup.  Workgroup
// column block cb owns channels cb*64 .. +63 of all three column blocks (192 GEMM columns =
// weight rows part*C + cb*64 + ch), so dfused stays on chip: the GEMM's 3 writes + the gate
// pass's 6 reads and 3 writes become 3 reads + 3 writes.  Streaming structure of
// conv1x1_stream_kernel (weights in registers, 64-row tiles walked grid-stride, next A image by
// LDS-DMA behind the current tile); the gate inputs of a tile are fetched ahead of its wait.
// Reference: models/unet_dfc_sa_res.py:102-110 (gate, fused, fusion_conv) backward.
// --------------------------------------------------------------------------------------------
struct GateEpi {
  const bf16_t* y3;
  const bf16_t* local;
  const bf16_t* attn;
  const float* sc;
  const float* sh;
  const float* mean;
  const float* invstd;
  bf16_t* dlocal;
  bf16_t* dattn;
  bf16_t* dz3;
  float* part;
};

__device__ __forceinline__ float gate_sigm(float x) { return 1.f / (1.f + __expf(-x)); }  // = block_ew sigm

// A-operand prologue (APRO, C = 64): the A image is DMA'd as [src | y] and turned into the BatchNorm
// backward apply  dy = gamma*invstd * (dz - coef0 - xhat*coef1),  xhat = (y - mean)*invstd, with
// dz = src (plain: dfcsa_bn_bwd_apply) or dz = src * (y*sc + sh > 0) (relu: dfcsa_bn_bwd_apply_relu),
// in LDS; dy is stored once (the weight gradient reads it) and multiplied from LDS.
struct ApplyPro {
  const bf16_t* y;
  const float* gamma;
  const float* coef;     // [2][64]
  const float* mean;
  const float* invstd;
  const float* sc;       // relu mask (nullptr: plain apply)
  const float* sh;
  bf16_t* dy;
};

// F.interpolate(bilinear, align_corners=False) source taps along one axis (= block_ew bilin_axis)
// scale = (float)in / (float)out, computed once on the host (the same correctly rounded quotient)
__device__ __forceinline__ void bilin_axis_c(int dst, int in, float scale, int& i0, int& i1, float& l0, float& l1) {
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  l0 = 1.f - l1;
}

// EPI_GATE: the gate backward above (192 columns: dfused | dlocal | dattn of channel block cb).
// EPI_ACC_RELU_BN (dfcsa_dgrad_acc_relu_bn): the gate conv's input gradient dy3 . W3t ADDED into
// [dlocal | dattn] (128 columns per workgroup; the same bf16 rounding as the accumulate-mode GEMM)
// and, on the final dlocal, the BN1-backward sums of dz1 = dlocal * (y1*sc1 + sh1 > 0) (the sums
// of dfcsa_bwd_relu_bn, whose read of dlocal and y1 it replaces by one read of y1).
enum { EPI_GATE = 0, EPI_ACC_RELU_BN = 1 };

// waves per SIMD the compiler budgets registers for: 2 for the variants whose allocation lands just
// above 256 VGPR+AGPR (one resident workgroup per CU otherwise): the 224^2 gate and acc/apply
// variants (280 and 264) and the 112^2 gate variant (272)
template <int KP, int EPI, bool APRO, bool SB = false>
constexpr int gate_wpe() { return (KP == 64 || (KP == 128 && EPI == 0) || SB) ? 2 : 1; }

// SB (single buffer, KP = 256; knob 44): one A-image slot, two workgroups per CU; the next tile's
// DMA is issued once every wave has finished its MFMA reads and flies during the epilogue
template <int KP, int EPI, bool APRO = false, bool SB = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(gate_wpe<KP, EPI, APRO, SB>())))
dgrad_gate_kernel(const ConvGemmArgs args, const GateEpi e, int mtiles, const ApplyPro ap) {
  using T = bf16_t;
  static_assert(!APRO || KP == 64, "A prologue: C = 64");
  constexpr int NWC = EPI == EPI_GATE ? 48 : 32, FN = NWC / 16, NWG = 4 * NWC;
  constexpr int KS = KP / 64, KG = KP / 32;
  constexpr int KSD = APRO ? 2 * KS : KS;   // K stages DMA'd per tile ([src | y] with the prologue)
  constexpr int IMG = 64 * 128, SLOT = KSD * IMG;
  constexpr int OSTR = NWG * 2 + 16;
  __shared__ __attribute__((aligned(16))) char smem[(SB ? 1 : 2) * SLOT];
  __shared__ __attribute__((aligned(16))) char otile[64 * OSTR];
  __shared__ __attribute__((aligned(16))) float red[4][2][64];
  static_assert(!SB || (!APRO && KP == 256), "single buffer: the non-prologue KP = 256 variants");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = args.M, C = args.Nd, K = args.K;
  const int cb = blockIdx.y;
  const int rsub = lane >> 3;
  const int cchunk = (lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7);

  // B fragments: local column lc = wave*48 + j*16 (+ lane&15) -> weight row (lc/64)*C + cb*64 + lc%64
  bf16x8_t bfr[FN][KG];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int lc = wave * NWC + j * 16;
    const int n = (lc >> 6) * C + cb * 64 + (lc & 63) + (lane & 15);
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      const int k = g * 32 + 8 * (lane >> 4);
      if (k < args.Kpad) bfr[j][g] = *(const bf16x8_t*)((const T*)args.Bw + (size_t)n * args.Kpad + k);
      else bfr[j][g] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  const void* zero = (const void*)g_zero_page;
  const T* a_src[2 * KSD];
#pragma unroll
  for (int i = 0; i < 2 * KSD; ++i) {
    const int st = i >> 1;
    const int k = (st % KS) * 64 + cchunk * 8;
    const T* base = (APRO && st >= KS) ? ap.y : (const T*)args.seg[0].ptr;
    a_src[i] = k < K ? base + k : nullptr;
  }
  auto issue = [&](int t, int slot) {
    char* base = smem + slot * SLOT;
#pragma unroll
    for (int i = 0; i < 2 * KSD; ++i) {
      const int st = i >> 1, rb = (i & 1) * 4 + wave;
      const int m = t * 64 + rb * 8 + rsub;
      const void* src = (m < M && a_src[i]) ? (const void*)(a_src[i] + (size_t)m * K) : zero;
      glds16(src, base + st * IMG + rb * 8 * 128);
    }
  };

  // epilogue items: channel chunk ck (8 channels), rows rr and rr + 32 of each tile
  const int ck = tid & 7, rr = tid >> 3;
  const int c0 = cb * 64 + ck * 8;
  float sc[8], sh[8], mu[8], is[8];
  load8<float>(e.sc + c0, sc);
  load8<float>(e.sh + c0, sh);
  load8<float>(e.mean + c0, mu);
  load8<float>(e.invstd + c0, is);
  float s0[8], s1[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { s0[q] = 0.f; s1[q] = 0.f; }
  // prologue constants of channel chunk ck (C = 64: the epilogue's chunk)
  float agk[8], ak0[8], ak1[8], amu[8], ais[8], asc[8], ash[8];
  if constexpr (APRO) {
    load8<float>(ap.gamma + ck * 8, agk);
    load8<float>(ap.coef + ck * 8, ak0);
    load8<float>(ap.coef + 64 + ck * 8, ak1);
    load8<float>(ap.mean + ck * 8, amu);
    load8<float>(ap.invstd + ck * 8, ais);
    if (ap.sc) { load8<float>(ap.sc + ck * 8, asc); load8<float>(ap.sh + ck * 8, ash); }
#pragma unroll
    for (int q = 0; q < 8; ++q) agk[q] *= ais[q];
  }

  // PIPE: the epilogue inputs of a tile (y3 / local / attn) are loaded one tile ahead, behind that
  // tile's A-image DMA, so the wait before a tile's MFMAs finds them arrived (loaded at the top of
  // the same iteration they cost a full memory latency per tile)
  auto load_pin = [&](int tt, uint4 (&p)[2][3]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = min(tt * 64 + rr + 32 * h, M - 1);
      const size_t off = (size_t)m * C + c0;
      p[h][0] = *(const uint4*)(e.y3 + off);   // y3 (gate) / y1 (acc)
      if constexpr (EPI == EPI_GATE) {
        p[h][1] = *(const uint4*)(e.local + off);
        p[h][2] = *(const uint4*)(e.attn + off);
      } else {   // the destination values the GEMM adds to
        p[h][1] = *(const uint4*)(e.dlocal + off);
        p[h][2] = *(const uint4*)(e.dattn + off);
      }
    }
  };
  // (measured per variant: a gain on the gate epilogue at K <= 128 -- 142.7 -> 133.4 us and
  // 83.2 -> 79.7 us -- and a loss of 2-5 % on the others, whose registers it raises further)
  constexpr bool PIPE = EPI == EPI_GATE && KP <= 128 && !APRO;
  int t = blockIdx.x;
  uint4 pin[2][3], pnx[2][3];
  if (t < mtiles) {
    issue(t, 0);
    if constexpr (PIPE) load_pin(t, pin);
  }
  int slot = 0;
  for (; t < mtiles; t += gridDim.x, slot ^= (SB ? 0 : 1)) {
    const int tn = t + gridDim.x;
    if constexpr (!PIPE) load_pin(t, pin);
    if constexpr (SB) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // DMA(t) was issued in the previous epilogue
    } else if (tn < mtiles) {
      issue(tn, slot ^ 1);
      if constexpr (PIPE) {
        load_pin(tn, pnx);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * KSD + 6) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * KSD) : "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();
    char* img = smem + slot * SLOT;
    if constexpr (APRO) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = rr + 32 * h, m = t * 64 + row;
        const int off = row * 128 + swz(row, ck) * 16;
        float dz[8], y[8], dy[8];
        load8<T>((const T*)(img + off), dz);
        load8<T>((const T*)(img + IMG + off), y);
        if (ap.sc) {
#pragma unroll
          for (int q = 0; q < 8; ++q) dz[q] = (y[q] * asc[q] + ash[q] > 0.f) ? dz[q] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float xh = (y[q] - amu[q]) * ais[q];
          dy[q] = agk[q] * (dz[q] - ak0[q] - xh * ak1[q]);
        }
        store8<T>((T*)(img + off), dy);
        if (m < M) store8<T>(ap.dy + (size_t)m * 64 + ck * 8, dy);
      }
      lds_barrier();
    }
    f32x4_t acc[4][FN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      Frag<T> fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) read_frag<T>(img + (g >> 1) * IMG, i * 16 + (lane & 15), g & 1, lane, fa[i]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].v, bfr[j][g], acc[i][j], 0, 0, 0);
    }
    if constexpr (SB) {
      lds_barrier();   // every wave's fragment reads of the slot are done
      if (tn < mtiles) issue(tn, 0);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wave * NWC + j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *(T*)(otile + (i * 16 + (lane >> 4) * 4 + r) * OSTR + col * 2) = f2bf(acc[i][j][r]);
    }
    lds_barrier();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = rr + 32 * h, m = t * 64 + row;
      if (m >= M) continue;
      const size_t off = (size_t)m * C + c0;
      if constexpr (EPI == EPI_ACC_RELU_BN) {
        float gl[8], ga[8], ol[8], oa[8], y[8];
        load8<T>((const T*)(otile + row * OSTR + ck * 16), gl);
        load8<T>((const T*)(otile + row * OSTR + 128 + ck * 16), ga);
        load8<T>((const T*)&pin[h][0], y);
        load8<T>((const T*)&pin[h][1], ol);
        load8<T>((const T*)&pin[h][2], oa);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          gl[q] = bf2f(f2bf(gl[q] + ol[q]));   // the value stored (and read back by the unfused pass)
          ga[q] += oa[q];
          const float z = (y[q] * sc[q] + sh[q] > 0.f) ? gl[q] : 0.f;
          s0[q] += z;
          s1[q] += z * ((y[q] - mu[q]) * is[q]);
        }
        store8<T>(e.dlocal + off, gl);
        store8<T>(e.dattn + off, ga);
        continue;
      }
      float df[8], dl[8], da[8], y[8], l[8], at[8], dz[8];
      load8<T>((const T*)(otile + row * OSTR + ck * 16), df);
      load8<T>((const T*)(otile + row * OSTR + 128 + ck * 16), dl);
      load8<T>((const T*)(otile + row * OSTR + 256 + ck * 16), da);
      load8<T>((const T*)&pin[h][0], y);
      load8<T>((const T*)&pin[h][1], l);
      load8<T>((const T*)&pin[h][2], at);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float g = gate_sigm(y[q] * sc[q] + sh[q]);
        const float dg = df[q] * (l[q] - at[q]);
        const float z = dg * g * (1.f - g);
        dz[q] = z;
        dl[q] += df[q] * g;
        da[q] += df[q] * (1.f - g);
        s0[q] += z;
        s1[q] += z * ((y[q] - mu[q]) * is[q]);
      }
      store8<T>(e.dlocal + off, dl);
      store8<T>(e.dattn + off, da);
      store8<T>(e.dz3 + off, dz);
    }
    if constexpr (PIPE) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int k = 0; k < 3; ++k) pin[h][k] = pnx[h][k];
    }
  }
  // per-workgroup sums: the 8 row lanes of a wave (butterfly), then the 4 waves in order
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float a0 = s0[q], a1 = s1[q];
    for (int o = 8; o < 64; o <<= 1) { a0 += __shfl_xor(a0, o, 64); a1 += __shfl_xor(a1, o, 64); }
    s0[q] = a0;
    s1[q] = a1;
  }
  if (lane < 8) {
    lds_st8(&red[wave][0][lane * 8], s0);
    lds_st8(&red[wave][1][lane * 8], s1);
  }
  __syncthreads();
  if (tid < 128) {
    const int s = tid >> 6, c = tid & 63;
    e.part[(size_t)blockIdx.x * 2 * C + s * C + cb * 64 + c] =
        (red[0][s][c] + red[1][s][c]) + (red[2][s][c] + red[3][s][c]);
  }
}

template <int KP, int EPI, bool APRO = false, bool SB = false>
int gate_occ() {
  static int occ = 0;
  if (!occ && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, dgrad_gate_kernel<KP, EPI, APRO, SB>, 256, 0) !=
                   hipSuccess ||
               occ < 1))
    occ = 1;
  return occ;
}

// workgroups of one dfcsa_dgrad_gate / _acc_relu_bn launch (= partial rows): every CU's resident
// slots, at most one per tile.  Knob 36: the C / 64 column blocks (grid.y) share the resident
// slots (grid.x = slots / column blocks), so every workgroup is resident from the start and loads
// its weight fragments once, instead of C / 64 successive grids of slot-many workgroups (0 = old).
// Same-box A/B (tools/gpu_r04_gate36.sh): the C = 256 kernels 105 -> 88 and 68 -> 51 us, C = 128
// acc 60 -> 54 us; step 1587 / 1597 / 1602 -> 1604 / 1607 / 1609 img/s.
int g_gate_grid_div = 1;   // knob 36
int g_gate_sb = 0;   // knob 44: 1 = the single-buffer KP = 256 gate dgrad kernels (two workgroups per CU)
template <int EPI>
int dgrad_gate_grid(int M, int C, bool apro = false) {
  const int kp = (C + 63) / 64 * 64;
  const int occ = apro ? gate_occ<64, EPI, true>() : kp == 64 ? gate_occ<64, EPI>() : kp == 128 ? gate_occ<128, EPI>()
                  : kp == 192 ? gate_occ<192, EPI>() : g_gate_sb ? gate_occ<256, EPI, false, true>()
                                                                 : gate_occ<256, EPI>();
  const int mtiles = (M + 63) / 64;
  int gx = 256 * occ;
  if (g_gate_grid_div) gx = std::max(1, gx / ((C + 63) / 64));
  return gx > mtiles ? mtiles : gx;
}

// --------------------------------------------------------------------------------------------
// Fusion conv forward with the gate fusion in its A-operand prologue (dfcsa_gate_fusion_fwd,
// C = 64): the A image of a 64-row tile is DMA'd as [y3 | local | attn] (three 64-channel K
// stages); after it lands, each lane turns its two (row, 8-channel) chunks of the y3 stage into
//   fused = g*local + (1-g)*attn,  g = sigmoid(y3*sc3 + sh3)        (dfcsa_gate_fuse's arithmetic)
// in place in LDS (and stores them: the fusion conv's weight gradient reads `fused`), then the
// tile is multiplied as by conv1x1_stream_kernel: y4 = [fused|local|attn] . W4^T + b4 with the
// BN4 partial statistics per 64-row tile.  The separate gate-fusion pass (3 reads + 1 write) and
// the GEMM's re-read of `fused` become one pass.  Reference models/unet_dfc_sa_res.py:102-110.
// --------------------------------------------------------------------------------------------
// PRO_GATE_FUSION (above).  PRO_LOCAL_ATTN (dfcsa_local_attn_gate_fwd): the gate conv, A = [y1 | y2]
// DMA'd; the prologue forms local = relu(bn1 y1) and attn = gamma * bilinear(o) + relu(bn2 y2)
// (dfcsa_block_local_attn's arithmetic) in place and stores both; then y3 = [local|attn] . W3^T + b3
// with BN3 statistics.  The o taps of a lane's two pixels are loaded ahead of the tile's wait.
enum { PRO_GATE_FUSION = 0, PRO_LOCAL_ATTN = 1 };

struct FwdPro {
  const float* sc0;   // gate fusion: bn3; local/attn: bn1
  const float* sh0;
  const float* sc1;   // local/attn: bn2
  const float* sh1;
  const float* o;     // [B][P][P][64] fp32 LightSelfAttention output
  const float* gamma;
  int P, H, W;
  bf16_t* out0;       // fused / local
  bf16_t* out1;       // - / attn
  DivMod dm_hw, dm_w; // pixel -> (image, row, column) by multiply-shift
  float sh, sw;       // bilinear source scales P / H, P / W
};

// SB (single buffer, C = 128; knob 43): one A-image slot instead of two, so two workgroups fit per
// CU (65 instead of 113 KiB of LDS); the next tile's DMA is issued once every wave has finished its
// MFMA reads of the slot and flies during the epilogue
// waves per SIMD the compiler budgets registers for (knob-free): 2 for the single-buffer C = 128 gate
// fusion (284 VGPR+AGPR unconstrained: one wave per SIMD, one workgroup per CU whatever its LDS)
template <int PRO, int C, bool SB>
constexpr int pro_wpe() { return (SB && PRO == 0 && C == 128) ? 2 : 1; }

template <int PRO, int C, bool SB = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(pro_wpe<PRO, C, SB>())))
gate_fusion_fwd_kernel(const ConvGemmArgs args, const FwdPro pr_, int mtiles) {
  using T = bf16_t;
  static_assert(C == 64 || C == 128, "prologue GEMM widths");
  constexpr int NSEG = PRO == PRO_GATE_FUSION ? 3 : 2;
  constexpr int SPS = C / 64;                       // 64-channel K stages per source
  constexpr int KS = NSEG * SPS, KG = 2 * KS;
  constexpr int NWC = C / 4, FN = NWC / 16, NWG = C;  // all C output columns in one workgroup
  constexpr int CPR = C / 8;                        // 8-channel chunks per pixel row
  constexpr int RSTEP = 256 / CPR, NITEM = 64 / RSTEP;   // prologue rows per pass, items per lane
  constexpr int NOUT = PRO == PRO_GATE_FUSION ? 1 : 2;   // prologue stores per item
  constexpr int IMG = 64 * 128, SLOT = KS * IMG;
  constexpr int OSTR = NWG * 2 + 16;
  constexpr int NSTORE = (64 * (NWG / 8)) / 256, OCH = NWG / 8;
  __shared__ __attribute__((aligned(16))) char smem[(SB ? 1 : 2) * SLOT];
  __shared__ __attribute__((aligned(16))) char otile[64 * OSTR];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = args.M;
  const int rsub = lane >> 3;
  const int cchunk = (lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7);
  bf16x8_t bfr[FN][KG];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = wave * NWC + j * 16 + (lane & 15);
#pragma unroll
    for (int g = 0; g < KG; ++g)
      bfr[j][g] = *(const bf16x8_t*)((const T*)args.Bw + (size_t)n * args.Kpad + g * 32 + 8 * (lane >> 4));
  }
  float bias[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bias[j] = args.bias ? args.bias[wave * NWC + j * 16 + (lane & 15)] : 0.f;
  const void* zero = (const void*)g_zero_page;
  // K stage st = source (st / SPS), channels (st % SPS) * 64 ..
  const T* a_src[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) a_src[i] = (const T*)args.seg[i / SPS].ptr + (i % SPS) * 64 + cchunk * 8;
  auto issue = [&](int t, int slot) {
    char* base = smem + slot * SLOT;
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i) {
      const int st = i >> 1, rb = (i & 1) * 4 + wave;
      const int m = t * 64 + rb * 8 + rsub;
      const void* src = m < M ? (const void*)(a_src[st] + (size_t)m * C) : zero;
      glds16(src, base + st * IMG + rb * 8 * 128);
    }
  };
  // prologue items: chunk pc (channels pc*8 ..) of rows pr + k*RSTEP; the chunk lives in K stage
  // (source*SPS + pc/8) at logical 16-B chunk pc%8 of the row
  const int pc = tid % CPR, pr = tid / CPR;
  const int pst = pc >> 3, pch = pc & 7;
  float sc[8], sh[8], sc2[8], sh2[8];
  load8<float>(pr_.sc0 + pc * 8, sc);
  load8<float>(pr_.sh0 + pc * 8, sh);
  float gam = 0.f;
  if constexpr (PRO == PRO_LOCAL_ATTN) {
    load8<float>(pr_.sc1 + pc * 8, sc2);
    load8<float>(pr_.sh1 + pc * 8, sh2);
    gam = *pr_.gamma;
  }
  T* o_base[NSTORE];
  int o_row[NSTORE];
#pragma unroll
  for (int it = 0; it < NSTORE; ++it) {
    const int e = tid + it * 256;
    o_row[it] = e / OCH;
    o_base[it] = (T*)args.dest[0] + (e - o_row[it] * OCH) * 8;
  }
  float st_s[FN], st_q[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) { st_s[j] = 0.f; st_q[j] = 0.f; }
  int t = blockIdx.x;
  if (t >= mtiles) return;   // never: the grid is at most one workgroup per tile
  issue(t, 0);
  int slot = 0;
  bool first_iter = true;
  for (; t < mtiles; t += gridDim.x, slot ^= (SB ? 0 : 1)) {
    const int tn = t + gridDim.x;
    // LightSelfAttention taps of this tile's pixels, loaded before the next tile's DMA
    float ov[NITEM][4][8], lw[NITEM][4];
    if constexpr (PRO == PRO_LOCAL_ATTN) {
#pragma unroll
      for (int h = 0; h < NITEM; ++h) {
        const int m = min(t * 64 + pr + RSTEP * h, M - 1);
        const int b = dm_div(pr_.dm_hw, m), rem = m - b * pr_.dm_hw.d, hh = dm_div(pr_.dm_w, rem), ww = rem - hh * pr_.W;
        int h0, h1, w0, w1;
        float lh0, lh1, lw0, lw1;
        bilin_axis_c(hh, pr_.P, pr_.sh, h0, h1, lh0, lh1);
        bilin_axis_c(ww, pr_.P, pr_.sw, w0, w1, lw0, lw1);
        const float* ob = pr_.o + (size_t)b * pr_.P * pr_.P * C + pc * 8;
        load8<float>(ob + (size_t)(h0 * pr_.P + w0) * C, ov[h][0]);
        load8<float>(ob + (size_t)(h0 * pr_.P + w1) * C, ov[h][1]);
        load8<float>(ob + (size_t)(h1 * pr_.P + w0) * C, ov[h][2]);
        load8<float>(ob + (size_t)(h1 * pr_.P + w1) * C, ov[h][3]);
        lw[h][0] = lh0; lw[h][1] = lh1; lw[h][2] = lw0; lw[h][3] = lw1;
      }
    }
    // outstanding, in issue order: DMA(t), [o taps], the previous tile's prologue + FN stats +
    // NSTORE output stores (no stats stores: kept in registers), DMA(tn): the counted wait retires DMA(t)
    if constexpr (SB) {
      // this tile's DMA was issued during the previous tile's epilogue (or before the loop)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (PRO == PRO_GATE_FUSION) {   // no loads besides the DMAs: leave the stores in flight
      if (tn < mtiles) {
        issue(tn, slot ^ 1);
        if (first_iter) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * KS) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * KS + NITEM * NOUT + NSTORE) : "memory");
      } else {
        if (first_iter) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NITEM * NOUT + NSTORE) : "memory");
      }
    } else {
      if (tn < mtiles) {
        issue(tn, slot ^ 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * KS) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    first_iter = false;
    lds_barrier();
    char* img = smem + slot * SLOT;
#pragma unroll
    for (int h = 0; h < NITEM; ++h) {
      const int row = pr + RSTEP * h, m = t * 64 + row;
      const int off = row * 128 + swz(row, pch) * 16;
      char* i0 = img + pst * IMG + off;                 // source 0 stage of this chunk
      char* i1 = i0 + SPS * IMG;                        // source 1
      float y[8], l[8], f[8];
      load8<T>((const T*)i0, y);
      load8<T>((const T*)i1, l);
      T* sink = (T*)(g_store_sink + 4 * (tid & 63));
      if constexpr (PRO == PRO_GATE_FUSION) {
        float at[8];
        load8<T>((const T*)(i1 + SPS * IMG), at);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float g = gate_sigm(y[q] * sc[q] + sh[q]);
          f[q] = g * l[q] + (1.f - g) * at[q];
        }
        store8<T>((T*)i0, f);
        // one store per item whatever m (rows past M go to the sink): a fixed count per tile
        store8<T>(m < M ? pr_.out0 + (size_t)m * C + pc * 8 : sink, f);
      } else {
        float a2[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          f[q] = fmaxf(y[q] * sc[q] + sh[q], 0.f);
          const float upv = lw[h][0] * (lw[h][2] * ov[h][0][q] + lw[h][3] * ov[h][1][q]) +
                            lw[h][1] * (lw[h][2] * ov[h][2][q] + lw[h][3] * ov[h][3][q]);
          const float v = l[q] * sc2[q] + sh2[q];
          a2[q] = gam * upv + fmaxf(v, 0.f);
        }
        store8<T>((T*)i0, f);
        store8<T>((T*)i1, a2);
        store8<T>(m < M ? pr_.out0 + (size_t)m * C + pc * 8 : sink, f);
        store8<T>(m < M ? pr_.out1 + (size_t)m * C + pc * 8 : sink, a2);
      }
    }
    lds_barrier();
    f32x4_t acc[4][FN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      Frag<T> fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) read_frag<T>(img + (g >> 1) * IMG, i * 16 + (lane & 15), g & 1, lane, fa[i]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].v, bfr[j][g], acc[i][j], 0, 0, 0);
    }
    if constexpr (SB) {
      lds_barrier();   // every wave's fragment reads of the slot are done
      if (tn < mtiles) issue(tn, 0);
    }
    const int m0 = t * 64;
    // BatchNorm partial sums of this workgroup's tiles, kept in registers (one slab row per
    // workgroup, written after the loop: the finalize then reads gridDim.x rows, not M/64)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          const float v = m < M ? acc[i][j][r] : 0.f;
          s += v;
          q += v * v;
        }
      s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
      st_s[j] += s;
      st_q[j] += q;
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wave * NWC + j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *(T*)(otile + (i * 16 + (lane >> 4) * 4 + r) * OSTR + col * 2) = f2bf(acc[i][j][r] + bias[j]);
    }
    lds_barrier();
#pragma unroll
    for (int it = 0; it < NSTORE; ++it) {
      const int e = tid + it * 256;
      const int row = o_row[it], cc = e - row * OCH;
      const int m = m0 + row;
      const uint4 v = *(const uint4*)(otile + row * OSTR + cc * 16);
      T* dst = m < M ? o_base[it] + (size_t)m * C : (T*)(g_store_sink + 4 * (tid & 63));
      *(uint4*)dst = v;
    }
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = wave * NWC + j * 16 + (lane & 15);
    if (lane < 32) {
      float* sp = args.stats + (size_t)blockIdx.x * 2 * C + (lane < 16 ? 0 : C) + n;
      if (args.fold.on) st_sc1_dw(sp, lane < 16 ? st_s[j] : st_q[j]);   // read by the fold's last workgroups
      else *sp = lane < 16 ? st_s[j] : st_q[j];
    }
  }
  // the BatchNorm of the C output columns finalised in the launch's tail (round 5): one
  // statistics row per workgroup, one column block of C
  if (args.fold.on) bn_fold_tail<256, C>(args.fold, args.stats, C, blockIdx.x, gridDim.x, 0, smem);
}

int g_stream_wgs = 0;   // workgroups per CU of the streaming kernel (0 = occupancy limit)
int g_debug = -1;
int g_stream_force = 0;  // knob 5: take the streaming kernel whenever it applies (tests)

template <int NWC, int KP>
int launch_stream(const ConvGemmArgs& a, hipStream_t st) {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv1x1_stream_kernel<NWC, KP, false>, 256, 0) != hipSuccess ||
        occ < 1)
      occ = 1;
  }
  const int mtiles = (a.M + 63) / 64;
  const int ny = (a.N + 4 * NWC - 1) / (4 * NWC);
  const int per_cu = g_stream_wgs > 0 ? g_stream_wgs : occ;
  int gx = (256 * per_cu + ny - 1) / ny;
  if (gx > mtiles) gx = mtiles;
  if (t_dry_rows) { *t_dry_rows = gx; if (t_dry_bn) *t_dry_bn = 4 * NWC; return 0; }   // one statistics row per workgroup column
  if (g_debug) fprintf(stderr, "[dfcsa] stream1x1 NWC=%d KP=%d occ=%d grid=%dx%d tiles=%d\n", NWC, KP, occ, gx, ny, mtiles);
  bool shifted = false;
  for (int i = 0; i < a.nseg; ++i) shifted = shifted || a.seg[i].dh || a.seg[i].dw;
  if (a.mode == CONV_STORE_SHUFFLE2) {
    if (a.accumulate || shifted) return DFCSA_EINVAL;
    hipLaunchKernelGGL((conv1x1_stream_kernel<NWC, KP, false, false, true>), dim3(gx, ny), dim3(256), 0, st, a, mtiles);
  } else if (shifted) {
    if (a.accumulate) return DFCSA_EINVAL;
    hipLaunchKernelGGL((conv1x1_stream_kernel<NWC, KP, false, true>), dim3(gx, ny), dim3(256), 0, st, a, mtiles);
  } else if (a.accumulate)
    hipLaunchKernelGGL((conv1x1_stream_kernel<NWC, KP, true>), dim3(gx, ny), dim3(256), 0, st, a, mtiles);
  else
    hipLaunchKernelGGL((conv1x1_stream_kernel<NWC, KP, false>), dim3(gx, ny), dim3(256), 0, st, a, mtiles);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// the streaming kernel serves 1x1 (no shift, stride 1, plain store) bf16 GEMMs with K <= 256
// (and, knob 30 on, the shifted-segment 3x3 with 9 * Cin <= 256: the first layer, Cin = 8)
int g_stream_shift = 1;   // knob 30
int g_stream_min_m = 4 * 64 * 256;   // knob 33: smallest M the streaming kernel takes
int g_stream_shuf = 1;               // knob 34: ConvTranspose2d (shuffle-store) GEMMs on the streaming kernel
bool stream_applies(const ConvGemmArgs& a) {
  const bool shuf = a.mode == CONV_STORE_SHUFFLE2 && g_stream_shuf && !a.accumulate && a.Nd % 8 == 0 &&
                    a.ndest == 1 && a.Hout == 2 * a.Ho && a.Wout == 2 * a.Wo;
  // M >= knob 33, or half of it with N >= 512 (the 56^2 N = 512 GEMMs and ConvTranspose: 25 / 32 / 30 us
  // against 28 / 35 / 38 us on the tile kernel since two K = 256 workgroups fit per CU,
  // profiles/r04d_ab_stream_otile.txt; N = 256 and the 28^2 shapes stay on the tile kernel)
  const bool big = a.M >= g_stream_min_m || (a.M >= g_stream_min_m / 2 && a.N >= 512);
  if ((a.mode != CONV_STORE_PLAIN && !shuf) || a.stride != 1 || a.Kpad > 256 || !big) return false;
  if (shuf)
    for (int i = 0; i < a.nseg; ++i)
      if (a.seg[i].dh || a.seg[i].dw) return false;
  bool shifted = false;
  for (int i = 0; i < a.nseg; ++i) shifted = shifted || a.seg[i].dh || a.seg[i].dw;
  if (shifted && (!g_stream_shift || a.accumulate || a.Cseg % 8)) return false;
  return a.Ho == a.Hi && a.Wo == a.Wi;
}

int try_stream(const ConvGemmArgs& a, hipStream_t st) {
  if (g_debug < 0) g_debug = getenv("DFCSA_DEBUG") ? 1 : 0;
  // measured (tools/stream_bench.py, B=16 shapes): since the streaming loop keeps its stores in
  // flight (fixed per-lane store counts, LDS-only barriers, hoisted argument-table reads) it is
  // at least as fast as the tile kernels on every 1x1 shape it serves (L1 N=64 K=128: 52 vs 77 us,
  // 3 destinations K=64: 96 vs 181 us), so it takes all of them
  (void)g_stream_force;
  if (!stream_applies(a)) return 1;
  // per-wave columns: register budget NWC/16 * KP/32 <= 16 fragments
  const int kp = a.Kpad;
  auto pick = [&](int nwc) {
    switch (kp) {
      case 64: return nwc == 16 ? launch_stream<16, 64>(a, st) : nwc == 32 ? launch_stream<32, 64>(a, st)
                      : nwc == 48 ? launch_stream<48, 64>(a, st) : launch_stream<64, 64>(a, st);
      case 128: return nwc == 16 ? launch_stream<16, 128>(a, st) : nwc == 32 ? launch_stream<32, 128>(a, st)
                      : nwc == 48 ? launch_stream<48, 128>(a, st) : launch_stream<64, 128>(a, st);
      case 192: return nwc == 16 ? launch_stream<16, 192>(a, st) : launch_stream<32, 192>(a, st);
      default: return nwc == 16 ? launch_stream<16, 256>(a, st) : launch_stream<32, 256>(a, st);
    }
  };
  const int maxf = 16 / (kp / 32);           // column fragments per wave that fit
  int nwc = 16;
  for (int c : {64, 48, 32, 16})
    if (c / 16 <= maxf && (a.N % (4 * c) == 0 || (c == 16))) { nwc = c; break; }
  if (kp >= 192 && nwc > 32) nwc = 32;
  return pick(nwc);
}

int g_conv_dbg = 0;  // knob 15: timing experiments (ConvGemmArgs::dbg)
int g_conv_cfg = 0;  // tuning override (dfcsa_set_tuning knob 1; 7 = no streaming 1x1 kernel)

// config ids: 1 reg 128x64, 2 reg 128x128, 3 dma 128x64, 4 dma 256x64, 5 dma 128x128, 6 dma 256x128
bool shifts_small(const ConvGemmArgs& a) {  // LDS-DMA kernels: segment shifts in [-1, 1]
  for (int i = 0; i < a.nseg; ++i)
    if (a.seg[i].dh < -1 || a.seg[i].dh > 1 || a.seg[i].dw < -1 || a.seg[i].dw > 1) return false;
  return true;
}

template <typename T>
int launch_t(const ConvGemmArgs& a, hipStream_t st) {
  if constexpr (sizeof(T) == 2) {
    switch (g_conv_cfg) {
      case 1: return launch_cfg<T, 128, 64, 4, 1>(a, st);
      case 2: return launch_cfg<T, 128, 128, 2, 2>(a, st);
      default: break;
    }
    // LDS-DMA kernels need shifts in [-1, 1] and 64-aligned segments (scalar address
    // generation); everything else (the 8-channel first layer) takes the register-staged tile
    // (the LDS-DMA tile kernel addresses its sources and weights with 32-bit buffer offsets)
    const bool glds_ok = shifts_small(a) && a.Cseg % 64 == 0 &&
                         (int64_t)(a.M / (a.Ho * a.Wo)) * a.Hi * a.Wi * a.Cseg * 2 < (1ll << 31) &&
                         (int64_t)a.N * a.Kpad * 2 < (1ll << 31);
    if (glds_ok) {
      switch (g_conv_cfg) {
        case 3: return launch_glds<128, 64, 2, 1>(a, st);
        case 4: return launch_glds<256, 64, 4, 1>(a, st);
        case 5: return launch_glds<128, 128, 2, 2>(a, st);
        case 6: return launch_glds<256, 128, 2, 2>(a, st);
        case 8: return launch_glds<128, 128, 2, 2, 3>(a, st);
        case 9: return launch_glds<128, 128, 2, 2, 4>(a, st);
        case 10: return launch_glds<256, 128, 4, 2, 3>(a, st);
        case 11: return launch_glds<256, 64, 4, 1, 3>(a, st);
        case 12: return launch_glds<128, 64, 2, 1, 4>(a, st);
        case 13: return launch_glds<256, 128, 4, 2, 2>(a, st);
        case 14: return launch_glds<128, 128, 4, 2, 2>(a, st);
        case 15: return launch_glds<128, 64, 4, 1, 2>(a, st);
        case 16: return launch_glds<128, 128, 4, 2, 3>(a, st);
        case 17: return launch_glds<256, 64, 8, 1, 2>(a, st);
        case 18: return launch_glds<256, 128, 8, 2, 2>(a, st);
        case 19: return launch_glds<64, 64, 2, 2, 2>(a, st);
        case 20: if (a.N % 256 == 0) return launch_pp<1, true, false>(a, st); break;
        case 21: if (a.N % 256 == 0) return launch_pp<1, true, true>(a, st); break;
        case 22: if (a.N % 256 == 0) return launch_pp<2, true, false>(a, st); break;
        case 23: if (a.N % 256 == 0) return launch_pp<2, false, true>(a, st); break;
        case 24: if (a.N % 256 == 0) return launch_pp<1, false, false>(a, st); break;
        case 25: if (a.N % 256 == 0) return launch_pp<2, true, true>(a, st); break;
        case 41: if ((a.kwork || t_dry_work) && a.N % 256 == 0) { const int gg = g_ppsk; g_ppsk = 1;
                   const bool ok = ppsk_applies(a); g_ppsk = gg; if (ok) return launch_ppsk(a, st); } break;
        case 29: { int ks, kp; const int g = g_splitk; g_splitk = 1; splitk_plan(a, &ks, &kp); g_splitk = g;
                   if (ks > 1 && (a.kwork || t_dry_work)) return launch_splitk(a, ks, kp, st); break; }
        case 30: return launch_glds32<128, 128, 4, 2, 4>(a, st);
        case 31: return launch_glds32<128, 128, 2, 2, 4>(a, st);
        case 32: return launch_glds32<128, 128, 4, 2, 5>(a, st);
        case 34: return launch_glds32<128, 64, 4, 1, 4>(a, st);
        case 35: return launch_glds32<128, 128, 4, 2, 3>(a, st);
        case 36: return launch_glds32<128, 128, 4, 2, 2>(a, st);
        case 37: return launch_glds32<128, 128, 2, 2, 2>(a, st);
        default: break;
      }
    }
    // measured on MI355X (tools/gemm_bench.py, the model's B=16 shapes): 8-wave LDS-DMA tiles
    // (waves of 32x64) beat 4-wave 64x64 ones -- twice the waves per SIMD hide the LDS and
    // DMA latency: 128x128/8 waves 690-730 TF on the 3x3 convs (vs ~600), 128x64/4 waves for
    // N <= 64 (530 TF on the L1 3x3, equal to the register-staged tile on the small-K 1x1s).
    if (g_conv_cfg == 0) {   // 3x3 fwd / fused dgrad with M >= knob 19: 2-D halo tiles
      HaloArgs h;
      int tw, tr;
      if (halo_plan(a, &h, &tw, &tr)) return launch_halo(h, tw, st);
    }
    if (g_conv_cfg != 7 && try_stream(a, st) == 0) return 0;
    if (!glds_ok) return a.N <= 64 ? launch_cfg<T, 128, 64, 4, 1>(a, st) : launch_cfg<T, 128, 128, 2, 2>(a, st);
    // few 128x128 tiles and a long K: split the K range (fixed-order reduction in the epilogue
    // launch; measured against the 64x64 / 128x64 tiles in profiles/r03b_splitk.jsonl)
    if (a.N > 64 && (a.kwork || t_dry_work)) {
      int ks, kp;
      splitk_plan(a, &ks, &kp);
      if (ks > 1) return launch_splitk(a, ks, kp, st);
    }
    // stream-K ping-pong tiles where whole 256x256 tiles leave a partial wave (the 28^2 / 56^2
    // grids of 98 / 196 / 392 tiles): every CU runs the same number of K-tiles
    if ((a.kwork || t_dry_work) && ppsk_applies(a)) return launch_ppsk(a, st);
    // N <= 64 with many rows: 256x64 / 8 waves (wave tile 32x64, twice the rows per B panel);
    // fewer than one workgroup of 128x128 per CU (the 14^2 level, 28^2 with N <= 256): 128x64 doubles the
    // workgroup count (gemm_bench: bottleneck dgrad 123 -> 108 us, bottleneck fwd 59 -> 52 us).
    if (a.N <= 64) return a.M >= 65536 ? launch_glds<256, 64, 8, 1, 2>(a, st) : launch_glds<128, 64, 4, 1, 2>(a, st);
    // 256x256 ping-pong tiles (one workgroup per CU: half the L2->LDS bytes per flop of two
    // 128x128 workgroups) wherever they still give >= 150 workgroups and a long K: measured
    // (tools/pp_check.py) 1.06-1.23x the 128x128 tile on the 3x3 fwd/dgrad of the 112^2-28^2
    // levels, slower below ~150 workgroups (one partial wave of tiles) and at K < 2048 (round 2:
    // the 112^2 decoder dgrad, K = 1408: 204 vs 175 us for the 128x128 tile; K = 1152: equal)
    if (a.N % 256 == 0 && a.K >= 2048 && ((a.M + 255) / 256) * (a.N / 256) >= 150)
      return launch_pp<2, true, false>(a, st);
    // the 14^2 bottleneck 3x3 fwd / dgrad (M = 3136, K >= 4608): 64x64 tiles give 392-784
    // workgroups instead of 200-400 (tools/gemm_bench.py round 2: 111 -> 102 us, 51 -> 48 us)
    if (a.M <= 4096 && a.N >= 512 && a.K >= 4096) return launch_glds<64, 64, 2, 2, 2>(a, st);
    if (((a.M + 127) / 128) * ((a.N + 127) / 128) < 256) {
      // still under one 128x64 workgroup per CU with a short K (the ViT GEMMs of TransUNet:
      // M = 8 x 196 rows, K = 768 / 3072): 64x64 tiles (4 waves of 32x32) double the workgroups
      // again (config 4: 499 -> 511 img/s).  Long-K GEMMs (the 14^2 3x3 dgrads) keep 128x64.
      if (a.K <= 3072 && ((a.M + 127) / 128) * ((a.N + 63) / 64) < 256)
        return launch_glds<64, 64, 2, 2, 2>(a, st);
      return launch_glds<128, 64, 4, 1, 2>(a, st);
    }
    return launch_glds<128, 128, 4, 2, 2>(a, st);
  }
  // fp32 (parity mode + the fp32 LightSelfAttention projections): few rows (M = B*P*P) -> the
  // split-reduction small-M kernel; other small problems get 64x64 tiles
  if (g_conv_cfg != 26 && small_conv_applies(a)) {
    if (t_dry_rows) { *t_dry_rows = 0; return 0; }   // (no statistics)
    const dim3 sg((a.M + 15) / 16, (a.N + 63) / 64);
    if (a.K >= 256 && g_small8) hipLaunchKernelGGL((small_conv_f32_kernel<8, 4>), sg, dim3(512), 0, st, a);
    else hipLaunchKernelGGL((small_conv_f32_kernel<4, 2>), sg, dim3(256), 0, st, a);
    DFCSA_CHECK_LAUNCH();
    return 0;
  }
  const int t128 = ((a.M + 127) / 128) * ((a.N + 127) / 128);
  if (t128 < 128) return launch_cfg<T, 64, 64, 2, 2>(a, st);
  if (a.N <= 64) return launch_cfg<T, 128, 64, 4, 1>(a, st);
  return launch_cfg<T, 128, 128, 2, 2>(a, st);
}

}  // namespace

namespace {
thread_local int t_fold_cw = 0;   // desc_args: the fold block width of the picked kernel (0: no fold)
// descriptor -> kernel arguments (validated); the statistics row count of the launch in *rows
int desc_args(const dfcsa_conv_desc* d, ConvGemmArgs& a, int* rows) {
  if (!d || d->nseg < 1 || d->nseg > DFCSA_MAX_SEG || d->M <= 0 || d->N <= 0) return DFCSA_EINVAL;
  const int chunk = d->dtype == DFCSA_DT_BF16 ? 8 : 4;
  const int kst = d->dtype == DFCSA_DT_BF16 ? 64 : 32;
  if (d->Cseg % chunk || d->Kpad % kst || d->Kpad < d->nseg * d->Cseg) return DFCSA_EINVAL;
  if (d->ndest < 1 || d->ndest > 3 || d->Nd % 8 || (d->mode == CONV_STORE_PLAIN && d->Nd * d->ndest != d->N))
    return DFCSA_EINVAL;
  if (d->mode == CONV_STORE_SHUFFLE2 && (d->ndest != 1 || d->N != 4 * d->Nd)) return DFCSA_EINVAL;
  std::memset(&a, 0, sizeof(a));
  a.M = d->M; a.N = d->N; a.K = d->nseg * d->Cseg; a.Kpad = d->Kpad; a.Cseg = d->Cseg;
  a.nseg = d->nseg;
  for (int i = 0; i < d->nseg; ++i) { a.seg[i].ptr = d->seg_ptr[i]; a.seg[i].dh = d->seg_dh[i]; a.seg[i].dw = d->seg_dw[i]; }
  a.Ho = d->Ho; a.Wo = d->Wo; a.Hi = d->Hi; a.Wi = d->Wi; a.stride = d->stride;
  a.dm_hw = make_divmod(d->Ho * d->Wo);
  a.dm_w = make_divmod(d->Wo);
  a.dm_cseg = make_divmod(d->Cseg);
  a.Bw = d->weight; a.bias = d->bias;
  a.mode = d->mode; a.ndest = d->ndest; a.Nd = d->Nd;
  for (int i = 0; i < 3; ++i) a.dest[i] = i < d->ndest ? d->dest[i] : nullptr;
  a.accumulate = d->accumulate; a.stats = d->stats;
  a.Hout = d->Hout; a.Wout = d->Wout;
  a.dbg = g_conv_dbg;
  a.kwork = d->work;
  a.kwork_floats = d->work ? d->work_floats : 0;
  // statistics rows of the kernel launch_t picks (a dry run of the selection)
  int r = 0, bw = 0;
  t_dry_rows = &r;
  t_dry_bn = &bw;
  if (d->dtype == DFCSA_DT_BF16) launch_t<bf16_t>(a, nullptr);
  else launch_t<float>(a, nullptr);
  t_dry_rows = nullptr;
  t_dry_bn = nullptr;
  *rows = r;
  t_fold_cw = bw;
  return 0;
}
}  // namespace

extern "C" int64_t dfcsa_conv_work_floats(const dfcsa_conv_desc* d) {
  ConvGemmArgs a;
  int rows = 0;
  int64_t need = 0;
  t_dry_work = &need;
  const int rc = desc_args(d, a, &rows);
  t_dry_work = nullptr;
  return rc ? rc : need;
}

extern "C" int dfcsa_conv_stats_rows(const dfcsa_conv_desc* d) {
  ConvGemmArgs a;
  int rows = 0;
  const int rc = desc_args(d, a, &rows);
  return rc ? rc : rows;
}

static int conv_launch(const dfcsa_conv_desc* d, const ConvGemmArgs& a, hipStream_t st);

extern "C" int dfcsa_conv_gemm(const dfcsa_conv_desc* d, void* stream) {
  ConvGemmArgs a;
  int rows = 0;
  if (const int rc = desc_args(d, a, &rows)) return rc;
  // statistics slab: [rows][2][N]
  if (d->stats && (int64_t)rows * 2 * d->N > d->stats_floats) return DFCSA_EINVAL;
  return conv_launch(d, a, (hipStream_t)stream);
}

int g_bn_fold = 1;   // knob 39: 0 = never fold the BatchNorm finalisation into the conv epilogue

// BnFold of a launch with `rows` statistics rows and fold column width cw (tickets and hand-off
// scratch from the shared rings); false when the fold is off or the rings cannot serve it
static bool make_fold(const dfcsa_bn_fold* f, int rows, int cw, BnFold& b) {
  std::memset(&b, 0, sizeof(b));
  if (!g_bn_fold || cw <= 0 || rows <= 0) return false;
  b.C = f->C;
  b.cw = cw;
  b.GS = 1;
  while ((int64_t)b.GS * b.GS < rows) ++b.GS;          // ~sqrt(T) rows per group, ~sqrt(T) groups
  b.ng = (rows + b.GS - 1) / b.GS;
  b.ncb = (f->C + cw - 1) / cw;
  b.cnt = dfcsa_ticket_alloc(b.ncb * b.ng + b.ncb);
  b.scr = dfcsa_scratch_alloc((int64_t)b.ncb * b.ng * 2 * cw);
  if (!b.cnt || !b.scr) {
    std::memset(&b, 0, sizeof(b));
    return false;
  }
  b.on = 1;
  b.count = f->count; b.bias = f->conv_bias; b.gamma = f->gamma; b.beta = f->beta;
  b.rmean = f->running_mean; b.rvar = f->running_var; b.nbt = f->num_batches_tracked;
  b.momentum = f->momentum; b.eps = f->eps;
  b.scale = f->scale; b.shift = f->shift; b.mean = f->mean; b.invstd = f->invstd;
  return true;
}

static bool fold_args_ok(const dfcsa_bn_fold* f) {
  return f && f->C > 0 && f->count > 0 && f->gamma && f->beta && f->running_mean && f->running_var && f->scale &&
         f->shift && f->mean && f->invstd;
}

extern "C" int dfcsa_conv_gemm_bn(const dfcsa_conv_desc* d, const dfcsa_bn_fold* f, void* stream) {
  if (!d || !f || !d->stats || f->C <= 0 || f->C > d->N || f->count <= 0 || !f->gamma || !f->beta ||
      !f->running_mean || !f->running_var || !f->scale || !f->shift || !f->mean || !f->invstd)
    return DFCSA_EINVAL;
  ConvGemmArgs a;
  int rows = 0;
  if (const int rc = desc_args(d, a, &rows)) return rc;
  if ((int64_t)rows * 2 * d->N > d->stats_floats) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (make_fold(f, rows, t_fold_cw, a.fold)) return conv_launch(d, a, st);
  // the picked kernel cannot fold (streaming / halo-tile kernels): conv, then the finalize launch
  if (const int rc = conv_launch(d, a, st)) return rc;
  return dfcsa_bn_finalize(d->stats, rows, f->C, d->N, f->count, f->conv_bias, f->gamma, f->beta, f->running_mean,
                           f->running_var, f->num_batches_tracked, f->momentum, f->eps, 1, f->scale, f->shift,
                           f->mean, f->invstd, stream);
}

static int conv_launch(const dfcsa_conv_desc* d, const ConvGemmArgs& a, hipStream_t st) {
  // profiling classes: the 1x1 streaming GEMMs are HBM-bound (their unit is bytes: A and the
  // weight panel read once, the output written once, read too when accumulating); the tile
  // kernels are MFMA-bound (2*M*N*K flop)
  const bool streamed = d->dtype == DFCSA_DT_BF16 && g_conv_cfg != 7 && g_conv_cfg < 1 && stream_applies(a);
  const double sbytes = 2.0 * ((double)a.M * a.Kpad + (double)a.N * a.Kpad + (double)a.M * a.N * (a.accumulate ? 2 : 1));
  ProfScope prof(streamed ? DFCSA_PROF_CONV_STREAM : DFCSA_PROF_CONV_GEMM, st,
                 streamed ? sbytes : 2.0 * a.M * a.N * a.K);
  if (dfcsa_shapelog())
    fprintf(stderr, "SHAPE conv M=%d N=%d K=%d Kpad=%d nseg=%d Cseg=%d Ho=%d Wo=%d acc=%d dt=%d\n", a.M, a.N, a.K,
            a.Kpad, a.nseg, a.Cseg, a.Ho, a.Wo, a.accumulate, d->dtype);
  return d->dtype == DFCSA_DT_BF16 ? launch_t<bf16_t>(a, st) : launch_t<float>(a, st);
}

namespace {

hipStream_t st_of(void* s) { return (hipStream_t)s; }

template <int EPI>
int launch_gate_epi(const ConvGemmArgs& a, const GateEpi& e, int64_t part_cap, hipStream_t st,
                    const ApplyPro* ap = nullptr) {
  const int M = a.M, C = a.Nd, Kpad = a.Kpad;
  const int mtiles = (M + 63) / 64;
  dim3 grid(dgrad_gate_grid<EPI>(M, C, ap != nullptr), C / 64);
  // one [2][C] partial row per workgroup column (blockIdx.x): refuse a slab shorter than the grid
  if ((int64_t)grid.x * 2 * C > part_cap) return DFCSA_EINVAL;
  // [M][C] tensors read + written besides A (with the prologue: y read, dy written)
  const double moved = (EPI == EPI_GATE ? 6.0 : 7.0) + (ap ? 2.0 : 0.0);
  ProfScope prof(DFCSA_PROF_CONV_STREAM, st, 2.0 * ((double)M * Kpad + (double)a.N * Kpad + moved * (double)M * C));
  ApplyPro none;
  std::memset(&none, 0, sizeof(none));
  if (ap) hipLaunchKernelGGL((dgrad_gate_kernel<64, EPI, true>), grid, dim3(256), 0, st, a, e, mtiles, *ap);
  else if (Kpad == 64) hipLaunchKernelGGL((dgrad_gate_kernel<64, EPI>), grid, dim3(256), 0, st, a, e, mtiles, none);
  else if (Kpad == 128) hipLaunchKernelGGL((dgrad_gate_kernel<128, EPI>), grid, dim3(256), 0, st, a, e, mtiles, none);
  else if (Kpad == 192) hipLaunchKernelGGL((dgrad_gate_kernel<192, EPI>), grid, dim3(256), 0, st, a, e, mtiles, none);
  else if (g_gate_sb)
    hipLaunchKernelGGL((dgrad_gate_kernel<256, EPI, false, true>), grid, dim3(256), 0, st, a, e, mtiles, none);
  else hipLaunchKernelGGL((dgrad_gate_kernel<256, EPI>), grid, dim3(256), 0, st, a, e, mtiles, none);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int dfcsa_dgrad_gate_parts(int M, int C) {
  if (M <= 0 || C <= 0) return DFCSA_EINVAL;
  return dgrad_gate_grid<EPI_GATE>(M, C);
}

extern "C" int dfcsa_dgrad_gate(int M, int C, const void* dy4, const void* w4t, int Kpad, const void* y3,
                                const float* sc3, const float* sh3, const float* mean3, const float* invstd3,
                                const void* local, const void* attn, void* dlocal, void* dattn, void* dz3,
                                float* partial, int64_t partial_floats, void* stream) {
  if (M <= 0 || C <= 0 || C % 64 || C > 256 || Kpad != (C + 63) / 64 * 64) return DFCSA_EINVAL;
  if (!dy4 || !w4t || !y3 || !sc3 || !sh3 || !mean3 || !invstd3 || !local || !attn || !dlocal || !dattn || !dz3 ||
      !partial)
    return DFCSA_EINVAL;
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.M = M; a.N = 3 * C; a.K = C; a.Kpad = Kpad; a.Cseg = C; a.nseg = 1; a.Nd = C;
  a.seg[0].ptr = dy4;
  a.Bw = w4t;
  GateEpi e;
  e.y3 = (const bf16_t*)y3; e.local = (const bf16_t*)local; e.attn = (const bf16_t*)attn;
  e.sc = sc3; e.sh = sh3; e.mean = mean3; e.invstd = invstd3;
  e.dlocal = (bf16_t*)dlocal; e.dattn = (bf16_t*)dattn; e.dz3 = (bf16_t*)dz3; e.part = partial;
  return launch_gate_epi<EPI_GATE>(a, e, partial_floats, st_of(stream));
}

extern "C" int dfcsa_dgrad_acc_relu_bn_parts(int M, int C) {
  if (M <= 0 || C <= 0) return DFCSA_EINVAL;
  return dgrad_gate_grid<EPI_ACC_RELU_BN>(M, C);
}

extern "C" int dfcsa_dgrad_acc_relu_bn(int M, int C, const void* dy3, const void* w3t, int Kpad, const void* y1,
                                       const float* sc1, const float* sh1, const float* mean1, const float* invstd1,
                                       void* dlocal, void* dattn, float* partial, int64_t partial_floats, void* stream) {
  if (M <= 0 || C <= 0 || C % 64 || C > 256 || Kpad != (C + 63) / 64 * 64) return DFCSA_EINVAL;
  if (!dy3 || !w3t || !y1 || !sc1 || !sh1 || !mean1 || !invstd1 || !dlocal || !dattn || !partial) return DFCSA_EINVAL;
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.M = M; a.N = 2 * C; a.K = C; a.Kpad = Kpad; a.Cseg = C; a.nseg = 1; a.Nd = C;
  a.seg[0].ptr = dy3;
  a.Bw = w3t;
  GateEpi e;
  std::memset(&e, 0, sizeof(e));
  e.y3 = (const bf16_t*)y1;
  e.sc = sc1; e.sh = sh1; e.mean = mean1; e.invstd = invstd1;
  e.dlocal = (bf16_t*)dlocal; e.dattn = (bf16_t*)dattn; e.part = partial;
  return launch_gate_epi<EPI_ACC_RELU_BN>(a, e, partial_floats, st_of(stream));
}

// dy = BatchNorm-backward apply of [src | y] (relu mask when sc != nullptr) formed in the A prologue
extern "C" int dfcsa_dgrad_gate_apply(int M, const void* dout, const void* y4, const float* gamma4,
                                      const float* coef4, const float* mean4, const float* invstd4,
                                      const float* sc4, const float* sh4, void* dy4, const void* w4t,
                                      const void* y3, const float* sc3, const float* sh3, const float* mean3,
                                      const float* invstd3, const void* local, const void* attn, void* dlocal,
                                      void* dattn, void* dz3, float* partial, int64_t partial_floats, void* stream) {
  const int C = 64, Kpad = 64;
  if (M <= 0 || !dout || !y4 || !gamma4 || !coef4 || !mean4 || !invstd4 || !dy4 || !w4t || !y3 || !sc3 || !sh3 ||
      !mean3 || !invstd3 || !local || !attn || !dlocal || !dattn || !dz3 || !partial || (!sc4 != !sh4))
    return DFCSA_EINVAL;
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.M = M; a.N = 3 * C; a.K = C; a.Kpad = Kpad; a.Cseg = C; a.nseg = 1; a.Nd = C;
  a.seg[0].ptr = dout;
  a.Bw = w4t;
  GateEpi e;
  e.y3 = (const bf16_t*)y3; e.local = (const bf16_t*)local; e.attn = (const bf16_t*)attn;
  e.sc = sc3; e.sh = sh3; e.mean = mean3; e.invstd = invstd3;
  e.dlocal = (bf16_t*)dlocal; e.dattn = (bf16_t*)dattn; e.dz3 = (bf16_t*)dz3; e.part = partial;
  ApplyPro ap;
  ap.y = (const bf16_t*)y4; ap.gamma = gamma4; ap.coef = coef4; ap.mean = mean4; ap.invstd = invstd4;
  ap.sc = sc4; ap.sh = sh4; ap.dy = (bf16_t*)dy4;
  return launch_gate_epi<EPI_GATE>(a, e, partial_floats, (hipStream_t)stream, &ap);
}

extern "C" int dfcsa_dgrad_acc_relu_bn_apply(int M, const void* dz3, const void* y3, const float* gamma3,
                                             const float* coef3, const float* mean3, const float* invstd3,
                                             void* dy3, const void* w3t, const void* y1, const float* sc1,
                                             const float* sh1, const float* mean1, const float* invstd1,
                                             void* dlocal, void* dattn, float* partial, int64_t partial_floats, void* stream) {
  const int C = 64, Kpad = 64;
  if (M <= 0 || !dz3 || !y3 || !gamma3 || !coef3 || !mean3 || !invstd3 || !dy3 || !w3t || !y1 || !sc1 || !sh1 ||
      !mean1 || !invstd1 || !dlocal || !dattn || !partial)
    return DFCSA_EINVAL;
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.M = M; a.N = 2 * C; a.K = C; a.Kpad = Kpad; a.Cseg = C; a.nseg = 1; a.Nd = C;
  a.seg[0].ptr = dz3;
  a.Bw = w3t;
  GateEpi e;
  std::memset(&e, 0, sizeof(e));
  e.y3 = (const bf16_t*)y1;
  e.sc = sc1; e.sh = sh1; e.mean = mean1; e.invstd = invstd1;
  e.dlocal = (bf16_t*)dlocal; e.dattn = (bf16_t*)dattn; e.part = partial;
  ApplyPro ap;
  std::memset(&ap, 0, sizeof(ap));
  ap.y = (const bf16_t*)y3; ap.gamma = gamma3; ap.coef = coef3; ap.mean = mean3; ap.invstd = invstd3;
  ap.dy = (bf16_t*)dy3;
  return launch_gate_epi<EPI_ACC_RELU_BN>(a, e, partial_floats, (hipStream_t)stream, &ap);
}

extern "C" int dfcsa_dgrad_apply_parts(int M, int epi) {
  if (M <= 0) return DFCSA_EINVAL;
  return epi == 0 ? dgrad_gate_grid<EPI_GATE>(M, 64, true) : dgrad_gate_grid<EPI_ACC_RELU_BN>(M, 64, true);
}

namespace {
int g_pro_sb = 1;   // knob 43: 1 = the single-buffer C = 128 prologue GEMMs (two workgroups per CU;
                    // same-box A/B 1644 / 1652 / 1638 vs 1630 / 1632 / 1628 img/s with 0)

template <int PRO, int C, bool SB = false>
int fwd_pro_grid_t(int M) {
  static int occ = 0;
  if (!occ &&
      (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, gate_fusion_fwd_kernel<PRO, C, SB>, 256, 0) != hipSuccess ||
       occ < 1))
    occ = 1;
  return std::min(256 * occ, (M + 63) / 64);
}
template <int PRO, int C>
int fwd_pro_grid(int M) {
  if constexpr (C == 128) {
    if (g_pro_sb) return fwd_pro_grid_t<PRO, C, true>(M);
  }
  return fwd_pro_grid_t<PRO, C>(M);
}

template <int PRO, int C>
int launch_fwd_pro(ConvGemmArgs& a, const FwdPro& pro, int64_t stats_cap, hipStream_t st,
                   const dfcsa_bn_fold* f = nullptr) {
  const int mtiles = (a.M + 63) / 64;
  const int gx = fwd_pro_grid<PRO, C>(a.M);
  // one [2][C] statistics row per workgroup: refuse a slab shorter than the grid
  if ((int64_t)gx * 2 * C > stats_cap) return DFCSA_EINVAL;
  if (f && !make_fold(f, gx, C, a.fold)) {
    // fold off or no ring space: the launch, then the finalize
    if (const int rc = launch_fwd_pro<PRO, C>(a, pro, stats_cap, st)) return rc;
    return dfcsa_bn_finalize(a.stats, gx, f->C, C, f->count, f->conv_bias, f->gamma, f->beta, f->running_mean,
                             f->running_var, f->num_batches_tracked, f->momentum, f->eps, 1, f->scale, f->shift,
                             f->mean, f->invstd, st);
  }
  const double moved = PRO == PRO_GATE_FUSION ? 2.0 : 3.0;   // prologue stores + the output
  ProfScope prof(DFCSA_PROF_CONV_STREAM, st, 2.0 * ((double)a.M * a.Kpad + (double)C * a.Kpad + moved * a.M * C));
  if constexpr (C == 128) {
    if (g_pro_sb) {
      hipLaunchKernelGGL((gate_fusion_fwd_kernel<PRO, C, true>), dim3(gx), dim3(256), 0, st, a, pro, mtiles);
      DFCSA_CHECK_LAUNCH();
      return 0;
    }
  }
  hipLaunchKernelGGL((gate_fusion_fwd_kernel<PRO, C>), dim3(gx), dim3(256), 0, st, a, pro, mtiles);
  DFCSA_CHECK_LAUNCH();
  return 0;
}
}  // namespace

extern "C" int dfcsa_fwd_pro_parts(int M, int C, int pro) {
  if (M <= 0) return DFCSA_EINVAL;
  if (pro == 0 && C == 64) return fwd_pro_grid<PRO_GATE_FUSION, 64>(M);
  if (pro == 0 && C == 128) return fwd_pro_grid<PRO_GATE_FUSION, 128>(M);
  if (pro == 1 && C == 64) return fwd_pro_grid<PRO_LOCAL_ATTN, 64>(M);
  if (pro == 1 && C == 128) return fwd_pro_grid<PRO_LOCAL_ATTN, 128>(M);
  return DFCSA_EINVAL;
}

static int gate_fusion_fwd(int M, int C, const void* y3, const float* sc3, const float* sh3, const void* local,
                           const void* attn, const void* w4, int Kpad, const float* b4, void* fused, void* y4,
                           float* stats4, int64_t stats4_floats, void* stream, const dfcsa_bn_fold* f) {
  if (f && (!fold_args_ok(f) || f->C != C)) return DFCSA_EINVAL;
  if (M <= 0 || (C != 64 && C != 128) || Kpad != 3 * C || !y3 || !sc3 || !sh3 || !local || !attn || !w4 || !fused ||
      !y4 || !stats4)
    return DFCSA_EINVAL;
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.M = M; a.N = C; a.K = 3 * C; a.Kpad = Kpad; a.Cseg = C; a.nseg = 3; a.Nd = C; a.ndest = 1;
  a.seg[0].ptr = y3; a.seg[1].ptr = local; a.seg[2].ptr = attn;
  a.Bw = w4; a.bias = b4; a.dest[0] = y4; a.stats = stats4;
  FwdPro pro;
  std::memset(&pro, 0, sizeof(pro));
  pro.sc0 = sc3; pro.sh0 = sh3; pro.out0 = (bf16_t*)fused;
  return C == 64 ? launch_fwd_pro<PRO_GATE_FUSION, 64>(a, pro, stats4_floats, (hipStream_t)stream, f)
                 : launch_fwd_pro<PRO_GATE_FUSION, 128>(a, pro, stats4_floats, (hipStream_t)stream, f);
}

extern "C" int dfcsa_gate_fusion_fwd(int M, int C, const void* y3, const float* sc3, const float* sh3,
                                     const void* local, const void* attn, const void* w4, int Kpad, const float* b4,
                                     void* fused, void* y4, float* stats4, int64_t stats4_floats, void* stream) {
  return gate_fusion_fwd(M, C, y3, sc3, sh3, local, attn, w4, Kpad, b4, fused, y4, stats4, stats4_floats, stream,
                         nullptr);
}

extern "C" int dfcsa_gate_fusion_fwd_bn(int M, int C, const void* y3, const float* sc3, const float* sh3,
                                        const void* local, const void* attn, const void* w4, int Kpad, const float* b4,
                                        void* fused, void* y4, float* stats4, int64_t stats4_floats,
                                        const dfcsa_bn_fold* f, void* stream) {
  if (!f) return DFCSA_EINVAL;
  return gate_fusion_fwd(M, C, y3, sc3, sh3, local, attn, w4, Kpad, b4, fused, y4, stats4, stats4_floats, stream, f);
}

static int local_attn_gate_fwd(int B, int H, int W, int C, const void* y1, const float* sc1, const float* sh1,
                               const void* y2, const float* sc2, const float* sh2, const float* o, int P,
                               const float* gamma, const void* w3, int Kpad, const float* b3, void* local, void* attn,
                               void* y3, float* stats3, int64_t stats3_floats, void* stream, const dfcsa_bn_fold* f) {
  if (f && (!fold_args_ok(f) || f->C != C)) return DFCSA_EINVAL;
  const int64_t M = (int64_t)B * H * W;
  if (M <= 0 || M >= (1ll << 31) || (C != 64 && C != 128) || Kpad != 2 * C || P <= 0 || !y1 || !sc1 || !sh1 || !y2 || !sc2 ||
      !sh2 || !o || !gamma || !w3 || !local || !attn || !y3 || !stats3)
    return DFCSA_EINVAL;
  ConvGemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.M = (int)M; a.N = C; a.K = 2 * C; a.Kpad = Kpad; a.Cseg = C; a.nseg = 2; a.Nd = C; a.ndest = 1;
  a.seg[0].ptr = y1; a.seg[1].ptr = y2;
  a.Bw = w3; a.bias = b3; a.dest[0] = y3; a.stats = stats3;
  FwdPro pro;
  std::memset(&pro, 0, sizeof(pro));
  pro.sc0 = sc1; pro.sh0 = sh1; pro.sc1 = sc2; pro.sh1 = sh2; pro.o = o; pro.gamma = gamma;
  pro.P = P; pro.H = H; pro.W = W;
  pro.dm_hw = make_divmod(H * W); pro.dm_w = make_divmod(W);
  pro.sh = (float)P / (float)H; pro.sw = (float)P / (float)W;
  pro.out0 = (bf16_t*)local; pro.out1 = (bf16_t*)attn;
  return C == 64 ? launch_fwd_pro<PRO_LOCAL_ATTN, 64>(a, pro, stats3_floats, (hipStream_t)stream, f)
                 : launch_fwd_pro<PRO_LOCAL_ATTN, 128>(a, pro, stats3_floats, (hipStream_t)stream, f);
}

extern "C" int dfcsa_local_attn_gate_fwd(int B, int H, int W, int C, const void* y1, const float* sc1,
                                         const float* sh1, const void* y2, const float* sc2, const float* sh2,
                                         const float* o, int P, const float* gamma, const void* w3, int Kpad,
                                         const float* b3, void* local, void* attn, void* y3, float* stats3, int64_t stats3_floats,
                                         void* stream) {
  return local_attn_gate_fwd(B, H, W, C, y1, sc1, sh1, y2, sc2, sh2, o, P, gamma, w3, Kpad, b3, local, attn, y3,
                             stats3, stats3_floats, stream, nullptr);
}

extern "C" int dfcsa_local_attn_gate_fwd_bn(int B, int H, int W, int C, const void* y1, const float* sc1,
                                            const float* sh1, const void* y2, const float* sc2, const float* sh2,
                                            const float* o, int P, const float* gamma, const void* w3, int Kpad,
                                            const float* b3, void* local, void* attn, void* y3, float* stats3,
                                            int64_t stats3_floats, const dfcsa_bn_fold* f, void* stream) {
  if (!f) return DFCSA_EINVAL;
  return local_attn_gate_fwd(B, H, W, C, y1, sc1, sh1, y2, sc2, sh2, o, P, gamma, w3, Kpad, b3, local, attn, y3,
                             stats3, stats3_floats, stream, f);
}

extern "C" int dfcsa_conv_gemm_mtile(int N) { (void)N; return 64; }

extern "C" int dfcsa_get_tuning(int knob) {
  switch (knob) {
    case 1: return g_conv_cfg;
    case 19: return g_halo_min_m;
    case 20: return g_wgrad_halo;
    case 31: return g_wgrad_coop;
    case 32: return g_wgrad_coop_launches;
    case 33: return g_stream_min_m;
    case 34: return g_stream_shuf;
    case 35: return g_lsa_cols_nt;
    case 46: return g_lsa_pool_one_slice;
    case 47: return g_lsa_pool_direct;
    case 48: return g_lsa_key_centre;
    case 49: return g_lsa_cols_flash;
    case 50: return g_gn_chunk;
    case 36: return g_gate_grid_div;
    case 37: return g_splitk_min_nk;
    case 39: return g_bn_fold;
    case 40: return g_ppsk;
    case 42: return g_wgrad_bd_nst;
    case 43: return g_pro_sb;
    case 44: return g_gate_sb;
    case 38: return g_splitk_target;
    default: return DFCSA_EINVAL;
  }
}

extern "C" int dfcsa_set_tuning(int knob, int value) {
  if (knob == 1) { g_conv_cfg = value; return 0; }
  if (knob == 2) { g_wgrad_target = value > 0 ? value : 512; return 0; }
  if (knob == 3) { g_stream_wgs = value; return 0; }
  if (knob == 4) { g_debug = value; return 0; }
  if (knob == 5) { g_stream_force = value; return 0; }
  if (knob == 6) { g_wgrad_waves = (value == 8 || value == 4) ? value : 0; return 0; }
  if (knob == 7) { g_wgrad_noglds = value; return 0; }
  if (knob == 8) { g_wgrad_narrow = value; return 0; }
  if (knob == 9) { g_fra_generic = value; return 0; }
  if (knob == 10) { g_fra_occ = value; return 0; }
  if (knob == 11) { g_ew_tile_elems = value >= 4096 ? value : 16384; return 0; }
  if (knob == 12) { g_wgrad_fuse_all = value; return 0; }
  if (knob == 13) { g_wgrad_fuse_max = value >= 0 ? (value <= 16 ? value : 16) : 0; return 0; }
  if (knob == 15) { g_conv_dbg = value; return 0; }
  if (knob == 21) { g_wgrad_nosimple = value; return 0; }
  if (knob == 22) { g_halo_variant = value; return 0; }
  if (knob == 23) { g_wgrad_reduce_old = value; return 0; }
  if (knob == 24) { g_wgrad_nst64 = value; return 0; }
  if (knob == 25) { g_splitk = value; return 0; }
  if (knob == 26) { g_wgrad_bd = value; return 0; }
  if (knob == 27) { g_small8 = value; return 0; }
  if (knob == 28) { g_lsa_rows_old = value; return 0; }
  if (knob == 30) { g_stream_shift = value; return 0; }
  if (knob == 31) { g_wgrad_coop = value; return 0; }
  if (knob == 33) { g_stream_min_m = value; return 0; }
  if (knob == 34) { g_stream_shuf = value; return 0; }
  if (knob == 35) { g_lsa_cols_nt = value; return 0; }
  if (knob == 46) { g_lsa_pool_one_slice = value ? 1 : 0; return 0; }
  if (knob == 47) { g_lsa_pool_direct = value ? 1 : 0; return 0; }
  if (knob == 48) { g_lsa_key_centre = value ? 1 : 0; return 0; }
  if (knob == 49) { g_lsa_cols_flash = value ? 1 : 0; return 0; }
  if (knob == 50) { g_gn_chunk = value ? 1 : 0; return 0; }
  if (knob == 36) { g_gate_grid_div = value; return 0; }
  if (knob == 39) { g_bn_fold = value; return 0; }
  if (knob == 40) { g_ppsk = value; return 0; }
  if (knob == 42) { g_wgrad_bd_nst = (value == 3 || value == 4) ? value : 2; return 0; }
  if (knob == 43) { g_pro_sb = value ? 1 : 0; return 0; }
  if (knob == 44) { g_gate_sb = value ? 1 : 0; return 0; }
  if (knob == 37) { g_splitk_min_nk = value > 0 ? value : 24; return 0; }
  if (knob == 38) { g_splitk_target = value > 0 ? value : 600; return 0; }
  if (knob == 16) { g_wgrad_noglds_f32small = value; return 0; }
  if (knob == 17) { g_wgrad_big = value; return 0; }
  if (knob == 18) { g_wgrad_wide_small = value; return 0; }
  if (knob == 14) { g_wgrad_nst = (value >= 2 && value <= 4) ? value : 2; return 0; }
  if (knob == 19) { g_halo_min_m = value; return 0; }
  if (knob == 20) { g_wgrad_halo = value; return 0; }
  return DFCSA_EINVAL;
}
