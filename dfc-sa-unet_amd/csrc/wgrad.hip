// Convolution weight gradient on MFMA: a reduction over pixels.
//
//   slab[s][i][j] = sum_{m in chunk s} G[m][i] * X[m][j]
//
// G is an NHWC gradient tensor (possibly the channel-concat of up to three tensors), X is the
// implicit im2col gather of the layer input (same segment/shift description as conv_gemm), so
// the reduction axis m is the slow (row) axis of BOTH operands.  Tiles are staged in LDS as
// [pixel][channel] images and the MFMA fragments (8 consecutive pixels per lane) are read with
// the gfx950 hardware-transposing ds_read_b64_tr_b16 (bf16).  An XOR swizzle of the 16-column
// blocks keeps those transposed reads bank-conflict-free.  The pixel axis is split into chunks
// (split-K).  With a destination (ndst > 0) and a modest split count the partials are reduced
// INSIDE the launch: each workgroup publishes its fp32 partial tile with write-through stores,
// takes a ticket on its output tile, and the last arriving workgroup sums the tile's partials in
// split order and adds them into the weight gradient in the reference layout (deterministic, no
// float atomics, no second launch, the partials read back from the on-die caches).  High split
// counts (the shallow, HBM-bound layers) keep the separate fixed-order reduction
// (dfcsa_wgrad_reduce).
//
// Replaces the weight half of ATen convolution_backward for the convolutions at reference
// models/unet_dfc_sa_res.py:58, 66, 74, 81, 88 and ConvTranspose2d at :147-156.
#include <cstdio>
#include <cstring>

#include "common.h"
#include "dfcsa_internal.h"
#include "small_gemm.h"

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s;

// physical 32-byte block of logical block `blk` in pixel row `r` (bf16 images)
template <int BW>
__device__ __forceinline__ int blk_swz(int r, int blk) {
  if constexpr (BW >= 128) return blk ^ ((r & 3) | (((r >> 3) & 1) << 2));
  else return blk ^ (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
}

// ---------------------------------------------------------------------------------------------
// Fused split-K epilogue
// ---------------------------------------------------------------------------------------------
constexpr int kCntRing = 1 << 18;       // ticket counters (one per output tile of a launch)
__device__ unsigned g_wg_cnt[kCntRing];

// dW element (i, j) of the GEMM -> the reference weight layout (dfcsa_wgrad_reduce's mapping)
__device__ __forceinline__ void wgrad_dst_add(const WgradArgs& a, int i, int j, float v) {
  if (i >= a.NI || j >= a.NJ) return;
  if (a.layout == 0) {
    const int rows = a.NI / a.ndst;
    const int d = i / rows, r = i - d * rows;
    const int tap = j / a.Ctot, cin = j - tap * a.Ctot;
    if (cin >= a.Creal || tap >= a.ntaps) return;
    float* dst = d == 0 ? a.dst[0] : (d == 1 ? a.dst[1] : a.dst[2]);
    dst[((int64_t)r * a.Creal + cin) * a.ntaps + tap] += v;
  } else if (a.layout == 2) {
    if (i >= 2 * a.Ctot + a.Creal) return;
    const int d = i < a.Ctot ? 0 : (i < 2 * a.Ctot ? 1 : 2);
    a.dst[d][(int64_t)(i - d * a.Ctot) * a.NJ + j] += v;
  } else if (a.layout == 3) {
    if (i < a.Ctot) a.dst[0][(int64_t)i * a.NJ + j] += v;
    else if (j >= a.Ctot) a.dst[1][(int64_t)(i - a.Ctot) * (a.NJ - a.Ctot) + (j - a.Ctot)] += v;
  } else {
    const int ij = j / a.Ctot, co = j - ij * a.Ctot;
    a.dst[0][((int64_t)i * a.Ctot + co) * 4 + ij] += v;
  }
}

// write-through (sc1) 16-B store: the bytes leave the XCD's L2 at once, so another XCD's
// workgroup reading them with sc1 loads after the ticket sees them (no L2 write-back fence).
// The s_nop covers the store-data hazard of >8-byte VMEM stores (the next VALU may not rewrite
// the data VGPRs for one wait state), which the compiler does not insert after inline asm.
__device__ __forceinline__ void st_sc1_x4(float* p, f32x4_t v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
// four sc1 16-B loads in flight, one wait
__device__ __forceinline__ void ld_sc1_x4x4(const float* p0, const float* p1, const float* p2, const float* p3,
                                            f32x4_t& v0, f32x4_t& v1, f32x4_t& v2, f32x4_t& v3) {
  asm volatile(
      "global_load_dwordx4 %0, %4, off sc1\n\t"
      "global_load_dwordx4 %1, %5, off sc1\n\t"
      "global_load_dwordx4 %2, %6, off sc1\n\t"
      "global_load_dwordx4 %3, %7, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
      : "v"(p0), "v"(p1), "v"(p2), "v"(p3)
      : "memory");
}

// The accumulator fragments of one wave: acc[i][j] holds rows rbase + i*16 + (lane>>4)*4 + r,
// column cbase + j*16 + (lane&15).  fuse == 0: plain [split][NI][NJ] partial slab.  Otherwise
// nsplit == 1 adds straight into dst; else partial tile -> ticket -> last arriver reduces.
// Partial tile layout (per output tile, per split): [wave][fragment][lane][4] -- every wave store
// is 1 KiB contiguous and the reducing lane reads exactly the elements it holds itself.
template <int FM, int FN, int NW>
__device__ __forceinline__ void wgrad_epilogue(const WgradArgs& a, f32x4_t (&acc)[FM][FN], int tile, int split,
                                               int rbase, int cbase, int lane, int wave, int tid, int* last_s) {
  constexpr int NF = FM * FN;
  if (!a.fuse) {
    float* out = a.slab + (size_t)split * a.NI * a.NJ;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = cbase + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rbase + i * 16 + (lane >> 4) * 4 + r;
          if (row < a.NI && col < a.NJ) out[(size_t)row * a.NJ + col] = acc[i][j][r];
        }
      }
    return;
  }
#ifndef DFCSA_NO_WGRAD_FUSE
  if (a.nsplit > 1) {
    constexpr int TILEF = NW * NF * 256;  // floats of one partial tile
    float* tbase = a.slab + (size_t)tile * a.nsplit * TILEF + (size_t)(wave * NF) * 256 + lane * 4;
#pragma unroll
    for (int f = 0; f < NF; ++f) st_sc1_x4(tbase + (size_t)split * TILEF + f * 256, acc[f / FN][f % FN]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(a.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last_s = (old == (unsigned)(a.nsplit - 1));
      if (*last_s) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __hip_atomic_store(a.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
      }
    }
    __syncthreads();
    if (!*last_s) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // sum the partials in split order 0..nsplit-1 (own one from registers: the same bits)
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      f32x4_t sum = {0.f, 0.f, 0.f, 0.f};
      const float* fb = tbase + f * 256;
      for (int p0 = 0; p0 < a.nsplit; p0 += 4) {
        f32x4_t v[4];
        const float* ptr[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) ptr[q] = fb + (size_t)min(p0 + q, a.nsplit - 1) * TILEF;
        ld_sc1_x4x4(ptr[0], ptr[1], ptr[2], ptr[3], v[0], v[1], v[2], v[3]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int p = p0 + q;
          if (p == split) sum += acc[f / FN][f % FN];
          else if (p < a.nsplit) sum += v[q];
        }
      }
      acc[f / FN][f % FN] = sum;
    }
  }
#endif
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = cbase + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) wgrad_dst_add(a, rbase + i * 16 + (lane >> 4) * 4 + r, col, acc[i][j][r]);
    }
}

// ---------------------------------------------------------------------------------------------
// Cooperative split-K reduction (args.coop; the host enables it only when the whole grid fits on
// the chip at once, so every split of a tile is resident or will become resident without waiting
// for a spinning workgroup).  Each workgroup
//   1. publishes its partial tile with write-through (sc1) stores, [tile][split][wave][frag][lane][4];
//   2. takes an arrival ticket on the tile's counter and waits (one lane, s_sleep poll of an sc1
//      load, bounded) until all nsplit partials are published, then one agent-scope acquire;
//   3. reduces ONE slice of the tile -- float4 positions [split*TQ/nsplit, (split+1)*TQ/nsplit) --
//      over all splits: the slice's positions x P parts of consecutive split ranges, each summed in
//      split order, the parts combined in LDS in part order (fixed order: bit-identical run to
//      run), and adds it into the weight gradient in the reference layout (each element owned by
//      exactly one lane: no atomics);
//   4. departs (second ticket); the last departure re-zeroes the counter for the next launch.
// So the reduction work is spread over every workgroup of the tile (each reads as many bytes as it
// wrote) instead of a serial last arriver or a separate reduction launch over an HBM slab.
// A poll that exceeds kCoopSpin (~0.1 s: never in a correct launch) sets g_wgrad_coop_err and
// proceeds -- a wrong gradient, reported by dfcsa_wgrad_coop_errors(), never a hung GPU.
// ---------------------------------------------------------------------------------------------
constexpr int kCoopSpin = 1 << 18;
__device__ int g_wgrad_coop_err;

template <int FM, int FN, int NW, int WN, int WTM, int WTN>
__device__ __forceinline__ void wgrad_coop(const WgradArgs& a, f32x4_t (&acc)[FM][FN], int tile, int split, int i0,
                                           int j0, int lane, int wave, int tid, float* lds) {
  constexpr int NF = FM * FN;
  constexpr int TILEF = NW * NF * 256;   // floats of one partial tile
  constexpr int TQ = TILEF / 4;          // float4 positions
  constexpr int NT = NW * 64;
  const int ns = a.nsplit;
  float* tb = a.slab + (size_t)tile * ns * TILEF;
  {
    float* mine = tb + (size_t)split * TILEF + (size_t)(wave * NF) * 256 + lane * 4;
#pragma unroll
    for (int f = 0; f < NF; ++f) st_sc1_x4(mine + f * 256, acc[f / FN][f % FN]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_fetch_add(a.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int it = 0;
    while (__hip_atomic_load(a.cnt + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)ns) {
      __builtin_amdgcn_s_sleep(2);
      if (++it > kCoopSpin) {
        __hip_atomic_store(&g_wgrad_coop_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const int q0 = (int)((int64_t)split * TQ / ns), q1 = (int)((int64_t)(split + 1) * TQ / ns);
  const int q = q1 - q0;
  if (q > 0) {
    const int P = q >= NT ? 1 : NT / q;                // parts (split ranges) per position
    const int part = q >= NT ? 0 : tid / q;
    const int s0 = (int)((int64_t)part * ns / P), s1 = (int)((int64_t)(part + 1) * ns / P);
    f32x4_t* red = (f32x4_t*)lds;                      // [P][q] partial sums when P > 1
    for (int p = (q >= NT ? tid : tid % q); p < q && part < P; p += (q >= NT ? NT : q)) {
      const float* src = tb + (size_t)(q0 + p) * 4;
      f32x4_t sum = {0.f, 0.f, 0.f, 0.f};
      for (int s = s0; s < s1; s += 4) {
        f32x4_t v[4];
        const float* ptr[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) ptr[u] = src + (size_t)min(s + u, s1 - 1) * TILEF;
        ld_sc1_x4x4(ptr[0], ptr[1], ptr[2], ptr[3], v[0], v[1], v[2], v[3]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (s + u < s1) sum += v[u];
      }
      if (P > 1) red[part * q + p] = sum;
      else {
        // position -> (wave, fragment, lane) of the accumulator layout -> (row, column)
        const int pw = (q0 + p) / (NF * 64), pf = ((q0 + p) / 64) % NF, pl = (q0 + p) & 63;
        const int row = i0 + (pw / WN) * WTM + (pf / FN) * 16 + (pl >> 4) * 4;
        const int col = j0 + (pw % WN) * WTN + (pf % FN) * 16 + (pl & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) wgrad_dst_add(a, row + r, col, sum[r]);
      }
    }
    if (P > 1) {
      __syncthreads();
      for (int p = tid; p < q; p += NT) {
        f32x4_t sum = red[p];
        for (int u = 1; u < P; ++u) sum += red[u * q + p];
        const int pw = (q0 + p) / (NF * 64), pf = ((q0 + p) / 64) % NF, pl = (q0 + p) & 63;
        const int row = i0 + (pw / WN) * WTM + (pf / FN) * 16 + (pl >> 4) * 4;
        const int col = j0 + (pw % WN) * WTN + (pf % FN) * 16 + (pl & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) wgrad_dst_add(a, row + r, col, sum[r]);
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(a.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned)(2 * ns - 1)) __hip_atomic_store(a.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// bf16: rows of BW channels = BW*2 bytes; chunk (8 channels) ch of row r
template <int BW>
__device__ __forceinline__ int chunk_off_bf16(int r, int ch) {
  int blk = ch >> 1;
  return r * (BW * 2) + ((blk_swz<BW>(r, blk) << 1) | (ch & 1)) * 16;
}

// transposed fragment read: 8 consecutive pixels (rows kb + 8*(lane>>4) ...) of column
// col0 + (lane & 15)
template <int BW>
__device__ __forceinline__ bf16x8_t tr_frag(const char* img, int kb, int col0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int blk = col0 >> 4;
  int r0 = kb + 8 * g + q, r1 = r0 + 4;
  const char* a0 = img + r0 * (BW * 2) + blk_swz<BW>(r0, blk) * 32 + 8 * p;
  const char* a1 = img + r1 * (BW * 2) + blk_swz<BW>(r1, blk) * 32 + 8 * p;
  v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a0);
  v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a1);
  bf16x8_t f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

// f32 fragment (parity mode): plain [pixel][BW] image, 8 scalar reads
template <int BW>
__device__ __forceinline__ void f32_frag(const char* img, int kb, int col0, int lane, float (&f)[8]) {
  const float* t = (const float*)img;
  const int col = col0 + (lane & 15), r = kb + 8 * (lane >> 4);
#pragma unroll
  for (int s = 0; s < 8; ++s) f[s] = t[(r + s) * BW + col];
}

template <typename T, int BI, int BJ, int NW>
__global__ void __launch_bounds__(NW * 64) wgrad_kernel(const WgradArgs args) {
  constexpr int NT = NW * 64;
  constexpr int EPC = ElemTraits<T>::kChunk;
  constexpr int KMS = (sizeof(T) == 2) ? 64 : 32;    // pixels per stage
  constexpr int NG = KMS / 32;
  constexpr int CPR_G = BI * (int)sizeof(T) / 16;    // 16-B chunks per G row
  constexpr int CPR_X = BJ * (int)sizeof(T) / 16;
  constexpr int RPP_G = NT / CPR_G, RPP_X = NT / CPR_X;    // rows per pass
  constexpr int NPG = KMS / RPP_G, NPX = KMS / RPP_X;       // passes per stage
  constexpr int GB = KMS * BI * (int)sizeof(T), XB = KMS * BJ * (int)sizeof(T);
  constexpr int WTM = BI / (NW / 2), WTN = BJ / 2;       // waves: NW/2 x 2
  constexpr int FM = WTM / 16, FN = WTN / 16;

  __shared__ __attribute__((aligned(16))) char smem[2 * (GB + XB)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int j0 = blockIdx.x * BJ, i0 = blockIdx.y * BI, split = blockIdx.z;
  const int mbeg = split * args.mchunk;
  const int mend = min(args.M, mbeg + args.mchunk);
  if (mbeg >= mend) {
    // still write zeros so the reduction can read every slab
  }

  // G loader: fixed channel chunk
  const int gcc = tid % CPR_G, grow = tid / CPR_G;
  const int gi = i0 + gcc * EPC;
  const bool g_ok = gi < args.NI;
  const T* gbase = nullptr;
  int gC = args.Cg;
  if (g_ok) {
    int src = dm_div(args.dm_cg, gi);
    gbase = (const T*)args.g_ptr[src] + (gi - src * args.Cg);
  }
  // X loader: fixed column chunk -> fixed segment
  const int xcc = tid % CPR_X, xrow = tid / CPR_X;
  const int xj = j0 + xcc * EPC;
  const bool x_ok = xj < args.NJ;
  ConvSeg xs = {nullptr, 0, 0};
  int xch = 0;
  if (x_ok) {
    int seg = dm_div(args.dm_cseg, xj);
    xch = xj - seg * args.Cseg;
    xs = args.seg[seg];
  }

  uint4 rg[NPG], rx[NPX];
  auto load_stage = [&](int kt) {
    const int mb = mbeg + kt * KMS;
#pragma unroll
    for (int p = 0; p < NPG; ++p) {
      int m = mb + grow + p * RPP_G;
      if (g_ok && m < mend) rg[p] = *(const uint4*)(gbase + (size_t)m * gC);
      else rg[p] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < NPX; ++p) {
      int m = mb + xrow + p * RPP_X;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (x_ok && m < mend) {
        int b = dm_div(args.dm_hw, m);
        int rem = m - b * args.dm_hw.d;
        int oh = dm_div(args.dm_w, rem);
        int ow = rem - oh * args.dm_w.d;
        int ih = oh * args.stride + xs.dh, iw = ow * args.stride + xs.dw;
        if (ih >= 0 && ih < args.Hi && iw >= 0 && iw < args.Wi)
          v = *(const uint4*)((const T*)xs.ptr + ((size_t)((b * args.Hi + ih) * args.Wi + iw) * args.Cseg + xch));
      }
      rx[p] = v;
    }
  };
  auto store_stage = [&](int s) {
    char* G = smem + s * (GB + XB);
    char* X = G + GB;
#pragma unroll
    for (int p = 0; p < NPG; ++p) {
      int r = grow + p * RPP_G;
      int off = (sizeof(T) == 2) ? chunk_off_bf16<BI>(r, gcc) : (r * BI * 4 + gcc * 16);
      *(uint4*)(G + off) = rg[p];
    }
#pragma unroll
    for (int p = 0; p < NPX; ++p) {
      int r = xrow + p * RPP_X;
      int off = (sizeof(T) == 2) ? chunk_off_bf16<BJ>(r, xcc) : (r * BJ * 4 + xcc * 16);
      *(uint4*)(X + off) = rx[p];
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};

  const int nk = (mend > mbeg) ? (mend - mbeg + KMS - 1) / KMS : 0;
  if (nk > 0) {
    load_stage(0);
    store_stage(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) load_stage(kt + 1);
    const char* G = smem + (kt & 1) * (GB + XB);
    const char* X = G + GB;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if constexpr (sizeof(T) == 2) {
        bf16x8_t fa[FM], fb[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[i] = tr_frag<BI>(G, 32 * g, wm * WTM + i * 16, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[j] = tr_frag<BJ>(X, 32 * g, wn * WTN + j * 16, lane);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      } else {
        float fa[FM][8], fb[FN][8];
#pragma unroll
        for (int i = 0; i < FM; ++i) f32_frag<BI>(G, 32 * g, wm * WTM + i * 16, lane, fa[i]);
#pragma unroll
        for (int j = 0; j < FN; ++j) f32_frag<BJ>(X, 32 * g, wn * WTN + j * 16, lane, fb[j]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int s = 0; s < 8; ++s)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
      }
    }
    if (more) store_stage((kt + 1) & 1);
    __syncthreads();
  }

  wgrad_epilogue<FM, FN, NW>(args, acc, blockIdx.y * gridDim.x + blockIdx.x, split, i0 + wm * WTM, j0 + wn * WTN,
                             lane, wave, tid, (int*)smem);   // smem is free after the main loop's last barrier
}


// --------------------------------------------------------------------------------------------
// bf16 weight gradient with LDS-DMA staging (global_load_lds_dwordx4): the [pixel][channel]
// images are filled directly from global memory; the XOR block swizzle of the transposed reads
// is applied on the source side (lane -> which logical 16-B chunk it fetches), so the images are
// bit-identical to the register-staged kernel's.  Per-lane gather state (group pointer / segment,
// swizzled channel) is fixed per DMA slot, only the pixel advances with the stage.
// --------------------------------------------------------------------------------------------
__device__ __attribute__((aligned(16))) uint4 g_wg_zero[64];

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void glb_void_t;

// LDS-DMA issued from inline asm (cdna_hip_programming.md, glds16_asm): the compiler does not
// count it, so it inserts no vmcnt(0) of its own before the next fragment reads -- with the
// builtin it cannot tell the stage being filled from the stage being read and drains every DMA
// before the MFMAs (measured in the round-2 ISA of this kernel: one vmcnt(0) per stage).  The
// kernel waits for its DMAs itself (counted vmcnt + barrier), and the loop issues no other
// vector-memory operation.  lds_dst: wave-uniform LDS byte address.
__device__ __forceinline__ void glds16_asm(const void* gsrc, const char* lds_dst) {
  const unsigned dst = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)lds_dst;
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(dst)
               : "memory");
}

template <int BI, int BJ, int WM, int WN, int NST, bool SIMPLE = false>
__global__ void __launch_bounds__(WM * WN * 64) wgrad_glds_kernel(const WgradArgs args, int nsplit) {
  constexpr int NW = WM * WN;
  using T = bf16_t;
  constexpr int KMS = 64;
  constexpr int GB = KMS * BI * 2, XB = KMS * BJ * 2, STAGE = GB + XB;
  constexpr int CPR_G = BI / 8, CPR_X = BJ / 8;            // 16-B chunks per image row
  constexpr int RPI_G = 64 / CPR_G, RPI_X = 64 / CPR_X;    // rows per DMA instruction
  constexpr int NI_G = CPR_G / NW, NI_X = CPR_X / NW;      // DMA instructions per wave per stage
  static_assert(NI_G >= 1 && NI_X >= 1, "wgrad glds tiling");
  constexpr int WTM = BI / WM, WTN = BJ / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int SMEM_MAIN = NST * STAGE;
  constexpr int OPS = NI_G + NI_X;   // DMA instructions per wave per stage (issued unconditionally)
  __shared__ __attribute__((aligned(16))) char smem[SMEM_MAIN + DFCSA_MAX_SEG * (int)sizeof(ConvSeg)];
  ConvSeg* segtab = (ConvSeg*)(smem + SMEM_MAIN);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int wv = __builtin_amdgcn_readfirstlane(wave);   // DMA destinations: scalar (M0)
  // XCD-aware order: all column/row tiles of one pixel split (and neighbouring splits) run on
  // one XCD, so the 9 shifted taps of a 3x3 gather hit that XCD's L2 instead of HBM
  const int nJ = (args.NJ + BJ - 1) / BJ, nI = (args.NI + BI - 1) / BI;
  const int L = xcd_remap(blockIdx.x, nJ * nI * nsplit);
  if (L < 0) return;
  const int j0 = (L % nJ) * BJ, i0 = ((L / nJ) % nI) * BI, split = L / (nJ * nI);
  const int mbeg = split * args.mchunk;
  const int mend = min(args.M, mbeg + args.mchunk);
  if (tid < args.nseg) segtab[tid] = args.seg[tid];
  __syncthreads();

  // G slots: row within the stage and source pointer (channel fixed), or null
  int g_row[NI_G];
  const T* g_src[NI_G];
#pragma unroll
  for (int q = 0; q < NI_G; ++q) {
    const int ins = q * NW + wave;
    const int r = ins * RPI_G + lane / CPR_G, pc = lane % CPR_G;
    const int lc = (blk_swz<BI>(r, pc >> 1) << 1) | (pc & 1);
    const int i = i0 + lc * 8;
    g_row[q] = r;
    g_src[q] = nullptr;
    if (i < args.NI) {
      const int grp = dm_div(args.dm_cg, i);
      g_src[q] = (const T*)args.g_ptr[grp] + (i - grp * args.Cg);
    }
  }
  // X slots: row, segment (LDS table) and channel
  int x_row[NI_X], x_seg[NI_X], x_ch[NI_X];
#pragma unroll
  for (int q = 0; q < NI_X; ++q) {
    const int ins = q * NW + wave;
    const int r = ins * RPI_X + lane / CPR_X, pc = lane % CPR_X;
    const int lc = (blk_swz<BJ>(r, pc >> 1) << 1) | (pc & 1);
    const int j = j0 + lc * 8;
    x_row[q] = r;
    x_seg[q] = -1;
    x_ch[q] = 0;
    if (j < args.NJ) {
      const int sg = dm_div(args.dm_cseg, j);
      x_seg[q] = sg;
      x_ch[q] = j - sg * args.Cseg;
    }
  }
  const void* zero = (const void*)g_wg_zero;
  // SIMPLE geometry: the X source of slot q at pixel m is x_base[q] + m*Cseg (the shift folded in),
  // valid while the shifted (row, column) stays inside the image; (row, column) of the slot's
  // pixel are advanced by 64 pixels per issued stage instead of divided out every stage
  const T* x_base[NI_X];
  int x_dh[NI_X], x_dw[NI_X], x_oh[NI_X], x_ow[NI_X];
  if constexpr (SIMPLE) {
#pragma unroll
    for (int q = 0; q < NI_X; ++q) {
      x_base[q] = nullptr;
      x_dh[q] = x_dw[q] = 0;
      const int m = mbeg + x_row[q];
      const int b = dm_div(args.dm_hw, m);
      const int rem = m - b * args.dm_hw.d;
      x_oh[q] = dm_div(args.dm_w, rem);
      x_ow[q] = rem - x_oh[q] * args.dm_w.d;
      if (x_seg[q] >= 0) {
        const ConvSeg sg = segtab[x_seg[q]];
        x_dh[q] = sg.dh;
        x_dw[q] = sg.dw;
        x_base[q] = (const T*)sg.ptr + ((sg.dh * args.Wi + sg.dw) * args.Cseg + x_ch[q]);
      }
    }
  }

  auto issue = [&](int kt, int buf) {
    char* G = smem + buf * STAGE;
    char* X = G + GB;
    const int mb = mbeg + kt * KMS;
#pragma unroll
    for (int q = 0; q < NI_G; ++q) {
      const int m = mb + g_row[q];
      const void* src = (g_src[q] && m < mend) ? (const void*)(g_src[q] + (size_t)m * args.Cg) : zero;
      glds16_asm(src, G + (q * NW + wv) * 1024);
    }
    if constexpr (SIMPLE) {
#pragma unroll
      for (int q = 0; q < NI_X; ++q) {
        const int m = mb + x_row[q];
        const bool ok = x_base[q] && m < mend && (unsigned)(x_oh[q] + x_dh[q]) < (unsigned)args.Hi &&
                        (unsigned)(x_ow[q] + x_dw[q]) < (unsigned)args.Wi;
        const void* src = ok ? (const void*)(x_base[q] + (size_t)m * args.Cseg) : zero;
        glds16_asm(src, X + (q * NW + wv) * 1024);
        int ow = x_ow[q] + args.adv_w, oh = x_oh[q] + args.adv_h;
        if (ow >= args.Wi) { ow -= args.Wi; ++oh; }
        if (oh >= args.Hi) oh -= args.Hi;
        x_ow[q] = ow;
        x_oh[q] = oh;
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < NI_X; ++q) {
      const int m = mb + x_row[q];
      const void* src = zero;
      if (x_seg[q] >= 0 && m < mend) {
        const ConvSeg sg = segtab[x_seg[q]];
        const int b = dm_div(args.dm_hw, m);
        const int rem = m - b * args.dm_hw.d;
        const int oh = dm_div(args.dm_w, rem);
        const int ow = rem - oh * args.dm_w.d;
        const int ih = oh * args.stride + sg.dh, iw = ow * args.stride + sg.dw;
        if (ih >= 0 && ih < args.Hi && iw >= 0 && iw < args.Wi)
          src = (const void*)((const T*)sg.ptr + ((size_t)((b * args.Hi + ih) * args.Wi + iw) * args.Cseg + x_ch[q]));
      }
      glds16_asm(src, X + (q * NW + wv) * 1024);
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};

  const int nk = (mend > mbeg) ? (mend - mbeg + KMS - 1) / KMS : 0;
  // NST-deep ring: stages kt+1 .. kt+NST-2 stay in flight while stage kt is multiplied; the DMAs
  // are the only vector-memory ops in the loop, so a counted vmcnt isolates stage kt
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s, s);
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
    __syncthreads();
    if (kt + NST - 1 < nk) issue(kt + NST - 1, (kt + NST - 1) % NST);
    const char* G = smem + (kt % NST) * STAGE;
    const char* X = G + GB;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      bf16x8_t fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = tr_frag<BI>(G, 32 * g, wm * WTM + i * 16, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = tr_frag<BJ>(X, 32 * g, wn * WTN + j * 16, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }

  if (args.coop) {
    wgrad_coop<FM, FN, NW, WN, WTM, WTN>(args, acc, L % (nJ * nI), split, i0, j0, lane, wave, tid, (float*)smem);
    return;
  }
  wgrad_epilogue<FM, FN, NW>(args, acc, L % (nJ * nI), split, i0 + wm * WTM, j0 + wn * WTN, lane, wave, tid,
                             (int*)smem);
}

// --------------------------------------------------------------------------------------------
// bf16 weight gradient with buffer-descriptor LDS-DMA on 64-channel sub-images (simple geometry:
// stride 1, same-size input, shifts in [-1, 1]; Cseg % 64 == 0 and Cg % 64 == 0).
//
// The stage images of wgrad_glds_kernel are [64 pixels][BI | BJ channels]; a 1-KB DMA then spans
// channel blocks of different sources / taps, so every lane carries its own 64-bit source pointer
// and zero-page select (~8 VALU per DMA, 7.9 VALU per MFMA measured on the 224^2 3x3 layer).  Here
// each operand tile is cut into [64 pixels][64 channels] sub-images (128-B rows, the blk_swz<64>
// swizzle of the BI = 64 images): one sub-image lies inside ONE dY tensor / ONE tap segment, so its
// source base, tap shift and channel offset are wave-uniform (a scalar buffer descriptor), the
// stage's pixel advance is the scalar soffset, and a lane adds only its fixed row/chunk offset and a
// tap-validity select (sel_oob: offset >= 2^31 reads zeros).  Wave w fills rows 8w .. 8w + 7 of
// every sub-image, so a lane's pixel is the same in all its DMAs of a stage: its (row, column) is
// tracked incrementally and the 9 tap-validity bits are formed once per stage.
// --------------------------------------------------------------------------------------------
// The DMA is issued from inline asm (as glds16_asm above): with the builtin the compiler cannot
// tell the ring slot being filled from the one the transposed reads use and drains every DMA
// (s_waitcnt vmcnt(0)) before the fragment reads.  Descriptor words: base, stride 0,
// num_records 2^31 - 1, the raw-buffer flags of __builtin_amdgcn_make_buffer_rsrc(.., 0x00020000).
typedef int wrsrc_t __attribute__((ext_vector_type(4)));
constexpr unsigned kWOOB = 0x80000000u;
__device__ __forceinline__ wrsrc_t wbuf(const void* base) {
  const uint64_t a = (uint64_t)base;
  wrsrc_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu));
  r[2] = 0x7fffffff;
  r[3] = 0x00020000;
  return r;
}
__device__ __forceinline__ void wblds16(wrsrc_t r, unsigned voff, unsigned soff, const char* lds_dst) {
  const unsigned dst = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)lds_dst;
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(r), "s"(soff), "s"(dst)
               : "memory");
}

// voff if bit `bit` of mask is set, else out of range
__device__ __forceinline__ unsigned sel_oob_w(unsigned mask, int bit, unsigned voff) {
  const unsigned m = (unsigned)__builtin_amdgcn_sbfe((int)mask, bit, 1);
  return (voff & m) | (kWOOB & ~m);
}

template <int BI, int NST>
__global__ void __launch_bounds__(512) wgrad_bd_kernel(const WgradArgs args, int nsplit) {
  using T = bf16_t;
  constexpr int BJ = 128, NW = 8;
  constexpr int WM = BI == 64 ? 2 : 4, WN = BI == 64 ? 4 : 2;
  constexpr int WTM = BI / WM, WTN = BJ / WN, FM = WTM / 16, FN = WTN / 16;
  constexpr int GS = BI / 64, XS = BJ / 64;            // sub-images per operand
  constexpr int SUB = 64 * 128;                        // bytes of one [64 px][64 ch] sub-image
  constexpr int STAGE = (GS + XS) * SUB;
  constexpr int OPS = GS + XS;                         // DMAs per wave per stage
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int nJ = (args.NJ + BJ - 1) / BJ, nI = (args.NI + BI - 1) / BI;
  const int L = xcd_remap(blockIdx.x, nJ * nI * nsplit);
  if (L < 0) return;
  const int j0 = (L % nJ) * BJ, i0 = ((L / nJ) % nI) * BI, split = L / (nJ * nI);
  const int mbeg = split * args.mchunk;
  const int mend = min(args.M, mbeg + args.mchunk);

  // lane -> (row, physical 16-B chunk) of its 1-KB DMA piece; logical channel via the swizzle
  const int prow = 8 * wave + (lane >> 3), pc = lane & 7;
  const int lc = ((blk_swz<64>(prow, pc >> 1) << 1) | (pc & 1)) * 8;
  // G sub-images: scalar bases (tensor, channel block); X sub-images: segment base + tap shift
  wrsrc_t gr[GS], xr[XS];
  int xtb[XS];
  bool gon[GS], xon[XS];
#pragma unroll
  for (int s = 0; s < GS; ++s) {
    const int i = i0 + s * 64;
    gon[s] = i < args.NI;
    const int grp = gon[s] ? i / args.Cg : 0;
    gr[s] = wbuf((const T*)args.g_ptr[grp] + (gon[s] ? i - grp * args.Cg : 0));
  }
#pragma unroll
  for (int s = 0; s < XS; ++s) {
    const int j = j0 + s * 64;
    xon[s] = j < args.NJ;
    const int sg = xon[s] ? j / args.Cseg : 0;
    const ConvSeg seg = args.seg[sg];
    const int ch0 = xon[s] ? j - sg * args.Cseg : 0;
    xr[s] = wbuf((const T*)seg.ptr + ((seg.dh * args.Wi + seg.dw) * args.Cseg + ch0));
    xtb[s] = (seg.dh + 1) * 3 + seg.dw + 1;
  }
  // lane offsets at the split's first pixel (+ 64 pixels per stage through soffset)
  const unsigned goff = 2u * (unsigned)((mbeg + prow) * args.Cg + lc);
  const unsigned xoff = 2u * (unsigned)((mbeg + prow) * args.Cseg + lc);
  const unsigned gstep = 2u * 64u * (unsigned)args.Cg, xstep = 2u * 64u * (unsigned)args.Cseg;
  // (row, column) of the lane's pixel, advanced 64 pixels per issued stage
  int oh, ow;
  {
    const int m = mbeg + prow;
    const int b = dm_div(args.dm_hw, m);
    const int rem = m - b * args.dm_hw.d;
    oh = dm_div(args.dm_w, rem);
    ow = rem - oh * args.dm_w.d;
  }

  auto issue = [&](int kt, int buf) {
    char* G = smem + buf * STAGE;
    char* X = G + GS * SUB;
    const bool in = mbeg + kt * 64 + prow < mend;
    // tap-validity bits of the lane's pixel: bit (dh + 1) * 3 + dw + 1
    const unsigned up = oh > 0, dn = oh + 1 < args.Hi, lf = ow > 0, rt = ow + 1 < args.Wi;
    const unsigned rowm = 0x7u & (0u - up), rowc = 0x38u, rowd = 0x1C0u & (0u - dn);
    const unsigned colm = 0x49u & (0u - lf), colc = 0x92u, colr = 0x124u & (0u - rt);
    const unsigned mask = in ? ((rowm | rowc | rowd) & (colm | colc | colr)) : 0u;
    const unsigned gmask = in ? 0x10u : 0u;   // G: the pixel row only (bit 4 = centre)
#pragma unroll
    for (int s = 0; s < GS; ++s)
      wblds16(gr[s], gon[s] ? sel_oob_w(gmask, 4, goff) : kWOOB, (unsigned)kt * gstep, G + s * SUB + wv * 1024);
#pragma unroll
    for (int s = 0; s < XS; ++s)
      wblds16(xr[s], xon[s] ? sel_oob_w(mask, xtb[s], xoff) : kWOOB, (unsigned)kt * xstep, X + s * SUB + wv * 1024);
    int nw = ow + args.adv_w, nh = oh + args.adv_h;
    if (nw >= args.Wi) { nw -= args.Wi; ++nh; }
    if (nh >= args.Hi) nh -= args.Hi;
    ow = nw;
    oh = nh;
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};

  const int nk = (mend > mbeg) ? (mend - mbeg + 63) / 64 : 0;
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    // stages issued behind this one: their DMAs may stay in flight
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
    lds_barrier();
    if (kt + NST - 1 < nk) issue(kt + NST - 1, (kt + NST - 1) % NST);
    const char* G = smem + (kt % NST) * STAGE;
    const char* X = G + GS * SUB;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      bf16x8_t fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int c = wm * WTM + i * 16;
        fa[i] = tr_frag<64>(G + (c >> 6) * SUB, 32 * g, c & 63, lane);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = wn * WTN + j * 16;
        fb[j] = tr_frag<64>(X + (c >> 6) * SUB, 32 * g, c & 63, lane);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();
  if (args.coop) {
    wgrad_coop<FM, FN, NW, WN, WTM, WTN>(args, acc, L % (nJ * nI), split, i0, j0, lane, wave, tid, (float*)smem);
    return;
  }
  wgrad_epilogue<FM, FN, NW>(args, acc, L % (nJ * nI), split, i0 + wm * WTM, j0 + wn * WTN, lane, wave, tid,
                             (int*)smem);
}

// --------------------------------------------------------------------------------------------
// 3x3 weight gradient on 2-D halo tiles (bf16).
//
//   dW[i][tap][c] = sum_m dY[m][i] * X[m shifted by tap][c]
//
// The row-tile kernel above stages, per 64-pixel K stage, a dY tile and ONE tap's shifted X rows:
// dY is re-read once per column tile (9 taps x Cin / 128) and the input 9 times, 32 KB per
// 2.1 MFLOP (64 flop/B).  Here a workgroup owns an output block of BI rows x (all 9 taps x one
// 64-channel chunk of one source) and walks 128-pixel 2-D tiles (TW x TR, TW | W, rows of the
// image-stacked grid) of its pixel range: per tile it DMAs the dY tile (128 x BI) and the X halo
// ((TW+2) x (TR+2) x 64 channels) ONCE and runs all 9 taps from LDS -- the tap's B fragments are
// transposed reads (ds_read_b64_tr_b16) of the halo rows p0(k) + dh*(TW+2) + dw, a tap leaving the
// pixel's image reads a zero row.  128 x 576 x 128 x 2 flop per 55 KB (343 flop/B at BI = 128).
// Pad pixels of a tile have zero dY rows (they add nothing).  Split-K over pixel ranges: each split
// writes its [BI][9 taps x 64] block of the [split][NI][NJ] slab (one split: added straight into
// the gradient), reduced in fixed split order by wgrad_reduce_kernel (deterministic).
// 8 waves, one workgroup per CU (~130 KB LDS), dY and halo double-buffered one tile ahead.
// --------------------------------------------------------------------------------------------
constexpr int WH_MAXPIECE = 32;                  // halo <= 256 pixels (32 DMA pieces of 8)
constexpr int WH_XB = WH_MAXPIECE * 1024;        // one halo image (64 channels = 128 B / pixel)

struct WHaloTap {
  int toff;   // dh*(TW+2) + dw
  int dh;
  int col;    // GEMM column of (tap, c = 0) for chunk 0: segment index * Cseg
};
struct WHaloGroup {
  const void* ptr;
  int ntaps;
  WHaloTap tap[9];
};
struct WHaloArgs {
  int M, NI, NJ, Cg, Cseg, BH, H, W;
  int TW, TR, HW2, nhalo;
  int tiles, tiles_x, per_split, splits;
  int ngroups, nchunk, nI;
  const void* g;
  WHaloGroup grp[4];
  float* slab;                                   // [splits][NI][NJ] (splits > 1)
  int layout, ntaps, Ctot, Creal, ndst;          // direct add (splits == 1): dfcsa_wgrad_reduce's mapping
  float* dst[3];
};

// transposed fragment read with explicit rows: lanes of group g = lane / 16 supply the addresses
// of tile pixels kb + 8g + q (rows ra) and + 4 (rows rb), q = (lane % 16) / 4; 16 columns from col0
template <int BW>
__device__ __forceinline__ bf16x8_t tr_frag_rows(const char* img, int ra, int rb, int col0, int lane) {
  const int p = lane & 3, blk = col0 >> 4;
  const char* a0 = img + ra * (BW * 2) + blk_swz<BW>(ra, blk) * 32 + 8 * p;
  const char* a1 = img + rb * (BW * 2) + blk_swz<BW>(rb, blk) * 32 + 8 * p;
  v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a0);
  v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a1);
  bf16x8_t f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

template <int BI>
__global__ void __launch_bounds__(512, 1) wgrad_halo_kernel(const WHaloArgs a) {
  using T = bf16_t;
  constexpr int WM = BI / 32, WN = 8 / WM;       // waves: 32 output rows x (64 / WN) channels each
  constexpr int WC = 64 / WN, FC = WC / 16;
  constexpr int GB = 128 * BI * 2;               // dY image: 128 pixels x BI channels
  constexpr int NIG = GB / 1024 / 8;             // dY DMA pieces per wave per tile
  constexpr int NIX = WH_MAXPIECE / 8;           // halo DMA pieces per wave per tile
  constexpr int CPR = BI / 8, RPI = 64 / CPR;    // dY: 16-B chunks per pixel row, rows per piece
  constexpr int STAGE = GB + WH_XB;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 256];
  char* const zrow = smem + 2 * STAGE;           // a zero halo row

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  // task = ((split * ngroups + g) * nchunk + cc) * nI + it: the row tiles of one (g, cc, split)
  // are neighbours (one XCD: they share the halo reads)
  const int ntask = a.splits * a.ngroups * a.nchunk * a.nI;
  const int L = xcd_remap(blockIdx.x, ntask);
  if (L < 0) return;
  const int it = L % a.nI;
  const int cc = (L / a.nI) % a.nchunk;
  const int g = (L / (a.nI * a.nchunk)) % a.ngroups;
  const int split = L / (a.nI * a.nchunk * a.ngroups);
  const int i0 = it * BI;
  const int t_beg = split * a.per_split, t_end = min(a.tiles, t_beg + a.per_split);
  const int TW = a.TW, HW2 = a.HW2, BH = a.BH, H = a.H, W = a.W, npx = a.TW * a.TR;
  if (tid < 16) *(uint4*)(zrow + tid * 16) = make_uint4(0, 0, 0, 0);

  // dY pieces: tile pixel r (row of the image), 16-B chunk (source-side swizzle of tr_frag<BI>)
  int g_r[NIG], g_c[NIG];
#pragma unroll
  for (int q = 0; q < NIG; ++q) {
    const int ins = q * 8 + wave;
    const int r = ins * RPI + lane / CPR, pc = lane % CPR;
    g_r[q] = r;
    g_c[q] = i0 + ((blk_swz<BI>(r, pc >> 1) << 1) | (pc & 1)) * 8;
  }
  // halo pieces: halo pixel q = ins*8 + lane/8, chunk (source-side swizzle of tr_frag<64>)
  int x_q[NIX], x_c[NIX];
#pragma unroll
  for (int q = 0; q < NIX; ++q) {
    const int ins = q * 8 + wave;
    const int hq = ins * 8 + (lane >> 3), pc = lane & 7;
    x_q[q] = hq;
    x_c[q] = cc * 64 + ((blk_swz<64>(hq, pc >> 1) << 1) | (pc & 1)) * 8;
  }
  const T* gsrc = (const T*)a.g;
  const T* xsrc = (const T*)a.grp[g].ptr;
  const void* zero = (const void*)g_wg_zero;
  auto issue = [&](int tile, int buf) {
    char* G = smem + buf * STAGE;
    char* X = G + GB;
    const int trow = tile / a.tiles_x, tcol = tile - trow * a.tiles_x;
    const int r0 = trow * a.TR, c0 = tcol * TW;
#pragma unroll
    for (int q = 0; q < NIG; ++q) {
      const int k = g_r[q], ty = k / TW, tx = k - ty * TW;
      const bool ok = k < npx && r0 + ty < BH && g_c[q] < a.NI;
      const void* src = ok ? (const void*)(gsrc + (size_t)((r0 + ty) * W + c0 + tx) * a.Cg + g_c[q]) : zero;
      __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(G + (q * 8 + wave) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < NIX; ++q) {
      const int hq = x_q[q], hy = hq / HW2, hx = hq - hy * HW2;
      const int gr = r0 - 1 + hy, ix = c0 - 1 + hx;
      const bool ok = hq < a.nhalo && gr >= 0 && gr < BH && ix >= 0 && ix < W;
      const void* src = ok ? (const void*)(xsrc + (size_t)(gr * W + ix) * a.Cseg + x_c[q]) : zero;
      __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(X + (q * 8 + wave) * 1024), 16, 0, 0);
    }
  };

  // B-operand rows of this lane: tile pixels k = kb + 8*(lane/16) + (lane%16)/4 (+4), kb = 32*ks
  int pa[4], pb[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int k0 = ks * 32 + 8 * (lane >> 4) + ((lane & 15) >> 2), k1 = k0 + 4;
    pa[ks] = (k0 / TW + 1) * HW2 + k0 % TW + 1;
    pb[ks] = (k1 / TW + 1) * HW2 + k1 % TW + 1;
  }

  f32x4_t acc[9][2][FC];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int fi = 0; fi < 2; ++fi)
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) acc[t][fi][fc] = {0.f, 0.f, 0.f, 0.f};

  const int ntap = a.grp[g].ntaps;
  if (t_beg < t_end) issue(t_beg, 0);
  for (int tile = t_beg, buf = 0; tile < t_end; ++tile, buf ^= 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tile + 1 < t_end) issue(tile + 1, buf ^ 1);
    // rows of the image edges: a tap with dh = -1 (+1) leaving the pixel's image reads zeros
    const int r0 = (tile / a.tiles_x) * a.TR;
    unsigned up = 0, dn = 0;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k0 = ks * 32 + 8 * (lane >> 4) + ((lane & 15) >> 2);
      const int y0 = (r0 + k0 / TW) % H, y1 = (r0 + (k0 + 4) / TW) % H;
      up |= (unsigned)(y0 == 0) << (2 * ks) | (unsigned)(y1 == 0) << (2 * ks + 1);
      dn |= (unsigned)(y0 == H - 1) << (2 * ks) | (unsigned)(y1 == H - 1) << (2 * ks + 1);
    }
    const char* G = smem + buf * STAGE;
    const char* X = G + GB;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8_t fa[2];
#pragma unroll
      for (int fi = 0; fi < 2; ++fi) fa[fi] = tr_frag<BI>(G, 32 * ks, wm * 32 + fi * 16, lane);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t < ntap) {
          const WHaloTap tp = a.grp[g].tap[t];
          const unsigned bad = tp.dh < 0 ? up : (tp.dh > 0 ? dn : 0u);
          const bool oka = !((bad >> (2 * ks)) & 1), okb = !((bad >> (2 * ks + 1)) & 1);
          const char* ia = oka ? X : zrow;
          const char* ib = okb ? X : zrow;
          const int ra = oka ? pa[ks] + tp.toff : 0, rb = okb ? pb[ks] + tp.toff : 0;
#pragma unroll
          for (int fc = 0; fc < FC; ++fc) {
            // two image bases per lane: the zero row is its own image of one 128-B row
            const int col = wn * WC + fc * 16;
            bf16x8_t fb;
            {
              const int p = lane & 3, blk = col >> 4;
              const char* a0 = ia + ra * 128 + blk_swz<64>(ra, blk) * 32 + 8 * p;
              const char* a1 = ib + rb * 128 + blk_swz<64>(rb, blk) * 32 + 8 * p;
              v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a0);
              v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a1);
              fb[0] = lo[0]; fb[1] = lo[1]; fb[2] = lo[2]; fb[3] = lo[3];
              fb[4] = hi[0]; fb[5] = hi[1]; fb[6] = hi[2]; fb[7] = hi[3];
            }
#pragma unroll
            for (int fi = 0; fi < 2; ++fi)
              acc[t][fi][fc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[fi], fb, acc[t][fi][fc], 0, 0, 0);
          }
        }
      }
    }
  }

  // ---- epilogue: acc[t][fi][fc][r] = dW[i0 + wm*32 + fi*16 + (lane/16)*4 + r][tap t][cc*64 + col] ----
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    if (t >= ntap) continue;
    const int jb = a.grp[g].tap[t].col + cc * 64;
#pragma unroll
    for (int fi = 0; fi < 2; ++fi)
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) {
        const int j = jb + wn * WC + fc * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + wm * 32 + fi * 16 + (lane >> 4) * 4 + r;
          if (i >= a.NI) continue;
          const float v = acc[t][fi][fc][r];
          if (a.splits > 1) {
            a.slab[((size_t)split * a.NI + i) * a.NJ + j] = v;
          } else {
            // dfcsa_wgrad_reduce's layout-0 mapping: row i -> dst[i / rows], column j -> (tap, cin)
            const int rows = a.NI / a.ndst, d = i / rows, rr = i - d * rows;
            const int tap = j / a.Ctot, cin = j - tap * a.Ctot;
            if (cin < a.Creal && tap < a.ntaps) {
              float* dst = d == 0 ? a.dst[0] : (d == 1 ? a.dst[1] : a.dst[2]);
              dst[((int64_t)rr * a.Creal + cin) * a.ntaps + tap] += v;
            }
          }
        }
      }
  }
}

// 64 output elements per workgroup, SUB split-ranges per element (threads sub*64 + el: each group
// of 64 threads reads 64 consecutive elements of one split -> coalesced; SUB grows with the split
// count so that high-split launches get enough threads), 8 loads in flight per thread; the SUB
// partial sums are combined in a fixed order through LDS (deterministic).
__device__ __forceinline__ void reduce_dst_add(int64_t e, int NI, int NJ, int layout, int ntaps, int Ctot, int Creal,
                                               int ndst, float* d0, float* d1, float* d2, float s) {
  int i = (int)(e / NJ), j = (int)(e % NJ);
  if (layout == 0) {
    int rows = NI / ndst;
    int d = i / rows, r = i - d * rows;
    int tap = j / Ctot, cin = j - tap * Ctot;
    if (cin >= Creal || tap >= ntaps) return;   // K-padding columns of the GEMM
    float* dst = d == 0 ? d0 : (d == 1 ? d1 : d2);
    dst[((int64_t)r * Creal + cin) * ntaps + tap] += s;
  } else if (layout == 2) {
    // 1x1 weights stacked by rows: [0, Ctot) -> d0, [Ctot, 2 Ctot) -> d1, [2 Ctot, 2 Ctot + Creal)
    // -> d2; later rows are GEMM padding
    if (i >= 2 * Ctot + Creal) return;
    const int d = i < Ctot ? 0 : (i < 2 * Ctot ? 1 : 2);
    float* dst = d == 0 ? d0 : (d == 1 ? d1 : d2);
    dst[(int64_t)(i - d * Ctot) * NJ + j] += s;
  } else if (layout == 3) {
    // two 1x1 weight gradients sharing their inputs' trailing columns (the DFC block's fusion conv
    // over [fused | local | attn] and gate conv over [local | attn]): rows [0, Ctot) -> d0 over all
    // NJ columns; rows [Ctot, 2 Ctot) -> d1 over the columns [Ctot, NJ)
    if (i < Ctot) d0[(int64_t)i * NJ + j] += s;
    else if (j >= Ctot) d1[(int64_t)(i - Ctot) * (NJ - Ctot) + (j - Ctot)] += s;
  } else {
    // ConvTranspose2d weight [Cin][Cout][2][2]; i = ci, j = ij*Cout + co (Ctot = Cout)
    int ij = j / Ctot, co = j - ij * Ctot;
    d0[((int64_t)i * Ctot + co) * 4 + ij] += s;
  }
}

// fp32 weight gradient over few pixel rows (the LightSelfAttention projections, M = B*P*P): the
// whole reduction in one launch (split over the 4 waves of a 16x64 tile, small_gemm.h), added
// straight into the destination layout -- no split-K slab, no reduce launch
template <int NWV, int UNR>
__device__ __forceinline__ void small_wgrad_tile(const WgradArgs& a, int bx, int by, float* lds) {
  auto st = [&](int i, int j, float v) {
    reduce_dst_add((int64_t)i * a.NJ + j, a.NI, a.NJ, a.layout, a.ntaps, a.Ctot, a.Creal, a.ndst, a.dst[0], a.dst[1],
                   a.dst[2], v);
  };
  small_gemm_tile<true, decltype(st), NWV, UNR>((const float*)a.g_ptr[0], a.NI, (const float*)a.seg[0].ptr, a.Cseg,
                                                a.NI, a.NJ, a.M, bx * 16, by * 64, lds, st);
  if (!a.bdst[0] || by != 0) return;
  // layout 2 bias gradients of this workgroup's 16 rows i: sum over the M pixel rows of G[m][i]
  // (fp64, parts of M/(4 NWV) rows in row order, then the parts in order -- fixed order)
  constexpr int NPART = NWV * 4;
  __syncthreads();   // lds is free again (the tile's partial sums were consumed)
  double* red = (double*)lds;   // [NPART][16]
  const int il = threadIdx.x & 15, part = threadIdx.x >> 4;
  const int i = bx * 16 + il;
  const float* __restrict__ g = (const float*)a.g_ptr[0];
  double sm = 0.0;
  if (i < a.NI) {
    const int per = (a.M + NPART - 1) / NPART, m0 = part * per, m1 = min(a.M, m0 + per);
    for (int m = m0; m < m1; ++m) sm += (double)g[(size_t)m * a.NI + i];
  }
  red[part * 16 + il] = sm;
  __syncthreads();
  if (part != 0 || i >= a.NI || i >= 2 * a.Ctot + a.Creal) return;
  double tot = 0.0;
  for (int q = 0; q < NPART; ++q) tot += red[q * 16 + il];
  const int d = i < a.Ctot ? 0 : (i < 2 * a.Ctot ? 1 : 2);
  a.bdst[d][i - d * a.Ctot] += (float)tot;
}

// fp32 weight gradient over few pixel rows (the LightSelfAttention projections, M = B*P*P): the
// whole reduction in one launch (split over the waves of a 16x64 tile, small_gemm.h), added
// straight into the destination layout -- no split-K slab, no reduce launch
template <int NWV, int UNR>
__global__ void __launch_bounds__(NWV * 64) small_wgrad_f32_kernel(const WgradArgs a) {
  __shared__ float lds[NWV * 16 * 64];
  small_wgrad_tile<NWV, UNR>(a, blockIdx.x, blockIdx.y, lds);
}

// The same weight gradient and, in the same launch, the 1x1 conv's input gradient from the same G:
// dx[m][n] = sum_i G[m][i] * wt[n][i] (wt: the transposed weight, rows of kpad floats).  Workgroups
// [0, nw) take the weight-gradient tiles, the rest the 16 x 64 input-gradient tiles -- the two
// GEMMs only read G, so one launch replaces two on the attention backward chain.
struct SmallDgrad {
  const float* wt;
  float* dx;
  int kpad, N, nwx, nw, ndx;
  // optional pool contraction (dfcsa_conv_wgrad_dgrad1x1_pool): wsum [M][2][N], rows [ndx][2][N]
  const float* wsum;
  const float* mean;
  const float* invstd;
  float* rows;
  int H, W, P;
};
template <int NWV, int UNR>
__global__ void __launch_bounds__(NWV * 64) small_wgrad_dgrad_f32_kernel(const WgradArgs a, const SmallDgrad d) {
  __shared__ float lds[NWV * 16 * 64];
  int b = blockIdx.x;
  if (b < d.nw) {
    small_wgrad_tile<NWV, UNR>(a, b % d.nwx, b / d.nwx, lds);
    return;
  }
  b -= d.nw;
  const int bx = b % d.ndx, by = b / d.ndx;
  if (!d.rows) {
    auto st = [&](int m, int n, float v) { d.dx[(size_t)m * d.N + n] = v; };
    small_gemm_tile<false, decltype(st), NWV, UNR>((const float*)a.g_ptr[0], a.NI, d.wt, d.kpad, a.M, d.N, a.NI,
                                                   bx * 16, by * 64, lds, st);
    return;
  }
  // with the pool contraction: each stored dpooled value also enters its column's two sums over the
  // tile's 16 rows (LDS [2][16][64], summed in row order below)
  __shared__ float cs[2][16][64];
  __shared__ float inv_area[16];
  const int NP = d.P * d.P;
  if (threadIdx.x < 16) {
    const int n = (bx * 16 + threadIdx.x) % NP, pi = n / d.P, pj = n - pi * d.P;
    inv_area[threadIdx.x] = 1.f / (float)((((pi + 1) * d.H + d.P - 1) / d.P - (pi * d.H) / d.P) *
                                         (((pj + 1) * d.W + d.P - 1) / d.P - (pj * d.W) / d.P));
  }
  for (int e = threadIdx.x; e < 2 * 16 * 64; e += NWV * 64) (&cs[0][0][0])[e] = 0.f;
  __syncthreads();
  auto st = [&](int m, int n, float v) {
    d.dx[(size_t)m * d.N + n] = v;
    const int r = m - bx * 16, c = n - by * 64;
    const float dd = v * inv_area[r];
    const float R = d.wsum[((size_t)m * 2) * d.N + n], Y = d.wsum[((size_t)m * 2 + 1) * d.N + n];
    cs[0][r][c] = dd * R;
    cs[1][r][c] = dd * d.invstd[n] * (Y - d.mean[n] * R);
  };
  small_gemm_tile<false, decltype(st), NWV, UNR>((const float*)a.g_ptr[0], a.NI, d.wt, d.kpad, a.M, d.N, a.NI,
                                                 bx * 16, by * 64, lds, st);
  __syncthreads();
  if (threadIdx.x < 128) {
    const int k = threadIdx.x >> 6, c = threadIdx.x & 63, n = by * 64 + c;
    if (n < d.N) {
      float s = 0.f;
      for (int r = 0; r < 16; ++r) s += cs[k][r][c];
      d.rows[((size_t)bx * 2 + k) * d.N + n] = s;
    }
  }
}

template <int SUB>
__global__ void __launch_bounds__(64 * SUB) wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int NI,
                                                                int NJ, int layout, int ntaps, int Ctot, int Creal,
                                                                int ndst, float* d0, float* d1, float* d2) {
  __shared__ float part[SUB][64];
  const int el = threadIdx.x & 63, sub = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + el;
  const int64_t total = (int64_t)NI * NJ;
  const int per = (splits + SUB - 1) / SUB, k0 = sub * per, k1 = min(splits, k0 + per);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f, a5 = 0.f, a6 = 0.f, a7 = 0.f;
  if (e < total) {
    int k = k0;
    for (; k + 7 < k1; k += 8) {
      const float* p = slab + (int64_t)k * total + e;
      a0 += p[0]; a1 += p[total]; a2 += p[2 * total]; a3 += p[3 * total];
      a4 += p[4 * total]; a5 += p[5 * total]; a6 += p[6 * total]; a7 += p[7 * total];
    }
    for (; k < k1; ++k) a0 += slab[(int64_t)k * total + e];
  }
  part[sub][el] = ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));
  __syncthreads();
  if (sub != 0 || e >= total) return;
  float s = part[0][el];
#pragma unroll
  for (int q = 1; q < SUB; ++q) s += part[q][el];
  reduce_dst_add(e, NI, NJ, layout, ntaps, Ctot, Creal, ndst, d0, d1, d2, s);
}

// Low split counts (the deep layers: 3-16 splits of a [NI][taps x Ctot] slab of up to 19 MB per
// split; multi-tap layers up to 64 splits, in chunks of MAXS): one workgroup per (row i, 64-channel chunk), its 4 waves take the taps round-robin, each
// lane issues all the split loads of its element at once (<= 16 in flight) and sums them in split
// order; the [64][T] tile is transposed through LDS so the read-modify-write of the weight
// gradient walks 64*T consecutive floats of the reference layout ([Cout][Cin][kh][kw]: taps
// fastest; ConvTranspose2d [Cin][Cout][2][2]) instead of 4-B scatters at a T-float stride.
// T == 1: the waves take four consecutive 64-channel chunks.
template <int MAXS>
__global__ void __launch_bounds__(256) wgrad_reduce_tap_kernel(const float* __restrict__ slab, int splits, int NI,
                                                               int NJ, int layout, int T, int Ctot, int Creal,
                                                               int ndst, float* d0, float* d1, float* d2) {
  __shared__ float tile[4 * 64 * 9 + 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = blockIdx.y;
  const int64_t total = (int64_t)NI * NJ;
  const int cw = T == 1 ? 256 : 64;                  // channels per workgroup
  const int c0 = blockIdx.x * cw;
  // taps handled by this wave: T > 1 -> t = wave, wave + 4, ...; T == 1 -> t = 0, channel block wave
  const int tstep = T == 1 ? T : 4;
  const int cl = T == 1 ? wave * 64 + lane : lane;   // channel within the chunk
  for (int t = T == 1 ? 0 : wave; t < T; t += tstep) {
    const int c = c0 + cl;
    const bool ok = c < Ctot;
    const float* p = slab + (int64_t)i * NJ + (int64_t)t * Ctot + c;
    float acc = 0.f;
    for (int s0 = 0; s0 < splits; s0 += MAXS) {   // MAXS loads in flight, summed in split order
      float v[MAXS];
#pragma unroll
      for (int s = 0; s < MAXS; ++s) v[s] = (ok && s0 + s < splits) ? p[(int64_t)(s0 + s) * total] : 0.f;
#pragma unroll
      for (int s = 0; s < MAXS; ++s)
        if (s0 + s < splits) acc += v[s];
    }
    tile[cl * T + t] = acc;
  }
  __syncthreads();
  // destination: rows of the reference layout, channels c0 .. c0 + cw (clipped to Creal), T
  // consecutive floats per channel
  float* dst;
  int r, creal;
  if (layout == 0) {
    const int rows = NI / ndst, d = i / rows;
    r = i - d * rows;
    dst = d == 0 ? d0 : (d == 1 ? d1 : d2);
    creal = Creal;
  } else {
    r = i;
    dst = d0;
    creal = Ctot;
  }
  const int nc = min(cw, creal - c0);
  if (nc <= 0) return;
  float* base = dst + ((int64_t)r * creal + c0) * T;
  for (int e = threadIdx.x; e < nc * T; e += 256) base[e] += tile[e];
}

int launch_reduce(const float* slab, int splits, int NI, int NJ, int layout, int ntaps, int Ctot, int Creal, int ndst,
                  float* d0, float* d1, float* d2, hipStream_t st) {
  const int64_t total = (int64_t)NI * NJ;
  const int blocks = (int)((total + 63) / 64);
  const int T = layout == 0 ? ntaps : 4;
  // (taps > 1 up to 64 splits: the 3x3 layers at 224^2 - 56^2 run 28 - 56; the high-split 1x1
  // reductions already write coalesced and keep the split-parallel kernel below)
  if (!g_wgrad_reduce_old && layout != 2 && layout != 3 && (splits <= 16 || (T > 1 && splits <= 64)) && T <= 9 &&
      (int64_t)T * Ctot <= NJ && NI <= 65535) {
    const int cw = T == 1 ? 256 : 64;
    dim3 grid((Ctot + cw - 1) / cw, NI);
    if (splits <= 4)
      hipLaunchKernelGGL(wgrad_reduce_tap_kernel<4>, grid, dim3(256), 0, st, slab, splits, NI, NJ, layout, T, Ctot,
                         Creal, ndst, d0, d1, d2);
    else if (splits <= 8)
      hipLaunchKernelGGL(wgrad_reduce_tap_kernel<8>, grid, dim3(256), 0, st, slab, splits, NI, NJ, layout, T, Ctot,
                         Creal, ndst, d0, d1, d2);
    else
      hipLaunchKernelGGL(wgrad_reduce_tap_kernel<16>, grid, dim3(256), 0, st, slab, splits, NI, NJ, layout, T, Ctot,
                         Creal, ndst, d0, d1, d2);
    DFCSA_CHECK_LAUNCH();
    return 0;
  }
  // >= ~16 splits per thread keeps the loads in flight; more sub-ranges when the blocks are few
  if (splits >= 128 && blocks < 1024)
    hipLaunchKernelGGL(wgrad_reduce_kernel<16>, dim3(blocks), dim3(1024), 0, st, slab, splits, NI, NJ, layout, ntaps,
                       Ctot, Creal, ndst, d0, d1, d2);
  else if (splits >= 32 && blocks < 2048)
    hipLaunchKernelGGL(wgrad_reduce_kernel<8>, dim3(blocks), dim3(512), 0, st, slab, splits, NI, NJ, layout, ntaps,
                       Ctot, Creal, ndst, d0, d1, d2);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel<4>, dim3(blocks), dim3(256), 0, st, slab, splits, NI, NJ, layout, ntaps,
                       Ctot, Creal, ndst, d0, d1, d2);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// big output tiles (knob 17) for the deep layers: one 512-thread workgroup per CU stages
// (BI + BJ) x 64 pixels per K stage for BI*BJ*64 MACs, so a 256x256 tile needs half the
// L2->LDS bytes per flop of a 128x128 one (the per-CU L2 fetch rate, ~70 GB/s, not the MFMA,
// bounds the 128x128 tile at ~0.46 of peak).  1: 256x256 (NI >= 256), 2: 256x128 (NI >= 256),
// 3: 128x256 (NI >= 128, NJ >= 256)
__host__ __device__ inline int wgrad_big_mode(int NI, int NJ, int big) {
  if (big == 1 && NI >= 256 && NJ >= 256) return 1;
  if (big == 2 && NI >= 256) return 2;
  if (big == 3 && NI >= 128 && NJ >= 256) return 3;
  return 0;
}

// 64-row (NI <= 64) bf16 tiles take 256 columns when NJ is wide (4 x 2 wave layout of 32x64
// tiles instead of 16x64: half the LDS fragment reads per MFMA)
// knob 18: also for 128 < NJ <= 256 (the 1x1 wgrads over three 64-channel sources at 224^2: one
// column tile, so G is read once instead of twice)
bool wide_j(const WgradArgs& a) {
  return a.NI <= 64 && ((a.NJ >= 512 && !g_wgrad_narrow) || (g_wgrad_wide_small && a.NJ > 128 && a.NJ <= 256));
}

// The halo launch of a bf16 3x3 weight gradient (layout 0, one dY tensor); false if it does not
// apply.  BI = 64 for NI <= 64, else 128; splits = pixel ranges so that ~256 workgroups run.
bool whalo_plan(const WgradArgs& a, int dtype, int layout, WHaloArgs* h, int* bi) {
  if (!g_wgrad_halo || dtype != DFCSA_DT_BF16 || layout != 0 || a.ng != 1 || a.stride != 1 || a.Ho != a.Hi ||
      a.Wo != a.Wi || a.Cseg % 64 || a.Cg % 8 || a.M < 32768)
    return false;
  if ((int64_t)a.M * a.Cseg >= (1ll << 31) || (int64_t)a.M * a.Cg >= (1ll << 31)) return false;
  std::memset(h, 0, sizeof(*h));
  bool shifted = false;
  for (int i = 0; i < a.nseg; ++i) {
    const ConvSeg& s = a.seg[i];
    if (s.dh < -1 || s.dh > 1 || s.dw < -1 || s.dw > 1) return false;
    shifted |= (s.dh || s.dw);
    int g = 0;
    while (g < h->ngroups && h->grp[g].ptr != s.ptr) ++g;
    if (g == h->ngroups) {
      if (g == 4) return false;
      h->grp[g].ptr = s.ptr;
      h->ngroups++;
    }
    WHaloGroup& G = h->grp[g];
    if (G.ntaps == 9) return false;
    G.tap[G.ntaps].dh = s.dh;
    G.tap[G.ntaps].toff = s.dw;          // + dh*(TW+2) below
    G.tap[G.ntaps].col = i * a.Cseg;
    G.ntaps++;
  }
  if (!shifted) return false;
  const int W = a.Wo, BH = a.M / a.Wo;
  int bTW = 0, bTR = 0, bHalo = 1 << 30;
  double best = 0.0;
  for (int TW = 4; TW <= 64 && TW <= W; ++TW) {
    if (W % TW) continue;
    const int TR = 128 / TW;
    const int halo = (TW + 2) * (TR + 2);
    const int pmax = (127 / TW + 2) * (TW + 2) + TW + 1;   // furthest halo row a (pad) lane reads
    if (halo > WH_MAXPIECE * 8 || pmax >= WH_MAXPIECE * 8) continue;
    const int tiles = (W / TW) * ((BH + TR - 1) / TR);
    const double eff = (double)a.M / ((double)tiles * 128.0);
    if (eff > best + 1e-9 || (eff > best - 1e-9 && halo < bHalo)) { best = eff; bTW = TW; bTR = TR; bHalo = halo; }
  }
  if (best < 0.85) return false;
  *bi = a.NI <= 64 ? 64 : 128;
  h->M = a.M; h->NI = a.NI; h->NJ = a.NJ; h->Cg = a.Cg; h->Cseg = a.Cseg; h->BH = BH; h->H = a.Ho; h->W = W;
  h->TW = bTW; h->TR = bTR; h->HW2 = bTW + 2; h->nhalo = bHalo;
  h->tiles_x = W / bTW;
  h->tiles = h->tiles_x * ((BH + bTR - 1) / bTR);
  h->nchunk = a.Cseg / 64;
  h->nI = (a.NI + *bi - 1) / *bi;
  const int groups = h->ngroups * h->nchunk * h->nI;
  int S = (256 + groups - 1) / groups;
  if (S > h->tiles / 2) S = h->tiles / 2;
  if (S < 1) S = 1;
  h->per_split = (h->tiles + S - 1) / S;
  h->splits = (h->tiles + h->per_split - 1) / h->per_split;
  for (int g = 0; g < h->ngroups; ++g)
    for (int t = 0; t < h->grp[g].ntaps; ++t) h->grp[g].tap[t].toff += h->grp[g].tap[t].dh * h->HW2;
  h->g = a.g_ptr[0];
  return true;
}

// LDS-DMA ring depth of the wgrad tile kernel: knob 14 forces it for every launch; knob 24 (>= 0)
// gives the 64-row tiles (NI <= 64: 24 KB stages, so three stages still leave two workgroups per
// CU) their own depth
inline int wgrad_nst(const WgradArgs& a, int BI) {
  if (BI == 64 && g_wgrad_nst64 >= 2) return g_wgrad_nst64;
  return g_wgrad_nst;
}

// ticket counters for `tiles` output tiles of one launch: a region of the ring per launch, so launches
// in flight on other streams never share one (each tile's counter is zero on entry and re-zeroed by
// the launch itself)
unsigned* wgrad_cnt_region(int tiles) {
  static unsigned* ring = nullptr;
  static int next = 0;
  if (tiles > kCntRing) return nullptr;
  if (!ring && hipGetSymbolAddress((void**)&ring, HIP_SYMBOL(g_wg_cnt)) != hipSuccess) return nullptr;
  if (next + tiles > kCntRing) next = 0;
  unsigned* r = ring + next;
  next += tiles;
  return r;
}

}  // namespace
int g_wgrad_coop_launches = 0;   // host count of cooperative launches (dfcsa_get_tuning(32), tests)
namespace {

// workgroups of `kern` (at `threads` per workgroup) that fit on the device at once (cached)
template <typename K>
int coop_capacity(K kern, int threads) {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cached[dev]) {
    int nb = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, threads, 0) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cached[dev] = nb * cus > 0 ? nb * cus : -1;
  }
  return cached[dev] > 0 ? cached[dev] : 0;
}

// launch `kern` on `grid` workgroups, with the cooperative split-K reduction when asked for and the
// whole grid fits on the device at once (otherwise the caller's separate reduction runs)
template <typename K>
int launch_wg(K kern, int grid, int threads, int BI, int BJ, const WgradArgs& a0, int splits, bool want_coop,
              bool* coop_used, hipStream_t st) {
  WgradArgs a = a0;
  a.coop = 0;
  if (want_coop && splits > 1 && grid <= coop_capacity(kern, threads)) {
    const int tiles = ((a.NI + BI - 1) / BI) * ((a.NJ + BJ - 1) / BJ);
    if ((a.cnt = wgrad_cnt_region(tiles)) != nullptr) {
      a.coop = 1;
      a.nsplit = splits;
    }
  }
  *coop_used = a.coop != 0;
  g_wgrad_coop_launches += a.coop;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, st, a, splits);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

template <typename T, int BI>
int launch_wgrad(const WgradArgs& a, int splits, hipStream_t st, bool want_coop, bool* coop_used) {
  constexpr int BJ = 128;
  *coop_used = false;
  dim3 grid((a.NJ + BJ - 1) / BJ, (a.NI + BI - 1) / BI, splits);
  // 8 waves (32x64 wave tiles) hide more latency: LDS-DMA + 8 waves measured best or equal on
  // every shape of the step (tools/wgrad_bench.py; 5-15 % on the 3x3 layers)
  const int waves = g_wgrad_waves ? g_wgrad_waves : 8;
  if constexpr (sizeof(T) == 2) {
    if (!g_wgrad_noglds) {
      if (const int bm = wgrad_big_mode(a.NI, a.NJ, g_wgrad_big)) {
        const int bi = bm == 3 ? 128 : 256, bj = bm == 2 ? 128 : 256;
        const int gb = xcd_pad(((a.NJ + bj - 1) / bj) * ((a.NI + bi - 1) / bi) * splits);
        if (bm == 1)
          return launch_wg(wgrad_glds_kernel<256, 256, 2, 4, 2>, gb, 512, bi, bj, a, splits, want_coop, coop_used, st);
        if (bm == 2)
          return launch_wg(wgrad_glds_kernel<256, 128, 4, 2, 2>, gb, 512, bi, bj, a, splits, want_coop, coop_used, st);
        return launch_wg(wgrad_glds_kernel<128, 256, 2, 4, 2>, gb, 512, bi, bj, a, splits, want_coop, coop_used, st);
      }
      // buffer-descriptor kernel on 64-channel sub-images (knob 26 = 0: the pointer-DMA kernel)
      if (g_wgrad_bd && a.simple && a.Cseg % 64 == 0 && a.Cg % 64 == 0 && !wide_j(a) &&
          (int64_t)a.M * a.Cseg * 2 < (1ll << 31) && (int64_t)a.M * a.Cg * 2 < (1ll << 31))
      {
        // knob 42: LDS-DMA ring depth of this kernel (2 = two workgroups per CU, the default; 3 / 4 =
        // one workgroup per CU with two / three stages in flight)
        const int bnst = g_wgrad_bd_nst;
        if (bnst == 4)
          return launch_wg(wgrad_bd_kernel<BI, 4>, xcd_pad(grid.x * grid.y * splits), 512, BI, BJ, a, splits,
                           want_coop, coop_used, st);
        if (bnst == 3)
          return launch_wg(wgrad_bd_kernel<BI, 3>, xcd_pad(grid.x * grid.y * splits), 512, BI, BJ, a, splits,
                           want_coop, coop_used, st);
        return launch_wg(wgrad_bd_kernel<BI, 2>, xcd_pad(grid.x * grid.y * splits), 512, BI, BJ, a, splits, want_coop,
                         coop_used, st);
      }
      // 1-D grid (x = padded tile count): see the XCD remap in the kernel
      if (BI == 64 && wide_j(a))
        return launch_wg(wgrad_glds_kernel<64, 256, 2, 4, 2>, xcd_pad(((a.NJ + 255) / 256) * ((a.NI + BI - 1) / BI) * splits),
                         512, BI, 256, a, splits, want_coop, coop_used, st);
      const int g1 = xcd_pad(grid.x * grid.y * splits);
      constexpr int WM8 = BI == 64 ? 2 : 4, WN8 = BI == 64 ? 4 : 2;
      const int nst = wgrad_nst(a, BI);
      if (waves == 8 && nst >= 4 && a.simple)
        return launch_wg(wgrad_glds_kernel<BI, BJ, WM8, WN8, 4, true>, g1, 512, BI, BJ, a, splits, want_coop, coop_used, st);
      if (waves == 8 && nst >= 4)
        return launch_wg(wgrad_glds_kernel<BI, BJ, WM8, WN8, 4>, g1, 512, BI, BJ, a, splits, want_coop, coop_used, st);
      if (waves == 8 && nst == 3 && a.simple)
        return launch_wg(wgrad_glds_kernel<BI, BJ, WM8, WN8, 3, true>, g1, 512, BI, BJ, a, splits, want_coop, coop_used, st);
      if (waves == 8 && nst == 3)
        return launch_wg(wgrad_glds_kernel<BI, BJ, WM8, WN8, 3>, g1, 512, BI, BJ, a, splits, want_coop, coop_used, st);
      if (waves == 8 && a.simple)
        return launch_wg(wgrad_glds_kernel<BI, BJ, WM8, WN8, 2, true>, g1, 512, BI, BJ, a, splits, want_coop, coop_used, st);
      if (waves == 8)
        return launch_wg(wgrad_glds_kernel<BI, BJ, WM8, WN8, 2>, g1, 512, BI, BJ, a, splits, want_coop, coop_used, st);
      return launch_wg(wgrad_glds_kernel<BI, BJ, 2, 2, 2>, g1, 256, BI, BJ, a, splits, want_coop, coop_used, st);
    }
  }
  if (waves == 8)
    hipLaunchKernelGGL((wgrad_kernel<T, BI, BJ, 8>), grid, dim3(512), 0, st, a);
  else
    hipLaunchKernelGGL((wgrad_kernel<T, BI, BJ, 4>), grid, dim3(256), 0, st, a);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

}  // namespace

int g_small8 = 1;            // knob 27: 0 = the 4-wave small fp32 GEMM tiles (LightSelfAttention projections)
int g_wgrad_bd = 1;          // knob 26: buffer-descriptor wgrad kernel (simple geometry)
int g_wgrad_coop = 0;        // knob 31: cooperative in-launch split-K reduction when the grid fits the chip
int g_wgrad_nst64 = 0;       // knob 24: ring depth of the 64-row tiles (0 = follow knob 14)
int g_wgrad_reduce_old = 0;  // knob 23: 1 = the element-order reduction for every split count
int g_wgrad_halo = 0;      // knob 20: 1 = 3x3 weight gradients on the 2-D halo-tile kernel (off: slower so far)
int g_wgrad_waves = 0;     // waves per wgrad workgroup (dfcsa_set_tuning knob 6; 0 = automatic)
int g_wgrad_noglds = 0;    // 1 = register-staged bf16 wgrad (dfcsa_set_tuning knob 7)
int g_wgrad_narrow = 1;    // 0 = allow the 64x256 wgrad tile (dfcsa_set_tuning knob 8; measured slower on the L1 3x3)
int g_wgrad_target = 512;  // workgroups per wgrad launch (dfcsa_set_tuning knob 2)
int g_wgrad_bd_nst = 2;    // knob 42: LDS-DMA ring depth of the buffer-descriptor wgrad kernel (2, 3, 4)
int g_wgrad_nst = 2;       // knob 14: LDS-DMA ring depth of the bf16 wgrad kernel (2, 3, 4)
int g_wgrad_fuse_all = 0;  // knob 12: 1 = reduce in-kernel at any split count, -1 = never (separate launch)
// knob 13: most splits reduced in-kernel.  Default 0 = never: measured on the headline step
// (tools/wgrad_shapes.py, bench A/B) the last arriver's serialized read of the partials costs more
// than the separate fixed-order reduction launch (W4 H14: 114 vs 72 us; step 1172 vs 1198 img/s at
// <= 4 splits, 1149 at <= 16), so the fused path stays selectable, tested, and off.
int g_wgrad_fuse_max = 0;
int g_wgrad_noglds_f32small = 0;  // knob 16: 1 = fp32 small-M wgrads take the generic tiles
int g_wgrad_nosimple = 0;         // knob 21: 1 = the divide-per-stage X addressing (A/B of the incremental one)

// output tile of the wgrad kernel a launch uses (launch_wgrad's choice)
int g_wgrad_big = 0;        // knob 17: big wgrad tiles (wgrad_big_mode)
int g_wgrad_wide_small = 0; // knob 18: 64x256 tile for NI <= 64, 128 < NJ <= 256 (wide_j)
void wgrad_tile(int NI, int NJ, int dtype, int* BI, int* BJ) {
  if (dtype == DFCSA_DT_BF16 && !g_wgrad_noglds) {
    if (const int bm = wgrad_big_mode(NI, NJ, g_wgrad_big)) {
      *BI = bm == 3 ? 128 : 256;
      *BJ = bm == 2 ? 128 : 256;
      return;
    }
  }
  *BI = NI <= 64 ? 64 : 128;
  *BJ = (dtype == DFCSA_DT_BF16 && !g_wgrad_noglds && NI <= 64 &&
         ((NJ >= 512 && !g_wgrad_narrow) || (g_wgrad_wide_small && NJ > 128 && NJ <= 256))) ? 256 : 128;
}

extern "C" int dfcsa_wgrad_fuse_max(void) { return g_wgrad_fuse_max; }

extern "C" int dfcsa_wgrad_coop_errors(int reset) {
  int v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_wgrad_coop_err), sizeof(int), 0, hipMemcpyDeviceToHost) != hipSuccess)
    return DFCSA_EINVAL;
  if (reset && v) {
    const int z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_wgrad_coop_err), &z, sizeof(int), 0, hipMemcpyHostToDevice) != hipSuccess)
      return DFCSA_EINVAL;
  }
  return v;
}

namespace {
void desc_to_args(const dfcsa_wgrad_desc* d, WgradArgs& a) {
  std::memset(&a, 0, sizeof(a));
  a.M = d->M; a.ng = d->ng; a.Cg = d->Cg; a.NI = d->ng * d->Cg;
  for (int i = 0; i < 3; ++i) a.g_ptr[i] = i < d->ng ? d->g_ptr[i] : nullptr;
  a.nseg = d->nseg; a.Cseg = d->Cseg; a.NJ = d->nseg * d->Cseg;
  for (int i = 0; i < d->nseg; ++i) { a.seg[i].ptr = d->seg_ptr[i]; a.seg[i].dh = d->seg_dh[i]; a.seg[i].dw = d->seg_dw[i]; }
  a.Ho = d->Ho; a.Wo = d->Wo; a.Hi = d->Hi; a.Wi = d->Wi; a.stride = d->stride;
}
}  // namespace

extern "C" int dfcsa_wgrad_plan_desc(const dfcsa_wgrad_desc* d, int* splits, int* mchunk, int64_t* slab_floats) {
  if (!d || d->nseg < 1 || d->nseg > DFCSA_MAX_SEG || d->ng < 1 || d->ng > 3 || !splits || !mchunk)
    return DFCSA_EINVAL;
  WgradArgs a;
  desc_to_args(d, a);
  WHaloArgs h;
  int bi;
  if (whalo_plan(a, d->dtype, d->layout, &h, &bi)) {
    *splits = h.splits;
    *mchunk = h.per_split * 128;
    if (slab_floats) *slab_floats = h.splits > 1 ? (int64_t)h.splits * a.NI * a.NJ : 0;
    return 0;
  }
  return dfcsa_wgrad_plan(d->M, a.NI, a.NJ, d->dtype, splits, mchunk, slab_floats);
}

extern "C" int dfcsa_wgrad_plan(int M, int NI, int NJ, int dtype, int* splits, int* mchunk, int64_t* slab_floats) {
  if (M <= 0 || NI <= 0 || NJ <= 0 || !splits || !mchunk) return DFCSA_EINVAL;
  const int kms = dtype == DFCSA_DT_BF16 ? 64 : 32;
  int BI, BJ;
  wgrad_tile(NI, NJ, dtype, &BI, &BJ);
  const int tiles = ((NI + BI - 1) / BI) * ((NJ + BJ - 1) / BJ);
  // splits trade occupancy against split-K slab traffic (each split writes NI*NJ fp32 that the
  // reduce reads back): ~2 workgroups per CU is enough to keep the MFMA pipes busy
  int s = g_wgrad_target / tiles;
  if (s < 1) s = 1;
  // few tiles (deep layers): at least ~3 workgroups per CU, else the chip is underfilled
  // (measured: 12544 x 512 x 9216 runs 276 us with 1 split, 180 us with 3)
  if (s <= 2) s = (768 + tiles - 1) / tiles;
  int max_s = M / (4 * kms);  // keep >= 4 stages per chunk
  if (max_s < 1) max_s = 1;
  if (s > max_s) s = max_s;
  // cap the slab at 256 MiB
  int64_t per = (int64_t)NI * NJ * 4;
  int64_t cap = ((int64_t)256 << 20) / per;
  if (cap < 1) cap = 1;
  if (s > cap) s = (int)cap;
  int mc = (M + s - 1) / s;
  mc = (mc + kms - 1) / kms * kms;
  s = (M + mc - 1) / mc;
  *splits = s;
  *mchunk = mc;
  if (slab_floats) {
    const int64_t plain = (int64_t)s * NI * NJ;
    const int64_t tiled = (int64_t)tiles * s * BI * BJ;
    *slab_floats = plain > tiled ? plain : tiled;
  }
  return 0;
}

namespace {
int launch_wgrad_any(WgradArgs& a, const dfcsa_wgrad_desc* d, hipStream_t st);
}  // namespace

extern "C" int dfcsa_conv_wgrad(const dfcsa_wgrad_desc* d, void* stream) {
  if (!d || d->nseg < 1 || d->nseg > DFCSA_MAX_SEG || d->ng < 1 || d->ng > 3) return DFCSA_EINVAL;
  if (d->Cg % 8 || d->Cseg % 8 || d->mchunk <= 0 || d->splits <= 0) return DFCSA_EINVAL;
  const int kms = d->dtype == DFCSA_DT_BF16 ? 64 : 32;
  if (d->mchunk % kms) return DFCSA_EINVAL;
  if (d->ndst < 0 || d->ndst > 3) return DFCSA_EINVAL;
  WgradArgs a;
  a.M = d->M; a.ng = d->ng; a.Cg = d->Cg; a.NI = d->ng * d->Cg;
  for (int i = 0; i < 3; ++i) a.g_ptr[i] = i < d->ng ? d->g_ptr[i] : nullptr;
  a.nseg = d->nseg; a.Cseg = d->Cseg; a.NJ = d->nseg * d->Cseg;
  for (int i = 0; i < d->nseg; ++i) { a.seg[i].ptr = d->seg_ptr[i]; a.seg[i].dh = d->seg_dh[i]; a.seg[i].dw = d->seg_dw[i]; }
  a.Ho = d->Ho; a.Wo = d->Wo; a.Hi = d->Hi; a.Wi = d->Wi; a.stride = d->stride;
  a.dm_hw = make_divmod(d->Ho * d->Wo); a.dm_w = make_divmod(d->Wo);
  a.dm_cseg = make_divmod(d->Cseg); a.dm_cg = make_divmod(d->Cg);
  a.slab = d->slab; a.mchunk = d->mchunk;
  a.nsplit = d->splits;
  a.simple = d->stride == 1 && d->Hi == d->Ho && d->Wi == d->Wo && !g_wgrad_nosimple;
  for (int i = 0; i < d->nseg && a.simple; ++i)
    a.simple = d->seg_dh[i] >= -1 && d->seg_dh[i] <= 1 && d->seg_dw[i] >= -1 && d->seg_dw[i] <= 1;
  if (a.simple) { a.adv_w = 64 % d->Wo; a.adv_h = (64 / d->Wo) % d->Ho; }
  a.layout = d->layout; a.ntaps = d->ntaps; a.Ctot = d->Ctot; a.Creal = d->Creal; a.ndst = d->ndst;
  for (int i = 0; i < 3; ++i) a.dst[i] = i < d->ndst ? d->dst[i] : nullptr;
  if (d->ndst > 0) {
    if (d->layout == 2 ? (d->ndst != 3 || d->Ctot <= 0 || 2 * d->Ctot > a.NI)
                       : d->layout == 3 ? (d->ndst != 2 || d->Ctot <= 0 || a.NI != 2 * d->Ctot || a.NJ <= d->Ctot)
                                        : (a.NI % d->ndst != 0))
      return DFCSA_EINVAL;
    if (d->Ctot <= 0) return DFCSA_EINVAL;
  }
  const bool want_bias = d->bias_dst[0] != nullptr;
  if (want_bias && (d->layout != 2 || d->ndst != 3 || d->ng != 1 || !d->bias_dst[1] || !d->bias_dst[2]))
    return DFCSA_EINVAL;
  for (int i = 0; i < 3; ++i) a.bdst[i] = nullptr;
  // one split: the kernel adds its tile straight into dst (no slab, no second launch)
  a.fuse = d->ndst > 0 && (d->splits == 1 ||
                           (g_wgrad_fuse_all >= 0 && (d->splits <= g_wgrad_fuse_max || g_wgrad_fuse_all > 0)));
  if (!a.fuse && !d->slab) return DFCSA_EINVAL;
  if (!a.fuse && d->slab_floats < (int64_t)d->splits * a.NI * a.NJ) return DFCSA_EINVAL;
  a.cnt = nullptr;
  a.coop = 0;
  bool want_coop = false;
  {
    int BI, BJ;
    wgrad_tile(a.NI, a.NJ, d->dtype, &BI, &BJ);
    const int tiles = ((a.NI + BI - 1) / BI) * ((a.NJ + BJ - 1) / BJ);
    const bool tiled_fits = d->slab && d->slab_floats >= (int64_t)tiles * d->splits * BI * BJ;
    if (a.fuse && d->splits > 1) {
      // the in-kernel reduction writes tiled partials [tile][split][BI][BJ] into the slab
      if (!tiled_fits) return DFCSA_EINVAL;
      if (!(a.cnt = wgrad_cnt_region(tiles))) return DFCSA_EINVAL;
    }
    // cooperative reduction (bf16 tile kernels; the launch function checks that the grid fits)
    want_coop = g_wgrad_coop && !a.fuse && d->ndst > 0 && d->splits > 1 && d->dtype == DFCSA_DT_BF16 && tiled_fits;
  }
  hipStream_t st = (hipStream_t)stream;
  double flops = 2.0 * a.M * a.NI * a.NJ;
  ProfScope prof(DFCSA_PROF_WGRAD, st, flops);   // the class covers the reduction launch too
  if (dfcsa_shapelog())
    fprintf(stderr, "SHAPE wgrad M=%d NI=%d NJ=%d nseg=%d Cseg=%d splits=%d mchunk=%d fuse=%d dt=%d\n", a.M, a.NI,
            a.NJ, a.nseg, a.Cseg, d->splits, d->mchunk, a.fuse, d->dtype);
  {
    WHaloArgs h;
    int bi;
    if (d->ndst > 0 && !want_bias && whalo_plan(a, d->dtype, d->layout, &h, &bi) && d->splits == h.splits &&
        d->mchunk == h.per_split * 128) {
      if (h.splits > 1 && (!d->slab || d->slab_floats < (int64_t)h.splits * a.NI * a.NJ)) return DFCSA_EINVAL;
      h.slab = d->slab;
      h.layout = d->layout; h.ntaps = d->ntaps; h.Ctot = d->Ctot; h.Creal = d->Creal; h.ndst = d->ndst;
      for (int i = 0; i < 3; ++i) h.dst[i] = a.dst[i];
      dim3 grid(xcd_pad(h.splits * h.ngroups * h.nchunk * h.nI));
      if (bi == 64) hipLaunchKernelGGL(wgrad_halo_kernel<64>, grid, dim3(512), 0, st, h);
      else hipLaunchKernelGGL(wgrad_halo_kernel<128>, grid, dim3(512), 0, st, h);
      DFCSA_CHECK_LAUNCH();
      if (h.splits > 1)
        return launch_reduce(d->slab, h.splits, a.NI, a.NJ, d->layout, d->ntaps, d->Ctot, d->Creal, d->ndst, a.dst[0],
                             a.dst[1], a.dst[2], st);
      return 0;
    }
  }
  if (d->dtype != DFCSA_DT_BF16 && a.M <= 4096 && a.ng == 1 && a.nseg == 1 && !a.seg[0].dh && !a.seg[0].dw &&
      a.stride == 1 && d->ndst > 0 && a.Ho == a.Hi && a.Wo == a.Wi && !g_wgrad_noglds_f32small) {
    const dim3 sg((a.NI + 15) / 16, (a.NJ + 63) / 64);
    if (want_bias) for (int i = 0; i < 3; ++i) a.bdst[i] = d->bias_dst[i];
    if (g_small8) hipLaunchKernelGGL((small_wgrad_f32_kernel<8, 4>), sg, dim3(512), 0, st, a);
    else hipLaunchKernelGGL((small_wgrad_f32_kernel<4, 2>), sg, dim3(256), 0, st, a);
    DFCSA_CHECK_LAUNCH();
    return 0;
  }
  a.coop = want_coop ? 1 : 0;   // (launch_wgrad_any's request flag; cleared before any launch)
  if (want_bias) {   // the other kernels: the column sums of G by one launch after the weight gradient
    const int rc = launch_wgrad_any(a, d, st);
    if (rc) return rc;
    return dfcsa_slab_colsum3((const float*)a.g_ptr[0], a.M, std::min(a.NI, 2 * d->Ctot + d->Creal), d->Ctot,
                              d->Ctot, d->bias_dst[0], d->bias_dst[1], d->bias_dst[2], stream);
  }
  return launch_wgrad_any(a, d, st);
}

namespace {
int launch_wgrad_any(WgradArgs& a, const dfcsa_wgrad_desc* d, hipStream_t st) {
  int rc;
  bool coop = false;
  const bool want_coop = a.coop != 0;
  a.coop = 0;
  if (d->dtype == DFCSA_DT_BF16)
    rc = a.NI <= 64 ? launch_wgrad<bf16_t, 64>(a, d->splits, st, want_coop, &coop)
                    : launch_wgrad<bf16_t, 128>(a, d->splits, st, want_coop, &coop);
  else
    rc = a.NI <= 64 ? launch_wgrad<float, 64>(a, d->splits, st, false, &coop)
                    : launch_wgrad<float, 128>(a, d->splits, st, false, &coop);
  if (rc) return rc;
  if (d->ndst > 0 && !a.fuse && !coop)
    return launch_reduce(d->slab, d->splits, a.NI, a.NJ, d->layout, d->ntaps, d->Ctot, d->Creal, d->ndst, a.dst[0],
                         a.dst[1], a.dst[2], st);
  return 0;
}
}  // namespace

extern "C" int dfcsa_wgrad_reduce(const float* slab, int splits, int NI, int NJ, int layout, int ntaps,
                                  int Ctot, int Creal, int ndst, float* const* dst, void* stream) {
  if (!slab || !dst || ndst < 1 || ndst > 3) return DFCSA_EINVAL;
  if (layout == 2 ? (ndst != 3 || Ctot <= 0 || 2 * Ctot > NI)
                  : layout == 3 ? (ndst != 2 || Ctot <= 0 || NI != 2 * Ctot || NJ <= Ctot) : (NI % ndst != 0))
    return DFCSA_EINVAL;
  return launch_reduce(slab, splits, NI, NJ, layout, ntaps, Ctot, Creal, ndst, dst[0], ndst > 1 ? dst[1] : nullptr,
                       ndst > 2 ? dst[2] : nullptr, (hipStream_t)stream);
}

// dfcsa_conv_wgrad(d) and dx = G * wt^T (a 1x1 conv's input gradient from the same G), one launch
// when the small fp32 kernels apply to both, else the two calls one after the other
extern "C" int dfcsa_conv_wgrad_dgrad1x1_pool(const dfcsa_wgrad_desc* d, const float* wt, int kpad, int N, float* dx,
                                              const dfcsa_pool_contract* pc, void* stream) {
  if (!d || !wt || !dx || N <= 0 || kpad < d->ng * d->Cg || kpad % 4) return DFCSA_EINVAL;
  if (pc && (!pc->wsum || !pc->mean || !pc->invstd || !pc->rows || pc->P <= 0 || pc->H <= 0 || pc->W <= 0 ||
             d->M % (pc->P * pc->P)))
    return DFCSA_EINVAL;
  const int NI = d->ng * d->Cg;
  const bool small = d->dtype != DFCSA_DT_BF16 && d->M <= 4096 && d->ng == 1 && d->nseg == 1 && !d->seg_dh[0] &&
                     !d->seg_dw[0] && d->stride == 1 && d->ndst > 0 && d->Ho == d->Hi && d->Wo == d->Wi &&
                     !g_wgrad_noglds_f32small && NI % 4 == 0;
  if (!small) {
    if (pc) return DFCSA_EINVAL;   // the contraction rows come from the small kernel only
    if (const int rc = dfcsa_conv_wgrad(d, stream)) return rc;
    dfcsa_conv_desc c;
    std::memset(&c, 0, sizeof(c));
    c.dtype = d->dtype; c.M = d->M; c.N = N; c.Kpad = kpad; c.Cseg = NI; c.nseg = 1;
    c.seg_ptr[0] = d->g_ptr[0];
    c.Ho = d->Ho; c.Wo = d->Wo; c.Hi = d->Ho; c.Wi = d->Wo; c.stride = 1;
    c.weight = wt; c.mode = 0; c.ndest = 1; c.dest[0] = dx; c.Nd = N;
    return dfcsa_conv_gemm(&c, stream);
  }
  // validation and argument setup of dfcsa_conv_wgrad, small-kernel path
  if (d->Cg % 8 || d->Cseg % 8) return DFCSA_EINVAL;
  if (d->layout == 2 ? (d->ndst != 3 || d->Ctot <= 0 || 2 * d->Ctot > NI)
                     : d->layout == 3 ? (d->ndst != 2 || d->Ctot <= 0 || NI != 2 * d->Ctot || d->Cseg <= d->Ctot)
                                      : (NI % d->ndst != 0 || d->Ctot <= 0))
    return DFCSA_EINVAL;
  const bool want_bias = d->bias_dst[0] != nullptr;
  if (want_bias && (d->layout != 2 || d->ndst != 3 || !d->bias_dst[1] || !d->bias_dst[2])) return DFCSA_EINVAL;
  WgradArgs a;
  std::memset(&a, 0, sizeof(a));
  a.M = d->M; a.ng = 1; a.Cg = d->Cg; a.NI = NI;
  a.g_ptr[0] = d->g_ptr[0];
  a.nseg = 1; a.Cseg = d->Cseg; a.NJ = d->Cseg;
  a.seg[0].ptr = d->seg_ptr[0];
  a.Ho = d->Ho; a.Wo = d->Wo; a.Hi = d->Hi; a.Wi = d->Wi; a.stride = 1;
  a.layout = d->layout; a.ntaps = d->ntaps; a.Ctot = d->Ctot; a.Creal = d->Creal; a.ndst = d->ndst;
  for (int i = 0; i < 3; ++i) a.dst[i] = i < d->ndst ? d->dst[i] : nullptr;
  if (want_bias) for (int i = 0; i < 3; ++i) a.bdst[i] = d->bias_dst[i];
  SmallDgrad s;
  std::memset(&s, 0, sizeof(s));
  s.wt = wt; s.dx = dx; s.kpad = kpad; s.N = N;
  if (pc) {
    s.wsum = pc->wsum; s.mean = pc->mean; s.invstd = pc->invstd; s.rows = pc->rows;
    s.H = pc->H; s.W = pc->W; s.P = pc->P;
  }
  s.nwx = (NI + 15) / 16;
  s.nw = s.nwx * ((a.NJ + 63) / 64);
  s.ndx = (d->M + 15) / 16;
  const int grid = s.nw + s.ndx * ((N + 63) / 64);
  hipStream_t st = (hipStream_t)stream;
  ProfScope prof(DFCSA_PROF_WGRAD, st, 2.0 * d->M * NI * (a.NJ + N));
  if (g_small8) hipLaunchKernelGGL((small_wgrad_dgrad_f32_kernel<8, 4>), dim3(grid), dim3(512), 0, st, a, s);
  else hipLaunchKernelGGL((small_wgrad_dgrad_f32_kernel<4, 2>), dim3(grid), dim3(256), 0, st, a, s);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_conv_wgrad_dgrad1x1(const dfcsa_wgrad_desc* d, const float* wt, int kpad, int N, float* dx,
                                         void* stream) {
  return dfcsa_conv_wgrad_dgrad1x1_pool(d, wt, kpad, N, dx, nullptr, stream);
}
