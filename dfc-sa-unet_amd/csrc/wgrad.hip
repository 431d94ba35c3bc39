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

template <int BI, int BJ, int WM, int WN, int NST>
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

  auto issue = [&](int kt, int buf) {
    char* G = smem + buf * STAGE;
    char* X = G + GB;
    const int mb = mbeg + kt * KMS;
#pragma unroll
    for (int q = 0; q < NI_G; ++q) {
      const int m = mb + g_row[q];
      const void* src = (g_src[q] && m < mend) ? (const void*)(g_src[q] + (size_t)m * args.Cg) : zero;
      __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(G + (q * NW + wave) * 1024), 16, 0, 0);
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
      __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(X + (q * NW + wave) * 1024), 16, 0, 0);
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

  wgrad_epilogue<FM, FN, NW>(args, acc, L % (nJ * nI), split, i0 + wm * WTM, j0 + wn * WTN, lane, wave, tid,
                             (int*)smem);
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
  } else {
    // ConvTranspose2d weight [Cin][Cout][2][2]; i = ci, j = ij*Cout + co (Ctot = Cout)
    int ij = j / Ctot, co = j - ij * Ctot;
    d0[((int64_t)i * Ctot + co) * 4 + ij] += s;
  }
}

// fp32 weight gradient over few pixel rows (the LightSelfAttention projections, M = B*P*P): the
// whole reduction in one launch (split over the 4 waves of a 16x64 tile, small_gemm.h), added
// straight into the destination layout -- no split-K slab, no reduce launch
__global__ void __launch_bounds__(256) small_wgrad_f32_kernel(const WgradArgs a) {
  __shared__ float lds[4 * 16 * 64];
  small_gemm_tile<true>((const float*)a.g_ptr[0], a.NI, (const float*)a.seg[0].ptr, a.Cseg, a.NI, a.NJ, a.M,
                        blockIdx.x * 16, blockIdx.y * 64, lds, [&](int i, int j, float v) {
                          reduce_dst_add((int64_t)i * a.NJ + j, a.NI, a.NJ, a.layout, a.ntaps, a.Ctot, a.Creal,
                                         a.ndst, a.dst[0], a.dst[1], a.dst[2], v);
                        });
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

int launch_reduce(const float* slab, int splits, int NI, int NJ, int layout, int ntaps, int Ctot, int Creal, int ndst,
                  float* d0, float* d1, float* d2, hipStream_t st) {
  const int64_t total = (int64_t)NI * NJ;
  const int blocks = (int)((total + 63) / 64);
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

template <typename T, int BI>
int launch_wgrad(const WgradArgs& a, int splits, hipStream_t st) {
  constexpr int BJ = 128;
  dim3 grid((a.NJ + BJ - 1) / BJ, (a.NI + BI - 1) / BI, splits);
  // 8 waves (32x64 wave tiles) hide more latency: LDS-DMA + 8 waves measured best or equal on
  // every shape of the step (tools/wgrad_bench.py; 5-15 % on the 3x3 layers)
  const int waves = g_wgrad_waves ? g_wgrad_waves : 8;
  if constexpr (sizeof(T) == 2) {
    if (!g_wgrad_noglds) {
      if (const int bm = wgrad_big_mode(a.NI, a.NJ, g_wgrad_big)) {
        const int bi = bm == 3 ? 128 : 256, bj = bm == 2 ? 128 : 256;
        dim3 gb(xcd_pad(((a.NJ + bj - 1) / bj) * ((a.NI + bi - 1) / bi) * splits));
        if (bm == 1) hipLaunchKernelGGL((wgrad_glds_kernel<256, 256, 2, 4, 2>), gb, dim3(512), 0, st, a, splits);
        else if (bm == 2) hipLaunchKernelGGL((wgrad_glds_kernel<256, 128, 4, 2, 2>), gb, dim3(512), 0, st, a, splits);
        else hipLaunchKernelGGL((wgrad_glds_kernel<128, 256, 2, 4, 2>), gb, dim3(512), 0, st, a, splits);
        DFCSA_CHECK_LAUNCH();
        return 0;
      }
      // 1-D grid (x = padded tile count, y = splits count carrier): see the XCD remap in the kernel
      if (BI == 64 && wide_j(a)) {
        dim3 g2(xcd_pad(((a.NJ + 255) / 256) * ((a.NI + BI - 1) / BI) * splits), splits);
        g2.y = 1;
        hipLaunchKernelGGL((wgrad_glds_kernel<64, 256, 2, 4, 2>), g2, dim3(512), 0, st, a, splits);
      } else {
        dim3 g1(xcd_pad(grid.x * grid.y * splits));
        constexpr int WM8 = BI == 64 ? 2 : 4, WN8 = BI == 64 ? 4 : 2;
        if (waves == 8 && g_wgrad_nst >= 4)
          hipLaunchKernelGGL((wgrad_glds_kernel<BI, BJ, WM8, WN8, 4>), g1, dim3(512), 0, st, a, splits);
        else if (waves == 8 && g_wgrad_nst == 3)
          hipLaunchKernelGGL((wgrad_glds_kernel<BI, BJ, WM8, WN8, 3>), g1, dim3(512), 0, st, a, splits);
        else if (waves == 8)
          hipLaunchKernelGGL((wgrad_glds_kernel<BI, BJ, WM8, WN8, 2>), g1, dim3(512), 0, st, a, splits);
        else
          hipLaunchKernelGGL((wgrad_glds_kernel<BI, BJ, 2, 2, 2>), g1, dim3(256), 0, st, a, splits);
      }
      DFCSA_CHECK_LAUNCH();
      return 0;
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

int g_wgrad_waves = 0;     // waves per wgrad workgroup (dfcsa_set_tuning knob 6; 0 = automatic)
int g_wgrad_noglds = 0;    // 1 = register-staged bf16 wgrad (dfcsa_set_tuning knob 7)
int g_wgrad_narrow = 1;    // 0 = allow the 64x256 wgrad tile (dfcsa_set_tuning knob 8; measured slower on the L1 3x3)
int g_wgrad_target = 512;  // workgroups per wgrad launch (dfcsa_set_tuning knob 2)
int g_wgrad_nst = 2;       // knob 14: LDS-DMA ring depth of the bf16 wgrad kernel (2, 3, 4)
int g_wgrad_fuse_all = 0;  // knob 12: 1 = reduce in-kernel at any split count, -1 = never (separate launch)
// knob 13: most splits reduced in-kernel.  Default 0 = never: measured on the headline step
// (tools/wgrad_shapes.py, bench A/B) the last arriver's serialized read of the partials costs more
// than the separate fixed-order reduction launch (W4 H14: 114 vs 72 us; step 1172 vs 1198 img/s at
// <= 4 splits, 1149 at <= 16), so the fused path stays selectable, tested, and off.
int g_wgrad_fuse_max = 0;
int g_wgrad_noglds_f32small = 0;  // knob 16: 1 = fp32 small-M wgrads take the generic tiles

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
  a.layout = d->layout; a.ntaps = d->ntaps; a.Ctot = d->Ctot; a.Creal = d->Creal; a.ndst = d->ndst;
  for (int i = 0; i < 3; ++i) a.dst[i] = i < d->ndst ? d->dst[i] : nullptr;
  if (d->ndst > 0) {
    if (d->layout == 2 ? (d->ndst != 3 || d->Ctot <= 0 || 2 * d->Ctot > a.NI) : (a.NI % d->ndst != 0)) return DFCSA_EINVAL;
    if (d->Ctot <= 0) return DFCSA_EINVAL;
  }
  // one split: the kernel adds its tile straight into dst (no slab, no second launch)
  a.fuse = d->ndst > 0 && (d->splits == 1 ||
                           (g_wgrad_fuse_all >= 0 && (d->splits <= g_wgrad_fuse_max || g_wgrad_fuse_all > 0)));
  if (!a.fuse && !d->slab) return DFCSA_EINVAL;
  a.cnt = nullptr;
  if (a.fuse && d->splits > 1) {
    // ticket counters: a ring region per launch, so launches in flight on other streams never
    // share one (each tile's last arriver re-zeroes its counter)
    static unsigned* ring = nullptr;
    static int next = 0;
    if (!ring && hipGetSymbolAddress((void**)&ring, HIP_SYMBOL(g_wg_cnt)) != hipSuccess) return DFCSA_EINVAL;
    int BI, BJ;
    wgrad_tile(a.NI, a.NJ, d->dtype, &BI, &BJ);
    const int tiles = ((a.NI + BI - 1) / BI) * ((a.NJ + BJ - 1) / BJ);
    if (tiles > kCntRing) return DFCSA_EINVAL;
    if (next + tiles > kCntRing) next = 0;
    a.cnt = ring + next;
    next += tiles;
  }
  hipStream_t st = (hipStream_t)stream;
  double flops = 2.0 * a.M * a.NI * a.NJ;
  ProfScope prof(DFCSA_PROF_WGRAD, st, flops);   // the class covers the reduction launch too
  if (d->dtype != DFCSA_DT_BF16 && a.M <= 4096 && a.ng == 1 && a.nseg == 1 && !a.seg[0].dh && !a.seg[0].dw &&
      a.stride == 1 && d->ndst > 0 && a.Ho == a.Hi && a.Wo == a.Wi && !g_wgrad_noglds_f32small) {
    hipLaunchKernelGGL(small_wgrad_f32_kernel, dim3((a.NI + 15) / 16, (a.NJ + 63) / 64), dim3(256), 0, st, a);
    DFCSA_CHECK_LAUNCH();
    return 0;
  }
  int rc;
  if (d->dtype == DFCSA_DT_BF16)
    rc = a.NI <= 64 ? launch_wgrad<bf16_t, 64>(a, d->splits, st) : launch_wgrad<bf16_t, 128>(a, d->splits, st);
  else
    rc = a.NI <= 64 ? launch_wgrad<float, 64>(a, d->splits, st) : launch_wgrad<float, 128>(a, d->splits, st);
  if (rc) return rc;
  if (d->ndst > 0 && !a.fuse)
    return launch_reduce(d->slab, d->splits, a.NI, a.NJ, d->layout, d->ntaps, d->Ctot, d->Creal, d->ndst, a.dst[0],
                         a.dst[1], a.dst[2], st);
  return 0;
}

extern "C" int dfcsa_wgrad_reduce(const float* slab, int splits, int NI, int NJ, int layout, int ntaps,
                                  int Ctot, int Creal, int ndst, float* const* dst, void* stream) {
  if (!slab || !dst || ndst < 1 || ndst > 3) return DFCSA_EINVAL;
  if (layout == 2 ? (ndst != 3 || Ctot <= 0 || 2 * Ctot > NI) : (NI % ndst != 0)) return DFCSA_EINVAL;
  return launch_reduce(slab, splits, NI, NJ, layout, ntaps, Ctot, Creal, ndst, dst[0], ndst > 1 ? dst[1] : nullptr,
                       ndst > 2 ? dst[2] : nullptr, (hipStream_t)stream);
}
