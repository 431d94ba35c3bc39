// DFC block elementwise stages and the train-mode BatchNorm machinery, NHWC, vectorised over
// 8-channel chunks (16-B bf16 / 32-B f32 accesses).
//
// Reference (models/unet_dfc_sa_res.py):
//   :57-62 local = ReLU(BN(conv3x3 x))           :65-69 a = ReLU(BN(conv1x1 x)) -> LSA
//   :36-38 attn = gamma * bilinear(o) + a        :73-77 g = Sigmoid(BN(conv1x1 [local, attn]))
//   :106  fused = g*local + (1-g)*attn           :80-84 ReLU(BN(conv1x1 [fused, local, attn]))
//   :113-114 out = out + res_scale * residual_conv(x)
// BatchNorm2d train semantics (torch.nn.BatchNorm2d, momentum 0.1, eps 1e-5): normalise with
// the biased batch variance, update running_var with the unbiased one.  The statistics come
// from the producing GEMM's epilogue (sums of the fp32 accumulator) so no extra pass is made.
//
// Backward: every BatchNorm backward is split into (1) an elementwise stage that forms
// dz = dL/d(BN output) and per-tile per-channel partial sums (sum dz, sum dz*xhat, ...), (2) a
// finalize that reduces the partial slabs in a fixed order (fp64) and (3) an apply stage
// dy = gamma*invstd*(dz - mean(dz) - xhat*mean(dz*xhat)) that also emits the conv-bias partial
// sums.  Nothing uses float atomics: results are bitwise reproducible.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "dfcsa_internal.h"

int g_ew_tile_elems = 16384;  // tuning knob 11: elements (pixels x channels) per reduction tile

namespace {

enum {
  EW_BN_ACT = 0,
  EW_LOCAL_ATTN,
  EW_GATE_FUSE,
  EW_BLOCK_OUT,
  EW_BWD_BLOCK_OUT,
  EW_BWD_RELU_BN,
  EW_BWD_GATE,
  EW_BWD_ATTN_ENTRY,
  EW_BN_BWD_APPLY,
  EW_CHANNEL_SUM,
  EW_SUM_OUT,       // ablation blocks: out = a0 (+ a1) + res_scale * a2
  EW_BWD_SUM_OUT,   // its backward: dres = res_scale * dout, partial sums of dout * res
  EW_BN_BWD_APPLY_RELU,   // BN_BWD_APPLY with dz = relu'(bn(y)) * dact recomputed (no dz tensor)
  EW_BN_BWD_APPLY_ENTRY,  // BN_BWD_APPLY with the attention-entry dz recomputed (no dz tensor)
};

struct EwArgs {
  int M, C, B, H, W, P, act;
  const void* a0;
  const void* a1;
  const void* a2;
  const void* a3;
  void* o0;
  void* o1;
  void* o2;
  void* o3;
  const float* sc;
  const float* sh;
  const float* sc2;
  const float* sh2;
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* coef;
  const float* tbl;     // o (fp32 [B][P][P][C]) or dpooled
  const float* scalar;  // gamma of LSA / res_scale
  float* partial;
  int64_t partial_cap;  // capacity of `partial` in floats (checked against the launch grid)
  int tile_px;          // pixels per reduction tile
  // adaptive-avg-pool backward lookups (pool_bwd_add): pixel -> (image, row, column) by
  // multiply-shift division; pool_exact: P divides H and W (one window per pixel, area pool_inv)
  DivMod dm_hw, dm_w, dm_ph, dm_pw;
  int pool_exact;
  int tbl16;     // tbl holds bf16 values (the bf16 flash layers' dpooled), else fp32
  float pool_inv;
  float bil_sh, bil_sw;   // bilinear upsample source scales P / H, P / W (host-computed quotients)
};

// host: fill the pool-backward lookup fields for an H x W map pooled to P x P
static void set_pool_geom(EwArgs& a) {
  a.dm_hw = make_divmod(a.H * a.W);
  a.dm_w = make_divmod(a.W);
  a.pool_exact = (a.P > 0 && a.H % a.P == 0 && a.W % a.P == 0) ? 1 : 0;
  a.dm_ph = make_divmod(a.pool_exact ? a.H / a.P : 1);
  a.dm_pw = make_divmod(a.pool_exact ? a.W / a.P : 1);
  a.pool_inv = a.pool_exact ? 1.f / (float)((a.H / a.P) * (a.W / a.P)) : 0.f;
  a.bil_sh = a.H > 0 ? (float)a.P / (float)a.H : 0.f;
  a.bil_sw = a.W > 0 ? (float)a.P / (float)a.W : 0.f;
}

__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// PyTorch upsample_bilinear2d (align_corners=False) source index/lambda for one axis.
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

// Raw 16-B (bf16) / 32-B (fp32) chunk of 8 elements: loads are issued as raw vectors and
// unpacked only when consumed, so a batch of U pixels costs 4 (bf16) VGPRs per input per pixel.
template <typename T> struct Raw;
template <> struct Raw<bf16_t> { uint4 v; };
template <> struct Raw<float> { float4 v0, v1; };
__device__ __forceinline__ Raw<bf16_t> ldraw(const bf16_t* p) { Raw<bf16_t> r; r.v = *(const uint4*)p; return r; }
__device__ __forceinline__ Raw<float> ldraw(const float* p) {
  Raw<float> r; r.v0 = *(const float4*)p; r.v1 = *(const float4*)(p + 4); return r;
}
__device__ __forceinline__ void unraw(const Raw<bf16_t>& r, float (&v)[8]) {
  const uint4 u = r.v;
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xffff0000u);
  v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xffff0000u);
}
__device__ __forceinline__ void unraw(const Raw<float>& r, float (&v)[8]) {
  v[0] = r.v0.x; v[1] = r.v0.y; v[2] = r.v0.z; v[3] = r.v0.w; v[4] = r.v1.x; v[5] = r.v1.y; v[6] = r.v1.z; v[7] = r.v1.w;
}

// ------------------------------- forward (no reductions) -------------------------------
// Each lane keeps ONE 8-channel chunk for the whole grid-stride loop (the stride, a multiple of
// 256 chunks, is a multiple of C/8 whenever C/8 divides 256 -- host-checked, `fixed`), so the
// per-channel BatchNorm parameters are loaded once; indices are 32-bit (M*C/8 < 2^31).
template <typename T, int MODE>
__global__ void __launch_bounds__(256) ew_fwd_kernel(const EwArgs a) {
  const T* __restrict__ A0 = (const T*)a.a0;
  const T* __restrict__ A1 = (const T*)a.a1;
  const T* __restrict__ A2 = (const T*)a.a2;
  T* __restrict__ O0 = (T*)a.o0;
  T* __restrict__ O1 = (T*)a.o1;
  const int cpp = a.C >> 3;
  const int total = a.M * cpp;
  const int first = blockIdx.x * 256 + threadIdx.x;
  const int stride = gridDim.x * 256;
  const bool fixed = (256 % cpp) == 0;
  float sc[8], sh[8], sc2[8], sh2[8];
  int c0 = (first % cpp) * 8;
  if (fixed) {
    if (a.a0 && a.sc) { ld8f(a.sc + c0, sc); ld8f(a.sh + c0, sh); }
    if constexpr (MODE == EW_LOCAL_ATTN) { ld8f(a.sc2 + c0, sc2); ld8f(a.sh2 + c0, sh2); }
  }
  if (fixed) {
    // batched: the loads of U chunks are issued before any of their stores (see ew_red_kernel)
    constexpr int U = sizeof(T) == 2 ? 4 : 2;
    constexpr int NIN = MODE == EW_GATE_FUSE || MODE == EW_SUM_OUT ? 3 : (MODE == EW_BN_ACT ? 1 : 2);
    const float scal = (a.scalar && (MODE == EW_LOCAL_ATTN || MODE == EW_BLOCK_OUT || MODE == EW_SUM_OUT))
                           ? *a.scalar : 0.f;
    const bool has0 = a.a0 != nullptr, has1 = a.a1 != nullptr, st0 = a.o0 != nullptr;
    const int elast = total - cpp + (first % cpp);   // last chunk of this lane's channel chunk
    for (int eb = first; eb < total; eb += U * stride) {
      Raw<T> in[U][NIN];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // unconditional loads (see ew_red_kernel): chunks past the end re-load a valid pixel of
        // this lane's channel chunk (stride is a multiple of cpp), their results are unused
        const int e = min(eb + u * stride, elast);
        {
          const size_t off = (size_t)(e / cpp) * a.C + c0;
          if (has0) in[u][0] = ldraw(A0 + off);
          if constexpr (MODE == EW_LOCAL_ATTN || MODE == EW_BLOCK_OUT || MODE == EW_GATE_FUSE) in[u][1] = ldraw(A1 + off);
          if constexpr (MODE == EW_GATE_FUSE) in[u][2] = ldraw(A2 + off);
          if constexpr (MODE == EW_SUM_OUT) {
            if (has1) in[u][1] = ldraw(A1 + off);
            in[u][2] = ldraw(A2 + off);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // keep every load of the batch ahead of its compute
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = eb + u * stride;
        if (e >= total) break;
        const int m = e / cpp;
        const size_t off = (size_t)m * a.C + c0;
        float y[8], out[8];
        if (has0) unraw(in[u][0], y);
        if constexpr (MODE == EW_BN_ACT) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float v = y[q] * sc[q] + sh[q];
            out[q] = a.act == 1 ? fmaxf(v, 0.f) : (a.act == 2 ? sigm(v) : v);
          }
          store8<T>(O0 + off, out);
        } else if constexpr (MODE == EW_LOCAL_ATTN) {
          if (st0) {
#pragma unroll
            for (int q = 0; q < 8; ++q) out[q] = fmaxf(y[q] * sc[q] + sh[q], 0.f);
            store8<T>(O0 + off, out);
          }
          float y2[8];
          unraw(in[u][1], y2);
          const int b = dm_div(a.dm_hw, m), rem = m - b * a.dm_hw.d, h = dm_div(a.dm_w, rem), w = rem - h * a.W;
          int h0, h1, w0, w1;
          float lh0, lh1, lw0, lw1;
          bilin_axis_s(h, a.P, a.bil_sh, h0, h1, lh0, lh1);
          bilin_axis_s(w, a.P, a.bil_sw, w0, w1, lw0, lw1);
          const float* ob = a.tbl + (size_t)b * a.P * a.P * a.C + c0;
          float o00[8], o01[8], o10[8], o11[8];
          ld8f(ob + (size_t)(h0 * a.P + w0) * a.C, o00);
          ld8f(ob + (size_t)(h0 * a.P + w1) * a.C, o01);
          ld8f(ob + (size_t)(h1 * a.P + w0) * a.C, o10);
          ld8f(ob + (size_t)(h1 * a.P + w1) * a.C, o11);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float upv = lh0 * (lw0 * o00[q] + lw1 * o01[q]) + lh1 * (lw0 * o10[q] + lw1 * o11[q]);
            const float v = y2[q] * sc2[q] + sh2[q];
            out[q] = scal * upv + (a.act ? fmaxf(v, 0.f) : v);
          }
          store8<T>(O1 + off, out);
        } else if constexpr (MODE == EW_GATE_FUSE) {
          float l[8], at[8];
          unraw(in[u][1], l);
          unraw(in[u][2], at);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float g = sigm(y[q] * sc[q] + sh[q]);
            out[q] = g * l[q] + (1.f - g) * at[q];
          }
          store8<T>(O0 + off, out);
        } else if constexpr (MODE == EW_BLOCK_OUT) {
          float r[8];
          unraw(in[u][1], r);
#pragma unroll
          for (int q = 0; q < 8; ++q) out[q] = fmaxf(y[q] * sc[q] + sh[q], 0.f) + scal * r[q];
          store8<T>(O0 + off, out);
        } else if constexpr (MODE == EW_SUM_OUT) {
          float r[8];
          unraw(in[u][2], r);
          if (has1) {
            float bb[8];
            unraw(in[u][1], bb);
#pragma unroll
            for (int q = 0; q < 8; ++q) y[q] += bb[q];
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) out[q] = y[q] + scal * r[q];
          store8<T>(O0 + off, out);
        }
      }
    }
    return;
  }
#pragma unroll 2
  for (int e = first; e < total; e += stride) {
    const int m = e / cpp;
    if (!fixed) {
      c0 = (e - m * cpp) * 8;
      if (a.a0 && a.sc) { ld8f(a.sc + c0, sc); ld8f(a.sh + c0, sh); }
      if constexpr (MODE == EW_LOCAL_ATTN) { ld8f(a.sc2 + c0, sc2); ld8f(a.sh2 + c0, sh2); }
    }
    const size_t off = (size_t)m * a.C + c0;
    float y[8], out[8];
    if (a.a0) load8<T>(A0 + off, y);
    if constexpr (MODE == EW_BN_ACT) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float v = y[q] * sc[q] + sh[q];
        out[q] = a.act == 1 ? fmaxf(v, 0.f) : (a.act == 2 ? sigm(v) : v);
      }
      store8<T>(O0 + off, out);
    } else if constexpr (MODE == EW_LOCAL_ATTN) {
      // a0 = y1 (sc, sh), a1 = y2 (sc2, sh2); tbl = o [B][P][P][C]; o0 = local, o1 = attn
      if (a.o0) {
#pragma unroll
        for (int q = 0; q < 8; ++q) out[q] = fmaxf(y[q] * sc[q] + sh[q], 0.f);
        store8<T>(O0 + off, out);
      }
      float y2[8];
      load8<T>(A1 + off, y2);
      const int b = dm_div(a.dm_hw, m), rem = m - b * a.dm_hw.d, h = dm_div(a.dm_w, rem), w = rem - h * a.W;
      int h0, h1, w0, w1;
      float lh0, lh1, lw0, lw1;
      bilin_axis_s(h, a.P, a.bil_sh, h0, h1, lh0, lh1);
      bilin_axis_s(w, a.P, a.bil_sw, w0, w1, lw0, lw1);
      const float* ob = a.tbl + (size_t)b * a.P * a.P * a.C + c0;
      float o00[8], o01[8], o10[8], o11[8];
      ld8f(ob + (size_t)(h0 * a.P + w0) * a.C, o00);
      ld8f(ob + (size_t)(h0 * a.P + w1) * a.C, o01);
      ld8f(ob + (size_t)(h1 * a.P + w0) * a.C, o10);
      ld8f(ob + (size_t)(h1 * a.P + w1) * a.C, o11);
      const float gm = *a.scalar;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float up = lh0 * (lw0 * o00[q] + lw1 * o01[q]) + lh1 * (lw0 * o10[q] + lw1 * o11[q]);
        const float v = y2[q] * sc2[q] + sh2[q];
        out[q] = gm * up + (a.act ? fmaxf(v, 0.f) : v);
      }
      store8<T>(O1 + off, out);
    } else if constexpr (MODE == EW_GATE_FUSE) {
      float l[8], at[8];
      load8<T>(A1 + off, l);
      load8<T>(A2 + off, at);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float g = sigm(y[q] * sc[q] + sh[q]);
        out[q] = g * l[q] + (1.f - g) * at[q];
      }
      store8<T>(O0 + off, out);
    } else if constexpr (MODE == EW_BLOCK_OUT) {
      float r[8];
      load8<T>(A1 + off, r);
      const float rs = *a.scalar;
#pragma unroll
      for (int q = 0; q < 8; ++q) out[q] = fmaxf(y[q] * sc[q] + sh[q], 0.f) + rs * r[q];
      store8<T>(O0 + off, out);
    } else if constexpr (MODE == EW_SUM_OUT) {
      // reference: fused = local + attn; out = fused + res_scale * res (fusion ablations)
      float r[8];
      load8<T>(A2 + off, r);
      if (a.a1) {
        float b[8];
        load8<T>(A1 + off, b);
#pragma unroll
        for (int q = 0; q < 8; ++q) y[q] += b[q];
      }
      const float rs = *a.scalar;
#pragma unroll
      for (int q = 0; q < 8; ++q) out[q] = y[q] + rs * r[q];
      store8<T>(O0 + off, out);
    }
  }
}

// ------------------------- backward stages with per-channel partial sums ----------------
template <int MODE> struct NSums { static constexpr int v = 2; };
template <> struct NSums<EW_BWD_BLOCK_OUT> { static constexpr int v = 3; };
template <> struct NSums<EW_BN_BWD_APPLY> { static constexpr int v = 1; };
template <> struct NSums<EW_BN_BWD_APPLY_RELU> { static constexpr int v = 1; };
template <> struct NSums<EW_BN_BWD_APPLY_ENTRY> { static constexpr int v = 1; };
template <> struct NSums<EW_CHANNEL_SUM> { static constexpr int v = 1; };
template <> struct NSums<EW_BWD_SUM_OUT> { static constexpr int v = 1; };

// Attention-entry gradient of pixel m (channels c0..c0+7): the adaptive-avg-pool backward of
// dpooled ([B][P][P][C] fp32), i.e. the sum over the pooling windows containing (h, w) of
// dpooled / window size (windows rows [floor(i*H/P), ceil((i+1)*H/P)) as torch's adaptive pool).
__device__ __forceinline__ void ld8_tbl(const EwArgs& a, size_t off, float (&v)[8]) {
  if (a.tbl16) {
    const uint4 u = *(const uint4*)((const bf16_t*)(const void*)a.tbl + off);
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
    v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xffff0000u);
    v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xffff0000u);
  } else {
    ld8f(a.tbl + off, v);
  }
}

__device__ __forceinline__ void pool_bwd_add(const EwArgs& a, int m, int c0, float (&add)[8]) {
  const int b = dm_div(a.dm_hw, m), rem = m - b * a.dm_hw.d, h = dm_div(a.dm_w, rem), w = rem - h * a.W;
  const int P = a.P;
  if (a.pool_exact) {
    // P divides H and W: the pixel lies in exactly one window of area (H/P)(W/P); the same
    // 1 / area as the general path below
    const int pi = dm_div(a.dm_ph, h), pj = dm_div(a.dm_pw, w);
    float v[8];
    ld8_tbl(a, ((size_t)(b * P + pi) * P + pj) * a.C + c0, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) add[q] = v[q] * a.pool_inv;
    return;
  }
  const int pi0 = (h * P) / a.H, pi1 = ((h + 1) * P + a.H - 1) / a.H - 1;
  const int pj0 = (w * P) / a.W, pj1 = ((w + 1) * P + a.W - 1) / a.W - 1;
#pragma unroll
  for (int q = 0; q < 8; ++q) add[q] = 0.f;
  for (int pi = pi0; pi <= pi1; ++pi) {
    const int hs = (pi * a.H) / P, he = ((pi + 1) * a.H + P - 1) / P;
    for (int pj = pj0; pj <= pj1; ++pj) {
      const int ws = (pj * a.W) / P, we = ((pj + 1) * a.W + P - 1) / P;
      const float inv = 1.f / (float)((he - hs) * (we - ws));
      float v[8];
      ld8_tbl(a, ((size_t)(b * P + pi) * P + pj) * a.C + c0, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) add[q] += v[q] * inv;
    }
  }
}

template <typename T, int MODE>
__device__ __forceinline__ void ew_red_body(const EwArgs& a, const int bx) {
  constexpr int NS = NSums<MODE>::v;
  const int cpp = a.C >> 3;                   // chunks per pixel (<= 256)
  const int pl = 256 / cpp;                   // pixel lanes
  const int tid = threadIdx.x;
  const int lane_px = tid / cpp, ck = tid - lane_px * cpp;
  const int c0 = ck * 8;
  const bool active = lane_px < pl;
  float acc[NS][8];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[s][q] = 0.f;

  // restrict-qualified views: the stores of one pixel cannot alias the loads of the next, so the
  // unrolled loop issues several pixels' loads back to back (memory-level parallelism)
  const T* __restrict__ A0 = (const T*)a.a0;
  const T* __restrict__ A1 = (const T*)a.a1;
  const T* __restrict__ A2 = (const T*)a.a2;
  const T* __restrict__ A3 = (const T*)a.a3;
  T* __restrict__ O0 = (T*)a.o0;
  T* __restrict__ O1 = (T*)a.o1;
  T* __restrict__ O2 = (T*)a.o2;
  const int mbeg = bx * a.tile_px;
  const int mend = min(a.M, mbeg + a.tile_px);
  float sc[8], sh[8], mu[8], is[8];
  float gk[8], k0[8], k1[8];   // BN_BWD_APPLY: gamma*invstd, coef0, coef1 (loop-invariant per lane)
  if (active) {
    if (a.sc) { ld8f(a.sc + c0, sc); ld8f(a.sh + c0, sh); }
    if (a.mean) { ld8f(a.mean + c0, mu); ld8f(a.invstd + c0, is); }
    if constexpr (MODE == EW_BN_BWD_APPLY || MODE == EW_BN_BWD_APPLY_RELU || MODE == EW_BN_BWD_APPLY_ENTRY) {
      ld8f(a.gamma + c0, gk);
      ld8f(a.coef + c0, k0);
      ld8f(a.coef + a.C + c0, k1);
#pragma unroll
      for (int q = 0; q < 8; ++q) gk[q] *= is[q];
    }
  }
  // Batched loop: all loads of U pixels are issued before any of their stores, so U pixels'
  // memory requests are in flight at once whatever alias analysis concludes (the compiler
  // otherwise orders every load after the previous pixel's stores: one round trip per pixel).
  constexpr int U = sizeof(T) == 2 ? 4 : 2;
  constexpr int NIN = MODE == EW_BWD_GATE ? 6 : (MODE == EW_BWD_BLOCK_OUT ? 3 : (MODE == EW_CHANNEL_SUM ? 1 : 2));
  const float scal = (a.scalar && (MODE == EW_BWD_BLOCK_OUT || MODE == EW_BWD_SUM_OUT)) ? *a.scalar : 0.f;
  const bool st0 = O0 != nullptr, st1 = O1 != nullptr;
  if (active) {
    for (int mb = mbeg + lane_px; mb < mend; mb += U * pl) {
      Raw<T> in[U][NIN];
      float add[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // no branch in the load phase (a conditional load makes the compiler merge registers
        // behind a wait): pixels past the tile re-load the last pixel, their results are unused
        const int m = min(mb + u * pl, mend - 1);
        {
          const size_t off = (size_t)m * a.C + c0;
          if constexpr (MODE == EW_CHANNEL_SUM) {
            in[u][0] = ldraw(A0 + off);
          } else if constexpr (MODE == EW_BWD_SUM_OUT) {
            in[u][0] = ldraw(A0 + off); in[u][1] = ldraw(A2 + off);
          } else if constexpr (MODE == EW_BWD_BLOCK_OUT) {
            in[u][0] = ldraw(A0 + off); in[u][1] = ldraw(A1 + off); in[u][2] = ldraw(A2 + off);
          } else if constexpr (MODE == EW_BWD_GATE) {
            in[u][0] = ldraw(A0 + off); in[u][1] = ldraw(A1 + off); in[u][2] = ldraw(A2 + off);
            in[u][3] = ldraw(A3 + off); in[u][4] = ldraw((const T*)O0 + off); in[u][5] = ldraw((const T*)O1 + off);
          } else {
            in[u][0] = ldraw(A0 + off); in[u][1] = ldraw(A1 + off);
          }
          if constexpr (MODE == EW_BWD_ATTN_ENTRY || MODE == EW_BN_BWD_APPLY_ENTRY) pool_bwd_add(a, m, c0, add[u]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // keep every load of the batch ahead of its compute
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = mb + u * pl;
        if (m >= mend) break;
        const size_t off = (size_t)m * a.C + c0;
        if constexpr (MODE == EW_CHANNEL_SUM) {
          float x[8];
          unraw(in[u][0], x);
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[0][q] += x[q];
        } else if constexpr (MODE == EW_BWD_SUM_OUT) {
          // a0 = dout, a2 = res; o1 = dres (optional)
          float d[8], r[8], dr[8];
          unraw(in[u][0], d);
          unraw(in[u][1], r);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            dr[q] = scal * d[q];
            acc[0][q] += d[q] * r[q];
          }
          if (st1) store8<T>(O1 + off, dr);
        } else if constexpr (MODE == EW_BWD_BLOCK_OUT) {
          // a0 = dout, a1 = y4, a2 = res; o0 = dz4 (optional), o1 = dres
          float d[8], y[8], r[8], dz[8], dr[8];
          unraw(in[u][0], d);
          unraw(in[u][1], y);
          unraw(in[u][2], r);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float z = (y[q] * sc[q] + sh[q] > 0.f) ? d[q] : 0.f;
            dz[q] = z;
            dr[q] = scal * d[q];
            acc[0][q] += z;
            acc[1][q] += z * ((y[q] - mu[q]) * is[q]);
            acc[2][q] += d[q] * r[q];
          }
          if (st0) store8<T>(O0 + off, dz);   // without dz4 the apply recomputes it
          store8<T>(O1 + off, dr);
        } else if constexpr (MODE == EW_BWD_RELU_BN) {
          float d[8], y[8], dz[8];
          unraw(in[u][0], d);
          unraw(in[u][1], y);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float z = (y[q] * sc[q] + sh[q] > 0.f) ? d[q] : 0.f;
            dz[q] = z;
            acc[0][q] += z;
            acc[1][q] += z * ((y[q] - mu[q]) * is[q]);
          }
          if (st0) store8<T>(O0 + off, dz);
        } else if constexpr (MODE == EW_BWD_GATE) {
          // a0 = dfused, a1 = y3, a2 = local, a3 = attn; o0 = dlocal(+=), o1 = dattn(+=), o2 = dz3
          float df[8], y[8], l[8], at[8], dl[8], da[8], dz[8];
          unraw(in[u][0], df);
          unraw(in[u][1], y);
          unraw(in[u][2], l);
          unraw(in[u][3], at);
          unraw(in[u][4], dl);
          unraw(in[u][5], da);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float g = sigm(y[q] * sc[q] + sh[q]);
            float dg = df[q] * (l[q] - at[q]);
            float z = dg * g * (1.f - g);
            dz[q] = z;
            dl[q] += df[q] * g;
            da[q] += df[q] * (1.f - g);
            acc[0][q] += z;
            acc[1][q] += z * ((y[q] - mu[q]) * is[q]);
          }
          store8<T>(O0 + off, dl);
          store8<T>(O1 + off, da);
          store8<T>(O2 + off, dz);
        } else if constexpr (MODE == EW_BWD_ATTN_ENTRY) {
          // a0 = dattn, a1 = y2, tbl = dpooled [B][P][P][C]; o0 = dz2 (optional)
          float d[8], y[8], dz[8];
          unraw(in[u][0], d);
          unraw(in[u][1], y);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float z = (!a.act || y[q] * sc[q] + sh[q] > 0.f) ? (d[q] + add[u][q]) : 0.f;
            dz[q] = z;
            acc[0][q] += z;
            acc[1][q] += z * ((y[q] - mu[q]) * is[q]);
          }
          if (st0) store8<T>(O0 + off, dz);
        } else if constexpr (MODE == EW_BN_BWD_APPLY || MODE == EW_BN_BWD_APPLY_RELU ||
                             MODE == EW_BN_BWD_APPLY_ENTRY) {
          // a0 = dz (APPLY) / the activation's output gradient (APPLY_RELU: dz = relu'(bn y) * a0;
          // APPLY_ENTRY: dz = act'(bn y) * (a0 + pool backward of tbl)), a1 = y; gamma, coef [2][C]
          // (hoisted); o0 = dy; sum dy (conv bias grad).  Recomputing dz costs a few VALU per
          // element and saves the dz tensor's write + read.
          float dz[8], y[8], dy[8];
          unraw(in[u][0], dz);
          unraw(in[u][1], y);
          if constexpr (MODE == EW_BN_BWD_APPLY_RELU) {
#pragma unroll
            for (int q = 0; q < 8; ++q) dz[q] = (y[q] * sc[q] + sh[q] > 0.f) ? dz[q] : 0.f;
          } else if constexpr (MODE == EW_BN_BWD_APPLY_ENTRY) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              dz[q] = (!a.act || y[q] * sc[q] + sh[q] > 0.f) ? (dz[q] + add[u][q]) : 0.f;
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float xh = (y[q] - mu[q]) * is[q];
            float v = gk[q] * (dz[q] - k0[q] - xh * k1[q]);
            dy[q] = v;
            acc[0][q] += v;
          }
          store8<T>(O0 + off, dy);
        }
      }
    }
  }
  if (!a.partial) return;  // sums not wanted (e.g. the analytically-zero conv-bias gradient)
  // deterministic in-workgroup reduction over pixel lanes
  __shared__ __attribute__((aligned(16))) float red[4 * 3 * 512];
  float* out = a.partial + (size_t)bx * NS * a.C;
  const bool pow2 = (cpp & (cpp - 1)) == 0;
  if (pow2 && cpp <= 64) {
    // lanes l and l ^ (k*cpp) hold the same channels: butterfly over the wave's pixel lanes,
    // then the 4 per-wave partials go through LDS
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float v = acc[s][q];
        for (int off = cpp; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
        acc[s][q] = v;
      }
    if (lane < cpp)   // 16-B stores (lds_st8): no 8-way bank conflicts
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        lds_st8(red + (wave * NS + s) * a.C + ck * 8, acc[s]);
      }
    __syncthreads();
    for (int e = tid; e < NS * a.C; e += 256) {
      const int s = e / a.C, c = e - s * a.C;
      out[e] = (red[(0 * NS + s) * a.C + c] + red[(1 * NS + s) * a.C + c]) +
               (red[(2 * NS + s) * a.C + c] + red[(3 * NS + s) * a.C + c]);
    }
    return;
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (active) {
      lds_st8(red + (lane_px * cpp + ck) * 8, acc[s]);
    }
    __syncthreads();
    for (int c = tid; c < a.C; c += 256) {
      const int k = c >> 3, q = c & 7;
      float v = 0.f;
      for (int p = 0; p < pl; ++p) v += red[(p * cpp + k) * 8 + q];
      out[s * a.C + c] = v;
    }
    __syncthreads();
  }
}

template <typename T, int MODE>
__global__ void __launch_bounds__(256) ew_red_kernel(const EwArgs a) {
  ew_red_body<T, MODE>(a, blockIdx.x);
}

// two independent reductions of one mode in one launch (workgroups [0, n0) take `a`, the rest `b`):
// e.g. the local branch's and the attention entry's BN-backward sums of a DFC block
template <typename T, int MODE>
__global__ void __launch_bounds__(256) ew_red_pair_kernel(const EwArgs a, const EwArgs b, int n0) {
  if ((int)blockIdx.x < n0) ew_red_body<T, MODE>(a, blockIdx.x);
  else ew_red_body<T, MODE>(b, blockIdx.x - n0);
}

// ---------------------------------------------------------------------------------------------
// Encoder block output fused with the 2x2 max-pool that follows it (reference
// models/unet_dfc_sa_res.py:113-114 then :165-172 MaxPool2d(2, 2); even H and W):
//   forward:  out = relu(bn4 y4) + res_scale*res for the 4 pixels of a window (stored: it is the
//             decoder's skip) and pooled = max over the window of the stored (rounded) values,
//             first maximum / NaN wins as ATen -- one pass instead of block_out + maxpool;
//   backward: dout = dskip + maxpool_bwd(dpooled) (ATen's routing to the first maximum of the
//             saved out) formed per window, stored, and the dfcsa_bwd_block_out stage on it
//             (dres = res_scale*dout; sums [dz4, dz4*xh4, dout*res]) -- one pass instead of the
//             pooling-gradient read-modify-write + the block-output backward.
// Thread = (pooled pixel, 8-channel chunk); the backward's per-channel sums are reduced per
// workgroup tile of pooled pixels as in ew_red_kernel (deterministic).
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) block_out_pool_kernel(int B, int H, int W, int C, const T* __restrict__ y4,
                                                             const float* __restrict__ sc4, const float* __restrict__ sh4,
                                                             const T* __restrict__ res, const float* __restrict__ rs,
                                                             T* __restrict__ out, T* __restrict__ pooled) {
  const int Ho = H / 2, Wo = W / 2, cpp = C >> 3;
  const int64_t total = (int64_t)B * Ho * Wo * cpp;
  const float scal = *rs;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ck = (int)(e % cpp);
    int64_t p = e / cpp;
    const int ow = (int)(p % Wo);
    p /= Wo;
    const int oh = (int)(p % Ho);
    const int b = (int)(p / Ho);
    float sc[8], sh[8];
    ld8f(sc4 + ck * 8, sc);
    ld8f(sh4 + ck * 8, sh);
    Raw<T> ry[4], rr[4];
    size_t off[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      off[t] = ((size_t)(b * H + 2 * oh + (t >> 1)) * W + 2 * ow + (t & 1)) * C + ck * 8;
      ry[t] = ldraw(y4 + off[t]);
      rr[t] = ldraw(res + off[t]);
    }
    float best[8];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float y[8], r[8], o[8];
      unraw(ry[t], y);
      unraw(rr[t], r);
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = fmaxf(y[q] * sc[q] + sh[q], 0.f) + scal * r[q];
      store8<T>(out + off[t], o);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = ElemTraits<T>::to_f(ElemTraits<T>::from_f(o[q]));   // the stored value
        if (t == 0 || v > best[q] || isnan(v)) best[q] = v;
      }
    }
    store8<T>(pooled + ((size_t)(b * Ho + oh) * Wo + ow) * C + ck * 8, best);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) bwd_block_out_pool_kernel(const EwArgs a, const T* __restrict__ xo,
                                                                 const T* __restrict__ dpool, T* __restrict__ dout) {
  // a: B, H, W (full resolution), C; a0 = dskip (nullable), a1 = y4, a2 = res; sc/sh/mean/invstd (BN4);
  // scalar = res_scale; o1 = dres; partial [ntiles][3][C]; tile_px = pooled pixels per workgroup
  constexpr int NS = 3;
  const int cpp = a.C >> 3;
  const int pl = 256 / cpp;
  const int tid = threadIdx.x;
  const int lane_px = tid / cpp, ck = tid - lane_px * cpp;
  const int c0 = ck * 8;
  const bool active = lane_px < pl;
  const int Ho = a.H / 2, Wo = a.W / 2;
  const int Mp = a.B * Ho * Wo;
  float acc[NS][8];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[s][q] = 0.f;
  const T* __restrict__ DS = (const T*)a.a0;
  const T* __restrict__ Y = (const T*)a.a1;
  const T* __restrict__ R = (const T*)a.a2;
  T* __restrict__ DR = (T*)a.o1;
  const int pbeg = blockIdx.x * a.tile_px;
  const int pend = min(Mp, pbeg + a.tile_px);
  if (active) {
    float sc[8], sh[8], mu[8], is[8];
    ld8f(a.sc + c0, sc); ld8f(a.sh + c0, sh); ld8f(a.mean + c0, mu); ld8f(a.invstd + c0, is);
    const float scal = *a.scalar;
    for (int pp = pbeg + lane_px; pp < pend; pp += pl) {
      const int ow = pp % Wo, t1 = pp / Wo, oh = t1 % Ho, b = t1 / Ho;
      size_t off[4];
      Raw<T> rx[4], ry[4], rr[4], rs[4];
      Raw<T> rg = ldraw(dpool + (size_t)pp * a.C + c0);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        off[t] = ((size_t)(b * a.H + 2 * oh + (t >> 1)) * a.W + 2 * ow + (t & 1)) * a.C + c0;
        rx[t] = ldraw(xo + off[t]);
        ry[t] = ldraw(Y + off[t]);
        rr[t] = ldraw(R + off[t]);
        if (DS) rs[t] = ldraw(DS + off[t]);
      }
      __builtin_amdgcn_sched_barrier(0);
      float best[8], g[8];
      int arg[8];
      unraw(rx[0], best);
      unraw(rg, g);
#pragma unroll
      for (int q = 0; q < 8; ++q) arg[q] = 0;
#pragma unroll
      for (int t = 1; t < 4; ++t) {
        float v[8];
        unraw(rx[t], v);
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (v[q] > best[q] || isnan(v[q])) { best[q] = v[q]; arg[q] = t; }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float d[8], y[8], r[8], dr[8];
        if (DS) unraw(rs[t], d);
        else {
#pragma unroll
          for (int q = 0; q < 8; ++q) d[q] = 0.f;
        }
        unraw(ry[t], y);
        unraw(rr[t], r);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          // dskip + pooled gradient at the window's first maximum, rounded as it is stored
          d[q] = ElemTraits<T>::to_f(ElemTraits<T>::from_f(d[q] + ((arg[q] == t) ? g[q] : 0.f)));
          const float z = (y[q] * sc[q] + sh[q] > 0.f) ? d[q] : 0.f;
          dr[q] = scal * d[q];
          acc[0][q] += z;
          acc[1][q] += z * ((y[q] - mu[q]) * is[q]);
          acc[2][q] += d[q] * r[q];
        }
        store8<T>(dout + off[t], d);
        store8<T>(DR + off[t], dr);
      }
    }
  }
  __shared__ __attribute__((aligned(16))) float red[4 * 3 * 512];
  float* outp = a.partial + (size_t)blockIdx.x * NS * a.C;
  const bool pow2 = (cpp & (cpp - 1)) == 0;
  if (pow2 && cpp <= 64) {
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float v = acc[s][q];
        for (int o = cpp; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
        acc[s][q] = v;
      }
    if (lane < cpp)   // 16-B stores (lds_st8): no 8-way bank conflicts
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        lds_st8(red + (wave * NS + s) * a.C + ck * 8, acc[s]);
      }
    __syncthreads();
    for (int e = tid; e < NS * a.C; e += 256) {
      const int s = e / a.C, c = e - s * a.C;
      outp[e] = (red[(0 * NS + s) * a.C + c] + red[(1 * NS + s) * a.C + c]) +
                (red[(2 * NS + s) * a.C + c] + red[(3 * NS + s) * a.C + c]);
    }
    return;
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (active) {
      lds_st8(red + (lane_px * cpp + ck) * 8, acc[s]);
    }
    __syncthreads();
    for (int c = tid; c < a.C; c += 256) {
      const int k = c >> 3, q = c & 7;
      float v = 0.f;
      for (int p2 = 0; p2 < pl; ++p2) v += red[(p2 * cpp + k) * 8 + q];
      outp[s * a.C + c] = v;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Column sums of per-tile partial rows, fused with the per-channel finalisation that consumes them
// (BatchNorm statistics, BatchNorm-backward coefficients, bias gradients): one launch instead of a
// row-reduction launch + a finalize launch.  grid (ceil(C/64), R), 1024 threads = 16 parts x 64
// channels; workgroup (x, g) sums rows [g*per, min(T, (g+1)*per)) of channel block x in double,
// 8 rows' loads in flight per thread.  R > 1: each group hands its NS double sums over through
// write-through (sc1) stores into a scratch ring, then takes an agent-scope ticket; the
// last-arriving group of block x reads all R hand-offs (sc1 loads) and combines them in a fixed
// order (deterministic), then finalises.  The partial rows are only read.
// ---------------------------------------------------------------------------------------------
constexpr int kRedRing = 1 << 16;          // ticket counters
constexpr int kRedScr = 1 << 20;           // hand-off doubles (8 MiB)
__device__ unsigned g_red_cnt[kRedRing];
__device__ double g_red_scr[kRedScr];

// twelve sc1 8-byte loads in flight, one wait
__device__ __forceinline__ void ld_sc1_d12(const double* const (&p)[12], double (&v)[12]) {
  asm volatile(
      "global_load_dwordx2 %0, %12, off sc1\n\t"
      "global_load_dwordx2 %1, %13, off sc1\n\t"
      "global_load_dwordx2 %2, %14, off sc1\n\t"
      "global_load_dwordx2 %3, %15, off sc1\n\t"
      "global_load_dwordx2 %4, %16, off sc1\n\t"
      "global_load_dwordx2 %5, %17, off sc1\n\t"
      "global_load_dwordx2 %6, %18, off sc1\n\t"
      "global_load_dwordx2 %7, %19, off sc1\n\t"
      "global_load_dwordx2 %8, %20, off sc1\n\t"
      "global_load_dwordx2 %9, %21, off sc1\n\t"
      "global_load_dwordx2 %10, %22, off sc1\n\t"
      "global_load_dwordx2 %11, %23, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]),
        "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7]), "v"(p[8]),
        "v"(p[9]), "v"(p[10]), "v"(p[11])
      : "memory");
}

// true (workgroup-uniform) if this workgroup finalises channel block x; part-0 threads then hold
// the column totals in tot[].  Column c of sum k of row t: src[t * rowlen + k * kstride + c].
template <int NS>
__device__ bool colred_block(const float* src, int T, int rowlen, int kstride, int C, int per, unsigned* cnt,
                             double* scr, double (&tot)[NS], double (*sh)[16][64], int* flag, int acq) {
  const int cl = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int R = gridDim.y, g = blockIdx.y;
  const int t0 = g * per, t1 = min(T, t0 + per);
  double s[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) s[k] = 0.0;
  if (c < C) {
    int t = t0 + part;
    for (; t + 7 * 16 < t1; t += 8 * 16) {  // 8 rows in flight, sequential order kept
      float v[8][NS];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < NS; ++k) v[j][k] = src[(size_t)(t + 16 * j) * rowlen + k * kstride + c];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < NS; ++k) s[k] += (double)v[j][k];
    }
    for (; t < t1; t += 16)
#pragma unroll
      for (int k = 0; k < NS; ++k) s[k] += (double)src[(size_t)t * rowlen + k * kstride + c];
  }
#pragma unroll
  for (int k = 0; k < NS; ++k) sh[k][part][cl] = s[k];
  __syncthreads();
  if (part == 0)
#pragma unroll
    for (int k = 0; k < NS; ++k)
      for (int p = 1; p < 16; ++p) s[k] += sh[k][p][cl];
  if (R == 1) {
#pragma unroll
    for (int k = 0; k < NS; ++k) tot[k] = s[k];
    return true;
  }
  if (part == 0) {   // scr[((x * R + g) * NS + k) * 64 + channel]
    double* slot = scr + ((size_t)(blockIdx.x * R + g) * NS) * 64 + cl;
#pragma unroll
    for (int k = 0; k < NS; ++k) st_sc1_d(slot + k * 64, s[k]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(cnt + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = old == (unsigned)(R - 1);
    if (*flag) {
      if (acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(cnt + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    }
  }
  __syncthreads();
  if (!*flag) return false;
  // part p combines groups p, p + 16, ... in order; the parts are then combined in order
  double gs[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) gs[k] = 0.0;
  if (R <= 16) {   // one group per part
    if (part < R) {
      const double* slot = scr + ((size_t)(blockIdx.x * R + part) * NS) * 64 + cl;
      double w[3];
      ld_sc1_d3(slot, slot + (NS > 1 ? 64 : 0), slot + (NS > 2 ? 128 : 0), w[0], w[1], w[2]);
#pragma unroll
      for (int k = 0; k < NS; ++k) gs[k] = w[k];
    }
  } else {  // groups part + 16 j (j < 4, R <= 64), every sum: one round of loads
    const double* p[12];
    const double* own = scr + ((size_t)(blockIdx.x * R + g) * NS) * 64 + cl;   // valid dummy
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int gg = part + 16 * j;
        p[j * 3 + k] = (gg < R && k < NS) ? scr + ((size_t)(blockIdx.x * R + gg) * NS + k) * 64 + cl : own;
      }
    double w[12];
    ld_sc1_d12(p, w);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < NS; ++k)
        if (part + 16 * j < R) gs[k] += w[j * 3 + k];
  }
#pragma unroll
  for (int k = 0; k < NS; ++k) sh[k][part][cl] = gs[k];
  __syncthreads();
  if (part == 0)
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      double v = 0.0;
      for (int p = 0; p < 16; ++p) v += sh[k][p][cl];
      tot[k] = v;
    }
  return true;
}

__global__ void __launch_bounds__(1024) bn_finalize_kernel(
    const float* __restrict__ stats, int ntiles, int per, unsigned* cnt, double* scr, int C, int ld, int count, const float* bias,
    const float* gamma, const float* beta, float* rmean, float* rvar, int64_t* nbt, float momentum, float eps,
    int training, float* scale, float* shift, float* mean, float* invstd, int acq) {
  __shared__ double sh[2][16][64];
  __shared__ int flag;
  const int cl = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double tot[2] = {0.0, 0.0};
  if (training && !colred_block<2>(stats, ntiles, 2 * ld, ld, C, per, cnt, scr, tot, sh, &flag, acq)) return;
  if (part == 0 && c < C) {
    float mu, var, istd;
    if (training) {
      const double n = (double)count;
      const double ma = tot[0] / n;
      double v = tot[1] / n - ma * ma;
      if (v < 0.0) v = 0.0;
      const double b = bias ? (double)bias[c] : 0.0;
      mu = (float)(ma + b);
      var = (float)v;
      istd = (float)(1.0 / sqrt(v + (double)eps));
      const double unb = count > 1 ? v * n / (n - 1.0) : v;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
      rvar[c] = (float)((1.0 - momentum) * (double)rvar[c] + momentum * unb);
    } else {
      mu = rmean[c];
      var = rvar[c];
      istd = 1.f / sqrtf(var + eps);
    }
    const float sc = gamma[c] * istd;
    scale[c] = sc;
    shift[c] = beta[c] - mu * sc;
    mean[c] = mu;
    invstd[c] = istd;
  }
  if (training && nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
}

// coef[0][c] = sum0 / count, coef[1][c] = sum1 / count; dgamma += sum1, dbeta += sum0; with a
// third sum (res_scale gradient) its channel total goes to third[c] and, once every channel block
// has finished (second ticket), the last one adds sum_c third[c] to *extra in channel order.
template <int NS>
__global__ void __launch_bounds__(1024) bn_bwd_finalize_kernel(const float* __restrict__ partial, int ntiles, int per,
                                                               unsigned* cnt, double* scr, int C, int count, float* coef,
                                                               float* dgamma, float* dbeta, float* third,
                                                               float* extra, int acq) {
  __shared__ double sh[NS][16][64];
  __shared__ int flag;
  const int cl = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double tot[NS];
  if (!colred_block<NS>(partial, ntiles, NS * C, C, C, per, cnt, scr, tot, sh, &flag, acq)) return;
  if (part == 0 && c < C) {
    coef[c] = (float)(tot[0] / count);
    coef[C + c] = (float)(tot[1] / count);
    if (dgamma) dgamma[c] += (float)tot[1];
    if (dbeta) dbeta[c] += (float)tot[0];
    if constexpr (NS > 2) {
      if (third) st_sc1_dw(third + c, (float)tot[2]);
    }
  }
  if constexpr (NS > 2) {
    if (!extra) return;
    unsigned* cnt2 = cnt + gridDim.x;
    if (gridDim.x > 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(cnt2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag = old == gridDim.x - 1;
        if (flag) {
          if (acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          __hip_atomic_store(cnt2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      __syncthreads();
      if (!flag) return;
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    // sum_c third[c], channel order: thread i adds channels i, i + 1024 (C <= 2048), then a tree
    double v = 0.0;
    for (int cc = threadIdx.x; cc < C; cc += 1024) v += (double)ld_sc1_f(third + cc);
    double* r = &sh[0][0][0];  // 1024 doubles (NS = 3: 3 x 16 x 64)
    r[threadIdx.x] = v;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
      if (threadIdx.x < o) r[threadIdx.x] += r[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) *extra += (float)r[0];
  }
}

// bn_bwd_finalize<2> for the attention entry of a DFC block, whose dz2 = r * (dattn + pool_bwd(dpooled))
// (r = relu'(bn2 y2)): the partial rows hold only the dattn part (dfcsa_bwd_relu_bn over dattn), and
// the pool part is the [B][N][C] contraction
//   sum_m r dz_pool = sum_{b,n} dpooled[b][n] / area_n * R[b][n],
//   sum_m r dz_pool xhat = sum_{b,n} dpooled[b][n] / area_n * invstd * (Y[b][n] - mean * R[b][n])
// with the forward pool's window sums R = sum r, Y = sum r*y2 (wsum [B][N][2][C]).  The 16 parts of
// the finalising workgroup take the (b, n) entries round-robin; parts combine in order (fp64).
__global__ void __launch_bounds__(1024) bn_bwd_finalize_pool_kernel(
    const float* __restrict__ partial, int ntiles, int per, unsigned* cnt, double* scr, int C, int count, float* coef,
    float* dgamma, float* dbeta, const float* __restrict__ dpooled, const float* __restrict__ wsum, int B, int H, int W,
    int P, const float* __restrict__ mean, const float* __restrict__ invstd, int acq) {
  __shared__ double sh[2][16][64];
  __shared__ int flag;
  const int cl = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double tot[2];
  if (!colred_block<2>(partial, ntiles, 2 * C, C, C, per, cnt, scr, tot, sh, &flag, acq)) return;
  __syncthreads();   // sh is reused below
  // 1 / window area per pooled position n (adaptive windows), once per workgroup
  __shared__ float inv_area[256];
  const int N = P * P;
  for (int n = threadIdx.x; n < N && n < 256; n += 1024) {
    const int pi = n / P, pj = n - pi * P;
    inv_area[n] = 1.f / (float)((((pi + 1) * H + P - 1) / P - (pi * H) / P) * (((pj + 1) * W + P - 1) / P - (pj * W) / P));
  }
  __syncthreads();
  double e0 = 0.0, e1 = 0.0;
  if (c < C) {
    const double mu = (double)mean[c], is = (double)invstd[c];
    const int BNn = B * N;
    const float rN = 1.f / (float)N;
    // part p takes entries p, p + 16, ...; eight entries' loads in flight per round, summed in order
    for (int eb = part; eb < BNn; eb += 16 * 8) {
      float d[8], r[8], y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = min(eb + 16 * u, BNn - 1);
        d[u] = dpooled[(size_t)e * C + c];
        r[u] = wsum[(size_t)e * 2 * C + c];
        y[u] = wsum[(size_t)e * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = eb + 16 * u;
        if (e >= BNn) break;
        const int n = e - N * (int)(((float)e + 0.5f) * rN);   // e mod N (exact: e < 2^20)
        const double dd = (double)d[u] * (double)(N <= 256 ? inv_area[n] : 0.f);
        e0 += dd * (double)r[u];
        e1 += dd * is * ((double)y[u] - mu * (double)r[u]);
      }
    }
  }
  sh[0][part][cl] = e0;
  sh[1][part][cl] = e1;
  __syncthreads();
  if (part != 0 || c >= C) return;
  for (int p = 0; p < 16; ++p) { tot[0] += sh[0][p][cl]; tot[1] += sh[1][p][cl]; }
  coef[c] = (float)(tot[0] / count);
  coef[C + c] = (float)(tot[1] / count);
  if (dgamma) dgamma[c] += (float)tot[1];
  if (dbeta) dbeta[c] += (float)tot[0];
}

// out[c] += sum_t slab[t][c]; columns split over up to three destinations at n0, n0 + n1
__global__ void __launch_bounds__(1024) slab_colsum_kernel(const float* __restrict__ slab, int ntiles, int per,
                                                           unsigned* cnt, double* scr, int C, int n0, int n1, float* d0,
                                                           float* d1, float* d2, int acq) {
  __shared__ double sh[1][16][64];
  __shared__ int flag;
  const int cl = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double tot[1];
  if (!colred_block<1>(slab, ntiles, C, 0, C, per, cnt, scr, tot, sh, &flag, acq)) return;
  if (part == 0 && c < C) {
    const double s = tot[0];
    if (c < n0) d0[c] += (float)s;
    else if (c < n0 + n1) d1[c - n0] += (float)s;
    else d2[c - n0 - n1] += (float)s;
  }
}

// dst[g][j] = sum over rows of group g of src[t][j]; grid (ceil(rowlen/256), G)
__global__ void __launch_bounds__(256) rows_reduce_kernel(const float* __restrict__ src, int T, int rowlen,
                                                          float* __restrict__ dst, int per) {
  const int j = blockIdx.x * 256 + threadIdx.x, g = blockIdx.y;
  if (j >= rowlen) return;
  const int t0 = g * per, t1 = min(T, t0 + per);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int t = t0;
  for (; t + 7 < t1; t += 8) {  // 8 rows in flight; same accumulation order as the 4-row step
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = src[(size_t)(t + k) * rowlen + j];
    s0 += v[0]; s1 += v[1]; s2 += v[2]; s3 += v[3];
    s0 += v[4]; s1 += v[5]; s2 += v[6]; s3 += v[7];
  }
  for (; t + 3 < t1; t += 4) {
    s0 += src[(size_t)t * rowlen + j];
    s1 += src[(size_t)(t + 1) * rowlen + j];
    s2 += src[(size_t)(t + 2) * rowlen + j];
    s3 += src[(size_t)(t + 3) * rowlen + j];
  }
  for (; t < t1; ++t) s0 += src[(size_t)t * rowlen + j];
  dst[(size_t)g * rowlen + j] = (s0 + s1) + (s2 + s3);
}

// one workgroup, fixed summation order; 4 independent loads in flight per thread for the long
// (per-pixel) vectors of the attention gammas (NT = 1024 there, 256 for per-channel vectors)
template <int NT>
__global__ void __launch_bounds__(NT) sum_scalar_kernel(const float* x, int n, float* out) {
  __shared__ double r[NT];
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  int i = threadIdx.x;
  for (; i + 3 * NT < n; i += 4 * NT) {
    s0 += x[i];
    s1 += x[i + NT];
    s2 += x[i + 2 * NT];
    s3 += x[i + 3 * NT];
  }
  for (; i < n; i += NT) s0 += x[i];
  r[threadIdx.x] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) r[threadIdx.x] += r[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out += (float)r[0];
}

void launch_sum_scalar(const float* x, int n, float* out, hipStream_t st) {
  if (n > 4096) hipLaunchKernelGGL(sum_scalar_kernel<1024>, dim3(1), dim3(1024), 0, st, x, n, out);
  else hipLaunchKernelGGL(sum_scalar_kernel<256>, dim3(1), dim3(256), 0, st, x, n, out);
}

// pixels per reduction tile: ~16 chunk-iterations per thread (fewer, fuller tiles than a fixed size)
inline int tile_px(int C) {
  const int cpp = C / 8, pl = 256 / (cpp > 0 ? cpp : 1);
  int t = g_ew_tile_elems / (C > 0 ? C : 1);
  if (t < pl) t = pl;
  return t;
}

template <int MODE>
int launch_fwd(int dtype, const EwArgs& a, hipStream_t st) {
  if (a.C % 8 || a.M <= 0 || (int64_t)a.M * (a.C / 8) >= (1ll << 31)) return DFCSA_EINVAL;
  int64_t chunks = (int64_t)a.M * (a.C / 8);
  // one batch (4 chunks) per thread where the grid allows (the kernel's batched loop)
  int blocks = (int)std::min<int64_t>((chunks + 1023) / 1024, 65535);
  if (dtype == DFCSA_DT_BF16) hipLaunchKernelGGL((ew_fwd_kernel<bf16_t, MODE>), dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((ew_fwd_kernel<float, MODE>), dim3(blocks), dim3(256), 0, st, a);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

template <int MODE>
int launch_red(int dtype, EwArgs a, hipStream_t st) {
  if (a.C % 8 || a.C > 2048 || a.M <= 0) return DFCSA_EINVAL;
  a.tile_px = tile_px(a.C);
  int blocks = (a.M + a.tile_px - 1) / a.tile_px;
  // the partial slab holds one [NS][C] row per workgroup: refuse a slab shorter than the grid
  if (a.partial && (int64_t)blocks * NSums<MODE>::v * a.C > a.partial_cap) return DFCSA_EINVAL;
  if (dtype == DFCSA_DT_BF16) hipLaunchKernelGGL((ew_red_kernel<bf16_t, MODE>), dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((ew_red_kernel<float, MODE>), dim3(blocks), dim3(256), 0, st, a);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

EwArgs zargs(int M, int C) {
  EwArgs a;
  std::memset(&a, 0, sizeof(a));
  a.M = M;
  a.C = C;
  return a;
}

}  // namespace

// row groups of a fused column reduction (colred_block): ~128 rows per group (one round of 8
// loads per thread), at most 64 groups; tickets: nblk (+ extra) counters from a ring (each last
// arriver re-zeroes its counter); hand-off scratch: nblk * R * ns * 64 doubles from a ring
struct RedPlan {
  int R = 1, per = 1;
  unsigned* cnt = nullptr;
  double* scr = nullptr;
  int acq = 1;   // 1: the last arriver takes an agent-scope acquire before reading the hand-offs
};
// Ticket counters and hand-off scratch.  With DFCSA_RED_ACQ=0 they are allocated with hipMalloc at
// first use (eager, before any graph capture): on that memory the hand-off is the measured acquire-free form of
// MI355X_MICROARCH.md (Valid forms, hand-off table row 1: every hand-off byte stored sc1 and drained
// by vmcnt(0) in every storing wave, one lane's agent-scope atomic add behind a workgroup barrier,
// the last adder told by the returned value, every load of the bytes an 8-B sc1 load after its add
// returned / behind the barrier it then joins), which saves the ~1.7 us buffer_inv of the acquire on
// every finalize.  Otherwise (default) the code object's arrays and the acquire are used.
static int red_mem(unsigned** ring, double** scr) {
  static unsigned* r = nullptr;
  static double* sc = nullptr;
  static int acq = -1;
  if (acq < 0) {
    unsigned* a = nullptr;
    double* b = nullptr;
    // default: the code-object arrays with the acquire; DFCSA_RED_ACQ=0 selects the acquire-free
    // form on hipMalloc memory (same-box A/B of the default bench: 1554 / 1554 img/s against 1571 /
    // 1558 with the acquire -- no gain, so the documented-safe form stays the default)
    const char* force = getenv("DFCSA_RED_ACQ");
    if (force && force[0] == '0' && hipMalloc((void**)&a, sizeof(unsigned) * kRedRing) == hipSuccess &&
        hipMalloc((void**)&b, sizeof(double) * kRedScr) == hipSuccess) {
      static unsigned zero[kRedRing];   // zero-initialised
      if (hipMemcpy(a, zero, sizeof(zero), hipMemcpyHostToDevice) == hipSuccess) {
        r = a;
        sc = b;
        acq = 0;
      }
    }
    if (acq < 0) {
      if (a) (void)hipFree(a);
      if (b) (void)hipFree(b);
      (void)hipGetLastError();
      if (hipGetSymbolAddress((void**)&r, HIP_SYMBOL(g_red_cnt)) != hipSuccess ||
          hipGetSymbolAddress((void**)&sc, HIP_SYMBOL(g_red_scr)) != hipSuccess)
        return -1;
      acq = 1;
    }
  }
  *ring = r;
  *scr = sc;
  return acq;
}

// next free word of the hand-off scratch ring (shared by red_plan and dfcsa_scratch_alloc)
static int64_t g_scr_next = 0;

static int red_plan(int T, int nblk, int ns, int extra, RedPlan* p) {
  int R = (T + 127) / 128;
  if (R > 64) R = 64;
  const int64_t rmax = (int64_t)(kRedScr / 4) / ((int64_t)(nblk > 0 ? nblk : 1) * (ns > 0 ? ns : 1) * 64);
  if (R > rmax) R = (int)rmax;
  if (R < 1) R = 1;
  int per = (T + R - 1) / R;
  while (R > 1 && T - (R - 1) * per < 1) {   // no empty group
    --R;
    per = (T + R - 1) / R;
  }
  p->R = R;
  p->per = per;
  p->cnt = nullptr;
  const int need = nblk + extra;
  unsigned* ring = nullptr;
  double* scr = nullptr;
  if (R > 1 || extra) {
    const int acq = red_mem(&ring, &scr);
    if (acq < 0) return DFCSA_EINVAL;
    p->acq = acq;
  }
  if (R > 1 || extra) {
    static int next = 0;
    if (need > kRedRing) return DFCSA_EINVAL;
    if (next + need > kRedRing) next = 0;
    p->cnt = ring + next;
    next += need;
  }
  if (R > 1) {
    const int64_t words = (int64_t)nblk * R * ns * 64;
    if (words > kRedScr) return DFCSA_EINVAL;
    if (g_scr_next + words > kRedScr) g_scr_next = 0;
    p->scr = scr + g_scr_next;
    g_scr_next += words;
  }
  return 0;
}

// tickets for other translation units' last-arriver hand-offs (same ring as the reductions here)
unsigned* dfcsa_ticket_alloc(int n) {
  RedPlan rp;
  return red_plan(1, 0, 0, n, &rp) ? nullptr : rp.cnt;
}

double* dfcsa_scratch_alloc(int64_t n) {
  unsigned* ring = nullptr;
  double* scr = nullptr;
  if (n <= 0 || n > kRedScr || red_mem(&ring, &scr) < 0) return nullptr;
  if (g_scr_next + n > kRedScr) g_scr_next = 0;
  double* p = scr + g_scr_next;
  g_scr_next += n;
  return p;
}

extern "C" int dfcsa_ew_ntiles(int M, int C) { return (M + tile_px(C) - 1) / tile_px(C); }

extern "C" int dfcsa_bn_finalize(const float* stats, int ntiles, int C, int ld, int count, const float* conv_bias,
                                 const float* gamma, const float* beta, float* running_mean, float* running_var,
                                 int64_t* nbt, float momentum, float eps, int training, float* scale,
                                 float* shift, float* mean, float* invstd, void* stream) {
  if (C <= 0 || (training && (!stats || count <= 0 || ntiles <= 0))) return DFCSA_EINVAL;
  const int nblk = (C + 63) / 64;
  RedPlan rp;
  if (training && red_plan(ntiles, nblk, 2, 0, &rp)) return DFCSA_EINVAL;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(nblk, rp.R), dim3(1024), 0, (hipStream_t)stream, stats, ntiles,
                     rp.per, rp.cnt, rp.scr, C, ld, count, conv_bias, gamma, beta, running_mean, running_var, nbt, momentum,
                     eps, training, scale, shift, mean, invstd, rp.acq);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_bn_act(int dtype, int M, int C, const void* y, const float* scale, const float* shift,
                            int act, void* out, void* stream) {
  EwArgs a = zargs(M, C);
  a.a0 = y; a.sc = scale; a.sh = shift; a.act = act; a.o0 = out;
  return launch_fwd<EW_BN_ACT>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_block_local_attn(int dtype, int B, int H, int W, int C, const void* y1, const float* sc1,
                                      const float* sh1, const void* y2, const float* sc2, const float* sh2,
                                      const float* o, int P, const float* gamma, int relu, void* local,
                                      void* attn, void* stream) {
  EwArgs a = zargs(B * H * W, C);
  a.B = B; a.H = H; a.W = W; a.P = P;
  a.a0 = y1; a.sc = sc1; a.sh = sh1; a.a1 = y2; a.sc2 = sc2; a.sh2 = sh2; a.tbl = o; a.scalar = gamma;
  a.o0 = y1 ? local : nullptr; a.o1 = attn; a.act = relu;
  set_pool_geom(a);
  return launch_fwd<EW_LOCAL_ATTN>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_gate_fuse(int dtype, int M, int C, const void* y3, const float* sc3, const float* sh3,
                               const void* local, const void* attn, void* fused, void* stream) {
  EwArgs a = zargs(M, C);
  a.a0 = y3; a.sc = sc3; a.sh = sh3; a.a1 = local; a.a2 = attn; a.o0 = fused;
  return launch_fwd<EW_GATE_FUSE>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_block_out(int dtype, int M, int C, const void* y4, const float* sc4, const float* sh4,
                               const void* res, const float* res_scale, void* out, void* stream) {
  EwArgs a = zargs(M, C);
  a.a0 = y4; a.sc = sc4; a.sh = sh4; a.a1 = res; a.scalar = res_scale; a.o0 = out;
  return launch_fwd<EW_BLOCK_OUT>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_bwd_block_out(int dtype, int M, int C, const void* dout, const void* y4, const float* sc4,
                                   const float* sh4, const float* mean4, const float* invstd4, const void* res,
                                   const float* res_scale, void* dz4, void* dres, float* partial, int64_t partial_floats, void* stream) {
  EwArgs a = zargs(M, C);
  a.a0 = dout; a.a1 = y4; a.a2 = res; a.sc = sc4; a.sh = sh4; a.mean = mean4; a.invstd = invstd4;
  a.scalar = res_scale; a.o0 = dz4; a.o1 = dres; a.partial = partial; a.partial_cap = partial_floats;
  return launch_red<EW_BWD_BLOCK_OUT>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_sum_out(int dtype, int M, int C, const void* a, const void* b, const void* res,
                              const float* res_scale, void* out, void* stream) {
  if (!a || !res || !res_scale || !out) return DFCSA_EINVAL;
  EwArgs e = zargs(M, C);
  e.a0 = a; e.a1 = b; e.a2 = res; e.scalar = res_scale; e.o0 = out;
  return launch_fwd<EW_SUM_OUT>(dtype, e, (hipStream_t)stream);
}

extern "C" int dfcsa_bwd_sum_out(int dtype, int M, int C, const void* dout, const void* res, const float* res_scale,
                                  void* dres, float* partial, int64_t partial_floats, void* stream) {
  if (!dout || !res || !res_scale || !partial) return DFCSA_EINVAL;
  EwArgs e = zargs(M, C);
  e.a0 = dout; e.a2 = res; e.scalar = res_scale; e.o1 = dres; e.partial = partial; e.partial_cap = partial_floats;
  return launch_red<EW_BWD_SUM_OUT>(dtype, e, (hipStream_t)stream);
}

extern "C" int dfcsa_sum_into(const float* x, int n, float* out, void* stream) {
  if (!x || !out || n <= 0) return DFCSA_EINVAL;
  launch_sum_scalar(x, n, out, (hipStream_t)stream);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_bwd_relu_bn(int dtype, int M, int C, const void* dact, const void* y, const float* sc,
                                 const float* sh, const float* mean, const float* invstd, void* dz,
                                 float* partial, int64_t partial_floats, void* stream) {
  EwArgs a = zargs(M, C);
  a.a0 = dact; a.a1 = y; a.sc = sc; a.sh = sh; a.mean = mean; a.invstd = invstd; a.o0 = dz; a.partial = partial; a.partial_cap = partial_floats;
  return launch_red<EW_BWD_RELU_BN>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_bwd_relu_bn_pair(int dtype, int M, int C, const void* dact0, const void* y0, const float* sc0,
                                      const float* sh0, const float* mean0, const float* invstd0, float* partial0,
                                      const void* dact1, const void* y1, const float* sc1, const float* sh1,
                                      const float* mean1, const float* invstd1, float* partial1,
                                      int64_t partial_floats, void* stream) {
  EwArgs a = zargs(M, C), b = zargs(M, C);
  a.a0 = dact0; a.a1 = y0; a.sc = sc0; a.sh = sh0; a.mean = mean0; a.invstd = invstd0;
  a.partial = partial0; a.partial_cap = partial_floats;
  b.a0 = dact1; b.a1 = y1; b.sc = sc1; b.sh = sh1; b.mean = mean1; b.invstd = invstd1;
  b.partial = partial1; b.partial_cap = partial_floats;
  if (C % 8 || C > 2048 || M <= 0 || !partial0 || !partial1) return DFCSA_EINVAL;
  a.tile_px = b.tile_px = tile_px(C);
  const int blocks = (M + a.tile_px - 1) / a.tile_px;
  if ((int64_t)blocks * 2 * C > partial_floats) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL((ew_red_pair_kernel<bf16_t, EW_BWD_RELU_BN>), dim3(2 * blocks), dim3(256), 0, st, a, b, blocks);
  else
    hipLaunchKernelGGL((ew_red_pair_kernel<float, EW_BWD_RELU_BN>), dim3(2 * blocks), dim3(256), 0, st, a, b, blocks);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_bwd_gate(int dtype, int M, int C, const void* dfused, const void* y3, const float* sc3,
                              const float* sh3, const float* mean3, const float* invstd3, const void* local,
                              const void* attn, void* dlocal, void* dattn, void* dz3, float* partial, int64_t partial_floats,
                              void* stream) {
  EwArgs a = zargs(M, C);
  a.a0 = dfused; a.a1 = y3; a.a2 = local; a.a3 = attn; a.sc = sc3; a.sh = sh3; a.mean = mean3;
  a.invstd = invstd3; a.o0 = dlocal; a.o1 = dattn; a.o2 = dz3; a.partial = partial; a.partial_cap = partial_floats;
  return launch_red<EW_BWD_GATE>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_bwd_attn_entry(int dtype, int B, int H, int W, int C, const void* dattn,
                                    const float* dpooled, int P, const void* y2, const float* sc2,
                                    const float* sh2, const float* mean2, const float* invstd2, int relu,
                                    void* dz2, float* partial, int64_t partial_floats, void* stream) {
  EwArgs a = zargs(B * H * W, C);
  a.B = B; a.H = H; a.W = W; a.P = P;
  a.a0 = dattn; a.a1 = y2; a.tbl = dpooled; a.sc = sc2; a.sh = sh2; a.mean = mean2; a.invstd = invstd2;
  a.o0 = dz2; a.partial = partial; a.partial_cap = partial_floats; a.act = relu;
  if (P <= 0) return DFCSA_EINVAL;
  set_pool_geom(a);
  return launch_red<EW_BWD_ATTN_ENTRY>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_bn_bwd_finalize(const float* partial, int ntiles, int nsum, int C, int count, float* coef,
                                     float* dgamma, float* dbeta, float* extra, void* stream) {
  if (nsum < 2 || nsum > 3 || C <= 0 || C > 2048 || ntiles <= 0) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int nblk = (C + 63) / 64;
  // the third per-channel sum (res_scale gradient) is stored in the tail of `coef` ([3][C]) and, with
  // `extra`, reduced to the scalar *extra by the last channel block (a second ticket level); without
  // it the caller sums coef[2C, 3C) off the critical path (dfcsa_sum_into on another stream)
  float* third = nsum == 3 ? coef + 2 * C : nullptr;
  RedPlan rp;
  if (red_plan(ntiles, nblk, nsum, extra && third ? 1 : 0, &rp)) return DFCSA_EINVAL;
  if (nsum == 3)
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<3>, dim3(nblk, rp.R), dim3(1024), 0, st, partial, ntiles, rp.per,
                       rp.cnt, rp.scr, C, count, coef, dgamma, dbeta, third, extra, rp.acq);
  else
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<2>, dim3(nblk, rp.R), dim3(1024), 0, st, partial, ntiles, rp.per,
                       rp.cnt, rp.scr, C, count, coef, dgamma, dbeta, nullptr, nullptr, rp.acq);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_bn_bwd_finalize_pool(const float* partial, int ntiles, int C, int count, float* coef,
                                          float* dgamma, float* dbeta, const float* dpooled, const float* wsum, int B,
                                          int H, int W, int P, const float* mean, const float* invstd, void* stream) {
  if (!partial || ntiles <= 0 || C <= 0 || count <= 0 || !coef || !dpooled || !wsum || !mean || !invstd || B <= 0 ||
      P <= 0 || P * P > 256 || H <= 0 || W <= 0 || (int64_t)B * P * P >= (1 << 20))
    return DFCSA_EINVAL;
  const int nblk = (C + 63) / 64;
  RedPlan rp;
  if (red_plan(ntiles, nblk, 2, 0, &rp)) return DFCSA_EINVAL;
  hipLaunchKernelGGL(bn_bwd_finalize_pool_kernel, dim3(nblk, rp.R), dim3(1024), 0, (hipStream_t)stream, partial,
                     ntiles, rp.per, rp.cnt, rp.scr, C, count, coef, dgamma, dbeta, dpooled, wsum, B, H, W, P, mean,
                     invstd, rp.acq);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_bn_bwd_apply(int dtype, int M, int C, const void* dz, const void* y, const float* mean,
                                  const float* invstd, const float* gamma, const float* coef, void* dy,
                                  float* bias_partial, int64_t bias_partial_floats, void* stream) {
  EwArgs a = zargs(M, C);
  a.a0 = dz; a.a1 = y; a.mean = mean; a.invstd = invstd; a.gamma = gamma; a.coef = coef; a.o0 = dy;
  a.partial = bias_partial; a.partial_cap = bias_partial_floats;
  return launch_red<EW_BN_BWD_APPLY>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_bn_bwd_apply_relu(int dtype, int M, int C, const void* dact, const void* y, const float* sc,
                                       const float* sh, const float* mean, const float* invstd, const float* gamma,
                                       const float* coef, void* dy, float* bias_partial, int64_t bias_partial_floats, void* stream) {
  if (!dact || !y || !sc || !sh || !mean || !invstd || !gamma || !coef || !dy) return DFCSA_EINVAL;
  EwArgs a = zargs(M, C);
  a.a0 = dact; a.a1 = y; a.sc = sc; a.sh = sh; a.mean = mean; a.invstd = invstd; a.gamma = gamma; a.coef = coef;
  a.o0 = dy; a.partial = bias_partial; a.partial_cap = bias_partial_floats;
  return launch_red<EW_BN_BWD_APPLY_RELU>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_bn_bwd_apply_entry(int dtype, int B, int H, int W, int C, const void* dattn,
                                        const float* dpooled, int P, const void* y, const float* sc,
                                        const float* sh, const float* mean, const float* invstd, int relu,
                                        const float* gamma, const float* coef, void* dy, float* bias_partial, int64_t bias_partial_floats,
                                        void* stream) {
  if (!dattn || !dpooled || P <= 0 || !y || !sc || !sh || !mean || !invstd || !gamma || !coef || !dy)
    return DFCSA_EINVAL;
  EwArgs a = zargs(B * H * W, C);
  a.B = B; a.H = H; a.W = W; a.P = P;
  a.a0 = dattn; a.a1 = y; a.tbl = dpooled; a.sc = sc; a.sh = sh; a.mean = mean; a.invstd = invstd; a.act = relu;
  a.gamma = gamma; a.coef = coef; a.o0 = dy; a.partial = bias_partial; a.partial_cap = bias_partial_floats;
  set_pool_geom(a);
  return launch_red<EW_BN_BWD_APPLY_ENTRY>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_bn_bwd_apply_entry16(int dtype, int B, int H, int W, int C, const void* dattn,
                                          const void* dpooled16, int P, const void* y, const float* sc,
                                          const float* sh, const float* mean, const float* invstd, int relu,
                                          const float* gamma, const float* coef, void* dy, float* bias_partial,
                                          int64_t bias_partial_floats, void* stream) {
  if (!dattn || !dpooled16 || P <= 0 || !y || !sc || !sh || !mean || !invstd || !gamma || !coef || !dy ||
      ((uintptr_t)dpooled16 & 15))
    return DFCSA_EINVAL;
  EwArgs a = zargs(B * H * W, C);
  a.B = B; a.H = H; a.W = W; a.P = P;
  a.a0 = dattn; a.a1 = y; a.tbl = (const float*)dpooled16; a.tbl16 = 1; a.sc = sc; a.sh = sh; a.mean = mean;
  a.invstd = invstd; a.act = relu;
  a.gamma = gamma; a.coef = coef; a.o0 = dy; a.partial = bias_partial; a.partial_cap = bias_partial_floats;
  set_pool_geom(a);
  return launch_red<EW_BN_BWD_APPLY_ENTRY>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_slab_colsum(const float* slab, int ntiles, int C, float* out, void* stream) {
  return dfcsa_slab_colsum3(slab, ntiles, C, C, 0, out, nullptr, nullptr, stream);
}

extern "C" int dfcsa_slab_colsum3(const float* slab, int ntiles, int C, int n0, int n1, float* d0, float* d1,
                                  float* d2, void* stream) {
  if (C <= 0 || ntiles <= 0 || n0 < 0 || n1 < 0 || n0 + n1 > C || !d0 || (n1 && !d1) || (n0 + n1 < C && !d2))
    return DFCSA_EINVAL;
  const int nblk = (C + 63) / 64;
  RedPlan rp;
  if (red_plan(ntiles, nblk, 1, 0, &rp)) return DFCSA_EINVAL;
  hipLaunchKernelGGL(slab_colsum_kernel, dim3(nblk, rp.R), dim3(1024), 0, (hipStream_t)stream, slab, ntiles, rp.per,
                     rp.cnt, rp.scr, C, n0, n1, d0, d1, d2, rp.acq);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_channel_sum(int dtype, int M, int C, const void* x, float* partial, int64_t partial_floats, void* stream) {
  EwArgs a = zargs(M, C);
  a.a0 = x; a.partial = partial; a.partial_cap = partial_floats;
  return launch_red<EW_CHANNEL_SUM>(dtype, a, (hipStream_t)stream);
}

extern "C" int dfcsa_rows_reduce(const float* src, int T, int rowlen, float* dst, int G, void* stream) {
  if (T <= 0 || rowlen <= 0 || G <= 0) return DFCSA_EINVAL;
  const int per = (T + G - 1) / G;
  hipLaunchKernelGGL(rows_reduce_kernel, dim3((rowlen + 255) / 256, G), dim3(256), 0, (hipStream_t)stream, src, T,
                     rowlen, dst, per);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_sum_to_scalar(const float* x, int n, float* out, void* stream) {
  if (n <= 0) return DFCSA_EINVAL;
  launch_sum_scalar(x, n, out, (hipStream_t)stream);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

// pooled pixels per workgroup tile of dfcsa_bwd_block_out_pool (a quarter of the elementwise tile)
static int pool_tile(int C) { int t = tile_px(C) / 4; const int pl = 256 / (C / 8 > 0 ? C / 8 : 1); return t < pl ? pl : t; }

extern "C" int dfcsa_block_out_pool(int dtype, int B, int H, int W, int C, const void* y4, const float* sc4,
                                    const float* sh4, const void* res, const float* res_scale, void* out,
                                    void* pooled, void* stream) {
  if (C % 8 || C > 2048 || (H & 1) || (W & 1) || B <= 0 || H <= 0 || W <= 0 || !y4 || !sc4 || !sh4 || !res ||
      !res_scale || !out || !pooled)
    return DFCSA_EINVAL;
  const int64_t n = (int64_t)B * (H / 2) * (W / 2) * (C / 8);
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 65535);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(block_out_pool_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, B, H, W, C, (const bf16_t*)y4, sc4,
                       sh4, (const bf16_t*)res, res_scale, (bf16_t*)out, (bf16_t*)pooled);
  else
    hipLaunchKernelGGL(block_out_pool_kernel<float>, dim3(blocks), dim3(256), 0, st, B, H, W, C, (const float*)y4, sc4,
                       sh4, (const float*)res, res_scale, (float*)out, (float*)pooled);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_bwd_block_out_pool_ntiles(int B, int H, int W, int C) {
  if (C <= 0 || (H & 1) || (W & 1)) return DFCSA_EINVAL;
  const int Mp = B * (H / 2) * (W / 2), t = pool_tile(C);
  return (Mp + t - 1) / t;
}

extern "C" int dfcsa_bwd_block_out_pool(int dtype, int B, int H, int W, int C, const void* dskip, const void* out,
                                        const void* dpooled, const void* y4, const float* sc4, const float* sh4,
                                        const float* mean4, const float* invstd4, const void* res,
                                        const float* res_scale, void* dout, void* dres, float* partial, int64_t partial_floats, void* stream) {
  if (C % 8 || C > 2048 || (H & 1) || (W & 1) || B <= 0 || !out || !dpooled || !y4 || !sc4 || !sh4 || !mean4 ||
      !invstd4 || !res || !res_scale || !dout || !dres || !partial)
    return DFCSA_EINVAL;
  EwArgs a = zargs(B * H * W, C);
  a.B = B; a.H = H; a.W = W;
  a.a0 = dskip; a.a1 = y4; a.a2 = res; a.sc = sc4; a.sh = sh4; a.mean = mean4; a.invstd = invstd4;
  a.scalar = res_scale; a.o1 = dres; a.partial = partial; a.partial_cap = partial_floats;
  a.tile_px = pool_tile(C);
  const int Mp = B * (H / 2) * (W / 2);
  const int blocks = (Mp + a.tile_px - 1) / a.tile_px;
  if ((int64_t)blocks * 3 * C > partial_floats) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DFCSA_DT_BF16)
    hipLaunchKernelGGL(bwd_block_out_pool_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, a, (const bf16_t*)out,
                       (const bf16_t*)dpooled, (bf16_t*)dout);
  else
    hipLaunchKernelGGL(bwd_block_out_pool_kernel<float>, dim3(blocks), dim3(256), 0, st, a, (const float*)out,
                       (const float*)dpooled, (float*)dout);
  DFCSA_CHECK_LAUNCH();
  return 0;
}
