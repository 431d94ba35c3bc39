// Small-M fp32 GEMM tile on the f32 MFMA (v_mfma_f32_16x16x4_f32) for the LightSelfAttention
// projections (M = B * P * P pooled tokens, e.g. 256 rows): C[p][q] = sum_r P(p, r) * Q(q, r).
// One 256-thread workgroup owns a 16 x 64 output tile; its 4 waves split the reduction range r
// into contiguous quarters (16-wide blocks) and their partial tiles are summed through LDS in
// wave order -- a fixed order, so results are bitwise reproducible.  Many more workgroups than a
// 64x64 tile with a serial K loop (the latency-bound 15-16 us launches this replaces).
//   NT (TN = false): P(p, r) = Pm[p * ldp + r], Q(q, r) = Qm[q * ldq + r]  (both rows contiguous
//                    in r; conv forward / dgrad; r % 4 == 0 rows, 16-B aligned)
//   TN (TN = true):  P(p, r) = Pm[r * ldp + p], Q(q, r) = Qm[r * ldq + q]  (weight gradient:
//                    reduction over the pixel rows of two NHWC tensors)
// MFMA operand layout (16x16x4 f32): lane l supplies A[i = l & 15][k = l >> 4] and
// B[k = l >> 4][j = l & 15]; reduction index of lane group kk at sub-step t: r = 16 rb + 4 kk + t.
#pragma once
#include "common.h"

typedef float sg_f32x4 __attribute__((ext_vector_type(4)));

// NWV waves (blockDim = 64 NWV) split the reduction; UNR blocks of 16 are loaded before any is
// multiplied (the K loop is latency-bound: one L2 round trip per UNR blocks).  lds: NWV*16*64 floats.
template <bool TN, class Store, int NWV = 4, int UNR = 2>
__device__ __forceinline__ void small_gemm_tile(const float* __restrict__ Pm, int ldp, const float* __restrict__ Qm,
                                                int ldq, int Pn, int Qn, int R, int p0, int q0, float* lds,
                                                Store store) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l16 = lane & 15, kk = lane >> 4;
  const int nb = (R + 15) / 16;
  const int b0 = (w * nb) / NWV, b1 = ((w + 1) * nb) / NWV;
  sg_f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = {0.f, 0.f, 0.f, 0.f};
  const int p = p0 + l16;
  const bool pin = p < Pn;
#pragma unroll UNR
  for (int rb = b0; rb < b1; ++rb) {
    const int r = rb * 16 + 4 * kk;
    float pa[4], qa[4][4];
    if constexpr (!TN) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (pin && r < R) v = *(const float4*)(Pm + (size_t)p * ldp + r);
      pa[0] = v.x; pa[1] = v.y; pa[2] = v.z; pa[3] = v.w;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = q0 + j * 16 + l16;
        float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
        if (q < Qn && r < R) u = *(const float4*)(Qm + (size_t)q * ldq + r);
        qa[j][0] = u.x; qa[j][1] = u.y; qa[j][2] = u.z; qa[j][3] = u.w;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) pa[t] = (pin && r + t < R) ? Pm[(size_t)(r + t) * ldp + p] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = q0 + j * 16 + l16;
#pragma unroll
        for (int t = 0; t < 4; ++t) qa[j][t] = (q < Qn && r + t < R) ? Qm[(size_t)(r + t) * ldq + q] : 0.f;
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[t], qa[j][t], acc[j], 0, 0, 0);
  }
  // partial tiles of the NWV waves -> LDS [NWV][16][64], summed in wave order
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) lds[(w * 16 + kk * 4 + rr) * 64 + j * 16 + l16] = acc[j][rr];
  __syncthreads();
  for (int e = tid; e < 1024; e += NWV * 64) {
    const int pr = e >> 6, qc = e & 63;
    float s;
    if constexpr (NWV == 4) {
      s = ((lds[e] + lds[1024 + e]) + lds[2048 + e]) + lds[3072 + e];
    } else {
      s = 0.f;
#pragma unroll
      for (int v = 0; v < NWV; ++v) s += lds[v * 1024 + e];
    }
    const int pp = p0 + pr, qq = q0 + qc;
    if (pp < Pn && qq < Qn) store(pp, qq, s);
  }
}
