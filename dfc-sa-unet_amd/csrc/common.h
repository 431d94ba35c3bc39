// Shared device/host helpers for libdfcsa (gfx950 / CDNA4 only).
//
// Element types: activations and packed weights are stored as T in {float, bf16 (uint16_t)};
// every reduction, accumulator and statistic is fp32 (fp64 where a whole-tensor sum is formed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DFCSA_DT_F32 0
#define DFCSA_DT_BF16 1

typedef uint16_t bf16_t;

// ---------------------------------------------------------------------------------------
// bf16 <-> f32.  The cast lowers to v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN-preserving).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}

template <typename T> struct ElemTraits;
template <> struct ElemTraits<float> {
  static constexpr int kChunk = 4;  // elements per 16-byte chunk
  __device__ __forceinline__ static float to_f(float v) { return v; }
  __device__ __forceinline__ static float from_f(float v) { return v; }
};
template <> struct ElemTraits<bf16_t> {
  static constexpr int kChunk = 8;
  __device__ __forceinline__ static float to_f(bf16_t v) { return bf2f(v); }
  __device__ __forceinline__ static bf16_t from_f(float v) { return f2bf(v); }
};

// 8 consecutive elements <-> 8 floats (16 B for bf16, 32 B for f32).  p must be 16-B aligned.
template <typename T> __device__ __forceinline__ void load8(const T* p, float (&v)[8]);
template <> __device__ __forceinline__ void load8<float>(const float* p, float (&v)[8]) {
  float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <> __device__ __forceinline__ void load8<bf16_t>(const bf16_t* p, float (&v)[8]) {
  uint4 u = *(const uint4*)p;
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xffff0000u);
  v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xffff0000u);
}
// 8 elements kept raw between the load and its use (bf16: one 16-B word, 4 VGPRs instead of 8),
// so that many loads can be in flight at a low register count
template <typename T> struct Raw8;
template <> struct Raw8<bf16_t> { uint4 a; };
template <> struct Raw8<float> { uint4 a, b; };
__device__ __forceinline__ void ld_raw8(const bf16_t* p, Raw8<bf16_t>& r) { r.a = *(const uint4*)p; }
__device__ __forceinline__ void ld_raw8(const float* p, Raw8<float>& r) {
  r.a = *(const uint4*)p;
  r.b = *(const uint4*)(p + 4);
}
__device__ __forceinline__ void cvt8(const Raw8<bf16_t>& r, float (&v)[8]) {
  const uint4 u = r.a;
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xffff0000u);
  v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xffff0000u);
}
__device__ __forceinline__ void cvt8(const Raw8<float>& r, float (&v)[8]) {
  v[0] = __uint_as_float(r.a.x); v[1] = __uint_as_float(r.a.y); v[2] = __uint_as_float(r.a.z);
  v[3] = __uint_as_float(r.a.w); v[4] = __uint_as_float(r.b.x); v[5] = __uint_as_float(r.b.y);
  v[6] = __uint_as_float(r.b.z); v[7] = __uint_as_float(r.b.w);
}
// base + a 32-bit byte offset: lets the compiler use the scalar-base + 32-bit-offset address form
// (one VGPR per address instead of two)
template <typename T> __device__ __forceinline__ const T* at_bytes(const T* base, unsigned byte_off) {
  return (const T*)((const char*)base + byte_off);
}
// 8 floats into LDS as two 16-B stores (p 16-B aligned).  Eight scalar stores at a lane stride of
// 8 words hit the same bank 8 lanes at a time; the wide stores are split over the banks.
__device__ __forceinline__ void lds_st8(float* p, const float (&v)[8]) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
template <typename T> __device__ __forceinline__ void store8(T* p, const float (&v)[8]);
template <> __device__ __forceinline__ void store8<float>(float* p, const float (&v)[8]) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}
template <> __device__ __forceinline__ void store8<bf16_t>(bf16_t* p, const float (&v)[8]) {
  uint4 u;
  u.x = pack2bf(v[0], v[1]); u.y = pack2bf(v[2], v[3]);
  u.z = pack2bf(v[4], v[5]); u.w = pack2bf(v[6], v[7]);
  *(uint4*)p = u;
}

// ---------------------------------------------------------------------------------------
// Fast unsigned division by a runtime constant (valid for 0 <= n < 2^31).
// ---------------------------------------------------------------------------------------
struct DivMod {
  int d;
  uint32_t mul;
  uint32_t shr;
};

static inline DivMod make_divmod(int d) {
  DivMod r;
  r.d = d;
  if (d <= 1) {
    r.mul = 0;
    r.shr = 0;
  } else {
    uint32_t l = 0;
    while ((1u << l) < (uint32_t)d) ++l;  // ceil(log2 d)
    uint32_t p = 31 + l;
    r.mul = (uint32_t)(((1ull << p) + (uint64_t)d - 1) / (uint64_t)d);
    r.shr = p - 32;
  }
  return r;
}

__device__ __forceinline__ int dm_div(const DivMod& dm, int n) {
  return dm.d == 1 ? n : (int)(__umulhi((uint32_t)n, dm.mul) >> dm.shr);
}

// ---------------------------------------------------------------------------------------
// wave reductions (wave64)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup fence + barrier and
// the fence drains vmcnt (outstanding global loads / stores / LDS-DMA) before the barrier, which
// serialises a DMA ring or a store stream; this waits for the wave's LDS operations only.  Global
// data (incl. LDS-DMA images) must be waited for explicitly with s_waitcnt vmcnt before it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Cross-workgroup hand-off helpers (last-arriver reductions): write-through (sc1) stores leave
// the XCD's L2 at once, sc1 loads do not hit a stale L2 line of another XCD; the writer waits for
// its stores (s_waitcnt vmcnt(0)) before taking an agent-scope ticket.
__device__ __forceinline__ void st_sc1_dw(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ float ld_sc1_f(const float* p) {
  float v;
  asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void st_sc1_d(double* p, double v) {
  asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
// three sc1 8-byte loads in flight, one wait
__device__ __forceinline__ void ld_sc1_d3(const double* p0, const double* p1, const double* p2, double& v0,
                                          double& v1, double& v2) {
  asm volatile(
      "global_load_dwordx2 %0, %3, off sc1\n\t"
      "global_load_dwordx2 %1, %4, off sc1\n\t"
      "global_load_dwordx2 %2, %5, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v0), "=&v"(v1), "=&v"(v2)
      : "v"(p0), "v"(p1), "v"(p2)
      : "memory");
}
// eight sc1 8-byte loads in flight, one wait
__device__ __forceinline__ void ld_sc1_d8(const double* const (&p)[8], double (&v)[8]) {
  asm volatile(
      "global_load_dwordx2 %0, %8, off sc1\n\t"
      "global_load_dwordx2 %1, %9, off sc1\n\t"
      "global_load_dwordx2 %2, %10, off sc1\n\t"
      "global_load_dwordx2 %3, %11, off sc1\n\t"
      "global_load_dwordx2 %4, %12, off sc1\n\t"
      "global_load_dwordx2 %5, %13, off sc1\n\t"
      "global_load_dwordx2 %6, %14, off sc1\n\t"
      "global_load_dwordx2 %7, %15, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7])
      : "memory");
}
// eight sc1 4-byte loads in flight, one wait (a last arriver's batched read of hand-off rows)
__device__ __forceinline__ void ld_sc1_f8(const float* const (&p)[8], float (&v)[8]) {
  asm volatile(
      "global_load_dword %0, %8, off sc1\n\t"
      "global_load_dword %1, %9, off sc1\n\t"
      "global_load_dword %2, %10, off sc1\n\t"
      "global_load_dword %3, %11, off sc1\n\t"
      "global_load_dword %4, %12, off sc1\n\t"
      "global_load_dword %5, %13, off sc1\n\t"
      "global_load_dword %6, %14, off sc1\n\t"
      "global_load_dword %7, %15, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7])
      : "memory");
}
typedef float f4v_t __attribute__((ext_vector_type(4)));
// sixteen sc1 16-byte loads in flight, one wait: rows r = 0..7 of a [row][ld] float matrix at p,
// 8 consecutive floats each (v[2r], v[2r + 1])
__device__ __forceinline__ void ld_sc1_f4x16(const float* p, int ld, f4v_t (&v)[16]) {
  const float* q[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) q[r] = p + (size_t)r * ld;
  asm volatile(
      "global_load_dwordx4 %0, %16, off sc1\n\t"
      "global_load_dwordx4 %1, %16, off offset:16 sc1\n\t"
      "global_load_dwordx4 %2, %17, off sc1\n\t"
      "global_load_dwordx4 %3, %17, off offset:16 sc1\n\t"
      "global_load_dwordx4 %4, %18, off sc1\n\t"
      "global_load_dwordx4 %5, %18, off offset:16 sc1\n\t"
      "global_load_dwordx4 %6, %19, off sc1\n\t"
      "global_load_dwordx4 %7, %19, off offset:16 sc1\n\t"
      "global_load_dwordx4 %8, %20, off sc1\n\t"
      "global_load_dwordx4 %9, %20, off offset:16 sc1\n\t"
      "global_load_dwordx4 %10, %21, off sc1\n\t"
      "global_load_dwordx4 %11, %21, off offset:16 sc1\n\t"
      "global_load_dwordx4 %12, %22, off sc1\n\t"
      "global_load_dwordx4 %13, %22, off offset:16 sc1\n\t"
      "global_load_dwordx4 %14, %23, off sc1\n\t"
      "global_load_dwordx4 %15, %23, off offset:16 sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]),
        "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]), "=&v"(v[12]), "=&v"(v[13]), "=&v"(v[14]), "=&v"(v[15])
      : "v"(q[0]), "v"(q[1]), "v"(q[2]), "v"(q[3]), "v"(q[4]), "v"(q[5]), "v"(q[6]), "v"(q[7])
      : "memory");
}
__device__ __forceinline__ float4 ld_sc1_f4(const float* p) {
  f4v_t v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(p) : "memory");
  return make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st_sc1_f4(float* p, float a, float b, float c, float d) {
  f4v_t v = {a, b, c, d};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// four sc1 16-byte loads in flight, one wait: p, p + ld, p + 2 ld, p + 3 ld
__device__ __forceinline__ void ld_sc1_f4x4(const float* p, int ld, f4v_t (&v)[4]) {
  asm volatile(
      "global_load_dwordx4 %0, %4, off sc1\n\t"
      "global_load_dwordx4 %1, %5, off sc1\n\t"
      "global_load_dwordx4 %2, %6, off sc1\n\t"
      "global_load_dwordx4 %3, %7, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
      : "v"(p), "v"(p + ld), "v"(p + 2 * ld), "v"(p + 3 * ld)
      : "memory");
}
// true in the workgroup that arrives last of `n` sharing *cnt (which it re-zeroes for the next
// launch); every thread calls it (contains barriers)
__device__ __forceinline__ bool wg_last_of(unsigned* cnt, unsigned n, int* flag_smem) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag_smem = old == n - 1;
    if (*flag_smem) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return *flag_smem != 0;
}

#define DFCSA_CHECK_LAUNCH() \
  do {                       \
    hipError_t e_ = hipGetLastError(); \
    if (e_ != hipSuccess) return -(int)e_; \
  } while (0)

#define DFCSA_EINVAL (-10000)

// XCD-aware workgroup order for 1-D grids padded to a multiple of 8: the hardware deals
// workgroup ids round-robin over the 8 XCDs (id % 8); this maps them so that each XCD walks
// one contiguous range of logical tiles (neighbouring tiles share halos / operand tiles in the
// XCD's own L2).  Returns -1 for padding ids.
__device__ __forceinline__ int xcd_remap(int lid, int total) {
  const int per = (total + 7) >> 3;
  const int L = (lid & 7) * per + (lid >> 3);
  return L < total ? L : -1;
}
__host__ __device__ inline int xcd_pad(int total) { return (total + 7) & ~7; }
