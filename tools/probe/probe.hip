#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
// one wave: C[16x16] = A[16x32] * B[32x16]^T  (A row-major k-contig, B stored [n][k])
__global__ void mfma_probe(const __hip_bfloat16* A, const __hip_bfloat16* B, float* C) {
  int l = threadIdx.x;
  bf16x8 a = *(const bf16x8*)(A + (l & 15) * 32 + 8 * (l >> 4));
  bf16x8 b = *(const bf16x8*)(B + (l & 15) * 32 + 8 * (l >> 4));
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  for (int j = 0; j < 4; ++j) C[((l >> 4) * 4 + j) * 16 + (l & 15)] = acc[j];
}
extern "C" int probe_mfma(const void* A, const void* B, void* C, void* stream) {
  hipLaunchKernelGGL(mfma_probe, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (const __hip_bfloat16*)A, (const __hip_bfloat16*)B, (float*)C);
  return (int)hipGetLastError();
}
