// clip_grad_norm_(max_norm) + SGD(momentum, weight_decay) over one flat fp32 parameter buffer.
//
// Reference: utils/trainer.py:149-151 (torch.nn.utils.clip_grad_norm_, optimizer.step()) with
// torch.optim.SGD(lr, momentum, weight_decay) from train.py:73-78.  Semantics kept:
//   total = ||g||_2 over all parameters; coef = min(1, max_norm / (total + 1e-6));
//   g <- g * coef (written back: p.grad holds the clipped gradient afterwards, as in torch);
//   d = g + wd * w;  buf = d (first step) | momentum * buf + d;  w <- w - lr * buf.
// The squared norm is reduced in two deterministic stages (per-block fp64 partials, then every
// SGD block re-reduces the partials itself), so the whole update is one read of g/w/buf and
// one write of g/w/buf with no host synchronisation.  A NaN loss flag skips the update on the
// device (the reference's NaN `continue`, trainer.py:134-139: only NaN skips; an inf loss
// still steps).  A NaN total norm gives a NaN clip coefficient, as torch's clip_grad_norm_
// does (max_norm / (NaN + 1e-6) clamped to <= 1 stays NaN).
#include <algorithm>

#include "common.h"
#include "dfcsa_internal.h"

namespace {

constexpr int kParts = 1024;

__global__ void __launch_bounds__(256) sumsq_kernel(int64_t n, const float* __restrict__ g, double* __restrict__ part) {
  double s = 0.0;
  const int64_t n4 = n / 4;
  const float4* g4 = (const float4*)g;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 v = g4[i];
    s += (double)(v.x * v.x + v.y * v.y) + (double)(v.z * v.z + v.w * v.w);
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    s += (double)g[i] * g[i];
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) clip_sgd_kernel(int64_t n, float* __restrict__ w, float* __restrict__ g,
                                                       float* __restrict__ buf, const double* __restrict__ part,
                                                       int nparts, float max_norm, float grad_scale, float lr,
                                                       float momentum, float wd, const int* mom_init,
                                                       const float* skip, float* norm_out) {
  __shared__ double red[256];
  __shared__ float coef_s;
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float total = (float)sqrt(red[0]) * grad_scale;
    float c = max_norm / (total + 1e-6f);
    c = isnan(c) ? c : fminf(c, 1.f);
    coef_s = c * grad_scale;
    if (blockIdx.x == 0 && norm_out) *norm_out = total;
  }
  __syncthreads();
  if (skip && isnan(*skip)) return;
  const float coef = coef_s;
  const bool first = (*mom_init == 0);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float gc = g[i] * coef;
    g[i] = gc;
    const float wv = w[i];
    const float d = gc + wd * wv;
    const float b = first ? d : momentum * buf[i] + d;
    buf[i] = b;
    w[i] = wv - lr * b;
  }
}

// dfcsa_clip_sgd2: the momentum buffer starts at zero (momentum * 0 + d == d: torch's first step,
// bit for bit, with no first-step flag and no flag launch); zero_grad != 0 also zeroes the gradient
// (the next step's zero_grad memset is then skipped) -- on a skipped (NaN) step too
__global__ void __launch_bounds__(256) clip_sgd2_kernel(int64_t n, float* __restrict__ w, float* __restrict__ g,
                                                        float* __restrict__ buf, const double* __restrict__ part,
                                                        int nparts, float max_norm, float grad_scale, float lr,
                                                        float momentum, float wd, int zero_grad, const float* skip,
                                                        float* norm_out) {
  __shared__ double red[256];
  __shared__ float coef_s;
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float total = (float)sqrt(red[0]) * grad_scale;
    float c = max_norm / (total + 1e-6f);
    c = isnan(c) ? c : fminf(c, 1.f);
    coef_s = c * grad_scale;
    if (blockIdx.x == 0 && norm_out) *norm_out = total;
  }
  __syncthreads();
  if (skip && isnan(*skip)) {
    if (zero_grad)
      for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) g[i] = 0.f;
    return;
  }
  const float coef = coef_s;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float gc = g[i] * coef;
    g[i] = zero_grad ? 0.f : gc;
    const float wv = w[i];
    const float d = gc + wd * wv;
    const float b = momentum * buf[i] + d;
    buf[i] = b;
    w[i] = wv - lr * b;
  }
}

__global__ void set_flag_kernel(int* flag, const float* skip) {
  if (skip && isnan(*skip)) return;
  *flag = 1;
}

}  // namespace

extern "C" int dfcsa_sumsq_nparts(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(kParts, (n / 4 + 255) / 256));
}

extern "C" int dfcsa_sumsq_partial(int64_t n, const float* g, double* partial, void* stream) {
  if (n <= 0) return DFCSA_EINVAL;
  hipLaunchKernelGGL(sumsq_kernel, dim3(dfcsa_sumsq_nparts(n)), dim3(256), 0, (hipStream_t)stream, n, g, partial);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_clip_sgd(int64_t n, float* w, float* g, float* buf, const double* partial, int nparts,
                              float max_norm, float grad_scale, float lr, float momentum, float weight_decay,
                              int* mom_init, const float* skip_if_nan, float* norm_out, void* stream) {
  if (n <= 0 || !mom_init) return DFCSA_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  int blocks = (int)std::min<int64_t>(2048, (n + 255) / 256);
  hipLaunchKernelGGL(clip_sgd_kernel, dim3(blocks), dim3(256), 0, st, n, w, g, buf, partial, nparts, max_norm,
                     grad_scale, lr, momentum, weight_decay, mom_init, skip_if_nan, norm_out);
  DFCSA_CHECK_LAUNCH();
  hipLaunchKernelGGL(set_flag_kernel, dim3(1), dim3(1), 0, st, mom_init, skip_if_nan);
  DFCSA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfcsa_clip_sgd2(int64_t n, float* w, float* g, float* buf, const double* partial, int nparts,
                               float max_norm, float grad_scale, float lr, float momentum, float weight_decay,
                               int zero_grad, const float* skip_if_nan, float* norm_out, void* stream) {
  if (n <= 0) return DFCSA_EINVAL;
  int blocks = (int)std::min<int64_t>(2048, (n + 255) / 256);
  hipLaunchKernelGGL(clip_sgd2_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, n, w, g, buf, partial, nparts,
                     max_norm, grad_scale, lr, momentum, weight_decay, zero_grad, skip_if_nan, norm_out);
  DFCSA_CHECK_LAUNCH();
  return 0;
}
