// Fused global-norm clip + Adagrad over the flat fp32 parameter buffer
// (reference model.py:288-305: clip_by_global_norm(max_grad_norm) then
// AdagradOptimizer(lr, initial_accumulator_value)).
//
// All trainable tensors live as views of ONE contiguous fp32 buffer (and their grads of
// one contiguous grad buffer, which is also the DP all-reduce bucket storage), so the
// whole optimizer is two launches with no host sync:
//   1. sumsq:   per-block partial sums of g^2 (deterministic two-level reduction)
//   2. adagrad: norm = gscale * sqrt(sum partials) (every block recomputes it from 1024
//               floats), scale = gscale * max_norm / max(norm, max_norm); g' = g*scale;
//               acc += g'^2; w -= lr * g' / sqrt(acc)
// gscale folds the data-parallel 1/world average of the summed gradient into the update
// (no separate pass over the 86 MB buffer after the all-reduce).
// A non-finite norm skips the update (NaN guard) and sets *flag = 1.  A
// non-zero *skip word (the persistent-LSTM hand-off error, sticky) also skips it and sets
// *flag |= 2: garbage gradients from a timed-out recurrence are never applied.
#include "common.h"

#define OPT_BLOCKS 1024

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, long n, float* __restrict__ part) {
  __shared__ float red[8];
  float s = 0.f;
  const long n4 = n / 4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float4 x = g4[i];
    s += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
  }
  for (long i = n4 * 4 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) s += g[i] * g[i];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void adagrad_kernel(float* __restrict__ w, float* __restrict__ acc,
                                                      const float* __restrict__ g, long n,
                                                      const float* __restrict__ part, int nparts, float lr,
                                                      float max_norm, float gscale, float* __restrict__ norm_out,
                                                      int* __restrict__ flag, const int* __restrict__ skip) {
  __shared__ float red[8];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  s = block_sum<256>(s, red);
  const float norm = gscale * sqrtf(s);
  const bool skipped = skip != nullptr && *skip != 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    norm_out[0] = norm;
    if (!isfinite(norm)) flag[0] |= 1;
    if (skipped) flag[0] |= 2;
  }
  if (!isfinite(norm) || skipped) return;
  const float scale = gscale * (max_norm > 0.f ? max_norm / fmaxf(norm, max_norm) : 1.0f);
  const long n4 = n / 4;
  float4* w4 = reinterpret_cast<float4*>(w);
  float4* a4 = reinterpret_cast<float4*>(acc);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 gg = g4[i], aa = a4[i], ww = w4[i];
    gg.x *= scale; gg.y *= scale; gg.z *= scale; gg.w *= scale;
    aa.x += gg.x * gg.x; aa.y += gg.y * gg.y; aa.z += gg.z * gg.z; aa.w += gg.w * gg.w;
    ww.x -= lr * gg.x * rsqrtf(aa.x); ww.y -= lr * gg.y * rsqrtf(aa.y);
    ww.z -= lr * gg.z * rsqrtf(aa.z); ww.w -= lr * gg.w * rsqrtf(aa.w);
    a4[i] = aa; w4[i] = ww;
  }
  for (long i = n4 * 4 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float gg = g[i] * scale;
    const float aa = acc[i] + gg * gg;
    acc[i] = aa;
    w[i] -= lr * gg * rsqrtf(aa);
  }
}

void launch_clip_adagrad(float* w, float* acc, const float* g, long n, float* part, float lr, float max_norm,
                         float gscale, float* norm_out, int* flag, const int* skip, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(OPT_BLOCKS), dim3(256), 0, st, g, n, part);
  hipLaunchKernelGGL(adagrad_kernel, dim3(OPT_BLOCKS), dim3(256), 0, st, w, acc, g, n, part, OPT_BLOCKS, lr, max_norm,
                     gscale, norm_out, flag, skip);
}
int opt_nparts() { return OPT_BLOCKS; }
