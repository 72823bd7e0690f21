// Measurement and test probes (not on any training / decode path):
//
//   cu_hold        one workgroup per CU holding the CU's whole LDS, spinning on the constant
//                  100 MHz clock for a bounded time -- stands in for RCCL collective kernels
//                  (one workgroup per channel) that hold CUs while the persistent encoder LSTM
//                  launches (train/trainer.py co-residency guard, tests/test_gpu_lstm.py).
//   tanh_eval      the attention kernels' tanh / sech^2 (attn_common.h rsig2: r = 1/(1 + 2^(2u log2 e)),
//                  tanh = 1 - 2r, sech^2 = 4 r (1 - r)) and, for comparison, a clamped odd/even
//                  rational tanh with one reciprocal (sech^2 = 1 - t^2), element by element.
//   tanh_tput      issue-rate of the two forms inside a score-like reduction e = sum_k v_k tanh(u_k)
//                  over register-resident data (no memory traffic in the loop): the cost per
//                  element that bounds the attention kernels' VALU work.
#include "attn_common.h"

// ------------------------------------------------------------------ CU hold
// Every workgroup requests `lds_bytes` of dynamic LDS (the whole CU's, 160 KB on gfx950), so no
// other workgroup that needs LDS can share its CU; the first wave spins with s_sleep (no issue
// pressure) until `ticks` of the constant clock have passed, then the workgroup exits -- every
// wave reaches the exit, so the grid drains whatever else runs.  times[2 i] / [2 i + 1]: the
// workgroup's start / end clock, for checking that the grid was resident all at once.
__global__ __launch_bounds__(64) void cu_hold_kernel(unsigned long long ticks, long long* times) {
  extern __shared__ float lds[];
  const unsigned long long t0 = wall_clock64();
  if (threadIdx.x == 0) lds[0] = 0.f;  // touch the allocation
  unsigned long long t = t0;
  while (t - t0 < ticks) {
    __builtin_amdgcn_s_sleep(64);
    t = wall_clock64();
  }
  if (threadIdx.x == 0) {
    times[2 * blockIdx.x] = (long long)t0;
    times[2 * blockIdx.x + 1] = (long long)t;
  }
}

int cu_hold_max_lds() {
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess) return 0;
  return v;
}

void launch_cu_hold(int grid, unsigned long long ticks, long long* times, int lds_bytes, hipStream_t st) {
  (void)hipFuncSetAttribute((const void*)cu_hold_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
  hipLaunchKernelGGL(cu_hold_kernel, dim3(grid), dim3(64), lds_bytes, st, ticks, times);
}

// ------------------------------------------------------------------ tanh forms
// Rational: tanh(u) ~= u P(u^2) / Q(u^2) on |u| <= 7.9053 (clamped outside), P degree 6, Q degree 3
// in u^2 (the float minimax fit of Eigen's ptanh_float): 1 mul + 9 FMAs + 2 muls + ONE rcp.
__device__ __forceinline__ f32x2 tanh_rat2(f32x2 u) {
  const float c = 7.90531110763549805f;
  u = f32x2{fminf(fmaxf(u.x, -c), c), fminf(fmaxf(u.y, -c), c)};
  const f32x2 z = u * u;
  f32x2 p = fma2(z, splat2(-2.76076847742355e-16f), splat2(2.00018790482477e-13f));
  p = fma2(z, p, splat2(-8.60467152213735e-11f));
  p = fma2(z, p, splat2(5.12229709037114e-08f));
  p = fma2(z, p, splat2(1.48572235717979e-05f));
  p = fma2(z, p, splat2(6.37261928875436e-04f));
  p = fma2(z, p, splat2(4.89352455891786e-03f));
  f32x2 q = fma2(z, splat2(1.19825839466702e-06f), splat2(1.18534705686654e-04f));
  q = fma2(z, q, splat2(2.26843463243900e-03f));
  q = fma2(z, q, splat2(4.89352518554385e-03f));
  return u * p * f32x2{__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
}

__global__ __launch_bounds__(256) void tanh_eval_kernel(const float* __restrict__ x, float* __restrict__ t,
                                                        float* __restrict__ s2, int n, int mode) {
  const int i = 2 * (blockIdx.x * 256 + threadIdx.x);
  if (i >= n) return;
  const f32x2 u = f32x2{x[i], i + 1 < n ? x[i + 1] : 0.f};
  f32x2 tv, sv;
  if (mode == 0) {
    const f32x2 r = rsig2(u * K2LOG2E);
    tv = fma2(splat2(-2.f), r, splat2(1.f));
    sv = 4.f * fma2(-r, r, r);
  } else {
    tv = tanh_rat2(u);
    sv = fma2(-tv, tv, splat2(1.f));
  }
  t[i] = tv.x;
  s2[i] = sv.x;
  if (i + 1 < n) {
    t[i + 1] = tv.y;
    s2[i + 1] = sv.y;
  }
}

// per thread 8 features (4 pairs) x `iters` positions of e = sum_k v_k tanh(x_k + c_i); the shift
// c_i differs per position so nothing is hoisted.  Mode 0 accumulates sum_k v_k r_k (the score is
// sum v - 2 sum v r, as in attn_fwd_row); mode 1 sum_k v_k tanh_rat(u_k).
template <int MODE>
__global__ __launch_bounds__(256) void tanh_tput_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                        int iters) {
  const int tid = blockIdx.x * 256 + threadIdx.x;
  f32x2 x[4], v[4], acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    x[j] = f32x2{in[(tid * 8 + 2 * j) & 1023], in[(tid * 8 + 2 * j + 1) & 1023]};
    v[j] = x[j] * 0.5f;
    acc[j] = splat2(0.f);
  }
  if (MODE == 0)
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = x[j] * K2LOG2E;
  for (int it = 0; it < iters; ++it) {
    const float c = (float)(it & 15) * 0.0625f - 0.5f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (MODE == 0) {
        const f32x2 r = rsig2(fma2(splat2(c), splat2(K2LOG2E), x[j]));
        acc[j] = fma2(v[j], r, acc[j]);
      } else {
        acc[j] = fma2(v[j], tanh_rat2(x[j] + c), acc[j]);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += acc[j].x + acc[j].y;
  out[tid] = s;
}

void launch_tanh_eval(const float* x, float* t, float* s2, int n, int mode, hipStream_t st) {
  hipLaunchKernelGGL(tanh_eval_kernel, dim3((n / 2 + 255) / 256 + 1), dim3(256), 0, st, x, t, s2, n, mode);
}

void launch_tanh_tput(const float* in, float* out, int threads, int iters, int mode, hipStream_t st) {
  if (mode == 0)
    hipLaunchKernelGGL(tanh_tput_kernel<0>, dim3(threads / 256), dim3(256), 0, st, in, out, iters);
  else
    hipLaunchKernelGGL(tanh_tput_kernel<1>, dim3(threads / 256), dim3(256), 0, st, in, out, iters);
}
