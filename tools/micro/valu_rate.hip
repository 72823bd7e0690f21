// VALU throughput probe on gfx950: wave-instructions per SIMD-cycle for v_exp_f32,
// v_rcp_f32, v_pk_fma_f32, v_fma_f32 and two tanh formulations (exp2 + rcp r-form vs a
// packed rational), every CU busy (2048 blocks x 256 threads, 8 independent chains per lane).
// Prints ns per element-op chip-wide and the implied cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
#define ITERS 4096
#define CH 8

__global__ __launch_bounds__(256) void k_exp(float* out, float seed) {
  float x[CH];
  for (int c = 0; c < CH; ++c) x[c] = seed * (threadIdx.x + c);
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = __builtin_amdgcn_exp2f(x[c]);
  float s = 0; for (int c = 0; c < CH; ++c) s += x[c];
  if (s == 12345.f) out[0] = s;
}
__global__ __launch_bounds__(256) void k_rcp(float* out, float seed) {
  float x[CH];
  for (int c = 0; c < CH; ++c) x[c] = seed * (threadIdx.x + c) + 1.0f;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = __builtin_amdgcn_rcpf(x[c]);
  float s = 0; for (int c = 0; c < CH; ++c) s += x[c];
  if (s == 12345.f) out[0] = s;
}
__global__ __launch_bounds__(256) void k_fma(float* out, float seed) {
  float x[CH];
  for (int c = 0; c < CH; ++c) x[c] = seed * (threadIdx.x + c);
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = fmaf(x[c], 0.999f, 0.001f);
  float s = 0; for (int c = 0; c < CH; ++c) s += x[c];
  if (s == 12345.f) out[0] = s;
}
__global__ __launch_bounds__(256) void k_pkfma(float* out, float seed) {
  f2 x[CH];
  for (int c = 0; c < CH; ++c) x[c] = f2{seed * (threadIdx.x + c), seed * c};
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = __builtin_elementwise_fma(x[c], f2{0.999f, 0.999f}, f2{0.001f, 0.001f});
  float s = 0; for (int c = 0; c < CH; ++c) s += x[c].x + x[c].y;
  if (s == 12345.f) out[0] = s;
}
// r-form: r = 1 / (1 + 2^y), q = r - r^2: 2 transcendentals + 2 FMA per element
__global__ __launch_bounds__(256) void k_rform(float* out, float seed) {
  float x[CH], acc[CH];
  for (int c = 0; c < CH; ++c) { x[c] = seed * (threadIdx.x + c); acc[c] = 0; }
  for (int i = 0; i < ITERS / 4; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const float r = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(x[c]) + 1.0f);
      acc[c] = fmaf(r, -r, r) + acc[c];
      x[c] += 0.01f;
    }
  float s = 0; for (int c = 0; c < CH; ++c) s += acc[c];
  if (s == 12345.f) out[0] = s;
}
// packed rational tanh (clamped), one rcp per element, pk_fma polynomial
__global__ __launch_bounds__(256) void k_prat(float* out, float seed) {
  f2 x[CH / 2], acc[CH / 2];
  for (int c = 0; c < CH / 2; ++c) { x[c] = f2{seed * (threadIdx.x + c), seed * c}; acc[c] = f2{0, 0}; }
  for (int i = 0; i < ITERS / 4; ++i)
#pragma unroll
    for (int c = 0; c < CH / 2; ++c) {
      f2 u = __builtin_elementwise_min(__builtin_elementwise_max(x[c], f2{-7.9f, -7.9f}), f2{7.9f, 7.9f});
      f2 u2 = u * u;
      f2 p = __builtin_elementwise_fma(u2, f2{-2.76e-16f, -2.76e-16f}, f2{2.0e-13f, 2.0e-13f});
      p = __builtin_elementwise_fma(u2, p, f2{-8.6e-11f, -8.6e-11f});
      p = __builtin_elementwise_fma(u2, p, f2{5.1e-8f, 5.1e-8f});
      p = __builtin_elementwise_fma(u2, p, f2{1.4e-5f, 1.4e-5f});
      p = __builtin_elementwise_fma(u2, p, f2{4.9e-3f, 4.9e-3f});
      p = p * u;
      f2 q = __builtin_elementwise_fma(u2, f2{1.2e-6f, 1.2e-6f}, f2{2.3e-4f, 2.3e-4f});
      q = __builtin_elementwise_fma(u2, q, f2{2.2e-3f, 2.2e-3f});
      q = __builtin_elementwise_fma(u2, q, f2{4.9e-3f, 4.9e-3f});
      f2 t = p * f2{__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
      acc[c] = __builtin_elementwise_fma(t, -t, acc[c] + f2{1.f, 1.f});
      x[c] += f2{0.01f, 0.01f};
    }
  float s = 0; for (int c = 0; c < CH / 2; ++c) s += acc[c].x + acc[c].y;
  if (s == 12345.f) out[0] = s;
}

template <typename K>
float timeit(K k, float* out, int blocks) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0.001f);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0.001f);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  float* out; hipMalloc(&out, 4);
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 8;  // 8 x 4 waves per CU = 8 waves/SIMD
  const double waves = blocks * 4.0, simds = cus * 4.0;
  struct { const char* n; float ms; double per; } r[] = {
    {"v_exp_f32", timeit(k_exp, out, blocks), (double)ITERS * CH},
    {"v_rcp_f32", timeit(k_rcp, out, blocks), (double)ITERS * CH},
    {"v_fma_f32", timeit(k_fma, out, blocks), (double)ITERS * CH},
    {"v_pk_fma_f32", timeit(k_pkfma, out, blocks), (double)ITERS * CH},
    {"rform_elem(exp+rcp+2fma)", timeit(k_rform, out, blocks), (double)ITERS / 4 * CH},
    {"packed_rational_elem", timeit(k_prat, out, blocks), (double)ITERS / 4 * CH},
  };
  for (auto& x : r) {
    const double winstr = waves * x.per;  // wave-level op count (per lane-op: x 64)
    const double ns_cyc = 1.0 / 2.1;      // assume ~2.1 GHz under load
    const double cyc_per = (x.ms * 1e6 / ns_cyc) * simds / winstr;
    printf("{\"op\": \"%s\", \"ms\": %.3f, \"elem_ops_per_ns\": %.1f, \"simd_cycles_per_wave_op_at_2.1GHz\": %.2f}\n", x.n, x.ms,
           winstr * 64 / (x.ms * 1e6), cyc_per);
  }
  return 0;
}
