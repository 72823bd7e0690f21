// Issue cost of the bf16 -> f32 "unpack + add" forms used by the attention score loops
// (one MI355X, hipEvent timing, 1024 workgroups x 256 threads, 8 independent chains per lane):
//   unpack : v_lshlrev + v_and + v_pk_add_f32       (y = bf2f(f) + t, two features)
//   dot2   : 2 x v_dot2_f32_bf16 with B = (1, 0) / (0, 1)
//   pkfma  : v_pk_fma_f32 alone (reference rate)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
constexpr int NCH = 8, IT = 4096;

__global__ __launch_bounds__(256) void k_unpack(const unsigned* in, float* out) {
  unsigned f[NCH];
  f32x2 t[NCH];
  for (int c = 0; c < NCH; ++c) { f[c] = in[threadIdx.x * NCH + c]; t[c] = f32x2{0.f, 0.f}; }
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const f32x2 x = f32x2{__uint_as_float(f[c] << 16), __uint_as_float(f[c] & 0xffff0000u)};
      t[c] = x + t[c] * 0.5f;  // pk_fma
      f[c] += 0x00010001u;
    }
  float s = 0.f;
  for (int c = 0; c < NCH; ++c) s += t[c].x + t[c].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_dot2(const unsigned* in, float* out) {
  unsigned f[NCH];
  f32x2 t[NCH];
  const bf16x2 lo = __builtin_bit_cast(bf16x2, 0x00003f80u), hi = __builtin_bit_cast(bf16x2, 0x3f800000u);
  for (int c = 0; c < NCH; ++c) { f[c] = in[threadIdx.x * NCH + c]; t[c] = f32x2{0.f, 0.f}; }
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const bf16x2 x = __builtin_bit_cast(bf16x2, f[c]);
      t[c].x = __builtin_amdgcn_fdot2_f32_bf16(x, lo, t[c].x * 0.5f, false);
      t[c].y = __builtin_amdgcn_fdot2_f32_bf16(x, hi, t[c].y * 0.5f, false);
      f[c] += 0x00010001u;
    }
  float s = 0.f;
  for (int c = 0; c < NCH; ++c) s += t[c].x + t[c].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_dot2n(const unsigned* in, float* out) {
  // dot2 with the accumulate operand t directly (no scaling): y = f + t
  unsigned f[NCH];
  f32x2 t[NCH];
  const bf16x2 lo = __builtin_bit_cast(bf16x2, 0x00003f80u), hi = __builtin_bit_cast(bf16x2, 0x3f800000u);
  for (int c = 0; c < NCH; ++c) { f[c] = in[threadIdx.x * NCH + c]; t[c] = f32x2{0.f, 0.f}; }
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const bf16x2 x = __builtin_bit_cast(bf16x2, f[c]);
      t[c].x = __builtin_amdgcn_fdot2_f32_bf16(x, lo, t[c].x, false);
      t[c].y = __builtin_amdgcn_fdot2_f32_bf16(x, hi, t[c].y, false);
      f[c] += 0x00010001u;
    }
  float s = 0.f;
  for (int c = 0; c < NCH; ++c) s += t[c].x + t[c].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_unpackn(const unsigned* in, float* out) {
  unsigned f[NCH];
  f32x2 t[NCH];
  for (int c = 0; c < NCH; ++c) { f[c] = in[threadIdx.x * NCH + c]; t[c] = f32x2{0.f, 0.f}; }
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const f32x2 x = f32x2{__uint_as_float(f[c] << 16), __uint_as_float(f[c] & 0xffff0000u)};
      t[c] = x + t[c];  // pk_add
      f[c] += 0x00010001u;
    }
  float s = 0.f;
  for (int c = 0; c < NCH; ++c) s += t[c].x + t[c].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  unsigned* in; float* out;
  hipMalloc(&in, 256 * NCH * 4); hipMalloc(&out, 1024 * 256 * 4);
  hipMemset(in, 0x3f, 256 * NCH * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](const char* name, void (*k)(const unsigned*, float*), int ops) {
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k, dim3(1024), dim3(256), 0, 0, in, out);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    // cycles per wave instruction per SIMD at 2.4 GHz: 1024 WG x 4 waves / (256 CU x 4 SIMD) = 4 waves per SIMD
    const double wave_ins = 4.0 * IT * NCH * ops;
    std::printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"cyc_per_pair_est\": %.2f}\n", name, best,
                best * 1e-3 * 2.4e9 / (4.0 * IT * NCH));
    (void)wave_ins;
  };
  run("unpack+pkfma", k_unpack, 1);
  run("unpack+pkadd", k_unpackn, 1);
  run("dot2x2(scaled acc)", k_dot2, 1);
  run("dot2x2", k_dot2n, 1);
  return 0;
}
