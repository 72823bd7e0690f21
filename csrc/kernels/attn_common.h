// Shared device helpers of the attention kernels (attention.hip: multi-block per row;
// attention_row.hip: one workgroup per row).
#pragma once
#include "common.h"

__device__ __forceinline__ float lo_bf(uint32_t r) { return __uint_as_float(r << 16); }
__device__ __forceinline__ float hi_bf(uint32_t r) { return __uint_as_float(r & 0xffff0000u); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
// tanh through r = 1 / (1 + 2^(y)), y = 2u*log2(e):  tanh(u) = 1 - 2r,  sech^2(u) = 4 r (1 - r).
// Scores become  e = sum_k v_k - 2 sum_k v_k r_k  (no clamp needed: 2^y -> inf gives r = 0,
// 2^y -> 0 gives r = 1), i.e. per element 2 packed FMAs + exp + add + rcp + packed FMA.
#define K2LOG2E 2.8853900817779268f
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 splat2(float x) { return f32x2{x, x}; }
__device__ __forceinline__ f32x2 rsig2(f32x2 y) {
  const f32x2 ex = f32x2{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)} + 1.0f;
  return f32x2{__builtin_amdgcn_rcpf(ex.x), __builtin_amdgcn_rcpf(ex.y)};
}
__device__ __forceinline__ f32x2 bf2pair(uint32_t r) { return f32x2{__uint_as_float(r << 16), __uint_as_float(r & 0xffff0000u)}; }
// The attention features F = enc_out . W_h are STORED pre-scaled by 2 log2(e) (the engine's
// F GEMM runs on W_h * K2LOG2E, pack.hip), so a score argument is y = F + t with t = 2 log2(e)
// (s + w cov) -- per feature pair two v_dot2_f32_bf16 against (1, 0) / (0, 1): the bf16 -> f32
// unpack and the add in ONE op per element instead of shift / and + packed FMA (12.4 vs 16.8
// cycles per pair, tools/micro/dot2_probe.cpp; the products are exact, one rounding of F + t).
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// The (1, 0) / (0, 1) selectors live in SGPRs made opaque once per kernel (dot2_sel()): left as
// constants, the compiler encodes (1, 0) as the inline constant 1.0, which the hardware does not
// expand to a bf16 1.0 in the low half (test_gpu_attention_ops failed with it).
struct Dot2Sel {
  uint32_t lo, hi;
};
__device__ __forceinline__ Dot2Sel dot2_sel() {
  uint32_t lo = 0x00003f80u, hi = 0x3f800000u;
  asm volatile("" : "+s"(lo), "+s"(hi));
  return Dot2Sel{lo, hi};
}
__device__ __forceinline__ f32x2 fadd_bf2(uint32_t r, f32x2 t, Dot2Sel sel) {
  const bf16x2_t x = __builtin_bit_cast(bf16x2_t, r);
  return f32x2{__builtin_amdgcn_fdot2_f32_bf16(x, __builtin_bit_cast(bf16x2_t, sel.lo), t.x, false),
               __builtin_amdgcn_fdot2_f32_bf16(x, __builtin_bit_cast(bf16x2_t, sel.hi), t.y, false)};
}

__device__ __forceinline__ float rdlane(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}

__device__ __forceinline__ float bfly8(const float (&x)[8], int b5, int b4, int b3) {
  float h4[4], h2[2], h1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float send = b5 ? x[i] : x[i + 4];
    const float keep = b5 ? x[i + 4] : x[i];
    h4[i] = keep + xor32_f(send);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float send = b4 ? h4[i] : h4[i + 2];
    const float keep = b4 ? h4[i + 2] : h4[i];
    h2[i] = keep + xor16_f(send);
  }
  {
    const float send = b3 ? h2[0] : h2[1];
    const float keep = b3 ? h2[1] : h2[0];
    h1 = keep + dpp_f<DPP_ROR8>(send);
  }
  h1 = dpp_sum8(h1);
  return h1;  // total of element q = 4*b5 + 2*b4 + b3, in all 8 lanes of that group
}

__device__ __forceinline__ float bfly4(const float (&x)[4], int b5, int b4) {
  float h2[2], h1;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float send = b5 ? x[i] : x[i + 2];
    const float keep = b5 ? x[i + 2] : x[i];
    h2[i] = keep + xor32_f(send);
  }
  {
    const float send = b4 ? h2[0] : h2[1];
    const float keep = b4 ? h2[1] : h2[0];
    h1 = keep + xor16_f(send);
  }
  h1 = dpp_sum16(h1);
  return h1;  // total of element q = 2*b5 + b4, in all 16 lanes of that group
}

