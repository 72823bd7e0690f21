// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Conventions used by every kernel in this directory:
//  * wave = 64 lanes; blocks are multiples of 64 threads.
//  * GEMM-shaped work uses v_mfma_f32_16x16x32_bf16 with fp32 accumulation.
//    Operand maps (cdna_hip_programming.md s3): lane l holds
//      A[row = l&15][k = 8*(l>>4) + j], B[k = 8*(l>>4) + j][col = l&15], j=0..7
//    and the accumulator holds C[row = (l>>4)*4 + r][col = l&15], r=0..3.
//  * Weight operands are stored "Bt" = [N][K] with K contiguous, so both A and B
//    fragments are one 16-byte load per lane straight from L2 (M <= a few hundred,
//    the operands are L2-resident and re-read every step of a recurrence).
//  * Recurrence GEMMs are latency-bound (a few MFLOP per step): each block's 4 waves
//    split K, every wave issues ALL of its fragment loads before its first MFMA (one
//    L2 round trip instead of K/32 dependent ones), and the 4 partial tiles are summed
//    through LDS.  See kslice_mma / ksplit_reduce.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dcheck.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define WAVE 64

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ f32x4 mfma16(const bf16x8 a, const bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// 8 fp32 -> one bf16x8 fragment (A operand taken from an fp32 activation).
__device__ __forceinline__ bf16x8 ld8f(const float* p) {
  const float4 x = *reinterpret_cast<const float4*>(p);
  const float4 y = *reinterpret_cast<const float4*>(p + 4);
  bf16x8 r;
  r[0] = f2bf(x.x); r[1] = f2bf(x.y); r[2] = f2bf(x.z); r[3] = f2bf(x.w);
  r[4] = f2bf(y.x); r[5] = f2bf(y.y); r[6] = f2bf(y.z); r[7] = f2bf(y.w);
  return r;
}

// the same for the sum of two fp32 partials p + q
__device__ __forceinline__ bf16x8 ld8f2(const float* p, const float* q) {
  const float4 x = *reinterpret_cast<const float4*>(p), y = *reinterpret_cast<const float4*>(p + 4);
  const float4 u = *reinterpret_cast<const float4*>(q), w = *reinterpret_cast<const float4*>(q + 4);
  bf16x8 r;
  r[0] = f2bf(x.x + u.x); r[1] = f2bf(x.y + u.y); r[2] = f2bf(x.z + u.z); r[3] = f2bf(x.w + u.w);
  r[4] = f2bf(y.x + w.x); r[5] = f2bf(y.y + w.y); r[6] = f2bf(y.z + w.z); r[7] = f2bf(y.w + w.w);
  return r;
}

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.0f;
  return z;
}

// Fast activations (fp32).  exp via v_exp_f32 (2^x).
__device__ __forceinline__ float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float fsigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + fexp(-x)); }
__device__ __forceinline__ float ftanh(float x) {
  // tanh(x) = 1 - 2/(exp(2x)+1); clamp keeps exp finite, exact to fp32 rounding for |x|>=9.
  x = fminf(fmaxf(x, -15.0f), 15.0f);
  float e = fexp(2.0f * x);
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
}

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

// Block-wide reductions for blockDim.x == NT (multiple of 64); scratch >= NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += scratch[i];
  return r;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* scratch) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, scratch[i]);
  return r;
}

// One 16x16 output tile, K loop of 32: acc += A[rows][k] * Bt[cols][k].
// a_row / b_row already point at this lane's row (A row l&15 / Bt row l&15) and k offset 8*(l>>4).
__device__ __forceinline__ f32x4 mfma_k(const bf16* a_row, const bf16* b_row, int K, f32x4 acc) {
  for (int k = 0; k < K; k += 32) acc = mfma16(ld8(a_row + k), ld8(b_row + k), acc);
  return acc;
}

// K-slice of NB tiles that share the A fragment: acc[j] += A[:, k0:k1] . Bt_j[:, k0:k1].
// Loads are issued in batches of KB k-steps before the MFMAs of the batch (one L2 round trip
// per batch); a batch step past k1 loads a valid (clamped) address and is zeroed, so the code
// is branch-free.  a(k) / b(j, k): pointers for this lane at absolute k (must include the
// 8*(l>>4) offset).
template <int NB, int KB = 4, typename FA, typename FB>
__device__ __forceinline__ void kslice_mma(FA a, FB b, int k0, int k1, f32x4 (&acc)[NB]) {
  for (int k = k0; k < k1; k += 32 * KB) {
    bf16x8 af[KB];
    bf16x8 bfr[NB][KB];
#pragma unroll
    for (int i = 0; i < KB; ++i) {
      const int kk = k + 32 * i;
      const int kc = kk < k1 ? kk : k0;
      af[i] = a(kc);
#pragma unroll
      for (int j = 0; j < NB; ++j) bfr[j][i] = b(j, kc);
    }
#pragma unroll
    for (int i = 0; i < KB; ++i) {
      if (k + 32 * i < k1) {
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[j] = mfma16(af[i], bfr[j][i], acc[j]);
      }
    }
  }
}

// Sum NB tiles across the 4 waves of a 256-thread block.  red: >= 4*NB*256 floats of LDS.
// Afterwards wave w owns accumulator register r = w of every tile: lane l holds the
// full sum for C[row = (l>>4)*4 + w][col = l&15] of tile j in out[j].
template <int NB>
__device__ __forceinline__ void ksplit_reduce(const f32x4 (&acc)[NB], float* red, float (&out)[NB]) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[((w * NB + j) * 4 + r) * 64 + l] = acc[j][r];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    float s = 0.f;
#pragma unroll
    for (int src = 0; src < 4; ++src) s += red[((src * NB + j) * 4 + w) * 64 + l];
    out[j] = s;
  }
}

// Cross-lane moves inside a 16-lane DPP row: a VALU operand modifier, no LDS round trip
// (a __shfl_xor is a ds_bpermute: ~100+ cycles of latency per dependent step).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xf, 0xf, false));
}
#define DPP_MIRROR 0x140       // l <-> 15 - l  (flips bits 0-3 of the row lane)
#define DPP_HALF_MIRROR 0x141  // l <-> 7 - l within each half (flips bits 0-2)
#define DPP_XOR2 0x4e          // quad_perm [2,3,0,1]
#define DPP_XOR1 0xb1          // quad_perm [1,0,3,2]
// all-reduce over the 8 lanes l, l^1, .., l^7 / the 16 lanes of the DPP row (partners xor 1,
// xor 2, then the mirrors: lanes of a quad already agree, so 7 - l acts as l ^ 4)
__device__ __forceinline__ float dpp_sum8(float x) {
  x += dpp_f<DPP_XOR1>(x);
  x += dpp_f<DPP_XOR2>(x);
  return x + dpp_f<DPP_HALF_MIRROR>(x);
}
__device__ __forceinline__ float dpp_sum16(float x) {
  x = dpp_sum8(x);
  return x + dpp_f<DPP_MIRROR>(x);
}
__device__ __forceinline__ float dpp_max16(float x) {
  x = fmaxf(x, dpp_f<DPP_XOR1>(x));
  x = fmaxf(x, dpp_f<DPP_XOR2>(x));
  x = fmaxf(x, dpp_f<DPP_HALF_MIRROR>(x));
  return fmaxf(x, dpp_f<DPP_MIRROR>(x));
}

#define DPP_ROR8 0x128         // row_ror:8 -- within a 16-lane row this is l ^ 8
// Value of lane l ^ 32 / l ^ 16 through the gfx950 v_permlane{32,16}_swap (VALU, no LDS).
// With both operands = v the swap returns {lower half, upper half} (rows {0,2} / {1,3}).
__device__ __forceinline__ float xor32_f(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 32) ? p[0] : p[1]);
}
__device__ __forceinline__ float xor16_f(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 16) ? p[0] : p[1]);
}
// v + v(l ^ 32), v + v(l ^ 16), max likewise (the two halves are summed in the same order on
// both sides, so every lane gets the bit-identical result)
// v_max3_f32 / v_max_f32 without the NaN-quieting canonicalisations fmaxf gets in IEEE mode
// (for finite or -inf operands: 8 instructions instead of ~29 for 16 values)
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmax2(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float sum_x32(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float sum_x16(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float max_x32(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}
__device__ __forceinline__ float max_x16(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}

#define HIP_LAUNCH_CHECK() (void)0
