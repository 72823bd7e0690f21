// Pointer-generator mixture loss, fused forward + backward (SURVEY K15-K18, K21;
// reference model.py:146-183, 249-268, 446-460).
//
// For decoder row n = (t, b) with gold extended-vocab id w:
//   P = p_gen * softmax(z)[w] * [w < V] + (1 - p_gen) * sum_i a_i [ext_i == w]
//   loss_n = -log P
// The [N, V+O] final distribution is never materialised: one block per row reduces
// the logits row to (max, sumexp) and gathers the copy mass, then writes
//   dz_k   = g * p_gen * pv_w / P * (softmax_k - [k == w])       (bf16, feeds 2 GEMMs)
//   dpre   = -g (pv_w - copy_w) / P * p_gen (1 - p_gen)          (p_gen pre-sigmoid)
//   dA_i   = -g (1 - p_gen) [ext_i == w] / P
// where g is the row's weight in the mean-over-examples loss (mask / (dec_len * B)).
// Baseline mode (pointer_gen=False, sequence_loss) is the same kernel with p_gen = 1.
// The output-projection bias is added on the fly (z = logits + bias), so the GEMM output
// is never re-written just to add it.
#include "common.h"

__global__ __launch_bounds__(256) void ptr_loss_kernel(
    const float* __restrict__ logits, const float* __restrict__ bias, const int* __restrict__ target, const float* __restrict__ rowg,
    const float* __restrict__ pgen, const float* __restrict__ attn, const int* __restrict__ ext,
    const int* __restrict__ lens, float* __restrict__ loss_row, bf16* __restrict__ dlogits,
    float* __restrict__ dpre, float* __restrict__ dA, int N, int B, int T, int V) {
  __shared__ float red[8];
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const int b = n % B;
  const float* z = logits + (size_t)n * V;
  const float g = rowg[n];
  const int w = target[n];
  // pass 1: row max and sum of exp
  float m = -INFINITY, s = 0.f;
  const int V4 = (V % 4 == 0) ? V : 0;  // float4 path needs 16-B aligned rows
  for (int k = tid * 4; k < V4; k += 1024) {
    float4 x = *reinterpret_cast<const float4*>(z + k);
    const float4 bb = *reinterpret_cast<const float4*>(bias + k);
    x.x += bb.x; x.y += bb.y; x.z += bb.z; x.w += bb.w;
    const float mx = fmaxf(fmaxf(x.x, x.y), fmaxf(x.z, x.w));
    if (mx > m) { s *= fexp(m - mx); m = mx; }
    s += fexp(x.x - m) + fexp(x.y - m) + fexp(x.z - m) + fexp(x.w - m);
  }
  for (int k = V4 + tid; k < V; k += 256) {
    const float x = z[k] + bias[k];
    if (x > m) { s *= fexp(m - x); m = x; }
    s += fexp(x - m);
  }
  const float M = block_max<256>(m, red);
  const float S = block_sum<256>(m == -INFINITY ? 0.f : s * fexp(m - M), red);
  const float lse = M + __logf(S);
  // copy mass of the gold id
  float c = 0.f;
  const float pg = pgen ? pgen[n] : 1.0f;
  if (pgen) {
    const int len = lens[b];
    const float* ar = attn + (size_t)n * T;
    const int* er = ext + (size_t)b * T;
    for (int i = tid; i < len; i += 256) c += er[i] == w ? ar[i] : 0.f;
    c = block_sum<256>(c, red);
  }
  const float pv = w < V ? fexp(z[w] + bias[w] - lse) : 0.f;
  const float P = pg * pv + (1.0f - pg) * c;
  if (tid == 0) loss_row[n] = g != 0.f ? -__logf(P) : 0.f;
  if (!dlogits) return;
  const float invP = 1.0f / P;
  const float alpha = g != 0.f ? g * pg * pv * invP : 0.f;
  bf16* dz = dlogits + (size_t)n * V;
  const int V8 = (V % 8 == 0) ? V : 0;
  for (int k = tid * 8; k < V8; k += 2048) {
    const float4 x0 = *reinterpret_cast<const float4*>(z + k);
    const float4 x1 = *reinterpret_cast<const float4*>(z + k + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(bias + k);
    const float4 b1 = *reinterpret_cast<const float4*>(bias + k + 4);
    const float xs[8] = {x0.x + b0.x, x0.y + b0.y, x0.z + b0.z, x0.w + b0.w,
                         x1.x + b1.x, x1.y + b1.y, x1.z + b1.z, x1.w + b1.w};
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(alpha * fexp(xs[j] - lse) - (k + j == w ? alpha : 0.f));
    *reinterpret_cast<bf16x8*>(dz + k) = o;
  }
  for (int k = V8 + tid; k < V; k += 256) {
    float d = alpha * fexp(z[k] + bias[k] - lse);
    if (k == w) d -= alpha;
    dz[k] = f2bf(d);
  }
  if (pgen) {
    if (tid == 0) dpre[n] = g != 0.f ? -g * (pv - c) * invP * pg * (1.0f - pg) : 0.f;
    const int len = lens[b];
    const float coef = g != 0.f ? -g * (1.0f - pg) * invP : 0.f;
    const int* er = ext + (size_t)b * T;
    float* dar = dA + (size_t)n * T;
    for (int i = tid; i < T; i += 256) dar[i] = (i < len && er[i] == w) ? coef : 0.f;
  }
}

void launch_ptr_loss(const float* logits, const float* bias, const int* target, const float* rowg, const float* pgen, const float* attn,
                     const int* ext, const int* lens, float* loss_row, bf16* dlogits, float* dpre, float* dA, int N,
                     int B, int T, int V, hipStream_t st) {
  hipLaunchKernelGGL(ptr_loss_kernel, dim3(N), dim3(256), 0, st, logits, bias, target, rowg, pgen, attn, ext, lens, loss_row,
                     dlogits, dpre, dA, N, B, T, V);
}
