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
    const int len = (int)DCHECK_IDX(lens[b], 0, T + 1, CHK_LOSS_LEN);
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
    const int len = (int)DCHECK_IDX(lens[b], 0, T + 1, CHK_LOSS_LEN);
    const float coef = g != 0.f ? -g * (1.0f - pg) * invP : 0.f;
    const int* er = ext + (size_t)b * T;
    float* dar = dA + (size_t)n * T;
    for (int i = tid; i < T; i += 256) dar[i] = (i < len && er[i] == w) ? coef : 0.f;
  }
}

// ---------------------------------------------------------------------------------------
// bf16 logits (bias already added by the GEMM epilogue), one read: each thread keeps its
// CH x 8 logits of the row in registers (V <= CH * 2048), so the row is read once for the
// log-sum-exp and the gold/copy gathers, and dz is written IN PLACE over the logits
// (dlogits may alias logits).  Traffic per row: 2V bytes in + 2V bytes out, versus 8V in
// + 2V out for the fp32 two-pass kernel above.
template <int CH>
__global__ __launch_bounds__(256) void ptr_loss_bf16_kernel(
    const bf16* logits, const int* __restrict__ target, const float* __restrict__ rowg,
    const float* __restrict__ pgen, const float* __restrict__ attn, const int* __restrict__ ext,
    const int* __restrict__ lens, float* __restrict__ loss_row, bf16* dlogits,
    float* __restrict__ dpre, float* __restrict__ dA, int N, int B, int T, int V) {
  __shared__ float red[8];
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const int b = n % B;
  const bf16* z = logits + (size_t)n * V;
  const float g = rowg[n];
  const int w = target[n];
  const int V8 = V & ~7;
  bf16x8 x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int k = (c * 256 + tid) * 8;
    if (k < V8) {
      x[c] = ld8(z + k);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[c][j] = k + j < V ? z[k + j] : f2bf(-INFINITY);
    }
  }
  const float zw = w < V ? bf2f(z[w]) : 0.f;  // read before any in-place write (syncs below)
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, bf2f(x[c][j]));
  const float M = block_max<256>(m, red);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += fexp(bf2f(x[c][j]) - M);
  const float lse = M + __logf(block_sum<256>(s, red));
  float cm = 0.f;
  const float pg = pgen ? pgen[n] : 1.0f;
  if (pgen) {
    const int len = (int)DCHECK_IDX(lens[b], 0, T + 1, CHK_LOSS_LEN);
    const float* ar = attn + (size_t)n * T;
    const int* er = ext + (size_t)b * T;
    for (int i = tid; i < len; i += 256) cm += er[i] == w ? ar[i] : 0.f;
    cm = block_sum<256>(cm, red);
  }
  const float pv = w < V ? fexp(zw - lse) : 0.f;
  const float P = pg * pv + (1.0f - pg) * cm;
  if (tid == 0) loss_row[n] = g != 0.f ? -__logf(P) : 0.f;
  if (!dlogits) return;
  const float invP = 1.0f / P;
  const float alpha = g != 0.f ? g * pg * pv * invP : 0.f;
  bf16* dz = dlogits + (size_t)n * V;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int k = (c * 256 + tid) * 8;
    if (k >= V) continue;
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(alpha * fexp(bf2f(x[c][j]) - lse) - (k + j == w ? alpha : 0.f));
    if (k < V8) {
      *reinterpret_cast<bf16x8*>(dz + k) = o;
    } else {
      for (int j = 0; j < 8 && k + j < V; ++j) dz[k + j] = o[j];
    }
  }
  if (pgen) {
    if (tid == 0) dpre[n] = g != 0.f ? -g * (pv - cm) * invP * pg * (1.0f - pg) : 0.f;
    const int len = (int)DCHECK_IDX(lens[b], 0, T + 1, CHK_LOSS_LEN);
    const float coef = g != 0.f ? -g * (1.0f - pg) * invP : 0.f;
    const int* er = ext + (size_t)b * T;
    float* dar = dA + (size_t)n * T;
    for (int i = tid; i < T; i += 256) dar[i] = (i < len && er[i] == w) ? coef : 0.f;
  }
}

int ptr_loss_bf16_max_vocab() { return 32 * 2048; }

void launch_ptr_loss_bf16(const bf16* logits, const int* target, const float* rowg, const float* pgen,
                          const float* attn, const int* ext, const int* lens, float* loss_row, bf16* dlogits,
                          float* dpre, float* dA, int N, int B, int T, int V, hipStream_t st) {
#define PLB(C) hipLaunchKernelGGL(ptr_loss_bf16_kernel<C>, dim3(N), dim3(256), 0, st, logits, target, rowg, pgen, attn, \
                                   ext, lens, loss_row, dlogits, dpre, dA, N, B, T, V)
  const int ch = (V + 2047) / 2048;
  if (ch <= 4) PLB(4);
  else if (ch <= 8) PLB(8);
  else if (ch <= 16) PLB(16);
  else if (ch <= 25) PLB(25);
  else PLB(32);
#undef PLB
}

void launch_ptr_loss(const float* logits, const float* bias, const int* target, const float* rowg, const float* pgen, const float* attn,
                     const int* ext, const int* lens, float* loss_row, bf16* dlogits, float* dpre, float* dA, int N,
                     int B, int T, int V, hipStream_t st) {
  hipLaunchKernelGGL(ptr_loss_kernel, dim3(N), dim3(256), 0, st, logits, bias, target, rowg, pgen, attn, ext, lens, loss_row,
                     dlogits, dpre, dA, N, B, T, V);
}
