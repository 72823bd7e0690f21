// Embedding gradient (reference model.py:211-214 -- TF's sparse IndexedSlices
// gradient of embedding_lookup, densified): gemb[ids[n], :] += src[n, :] for the encoder and
// the decoder token lists in ONE launch.  One wave per token row (lane strides of 64 over E), fp32
// hardware atomics in L2 (-munsafe-fp-atomics: global_atomic_add_f32, no return value).
// Replaces two generic index_add launches (~0.28 ms each at B = 256: 102k + 26k rows).
#include "common.h"

__global__ __launch_bounds__(256) void emb_grad_kernel(float* __restrict__ gemb, const int64_t* __restrict__ ids0,
                                                       const float* __restrict__ src0, int n0,
                                                       const int64_t* __restrict__ ids1,
                                                       const float* __restrict__ src1, int n1, int E, int V) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= n0 + n1) return;
  const bool first = row < n0;
  const int r = first ? row : row - n0;
  const int64_t id = first ? ids0[r] : ids1[r];
  DCHECK_IN(id, 0, V, CHK_EMB_ID);
  if (id < 0 || id >= V) return;  // defensive: ids come from the vocab (< V)
  const float* s = (first ? src0 : src1) + (size_t)r * E;
  float* d = gemb + (size_t)id * E;
  for (int c = lane; c < E; c += 64) {  // coalesced 256-B atomics per wave instruction
    const float x = s[c];
    if (x != 0.f) atomicAdd(d + c, x);
  }
}

void launch_emb_grad(float* gemb, const int64_t* ids0, const float* src0, int n0, const int64_t* ids1,
                     const float* src1, int n1, int E, int V, hipStream_t st) {
  const int rows = n0 + n1;
  if (rows <= 0) return;
  hipLaunchKernelGGL(emb_grad_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, gemb, ids0, src0, n0, ids1, src1, n1, E,
                     V);
}

// Sorted variant: token rows visited in id order (perm = argsort of the concatenated
// [encoder; decoder] id list), 64 consecutive sorted rows per wave, each lane summing its
// E/64 columns in registers and issuing atomics only when the id changes.  Zipf-distributed
// text sends thousands of rows to the few hottest ids; the unsorted kernel serialises them on
// one address each (~0.32 ms at B = 256), here a hot id costs one atomic per 64-row chunk.
template <int PER>
__global__ __launch_bounds__(256) void emb_grad_sorted_kernel(float* __restrict__ gemb,
                                                              const int* __restrict__ sid,
                                                              const int* __restrict__ perm,
                                                              const float* __restrict__ src0, int n0,
                                                              const float* __restrict__ src1, int n1, int E, int V) {
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int n = n0 + n1, r0 = wv * 64;
  if (r0 >= n) return;
  const int r1 = min(r0 + 64, n);
  float acc[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) acc[j] = 0.f;
  int cur = sid[r0];
  for (int rb = r0; rb < r1; rb += 8) {
    // 8 rows' ids, source rows and values in flight before the (id-ordered) accumulation
    int idv[8];
    float xv[8][PER];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = min(rb + u, r1 - 1);
      idv[u] = rb + u < r1 ? sid[r] : -1;
      if (rb + u < r1) DCHECK_IN(idv[u], 0, V, CHK_EMB_ID);
      const int q = perm[r];
      const float* srow = q < n0 ? src0 + (size_t)q * E : src1 + (size_t)(q - n0) * E;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int c = lane + 64 * j;
        xv[u][j] = c < E ? srow[c] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int id = idv[u];  // wave-uniform
      if (id < 0) break;
      if (id != cur) {
        if (cur >= 0 && cur < V) {
#pragma unroll
          for (int j = 0; j < PER; ++j) {
            const int c = lane + 64 * j;
            if (c < E && acc[j] != 0.f) atomicAdd(gemb + (size_t)cur * E + c, acc[j]);
            acc[j] = 0.f;
          }
        }
        cur = id;
      }
#pragma unroll
      for (int j = 0; j < PER; ++j) acc[j] += xv[u][j];
    }
  }
  if (cur >= 0 && cur < V) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = lane + 64 * j;
      if (c < E && acc[j] != 0.f) atomicAdd(gemb + (size_t)cur * E + c, acc[j]);
    }
  }
}

void launch_emb_grad_sorted(float* gemb, const int* sid, const int* perm, const float* src0, int n0,
                            const float* src1, int n1, int E, int V, hipStream_t st) {
  const int n = n0 + n1;
  if (n <= 0) return;
  const int waves = (n + 63) / 64;
  const dim3 grid((waves + 3) / 4);
  const int per = (E + 63) / 64;
#define LE(P) hipLaunchKernelGGL(emb_grad_sorted_kernel<P>, grid, dim3(256), 0, st, gemb, sid, perm, src0, n0, src1, n1, E, V)
  if (per <= 1) LE(1);
  else if (per <= 2) LE(2);
  else if (per <= 4) LE(4);
  else LE(8);
#undef LE
}
