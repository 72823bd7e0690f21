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

// ------------------------------------------------------------- deterministic variant
// TSAMD_DETERMINISTIC: the same id-ordered rows, summed in a fixed order with no atomics.
// Pass 1: wave w sums its 64 sorted rows segment by segment (in row order).  A segment wholly
// inside the chunk is stored straight into gemb (its only writer); the chunk's first segment,
// when it began in an earlier chunk, goes to pf[w]; its last segment, when it began here and
// continues into the next chunk, goes to pl[w].  Pass 2: the chunk where such a segment starts
// adds pl[w] + pf[w+1] + pf[w+2] + ... along the chunks it spans (in chunk order) and stores
// the total.  Summation order depends only on the (host-sorted, stable) row order.
namespace {
struct ChunkInfo {
  int r0, r1, first, last;
  bool cont, conts;  // the first segment began earlier / the last segment continues later
};
__device__ __forceinline__ ChunkInfo chunk_info(const int* sid, int w, int n) {
  ChunkInfo c;
  c.r0 = w * 64;
  c.r1 = min(c.r0 + 64, n);
  c.first = sid[c.r0];
  c.last = sid[c.r1 - 1];
  c.cont = c.r0 > 0 && sid[c.r0 - 1] == c.first;
  c.conts = c.r1 < n && sid[c.r1] == c.last;
  return c;
}
}  // namespace

template <int PER>
__global__ __launch_bounds__(256) void emb_grad_det_pass1(float* __restrict__ gemb, const int* __restrict__ sid,
                                                          const int* __restrict__ perm, const float* __restrict__ src0,
                                                          int n0, const float* __restrict__ src1, int n1, int E,
                                                          int V, float* __restrict__ pf, float* __restrict__ pl) {
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int n = n0 + n1;
  if (wv * 64 >= n) return;
  const ChunkInfo ci = chunk_info(sid, wv, n);
  float acc[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) acc[j] = 0.f;
  int cur = ci.first;
  bool first_seg = true;
  auto emit = [&](bool is_last) {
    float* dst;
    if (first_seg && ci.cont) dst = pf + (size_t)wv * E;
    else if (is_last && ci.conts) dst = pl + (size_t)wv * E;
    else dst = (cur >= 0 && cur < V) ? gemb + (size_t)cur * E : nullptr;
    if (dst) {
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int c = lane + 64 * j;
        if (c < E) dst[c] = acc[j];
      }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) acc[j] = 0.f;
    first_seg = false;
  };
  for (int r = ci.r0; r < ci.r1; ++r) {
    const int id = sid[r];
    if (id != cur) {
      emit(false);
      cur = id;
    }
    const int q = perm[r];
    const float* srow = q < n0 ? src0 + (size_t)q * E : src1 + (size_t)(q - n0) * E;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = lane + 64 * j;
      if (c < E) acc[j] += srow[c];
    }
  }
  emit(true);
}

__global__ __launch_bounds__(256) void emb_grad_det_pass2(float* __restrict__ gemb, const int* __restrict__ sid,
                                                          int n, int E, int V, const float* __restrict__ pf,
                                                          const float* __restrict__ pl) {
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nw = (n + 63) / 64;
  if (wv >= nw) return;
  const ChunkInfo ci = chunk_info(sid, wv, n);
  // pl[wv] holds a segment that starts in this chunk and continues
  if (!ci.conts || (ci.first == ci.last && ci.cont)) return;
  const int id = ci.last;
  for (int c = lane; c < E; c += 64) {
    float s = pl[(size_t)wv * E + c];
    for (int w2 = wv + 1; w2 < nw; ++w2) {
      s += pf[(size_t)w2 * E + c];
      const int r1 = min(w2 * 64 + 64, n);
      const bool middle = sid[r1 - 1] == id && r1 < n && sid[r1] == id;
      if (!middle) break;
    }
    if (id >= 0 && id < V) gemb[(size_t)id * E + c] = s;
  }
}

int emb_grad_det_chunks(int n) { return (n + 63) / 64; }

void launch_emb_grad_det(float* gemb, const int* sid, const int* perm, const float* src0, int n0, const float* src1,
                         int n1, int E, int V, float* pf, float* pl, hipStream_t st) {
  const int n = n0 + n1;
  if (n <= 0) return;
  const int waves = (n + 63) / 64;
  const dim3 grid((waves + 3) / 4);
  const int per = (E + 63) / 64;
#define LD(P) hipLaunchKernelGGL(emb_grad_det_pass1<P>, grid, dim3(256), 0, st, gemb, sid, perm, src0, n0, src1, n1, E, \
                                 V, pf, pl)
  if (per <= 1) LD(1);
  else if (per <= 2) LD(2);
  else if (per <= 4) LD(4);
  else LD(8);
#undef LD
  hipLaunchKernelGGL(emb_grad_det_pass2, grid, dim3(256), 0, st, gemb, sid, n, E, V, pf, pl);
}
