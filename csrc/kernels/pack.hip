// Weight repack after every optimizer step: fp32 master views -> the bf16 kernel
// layouts (plain copies, transposes, gate-interleaved permutations, concatenations) and a few
// fp32 copies, as ONE launch over a device table of jobs.  Replaces ~50 torch cast / copy /
// cat launches (~5 us each) in the optimizer graph.  Casts round to nearest even.
//
// A block finds its job by binary search over the (LDS-staged) first blocks of the jobs.
#include "common.h"

#define PACK_MAXJ 64
#define PACK_COLS 16  // int64 per job row

// Job row (PACK_COLS int64): src, dst, d0, d1, d2, src strides s0..s2, dst strides t0..t2
// (elements), first block, kind, dst dtype (0 bf16, 1 fp32), element count, scale (the bits of an
// fp32 factor applied before the cast in the low 32 bits; 0 = 1.0).  Kinds (host-classified):
//   0 generic strided copy: 256 elements per block, one per thread (index math per element);
//   1 contiguous src and dst: 2048 elements per block, 8 per thread (two 16-byte loads, one
//     16-byte bf16 store);
//   2 transpose: dst [d1][d2] contiguous, src its transpose view of a contiguous [d2][d1]
//     matrix (strides (1, d1)): 64 x 64 tiles through LDS, both sides coalesced;
//   3 row-strided 2-D copy (unit column strides, d2 % 8 == 0, 16-byte aligned rows): kind 1's
//     8 per thread with a row stride on either side -- the vocab W into its 128-aligned [H][Vp]
//     image (as kind 0 it took the repack from 50 to 85 us).
// Round 3's single element-per-thread kernel spent 194 us per step on the 32M-element repack
// (the 12.8M-element vocab W^T transpose and two plain 6.4M / 12.8M copies dominate).
__global__ __launch_bounds__(256) void pack_cast_kernel(const long* __restrict__ jobs, int nj, long total) {
  __shared__ long start[PACK_MAXJ + 1];
  __shared__ float tile[64][65];
  for (int j = threadIdx.x; j < nj; j += 256) start[j] = jobs[(size_t)j * PACK_COLS + 11];
  if (threadIdx.x == 0) start[nj] = total;
  __syncthreads();
  const long blk = blockIdx.x;
  int lo = 0, hi = nj - 1;  // last job whose first block <= blk
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (start[mid] <= blk) lo = mid;
    else hi = mid - 1;
  }
  const long* J = jobs + (size_t)lo * PACK_COLS;
  const long jb = blk - start[lo];
  const int kind = (int)J[12], f32o = (int)J[13];
  const long n = J[14];
  const float sc = J[15] ? __int_as_float((int)J[15]) : 1.f;
  const float* src = reinterpret_cast<const float*>(J[0]);
  if (kind == 1) {
    const long e0 = jb * 2048 + (long)threadIdx.x * 8;
    if (e0 >= n) return;
    if (e0 + 8 <= n) {
      float4 a = *reinterpret_cast<const float4*>(src + e0);
      float4 b = *reinterpret_cast<const float4*>(src + e0 + 4);
      a.x *= sc; a.y *= sc; a.z *= sc; a.w *= sc;
      b.x *= sc; b.y *= sc; b.z *= sc; b.w *= sc;
      if (f32o) {
        float* d = reinterpret_cast<float*>(J[1]) + e0;
        *reinterpret_cast<float4*>(d) = a;
        *reinterpret_cast<float4*>(d + 4) = b;
      } else {
        bf16x8 o;
        o[0] = f2bf(a.x); o[1] = f2bf(a.y); o[2] = f2bf(a.z); o[3] = f2bf(a.w);
        o[4] = f2bf(b.x); o[5] = f2bf(b.y); o[6] = f2bf(b.z); o[7] = f2bf(b.w);
        *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(J[1]) + e0) = o;
      }
    } else {
      for (long e = e0; e < n; ++e) {
        if (f32o) reinterpret_cast<float*>(J[1])[e] = src[e] * sc;
        else reinterpret_cast<bf16*>(J[1])[e] = f2bf(src[e] * sc);
      }
    }
    return;
  }
  if (kind == 2) {  // dst [R = d1][C = d2]; base = the contiguous [C][R] matrix src views
    const long R = J[3], C = J[4];
    const long tr = (R + 63) / 64;
    const long i0 = (jb % tr) * 64, c0 = (jb / tr) * 64;  // dst rows i0.., dst cols (base rows) c0..
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int k = ty; k < 64; k += 4) {  // base row c0 + k, base cols (dst rows) i0 + tx: coalesced
      const long c = c0 + k, i = i0 + tx;
      tile[k][tx] = (c < C && i < R) ? src[c * R + i] : 0.f;
    }
    __syncthreads();
    for (int k = ty; k < 64; k += 4) {  // dst row i0 + k, cols c0 + tx: coalesced
      const long i = i0 + k, c = c0 + tx;
      if (i < R && c < C) {
        const float v = tile[tx][k] * sc;
        if (f32o) reinterpret_cast<float*>(J[1])[i * C + c] = v;
        else reinterpret_cast<bf16*>(J[1])[i * C + c] = f2bf(v);
      }
    }
    return;
  }
  if (kind == 3) {  // 2-D [R][C] with row strides J[6] (src) / J[9] (dst), C % 8 == 0: 8 per thread
    const long e0 = jb * 2048 + (long)threadIdx.x * 8;
    if (e0 >= n) return;
    const long C = J[4], r = e0 / C, c = e0 - r * C;
    const float* sp = src + r * J[6] + c;
    float4 a = *reinterpret_cast<const float4*>(sp);
    float4 b = *reinterpret_cast<const float4*>(sp + 4);
    a.x *= sc; a.y *= sc; a.z *= sc; a.w *= sc;
    b.x *= sc; b.y *= sc; b.z *= sc; b.w *= sc;
    const long o = r * J[9] + c;
    if (f32o) {
      float* d = reinterpret_cast<float*>(J[1]) + o;
      *reinterpret_cast<float4*>(d) = a;
      *reinterpret_cast<float4*>(d + 4) = b;
    } else {
      bf16x8 v;
      v[0] = f2bf(a.x); v[1] = f2bf(a.y); v[2] = f2bf(a.z); v[3] = f2bf(a.w);
      v[4] = f2bf(b.x); v[5] = f2bf(b.y); v[6] = f2bf(b.z); v[7] = f2bf(b.w);
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(J[1]) + o) = v;
    }
    return;
  }
  const long li = jb * 256 + threadIdx.x;
  if (li >= n) return;
  const unsigned d1 = (unsigned)J[3], d2 = (unsigned)J[4];
  const unsigned ul = (unsigned)li, i2 = ul % d2, r = ul / d2, i1 = r % d1, i0 = r / d1;
  const float v = src[i0 * J[5] + i1 * J[6] + i2 * J[7]] * sc;
  const long o = i0 * J[8] + i1 * J[9] + i2 * J[10];
  if (f32o) reinterpret_cast<float*>(J[1])[o] = v;
  else reinterpret_cast<bf16*>(J[1])[o] = f2bf(v);
}

int pack_max_jobs() { return PACK_MAXJ; }
int pack_job_cols() { return PACK_COLS; }

// total: blocks over all jobs (the host's sum of the per-job block counts)
void launch_pack_cast(const long* jobs, int nj, long total, hipStream_t st) {
  if (total <= 0) return;
  hipLaunchKernelGGL(pack_cast_kernel, dim3((unsigned)total), dim3(256), 0, st, jobs, nj, total);
}
