// Weight repack after every optimizer step: fp32 master views -> the bf16 kernel
// layouts (plain copies, transposes, gate-interleaved permutations, concatenations) and a few
// fp32 copies, as ONE launch over a device table of jobs.  Replaces ~50 torch cast / copy /
// cat launches (~5 us each) in the optimizer graph.  Casts round to nearest even.
//
// Job (13 int64): src, dst, d0, d1, d2, src strides s0..s2, dst strides t0..t2 (elements),
// first flat element of the job, dst dtype (0 bf16, 1 fp32).  Jobs are laid out back to back in
// a flat element space; a thread finds its job by binary search over the (LDS-staged) starts.
#include "common.h"

#define PACK_MAXJ 64

__global__ __launch_bounds__(256) void pack_cast_kernel(const long* __restrict__ jobs, int nj, long total) {
  __shared__ long start[PACK_MAXJ + 1];
  for (int j = threadIdx.x; j < nj; j += 256) start[j] = jobs[(size_t)j * 13 + 11];
  if (threadIdx.x == 0) start[nj] = total;
  __syncthreads();
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    int lo = 0, hi = nj - 1;  // last job with start <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (start[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    const long* J = jobs + (size_t)lo * 13;
    const unsigned li = (unsigned)(i - start[lo]);
    const unsigned d1 = (unsigned)J[3], d2 = (unsigned)J[4];
    const unsigned i2 = li % d2, r = li / d2, i1 = r % d1, i0 = r / d1;
    const float v = reinterpret_cast<const float*>(J[0])[i0 * J[5] + i1 * J[6] + i2 * J[7]];
    const long o = i0 * J[8] + i1 * J[9] + i2 * J[10];
    if (J[12]) reinterpret_cast<float*>(J[1])[o] = v;
    else reinterpret_cast<bf16*>(J[1])[o] = f2bf(v);
  }
}

int pack_max_jobs() { return PACK_MAXJ; }

void launch_pack_cast(const long* jobs, int nj, long total, hipStream_t st) {
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pack_cast_kernel, dim3((unsigned)blocks), dim3(256), 0, st, jobs, nj, total);
}
