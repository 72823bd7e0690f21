// Weight-gradient GEMM  out[M][N] += sum_k a[k][m] b[k][n]  (both operands K-major: rows are
// tokens / decoder steps x batch, K = 25.6k-102k; M <= 1024, N up to the 50k vocabulary),
// split-K over workgroups with fp32 atomics into the pre-zeroed gradient buffer (SURVEY K22
// weight gradients, incl. the vocab projection dW = X^T . dlogits of model.py:229-236).
//
// Why not the library GEMM: hipBLASLt runs these shapes as stream-K kernels whose tile owners
// spin on flags of higher-numbered workgroups.  Beside another spinning kernel (a second
// stream-K GEMM, the persistent LSTM BPTT) each can hold CUs the other's waiting workgroups
// need -- two concurrent library GEMMs did hang on MI355X.  This kernel never waits on another
// workgroup, so it can run on a side stream beside the encoder BPTT (pointer_generator.py,
// TSAMD_DEFER_WGRAD).
//
// Tile 128 (m) x 128 (n) per workgroup, 4 waves of 64 x 64, k-steps of 64 (32: 3-5% slower) staged through
// double-buffered LDS as [k][m] / [k][n] rows (coalesced 16-byte global loads).  The MFMA wants
// each lane's 8 consecutive k of one m (A) or one n (B): gfx950's ds_read_b64_tr_b16 reads a
// 4-row x 16-column block and hands lane i of each 16-lane group column i of the 4 rows, so two
// transposed reads per fragment turn the k-major image into MFMA operands without a transpose
// pass.
#include "common.h"
#include <stdlib.h>

namespace {

constexpr int WBM = 128, WBN = 128;
constexpr int WPAD = 16;  // bf16 per LDS row: 288-byte rows put rows r and r + 1 eight banks apart
constexpr int WLD = WBM + WPAD;

typedef short v4i16 __attribute__((ext_vector_type(4)));

// lane l: rows 8 (l >> 4) + 4 half + ((l & 15) >> 2) and columns c0 + 4 (l & 3) of the image;
// returns 4 bf16 of column c0 + (l & 15), rows 8 (l >> 4) + 4 half .. + 3
__device__ __forceinline__ v4i16 tr_read(const bf16* img, int c0, int half, int lane) {
  const int row = 8 * (lane >> 4) + 4 * half + ((lane & 15) >> 2);  // within a 32-row k-slice
  const bf16* p = img + row * WLD + c0 + 4 * (lane & 3);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(const_cast<bf16*>(p)));
}

__device__ __forceinline__ bf16x8 frag(const bf16* img, int c0, int lane) {
  const v4i16 lo = tr_read(img, c0, 0, lane), hi = tr_read(img, c0, 1, lane);
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 v = v8i16{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

}  // namespace

// 1-D grid of gm x ceil8(ny) blocks, ny = ceil(N / 128) x splits (see the block map below); M a
// multiple of 128, N a multiple of 8 (column chunks past N are zero-filled and not stored), any
// K (rows past the chunk end are zero-filled); lda / ldb / ldo in elements
template <int WBK>
__global__ __launch_bounds__(256) void wgrad_tn_kernel(const bf16* __restrict__ a, int lda, const bf16* __restrict__ b,
                                                       int ldb, float* __restrict__ out, int ldo, int N, int K,
                                                       int kchunk, int gm, int gn, int ny) {
  constexpr int CPT = WBK * 16 / 256;  // 16-byte chunks per thread per operand and stage
  __shared__ __attribute__((aligned(16))) bf16 As[2][WBK * WLD];
  __shared__ __attribute__((aligned(16))) bf16 Bs[2][WBK * WLD];
  // XCD-aware block map: workgroups are dealt to the 8 XCDs round-robin by linear id, so
  // blocks L and L + 8 share an XCD.  The gm row tiles of one (column tile, k-chunk) pair get
  // ids 8 (gm j + i) + x (i < gm): they run on ONE XCD at about the same time and the b-operand
  // rows (the tall K x N operand, e.g. the 2.56 GB vocab dlogits) come from HBM once and from
  // that XCD's L2 for the other row tiles.
  const int L = blockIdx.x, xcd = L & 7, q = L >> 3;
  const int yi = (q / gm) * 8 + xcd;
  if (yi >= ny) return;  // padding of ny to a multiple of 8 (uniform per block, before any barrier)
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int m0 = (q % gm) * WBM, n0 = (yi % gn) * WBN;
  const int k0 = (yi / gn) * kchunk, k1 = min(K, k0 + kchunk);
  if (k0 >= k1) return;
  const int wm = (wid & 1) * 64, wn = (wid >> 1) * 64;
  // staging: WBK rows x 128 columns = WBK * 16 chunks of 16 B per operand, CPT per thread
  bf16x8 ra[CPT], rb[CPT];
  auto fetch = [&](int kb) {
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const int c = tid + 256 * u, r = c >> 4, col = (c & 15) * 8, k = kb + r;
      if (k < k1) {
        ra[u] = ld8(a + (size_t)k * lda + m0 + col);
        rb[u] = n0 + col < N ? ld8(b + (size_t)k * ldb + n0 + col) : zero8();
      } else {
        ra[u] = zero8();
        rb[u] = zero8();
      }
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const int c = tid + 256 * u, r = c >> 4, col = (c & 15) * 8;
      *reinterpret_cast<bf16x8*>(&As[buf][r * WLD + col]) = ra[u];
      *reinterpret_cast<bf16x8*>(&Bs[buf][r * WLD + col]) = rb[u];
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  fetch(k0);
  stash(0);
  __syncthreads();
  int buf = 0;
  for (int kb = k0; kb < k1; kb += WBK) {
    const bool more = kb + WBK < k1;
    if (more) fetch(kb + WBK);  // in flight during this step's MFMAs
#pragma unroll
    for (int ks = 0; ks < WBK / 32; ++ks) {
      const bf16* Ak = As[buf] + ks * 32 * WLD;
      const bf16* Bk = Bs[buf] + ks * 32 * WLD;
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag(Ak, wm + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag(Bk, wn + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
    }
    if (more) stash(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // accumulator (i, j, r): m = wm + 16 i + 4 (lane >> 4) + r, n = wn + 16 j + (lane & 15)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float* row = out + (size_t)(m0 + wm + 16 * i + 4 * (lane >> 4) + r) * ldo + n0 + wn + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n0 + wn + 16 * j + (lane & 15) < N) atomicAdd(row + 16 * j, acc[i][j][r]);
    }
}

// splits: enough workgroups for ~2 per CU, each at least 512 rows of K
int wgrad_tn_splits(int M, int N, int K) {
  const int tiles = (M / WBM) * ((N + WBN - 1) / WBN);
  int s = (512 + tiles - 1) / tiles;
  const int smax = (K + 511) / 512;
  return s < 1 ? 1 : (s > smax ? smax : s);
}

void launch_wgrad_tn(const bf16* a, int lda, const bf16* b, int ldb, float* out, int ldo, int M, int N, int K,
                     hipStream_t st) {
  constexpr int WBK = 64;
  const int s = wgrad_tn_splits(M, N, K);
  const int kchunk = ((K + s - 1) / s + WBK - 1) / WBK * WBK;
  const int splits = (K + kchunk - 1) / kchunk;
  const int gm = M / WBM, gn = (N + WBN - 1) / WBN, ny = gn * splits;
  const dim3 grid(gm * ((ny + 7) / 8 * 8));
  hipLaunchKernelGGL(wgrad_tn_kernel<WBK>, grid, dim3(256), 0, st, a, lda, b, ldb, out, ldo, N, K, kchunk, gm, gn, ny);
}
