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
#include "lds_frag.h"
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

// ---------------------------------------------------------------------------------------------
// wgrad_tt: the long-K weight-gradient GEMM as 256 x BN tiles with a deterministic split-K
// (round-6 review item 2; reference model.py:290-297 -- tf.gradients over the encoder LSTM input
// / recurrent kernels, model.py:89-93):
//
//   slab[s][m][n] = sum_{k in chunk s} a[k][m] b[k][n]      (this kernel, fp32, no atomics)
//   out[m][n]     = sum_s slab[s][m][n]  in s order         (wgrad_sum_kernel)
//
// so the result does not depend on scheduling (the torch split-K path's bmm + torch.sum and the
// fp32-atomic wgrad_tn above are replaced for the encoder weight gradients).
//
// Geometry: 512 threads = 8 waves as 2 (m) x 4 (n), a wave 128 (m) x BN/4 (n) of
// v_mfma_f32_16x16x32_bf16 accumulators; K steps of 64.  Both operands are K-major ([k][m] /
// [k][n] rows of 512 bytes); each K tile is staged by global_load_lds_dwordx4 (1 KB per wave
// instruction: 4 rows of a 128-column half image) into two LDS stages; the MFMA operands are read
// transposed by ds_read_b64_tr_b16 (two per fragment).  Half images of 128 columns use
// 256-byte rows with the 16-byte chunk ch of row r at ch ^ (((r & 3) << 2) | ((r >> 2) & 3))
// (cdna_hip_programming.md T10 (b)): the two 4-row blocks a 32-lane half reads, 8 rows apart in
// the same columns, hit distinct banks.  The XOR is applied to the per-lane GLOBAL source
// address, so the LDS-DMA image stays lane-linear.
//
// Workgroup order: lin (the bijective XCD remap) -> split s = lin / tiles, tile = lin % tiles, so
// the tiles of one K chunk are consecutive in lin, i.e. on one XCD: that XCD's L2 serves the
// chunk's a / b panels to all of its tiles (HBM reads each operand once).

template <int BN>
__global__ __launch_bounds__(512, 1) void wgrad_tt_kernel(const bf16* __restrict__ a, int lda, const bf16* __restrict__ b,
                                                          int ldb, float* __restrict__ dst, long sstride, int ldd,
                                                          int nv, int M, int N, int kchunk, int K) {
  constexpr int BM = 256, BK = 64, HI = 64 * 256;           // half-image bytes (64 rows x 256 B)
  constexpr int NHA = BM / 128, NHB = BN / 128;             // half images per operand
  constexpr int STAGE = (NHA + NHB) * HI;
  constexpr int WN = BN / 4, NJ = WN / 16;                  // wave columns, 16-col subtiles
  constexpr int PPW = (NHA + NHB) * 16 / 8;                 // glds pieces per wave per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int tm = M / BM, tn = N / BN, tiles = tm * tn;
  const int nwg = gridDim.x, id = blockIdx.x, xcd = id & 7, qq = nwg >> 3, r8 = nwg & 7;
  const int lin = (xcd < r8 ? xcd * (qq + 1) : r8 * (qq + 1) + (xcd - r8) * qq) + (id >> 3);
  const int s = lin / tiles, tile = lin - s * tiles;
  const int m0 = (tile / tn) * BM, n0 = (tile % tn) * BN;
  const int k0 = s * kchunk, nk = (min(K, k0 + kchunk) - k0) / BK;
  // glds piece pc (0 .. 16 (NHA + NHB) - 1) of a stage: half image h = pc / 16, rows 4 (pc % 16) ..
  // + 3; lane l: row 4 (pc % 16) + (l >> 4), physical chunk l & 15 <- logical chunk (l & 15) ^ sw(row)
  const bf16* src[PPW];
  size_t kstep[PPW];  // elements per K step of the piece's operand
  int ldst[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int pc = wid * PPW + j, h = pc >> 4, row = 4 * (pc & 15) + (lane >> 4);
    const int ch = (lane & 15) ^ tt_sw(row);
    src[j] = h < NHA ? a + (size_t)(k0 + row) * lda + m0 + 128 * h + 8 * ch
                     : b + (size_t)(k0 + row) * ldb + n0 + 128 * (h - NHA) + 8 * ch;
    kstep[j] = (size_t)BK * (h < NHA ? lda : ldb);
    ldst[j] = h * HI + (pc & 15) * 1024;
  }
  const unsigned sbase = (unsigned)(uintptr_t)(tt_lds_t)smem;
  auto stage = [&](int buf, int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PPW; ++j)
      glds16_asm(src[j] + kt * kstep[j], __builtin_amdgcn_readfirstlane(sbase + buf * STAGE + ldst[j]));
  };
  const int wr = wid >> 2, wc = wid & 3;
  // the wave's images: a half image wr (its 128 m), b half image (wc * WN) / 128 at column offset
  const int bimg = NHA + (wc * WN) / 128, bcol = (wc * WN) % 128;
  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  // Measured and not kept (profiles/r6/wgrad_tt.md): a ping-pong schedule (the two wave groups
  // one barrier apart, reads of one beside the MFMAs of the other: 256 VGPRs + 36 bytes of
  // scratch, 1.6x slower) and a 4-wave 128 x 128-per-wave kernel with register-double-buffered
  // fragments (452 registers, 7-13 % slower at the config #5 shapes).
  if (nk > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(buf ^ 1, kt + 1);
    const char* Ai = smem + buf * STAGE + wr * HI;
    const char* Bi = smem + buf * STAGE + bimg * HI;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 fb[NJ], fa[8];
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[j] = tt_frag(Bi, 32 * kk, bcol + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = tt_frag(Ai, 32 * kk, 16 * i, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // accumulator (i, j, r): m = m0 + 128 wr + 16 i + 4 (l >> 4) + r, n = n0 + wc WN + 16 j + (l & 15);
  // to split s's slab (sstride apart, rows of ldd = N) or, unsplit, straight to the output rows
  // (ldd = ldo), columns n < nv
  float* sl = dst + (size_t)s * sstride;
  const int nl = n0 + wc * WN + (lane & 15);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float* row = sl + (size_t)(m0 + 128 * wr + 16 * i + 4 * (lane >> 4) + r) * ldd + nl;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if (nl + 16 * j < nv) row[16 * j] = acc[i][j][r];
    }
}

// out[m][n] (= or +=) sum_{s < S} slab[s][m][n], s ascending; trans: slab is [S][N][M] (the roles
// of the operands were swapped) and out[m][n] = sum_s slab[s][n][m] through a 64 x 64 LDS tile
template <bool TRANS>
__global__ __launch_bounds__(256) void wgrad_sum_kernel(const float* __restrict__ slab, float* __restrict__ out, int ldo,
                                                        int M, int N, int S, bool acc, int nv) {
  if constexpr (!TRANS) {  // out columns n < nv (nv % 4 == 0)
    const size_t i4 = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4, MN = (size_t)M * N;
    if (i4 >= MN || (int)(i4 % N) >= nv) return;
    float4 t = *reinterpret_cast<const float4*>(slab + i4);
    for (int s = 1; s < S; ++s) {
      const float4 u = *reinterpret_cast<const float4*>(slab + (size_t)s * MN + i4);
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    const int m = (int)(i4 / N), n = (int)(i4 % N);
    float* op = out + (size_t)m * ldo + n;
    if (((uintptr_t)op & 15) == 0) {
      float4* o = reinterpret_cast<float4*>(op);
      if (acc) {
        const float4 u = *o;
        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
      }
      *o = t;
    } else {  // an output slice of the flat gradient buffer need not be 16-byte aligned
      if (acc) {
        t.x += op[0]; t.y += op[1]; t.z += op[2]; t.w += op[3];
      }
      op[0] = t.x; op[1] = t.y; op[2] = t.z; op[3] = t.w;
    }
  } else {
    // slab [S][N][M] -> out [M][N]; block = 64 (n) x 64 (m) of the slab
    __shared__ float tile[64][65];
    const int nb = blockIdx.x % (N / 64), mb = blockIdx.x / (N / 64);
    const size_t MN = (size_t)M * N;
    const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
    float t[16];  // slab rows n = nb 64 + r0 + 4 e, column m = mb 64 + c: 16 independent loads per split
    const float* base = slab + (size_t)(nb * 64 + r0) * M + mb * 64 + c;
#pragma unroll
    for (int e = 0; e < 16; ++e) t[e] = base[(size_t)4 * e * M];
    for (int s = 1; s < S; ++s) {
#pragma unroll
      for (int e = 0; e < 16; ++e) t[e] += base[s * MN + (size_t)4 * e * M];
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) tile[r0 + 4 * e][c] = t[e];
    __syncthreads();
    for (int rr = r0; rr < 64; rr += 4) {  // out row m = mb 64 + rr, column n = nb 64 + c
      float* o = out + (size_t)(mb * 64 + rr) * ldo + nb * 64 + c;
      *o = acc ? *o + tile[c][rr] : tile[c][rr];
    }
  }
}

// out[m][n] (= or +=) sum_s slab[s][m][n] in split order ([S][M][N] fp32; the split-K gemm_bt)
void launch_slab_sum(const float* slab, float* out, int ldo, int M, int N, int S, bool acc, hipStream_t st) {
  const size_t n4 = (size_t)M * N / 4;
  hipLaunchKernelGGL(wgrad_sum_kernel<false>, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, slab, out, ldo, M, N,
                     S, acc, N);
}

// the split of K: ~1 workgroup per CU (tiles x S >= 256), chunks of whole 64-row steps
int wgrad_tt_splits(int M, int N, int K) {
  const int BN = N % 256 == 0 ? 256 : 128;
  const int tiles = (M / 256) * (N / BN), steps = K / 64;
  int s = (256 + tiles - 1) / tiles;
  s = s < 1 ? 1 : (s > steps ? steps : s);
  const int kc = (steps + s - 1) / s;
  return (steps + kc - 1) / kc;
}
bool wgrad_tt_ok(int M, int N, int K) { return M % 256 == 0 && N % 128 == 0 && K % 64 == 0 && K >= 64; }
bool wgrad_tt_direct(int M, int N, int K, bool trans, bool acc) { return !trans && !acc && wgrad_tt_splits(M, N, K) == 1; }

void launch_wgrad_tt(const bf16* a, int lda, const bf16* b, int ldb, float* slab, float* out, int ldo, int M, int N,
                     int K, bool trans, bool acc, int nv, hipStream_t st) {
  const int BN = N % 256 == 0 ? 256 : 128;
  const int S = wgrad_tt_splits(M, N, K), steps = K / 64, kc = (steps + S - 1) / S;
  const int grid = (M / 256) * (N / BN) * S;
  const size_t lds = (size_t)(2 + BN / 128) * 64 * 256 * 2;
  // one split and a plain store: the tiles go straight to out (no slab pass)
  const bool direct = wgrad_tt_direct(M, N, K, trans, acc);
  float* dst = direct ? out : slab;
  const long sstride = direct ? 0 : (long)M * N;
  const int ldd = direct ? ldo : N, nvk = direct ? nv : N;
  if (BN == 256) {
    (void)hipFuncSetAttribute((const void*)wgrad_tt_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(wgrad_tt_kernel<256>, dim3(grid), dim3(512), lds, st, a, lda, b, ldb, dst, sstride, ldd, nvk, M, N,
                       kc * 64, K);
  } else {
    (void)hipFuncSetAttribute((const void*)wgrad_tt_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(wgrad_tt_kernel<128>, dim3(grid), dim3(512), lds, st, a, lda, b, ldb, dst, sstride, ldd, nvk, M, N,
                       kc * 64, K);
  }
  if (direct) return;
  if (!trans) {
    const size_t n4 = (size_t)M * N / 4;
    hipLaunchKernelGGL(wgrad_sum_kernel<false>, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, slab, out, ldo, M, N,
                       S, acc, nv);
  } else {  // out is [N][M] (ldo), the slab [S][M][N]: out[n][m] = sum slab[s][m][n]
    hipLaunchKernelGGL(wgrad_sum_kernel<true>, dim3((M / 64) * (N / 64)), dim3(256), 0, st, slab, out, ldo, N, M, S, acc,
                       M);
  }
}
