// Batched attention-context GEMMs of the training step (reference attention_decoder.py:117-127
// context = sum_i a_i h_i and its gradients through tf.gradients, model.py:290-297), one launch
// each over the whole decoder (all D steps at once), bf16 MFMA (v_mfma_f32_16x16x32_bf16), fp32
// accumulate:
//
//   ctx_fwd  CTX[d][b][n]  = sum_t att[d][b][t] . enc[b][t][n]   (+ the bf16 twin CTXb)
//   ctx_da   dA[d][b][t] (+)= sum_n dctx[d][b][n] . enc[b][t][n]
//   ctx_de   dE[b][t][n]   = sum_d att[d][b][t] . dctx[d][b][n]
//
// att / dctx are the step-major [D][B][*] buffers the decoder loop writes, enc the encoder output
// [B][T][A].  They replace three torch.bmm calls (strided per-batch views of those buffers) and
// the two tr01 layout passes that moved their [B][D][*] outputs to step-major: the outputs are
// stored step-major here.  All three are memory-bound (K = T, A or D against 100-row tiles): the
// design goal is one HBM pass over the large operand (enc_out, or the dE output) per launch.
//
// Staging: every operand K-tile goes global -> LDS by global_load_lds_dwordx4 (inline-asm form,
// lds_frag.h) into
//   * K-major images (rows of 64 bf16 = 128 B, chunk c of row r at c ^ ((r >> 1) & 7)): operands
//     whose rows run along K (att for ctx_fwd, dctx / enc for ctx_da), read as fragments by
//     ds_read_b128 -- 16 rows of one 16-lane group land on 16 distinct 16-byte bank slots;
//   * half images (rows of 128 bf16 = 256 B, tt_sw swizzle): operands whose rows run along M or N
//     (enc for ctx_fwd, att / dctx for ctx_de), read transposed by ds_read_b64_tr_b16 (tt_frag).
// Workgroup order: blockIdx is remapped XCD-bijectively so the column tiles of one batch row b are
// consecutive, i.e. on one XCD: its L2 serves the shared operand (att / dctx rows of b) to them.
#include "common.h"
#include "launchers.h"
#include "lds_frag.h"
#include <stdlib.h>

namespace {

__device__ __forceinline__ int km_sw(int r) { return (r >> 1) & 7; }

// MFMA operand (rows r0 .. r0 + 15, k-sub-step kk of a 64-wide K tile) from a K-major image
__device__ __forceinline__ bf16x8 km_frag(const char* img, int r0, int kk, int lane) {
  const int r = r0 + (lane & 15), c = kk * 4 + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(img + r * 128 + 16 * (c ^ km_sw(r)));
}

// bijective XCD remap of blockIdx (cdna_hip_programming.md s5): consecutive lin share an XCD
__device__ __forceinline__ int xcd_lin() {
  const int nwg = gridDim.x, id = blockIdx.x, xcd = id & 7, q = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (id >> 3);
}

__device__ __forceinline__ unsigned lds_addr(const char* p) { return (unsigned)(uintptr_t)(tt_lds_t)p; }

constexpr int CB_MT = 8;  // 16-row m tiles of the D (<= 128) side

}  // namespace

// one workgroup per (b, 128 output columns n0..): 4 waves, wave w owns columns n0 + 32 w .. + 31
// (2 n tiles) of all ceil(D / 16) row tiles.  K = T in steps of 64, double-buffered; the K tail
// (T % 64) is zeroed in the enc fragments (T % 8 == 0).
__global__ __launch_bounds__(256) void ctx_fwd_kernel(const bf16* __restrict__ att, const bf16* __restrict__ enc,
                                                      float* __restrict__ ctx, bf16* __restrict__ ctxb, int B, int T,
                                                      int D, int A) {
  constexpr int AI = 128 * 128, EI = 64 * 256, STAGE = AI + EI;  // att K-major image, enc half image
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int ntn = A / 128, lin = xcd_lin(), b = lin / ntn, n0 = (lin - b * ntn) * 128;
  const int mt = (D + 15) >> 4, nk = (T + 63) / 64;
  // glds pieces: att image pieces p = 4 wid + j (rows 8 p .. + 7, lane row 8 p + (l >> 3), slot l & 7);
  // enc image pieces p (rows 4 p .. + 3, lane row 4 p + (l >> 4), slot l & 15)
  const bf16* asrc[4];
  bool aon[4];
  int ar[4], er[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = 4 * wid + j, row = 8 * p + (lane >> 3);
    aon[j] = 8 * p < D;  // pieces wholly past D are not loaded (their rows are never stored)
    ar[j] = (lane & 7) ^ km_sw(row);  // the logical k chunk this lane's slot holds
    asrc[j] = att + ((size_t)min(row, D - 1) * B + b) * T;
    er[j] = 4 * p + (lane >> 4);
  }
  const int ech = (lane & 15);
  const unsigned sbase = lds_addr(smem);
  auto stage = [&](int buf, int kt) __attribute__((always_inline)) {
    const int k0 = kt * 64;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = 4 * wid + j;
      if (aon[j])
        glds16_asm(asrc[j] + min(k0 + 8 * ar[j], T - 8), __builtin_amdgcn_readfirstlane(sbase + buf * STAGE + p * 1024));
      const int row = er[j], t = min(k0 + row, T - 1);
      glds16_asm(enc + ((size_t)b * T + t) * A + n0 + 8 * (ech ^ tt_sw(row)),
                 __builtin_amdgcn_readfirstlane(sbase + buf * STAGE + AI + p * 1024));
    }
  };
  f32x4 acc[CB_MT][2];
#pragma unroll
  for (int i = 0; i < CB_MT; ++i) acc[i][0] = acc[i][1] = f32x4{0, 0, 0, 0};
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(buf ^ 1, kt + 1);
    const char* Ai = smem + buf * STAGE;
    const char* Ei = Ai + AI;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int kb = kt * 64 + 32 * kk;
      if (kb >= T) break;  // (uniform) the K tail's empty half
      bf16x8 fb[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        fb[j] = tt_frag(Ei, 32 * kk, 32 * wid + 16 * j, lane);
        if (kb + 8 * (lane >> 4) >= T) fb[j] = zero8();  // rows past T (clamped loads)
      }
#pragma unroll
      for (int i = 0; i < CB_MT; ++i) {
        if (i < mt) {
          const bf16x8 fa = km_frag(Ai, 16 * i, kk, lane);
          acc[i][0] = mfma16(fa, fb[0], acc[i][0]);
          acc[i][1] = mfma16(fa, fb[1], acc[i][1]);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // accumulator (i, j, r): d = 16 i + 4 (l >> 4) + r, n = n0 + 32 w + 16 j + (l & 15)
  const int nl = n0 + 32 * wid + (lane & 15);
#pragma unroll
  for (int i = 0; i < CB_MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int d = 16 * i + 4 * (lane >> 4) + r;
      if (i < mt && d < D) {
        const size_t o = ((size_t)d * B + b) * A + nl;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          ctx[o + 16 * j] = acc[i][j][r];
          ctxb[o + 16 * j] = f2bf(acc[i][j][r]);
        }
      }
    }
}

// one workgroup of NW waves per (b, 32 NW t columns t0..): the dctx rows of b and the enc rows t0..
// as K-major images, K = A in steps of 64 (A % 64 == 0); wave w owns t columns t0 + 32 w .. + 31.
// NW = 8 halves the L2 re-reads of the dctx rows (one image per 256 t instead of per 128).
template <int NW>
__global__ __launch_bounds__(NW * 64) void ctx_da_kernel(const bf16* __restrict__ dctx, const bf16* __restrict__ enc,
                                                         float* __restrict__ da, int B, int T, int D, int A,
                                                         int acc_out) {
  constexpr int DI = 128 * 128, EI = 32 * NW * 128, STAGE = DI + EI, DPW = 16 / NW;  // dctx pieces per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int TT = 32 * NW, ntn = (T + TT - 1) / TT, lin = xcd_lin(), b = lin / ntn, t0 = (lin - b * ntn) * TT;
  const int mt = (D + 15) >> 4, nk = A / 64;
  const bf16* dsrc[DPW];
  const bf16* esrc[4];
  bool don[DPW], eon[4];
#pragma unroll
  for (int j = 0; j < DPW; ++j) {
    const int p = DPW * wid + j, row = 8 * p + (lane >> 3), c = (lane & 7) ^ km_sw(row);
    don[j] = 8 * p < D;
    dsrc[j] = dctx + ((size_t)min(row, D - 1) * B + b) * A + 8 * c;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = 4 * wid + j, row = 8 * p + (lane >> 3), c = (lane & 7) ^ km_sw(row);
    eon[j] = t0 + 8 * p < T;
    esrc[j] = enc + ((size_t)b * T + min(t0 + row, T - 1)) * A + 8 * c;
  }
  const unsigned sbase = lds_addr(smem);
  auto stage = [&](int buf, int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < DPW; ++j)
      if (don[j])
        glds16_asm(dsrc[j] + kt * 64, __builtin_amdgcn_readfirstlane(sbase + buf * STAGE + (DPW * wid + j) * 1024));
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (eon[j])
        glds16_asm(esrc[j] + kt * 64, __builtin_amdgcn_readfirstlane(sbase + buf * STAGE + DI + (4 * wid + j) * 1024));
  };
  const bool live = t0 + 32 * wid < T;  // (uniform) this wave has columns before T
  f32x4 acc[CB_MT][2];
#pragma unroll
  for (int i = 0; i < CB_MT; ++i) acc[i][0] = acc[i][1] = f32x4{0, 0, 0, 0};
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(buf ^ 1, kt + 1);
    const char* Di = smem + buf * STAGE;
    const char* Ei = Di + DI;
    if (live) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 fb0 = km_frag(Ei, 32 * wid, kk, lane), fb1 = km_frag(Ei, 32 * wid + 16, kk, lane);
#pragma unroll
        for (int i = 0; i < CB_MT; ++i) {
          if (i < mt) {
            const bf16x8 fa = km_frag(Di, 16 * i, kk, lane);
            acc[i][0] = mfma16(fa, fb0, acc[i][0]);
            acc[i][1] = mfma16(fa, fb1, acc[i][1]);
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int tl = t0 + 32 * wid + (lane & 15);
#pragma unroll
  for (int i = 0; i < CB_MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int d = 16 * i + 4 * (lane >> 4) + r;
      if (i < mt && d < D) {
        float* o = da + ((size_t)d * B + b) * T + tl;
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (tl + 16 * j < T) o[16 * j] = acc_out ? o[16 * j] + acc[i][j][r] : acc[i][j][r];
      }
    }
}

// one workgroup per (b, 128 t rows t0..), looping over the 128-column blocks n0 = 0, 128, .. of A:
// K = D <= 128 in one stage.  The att rows [d][t0 ..] stay in LDS as one half image for the whole
// loop; the dctx rows [d][n0 ..] of the next block are staged into the (single) dctx image while
// the current block's tile is stored -- the fp32 dE output is the traffic that matters; 64 KB of
// LDS keeps 2 workgroups per CU.  Measured (profiles/r6/ctx_bmm.md): one tile per workgroup
// 56.3 / 2128 us (headline / config #5), this loop 58.6 / 1726, the loop with a second dctx buffer
// (96 KB, 1 workgroup per CU) 71.6 / 2024.  Rows past D of the att image are zero, both operands
// are read transposed; waves 2 x 2, each 64 t x 64 n.
// deb (bf16 mode): the product stored in bf16 (the engine's bf16 encoder-output gradient, to which
// the W_h GEMM then adds dF . W_h^T with beta = 1).  An in-place bf16 accumulate here measured
// 3023 vs 1729 us at config #5 (64 two-byte reads per lane in the epilogue).
__global__ __launch_bounds__(256) void ctx_de_kernel(const bf16* __restrict__ att, const bf16* __restrict__ dctx,
                                                     float* __restrict__ de, bf16* __restrict__ deb, int B, int T,
                                                     int D, int A) {
  constexpr int IMG = 128 * 256;
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG];  // att image, dctx image
  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int ntt = (T + 127) / 128, ntn = A / 128;
  const int lin = xcd_lin(), b = lin / ntt, t0 = (lin - b * ntt) * 128;
  const unsigned sbase = lds_addr(smem);
  const int np = (D + 3) / 4;  // 4-row pieces holding rows < D
  // 32 pieces (4 rows x 256 B) per image, 8 per wave
  auto stage_dctx = [&](int n0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = 8 * wid + j, row = 4 * p + (lane >> 4), ch = (lane & 15) ^ tt_sw(row);
      if (p < np)
        glds16_asm(dctx + ((size_t)min(row, D - 1) * B + b) * A + n0 + 8 * ch,
                   __builtin_amdgcn_readfirstlane(sbase + IMG + p * 1024));
    }
  };
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int p = 8 * wid + j, row = 4 * p + (lane >> 4), ch = (lane & 15) ^ tt_sw(row);
    if (p < np)
      glds16_asm(att + ((size_t)min(row, D - 1) * B + b) * T + min(t0 + 8 * ch, T - 8),
                 __builtin_amdgcn_readfirstlane(sbase + p * 1024));
  }
  stage_dctx(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // rows D .. 127 of both images -> 0 (plain LDS stores, once).  Only the att image's must stay
  // zero: a partial last piece (D % 4) re-lands clamped copies of row D - 1 in the dctx image,
  // finite, so their products with the zero att rows are exact zeros.
  if (D < 128) {
    for (int e = tid; e < 2 * 128 * 16; e += 256) {
      const int img = e >> 11, row = (e >> 4) & 127;
      if (row >= D) *reinterpret_cast<bf16x8*>(smem + img * IMG + row * 256 + 16 * (e & 15)) = zero8();
    }
    __syncthreads();
  }
  const int wr = wid >> 1, wc = wid & 1, nkk = (D + 31) / 32;
  for (int nb = 0; nb < ntn; ++nb) {
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
    for (int kk = 0; kk < nkk; ++kk) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = tt_frag(smem, 32 * kk, 64 * wr + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = tt_frag(smem + IMG, 32 * kk, 64 * wc + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
    }
    if (nb + 1 < ntn) {  // every wave's reads of this dctx image done -> stage the next block
      __syncthreads();
      stage_dctx((nb + 1) * 128);
    }
    const int nl = nb * 128 + 64 * wc + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = t0 + 64 * wr + 16 * i + 4 * (lane >> 4) + r;
        if (t < T) {
          const size_t o = ((size_t)b * T + t) * A + nl;
          if (deb) {
#pragma unroll
            for (int j = 0; j < 4; ++j) deb[o + 16 * j] = f2bf(acc[i][j][r]);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) de[o + 16 * j] = acc[i][j][r];
          }
        }
      }
    if (nb + 1 < ntn) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next block's dctx has landed
      __syncthreads();
    }
  }
}

bool ctx_bmm_ok(int B, int T, int D, int A) {
  return B >= 1 && D >= 1 && D <= 128 && T >= 8 && T % 8 == 0 && A >= 128 && A % 128 == 0;
}

void launch_ctx_fwd(const bf16* att, const bf16* enc, float* ctx, bf16* ctxb, int B, int T, int D, int A,
                    hipStream_t st) {
  hipLaunchKernelGGL(ctx_fwd_kernel, dim3(B * (A / 128)), dim3(256), 0, st, att, enc, ctx, ctxb, B, T, D, A);
}

void launch_ctx_da(const bf16* dctx, const bf16* enc, float* da, int B, int T, int D, int A, bool acc, hipStream_t st) {
  static const int nw_env = [] {
    const char* e = getenv("TSAMD_CTX_DA_NW");
    return e ? atoi(e) : 0;
  }();
  const int nw = nw_env == 4 || nw_env == 8 ? nw_env : 8;
  const int lds = 2 * (128 * 128 + 32 * nw * 128);
  if (nw == 8) {
    (void)hipFuncSetAttribute((const void*)ctx_da_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(ctx_da_kernel<8>, dim3(B * ((T + 255) / 256)), dim3(512), lds, st, dctx, enc, da, B, T, D, A,
                       (int)acc);
  } else {
    hipLaunchKernelGGL(ctx_da_kernel<4>, dim3(B * ((T + 127) / 128)), dim3(256), lds, st, dctx, enc, da, B, T, D, A,
                       (int)acc);
  }
}

void launch_ctx_de(const bf16* att, const bf16* dctx, float* de, bf16* deb, int B, int T, int D, int A, hipStream_t st) {
  hipLaunchKernelGGL(ctx_de_kernel, dim3(B * ((T + 127) / 128)), dim3(256), 0, st, att, dctx, de, deb, B, T, D, A);
}
