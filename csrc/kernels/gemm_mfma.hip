// Hand-written MFMA GEMM for the encoder's activation GEMMs (SURVEY K4 / K2 "hoist x.W_x for all T
// as one MFMA GEMM"; reference model.py:89-93 bidirectional_dynamic_rnn input kernels,
// attention_decoder.py:64-66 W_h features):
//
//     C[m, 0:N] (+)= A[arow(m), 0:K] . Bt[0:N, 0:K]^T  (+ bias)      bf16 operands, fp32 accumulate
//
// with the A rows GATHERED in the prologue, so the layout pass that fed the library GEMM is gone:
//   AMODE 0  plain rows:  arow(m) = m
//   AMODE 1  step frame:  m = t * B + b of direction d;  tt = t (d = 0) or rev[b][t] (d = 1, the bw
//            direction reversed within each length);  arow = ids ? ids[b][tt] (embedding table
//            rows: layer 0 reads the token embeddings straight from the table) : b * T + tt
//            (the layer below's batch-frame output) -- what to_step_frame wrote and the library
//            GEMM re-read.  With xsf set the gathered rows are also stored there ([M][K], the
//            step-frame copy the weight gradient reads later): the N-tile workgroups of an M tile
//            each store an interleaved 1/ntn of its rows from the landed LDS stage.
//   AMODE 2  two-direction merge (the encoder input-gradient GEMM): K = 2 Kh, A = the BPTT's dz
//            [2][T][B][Kh] (step frame); output row m = (t, b) -- step frame t * B + b, or batch
//            frame b * T + t with dir bit 2 -- and k-half h reads dz[h] at step t, or at rev[b][t]
//            with dir bit h.  One GEMM over [dz_fw | dz_bw] . [Kx_fw ; Kx_bw] replaces the two
//            per-direction GEMMs and the from_step_frame / step_frame_hop pass that added them.
//
// Geometry (cdna_hip_programming.md s5): 256 x BN x 64 tiles, 8 waves as 2 (M) x 4 (N), each wave
// 128 x BN/4 of v_mfma_f32_16x16x32_bf16 accumulators.  Both operand tiles are staged global -> LDS
// by global_load_lds_dwordx4 (16 B per lane, lane-linear 1 KB per wave instruction; the per-lane
// GLOBAL address carries the row gather and the XOR swizzle, so LDS stays lane-linear) into two
// LDS stages: tile k + 1 is in flight while tile k is multiplied; one barrier per K step.  LDS
// image: row r's k-chunk c (8 bf16) sits in slot c ^ (r & 7) of its 128-byte row, so the 16 rows
// of one fragment read spread over 8 slots.  Epilogue through LDS: each wave's tile is written
// row-major to LDS and stored as 16-byte row runs (fp32 or bf16, + bias, beta = 1 accumulate).
// Workgroup order: the (M tiles x N tiles) grid is walked N-fastest within groups of M tiles that
// share an XCD (blockIdx % 8 = XCD under round-robin dispatch), so the N tiles of one A row block
// run on one XCD and read the block from its L2.
#include "common.h"
#include "launchers.h"

namespace {

constexpr int GM_BM = 256, GM_BK = 64, GM_THREADS = 512;

struct GemmP {
  const bf16* A;
  const bf16* Bt;
  void* C;
  const float* bias;
  const int64_t* ids;  // AMODE 1: token ids [B][T] (nullable)
  const int64_t* rev;  // AMODE 1: [B][T] reversed position of (b, t)
  bf16* xsf;           // AMODE 1, nullable: the gathered A rows [M][K]
  long lda, ldb, ldc, nsrc;
  int M, N, K, B, T, dir;
  int kchunk;    // split-K (AMODE 0, fp32 out): K columns per split (multiple of 64; K when unsplit)
  long sstride;  // split s writes its partial tile to C + s * sstride (a slab summed afterwards)
};

__device__ __forceinline__ const bf16* a_row(const GemmP& p, int m, int AMODE) {
  m = min(m, p.M - 1);
  if (AMODE == 0) return p.A + (size_t)m * p.lda;
  const int t = m / p.B, b = m - t * p.B;
  const int tt = p.dir == 0 ? t : (int)DCHECK_IDX(p.rev[(size_t)b * p.T + t], 0, p.T, CHK_FRAME_REV);
  const long src = p.ids ? DCHECK_IDX(p.ids[(size_t)b * p.T + tt], 0, p.nsrc, CHK_FRAME_ID) : (long)b * p.T + tt;
  return p.A + (size_t)src * p.lda;
}

__device__ __forceinline__ const bf16* a_row2(const GemmP& p, int m, int h) {
  m = min(m, p.M - 1);
  int t, b;
  if (p.dir & 4) {
    b = m / p.T;
    t = m - b * p.T;
  } else {
    t = m / p.B;
    b = m - t * p.B;
  }
  const int tt = (p.dir >> h) & 1 ? (int)DCHECK_IDX(p.rev[(size_t)b * p.T + t], 0, p.T, CHK_FRAME_REV) : t;
  return p.A + (((size_t)h * p.T + tt) * p.B + b) * p.lda;
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

}  // namespace

// epilogue: per wave, 32-row slabs of its 128 x WN tile through LDS -> 16-byte row runs
template <int BN, int OUT, bool BETA>
__device__ __forceinline__ void gemm_epilogue(const GemmP& p, const f32x4 (&acc)[8][BN / 64], char* smem, int m0, int n0,
                                              int wr, int wc, int wid, int lane) {
  constexpr int WN = BN / 4, NI = WN / 16;
  const int fr = lane & 15, fq = lane >> 4;
  float* ep = reinterpret_cast<float*>(smem) + wid * (32 * WN);
  constexpr int RUN = 4;                 // fp32 elements per lane store (16 bytes)
  constexpr int LPR = WN / RUN;          // lanes per row
  constexpr int RPP = 64 / LPR;          // rows per pass
  float bv[RUN];
  const int col = n0 + wc * WN + (lane % LPR) * RUN;
  constexpr int ES = OUT == 1 ? 2 : 4;  // output element bytes
  // buffer resource over this workgroup's output rows [m0, min(M, m0 + BM)): stores past M drop
  const long rows = min((long)GM_BM, (long)p.M - m0);
  const __amdgpu_buffer_rsrc_t crsrc = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char*>(p.C) + (size_t)m0 * p.ldc * ES, 0, (int)(rows * p.ldc * ES), 0x00020000);
  const int voff = (int)(((size_t)(wr * 128 + lane / LPR) * p.ldc + col) * ES);
#pragma unroll
  for (int e = 0; e < RUN; ++e) bv[e] = p.bias ? p.bias[col + e] : 0.f;
#pragma unroll
  for (int slab = 0; slab < 4; ++slab) {
    // accumulators of subtiles i = 2 slab, 2 slab + 1 -> LDS [32][WN]
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) ep[(ii * 16 + fq * 4 + rr) * WN + j * 16 + fr] = acc[2 * slab + ii][j][rr];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's slab writes done (wave-private)
    // all passes' row runs first, then buffer stores: one VGPR offset for every pass (the pass
    // and slab offsets are SGPR soffsets), distinct data registers, and rows past M dropped by
    // the resource's range check instead of branches
    float4 v[32 / RPP];
#pragma unroll
    for (int pass = 0; pass < 32 / RPP; ++pass)
      v[pass] = *reinterpret_cast<const float4*>(ep + (pass * RPP + lane / LPR) * WN + (lane % LPR) * RUN);
#pragma unroll
    for (int pass = 0; pass < 32 / RPP; ++pass) {
      const int soff = (int)(((size_t)(slab * 32 + pass * RPP) * p.ldc) * ES);
      if (BETA) {
        const auto c = __builtin_amdgcn_raw_buffer_load_b128(crsrc, voff, soff, 0);
        v[pass].x += __uint_as_float(c[0]); v[pass].y += __uint_as_float(c[1]);
        v[pass].z += __uint_as_float(c[2]); v[pass].w += __uint_as_float(c[3]);
      }
      const float o0 = v[pass].x + bv[0], o1 = v[pass].y + bv[1], o2 = v[pass].z + bv[2], o3 = v[pass].w + bv[3];
      if (OUT == 1) {
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
        const bf16x4 h{f2bf(o0), f2bf(o1), f2bf(o2), f2bf(o3)};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, h), crsrc, voff, soff, 0);
      } else {
        typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4v{__float_as_uint(o0), __float_as_uint(o1), __float_as_uint(o2), __float_as_uint(o3)}, crsrc, voff, soff, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slab read before the next slab's writes
  }
}

// BN: 256 or 128 output columns per workgroup; OUT: 0 fp32, 1 bf16; BETA: C += (fp32 only)
template <int AMODE, int BN, int OUT, bool BETA>
__global__ __launch_bounds__(GM_THREADS, 1) void gemm_bt_kernel(GemmP p) {
  constexpr int BM = GM_BM, BK = GM_BK;
  constexpr int WN = BN / 4;           // columns per wave
  constexpr int NI = WN / 16;          // 16-column subtiles per wave (4 or 2)
  constexpr int MI = 128 / 16;         // 16-row subtiles per wave
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int A_PER_WAVE = BM / 8 / 8;  // glds (8 rows each) per wave for A
  constexpr int B_PER_WAVE = BN / 8 / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 stages (and the epilogue tile)

  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int wr = wid >> 2, wc = wid & 3;
  // workgroup -> (m tile, n tile): groups of 8 consecutive ids = one id per XCD; within an XCD the
  // ids walk the N tiles of one M tile before the next M tile
  const int ntn = p.N / BN, ntm = (p.M + BM - 1) / BM;
  const int nwg = gridDim.x;  // ntn x ntm tiles x the K splits
  const int id = blockIdx.x;
  const int xcd = id & 7, per = (nwg + 7) >> 3, q = nwg >> 3, r8 = nwg & 7;
  // bijective remap (cdna_hip_programming.md s5, XCD swizzle)
  const int lin0 = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (id >> 3);
  (void)per;
  // split-K: split sk = lin0 / tiles (the tiles of one split are consecutive, so one XCD's L2
  // serves a K chunk's B panel to the M tiles it runs)
  const int sk = lin0 / (ntn * ntm), lin = lin0 - sk * (ntn * ntm);
  const int tm = lin / ntn, tn = lin - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = sk * p.kchunk;

  // per-lane source pointers of the glds pieces: piece i of this wave covers 8 rows; lane l
  // loads row (piece row0 + l / 8), k-chunk (l % 8) ^ (row & 7) of the current K tile
  const int lr = lane >> 3, lc = lane & 7;
  const bf16* asrc[A_PER_WAVE];
  const bf16* asrc1[AMODE == 2 ? A_PER_WAVE : 1];  // AMODE 2: the second k-half's rows
#pragma unroll
  for (int i = 0; i < A_PER_WAVE; ++i) {
    const int row = (wid * A_PER_WAVE + i) * 8 + lr;
    if constexpr (AMODE == 2) {
      asrc[i] = a_row2(p, m0 + row, 0) + ((lc ^ (row & 7)) * 8);
      asrc1[i] = a_row2(p, m0 + row, 1) + ((lc ^ (row & 7)) * 8);
    } else {
      asrc[i] = a_row(p, m0 + row, AMODE) + kbeg + ((lc ^ (row & 7)) * 8);
    }
  }
  const int nkh = p.K / (2 * BK);  // AMODE 2: k tiles per half
  const bf16* bsrc[B_PER_WAVE];
#pragma unroll
  for (int i = 0; i < B_PER_WAVE; ++i) {
    const int row = (wid * B_PER_WAVE + i) * 8 + lr;
    bsrc[i] = p.Bt + (size_t)(n0 + row) * p.ldb + kbeg + ((lc ^ (row & 7)) * 8);
  }
  auto stage_load = [&](int s, int kt) {
    char* base = smem + s * STAGE;
#pragma unroll
    for (int i = 0; i < A_PER_WAVE; ++i) {
      const bf16* src = (AMODE == 2 && kt >= nkh) ? asrc1[AMODE == 2 ? i : 0] + (kt - nkh) * BK : asrc[i] + kt * BK;
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(base + ((wid * A_PER_WAVE + i) * 8) * (BK * 2)), 16, 0,
                                       0);
    }
#pragma unroll
    for (int i = 0; i < B_PER_WAVE; ++i)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bsrc[i] + kt * BK),
                                       (lds_ptr_t)(base + A_BYTES + ((wid * B_PER_WAVE + i) * 8) * (BK * 2)), 16, 0, 0);
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (min(p.K, kbeg + p.kchunk) - kbeg) / BK;
  // fragment read offsets: lane reads row (l & 15) of a subtile, k-chunk kb * 4 + (l >> 4)
  const int fr = lane & 15, fq = lane >> 4;
  stage_load(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int s = kt & 1;
    if (kt + 1 < nk) stage_load(s ^ 1, kt + 1);
    const char* As = smem + s * STAGE;
    const char* Bs = As + A_BYTES;
    if (AMODE == 1 && p.xsf) {  // this workgroup's share of the landed A tile -> the step-frame copy
      const int nrows = (BM - tn + ntn - 1) / ntn;
      for (int pc = tid; pc < nrows * 8; pc += GM_THREADS) {
        const int r = (pc >> 3) * ntn + tn, c = pc & 7, m = m0 + r;
        if (m < p.M)
          *reinterpret_cast<bf16x8*>(p.xsf + (size_t)m * p.K + kt * BK + c * 8) =
              *reinterpret_cast<const bf16x8*>(As + r * (BK * 2) + ((c ^ (r & 7)) * 16));
      }
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      // every fragment of this 32-deep k block first (one LDS round trip), then its MFMAs at raised
      // priority: the other wave of the SIMD issues its reads under them
      const int chunk = kb * 4 + fq;
      bf16x8 bfrag[NI], afrag[MI];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int row = wc * WN + j * 16 + fr;
        bfrag[j] = *reinterpret_cast<const bf16x8*>(Bs + row * (BK * 2) + ((chunk ^ (row & 7)) * 16));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wr * 128 + i * 16 + fr;
        afrag[i] = *reinterpret_cast<const bf16x8*>(As + row * (BK * 2) + ((chunk ^ (row & 7)) * 16));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(afrag[i], bfrag[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  GemmP ps = p;  // split sk's partial tile: its slab
  ps.C = reinterpret_cast<char*>(p.C) + (size_t)sk * p.sstride * (OUT == 1 ? 2 : 4);
  gemm_epilogue<BN, OUT, BETA>(ps, acc, smem, m0, n0, wr, wc, wid, lane);
}

bool gemm_bt_supported(int M, int N, int K, int BN) {
  return M >= 1 && K >= 64 && K % 64 == 0 && (BN == 256 || BN == 128) && N % BN == 0;
}

size_t gemm_bt_lds(int BN) { return 2 * (size_t)(GM_BM * GM_BK * 2 + BN * GM_BK * 2); }

void launch_gemm_bt(const bf16* A, long lda, const bf16* Bt, long ldb, void* C, long ldc, bool out_bf16, bool beta,
                    const float* bias, int M, int N, int K, int amode, const int64_t* ids, const int64_t* rev,
                    bf16* xsf, long nsrc, int B, int T, int dir, hipStream_t st) {
  GemmP p{A, Bt, C, bias, ids, rev, xsf, lda, ldb, ldc, nsrc, M, N, K, B, T, dir, K, 0};
  const int BN = N % 256 == 0 ? 256 : 128;
  const int grid = ((M + GM_BM - 1) / GM_BM) * (N / BN);
  const size_t lds = gemm_bt_lds(BN);
#define GL(AM, BNN, O, BE)                                                                                    \
  do {                                                                                                        \
    auto kfn = gemm_bt_kernel<AM, BNN, O, BE>;                                                                \
    (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);      \
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(GM_THREADS), lds, st, p);                                        \
  } while (0)
#define GL_OUT(AM, BNN)                 \
  if (out_bf16) GL(AM, BNN, 1, false);  \
  else if (beta) GL(AM, BNN, 0, true);  \
  else GL(AM, BNN, 0, false);
  if (amode == 2) {  // merge: fp32 out, no beta
    if (BN == 256) GL(2, 256, 0, false);
    else GL(2, 128, 0, false);
    return;
  }
  if (amode == 0) {
    if (BN == 256) { GL_OUT(0, 256) } else { GL_OUT(0, 128) }
  } else {
    if (BN == 256) { GL_OUT(1, 256) } else { GL_OUT(1, 128) }
  }
#undef GL_OUT
#undef GL
}

// Split-K (long K, few output tiles: the vocab input gradient dX = dlogits . W, K = V): S
// splits of the K range as S x the tiles, each storing its fp32 partial tile to slab[s]
// ([S][M][N]), then the slab sum (wgrad.hip) adds the splits in order into out -- deterministic,
// no atomics.  S fills about one round of the 256 CUs (one 512-thread workgroup per CU).
int gemm_bt_splits(int M, int N, int K) {
  const int BN = N % 256 == 0 ? 256 : 128, tiles = ((M + GM_BM - 1) / GM_BM) * (N / BN), steps = K / GM_BK;
  int s = 256 / tiles;
  if (s > steps / 16) s = steps / 16;  // >= 16 K steps per split
  if (s < 2) return 1;
  const int kc = (steps + s - 1) / s;
  return (steps + kc - 1) / kc;
}

void launch_gemm_bt_splitk(const bf16* A, long lda, const bf16* Bt, long ldb, float* slab, float* out, long ldo, int M,
                           int N, int K, bool acc, hipStream_t st) {
  const int S = gemm_bt_splits(M, N, K), steps = K / GM_BK, kc = (steps + S - 1) / S;
  GemmP p{A, Bt, slab, nullptr, nullptr, nullptr, nullptr, lda, ldb, (long)N, 0, M, N, K, 0, 0, 0, kc * GM_BK,
          (long)M * N};
  const int BN = N % 256 == 0 ? 256 : 128;
  const int grid = ((M + GM_BM - 1) / GM_BM) * (N / BN) * S;
  const size_t lds = gemm_bt_lds(BN);
  if (BN == 256) {
    (void)hipFuncSetAttribute((const void*)gemm_bt_kernel<0, 256, 0, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    hipLaunchKernelGGL((gemm_bt_kernel<0, 256, 0, false>), dim3(grid), dim3(GM_THREADS), lds, st, p);
  } else {
    (void)hipFuncSetAttribute((const void*)gemm_bt_kernel<0, 128, 0, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    hipLaunchKernelGGL((gemm_bt_kernel<0, 128, 0, false>), dim3(grid), dim3(GM_THREADS), lds, st, p);
  }
  launch_slab_sum(slab, out, (int)ldo, M, N, S, acc, st);
}
