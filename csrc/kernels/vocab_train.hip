// Training vocab head without materialised logits (hard part 7.5-2;
// reference model.py:229-268, 146-183, 446-460).
//
// The library path writes the [N, V] bf16 logits (N = D*B rows: 2.56 GB at B = 256) from a
// K = 256 GEMM that is store-bound, then a loss kernel reads them back and overwrites them
// with dlogits.  Here the logits only ever exist in MFMA accumulators:
//
//   pass 1  vocab_train_kernel<false>: logits tile (32 rows x 256 columns, K = H) ->
//           per-row (max, sum exp) partial of the tile -> part[vt][row]; the tile holding a
//           row's gold id also records its logit z_w.  No [N, V] traffic at all.
//   rows    vocab_rowstats_kernel: lse = combine(partials), p_vocab(w) = exp(z_w - lse).
//           ptr_rowfin_kernel: copy mass of w, P = p_gen p_vocab + (1 - p_gen) copy,
//           loss, alpha = g p_gen p_vocab / P, dpre, dA (one wave per row).
//   pass 2  vocab_train_kernel<true>: recompute the tile, dz = alpha (exp(z - lse) - [k == w])
//           -> bf16 dlogits (the only [N, V] traffic: one write, read by the two weight /
//           input gradient GEMMs).
//
// Both passes run a persistent grid: the (vocab tile, row block) units are laid out vocab-
// tile-major and every workgroup takes one contiguous range, so a workgroup keeps one W^T
// tile's fragments in registers (128 VGPRs) across many row blocks and reloads them only at a
// tile boundary; the 32 x H row block of X is staged in LDS per unit (shared by the 4 waves).
// Each wave owns NI 16-column MFMA tiles: NI = 4 (a 256-column vocab tile) up to H = 256, NI = 2
// (128 columns) at H = 512, so the W^T fragments stay at KS x NI = 32 registers of 8 bf16 either
// way (config #5, reference model.py:229 with hidden 512).
#include "common.h"
#include "attn_common.h"  // f32x2 packed-FP32 helpers

#define VR_ROWS 32   // rows per unit (2 MFMA row tiles)

// 16-column MFMA tiles per wave and vocab columns per unit (4 waves) at hidden size H
__host__ __device__ constexpr int vr_ni(int H) { return H <= 256 ? 4 : 2; }
__host__ __device__ constexpr int vr_cols(int H) { return 64 * vr_ni(H); }
#define LOG2E_F 1.4426950408889634f
#define LN2_F 0.6931471805599453f

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ void ms_merge(float& m, float& s, float m2, float s2) {
  const float M = fmaxf(m, m2);
  if (M == -INFINITY) return;
  s = (m == -INFINITY ? 0.f : s * fexp(m - M)) + (m2 == -INFINITY ? 0.f : s2 * fexp(m2 - M));
  m = M;
}

// max / sum over the 16 lanes of one accumulator column group (one DPP row)
__device__ __forceinline__ float max16(float x) { return dpp_max16(x); }
__device__ __forceinline__ float sum16(float x) { return dpp_sum16(x); }

// 16 values per lane (index q = 4i + r) summed over the 16 lanes of a DPP row; lane l returns
// the total of value q = l & 15.  Each step sends the half of the values the partner keeps.
__device__ __forceinline__ float row_transpose_sum(float (&v)[16], int c16) {
  const bool b3 = c16 & 8, b2 = c16 & 4, b1 = c16 & 2, b0 = c16 & 1;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const float keep = b3 ? v[a + 8] : v[a], send = b3 ? v[a] : v[a + 8];
    v[a] = keep + dpp_f<DPP_MIRROR>(send);
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const float keep = b2 ? v[a + 4] : v[a], send = b2 ? v[a] : v[a + 4];
    v[a] = keep + dpp_f<DPP_HALF_MIRROR>(send);
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const float keep = b1 ? v[a + 2] : v[a], send = b1 ? v[a] : v[a + 2];
    v[a] = keep + dpp_f<DPP_XOR2>(send);
  }
  const float keep = b0 ? v[1] : v[0], send = b0 ? v[0] : v[1];
  return keep + dpp_f<DPP_XOR1>(send);
}

// 8 values per lane (q = 4i + r) summed over the 16 lanes of a DPP row: lane l returns the total
// of value q = 4 b3 + 2 b2 + b1 (bits of l & 15); lanes l and l ^ 1 return the same total.
__device__ __forceinline__ float row_transpose_sum8(float (&v)[8], int c16) {
  const bool b3 = c16 & 8, b2 = c16 & 4, b1 = c16 & 2;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const float keep = b3 ? v[a + 4] : v[a], send = b3 ? v[a] : v[a + 4];
    v[a] = keep + dpp_f<DPP_MIRROR>(send);
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const float keep = b2 ? v[a + 2] : v[a], send = b2 ? v[a] : v[a + 2];
    v[a] = keep + dpp_f<DPP_HALF_MIRROR>(send);
  }
  const float keep = b1 ? v[1] : v[0], send = b1 ? v[0] : v[1];
  const float t = keep + dpp_f<DPP_XOR2>(send);
  return t + dpp_f<DPP_XOR1>(t);
}

}  // namespace

// Operands are swapped relative to a plain logits GEMM: A = W^T fragments (16 vocab
// columns x 32 k, held in registers), B = X fragments (32 k x 16 rows, from LDS), so
// accumulator (i, j, r) holds logit[row = rb + 16j + (lane & 15)][col = cw + 16i + 4(lane>>4) + r]:
// every lane owns 16 columns of each of its rows, so a row's softmax partial is 15 in-lane
// ops + 2 cross-lane steps (the 4 lanes l, l^16, l^32, l^48), and each lane's 4 consecutive
// columns are one 8-byte bf16 store in pass 2.
//
// Per unit ONE barrier: the X rows of unit u+1 are loaded into registers before unit u's
// MFMAs and written to the other LDS buffer after its epilogue; the cross-wave (max, sum)
// merge of unit u is done by wave 0 after the barrier (double-buffered Pm/Ps).
template <int H, bool GRAD>
__global__ __launch_bounds__(256, 2) void vocab_train_kernel(
    const bf16* __restrict__ X,       // [N][ldx] output-projection activations (first H columns)
    const bf16* __restrict__ WT,      // [V][H]   output_projection/w transposed
    const float* __restrict__ bias,   // [V]
    const int* __restrict__ target,   // [N]      gold extended-vocab id
    float* __restrict__ part,         // [nt][N][2]  pass 1: per-tile (max, sum exp)
    float* __restrict__ zg,           // [N]      pass 1: gold logit (rows with w < V)
    const float* __restrict__ lse,    // [N]      pass 2
    const float* __restrict__ alpha,  // [N]      pass 2
    bf16* __restrict__ dl,            // [N][ldd] pass 2: dlogits (columns V .. ldd - 1 never written)
    float* __restrict__ dbias,        // [V]      pass 2 (nullable): += column sums of dlogits
    int N, int V, int ldx, int ldd,
    const int* __restrict__ vblk,     // nullable: the live 32-row blocks (EngineConfig.skip_pad_steps),
    const int* __restrict__ vblk_n,   // *vblk_n of them; the units enumerate only those
    int compact) {                    // pass 2: live block j's dlogits go to rows 32 j .. (compacted)
  constexpr int KS = H / 32;          // k-steps of 32
  constexpr int NI = vr_ni(H), VR_COLS = vr_cols(H);
  // LDS X row stride = 2 16-byte slots past a multiple of 256 bytes: the 16-lane groups of a
  // ds_read_b128 fragment read (lanes {0-3,12-15,20-27}, ...: rows 16 j + (lane & 15), chunk
  // 4 h + (lane >> 4)) put their 8 rows of one chunk on the even slots and the other 8 on the odd
  // ones -- the 64 banks once.  (An H + 8 pad, 1 slot, left every group 2-way conflicted: PMC
  // SQ_LDS_BANK_CONFLICT 36 % of the LDS cycles, profiles/r6/vocab_train_pmc.md)
  constexpr int XS = H + 16;
  constexpr int RJ = VR_ROWS / 16;    // 16-row MFMA tiles per unit
  constexpr int CH = VR_ROWS * H / 8 / 256;  // 16-byte X chunks per thread per unit
  static_assert(CH >= 1 && VR_ROWS * H / 8 % 256 == 0, "X staging");
  __shared__ __attribute__((aligned(16))) bf16 Xs[2][VR_ROWS * XS];
  __shared__ float Pm[2][4][VR_ROWS], Ps[2][4][VR_ROWS];
  __shared__ int Tg[2][VR_ROWS];
  __shared__ float Ls[2][VR_ROWS], Al[2][VR_ROWS];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int RB = vblk ? *vblk_n : (N + VR_ROWS - 1) / VR_ROWS, nt = (V + VR_COLS - 1) / VR_COLS;
  const long units = (long)RB * nt;
  auto row0 = [&](int u) { return (vblk ? vblk[u % RB] : u % RB) * VR_ROWS; };  // unit u's first row
  const int u0 = (int)(units * blockIdx.x / gridDim.x), u1 = (int)(units * (blockIdx.x + 1) / gridDim.x);
  if (u0 >= u1) return;
  const int kof = 8 * (lane >> 4), c16 = lane & 15, q4 = 4 * (lane >> 4);
  bf16x8 wa[KS][NI];  // A fragments: W^T rows (vocab columns) of this wave's NI column tiles
  f32x2 bc2[NI][2];   // log2(e) x bias of the lane's columns cw + 16i + q4 + r, pairs (r = 2h, 2h + 1)
                      // (-inf past V in pass 1)
  int cur_vt = -1;
  // pass 2: the output-projection bias gradient db = sum_rows dlogits.  Per unit the lane's
  // 4 NI column partials (its 2 rows) are folded across the 16 lanes that share those columns
  // by a halving butterfly (8 + 4 + 2 + 1 DPP exchanges), which leaves lane l with the full
  // column sum for column index c16 = l & 15 (NI = 2: q = c16 >> 1, lane pairs agree) -- ONE
  // accumulator register per lane, carried over the workgroup's units of a vocab tile and
  // flushed with one atomic per column when the tile changes (a 16-register accumulator
  // spilled at 256 VGPRs).
  float cacc = 0.f;
  auto flush_bias = [&](int vt_old) {
    const int q = NI == 4 ? c16 : c16 >> 1;
    const int col = vt_old * VR_COLS + 16 * NI * wid + 16 * (q >> 2) + q4 + (q & 3);
    if (col < V && (NI == 4 || !(c16 & 1))) atomicAdd(dbias + col, cacc);
    cacc = 0.f;
  };
  bf16x8 xr[CH];      // prefetched X chunks of the next unit
  int tg_r = 0;
  float ls_r = 0.f, al_r = 0.f;
  auto fetch = [&](int u) {  // global -> registers (unit u's X rows, targets, row scalars)
    const int rb = row0(u);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = c * 256 + threadIdx.x, rr = idx / (H / 8), k8 = (idx % (H / 8)) * 8;
      xr[c] = ld8(X + (size_t)min(rb + rr, N - 1) * ldx + k8);
    }
    if (threadIdx.x < VR_ROWS) {
      const int row = min(rb + threadIdx.x, N - 1);
      tg_r = target[row];
      if (GRAD) {
        ls_r = lse[row];
        al_r = alpha[row];
      }
    }
  };
  auto stash = [&](int buf) {  // registers -> LDS buffer
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = c * 256 + threadIdx.x, rr = idx / (H / 8), k8 = (idx % (H / 8)) * 8;
      *reinterpret_cast<bf16x8*>(&Xs[buf][rr * XS + k8]) = xr[c];
    }
    if (threadIdx.x < VR_ROWS) {
      Tg[buf][threadIdx.x] = tg_r;
      if (GRAD) {
        Ls[buf][threadIdx.x] = ls_r;
        Al[buf][threadIdx.x] = al_r;
      }
    }
  };
  auto merge_store = [&](int buf, int u) {  // pass 1: cross-wave (max, sum) of unit u -> part
    const int vt = u / RB, rb = row0(u);
    if (wid == 0 && lane < VR_ROWS && rb + lane < N) {
      float m = Pm[buf][0][lane], sm = Ps[buf][0][lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) ms_merge(m, sm, Pm[buf][w][lane], Ps[buf][w][lane]);
      *reinterpret_cast<float2*>(part + ((size_t)vt * N + rb + lane) * 2) = make_float2(m, sm);
    }
  };
  fetch(u0);
  stash(0);
  __syncthreads();
  for (int u = u0; u < u1; ++u) {
    const int buf = (u - u0) & 1;
    const int vt = u / RB, rb = row0(u);
    const int cw = vt * VR_COLS + 16 * NI * wid;  // this wave's first column
    if (vt != cur_vt) {  // new vocab tile: its A fragments and bias into registers
      if (GRAD && dbias && cur_vt >= 0) flush_bias(cur_vt);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const bf16* arow = WT + (size_t)min(cw + 16 * i + c16, V - 1) * H + kof;
#pragma unroll
        for (int h = 0; h < KS; ++h) wa[h][i] = ld8(arow + 32 * h);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int col = cw + 16 * i + q4 + r;
          const float b = col < V ? bias[col] * LOG2E_F : (GRAD ? 0.f : -INFINITY);
          if (r & 1) bc2[i][r >> 1].y = b;
          else bc2[i][r >> 1].x = b;
        }
      }
      cur_vt = vt;
    }
    if (u + 1 < u1) fetch(u + 1);
    f32x4 acc[NI][RJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < RJ; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int h = 0; h < KS; ++h)
#pragma unroll
      for (int j = 0; j < RJ; ++j) {
        const bf16x8 xb = *reinterpret_cast<const bf16x8*>(&Xs[buf][(16 * j + c16) * XS + 32 * h + kof]);
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i][j] = mfma16(wa[h][i], xb, acc[i][j]);
      }
    if constexpr (!GRAD) {
#pragma unroll
      for (int j = 0; j < RJ; ++j) {
        const int rr = 16 * j + c16, row = rb + rr;
        const int wo = Tg[buf][rr] - cw - q4;  // gold column relative to the lane's first one
        // y = log2(e) x logit (base-2 domain: one packed FMA per element pair, exp2 without a
        // multiply); -inf for columns >= V
        f32x2 y[NI][2];
        float m = -INFINITY;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            y[i][h] = fma2(f32x2{acc[i][j][2 * h], acc[i][j][2 * h + 1]}, splat2(LOG2E_F), bc2[i][h]);
            m = vmax3(m, y[i][h].x, y[i][h].y);
          }
        // the gold logit: at most one of the row's columns lies among the lane's 16
        // (offsets 16i + r), so the selection runs only on the rare hit
        if ((unsigned)wo < 16u * NI && (wo & 12) == 0 && row < N) {
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (wo == 16 * i + r) zg[row] = (r & 1 ? y[i][r >> 1].y : y[i][r >> 1].x) * LN2_F;
        }
        m = max_x32(max_x16(m));
        f32x2 s2 = splat2(0.f);
        if (m > -INFINITY) {
          const f32x2 mm = splat2(m);
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const f32x2 t = y[i][h] - mm;
              s2 += f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
            }
        }
        const float sm = sum_x32(sum_x16(s2.x + s2.y));
        if (lane < 16) {
          Pm[buf][wid][rr] = m * LN2_F;  // natural-log domain for the partial
          Ps[buf][wid][rr] = sm;
        }
      }
    } else {
      const bool full = (V % 4 == 0) && cw + 16 * NI <= V;  // wave-uniform: no column guards
      f32x2 cs[NI][2];  // this unit's column partials, index (i, r / 2)
#pragma unroll
      for (int i = 0; i < NI; ++i) cs[i][0] = cs[i][1] = splat2(0.f);
#pragma unroll
      for (int j = 0; j < RJ; ++j) {
        const int rr = 16 * j + c16, row = rb + rr;
        const int wo = Tg[buf][rr] - cw - q4;
        const float al = Al[buf][rr];
        // alpha exp(z - lse) = exp2(log2(e) z + log2(alpha) - log2(e) lse)   (alpha >= 0)
        const float c = al > 0.f ? __log2f(al) - Ls[buf][rr] * LOG2E_F : -INFINITY;
        if (row < N) {
          f32x2 d[NI][2];
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const f32x2 t = fma2(f32x2{acc[i][j][2 * h], acc[i][j][2 * h + 1]}, splat2(LOG2E_F), bc2[i][h] + c);
              d[i][h] = f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
            }
          // - alpha at the gold column (rare: see pass 1)
          if ((unsigned)wo < 16u * NI && (wo & 12) == 0) {
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (wo == 16 * i + r) {
                  if (r & 1) d[i][r >> 1].y -= al;
                  else d[i][r >> 1].x -= al;
                }
          }
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            cs[i][0] += d[i][0];
            cs[i][1] += d[i][1];
          }
          bf16* dst = dl + (size_t)(compact ? (u % RB) * VR_ROWS + rr : row) * ldd + cw + q4;
          if (full) {
            // (plain stores: the 4 stores of a row's 128-byte line are merged in L2; non-temporal
            // stores went to HBM as 32-byte pieces, 1.31 -> 1.75 ms)
#pragma unroll
            for (int i = 0; i < NI; ++i)
              *reinterpret_cast<bf16x4*>(dst + 16 * i) =
                  bf16x4{f2bf(d[i][0].x), f2bf(d[i][0].y), f2bf(d[i][1].x), f2bf(d[i][1].y)};
          } else {
#pragma unroll
            for (int i = 0; i < NI; ++i) {
              const int col = cw + 16 * i + q4;
              const float dv[4] = {d[i][0].x, d[i][0].y, d[i][1].x, d[i][1].y};
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (col + r < V) dst[16 * i + r] = f2bf(dv[r]);
            }
          }
        }
      }
      if (dbias) {
        float cv[4 * NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          cv[4 * i] = cs[i][0].x;
          cv[4 * i + 1] = cs[i][0].y;
          cv[4 * i + 2] = cs[i][1].x;
          cv[4 * i + 3] = cs[i][1].y;
        }
        if constexpr (NI == 4) cacc += row_transpose_sum(cv, c16);
        else cacc += row_transpose_sum8(cv, c16);
      }
    }
    if (u + 1 < u1) stash(buf ^ 1);
    __syncthreads();
    if constexpr (!GRAD) merge_store(buf, u);
  }
  if (GRAD && dbias) flush_bias(cur_vt);
}

// Rows past their last live decoder step are not enumerated by pass 2, so their dlogits keep what
// an earlier batch wrote there.  Before pass 2, a 32-row block that is dead now but was written by
// the previous pass 2 (state[b]) is zeroed -- the gradient GEMMs read every row -- and state[]
// becomes this batch's liveness.  Consecutive batches have similar length profiles (rows sorted
// by live steps), so few blocks change.
__global__ __launch_bounds__(256) void vocab_zero_dead_kernel(bf16* __restrict__ dl, const int* __restrict__ vlive,
                                                              int* __restrict__ state, int N, int ldd) {
  const int b = blockIdx.x;
  const int live = vlive[b];
  if (!live && state[b]) {
    const size_t r0 = (size_t)b * VR_ROWS, r1 = min((size_t)N, r0 + VR_ROWS);
    bf16* p = dl + r0 * ldd;
    const size_t n = (r1 - r0) * (size_t)ldd;
    const size_t head = (16 - ((uintptr_t)p & 15)) & 15;  // bytes to 16-byte alignment
    const size_t h = min(n, head / 2);
    for (size_t i = threadIdx.x; i < h; i += 256) p[i] = f2bf(0.f);
    typedef uint32_t u32x4z __attribute__((ext_vector_type(4)));
    u32x4z* q = reinterpret_cast<u32x4z*>(p + h);
    const size_t nv = (n - h) / 8;
    for (size_t i = threadIdx.x; i < nv; i += 256) q[i] = u32x4z{0, 0, 0, 0};
    for (size_t i = h + nv * 8 + threadIdx.x; i < n; i += 256) p[i] = f2bf(0.f);
  }
  if (threadIdx.x == 0) state[b] = live;
}

// lse and p_vocab(gold) per row: 32 rows x 8 tile slices per workgroup (slice j merges the
// row's partials of tiles j, j + 8, ...: each warp-wide load is 32 consecutive rows' float2,
// coalesced), the 8 slice partials merged through LDS.  N/32 workgroups instead of N/256 with a
// 196-long serial merge per thread (74 -> ~10 us at N = 25600).
__global__ __launch_bounds__(256) void vocab_rowstats_kernel(const float* __restrict__ part, const float* __restrict__ zg,
                                                             const int* __restrict__ target, float* __restrict__ lse,
                                                             float* __restrict__ pv, int N, int V, int nt) {
  __shared__ float sm_m[8][32], sm_s[8][32];
  const int rl = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int n = blockIdx.x * 32 + rl;
  float m = -INFINITY, s = 0.f;
  if (n < N)
    for (int vt = sl; vt < nt; vt += 8) {
      const float2 p = *reinterpret_cast<const float2*>(part + ((size_t)vt * N + n) * 2);
      ms_merge(m, s, p.x, p.y);
    }
  sm_m[sl][rl] = m;
  sm_s[sl][rl] = s;
  __syncthreads();
  if (sl == 0 && n < N) {
#pragma unroll
    for (int j = 1; j < 8; ++j) ms_merge(m, s, sm_m[j][rl], sm_s[j][rl]);
    const float L = m + __logf(s);
    lse[n] = L;
    const int w = target[n];
    pv[n] = w < V ? fexp(zg[n] - L) : 0.f;
  }
}

// Pointer mixture per row (one wave per row): copy mass of the gold id, P, loss, the
// dlogits scale alpha, dpre (p_gen pre-sigmoid) and dA (attention), as ptr_loss.
__global__ __launch_bounds__(256) void ptr_rowfin_kernel(
    const float* __restrict__ pv_in, const int* __restrict__ target, const float* __restrict__ rowg,
    const float* __restrict__ pgen, const float* __restrict__ attn, const int* __restrict__ ext,
    const int* __restrict__ lens, float* __restrict__ loss_row, float* __restrict__ alpha, float* __restrict__ dpre,
    float* __restrict__ dA, int N, int B, int T) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  const int b = n % B, w = target[n], len = (int)DCHECK_IDX(lens[b], 0, T + 1, CHK_LOSS_LEN);
  const float g = rowg[n], pv = pv_in[n];
  const float pg = pgen ? pgen[n] : 1.0f;
  const int* er = ext + (size_t)b * T;
  float cm = 0.f;
  if (pgen) {
    const float* ar = attn + (size_t)n * T;
    for (int i = lane; i < len; i += 64) cm += er[i] == w ? ar[i] : 0.f;
    cm = wave_sum(cm);
  }
  const float P = pg * pv + (1.0f - pg) * cm;
  const float invP = 1.0f / P;
  if (lane == 0) {
    loss_row[n] = g != 0.f ? -__logf(P) : 0.f;
    if (alpha) alpha[n] = g != 0.f ? g * pg * pv * invP : 0.f;
    if (pgen && dpre) dpre[n] = g != 0.f ? -g * (pv - cm) * invP * pg * (1.0f - pg) : 0.f;
  }
  if (pgen && dA) {
    const float coef = g != 0.f ? -g * (1.0f - pg) * invP : 0.f;
    float* dar = dA + (size_t)n * T;
    for (int i = lane; i < T; i += 64) dar[i] = (i < len && er[i] == w) ? coef : 0.f;
  }
}

int vocab_train_tiles(int V, int H) { return (V + vr_cols(H) - 1) / vr_cols(H); }

// 2 workgroups per CU (<= 256 VGPRs, ~36 KB LDS each at H = 256, ~67 KB at H = 512): 512
// persistent workgroups
static int vocab_train_grid(int N, int V, int H) {
  const long units = (long)((N + VR_ROWS - 1) / VR_ROWS) * vocab_train_tiles(V, H);
  return (int)(units < 512 ? units : 512);
}

void launch_vocab_train_fwd(const bf16* X, int ldx, const bf16* WT, const float* bias, const int* target, float* part,
                            float* zg, float* lse, float* pv, int N, int V, int H, const int* vblk, const int* vblk_n,
                            hipStream_t st) {
  const int grid = vocab_train_grid(N, V, H);
#define VF(HH) hipLaunchKernelGGL((vocab_train_kernel<HH, false>), dim3(grid), dim3(256), 0, st, X, WT, bias, target, \
                                  part, zg, nullptr, nullptr, nullptr, nullptr, N, V, ldx, V, vblk, vblk_n, 0)
  if (H == 512) VF(512);
  else if (H == 256) VF(256);
  else VF(128);
#undef VF
  hipLaunchKernelGGL(vocab_rowstats_kernel, dim3((N + 31) / 32), dim3(256), 0, st, part, zg, target, lse, pv, N, V,
                     vocab_train_tiles(V, H));
}

void launch_vocab_train_bwd(const bf16* X, int ldx, const bf16* WT, const float* bias, const int* target,
                            const float* lse, const float* alpha, bf16* dl, int ldd, float* dbias, int N, int V, int H,
                            const int* vblk, const int* vblk_n, const int* vlive, int* vstate, hipStream_t st) {
  const int grid = vocab_train_grid(N, V, H);
  // with the live-block list: either the dead blocks an earlier pass wrote are zeroed (vlive /
  // vstate; dlogits in place) or, without them, the live blocks' rows are written compacted
  const int compact = vblk && !vlive;
  if (vblk && vlive)
    hipLaunchKernelGGL(vocab_zero_dead_kernel, dim3((N + VR_ROWS - 1) / VR_ROWS), dim3(256), 0, st, dl, vlive, vstate,
                       N, ldd);
#define VB(HH) hipLaunchKernelGGL((vocab_train_kernel<HH, true>), dim3(grid), dim3(256), 0, st, X, WT, bias, target, \
                                  nullptr, nullptr, lse, alpha, dl, dbias, N, V, ldx, ldd, vblk, vblk_n, compact)
  if (H == 512) VB(512);
  else if (H == 256) VB(256);
  else VB(128);
#undef VB
}

void launch_ptr_rowfin(const float* pv, const int* target, const float* rowg, const float* pgen, const float* attn,
                       const int* ext, const int* lens, float* loss_row, float* alpha, float* dpre, float* dA, int N,
                       int B, int T, hipStream_t st) {
  hipLaunchKernelGGL(ptr_rowfin_kernel, dim3((N + 3) / 4), dim3(256), 0, st, pv, target, rowg, pgen, attn, ext, lens,
                     loss_row, alpha, dpre, dA, N, B, T);
}
