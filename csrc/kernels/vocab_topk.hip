// Decode vocab head for the device beam search (reference
// model.py:229-243, 146-183, 280-285).
//
//   vocab_logits_kernel grid (ceil(R/64), ceil(V/256)), 4 waves: a 64-row x 256-column tile of
//                       logits = X . W_out + b by MFMA (K = H), stored fp32 straight from the
//                       accumulators, plus the tile's per-row (max, sum exp) partials;
//   vocab_select_kernel grid R: log-sum-exp from the partials; the K tiles with the largest
//                       maxima hold the row's plain top-K, so only those K x 256 logits are
//                       read (x >= tau = K-th largest tile max); then the pointer copy mass
//                       (LDS hash) and the exact top-K of the extended-vocab final
//                       distribution (same argument as final_topk in beam.hip: plain top-K
//                       union copied ids).
// Replaces a library GEMM + a separate per-element top-k pass over the logits.
#include "common.h"
#include <stdlib.h>
#include <type_traits>
#include "attn_common.h"  // f32x2 packed-FP32 helpers
#include "beam_common.h"  // beam bookkeeping fused into the select kernel's tail
#include "launchers.h"

#define VT_ROWS 64    // rows per workgroup half
#define VT_K 8        // max K (= 2 * beam, beam <= 4)
#define VM_CAND 4096  // tile maxima (nt <= 4096), then <= K * 256 survivors + copied ids
#define VM_HASH 2048

// vocab columns per workgroup: 4 MFMA column tiles per wave up to hidden 256, 2 at hidden 512
// (the wave's W^T fragments stay at 32 registers of 8 bf16: H/32 k-steps x NI tiles)
__host__ __device__ constexpr int vt_ni(int HMAX) { return HMAX <= 256 ? 4 : 2; }
__host__ __device__ constexpr int vt_cols(int HMAX) { return 64 * vt_ni(HMAX); }

namespace {

__device__ __forceinline__ bool vbetter(float v1, int i1, float v2, int i2) {
  return v1 > v2 || (v1 == v2 && i1 < i2);
}

__device__ __forceinline__ void ms_combine(float& m, float& s, float m2, float s2) {
  const float M = fmaxf(m, m2);
  if (M == -INFINITY) return;
  s = (m == -INFINITY ? 0.f : s * fexp(m - M)) + (m2 == -INFINITY ? 0.f : s2 * fexp(m2 - M));
  m = M;
}

}  // namespace

// vocab_logits epilogue for one wave and one 16-row tile jr.  Operands are swapped relative
// to a plain logits GEMM (A = W^T fragments, B = X rows, as in vocab_train.hip), so
// accumulator (i, jr, r) holds logit[row = rb + 16 jr + (lane & 15)][col = cw + 16 i + 4 q + r],
// q = lane >> 4: every lane owns 16 columns of one row.  The row's (max, sum exp) over the
// wave's 64 columns is 15 in-lane ops + 2 cross-lane steps (lanes l, l^16, l^32, l^48), and the
// lane's 4 consecutive columns per i are one 16-byte store (a row's 64 columns = one 256-byte
// run over the 4 i and 4 q).  Replaced a [row = lane group] layout whose per-row reductions
// took 16-lane DPP trees for each of the lane's 16 rows and an LDS staging pass for stores.
template <bool FULL, int NI, bool NTS = false>
__device__ __forceinline__ void vl_epilogue(const f32x4 (&acc)[NI][4], int jr, const f32x2 (&bc)[NI][2],
                                            float* __restrict__ logits, float* Pm, float* Ps, int rb, int cw,
                                            int lane, int R, int V) {
  constexpr float L2E = 1.4426950408889634f;
  const int row = rb + 16 * jr + (lane & 15), q4 = 4 * (lane >> 4);
  f32x2 x[NI][2];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      x[i][h] = f32x2{acc[i][jr][2 * h], acc[i][jr][2 * h + 1]} + bc[i][h];  // bc = -inf past V
      m = vmax3(m, x[i][h].x, x[i][h].y);
    }
  m = max_x32(max_x16(m));
  f32x2 s2 = f32x2{0.f, 0.f};
  if (FULL || m > -INFINITY) {
    const f32x2 mb = f32x2{-m * L2E, -m * L2E};
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x2 t = __builtin_elementwise_fma(x[i][h], f32x2{L2E, L2E}, mb);
        s2 += f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};  // exp(-inf) = 0
      }
  }
  const float sm = sum_x32(sum_x16(s2.x + s2.y));
  if (lane < 16) {
    Pm[16 * jr + lane] = m;
    Ps[16 * jr + lane] = sm;
  }
  if (FULL) {
    float* dst = logits + (size_t)row * V + cw + q4;
#pragma unroll
    for (int i = 0; i < NI; ++i)
      if constexpr (NTS)
        __builtin_nontemporal_store(f32x4{x[i][0].x, x[i][0].y, x[i][1].x, x[i][1].y},
                                    reinterpret_cast<f32x4*>(dst + 16 * i));
      else
        *reinterpret_cast<float4*>(dst + 16 * i) = make_float4(x[i][0].x, x[i][0].y, x[i][1].x, x[i][1].y);
  } else if (row < R) {
    float* dst = logits + (size_t)row * V;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int col = cw + 16 * i + q4;
      const float xv[4] = {x[i][0].x, x[i][0].y, x[i][1].x, x[i][1].y};
      if ((V & 3) == 0 && col + 4 <= V) {
        *reinterpret_cast<float4*>(dst + col) = make_float4(xv[0], xv[1], xv[2], xv[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (col + e < V) dst[col + e] = xv[e];
      }
    }
  }
}

// 35 KB (RH = 1) / 70 KB (RH = 2) of LDS, 2 workgroups per CU (<= 256 VGPRs): all 32 W^T fragments
// of a wave in flight at once.  (A 4-per-CU variant, 128
// VGPRs, measured the same before this layout and spills with it.)
// RH = 2: 128 rows per workgroup, the W^T fragments reused for two 64-row halves (half the
// workgroups and W^T fetches: 392 tiles at R = 256 = one round), X tile 68 KB of LDS.
// HFIX: H == HMAX, known at compile time (the X-staging row / chunk split by H / 8 is then a
// shift instead of an integer division per 16-byte chunk)
// NTS: the logits stores are non-temporal -- the select kernel re-reads only the K best tiles
// and the copied words of each row, so 51 MB per step (R = 256) need not displace L2 lines:
// 25.1 -> 23.6 us, decode 6092-6102 -> 6143-6155 summaries/s (profiles/r4/ab/decode_logits_nt.md)
template <int OCC, int RH, int HMAX, bool HFIX = false, bool NTS = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void vocab_logits_kernel(
    const bf16* __restrict__ X,     // [R][H]  output-projection activations (bf16)
    const bf16* __restrict__ WT,    // [V][H]  output_projection/w transposed ("Bt")
    const float* __restrict__ bias, // [V]
    float* __restrict__ logits,     // [R][V]  fp32 (bias added)
    float* __restrict__ part_ms,    // [R][nt][2]  per tile (max, sum exp)
    int R, int V, int Hrt) {
  const int H = HFIX ? HMAX : Hrt;
  constexpr int BR = VT_ROWS * RH;  // rows per block
  constexpr int NI = vt_ni(HMAX), VT_COLS = vt_cols(HMAX), KS = HMAX / 32;
  __shared__ float Pm[4][BR], Ps[4][BR];
  __shared__ __attribute__((aligned(16))) bf16 Xs[BR * (HMAX + 8)];  // X tile of the block
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // XCD-aware order: the RB row blocks of one vocab tile get block ids equal mod 8 (one XCD
  // under round-robin dealing), so the tile's W^T columns come from HBM once and are then
  // served from that XCD's L2 to the other row blocks
  const int RB = (R + BR - 1) / BR, nt = (V + VT_COLS - 1) / VT_COLS;
  const int slot = blockIdx.x >> 3, vt = (slot / RB) * 8 + (blockIdx.x & 7);
  if (vt >= nt) return;
  const int rb = (slot % RB) * BR;
  const int cw = vt * VT_COLS + 16 * NI * wid;  // this wave's first column
  // X rows of this block -> LDS once (shared by the 4 waves)
  const int kof = 8 * (lane >> 4), c16 = lane & 15, q4 = 4 * (lane >> 4);
  constexpr int XPT = BR * HMAX / 8 / 256;  // 16-byte X chunks per thread (H <= HMAX)
  bf16x8 xr[XPT];
#pragma unroll
  for (int u = 0; u < XPT; ++u) {
    const int c = threadIdx.x + 256 * u, rr = c / (H / 8), k8 = (c % (H / 8)) * 8;
    if (c < BR * (H / 8)) xr[u] = ld8(X + (size_t)min(rb + rr, R - 1) * H + k8);
  }
  // every A fragment of the wave (W^T rows = its 4 x 16 vocab columns, H/32 k-steps, H <= 256:
  // 128 VGPRs) is issued right behind the X loads, before their LDS stores: one memory round
  // trip for both
  const bf16* arow[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) arow[i] = WT + (size_t)min(cw + 16 * i + c16, V - 1) * H + kof;
  bf16x8 wa[KS][NI];
#pragma unroll
  for (int h = 0; h < KS; ++h)
#pragma unroll
    for (int i = 0; i < NI; ++i) wa[h][i] = ld8(arow[i] + min(32 * h, H - 32));
  // bias of the lane's columns cw + 16 i + q4 + r, pairs (r = 2h, 2h + 1); -inf past V
  f32x2 bc[NI][2];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int col = cw + 16 * i + q4 + 2 * h;
      bc[i][h] = f32x2{col < V ? bias[col] : -INFINITY, col + 1 < V ? bias[col + 1] : -INFINITY};
    }
#pragma unroll
  for (int u = 0; u < XPT; ++u) {
    const int c = threadIdx.x + 256 * u, rr = c / (H / 8), k8 = (c % (H / 8)) * 8;
    if (c < BR * (H / 8)) *reinterpret_cast<bf16x8*>(&Xs[rr * (H + 8) + k8]) = xr[u];
  }
  __syncthreads();
#pragma unroll
  for (int h2 = 0; h2 < RH; ++h2) {
    const int rbh = rb + VT_ROWS * h2;
    f32x4 acc[NI][4];  // [vocab column tile i][row tile jr]
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int jr = 0; jr < 4; ++jr) acc[i][jr] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int h = 0; h < KS; ++h) {
      if (32 * h < H) {
#pragma unroll
        for (int jr = 0; jr < 4; ++jr) {
          const bf16x8 xb =
              *reinterpret_cast<const bf16x8*>(&Xs[(VT_ROWS * h2 + 16 * jr + c16) * (H + 8) + 32 * h + kof]);
#pragma unroll
          for (int i = 0; i < NI; ++i) acc[i][jr] = mfma16(wa[h][i], xb, acc[i][jr]);
        }
      }
    }
    // ---- epilogue: + bias, store fp32, per-row (max, sum exp) over this wave's 64 columns.
    // FULL (every tile but the last vocab tile / row block): no column or row guards.
    const bool full = (vt + 1) * VT_COLS <= V && rbh + VT_ROWS <= R && (V & 3) == 0;
#pragma unroll
    for (int jr = 0; jr < 4; ++jr) {
      if (full)
        vl_epilogue<true, NI, NTS>(acc, jr, bc, logits, Pm[wid] + VT_ROWS * h2, Ps[wid] + VT_ROWS * h2, rbh, cw, lane, R, V);
      else
        vl_epilogue<false, NI>(acc, jr, bc, logits, Pm[wid] + VT_ROWS * h2, Ps[wid] + VT_ROWS * h2, rbh, cw, lane, R, V);
    }
  }
  __syncthreads();
  for (int rr = threadIdx.x; rr < BR; rr += 256) {
    const int row = rb + rr;
    float m = Pm[0][rr], sm = Ps[0][rr];
#pragma unroll
    for (int w = 1; w < 4; ++w) ms_combine(m, sm, Pm[w][rr], Ps[w][rr]);
    if (row < R) {
      part_ms[((size_t)row * nt + vt) * 2] = m;
      part_ms[((size_t)row * nt + vt) * 2 + 1] = sm;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Column-span logits kernel (H = 128 / 256 / 512): every W^T byte is fetched by ONE wave.
//
// The tile kernel above re-reads W^T once per row block and X once per workgroup: at R = 256,
// V = 50k, H = 256 that is 392 x (128 KB of W^T + 64 KB of X) = 75 MB pulled into the CUs for
// 25.6 MB of unique data, ~384 KB per CU.  A prologue burst of every CU sustains ~11 B/cycle/CU
// (MI355X_MICROARCH.md, "prologue HBM burst"), so the fetch alone is ~15 us of its 20.8 us
// no-store time (profiles/r6/decode_vocab_span.md).
//
// Here the grid is one workgroup per CU (G = 256 for V = 50k), 8 waves, and wave q of the grid
// owns the 16-column tiles [q nt16 / NW, (q + 1) nt16 / NW) (1 or 2 tiles; NW = 8 G): it holds
// their W^T fragments in registers for the whole launch and multiplies them against ALL rows of
// X, which the workgroup stages into LDS once (R x H bf16: 128 KB at R = 256, H = 256; rows
// beyond what fits run as further chunks).  Per CU that is ~100 KB of W^T (HBM) + 128 KB of X
// (L2): 58 MB chip-wide instead of 75 MB, with the W^T part read exactly once.
//
// LDS image of X: row r's 16-byte chunk c sits at chunk slot c ^ (r & 15) of its 2H-byte row (no
// padding, glds-fillable): the B-fragment read (rows 16 jr + (l & 15), chunk 4 h + (l >> 4)) hits
// 16 distinct 16-byte bank slots in each of ds_read_b128's four 16-lane groups.
//
// Same MFMA sequence as the tile kernel (acc from zero, k-steps ascending, + bias): the logits are
// bit-identical to it.  Partials: one (max, sum exp) per (row, wave), laid out [G][R][8] so a
// workgroup's 8 waves write 64 contiguous bytes per row; the select kernel maps partial q back
// to its column span (vp_span).
#define VP_WAVES 8
#define VP_THREADS (64 * VP_WAVES)
#define VP_NI 2                 // 16-column tiles per wave, at most
#define VP_LDS (150 * 1024)     // X chunk + per-wave row partials (RB + 64 bytes per row)
// rows per X chunk: a multiple of the sub-chunk rows within VP_LDS
__host__ __device__ constexpr int vp_subr(int H) { return H >= 512 ? 32 : 64; }
__host__ __device__ constexpr int vp_rows(int H) { return VP_LDS / (2 * H + 8 * VP_WAVES) / vp_subr(H) * vp_subr(H); }
__host__ __device__ inline int vp_xrows(int H, int R) { return min(vp_rows(H), (R + vp_subr(H) - 1) / vp_subr(H) * vp_subr(H)); }
#define VP_CUS 256

__host__ __device__ inline int vp_groups(int V) {
  const int nt16 = (V + 15) / 16;
  const int g = nt16 > VP_CUS * VP_WAVES * VP_NI ? (nt16 + VP_WAVES * VP_NI - 1) / (VP_WAVES * VP_NI) : VP_CUS;
  return min(g, (nt16 + VP_WAVES - 1) / VP_WAVES);
}
__host__ __device__ inline bool vp_supported(int H) { return H == 128 || H == 256 || H == 512; }
// TSAMD_VL_TILE=1: the tile kernel above (A/B switch)
static inline bool vp_use(int H) {
  static const bool tile = getenv("TSAMD_VL_TILE") && getenv("TSAMD_VL_TILE")[0] == '1';
  return vp_supported(H) && !tile;
}
// first 16-column tile of partial q (q in [0, NW]; NW = 8 * vp_groups(V))
__device__ __forceinline__ int vp_lo(int q, int nt16, int NW) { return (int)(((long)q * nt16) / NW); }

// s_barrier with release / acquire fences on LDS only: the workgroup-wide __syncthreads fence
// also waits for every global load and store in flight (vmcnt(0)), which would end the overlap
// of the X staging and the logits stores with the MFMAs
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// PROBE (attribution builds only, vocab_span_probe): bit 0 no logits stores, bit 1 no epilogue
// math (partials from the raw row max), bit 2 no MFMAs (loads + epilogue only)
//
// Pipeline: X is staged in sub-chunks of SUBR rows through registers (global_load_dwordx4 ->
// ds_write_b128), VP_LOOK sub-chunks ahead of the one being multiplied, so the compiler counts
// every wait exactly (loads, stores and the staging are all visible to it; an LDS-DMA fill is
// not counted by it and turns the wait for the W^T registers into vmcnt(0)); each CU starts its
// 1 KB pieces at a different offset; the epilogue of a group runs its row tiles side by side
// (max, cross-lane steps, exp sums, stores), not one dependent chain per tile.
#define VP_LOOK 2
template <int H, int PROBE = 0>
__global__ __launch_bounds__(VP_THREADS, 1) void vocab_logits_span_kernel(
    const bf16* __restrict__ X, const bf16* __restrict__ WT, const float* __restrict__ bias,
    float* __restrict__ logits, float* __restrict__ part_ms, int R, int V) {
  constexpr float L2E = 1.4426950408889634f;
  constexpr int KS = H / 32, RB = 2 * H;             // k-steps, LDS row bytes
  constexpr int SUBR = vp_subr(H), NJ = SUBR / 16;
  constexpr int RS = vp_rows(H);                     // rows per X chunk
  constexpr int PS = SUBR * RB / 1024;               // 1 KB pieces per sub-chunk (a multiple of 8)
  constexpr int PPW = PS / VP_WAVES;                 // pieces per wave per sub-chunk
  constexpr int MAXSUB = RS / SUBR;
  extern __shared__ __attribute__((aligned(16))) char Xs[];
  // per-wave (max, sum exp) of the chunk's rows, after the X image: [VP_WAVES][xrows]
  float2* Pw = reinterpret_cast<float2*>(Xs + (size_t)vp_xrows(H, R) * RB);
  const int xrows = vp_xrows(H, R);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nt16 = (V + 15) >> 4, NW = gridDim.x * VP_WAVES, q = blockIdx.x * VP_WAVES + wid;
  const int lo = vp_lo(q, nt16, NW), ni = vp_lo(q + 1, nt16, NW) - lo;
  const int cw = 16 * lo;  // this wave's first column
  const int c16 = lane & 15, qd = lane >> 4, kof = 8 * qd;
  const int rot = (blockIdx.x >> 3) % PS;  // piece rotation of this CU (blockIdx % 8 = XCD)
  // the wave's W^T fragments: loaded once, before the first X chunk's LDS fill
  bf16x8 wa[KS][VP_NI];
#pragma unroll
  for (int i = 0; i < VP_NI; ++i) {
    const bf16* arow = WT + (size_t)min(cw + 16 * i + c16, V - 1) * H + kof;
#pragma unroll
    for (int h = 0; h < KS; ++h) wa[h][i] = i < ni ? ld8(arow + 32 * h) : bf16x8{};
  }
  f32x2 bc[VP_NI][2];
#pragma unroll
  for (int i = 0; i < VP_NI; ++i)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int col = cw + 16 * i + 4 * qd + 2 * hh;
      const bool ok = i < ni;
      bc[i][hh] = f32x2{ok && col < V ? bias[col] : -INFINITY, ok && col + 1 < V ? bias[col + 1] : -INFINITY};
    }
  const bool colfull = (V & 3) == 0 && cw + 16 * ni <= V;

  // sub-chunk s of the chunk at r0: piece j of this wave -> registers, then -> its LDS slot
  auto issue = [&](int r0, int s, bf16x8 (&st)[PPW]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int pc = s * PS + (wid + VP_WAVES * j + rot) % PS;
      const int b = pc * 1024 + lane * 16, rr = b / RB, slot = (b % RB) >> 4;
      st[j] = ld8(X + (size_t)min(r0 + rr, R - 1) * H + ((slot ^ (rr & 15)) << 3));
    }
  };
  auto land = [&](int s, const bf16x8 (&st)[PPW]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int pc = s * PS + (wid + VP_WAVES * j + rot) % PS;
      *reinterpret_cast<bf16x8*>(Xs + pc * 1024 + lane * 16) = st[j];
    }
  };
  // the multiply + epilogue of sub-chunk s (row tiles 4 s .. of the chunk at r0)
  auto compute = [&](int r0, int s, int nrt) __attribute__((always_inline)) {
    const int jg = NJ * s, nj = min(NJ, nrt - jg);
    f32x4 acc[VP_NI][NJ];
#pragma unroll
    for (int i = 0; i < VP_NI; ++i)
#pragma unroll
      for (int jr = 0; jr < NJ; ++jr) acc[i][jr] = f32x4{0, 0, 0, 0};
    // per k-step: the group's NJ fragments first (one LDS round trip), then its MFMAs; the next
    // k-step's fragments are read under them (xn), so no MFMA waits on a single read
    auto frag = [&](int h, int jr) __attribute__((always_inline)) {
      const int rr = 16 * (jg + min(jr, nj - 1)) + c16;
      return *reinterpret_cast<const bf16x8*>(Xs + rr * RB + (((4 * h + qd) ^ (rr & 15)) << 4));
    };
    bf16x8 xb[NJ];
#pragma unroll
    for (int jr = 0; jr < NJ; ++jr) xb[jr] = frag(0, jr);
#pragma unroll
    for (int h = 0; h < KS; ++h) {
      bf16x8 xn[NJ];
      if (h + 1 < KS) {
#pragma unroll
        for (int jr = 0; jr < NJ; ++jr) xn[jr] = frag(h + 1, jr);
      }
#pragma unroll
      for (int jr = 0; jr < NJ; ++jr) {
        if (PROBE & 4) {
          acc[0][jr][0] += (float)xb[jr][0];
        } else {
          acc[0][jr] = mfma16(wa[h][0], xb[jr], acc[0][jr]);
          if (ni > 1) acc[1][jr] = mfma16(wa[h][1], xb[jr], acc[1][jr]);
        }
      }
      if (h + 1 < KS) {
#pragma unroll
        for (int jr = 0; jr < NJ; ++jr) xb[jr] = xn[jr];
      }
    }
    f32x2 x[NJ][VP_NI][2];
    float m[NJ], sm[NJ];
#pragma unroll
    for (int jr = 0; jr < NJ; ++jr) {
      m[jr] = -INFINITY;
#pragma unroll
      for (int i = 0; i < VP_NI; ++i)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          x[jr][i][hh] = f32x2{acc[i][jr][2 * hh], acc[i][jr][2 * hh + 1]} + bc[i][hh];  // -inf past V / ni
          m[jr] = vmax3(m[jr], x[jr][i][hh].x, x[jr][i][hh].y);
        }
    }
    if (!(PROBE & 2)) {
#pragma unroll
      for (int jr = 0; jr < NJ; ++jr) m[jr] = max_x16(m[jr]);
#pragma unroll
      for (int jr = 0; jr < NJ; ++jr) m[jr] = max_x32(m[jr]);
      f32x2 s2[NJ];
#pragma unroll
      for (int jr = 0; jr < NJ; ++jr) {
        s2[jr] = f32x2{0.f, 0.f};
        const f32x2 mb = f32x2{-m[jr] * L2E, -m[jr] * L2E};
#pragma unroll
        for (int i = 0; i < VP_NI; ++i)
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const f32x2 t = __builtin_elementwise_fma(x[jr][i][hh], f32x2{L2E, L2E}, mb);
            s2[jr] += f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};  // exp(-inf) = 0
          }
      }
#pragma unroll
      for (int jr = 0; jr < NJ; ++jr) sm[jr] = sum_x16(s2[jr].x + s2[jr].y);
#pragma unroll
      for (int jr = 0; jr < NJ; ++jr) sm[jr] = sum_x32(sm[jr]);
    } else {
#pragma unroll
      for (int jr = 0; jr < NJ; ++jr) sm[jr] = 0.f;
    }
#pragma unroll
    for (int jr = 0; jr < NJ; ++jr) {
      if (jr >= nj) break;
      const int row = r0 + 16 * (jg + jr) + c16;
      if (row >= R) break;
      if (lane < 16) Pw[wid * xrows + row - r0] = make_float2(m[jr], sm[jr]);
      if (PROBE & 1) continue;
      float* dst = logits + (size_t)row * V;
#pragma unroll
      for (int i = 0; i < VP_NI; ++i) {
        if (i >= ni) break;
        const int col = cw + 16 * i + 4 * qd;
        if (PROBE & 8) {  // plain (temporal) stores
          *reinterpret_cast<f32x4*>(dst + col) = f32x4{x[jr][i][0].x, x[jr][i][0].y, x[jr][i][1].x, x[jr][i][1].y};
        } else if (PROBE & 16) {  // span-major [NW][R][32]: a row's span is one 128-byte line
          f32x4* d = reinterpret_cast<f32x4*>(logits + (((size_t)q * R + row) * 32) + 8 * qd + 4 * i);
          __builtin_nontemporal_store(f32x4{x[jr][i][0].x, x[jr][i][0].y, x[jr][i][1].x, x[jr][i][1].y}, d);
        } else if (PROBE & 32) {  // bf16 logits (half the bytes)
          typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
          const unsigned a = (unsigned)__builtin_bit_cast(unsigned short, f2bf(x[jr][i][0].x)) |
                             ((unsigned)__builtin_bit_cast(unsigned short, f2bf(x[jr][i][0].y)) << 16);
          const unsigned b = (unsigned)__builtin_bit_cast(unsigned short, f2bf(x[jr][i][1].x)) |
                             ((unsigned)__builtin_bit_cast(unsigned short, f2bf(x[jr][i][1].y)) << 16);
          __builtin_nontemporal_store(u32x2v{a, b}, reinterpret_cast<u32x2v*>(reinterpret_cast<bf16*>(logits) + (size_t)row * V + col));
        } else if (colfull) {
          __builtin_nontemporal_store(f32x4{x[jr][i][0].x, x[jr][i][0].y, x[jr][i][1].x, x[jr][i][1].y},
                                      reinterpret_cast<f32x4*>(dst + col));
        } else {
          const float xv[4] = {x[jr][i][0].x, x[jr][i][0].y, x[jr][i][1].x, x[jr][i][1].y};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e < V) dst[col + e] = xv[e];
        }
      }
    }
  };
  // one X chunk (rows [r0, r0 + RS)).  FULL: all MAXSUB sub-chunks hold rows (no run-time guard
  // around a load, so the compiler's wait counts stay exact); otherwise sub-chunks past the
  // chunk's rows are neither loaded nor multiplied
  auto chunk = [&](const int r0, auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
    const int nrt = (min(RS, R - r0) + 15) >> 4;  // 16-row tiles of this chunk
    const int nsub = FULL ? MAXSUB : (nrt + NJ - 1) / NJ;
    if (r0 > 0) lds_barrier();  // the previous chunk's fragment reads are done
    bf16x8 st[VP_LOOK][PPW];
#pragma unroll
    for (int s = 0; s < VP_LOOK && s < MAXSUB; ++s)
      if (FULL || s < nsub) issue(r0, s, st[s]);
#pragma unroll
    for (int s = 0; s < MAXSUB; ++s) {
      if (FULL || s < nsub) {
        land(s, st[s % VP_LOOK]);
        lds_barrier();
        if (s + VP_LOOK < MAXSUB && (FULL || s + VP_LOOK < nsub)) issue(r0, s + VP_LOOK, st[s % VP_LOOK]);
        if (ni > 0) compute(r0, s, nrt);
      }
    }
    // the workgroup's (max, sum exp) per row over its 8 waves' spans -> part_ms[row][G] (waves with
    // an empty span wrote nothing)
    lds_barrier();
    const int nr = min(RS, R - r0), q0 = blockIdx.x * VP_WAVES;
    for (int rr = threadIdx.x; rr < nr; rr += VP_THREADS) {
      float mm = -INFINITY, ss = 0.f;
#pragma unroll
      for (int w = 0; w < VP_WAVES; ++w)
        if (vp_lo(q0 + w + 1, nt16, NW) > vp_lo(q0 + w, nt16, NW)) ms_combine(mm, ss, Pw[w * xrows + rr].x, Pw[w * xrows + rr].y);
      *reinterpret_cast<float2*>(part_ms + ((size_t)(r0 + rr) * gridDim.x + blockIdx.x) * 2) = make_float2(mm, ss);
    }
  };
  int r0 = 0;
  for (; r0 + RS <= R; r0 += RS) chunk(r0, std::integral_constant<bool, true>{});
  if (r0 < R) chunk(r0, std::integral_constant<bool, false>{});
}

namespace {
__device__ __forceinline__ int vhslot(int w) { return (int)(((unsigned)w * 2654435761u) >> 21) & (VM_HASH - 1); }

}  // namespace

#define VS_THREADS 1024  // 256 threads measured 16.6 us vs 14.0 at R = 256 (fewer loads in flight)
#define VS_NONE 0x7fffffff  // sentinel id: (-inf, VS_NONE) never beats anything

namespace {
// Top-K of n4 (multiple of 4, padded with sentinels) LDS entries by rank counting: every
// entry counts the entries that beat it (value desc, id asc -- a strict order for distinct
// pairs) with broadcast float4/int4 LDS reads; entries of rank < K land in ov/oi[rank].
// Used on small, pre-pruned sets (typically K to a few K entries).  ov/oi
// must be pre-filled with (-inf, VS_NONE).
// vbetter without short-circuit branches (the rank loop stays straight-line)
__device__ __forceinline__ int beats(float a, int ai, float x, int xi) {
  return (int)(a > x) | ((int)(a == x) & (int)(ai < xi));
}

// order-preserving float -> int key (for LDS atomicMax)
__device__ __forceinline__ int okey(float f) {
  const int b = __float_as_int(f);
  return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float okey_inv(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff); }

__device__ __forceinline__ void rank_select(const float* v, const int* id, int n4, int K, float* ov, int* oi) {
  for (int i = threadIdx.x; i < n4; i += VS_THREADS) {
    const float x = v[i];
    const int xi = id[i];
    if (xi == VS_NONE) continue;
    int rank = 0;
#pragma unroll 4
    for (int j = 0; j < n4; j += 4) {  // no early exit: the loads stay independent and pipelined
      const float4 a = *reinterpret_cast<const float4*>(v + j);
      const int4 b = *reinterpret_cast<const int4*>(id + j);
      rank += beats(a.x, b.x, x, xi) + beats(a.y, b.y, x, xi) + beats(a.z, b.z, x, xi) + beats(a.w, b.w, x, xi);
    }
    if (rank < K) {
      ov[rank] = x;
      oi[rank] = xi;
    }
  }
}

__device__ __forceinline__ void pad4(float* v, int* id, int n) {
  if (threadIdx.x < 4) {
    v[n + threadIdx.x] = -INFINITY;
    id[n + threadIdx.x] = VS_NONE;
  }
}
}  // namespace

// grid R, 1024 threads.  Two global round trips: (partials, copy ids, attention) issued
// together, then (the K best tiles' logits, the copied words' logits) issued together.
// With pg.w set the kernel also computes p_gen = sigmoid([ctx, c, h, x] . w + b) of its row
// (reference attention_decoder.py:164-168; one launch less per decode step) and stores it
// to pg.out; otherwise p_gen comes from ``pgen`` (nullptr for both: baseline, no pointer).
//
// BeamTail (bt.lp_sum set): the last of an article's ``beam`` row workgroups to finish (one
// arrival counter per article) then runs that article's beam bookkeeping (beam_common.h) --
// one kernel boundary less per decode step than a separate beam_step launch.
// attribution builds (tools/vocab_select_stamps.py): thread 0 of each row stamps s_memtime at the
// phase boundaries into vs_stamps[row][16] (a buffer only the tool reads)
__device__ unsigned long long* vs_stamps = nullptr;
#define VS_ST(k)                                                                       \
  do {                                                                                 \
    if constexpr (STAMP) {                                                             \
      if (tid == 0) vs_stamps[(size_t)r * 16 + (k)] = __builtin_amdgcn_s_memtime();    \
    }                                                                                  \
  } while (0)
template <bool STAMP = false>
__global__ __launch_bounds__(VS_THREADS) void vocab_select_kernel(
    const float* __restrict__ logits, const float* __restrict__ part_ms, const float* __restrict__ pgen,
    const float* __restrict__ attn, const int* __restrict__ ext, const int* __restrict__ lens,
    int* __restrict__ out_ids, float* __restrict__ out_lp, int V, int T, int K, int beam, int nt, int tcols, PgIn pgi,
    BeamTail bt, int span) {  // span: partials of vocab_logits_span_kernel (nt = NW waves, [G][R][8], vp_lo columns)
  __shared__ float bt_cval[64];
  __shared__ int bt_cid[64], bt_srt[64];
  __shared__ int bt_last;
  __shared__ int hkey[VM_HASH];
  __shared__ float hmass[VM_HASH];
  __shared__ __attribute__((aligned(16))) float cv[VM_CAND + 8];
  __shared__ __attribute__((aligned(16))) int ci[VM_CAND + 8];
  __shared__ float red[16];
  __shared__ float pv_s[3][VT_K];
  __shared__ int pi_s[3][VT_K];
  __shared__ int gkey[VT_K], gkey2[VT_K], gkey3[VT_K];
  __shared__ int ncand, ncopy;
  const int r = blockIdx.x, tid = threadIdx.x;
  const int art = r / beam;
  const float* z = logits + (size_t)r * V;
  VS_ST(0);
  constexpr int PPT = VM_CAND / VS_THREADS;  // tile partials per thread (nt <= 4096)
  constexpr int TPT = 2048 / VS_THREADS;     // source positions per thread (T <= 2048)
  constexpr int SPT = VM_HASH / VS_THREADS;  // hash slots per thread
  // ---- round trip 1: tile partials, copy ids and attention, all in flight together
  const bool ptr = pgen || pgi.w;
  float pg = pgen ? pgen[r] : 1.0f;
  float pgd = 0.f;  // this thread's share of the p_gen pre-activation
  if (pgi.w) {
    const int A = pgi.A, H = pgi.H;
    for (int i = tid; i < A + 2 * H + pgi.E; i += VS_THREADS) {
      const float x = i < A ? pgi.ctx[(size_t)r * A + i]
                    : i < A + H ? pgi.c[(size_t)r * H + i - A]
                    : i < A + 2 * H ? bf2f(pgi.h[(size_t)r * H + i - A - H])
                    : pgi.x[(size_t)r * pgi.E + i - A - 2 * H];
      pgd += x * pgi.w[i];
    }
  }
  const int len = ptr ? (int)DCHECK_IDX(lens[art], 0, T + 1, CHK_LOSS_LEN) : 0;
  float2 pm[PPT];
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const int q = tid + u * VS_THREADS;
    pm[u] = q < nt ? *reinterpret_cast<const float2*>(part_ms + ((size_t)r * nt + q) * 2) : make_float2(-INFINITY, 0.f);
  }
  int ew[TPT];
  float ea[TPT];
#pragma unroll
  for (int u = 0; u < TPT; ++u) {
    const int i = tid + u * VS_THREADS;
    ew[u] = i < len ? ext[(size_t)art * T + i] : -1;
    ea[u] = i < len ? attn[(size_t)r * T + i] : 0.f;
  }
  for (int i = tid; i < VM_HASH; i += VS_THREADS) { hkey[i] = -1; hmass[i] = 0.f; }
  if (tid < 3 * VT_K) { (&pv_s[0][0])[tid] = -INFINITY; (&pi_s[0][0])[tid] = VS_NONE; }
  if (tid == 0) { ncand = 0; ncopy = 0; }
  if (tid < VT_K) { gkey[tid] = okey(-INFINITY); gkey2[tid] = okey(-INFINITY); gkey3[tid] = okey(-INFINITY); }
  float m = -INFINITY;
#pragma unroll
  for (int u = 0; u < PPT; ++u) m = fmaxf(m, pm[u].x);
  if (pgi.w) {  // uniform branch: block_sum's barriers are reached by every thread
    pg = fsigmoid(block_sum<VS_THREADS>(pgd, red) + pgi.b[0]);
    if (tid == 0 && pgi.out) pgi.out[r] = pg;
  }
  __syncthreads();  // hash cleared before the inserts below (and red free for block_max)
  VS_ST(1);
  // pointer copy mass per extended-vocab word (LDS hash)
#pragma unroll
  for (int u = 0; u < TPT; ++u) {
    const int w = ew[u];
    if (w < 0) continue;
    int h = vhslot(w);
    for (int probe = 0; probe < VM_HASH; ++probe) {
      const int prev = atomicCAS(&hkey[h], -1, w);
      if (prev == -1 || prev == w) {
        atomicAdd(&hmass[h], ea[u]);
        break;
      }
      h = (h + 1) & (VM_HASH - 1);
    }
  }
  // log-sum-exp of the row from the partials
  VS_ST(2);
  const float M = block_max<VS_THREADS>(m, red);
  VS_ST(3);
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < PPT; ++u)
    if (pm[u].x > -INFINITY) s += pm[u].y * fexp(pm[u].x - M);
  // prune the tiles: the maxima of K disjoint tile groups (q mod K) are K distinct tile maxima,
  // so their minimum is <= the K-th largest tile max; only tiles at or above it can matter
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const int q = tid + u * VS_THREADS;
    if (q < nt) atomicMax(&gkey[q % K], okey(pm[u].x));
  }
  const float lse = M + __logf(block_sum<VS_THREADS>(s, red));  // (its syncs also close the hash inserts)
  VS_ST(4);
  float gmin = INFINITY;
  for (int g = 0; g < K; ++g) gmin = fminf(gmin, okey_inv(gkey[g]));
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const int q = tid + u * VS_THREADS;
    if (q < nt && pm[u].x >= gmin) {
      const int slot = atomicAdd(&ncand, 1);
      cv[slot] = pm[u].x;
      ci[slot] = q;
    }
  }
  __syncthreads();
  const int ntile = ncand;
  pad4(cv, ci, ntile);
  __syncthreads();
  // the K tiles with the largest maxima hold the plain top-K (value desc, index asc): an
  // element of any other tile is <= its tile max <= tau, and each selected tile max beats it
  VS_ST(5);
  rank_select(cv, ci, (ntile + 3) & ~3, K, pv_s[0], pi_s[0]);
  __syncthreads();
  VS_ST(6);
  if (tid == 0) ncand = 0;
  const float tau = pv_s[0][K - 1];
  // ---- round trip 2: the K selected tiles' logits and the copied words' logits
  constexpr int EPT = VT_K * 256 / VS_THREADS;  // tiles of <= 256 columns
  float zs[EPT];
  int cs[EPT];
#pragma unroll
  for (int u = 0; u < EPT; ++u) {
    const int e = tid + u * VS_THREADS;
    const int tq = e < K * tcols ? pi_s[0][e / tcols] : VS_NONE;
    if (span) {  // tile tq = workgroup tq's columns [16 vp_lo(8 tq), 16 vp_lo(8 tq + 8)), tcols its maximum
      const int nt16 = (V + 15) >> 4, nw = VP_WAVES * nt;
      const int c = tq < nt ? 16 * vp_lo(VP_WAVES * tq, nt16, nw) + (e % tcols) : V;
      cs[u] = tq < nt && c < 16 * vp_lo(VP_WAVES * tq + VP_WAVES, nt16, nw) ? c : V;
    } else {
      cs[u] = tq < nt ? tq * tcols + (e % tcols) : V;
    }
    zs[u] = cs[u] < V ? z[cs[u]] : -INFINITY;
  }
  int wk[SPT];
  float zk[SPT];
#pragma unroll
  for (int u = 0; u < SPT; ++u) {
    wk[u] = hkey[tid + VS_THREADS * u];
    zk[u] = (wk[u] >= 0 && wk[u] < V) ? z[wk[u]] : -INFINITY;
  }
  // a tighter bound than tau: the maxima of K disjoint groups of the selected tiles' entries
  // (entry index mod K) are K distinct entries, so the K-th largest logit is >= their minimum.
  // With trained weights the best tiles are the frequent-word tiles, nearly all of whose
  // entries are >= tau: ~2000 candidates for the quadratic rank select instead of a few K
  // (vocab_select 20.7 -> 29.4 us per step before this bound: profiles/r4/ab/decode_trained.md)
#pragma unroll
  for (int u = 0; u < EPT; ++u)
    if (cs[u] < V) atomicMax(&gkey3[(tid + u * VS_THREADS) % K], okey(zs[u]));
  __syncthreads();  // ncand reset, the tile list and the group maxima read by everyone before the appends
  VS_ST(7);
  float tau2 = INFINITY;
  for (int g = 0; g < K; ++g) tau2 = fminf(tau2, okey_inv(gkey3[g]));
  tau2 = fmaxf(tau2, tau);
#pragma unroll
  for (int u = 0; u < EPT; ++u)
    if (cs[u] < V && zs[u] >= tau2) {
      const int slot = atomicAdd(&ncand, 1);
      cv[slot] = zs[u];
      ci[slot] = cs[u];
    }
  __syncthreads();
  const int nc = ncand;
  pad4(cv, ci, nc);
  __syncthreads();
  VS_ST(8);
  rank_select(cv, ci, (nc + 3) & ~3, K, pv_s[1], pi_s[1]);  // plain top-K
  __syncthreads();
  VS_ST(9);
  // final candidates: plain top-K (copied words masked: their entry below is exact) U copied words
  if (tid < K) {
    const int w = pi_s[1][tid];
    bool incopy = false;
    if (len > 0 && w != VS_NONE) {
      int h = vhslot(w);
      for (int probe = 0; probe < VM_HASH; ++probe) {
        const int kk = hkey[h];
        if (kk == -1) break;
        if (kk == w) { incopy = true; break; }
        h = (h + 1) & (VM_HASH - 1);
      }
    }
    cv[tid] = (incopy || w == VS_NONE) ? -INFINITY : pg * fexp(pv_s[1][tid] - lse);
    ci[tid] = w;
  }
  // every plain top-K word has a final probability >= theta (the smallest plain term
  // pg * p_vocab among them), so a copied word below theta cannot make the top-K; and the
  // maxima of K disjoint groups of copied words are K distinct entries, so nothing below
  // their minimum can either
  float theta = INFINITY;
  for (int k = 0; k < K; ++k)
    theta = fminf(theta, pi_s[1][k] == VS_NONE ? -INFINITY : pg * fexp(pv_s[1][k] - lse));
  float fin[SPT];
#pragma unroll
  for (int u = 0; u < SPT; ++u) {
    const float pv = (wk[u] >= 0 && wk[u] < V) ? fexp(zk[u] - lse) : 0.f;
    fin[u] = wk[u] < 0 ? -INFINITY : pg * pv + (1.0f - pg) * hmass[tid + VS_THREADS * u];
    if (fin[u] >= theta) atomicMax(&gkey2[(tid + VS_THREADS * u) % K], okey(fin[u]));
  }
  __syncthreads();
  float thr = INFINITY;
  for (int g = 0; g < K; ++g) thr = fminf(thr, okey_inv(gkey2[g]));
  thr = fmaxf(thr, theta);
#pragma unroll
  for (int u = 0; u < SPT; ++u) {
    if (wk[u] >= 0 && fin[u] >= thr) {
      const int slot = atomicAdd(&ncopy, 1);
      cv[K + slot] = fin[u];
      ci[K + slot] = wk[u];
    }
  }
  __syncthreads();
  const int nf = K + ncopy;
  pad4(cv, ci, nf);
  __syncthreads();
  VS_ST(10);
  rank_select(cv, ci, (nf + 3) & ~3, K, pv_s[2], pi_s[2]);
  __syncthreads();
  VS_ST(11);
  if (tid < K) {
    out_ids[(size_t)r * K + tid] = pi_s[2][tid];
    out_lp[(size_t)r * K + tid] = __logf(pv_s[2][tid]);
  }
  if (bt.lp_sum) {  // uniform
    // this row's own p_gen history entry (the article tail must not read the p_gen of the
    // article's other rows: those are plain stores of other workgroups of this launch)
    if (tid == 0 && bt.pg_hist) {
      const size_t th = (size_t)min(*bt.step - 1, bt.max_dec - 1);
      bt.pg_hist[th * ((size_t)bt.Na * beam) + r] = pg;
    }
    if (tid < K) {  // this row's candidates as tagged granules (see beam_article_tail)
      const unsigned long long hi = ((unsigned long long)((unsigned)(*bt.step) & 0x7fffu) << 17) |
                                    (unsigned)(pi_s[2][tid] & 0x1ffff);
      __hip_atomic_store(bt.gran + (size_t)r * K + tid, (hi << 32) | __float_as_uint(__logf(pv_s[2][tid])),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (tid == 0)
      bt_last = __hip_atomic_fetch_add(&bt.art_ctr[art], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                (unsigned)(beam - 1);
    __syncthreads();
    if (bt_last) {
      if (tid == 0) __hip_atomic_store(&bt.art_ctr[art], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      beam_article_tail(bt, art, bt_cval, bt_cid, bt_srt);
    }
  }
  VS_ST(12);
}

// attribution probe: one span-kernel launch with PROBE bits (H = 256)
void launch_vocab_span_probe(const bf16* X, const bf16* WT, const float* bias, float* logits, float* part_ms, int R, int V,
                             int probe, hipStream_t st) {
  const int nt = vp_groups(V);
  const size_t lds = (size_t)vp_xrows(256, R) * (512 + 8 * VP_WAVES);
#define VPP(PB)                                                                                               \
  do {                                                                                                        \
    auto kfn = vocab_logits_span_kernel<256, PB>;                                                             \
    (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);      \
    hipLaunchKernelGGL(kfn, dim3(nt), dim3(VP_THREADS), lds, st, X, WT, bias, logits, part_ms, R, V); \
  } while (0)
  switch (probe) {
    case 0: VPP(0); break;
    case 1: VPP(1); break;
    case 3: VPP(3); break;
    case 4: VPP(4); break;
    case 5: VPP(5); break;
    case 8: VPP(8); break;
    case 16: VPP(16); break;
    case 32: VPP(32); break;
    default: VPP(7); break;
  }
#undef VPP
}

static bool vs_stamp_host = false;
// attribution: stamps of the span-path select kernel go to buf ([R][16] u64); nullptr turns them off
void set_vocab_select_stamps(unsigned long long* buf) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(vs_stamps), &buf, sizeof(buf));
  vs_stamp_host = buf != nullptr;
}

int vocab_topk_tiles(int V, int H) { return vp_use(H) ? vp_groups(V) : (V + vt_cols(H) - 1) / vt_cols(H); }

void launch_vocab_topk(const bf16* X, const bf16* WT, const float* bias, const float* pgen, const float* attn,
                       const int* ext, const int* lens, int* out_ids, float* out_lp, float* logits, float* part_ms,
                       int R, int V, int H, int T, int K, int beam, PgIn pgi, hipStream_t st, const BeamTail* bt) {
  const int nt = vocab_topk_tiles(V, H);
  const BeamTail none{};
  const bool span = vp_use(H);
  if (span) {
    const size_t lds = (size_t)vp_xrows(H, R) * (2 * H + 8 * VP_WAVES);
#define VPL(HH)                                                                                             \
  do {                                                                                                      \
    auto kfn = vocab_logits_span_kernel<HH>;                                                                \
    (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);    \
    hipLaunchKernelGGL(kfn, dim3(nt), dim3(VP_THREADS), lds, st, X, WT, bias, logits, part_ms, R, V); \
  } while (0)
    if (H == 128) VPL(128);
    else if (H == 256) VPL(256);
    else VPL(512);
#undef VPL
    if (vs_stamp_host)
      hipLaunchKernelGGL(vocab_select_kernel<true>, dim3(R), dim3(VS_THREADS), 0, st, logits, part_ms, pgen, attn, ext, lens,
                         out_ids, out_lp, V, T, K, beam, nt, 16 * VP_NI * VP_WAVES, pgi, bt ? *bt : none, 1);
    else
      hipLaunchKernelGGL(vocab_select_kernel<false>, dim3(R), dim3(VS_THREADS), 0, st, logits, part_ms, pgen, attn, ext, lens,
                         out_ids, out_lp, V, T, K, beam, nt, 16 * VP_NI * VP_WAVES, pgi, bt ? *bt : none, 1);
    return;
  }
  const int tcols = vt_cols(H);
  // default: 128-row workgroups (392 at R = 256, V = 50k: one round at 2 per CU; W^T fragments
  // fetched once per 128 rows): decode 5610 -> 5927 summaries/s at 64 articles, 6940 -> 7300 at
  // 128 (64-row workgroups, 784 at R = 256, run 1.5 rounds)
  // hidden 512: 64-row workgroups (the X tile is 66 KB), 128 columns each
  if (H <= 256) {
    const int RB = (R + VT_ROWS * 2 - 1) / (VT_ROWS * 2);
    // (HFIX at 256 spills 16 VGPRs: the constant split lets all 16 X chunks be hoisted in flight)
    hipLaunchKernelGGL((vocab_logits_kernel<2, 2, 256>), dim3(8 * RB * ((nt + 7) / 8)), dim3(256), 0, st, X, WT, bias,
                       logits, part_ms, R, V, H);
  } else {
    const int RB = (R + VT_ROWS - 1) / VT_ROWS;
    hipLaunchKernelGGL((vocab_logits_kernel<2, 1, 512, true>), dim3(8 * RB * ((nt + 7) / 8)), dim3(256), 0, st, X, WT,
                       bias, logits, part_ms, R, V, H);
  }
  hipLaunchKernelGGL(vocab_select_kernel<false>, dim3(R), dim3(VS_THREADS), 0, st, logits, part_ms, pgen, attn, ext, lens,
                     out_ids, out_lp, V, T, K, beam, nt, tcols, pgi, bt ? *bt : none, 0);
}
