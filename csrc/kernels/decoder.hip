// Attention-decoder recurrence, train/eval direction (SURVEY K5-K7, K13/K14 hoisted;
// reference attention_decoder.py:131-174).  Per decoder step t the reference computes
//   x_t  = [emb_t, ctx_{t-1}] . W_in + b_in
//   z    = [x_t, h_{t-1}] . W_cell + b_cell ; (c_t, h_t) = LSTMCell(z, c_{t-1})
//   s_t  = [c_t, h_t] . W_s + b_s                     (attention query features)
// Only z is on the recurrent critical path, and x_t enters it linearly, so the loop
// computes   z = XG_t + ctx_{t-1} . W_comb + h_{t-1} . W_cell[E:]
// with XG_t = (emb_t.W_in[:E] + b_in).W_cell[:E] + b_cell for all t as ONE GEMM before the
// loop and W_comb = W_in[E:] . W_cell[:E] precomputed per optimizer step.  x_t itself is
// rebuilt after the loop (one GEMM) for p_gen and the weight gradients.  Mathematically
// identical to the reference; it removes a dependent GEMM (and a ~1.5 us kernel boundary)
// from every decoder step.  Backward mirrors it: one GEMM per step produces
//   [dx_t | dh_{t-1} | dctx_{t-1}] = dz_t . [W_cell | W_comb]^T
// (dctx additionally gets dCTX_dir and the p_gen path dX_dir.W_in[E:]^T, both hoisted).
//
// Every kernel: one block = 4 waves on a 16x16 output tile (x 4 gates for the cell),
// K split across the waves (kslice_mma) and summed in LDS (ksplit_reduce).
#include "common.h"
#include "launchers.h"
#include <stdlib.h>

// XCD-aware tile order for the (column tile, row tile) grids below.  Blocks are dealt to
// the 8 XCDs round-robin by linear id; every block of a column tile re-reads that tile's
// weight rows, so the column tiles are split into 8 contiguous ranges, one per XCD: each
// XCD's L2 then holds 1/8 of the weight matrix (at hidden 512 the cell / dz weights are
// 6-7 MB, more than one XCD's 4 MB L2).  Falls back to the plain order when gx % 8 != 0.
__device__ __forceinline__ void xcd_tile(int& tx, int& ty) {
  const int gx = gridDim.x, gy = gridDim.y;
  tx = blockIdx.x;
  ty = blockIdx.y;
  if (gx % 8) return;
  const int L = blockIdx.y * gx + blockIdx.x, xcd = L & 7, q = L >> 3, cpx = gx >> 3;
  tx = xcd * cpx + q % cpx;
  ty = q / cpx;
  (void)gy;
}

// z = XG + [ctx, h] . WcT^T ; cell update.  WcT: [4H][A+H] (cols 0..A-1 = W_comb^T, A.. = W_cell[E:]^T).
// grid (H/16, ceil(B/16)).  KB: k-steps per load batch (kslice_mma) -- 6 covers a wave's
// K / 4 = 192 at hidden 256 in one L2 round trip instead of two.
// Beam-decode gather (optional): row r of the step reads its parent row g = gidx[r] of the
// previous state set (c, h, ctx) and the per-token table row of its latest token (in-article
// OOV ids -> [UNK]); thread 0 of block 0 advances the decode-step counter.  Replaces a separate
// beam_gather launch per decode step (device_beam.py).
struct BeamGather {
  const int* gidx;      // [B] parent rows (nullptr: no gather, row r reads row r)
  const int* latest;    // [B] latest token ids
  const float* XGtab;   // [V][4H] per-token gate inputs (replaces XG)
  int V, unk;
  int* step;            // decode-step counter (nullable)
};

// Training: a 16-row tile whose rows are all past their last loss-weighted decoder step
// (step >= dlen[r], EngineConfig.skip_pad_steps) has nothing to compute.  Every wave of the
// block votes on the same 16 rows, so the result is block-uniform (safe before barriers).
__device__ __forceinline__ bool tile_dead(const int* dlen, int step, int r0, int B) {
  if (!dlen) return false;
  const int r = min(r0 + (int)(threadIdx.x & 15), B - 1);
  return __all(step >= dlen[r]);
}

__device__ __forceinline__ int bg_tok(const BeamGather& bg, int r) {
  const int t = (int)DCHECK_IDX(bg.latest[r], 0, 0x7fffffff, CHK_BEAM_TOKEN);
  return t < bg.V ? t : bg.unk;
}

template <int KB>
__global__ __launch_bounds__(256) void dec_cell_fwd_kernel(
    const float* __restrict__ XG,      // [B][4H]
    const bf16* __restrict__ ctxp,     // [B][A]   ctx_{t-1} (nullptr at t==0)
    const bf16* __restrict__ hprev,    // [B][H]
    const float* __restrict__ cprev,   // [B][H]
    const bf16* __restrict__ WcT,      // [4H][A+H]
    float* __restrict__ c_out, bf16* __restrict__ cb_out, bf16* __restrict__ hb_out,  // [B][H]
    float* __restrict__ act,           // [B][4H] (nullable)
    int B, int H, int A, BeamGather bg, const int* __restrict__ dlen, int step) {
  __shared__ float red[4 * 4 * 256];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (bg.step && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *bg.step += 1;
  int tx, ty;
  xcd_tile(tx, ty);
  const int u0 = tx * 16, r0 = ty * 16;
  const int G = 4 * H, K = A + H;
  const int r = r0 + (lane >> 4) * 4 + wid, u = u0 + (lane & 15);
  const bool rok = r < B;
  const size_t ri = (size_t)(rok ? r : 0) * H + u;
  if (tile_dead(dlen, step, r0, B)) {  // finite zeros: the head reads every row's state
    if (rok) {
      c_out[ri] = 0.f;
      cb_out[ri] = f2bf(0.f);
      hb_out[ri] = f2bf(0.f);
      if (act) {
        float* a4 = act + (size_t)r * G;
        a4[u] = 0.f; a4[H + u] = 0.f; a4[2 * H + u] = 0.f; a4[3 * H + u] = 0.f;
      }
    }
    return;
  }
  // parent row of r (gather mode) for the previous state
  const int rp = bg.gidx ? (int)DCHECK_IDX(bg.gidx[rok ? r : 0], 0, B, CHK_BEAM_PARENT) : (rok ? r : 0);
  float xg[4], cp;
  {
    const float* xr = bg.gidx ? bg.XGtab + (size_t)bg_tok(bg, rok ? r : 0) * G : XG + (size_t)(rok ? r : 0) * G;
#pragma unroll
    for (int g = 0; g < 4; ++g) xg[g] = xr[g * H + u];
    cp = cprev[(size_t)rp * H + u];
  }
  const int ar0 = min(r0 + (lane & 15), B - 1);
  const int ar = bg.gidx ? (int)DCHECK_IDX(bg.gidx[ar0], 0, B, CHK_BEAM_PARENT) : ar0;
  const int kof = 8 * (lane >> 4);
  const bf16* crow = ctxp ? ctxp + (size_t)ar * A + kof : nullptr;
  const bf16* hrow = hprev + (size_t)ar * H + kof - A;  // indexed with absolute k >= A
  const bf16* W = WcT + (size_t)(u0 + (lane & 15)) * K + kof;
  const int kbeg = ctxp ? 0 : A;
  const int nst = (K - kbeg) / 32;
  const int k0 = kbeg + (wid * nst / 4) * 32, k1 = kbeg + ((wid + 1) * nst / 4) * 32;
  f32x4 acc[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) acc[g] = f32x4{0, 0, 0, 0};
  kslice_mma<4, KB>([&](int k) { return k < A ? ld8(crow + k) : ld8(hrow + k); },
                [&](int g, int k) { return ld8(W + (size_t)g * H * K + k); }, k0, k1, acc);
  float z[4];
  ksplit_reduce<4>(acc, red, z);
  if (!rok) return;
  const float ig = fsigmoid(z[0] + xg[0]), jg = ftanh(z[1] + xg[1]);
  const float fg = fsigmoid(z[2] + xg[2] + 1.0f), og = fsigmoid(z[3] + xg[3]);
  const float c = fg * cp + ig * jg;
  const float h = og * ftanh(c);
  c_out[ri] = c;
  cb_out[ri] = f2bf(c);
  hb_out[ri] = f2bf(h);
  if (act) {
    float* a4 = act + (size_t)r * G;
    a4[u] = ig; a4[H + u] = jg; a4[2 * H + u] = fg; a4[3 * H + u] = og;
  }
}

// Generic small-M linear on two concatenated bf16 inputs (the shape of every per-step
// projection of the decoder: s = [c,h].W_s + b, out = [h,ctx].W_o + b, x = x0 + ctx.W_in[E:]):
//   out[r][n] = sum_{k<K1} a1[r][k] Wt[n][k] + sum_{k<K2} a2[r][k] Wt[n][K1+k] + bias[n] + add[r][n]
// Wt: [N][K1+K2] bf16 ("Bt" layout).  fp32 and/or bf16 outputs.  grid (N/16, ceil(B/16)),
// 4 waves split K (kslice_mma) and reduce in LDS.  add may alias out (same element, same lane).
// Beam-decode gathers (optional): ga -- operand rows read through a parent index (a1 / a2 row
// ga[r]); gtok -- the add term is a per-token table (add row = table row of token gtok[r], ids
// >= V -> unk), as the x-merge x = x0[token] + ctx_parent . W_in[E:].
struct L2Args {
  const bf16* a1; int K1; const bf16* a2; int K2; const bf16* Wt;
  const float* bias; const float* add; float* out; bf16* outb; int N;
  const int* ga = nullptr; const int* gtok = nullptr; int V = 0, unk = 0;
  const int* dlen = nullptr; int step = 0;  // training: skip tiles of rows past their last live step
};

template <int KB>
__device__ __forceinline__ void linear2_body(const L2Args& p, int B, int n0, int r0, float* red) {
  if (tile_dead(p.dlen, p.step, r0, B)) return;  // (nothing reads a dead row's s)
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ar0 = min(r0 + (lane & 15), B - 1);
  const int ar = p.ga ? (int)DCHECK_IDX(p.ga[ar0], 0, B, CHK_BEAM_PARENT) : ar0;
  const int kof = 8 * (lane >> 4);
  const int K1 = p.K1, K = p.K1 + p.K2, N = p.N;
  const bf16* r1 = p.a1 + (size_t)ar * K1 + kof;
  const bf16* r2 = p.a2 ? p.a2 + (size_t)ar * p.K2 + kof - K1 : nullptr;
  const bf16* brow = p.Wt + (size_t)(n0 + (lane & 15)) * K + kof;
  const int nst = K / 32;
  const int k0 = (wid * nst / 4) * 32, k1 = ((wid + 1) * nst / 4) * 32;
  f32x4 acc[1] = {f32x4{0, 0, 0, 0}};
  kslice_mma<1, KB>([&](int k) { return k < K1 ? ld8(r1 + k) : ld8(r2 + k); },
                [&](int, int k) { return ld8(brow + k); }, k0, k1, acc);
  float o[1];
  ksplit_reduce<1>(acc, red, o);
  const int r = r0 + (lane >> 4) * 4 + wid, n = n0 + (lane & 15);
  if (r >= B) return;
  const size_t ix = (size_t)r * N + n;
  size_t ia = ix;
  if (p.gtok) {
    const int t = (int)DCHECK_IDX(p.gtok[r], 0, 0x7fffffff, CHK_BEAM_TOKEN);
    ia = (size_t)(t < p.V ? t : p.unk) * N + n;
  }
  const float v = o[0] + (p.bias ? p.bias[n] : 0.f) + (p.add ? p.add[ia] : 0.f);
  if (p.out) p.out[ix] = v;
  if (p.outb) p.outb[ix] = f2bf(v);
}

template <int KB>
__global__ __launch_bounds__(256) void linear2_kernel(L2Args p, int B) {
  __shared__ float red[4 * 256];
  int tx, ty;
  xcd_tile(tx, ty);
  linear2_body<KB>(p, B, tx * 16, ty * 16, red);
}

// Two independent linear2 problems on the same rows in one launch (blockIdx.z picks the
// problem; column tiles past a problem's N exit): the beam-decode step pairs the attention
// query projection with the x-merge of the previous context, saving a kernel boundary.
template <int KB>
__global__ __launch_bounds__(256) void linear2_pair_kernel(L2Args p0, L2Args p1, int B) {
  __shared__ float red[4 * 256];
  const L2Args& p = blockIdx.z ? p1 : p0;
  const int n0 = blockIdx.x * 16;
  if (n0 >= p.N) return;  // uniform per block, before any barrier
  linear2_body<KB>(p, B, n0, blockIdx.y * 16, red);
}

// p_gen = sigmoid([ctx, c, h, x] . w + b), one wave per row (reference attention_decoder.py:164-168).
__global__ __launch_bounds__(256) void pgen_kernel(const float* __restrict__ ctx, const float* __restrict__ c,
                                                   const bf16* __restrict__ h, const float* __restrict__ x,
                                                   const float* __restrict__ w, const float* __restrict__ b,
                                                   float* __restrict__ pg, int R, int A, int H, int E) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= R) return;
  float s = 0.f;
  for (int k = lane; k < A; k += 64) s += ctx[(size_t)r * A + k] * w[k];
  for (int k = lane; k < H; k += 64) s += c[(size_t)r * H + k] * w[A + k] + bf2f(h[(size_t)r * H + k]) * w[A + H + k];
  for (int k = lane; k < E; k += 64) s += x[(size_t)r * E + k] * w[A + 2 * H + k];
  s = wave_sum(s);
  if (lane == 0) pg[r] = fsigmoid(s + b[0]);
}

// p_gen weight gradient: gw[k] = sum_n dpre[n] * [ctx, c, h, x][n][k]  (k < A+2H+E).
// grid (ceil(Ktot/256), nsplit): each thread owns one column (coalesced row reads),
// loops its row chunk, then one atomicAdd.  Replaces four fp32 GEMVs (transposed
// large-N GEMV is a slow path in the BLAS library).  gw must be zeroed by the caller.
// p_gen weight gradient, stage 1: column k's partial sum over rows [n0, n0 + rows_per) of split
// blockIdx.y into part[split][k] (4 independent accumulators); stage 2 (colsum_det) adds the
// splits in a fixed order.  The round-5 form added every split's partial into gw with an atomic:
// 400 adds per column address serialised at the memory side (45 us at N = 25600); deterministic
// now in every mode.
__global__ __launch_bounds__(256) void pgen_bwd_kernel(const float* __restrict__ ctx, const float* __restrict__ c,
                                                       const bf16* __restrict__ h, const float* __restrict__ x,
                                                       const float* __restrict__ dpre, float* __restrict__ part,
                                                       int N, int A, int H, int E, int rows_per) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  const int Kt = A + 2 * H + E;
  if (k >= Kt) return;
  const int n0 = blockIdx.y * rows_per, n1 = min(N, n0 + rows_per);
  float a4[4] = {0.f, 0.f, 0.f, 0.f};
  auto sweep = [&](auto ld) {
    int n = n0;
    for (; n + 4 <= n1; n += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a4[u] += dpre[n + u] * ld(n + u);
    }
    for (; n < n1; ++n) a4[0] += dpre[n] * ld(n);
  };
  if (k < A) sweep([&](int n) { return ctx[(size_t)n * A + k]; });
  else if (k < A + H) sweep([&](int n) { return c[(size_t)n * H + (k - A)]; });
  else if (k < A + 2 * H) sweep([&](int n) { return bf2f(h[(size_t)n * H + (k - A - H)]); });
  else sweep([&](int n) { return x[(size_t)n * E + (k - A - 2 * H)]; });
  part[(size_t)blockIdx.y * Kt + k] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
}

// p_gen gradient into the decoder inputs, all D*B rows in one launch (the hoisted per-step
// "direct" terms of the reverse loop):  with dp = dL/d(p_gen pre-activation) and the p_gen
// weight w = [w_ctx | w_c | w_h | w_x],
//   dCTX_dir += dp w_ctx,  dC_dir = dp w_c,  dH_dir += dp w_h,  dX_dir = dp w_x,
// plus the p_gen bias gradient sum(dp) (one atomic per workgroup).  Replaces a reduction,
// four broadcast products, two adds and two copies.  One wave per row.
__global__ __launch_bounds__(256) void pgen_dirs_kernel(const float* __restrict__ dpre, const float* __restrict__ w,
                                                        float* __restrict__ dctx, float* __restrict__ dc,
                                                        float* __restrict__ dh, float* __restrict__ dx,
                                                        float* __restrict__ gb, int N, int A, int H, int E) {
  __shared__ float red[4];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + wid;
  float d = 0.f;
  if (n < N) {
    d = dpre[n];
    const float* wc = w + A;
    const float* wh = w + A + H;
    const float* wx = w + A + 2 * H;
    for (int k = lane; k < A; k += 64) dctx[(size_t)n * A + k] += d * w[k];
    for (int k = lane; k < H; k += 64) {
      dc[(size_t)n * H + k] = d * wc[k];
      dh[(size_t)n * H + k] += d * wh[k];
    }
    for (int k = lane; k < E; k += 64) dx[(size_t)n * E + k] = d * wx[k];
  }
  if (lane == 0) red[wid] = d;
  __syncthreads();
  if (gb && threadIdx.x == 0) atomicAdd(gb, (red[0] + red[1]) + (red[2] + red[3]));
}

// Backward of s-projection + LSTM cell for step t.  grid (H/16, ceil(B/16)).
//   dc_t = ds . W_s[0:H]^T + dC_dir + dc_carry ;  dh_t = ds . W_s[H:2H]^T + dH_dir + dh_rec
//   cell backward -> dz_t (bf16), dc_carry <- dc_total * f
// ds (fp32 [B][A]) was accumulated by attn_bwd_step's blocks with atomics, or stored by
// attn_bwd_row.
__global__ __launch_bounds__(256) void dec_bwd_cell_kernel(
    const float* __restrict__ ds,
    const bf16* __restrict__ Ws,                                               // Ws: [2H][A] (TF Matrix)
    const float* __restrict__ dC_dir, const float* __restrict__ dH_dir,       // [B][H] (nullable)
    const float* __restrict__ dh_rec, float* __restrict__ dc_carry,            // [B][H]
    const float* __restrict__ act, const float* __restrict__ c_now, const float* __restrict__ c_prev,
    bf16* __restrict__ dz, int B, int H, int A, const int* __restrict__ dlen, int step) {
  __shared__ float red[4 * 2 * 256];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int tx, ty;
  xcd_tile(tx, ty);
  const int u0 = tx * 16, r0 = ty * 16;
  const int r = r0 + (lane >> 4) * 4 + wid, u = u0 + (lane & 15);
  const bool rok = r < B;
  if (tile_dead(dlen, step, r0, B)) {  // dz = 0 (read by the weight-gradient GEMMs); dc_carry stays 0
    if (rok) {
      bf16* dzr = dz + (size_t)r * 4 * H;
      dzr[u] = f2bf(0.f); dzr[H + u] = f2bf(0.f); dzr[2 * H + u] = f2bf(0.f); dzr[3 * H + u] = f2bf(0.f);
    }
    return;
  }
  const size_t ri = (size_t)(rok ? r : 0) * H + u;
  float dh0, dc0, a4[4], cn, cpv;
  {
    dh0 = dh_rec[ri] + (dH_dir ? dH_dir[ri] : 0.f);
    dc0 = dc_carry[ri] + (dC_dir ? dC_dir[ri] : 0.f);
    const float* ap = act + (size_t)(rok ? r : 0) * 4 * H;
#pragma unroll
    for (int g = 0; g < 4; ++g) a4[g] = ap[g * H + u];
    cn = c_now[ri];
    cpv = c_prev[ri];
  }
  const int ar = min(r0 + (lane & 15), B - 1);
  const int kof = 8 * (lane >> 4);
  const float* arow = ds + (size_t)ar * A + kof;
  const bf16* bc = Ws + (size_t)(u0 + (lane & 15)) * A + kof;
  const bf16* bh = Ws + (size_t)(H + u0 + (lane & 15)) * A + kof;
  const int nst = A / 32;
  const int k0 = (wid * nst / 4) * 32, k1 = ((wid + 1) * nst / 4) * 32;
  f32x4 acc[2] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
  kslice_mma<2>([&](int k) { return ld8f(arow + k); },
                [&](int j, int k) { return ld8((j == 0 ? bc : bh) + k); }, k0, k1, acc);
  float o[2];  // ds . W_s[0:H]^T, ds . W_s[H:2H]^T
  ksplit_reduce<2>(acc, red, o);
  if (!rok) return;
  const float dh = dh0 + o[1];
  float dc = dc0 + o[0];
  const float ig = a4[0], jg = a4[1], fg = a4[2], og = a4[3];
  const float tc = ftanh(cn);
  dc += dh * og * (1.0f - tc * tc);
  const float dzo = dh * tc * og * (1.0f - og);
  const float dzi = dc * jg * ig * (1.0f - ig);
  const float dzj = dc * ig * (1.0f - jg * jg);
  const float dzf = dc * cpv * fg * (1.0f - fg);
  dc_carry[ri] = dc * fg;
  bf16* dzr = dz + (size_t)r * 4 * H;
  dzr[u] = f2bf(dzi); dzr[H + u] = f2bf(dzj); dzr[2 * H + u] = f2bf(dzf); dzr[3 * H + u] = f2bf(dzo);
}

// [dx_t | dh_{t-1} | dctx_{t-1}] = dz_t . Wbig^T, Wbig = [W_cell ; W_comb]: [E+H+A][4H].
// grid ((E+H+A)/16, ceil(B/16)).  KB: k-steps per load batch (see the launcher).
template <int KB>
__global__ __launch_bounds__(256) void dec_bwd_dz_kernel(
    const bf16* __restrict__ dz, const bf16* __restrict__ Wbig,
    const float* __restrict__ dX_dir,        // [B][E] nullable
    const float* __restrict__ dCTX_dir_prev, // [B][A] nullable (already includes dX_dir[t].W_in[E:]^T)
    float* __restrict__ dx_out,              // [B][E]
    float* __restrict__ dctx_prev_out,       // [B][A] nullable (t == 0)
    float* __restrict__ dh_rec, int B, int E, int H, int A, const int* __restrict__ dlen, int step) {
  __shared__ float red[4 * 256];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int tx, ty;
  xcd_tile(tx, ty);
  const int n0 = tx * 16, r0 = ty * 16;
  if (n0 >= E + H && !dctx_prev_out) return;  // uniform per block
  if (tile_dead(dlen, step, r0, B)) {  // every output is an exact zero past the last live step
    const int r = r0 + (lane >> 4) * 4 + wid, n = n0 + (lane & 15);
    if (r < B) {
      if (n < E) dx_out[(size_t)r * E + n] = 0.f;
      else if (n < E + H) dh_rec[(size_t)r * H + n - E] = 0.f;
      else dctx_prev_out[(size_t)r * A + n - E - H] = 0.f;
    }
    return;
  }
  const int G = 4 * H;
  const int ar = min(r0 + (lane & 15), B - 1);
  const int kof = 8 * (lane >> 4);
  const bf16* arow = dz + (size_t)ar * G + kof;
  const bf16* brow = Wbig + (size_t)(n0 + (lane & 15)) * G + kof;
  const int nst = G / 32;
  const int k0 = (wid * nst / 4) * 32, k1 = ((wid + 1) * nst / 4) * 32;
  f32x4 acc[1] = {f32x4{0, 0, 0, 0}};
  kslice_mma<1, KB>([&](int k) { return ld8(arow + k); }, [&](int, int k) { return ld8(brow + k); }, k0, k1, acc);
  float o[1];
  ksplit_reduce<1>(acc, red, o);
  const int r = r0 + (lane >> 4) * 4 + wid, n = n0 + (lane & 15);
  if (r >= B) return;
  if (n < E) {
    dx_out[(size_t)r * E + n] = o[0] + (dX_dir ? dX_dir[(size_t)r * E + n] : 0.f);
  } else if (n < E + H) {
    dh_rec[(size_t)r * H + n - E] = o[0];
  } else {
    const int a = n - E - H;
    dctx_prev_out[(size_t)r * A + a] = o[0] + (dCTX_dir_prev ? dCTX_dir_prev[(size_t)r * A + a] : 0.f);
  }
}

// dec_cell_fwd with 6-step load batches: 7.67 -> 6.79 us per call at hidden 256 / 128 rows (one
// L2 round trip instead of two with 4-step batches), equal at hidden 512; B = 256 train
// 19.71-19.77 -> 19.63-19.67 ms (profiles/r2/ab/dec_cell_kb.jsonl)
void launch_dec_cell_fwd(const float* XG, const bf16* ctxp, const bf16* hprev, const float* cprev, const bf16* WcT,
                         float* c_out, bf16* cb_out, bf16* hb_out, float* act, int B, int H, int A, const int* dlen,
                         int step, hipStream_t st) {
  dim3 grid(H / 16, (B + 15) / 16);
  hipLaunchKernelGGL(dec_cell_fwd_kernel<6>, grid, dim3(256), 0, st, XG, ctxp, hprev, cprev, WcT, c_out, cb_out,
                     hb_out, act, B, H, A, BeamGather{nullptr, nullptr, nullptr, 0, 0, nullptr}, dlen, step);
}
void launch_dec_cell_fwd_beam(const int* gidx, const int* latest, const float* XGtab, const bf16* ctxp,
                              const bf16* hprev, const float* cprev, const bf16* WcT, float* c_out, bf16* cb_out,
                              bf16* hb_out, int* step, int B, int H, int A, int V, int unk, hipStream_t st) {
  dim3 grid(H / 16, (B + 15) / 16);
  hipLaunchKernelGGL(dec_cell_fwd_kernel<6>, grid, dim3(256), 0, st, nullptr, ctxp, hprev, cprev, WcT, c_out, cb_out,
                     hb_out, nullptr, B, H, A, BeamGather{gidx, latest, XGtab, V, unk, step}, nullptr, 0);
}
// the beam-decode pair: s = [cb, hb] . WsT^T + bs, and x = Xtab[token] + ctx_parent . WicT^T
// k-steps per load batch of linear2: a wave's whole K / 4 slice in one batch (one L2 round trip)
// when it is at most 8 k-steps (the output projection's K = H + A = 768 at hidden 256: 6; the
// query projection's K = 2H = 1024 at hidden 512: 8), else batches of 4
static int l2_kb(int K) {
  const int ks = (K / 32 + 3) / 4;
  return ks <= 4 ? 4 : ks <= 6 ? 6 : ks <= 8 ? 8 : 4;
}
#define L2_LAUNCH(KERN, K, GRID, ST, ...)                                                          \
  do {                                                                                           \
    const int kb_ = l2_kb(K);                                                                    \
    if (kb_ == 6) hipLaunchKernelGGL(KERN<6>, GRID, dim3(256), 0, ST, __VA_ARGS__);              \
    else if (kb_ == 8) hipLaunchKernelGGL(KERN<8>, GRID, dim3(256), 0, ST, __VA_ARGS__);         \
    else hipLaunchKernelGGL(KERN<4>, GRID, dim3(256), 0, ST, __VA_ARGS__);                       \
  } while (0)

void launch_beam_sproj_xmerge(const bf16* cb, const bf16* hb, const bf16* WsT, const float* bs, float* s_out,
                              const bf16* ctx_src, const bf16* WicT, const float* Xtab, const int* gidx,
                              const int* latest, float* x_out, int B, int H, int A, int E, int V, int unk,
                              hipStream_t st) {
  dim3 grid((A > E ? A : E) / 16, (B + 15) / 16, 2);
  L2Args p0{cb, H, hb, H, WsT, bs, nullptr, s_out, nullptr, A};
  L2Args p1{ctx_src, A, nullptr, 0, WicT, nullptr, Xtab, x_out, nullptr, E};
  p1.ga = gidx;
  p1.gtok = latest;
  p1.V = V;
  p1.unk = unk;
  L2_LAUNCH(linear2_pair_kernel, H + H > A ? H + H : A, grid, st, p0, p1, B);
}
void launch_linear2(const bf16* a1, int K1, const bf16* a2, int K2, const bf16* Wt, const float* bias,
                    const float* add, float* out, bf16* outb, int B, int N, hipStream_t st) {
  dim3 grid(N / 16, (B + 15) / 16);
  const L2Args p{a1, K1, a2, K2, Wt, bias, add, out, outb, N};
  L2_LAUNCH(linear2_kernel, K1 + K2, grid, st, p, B);
}
void launch_linear2_pair(const bf16* a1, int K1, const bf16* a2, int K2, const bf16* Wt, const float* bias,
                         const float* add, float* out, bf16* outb, int N, const bf16* c1, int L1, const bf16* c2,
                         int L2, const bf16* Vt, const float* vbias, const float* vadd, float* vout, bf16* voutb,
                         int M, int B, hipStream_t st) {
  dim3 grid((N > M ? N : M) / 16, (B + 15) / 16, 2);
  const L2Args p0{a1, K1, a2, K2, Wt, bias, add, out, outb, N};
  const L2Args p1{c1, L1, c2, L2, Vt, vbias, vadd, vout, voutb, M};
  L2_LAUNCH(linear2_pair_kernel, K1 + K2 > L1 + L2 ? K1 + K2 : L1 + L2, grid, st, p0, p1, B);
}
void launch_dec_sproj(const bf16* cb, const bf16* hb, const bf16* WsT, const float* bs, float* s_out, int B, int H,
                      int A, const int* dlen, int step, hipStream_t st) {
  dim3 grid(A / 16, (B + 15) / 16);
  L2Args p{cb, H, hb, H, WsT, bs, nullptr, s_out, nullptr, A};
  p.dlen = dlen;
  p.step = step;
  L2_LAUNCH(linear2_kernel, H + H, grid, st, p, B);
}
int pgen_bwd_splits(int N, int A, int H, int E) {
  const int cols = (A + 2 * H + E + 255) / 256;
  return max(1, min((N + 63) / 64, 2048 / cols));
}
// part: [pgen_bwd_splits][Kt] fp32, cpart: [colsum_det_chunks(splits, Kt)][Kt] fp32 (workspaces)
void launch_pgen_bwd(const float* ctx, const float* c, const bf16* h, const float* x, const float* dpre, float* gw,
                     float* part, float* cpart, int N, int A, int H, int E, hipStream_t st) {
  const int Kt = A + 2 * H + E;
  const int cols = (Kt + 255) / 256;
  const int nsplit = pgen_bwd_splits(N, A, H, E);
  const int rows_per = (N + nsplit - 1) / nsplit;
  hipLaunchKernelGGL(pgen_bwd_kernel, dim3(cols, nsplit), dim3(256), 0, st, ctx, c, h, x, dpre, part, N, A, H, E,
                     rows_per);
  launch_colsum_det(part, false, cpart, gw, nsplit, Kt, true, st);
}
void launch_pgen_dirs(const float* dpre, const float* w, float* dctx, float* dc, float* dh, float* dx, float* gb,
                      int N, int A, int H, int E, hipStream_t st) {
  hipLaunchKernelGGL(pgen_dirs_kernel, dim3((N + 3) / 4), dim3(256), 0, st, dpre, w, dctx, dc, dh, dx, gb, N, A, H, E);
}
void launch_pgen(const float* ctx, const float* c, const bf16* h, const float* x, const float* w, const float* b,
                 float* pg, int R, int A, int H, int E, hipStream_t st) {
  hipLaunchKernelGGL(pgen_kernel, dim3((R + 3) / 4), dim3(256), 0, st, ctx, c, h, x, w, b, pg, R, A, H, E);
}
void launch_dec_bwd_cell(const float* ds, const bf16* Ws, const float* dC_dir, const float* dH_dir,
                         const float* dh_rec, float* dc_carry, const float* act, const float* c_now,
                         const float* c_prev, bf16* dz, int B, int H, int A, const int* dlen, int step,
                         hipStream_t st) {
  dim3 grid(H / 16, (B + 15) / 16);
  hipLaunchKernelGGL(dec_bwd_cell_kernel, grid, dim3(256), 0, st, ds, Ws, dC_dir, dH_dir, dh_rec, dc_carry, act,
                     c_now, c_prev, dz, B, H, A, dlen, step);
}
void launch_dec_bwd_dz(const bf16* dz, const bf16* Wbig, const float* dX_dir, const float* dCTX_dir_prev,
                       float* dx_out, float* dctx_prev_out, float* dh_rec, int B, int E, int H, int A,
                       const int* dlen, int step, hipStream_t st) {
  dim3 grid((E + H + A) / 16, (B + 15) / 16);
  // KB = 8 measured equal (5.68 vs 5.74 us at 128 rows, tools/dec_kernels_micro.py) at 96 instead
  // of 41 VGPRs, so this one keeps 4-step batches
  hipLaunchKernelGGL(dec_bwd_dz_kernel<4>, grid, dim3(256), 0, st, dz, Wbig, dX_dir, dCTX_dir_prev, dx_out,
                     dctx_prev_out, dh_rec, B, E, H, A, dlen, step);
}
