// Attention-decoder recurrence, train/eval direction (SURVEY K5-K7, K13/K14 hoisted;
// reference attention_decoder.py:131-174).  Per decoder step t the forward chain is
//   x_t  = xe_t + ctx_{t-1} . W_in[E:E+A]            (xe_t = emb_t . W_in[0:E] + b, hoisted)
//   z    = [x_t, h_{t-1}] . W_cell + b ; (c_t, h_t) = LSTMCell(z, c_{t-1})
//   s_t  = [c_t, h_t] . W_s + b_s                     (attention query features)
// followed by the two attention kernels.  p_gen and the output projection depend only
// on per-step values, so they are computed after the loop as batched GEMMs.
//
// dec_xcell_fwd fuses the input merge into the cell kernel: every 64-unit block
// recomputes x_t for its 16 rows (a 16x128x512 MFMA tile set, ~32 MFMA per wave) into
// LDS instead of paying a dependent-kernel boundary (~1.5 us) for a separate x launch.
// Likewise dec_bwd_dz fuses dctx_{t-1} = dx_t . W_in[E:]^T into the block that owns dx.
#include "common.h"

#define XPAD 8

// grid (ceil(H/64), ceil(B/16)); 4 waves.
__global__ __launch_bounds__(256) void dec_xcell_fwd_kernel(
    const float* __restrict__ xe,      // [B][E]   this step's emb.W + b
    const bf16* __restrict__ ctxp,     // [B][A]   ctx_{t-1} (nullptr at t==0)
    const bf16* __restrict__ WicT,     // [E][A]   W_in[E:E+A]^T
    const bf16* __restrict__ WcT,      // [4H][E+H] W_cell^T
    const float* __restrict__ bc,      // [4H]
    const bf16* __restrict__ hprev,    // [B][H]
    const float* __restrict__ cprev,   // [B][H]
    float* __restrict__ x_out, bf16* __restrict__ xb_out,  // [B][E]
    float* __restrict__ c_out, bf16* __restrict__ cb_out, bf16* __restrict__ hb_out,  // [B][H]
    float* __restrict__ act,           // [B][4H]
    int B, int E, int H, int A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xs = reinterpret_cast<bf16*>(smem);  // [16][E+XPAD]
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r0 = blockIdx.y * 16;
  const int ar = min(r0 + (lane & 15), B - 1);
  const int kof = 8 * (lane >> 4);
  const int XS = E + XPAD;
  // ---- phase 1: x rows for this block
  for (int ct = wid; ct < E / 16; ct += 4) {
    f32x4 acc = {0, 0, 0, 0};
    if (ctxp) acc = mfma_k(ctxp + (size_t)ar * A + kof, WicT + (size_t)(ct * 16 + (lane & 15)) * A + kof, A, acc);
    const int col = ct * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int rr = (lane >> 4) * 4 + j, r = r0 + rr;
      const float xv = acc[j] + (r < B ? xe[(size_t)r * E + col] : 0.f);
      xs[rr * XS + col] = f2bf(xv);
      if (blockIdx.x == 0 && r < B) {
        x_out[(size_t)r * E + col] = xv;
        xb_out[(size_t)r * E + col] = f2bf(xv);
      }
    }
  }
  __syncthreads();
  // ---- phase 2: gates for 16 units x 4 gates, K = E (LDS) + H (global h)
  const int u0 = blockIdx.x * 64 + wid * 16;
  if (u0 >= H) return;
  const int K = E + H;
  f32x4 acc[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) acc[g] = f32x4{0, 0, 0, 0};
  const bf16* xa = xs + (lane & 15) * XS + kof;
  for (int k = 0; k < E; k += 32) {
    bf16x8 a = *reinterpret_cast<const bf16x8*>(xa + k);
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = mfma16(a, ld8(WcT + ((size_t)g * H + u0 + (lane & 15)) * K + kof + k), acc[g]);
  }
  const bf16* ha = hprev + (size_t)ar * H + kof;
  for (int k = 0; k < H; k += 32) {
    bf16x8 a = ld8(ha + k);
#pragma unroll
    for (int g = 0; g < 4; ++g)
      acc[g] = mfma16(a, ld8(WcT + ((size_t)g * H + u0 + (lane & 15)) * K + E + kof + k), acc[g]);
  }
  const int u = u0 + (lane & 15);
  const float bi = bc[u], bj = bc[H + u], bff = bc[2 * H + u], bo = bc[3 * H + u];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = r0 + (lane >> 4) * 4 + j;
    if (r >= B) continue;
    const size_t ri = (size_t)r * H + u;
    const float ig = fsigmoid(acc[0][j] + bi), jg = ftanh(acc[1][j] + bj);
    const float fg = fsigmoid(acc[2][j] + bff + 1.0f), og = fsigmoid(acc[3][j] + bo);
    const float c = fg * cprev[ri] + ig * jg;
    const float h = og * ftanh(c);
    c_out[ri] = c;
    cb_out[ri] = f2bf(c);
    hb_out[ri] = f2bf(h);
    float* a4 = act + (size_t)r * 4 * H;
    a4[u] = ig; a4[H + u] = jg; a4[2 * H + u] = fg; a4[3 * H + u] = og;
  }
}

// s = [c, h] . W_s + b_s  -> [B][A] fp32.  grid (ceil(A/64), ceil(B/16)).
__global__ __launch_bounds__(256) void dec_sproj_kernel(
    const bf16* __restrict__ cb, const bf16* __restrict__ hb, const bf16* __restrict__ WsT,  // [A][2H]
    const float* __restrict__ bs, float* __restrict__ s_out, int B, int H, int A) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = blockIdx.x * 64 + wid * 16;
  if (n0 >= A) return;
  const int r0 = blockIdx.y * 16;
  const int ar = min(r0 + (lane & 15), B - 1);
  const int kof = 8 * (lane >> 4);
  const bf16* brow = WsT + (size_t)(n0 + (lane & 15)) * 2 * H + kof;
  f32x4 acc = {0, 0, 0, 0};
  acc = mfma_k(cb + (size_t)ar * H + kof, brow, H, acc);
  acc = mfma_k(hb + (size_t)ar * H + kof, brow + H, H, acc);
  const int n = n0 + (lane & 15);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = r0 + (lane >> 4) * 4 + j;
    if (r < B) s_out[(size_t)r * A + n] = acc[j] + bs[n];
  }
}

// Backward of s-projection + LSTM cell for step t.  grid (ceil(H/64), ceil(B/16)).
//   ds   = sum over position chunks of dsp                     (also stored: ds_out)
//   dc_t = ds . W_s[0:H]^T + dC_dir + dc_carry ;  dh_t = ds . W_s[H:2H]^T + dH_dir + dh_rec
//   cell backward -> dz_t (bf16), dc_carry <- dc_total * f
__global__ __launch_bounds__(256) void dec_bwd_cell_kernel(
    const float* __restrict__ dsp, int nchunk, const bf16* __restrict__ Ws,  // Ws: [2H][A] (TF Matrix)
    const float* __restrict__ dC_dir, const float* __restrict__ dH_dir,       // [B][H] (nullable)
    const float* __restrict__ dh_rec, float* __restrict__ dc_carry,            // [B][H]
    const float* __restrict__ act, const float* __restrict__ c_now, const float* __restrict__ c_prev,
    float* __restrict__ ds_out, bf16* __restrict__ dz, int B, int H, int A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* dss = reinterpret_cast<bf16*>(smem);  // [16][A+XPAD]
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int r0 = blockIdx.y * 16;
  const int AS = A + XPAD;
  for (int idx = tid; idx < 16 * A; idx += 256) {
    const int rr = idx / A, k = idx - rr * A, r = r0 + rr;
    float x = 0.f;
    if (r < B) {
      const float* p = dsp + (size_t)r * nchunk * A + k;
      for (int c = 0; c < nchunk; ++c) x += p[(size_t)c * A];
      if (blockIdx.x == 0) ds_out[(size_t)r * A + k] = x;
    }
    dss[rr * AS + k] = f2bf(x);
  }
  __syncthreads();
  const int u0 = blockIdx.x * 64 + wid * 16;
  if (u0 >= H) return;
  const int kof = 8 * (lane >> 4);
  const bf16* aptr = dss + (lane & 15) * AS + kof;
  f32x4 adc = {0, 0, 0, 0}, adh = {0, 0, 0, 0};
  const bf16* bc = Ws + (size_t)(u0 + (lane & 15)) * A + kof;
  const bf16* bh = Ws + (size_t)(H + u0 + (lane & 15)) * A + kof;
  for (int k = 0; k < A; k += 32) {
    bf16x8 a = *reinterpret_cast<const bf16x8*>(aptr + k);
    adc = mfma16(a, ld8(bc + k), adc);
    adh = mfma16(a, ld8(bh + k), adh);
  }
  const int u = u0 + (lane & 15);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = r0 + (lane >> 4) * 4 + j;
    if (r >= B) continue;
    const size_t ri = (size_t)r * H + u;
    float dh = adh[j] + dh_rec[ri] + (dH_dir ? dH_dir[ri] : 0.f);
    float dc = adc[j] + dc_carry[ri] + (dC_dir ? dC_dir[ri] : 0.f);
    const float* a4 = act + (size_t)r * 4 * H;
    const float ig = a4[u], jg = a4[H + u], fg = a4[2 * H + u], og = a4[3 * H + u];
    const float tc = ftanh(c_now[ri]);
    dc += dh * og * (1.0f - tc * tc);
    const float dzo = dh * tc * og * (1.0f - og);
    const float dzi = dc * jg * ig * (1.0f - ig);
    const float dzj = dc * ig * (1.0f - jg * jg);
    const float dzf = dc * c_prev[ri] * fg * (1.0f - fg);
    dc_carry[ri] = dc * fg;
    bf16* dzr = dz + (size_t)r * 4 * H;
    dzr[u] = f2bf(dzi); dzr[H + u] = f2bf(dzj); dzr[2 * H + u] = f2bf(dzf); dzr[3 * H + u] = f2bf(dzo);
  }
}

// [dx_t | dh_{t-1}] = dz_t . W_cell^T, plus dctx_{t-1} = dx_t . W_in[E:E+A]^T + dCTX_dir.
// grid (1 + ceil(H/64), ceil(B/16)); block x==0 owns dx and dctx, x>=1 own 64 units of dh.
__global__ __launch_bounds__(256) void dec_bwd_dz_kernel(
    const bf16* __restrict__ dz, const bf16* __restrict__ Wc,   // Wc: [E+H][4H] (TF kernel)
    const bf16* __restrict__ Wic,                                 // [A][E] = W_in rows E..E+A-1
    const float* __restrict__ dX_dir,                             // [B][E] nullable
    const float* __restrict__ dCTX_dir_prev,                      // [B][A] nullable (for t-1)
    float* __restrict__ dx_out,                                   // [B][E]
    float* __restrict__ dctx_prev_out,                            // [B][A] nullable (t==0)
    float* __restrict__ dh_rec, int B, int E, int H, int A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r0 = blockIdx.y * 16;
  const int ar = min(r0 + (lane & 15), B - 1);
  const int kof = 8 * (lane >> 4);
  const int G = 4 * H;
  const bf16* arow = dz + (size_t)ar * G + kof;
  if (blockIdx.x > 0) {
    const int u0 = (blockIdx.x - 1) * 64 + wid * 16;
    if (u0 >= H) return;
    f32x4 acc = mfma_k(arow, Wc + (size_t)(E + u0 + (lane & 15)) * G + kof, G, f32x4{0, 0, 0, 0});
    const int u = u0 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + (lane >> 4) * 4 + j;
      if (r < B) dh_rec[(size_t)r * H + u] = acc[j];
    }
    return;
  }
  bf16* dxs = reinterpret_cast<bf16*>(smem);  // [16][E+XPAD]
  const int XS = E + XPAD;
  for (int ct = wid; ct < E / 16; ct += 4) {
    f32x4 acc = mfma_k(arow, Wc + (size_t)(ct * 16 + (lane & 15)) * G + kof, G, f32x4{0, 0, 0, 0});
    const int col = ct * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int rr = (lane >> 4) * 4 + j, r = r0 + rr;
      float v = acc[j] + ((r < B && dX_dir) ? dX_dir[(size_t)r * E + col] : 0.f);
      if (r < B) dx_out[(size_t)r * E + col] = v;
      dxs[rr * XS + col] = f2bf(r < B ? v : 0.f);
    }
  }
  if (!dctx_prev_out) return;
  __syncthreads();
  const bf16* xa = dxs + (lane & 15) * XS + kof;
  for (int ct = wid; ct < A / 16; ct += 4) {
    f32x4 acc = {0, 0, 0, 0};
    const bf16* brow = Wic + (size_t)(ct * 16 + (lane & 15)) * E + kof;
    for (int k = 0; k < E; k += 32) acc = mfma16(*reinterpret_cast<const bf16x8*>(xa + k), ld8(brow + k), acc);
    const int col = ct * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + (lane >> 4) * 4 + j;
      if (r < B) dctx_prev_out[(size_t)r * A + col] = acc[j] + (dCTX_dir_prev ? dCTX_dir_prev[(size_t)r * A + col] : 0.f);
    }
  }
}

void launch_dec_xcell_fwd(const float* xe, const bf16* ctxp, const bf16* WicT, const bf16* WcT, const float* bc,
                          const bf16* hprev, const float* cprev, float* x_out, bf16* xb_out, float* c_out,
                          bf16* cb_out, bf16* hb_out, float* act, int B, int E, int H, int A, hipStream_t st) {
  dim3 grid((H + 63) / 64, (B + 15) / 16);
  size_t sm = 16 * (E + XPAD) * sizeof(bf16);
  hipLaunchKernelGGL(dec_xcell_fwd_kernel, grid, dim3(256), sm, st, xe, ctxp, WicT, WcT, bc, hprev, cprev, x_out,
                     xb_out, c_out, cb_out, hb_out, act, B, E, H, A);
}
void launch_dec_sproj(const bf16* cb, const bf16* hb, const bf16* WsT, const float* bs, float* s_out, int B, int H,
                      int A, hipStream_t st) {
  dim3 grid((A + 63) / 64, (B + 15) / 16);
  hipLaunchKernelGGL(dec_sproj_kernel, grid, dim3(256), 0, st, cb, hb, WsT, bs, s_out, B, H, A);
}
void launch_dec_bwd_cell(const float* dsp, int nchunk, const bf16* Ws, const float* dC_dir, const float* dH_dir,
                         const float* dh_rec, float* dc_carry, const float* act, const float* c_now,
                         const float* c_prev, float* ds_out, bf16* dz, int B, int H, int A, hipStream_t st) {
  dim3 grid((H + 63) / 64, (B + 15) / 16);
  size_t sm = 16 * (A + XPAD) * sizeof(bf16);
  hipLaunchKernelGGL(dec_bwd_cell_kernel, grid, dim3(256), sm, st, dsp, nchunk, Ws, dC_dir, dH_dir, dh_rec, dc_carry,
                     act, c_now, c_prev, ds_out, dz, B, H, A);
}
void launch_dec_bwd_dz(const bf16* dz, const bf16* Wc, const bf16* Wic, const float* dX_dir,
                       const float* dCTX_dir_prev, float* dx_out, float* dctx_prev_out, float* dh_rec, int B, int E,
                       int H, int A, hipStream_t st) {
  dim3 grid(1 + (H + 63) / 64, (B + 15) / 16);
  size_t sm = 16 * (E + XPAD) * sizeof(bf16);
  hipLaunchKernelGGL(dec_bwd_dz_kernel, grid, dim3(256), sm, st, dz, Wc, Wic, dX_dir, dCTX_dir_prev, dx_out,
                     dctx_prev_out, dh_rec, B, E, H, A);
}
