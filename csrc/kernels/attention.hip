// Bahdanau attention with coverage, one decoder step per launch pair
// (reference attention_decoder.py:79-129, model.py:463-480).
//
//   e_i   = sum_k v_k tanh(F[i,k] + s[k] + w_c[k] * cov_i)      (F = W_h enc_out, s = W_s[c;h] + b)
//   a     = masked softmax(e)                                    (== softmax*mask renormalised)
//   cov'  = cov + a           covloss = sum_i min(a_i, cov_i)
//   ctx   = sum_i a_i E[i,:]
//
// Two layouts of the [B,T,A] encoder features are used (both fit trivially in HBM):
//  * row-major F/E [B][T][A] -- lanes on the feature axis (8 bf16 = one 16-B load);
//  * transposed Ft [B][A][T] (score kernel) -- lanes on the position axis, so the score e_i
//    reduces over k inside a lane (no cross-lane reduction at all), the per-k parameters
//    (s_k, v_k, w_c_k) are wave-uniform scalar loads, and the 8 waves of a block split the
//    k axis (summed once in LDS).
// These multi-block-per-row kernels serve B < 128 and the A = 1024 backward; the row-resident
// kernels of attention_row.hip take the rest.
// The v / w_c / F gradients are NOT accumulated per step: the backward step stores
// de_t, and attn_bwd_feat recomputes tanh once over all steps after the loop.  The
// recurrent path only carries ds_t (atomically accumulated across position chunks) and
// dcov_t.
#include "common.h"
#include <stdlib.h>

#define SCORE_POS 128  // positions per block in the lanes-over-positions kernels (2 per lane)
// waves per block (template SW): each takes A/SW of the feature axis.  16 waves (A % 128 == 0)
// keep 4 waves per SIMD resident at B = 64 -- these kernels are latency-bound there.

#include "attn_common.h"

// ---------------------------------------------------------------- forward: scores
// grid (ceil(T/128), B / REP), SW*64 threads.  Ft: [B/REP][A][T] bf16, T even.  Each lane owns
// 2 positions; the SW waves split the feature axis; per 8-feature batch all 8 Ft loads are
// issued before the tanh work and s/v/w_c come in as wave-uniform vectors.  REP rows share
// one Ft row (beam search: the beam hypotheses of an article attend over the same encoder
// features), so Ft is read once per article instead of once per hypothesis.
template <int SW, int REP>
__global__ __launch_bounds__(SW * 64) void attn_score_kernel(
    const bf16* __restrict__ Ft, const float* __restrict__ s, const float* __restrict__ v,
    const float* __restrict__ wc, const float* __restrict__ cov, const int* __restrict__ lens,
    float* __restrict__ e, int T, int A, int xcd) {
  const Dot2Sel dsel = dot2_sel();  // F pair selectors for fadd_bf2
  __shared__ float red[SW][REP][SCORE_POS];
  // XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs, so consecutive
  // ids would put the position chunks of one Ft row on different XCDs.  A row is T*2 bytes
  // (800 at T = 400, not a multiple of the 128-byte line): the lines two chunks share were
  // then fetched from HBM once per XCD (FETCH_SIZE 1.45x the Ft bytes).  Giving each XCD a
  // contiguous range of (row, chunk) keeps the shared lines in one L2.
  int bx = blockIdx.x, by = blockIdx.y;
  {
    const int nx = gridDim.x, ntot = nx * gridDim.y;
    if (xcd && (ntot & 7) == 0) {
      const int id = blockIdx.y * nx + blockIdx.x;
      const int L = (id & 7) * (ntot >> 3) + (id >> 3);
      by = L / nx;
      bx = L - by * nx;
    }
  }
  const int b = by;  // Ft row (article)
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int len = (int)DCHECK_IDX(lens[b], 1, T + 1, CHK_ATTN_LEN);
  const int pb = bx * SCORE_POS;
  if (pb >= len) return;  // uniform: masked positions are never read by the softmax
  const int p = pb + 2 * lane;
  const int pc = p < T ? p : 0;
  f32x2 cc[REP];
#pragma unroll
  for (int q = 0; q < REP; ++q) {
    cc[q] = f32x2{0.f, 0.f};
    if (cov) {
      const float2 c2 = *reinterpret_cast<const float2*>(cov + ((size_t)b * REP + q) * T + pc);
      cc[q] = f32x2{c2.x, c2.y};
    }
  }
  const int ka = wid * (A / SW), kb = ka + A / SW;
  const bf16* fp = Ft + ((size_t)b * A) * T + pc;
  f32x2 acc[REP];
#pragma unroll
  for (int q = 0; q < REP; ++q) acc[q] = f32x2{0.f, 0.f};
  float vsum = 0.f;
  for (int k = ka; k < kb; k += 8) {
    uint32_t raw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) raw[i] = *reinterpret_cast<const uint32_t*>(fp + (size_t)(k + i) * T);
    float vk[8], wk[8];
    *reinterpret_cast<float4*>(vk) = *reinterpret_cast<const float4*>(v + k);
    *reinterpret_cast<float4*>(vk + 4) = *reinterpret_cast<const float4*>(v + k + 4);
    if (wc) {
      *reinterpret_cast<float4*>(wk) = *reinterpret_cast<const float4*>(wc + k);
      *reinterpret_cast<float4*>(wk + 4) = *reinterpret_cast<const float4*>(wc + k + 4);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) wk[i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) vsum += vk[i];
#pragma unroll
    for (int q = 0; q < REP; ++q) {
      const float* sb = s + ((size_t)b * REP + q) * A;
      float sk[8];
      *reinterpret_cast<float4*>(sk) = *reinterpret_cast<const float4*>(sb + k);
      *reinterpret_cast<float4*>(sk + 4) = *reinterpret_cast<const float4*>(sb + k + 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        // y = 2 log2(e) (F + s_k + w_k cov) for both positions at once (F stored pre-scaled)
        const f32x2 base = fma2(splat2(wk[i] * K2LOG2E), cc[q], splat2(sk[i] * K2LOG2E));
        const f32x2 y = fadd_bf2(raw[i], base, dsel);
        acc[q] = fma2(splat2(vk[i]), rsig2(y), acc[q]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < REP; ++q) {
    red[wid][q][2 * lane] = vsum - 2.0f * acc[q].x;
    red[wid][q][2 * lane + 1] = vsum - 2.0f * acc[q].y;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < REP * SCORE_POS; t += SW * 64) {
    const int q = t / SCORE_POS, pp = t % SCORE_POS, pos = pb + pp;
    float r = 0.f;
#pragma unroll
    for (int w = 0; w < SW; ++w) r += red[w][q][pp];
    if (pos < len) e[((size_t)b * REP + q) * T + pos] = r;
  }
}

// ------------------------------------------------- forward: softmax, coverage, context
// grid (A/64 feature chunks, B / REP).  Every block recomputes the softmax of its REP rows
// (T floats each); block x==0 also publishes a_t, cov_{t+1} and the coverage loss.  The REP
// rows share one E row, read once for all of them.
#define MAXT 2048
template <int REP>
__global__ __launch_bounds__(256) void attn_softmax_ctx_kernel(
    const float* __restrict__ e, const bf16* __restrict__ E, const int* __restrict__ lens,
    const float* __restrict__ cov, float* __restrict__ a_out, float* __restrict__ cov_out,
    float* __restrict__ covloss, float* __restrict__ ctx, bf16* __restrict__ ctx_bf, int T, int A) {
  __shared__ float sa[REP][MAXT / (REP > 1 ? 2 : 1)];
  __shared__ float red[8];
  __shared__ float part[4][REP][64];
  const int b = blockIdx.y;  // E row (article)
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int len = (int)DCHECK_IDX(lens[b], 1, T + 1, CHK_ATTN_LEN);
#pragma unroll
  for (int q = 0; q < REP; ++q) {
    const size_t row = (size_t)b * REP + q;
    const float* er = e + row * T;
    float m = -INFINITY;
    for (int i = tid; i < len; i += 256) m = fmaxf(m, er[i]);
    m = block_max<256>(m, red);
    float sum = 0.f;
    for (int i = tid; i < len; i += 256) {
      float x = fexp(er[i] - m);
      sa[q][i] = x;
      sum += x;
    }
    sum = block_sum<256>(sum, red);
    const float inv = 1.0f / sum;
    for (int i = tid; i < len; i += 256) sa[q][i] *= inv;
  }
  __syncthreads();
  if (blockIdx.x == 0) {
#pragma unroll
    for (int q = 0; q < REP; ++q) {
      const size_t row = (size_t)b * REP + q;
      float cl = 0.f;
      for (int i = tid; i < T; i += 256) {
        const float a = i < len ? sa[q][i] : 0.f;
        a_out[row * T + i] = a;
        if (cov_out) {
          const float c = cov ? cov[row * T + i] : 0.f;
          cov_out[row * T + i] = c + a;
          cl += fminf(a, c);
        }
      }
      if (covloss) {
        cl = block_sum<256>(cl, red);
        if (tid == 0) covloss[row] = cl;
      }
    }
  }
  // context: 64 features per block; lane = (pos sub-index 0..7, feature group 0..7)
  const int f0 = blockIdx.x * 64;
  const int ps = lane >> 3, fg = lane & 7;
  float acc[REP][8];
#pragma unroll
  for (int q = 0; q < REP; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[q][j] = 0.f;
  const bf16* Eb = E + (size_t)b * T * A + f0 + fg * 8;
#pragma unroll 4
  for (int i = wid * 8 + ps; i < len; i += 32) {
    bf16x8 x = ld8(Eb + (size_t)i * A);
#pragma unroll
    for (int q = 0; q < REP; ++q) {
      const float a = sa[q][i];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[q][j] += a * bf2f(x[j]);
    }
  }
#pragma unroll
  for (int q = 0; q < REP; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = acc[q][j];
      x += dpp_f<DPP_ROR8>(x);
      x = sum_x32(sum_x16(x));
      acc[q][j] = x;
    }
  if (ps == 0) {
#pragma unroll
    for (int q = 0; q < REP; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) part[wid][q][fg * 8 + j] = acc[q][j];
  }
  __syncthreads();
  if (tid < 64 * REP) {
    const int q = tid >> 6, f = tid & 63;
    const size_t row = (size_t)b * REP + q;
    const float c = part[0][q][f] + part[1][q][f] + part[2][q][f] + part[3][q][f];
    ctx[row * A + f0 + f] = c;
    if (ctx_bf) ctx_bf[row * A + f0 + f] = f2bf(c);
  }
}


// ------------------------------------------ backward step, fused: da, de, ds, dcov
// One pass over the rows E_i (encoder outputs) and F_i (W_h features) of a block's positions:
//   da_i   = r_i + dctx . E_i,        r_i = Ga_i + dcov_next_i + g_cl [a_i <= cov_i]
//   S      = sum_j a_j da_j = sum_j a_j r_j + dctx . ctx     (ctx = sum_j a_j E_j, forward)
//   de_i   = a_i (da_i - S)
//   ds_k  += sum_i de_i v_k sech2(u_ik)                        (atomic, ds pre-zeroed)
//   dcov_i = dcov_next_i + g_cl [a_i > cov_i] + de_i sum_k v_k w_c_k sech2(u_ik)
// S needs no pass over da (its dctx.E half is dctx.ctx), so every block is independent and one
// launch per decoder step does it all.  Lanes on the feature axis (8 per lane, NK blocks of 512);
// per group of positions the partial dctx.E_i dots are reduced with a butterfly
// reduce-scatter (the lanes of position q end up holding its total), de_q is broadcast with
// v_readlane, then the r-form tanh pass (packed fp32, see rsig2) accumulates ds and the dcov
// partials, reduced the same way.   v_k sech2(u) = 4 v_k r (1 - r)  ->  ds_k = 4 v_k sum_i de_i q_ik.
// The row-resident attn_bwd_row (attention_row.hip) replaces this kernel at A = 512 and B >= 128.

// Same math with 4 positions per group (NG4 groups per wave): the E/F rows in flight per
// lane halve (32 instead of 64 VGPRs), which buys a third wave per SIMD at the 168-VGPR cap.
// NK feature blocks of 512 per lane (NK = 2: A = 1024, config #5).
template <int NG4, int OCC, int NK>
__global__ __launch_bounds__(256, OCC) void attn_bwd_step4_kernel(
    const bf16* __restrict__ E, const bf16* __restrict__ F, const float* __restrict__ s,
    const float* __restrict__ v, const float* __restrict__ wc, const float* __restrict__ cov,
    const float* __restrict__ a, const float* __restrict__ dctx, const float* __restrict__ ctx,
    const float* __restrict__ Ga, const float* __restrict__ dcov_next, const float* __restrict__ gcl,
    const int* __restrict__ lens, float* __restrict__ de_out, float* __restrict__ ds,
    float* __restrict__ dcov_out, int T, int A) {
  const Dot2Sel dsel = dot2_sel();  // F pair selectors for fadd_bf2
  constexpr int PW = 4 * NG4;  // positions per wave
  constexpr int PB = 4 * PW;   // positions per block
  static_assert(PW == 32 || PW == 16 || PW == 64, "lane -> position map needs a power of two <= 64");
  __shared__ float red[8];
  __shared__ float part[4][512 * NK];
  const int b = blockIdx.y;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int len = (int)DCHECK_IDX(lens[b], 1, T + 1, CHK_ATTN_LEN);
  const size_t rb = (size_t)b * T;
  const int p0 = blockIdx.x * PB + wid * PW;
  if (blockIdx.x * PB >= len) {  // whole block masked: only pass dcov through
    for (int i = tid; i < PB; i += 256) {
      const int p = blockIdx.x * PB + i;
      if (p < T) {
        if (dcov_out) dcov_out[rb + p] = dcov_next ? dcov_next[rb + p] : 0.f;
        de_out[rb + p] = 0.f;
      }
    }
    return;
  }
  const float g = gcl ? gcl[b] : 0.f;
  const bf16* Eb = E + (size_t)b * T * A;
  const bf16* Fb = F + (size_t)b * T * A;
  int k0c[NK];
#pragma unroll
  for (int kb = 0; kb < NK; ++kb) k0c[kb] = min(kb * 512 + lane * 8, A - 8);
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 fr[NK][4], er[NK][4];
#define LOAD4(dst, base, pg)                                                               \
  {                                                                                        \
    _Pragma("unroll") for (int q = 0; q < 4; ++q) {                                        \
      const int pq = min((pg) + q, len - 1);                                               \
      _Pragma("unroll") for (int kb = 0; kb < NK; ++kb) dst[kb][q] =                       \
          __builtin_bit_cast(u32x4, ld8(base + (size_t)pq * A + k0c[kb]));                 \
    }                                                                                      \
  }
  if (p0 < len) {
    LOAD4(er, Eb, p0);
    LOAD4(fr, Fb, p0);
  }
  float dk[NK][8];
  f32x2 s2[NK][4], w2[NK][4], v4w[NK][4], acc[NK][4];
#pragma unroll
  for (int kb = 0; kb < NK; ++kb) {
    const int k0 = kb * 512 + lane * 8;
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      float sv[2], wv[2], vv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = k0 + 2 * jp + h;
        const bool ok = k < A;
        sv[h] = ok ? s[(size_t)b * A + k] : 0.f;
        vv[h] = ok ? v[k] : 0.f;
        wv[h] = (ok && wc) ? wc[k] : 0.f;
        dk[kb][2 * jp + h] = ok ? dctx[(size_t)b * A + k] : 0.f;
      }
      s2[kb][jp] = f32x2{sv[0], sv[1]} * K2LOG2E;
      w2[kb][jp] = f32x2{wv[0], wv[1]} * K2LOG2E;
      v4w[kb][jp] = f32x2{4.f * vv[0] * wv[0], 4.f * vv[1] * wv[1]};
      acc[kb][jp] = f32x2{0.f, 0.f};
    }
  }
  float a_l = 0.f, r_l = 0.f, c_l = 0.f, dn_l = 0.f;
  {
    const int p = p0 + (lane & (PW - 1));
    if (p < len) {
      const size_t ix = rb + p;
      a_l = a[ix];
      c_l = cov ? cov[ix] : 0.f;
      r_l = (Ga ? Ga[ix] : 0.f) + (dcov_next ? dcov_next[ix] : 0.f);
      if (gcl && a_l <= c_l) r_l += g;
    }
    if (p < T && dcov_next) dn_l = dcov_next[rb + p];
  }
  float S = 0.f;
  for (int i = tid; i < len; i += 256) {
    const size_t ix = rb + i;
    const float ai = a[ix];
    float r = (Ga ? Ga[ix] : 0.f) + (dcov_next ? dcov_next[ix] : 0.f);
    if (gcl && ai <= (cov ? cov[ix] : 0.f)) r += g;
    S += ai * r;
  }
  for (int k = tid; k < A; k += 256) S += dctx[(size_t)b * A + k] * ctx[(size_t)b * A + k];
  S = block_sum<256>(S, red);
  const int b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1;
  const int qm = 2 * b5 + b4;
#pragma unroll
  for (int grp = 0; grp < NG4; ++grp) {
    const int pg = p0 + grp * 4;
    if (pg >= len) {
      for (int i = lane; i < 4 * (NG4 - grp); i += 64) {
        const int p = pg + i;
        if (p < T) {
          de_out[rb + p] = 0.f;
          if (dcov_out) dcov_out[rb + p] = dcov_next ? dcov_next[rb + p] : 0.f;
        }
      }
      break;
    }
    const bool more = grp + 1 < NG4 && pg + 4 < len;
    float pd[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x2 d2 = f32x2{0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < NK; ++kb)
#pragma unroll
        for (int jp = 0; jp < 4; ++jp)
          d2 = fma2(bf2pair(er[kb][q][jp]), f32x2{dk[kb][2 * jp], dk[kb][2 * jp + 1]}, d2);
      pd[q] = d2.x + d2.y;
    }
    if (more) LOAD4(er, Eb, pg + 4);
    const float dot = bfly4(pd, b5, b4);
    const int src = grp * 4 + qm;
    const float a_q = __shfl(a_l, src, 64), r_q = __shfl(r_l, src, 64);
    const float c_q = __shfl(c_l, src, 64), dn_q = __shfl(dn_l, src, 64);
    const float de_q = (pg + qm < len) ? a_q * (r_q + dot - S) : 0.f;
    float dcv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float de = rdlane(de_q, ((q >> 1) << 5) | ((q & 1) << 4));
      const float c = rdlane(c_l, grp * 4 + q);
      f32x2 dc2 = f32x2{0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < NK; ++kb)
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
          const f32x2 y = fadd_bf2(fr[kb][q][jp], fma2(w2[kb][jp], splat2(c), s2[kb][jp]), dsel);
          const f32x2 r = rsig2(y);
          const f32x2 qv = fma2(-r, r, r);
          acc[kb][jp] = fma2(qv, splat2(de), acc[kb][jp]);
          dc2 = fma2(qv, v4w[kb][jp], dc2);
        }
      dcv[q] = dc2.x + dc2.y;
    }
    if (more) LOAD4(fr, Fb, pg + 4);
    const float hc = bfly4(dcv, b5, b4);
    if ((lane & 15) == 0) {
      const int p = pg + qm;
      if (p < T) {
        const size_t ix = rb + p;
        de_out[ix] = de_q;
        if (dcov_out) {
          float r = dn_q;
          if (p < len) {
            r += de_q * hc;
            if (gcl && a_q > c_q) r += g;
          }
          dcov_out[ix] = r;
        }
      }
    }
  }
#undef LOAD4
#pragma unroll
  for (int kb = 0; kb < NK; ++kb) {
    const int k0 = kb * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = k0 + j < A;
      part[wid][kb * 512 + lane * 8 + j] = ok ? 4.f * v[ok ? k0 + j : 0] * acc[kb][j >> 1][j & 1] : 0.f;
    }
  }
  __syncthreads();
  float* out = ds + (size_t)b * A;
  for (int k = tid; k < A; k += 256) {
    const float x = part[0][k] + part[1][k] + part[2][k] + part[3][k];
    atomicAdd(out + k, x);
  }
}

// ------------------------------------------------------ post-loop: dF, dv, dw_c
// dF[b,i,k] = sum_t de[t,b,i] v_k sech2(u_tik); dv_k = sum de tanh(u); dwc_k = sum de v_k sech2 cov.
// Lanes on features (8 per lane), each wave keeps 4 positions x 8 features of dF in
// registers across all D steps; de / cov are wave-uniform scalar loads.
template <int NPW, int OCC>
__global__ __launch_bounds__(256, OCC) void attn_bwd_feat_kernel(
    const bf16* __restrict__ F, const float* __restrict__ S_all, const float* __restrict__ v,
    const float* __restrict__ wc, const float* __restrict__ cov_all, const float* __restrict__ de_all,
    const int* __restrict__ lens, bf16* __restrict__ dF, float* __restrict__ dv, float* __restrict__ dwc,
    int D, int B, int T, int A, int nslot, const int* __restrict__ dlen) {
  __shared__ float pv[4][512];
  __shared__ float pw[4][512];
  const int b = blockIdx.y;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int len = (int)DCHECK_IDX(lens[b], 1, T + 1, CHK_ATTN_LEN);
  const int kbase = blockIdx.z * 512;
  const int k0 = kbase + lane * 8;
  const bool kok = k0 < A;
  const int p0 = blockIdx.x * (4 * NPW) + wid * NPW;  // NPW positions per wave
  // r-form (see rsig2): with r = 1/(1 + 2^y),
  //   dF  = 4 v sum_t de r(1-r),  dv = sum_t de - 2 sum_t de r,  dwc = 4 v sum_t de cov r(1-r)
  f32x2 w2[4], accv[4], accw[4];
  float vk[8], sum_de = 0.f;
#pragma unroll
  for (int jp = 0; jp < 4; ++jp) {
    float wv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = 2 * jp + h;
      const bool ok = kok && k0 + j < A;
      vk[j] = ok ? v[k0 + j] : 0.f;
      wv[h] = (ok && wc) ? wc[k0 + j] : 0.f;
    }
    w2[jp] = f32x2{wv[0], wv[1]} * K2LOG2E;
    accv[jp] = f32x2{0.f, 0.f};
    accw[jp] = f32x2{0.f, 0.f};
  }
  float adv[8], adw[8];
  if (p0 < len && kok) {
    const int np = min(NPW, len - p0);
    f32x2 fs[NPW][4], acc[NPW][4];
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      const int p = min(p0 + q, T - 1);
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 fw = __builtin_bit_cast(u32x4, ld8(F + ((size_t)b * T + p) * A + k0));
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        fs[q][jp] = bf2pair(fw[jp]);  // F is stored pre-scaled (attn_common.h)
        acc[q][jp] = f32x2{0.f, 0.f};
      }
    }
    // steps past the row's last loss-weighted decoder step have de = 0 (dlen, nullable)
    const int Dl = dlen ? min(D, dlen[b]) : D;
    for (int t = 0; t < Dl; ++t) {
      const float* st = S_all + ((size_t)t * B + b) * A + k0;
      const float4 s0 = *reinterpret_cast<const float4*>(st);
      const float4 s1 = *reinterpret_cast<const float4*>(st + 4);
      const f32x2 s2[4] = {f32x2{s0.x, s0.y} * K2LOG2E, f32x2{s0.z, s0.w} * K2LOG2E,
                           f32x2{s1.x, s1.y} * K2LOG2E, f32x2{s1.z, s1.w} * K2LOG2E};
      const size_t rb = ((size_t)t * B + b) * T + p0;
#pragma unroll
      for (int q = 0; q < NPW; ++q) {
        if (q < np) {
          const float de = de_all[rb + q];
          const float c = cov_all ? cov_all[rb + q] : 0.f;
          const float dec = de * c;
          sum_de += de;
#pragma unroll
          for (int jp = 0; jp < 4; ++jp) {
            const f32x2 y = fma2(w2[jp], splat2(c), s2[jp]) + fs[q][jp];
            const f32x2 r = rsig2(y);
            const f32x2 qv = fma2(-r, r, r);
            acc[q][jp] = fma2(qv, splat2(de), acc[q][jp]);
            accv[jp] = fma2(r, splat2(de), accv[jp]);
            accw[jp] = fma2(qv, splat2(dec), accw[jp]);
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      if (p0 + q < T) {  // bf16 straight into the GEMM operand; zeros past len
        bf16x8 o8;
#pragma unroll
        for (int j = 0; j < 8; ++j) o8[j] = f2bf(q < np ? 4.0f * vk[j] * acc[q][j >> 1][j & 1] : 0.f);
        *reinterpret_cast<bf16x8*>(dF + ((size_t)b * T + p0 + q) * A + k0) = o8;
      }
    }
  } else if (kok) {  // fully masked positions of this wave: dF = 0 (no separate memset)
#pragma unroll
    for (int q = 0; q < NPW; ++q)
      if (p0 + q < T) *reinterpret_cast<bf16x8*>(dF + ((size_t)b * T + p0 + q) * A + k0) = zero8();
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    adv[j] = sum_de - 2.0f * accv[j >> 1][j & 1];
    adw[j] = 4.0f * vk[j] * accw[j >> 1][j & 1];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    pv[wid][lane * 8 + j] = adv[j];
    pw[wid][lane * 8 + j] = adw[j];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 512; k += 256) {
    const int kk = kbase + k;
    if (kk < A) {
      const float x = pv[0][k] + pv[1][k] + pv[2][k] + pv[3][k];
      const float y = pw[0][k] + pw[1][k] + pw[2][k] + pw[3][k];
      // nslot (power of two) partial rows: the B x T/16 workgroups would otherwise all add
      // into the same A addresses, and same-address atomics serialise at L2
      const size_t so = (size_t)((blockIdx.x + blockIdx.y * gridDim.x) & (nslot - 1)) * A;
      if (x != 0.f) atomicAdd(dv + so + kk, x);
      if (dwc && y != 0.f) atomicAdd(dwc + so + kk, y);
    }
  }
}

void launch_attn_score(const bf16* Ft, const float* s, const float* v, const float* wc, const float* cov,
                       const int* lens, float* e, int B, int T, int A, int rep, hipStream_t st) {
  dim3 grid((T + SCORE_POS - 1) / SCORE_POS, B / rep);
  // rep = 1 (training, B < 128): 8 waves per block measured 23.3 vs 24.5 us; rep = 4 (beam
  // decode through these kernels): 16 waves when A % 128 == 0, 14.5 vs 14.7 ms per batch
  const bool w16 = A % 128 == 0 && rep > 1;
#define LS(SW, RP) hipLaunchKernelGGL((attn_score_kernel<SW, RP>), grid, dim3(SW * 64), 0, st, Ft, s, v, wc, cov, lens, e, T, A, 1)
  if (rep == 4) { if (w16) LS(16, 4); else LS(8, 4); }
  else if (rep == 2) { if (w16) LS(16, 2); else LS(8, 2); }
  else { if (w16) LS(16, 1); else LS(8, 1); }
#undef LS
}
void launch_attn_softmax_ctx(const float* e, const bf16* E, const int* lens, const float* cov, float* a_out,
                             float* cov_out, float* covloss, float* ctx, bf16* ctx_bf, int B, int T, int A, int rep,
                             hipStream_t st) {
  dim3 grid(A / 64, B / rep);
#define LC(RP) hipLaunchKernelGGL(attn_softmax_ctx_kernel<RP>, grid, dim3(256), 0, st, e, E, lens, cov, a_out, cov_out, \
                                  covloss, ctx, ctx_bf, T, A)
  if (rep == 4) LC(4);
  else if (rep == 2) LC(2);
  else LC(1);
#undef LC
}
int attn_nchunk(int T) { return (T + 63) / 64; }
void launch_attn_bwd_step(const bf16* E, const bf16* F, const float* s, const float* v, const float* wc,
                          const float* cov, const float* a, const float* dctx, const float* ctx, const float* Ga,
                          const float* dcov_next, const float* gcl, const int* lens, float* de_out, float* ds,
                          float* dcov_out, int B, int T, int A, hipStream_t st) {
  // A <= 512: 4-position groups, 8 groups per wave (128 positions per block), 2 waves per SIMD
  // cap: 54 us vs 61 us for an 8-position kernel at B = 256, T = 400 (tools/attn_micro.py).
  // A = 1024 (config #5): 16 features per lane at 208 VGPRs (2 waves per SIMD), 64 positions
  // per wave = 256 per block so each row's S prologue is paid by 4 blocks, not 7: 198 us vs
  // 250 us per launch at 256 rows x T = 800 (tools/attn_bwd_a1024_micro.py).
  if (A <= 512)
    hipLaunchKernelGGL((attn_bwd_step4_kernel<8, 2, 1>), dim3((T + 127) / 128, B), dim3(256), 0, st, E, F, s, v, wc,
                       cov, a, dctx, ctx, Ga, dcov_next, gcl, lens, de_out, ds, dcov_out, T, A);
  else
    hipLaunchKernelGGL((attn_bwd_step4_kernel<16, 2, 2>), dim3((T + 255) / 256, B), dim3(256), 0, st, E, F, s, v, wc,
                       cov, a, dctx, ctx, Ga, dcov_next, gcl, lens, de_out, ds, dcov_out, T, A);
}
void launch_attn_bwd_feat(const bf16* F, const float* S_all, const float* v, const float* wc, const float* cov_all,
                          const float* de_all, const int* lens, bf16* dF, float* dv, float* dwc, int D, int B, int T,
                          int A, int nslot, hipStream_t st, const int* dlen) {
  // 4 positions per wave capped at 128 VGPRs = 4 waves/SIMD (a few prologue spills): 1.51 ms
  // vs 1.64 ms uncapped at 3 waves/SIMD and 1.65 ms with 2 positions per wave (B = 256,
  // T = 400, D = 100)
  dim3 grid((T + 15) / 16, B, (A + 511) / 512);
  hipLaunchKernelGGL((attn_bwd_feat_kernel<4, 4>), grid, dim3(256), 0, st, F, S_all, v, wc, cov_all, de_all, lens, dF,
                     dv, dwc, D, B, T, A, nslot, dlen);
}
