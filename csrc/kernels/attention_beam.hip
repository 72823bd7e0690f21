// Beam-decode attention with coverage, one article's encoder rows read ONCE for all its beam
// hypotheses (SURVEY K8-K12 in decode mode; reference attention_decoder.py:79-129,
// model.py:367-443 -- the decode graph runs the attention of all beam_size hypotheses of one
// article against the same encoder states).
//
// The row kernel (attention_row.hip) runs one workgroup per hypothesis, so the beam hypotheses
// of an article each pull its F = W_h enc_out and E = enc_out rows (800 KB at T = 400, A = 512)
// through L2: 4x the encoder bytes per step.  Here:
//
//   attn_beam_part  grid (articles x S chunks of the article's positions): a workgroup streams
//                   the chunk's F / E rows once and computes, for every hypothesis r of the
//                   article, the scores e_ri = sum_k v_k tanh(F_ik + s_rk + w_k cov_ri) (the r-form
//                   of attn_common.h), an online softmax (chunk max m, sum l) and the context
//                   partial sum_i exp(e_ri - m) E_i; raw scores go to e_buf, (m, l) and the partial
//                   to pm / pctx.  The coverage gather of the beam step happens here too:
//                   cov_ri = cov_src[g_r, i] + a_src[g_r, i] (g_r = the hypothesis' parent row),
//                   kept in cov_keep for the next step.
//   attn_beam_merge grid R (hypotheses): M = max_c m_c, L = sum_c l_c e^(m_c - M),
//                   ctx = sum_c e^(m_c - M) pctx_c / L, a_i = e^(e_i - M) / L.
//
// S chunks per article keep >= 512 workgroups busy at 64 articles (the scores are tanh-bound:
// 4 hypotheses x 8 features x 2 transcendentals per lane and position).
#include "attn_common.h"
#include "launchers.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBeamRB = 4;   // hypotheses per article (rep)
constexpr int kBeamNW = 4;   // waves per workgroup (2 workgroups per CU at <= 256 VGPRs)

struct Rows1 {
  u32x4 x[4];  // 4 positions x 8 bf16 features of one tensor (A = 512: lane * 8)
};

__device__ __forceinline__ void load_rows1(Rows1& r, const bf16* base, int p0, int plast, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = min(p0 + q, plast);
    r.x[q] = __builtin_bit_cast(u32x4, ld8(base + (size_t)p * 512 + lane * 8));
  }
}

}  // namespace

// grid Na * S; block kBeamNW waves.  A = 512 (8 features per lane), RB = 4 hypotheses per article.
template <int NW, int RB>
__global__ __launch_bounds__(NW * 64) void attn_beam_part_kernel(
    const bf16* __restrict__ F, const bf16* __restrict__ E, const float* __restrict__ s,
    const float* __restrict__ v, const float* __restrict__ wc,
    const float* __restrict__ cov,      // [R][T] coverage as is (no gather), or nullptr
    const float* __restrict__ cov_src,  // [R][T] parent coverage (gather mode), or nullptr
    const float* __restrict__ a_src,    // [R][T] parent attention (gather mode)
    float* __restrict__ cov_keep,       // [R][T] gathered coverage out (gather mode)
    const int* __restrict__ cg,         // [R] parent rows (gather mode)
    const int* __restrict__ lens,       // [Na]
    float* __restrict__ e_buf,          // [R][T] raw scores
    float* __restrict__ pm,             // [R][S][2] chunk (max, sum exp)
    float* __restrict__ pctx,           // [R][S][512] chunk context partials (relative to the chunk max)
    int T, int S) {
  constexpr int A = 512;
  __shared__ float part[NW][RB][A];
  __shared__ float wm[NW][RB], wl[NW][RB];
  const int a = blockIdx.x / S, c = blockIdx.x % S;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int len = (int)DCHECK_IDX(lens[a], 1, T + 1, CHK_ATTN_LEN);
  // chunk c of the article's len positions, in whole 4-position groups
  const int ng = (len + 3) >> 2, gpc = (ng + S - 1) / S;
  const int p0 = 4 * gpc * c, p1 = min(len, 4 * gpc * (c + 1));
  const int ngrp = p1 > p0 ? (p1 - p0 + 3) >> 2 : 0;
  const bf16* Fb = F + (size_t)a * T * A;
  const bf16* Eb = E + (size_t)a * T * A;
  const int qm = lane >> 4, b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1;
  const int r0 = a * RB;
  const bool gather = cg != nullptr;
  size_t cb[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r)
    cb[r] = gather ? (size_t)DCHECK_IDX(cg[r0 + r], 0, (int)gridDim.x / S * RB, CHK_BEAM_PARENT) * T
                   : (size_t)(r0 + r) * T;
  Rows1 fA, eA, fB, eB;
  float cA[RB], cBv[RB];
  auto load = [&](int grp, Rows1& f, Rows1& e, float (&cv)[RB]) {
    const int q0 = p0 + 4 * grp;
    load_rows1(f, Fb, q0, len - 1, lane);
    load_rows1(e, Eb, q0, len - 1, lane);
    const int p = min(q0 + qm, len - 1);
#pragma unroll
    for (int r = 0; r < RB; ++r)
      cv[r] = gather ? cov_src[cb[r] + p] + a_src[cb[r] + p] : (cov ? cov[cb[r] + p] : 0.f);
  };
  if (wid < ngrp) load(wid, fA, eA, cA);
  // per-lane feature parameters (pre-scaled for the r-form) and per-hypothesis query
  f32x2 w2[4], v2[4], s2[RB][4], acc[RB][4];
  float vsum = 0.f;
  const int k0 = lane * 8;
#pragma unroll
  for (int jp = 0; jp < 4; ++jp) {
    const float2 vv = *reinterpret_cast<const float2*>(v + k0 + 2 * jp);
    const float2 wv = wc ? *reinterpret_cast<const float2*>(wc + k0 + 2 * jp) : make_float2(0.f, 0.f);
    w2[jp] = f32x2{wv.x, wv.y} * K2LOG2E;
    v2[jp] = f32x2{vv.x, vv.y};
    vsum += vv.x + vv.y;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const float2 sv = *reinterpret_cast<const float2*>(s + (size_t)(r0 + r) * A + k0 + 2 * jp);
      s2[r][jp] = f32x2{sv.x, sv.y} * K2LOG2E;
      acc[r][jp] = f32x2{0.f, 0.f};
    }
  }
  float m_w[RB], l_w[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) { m_w[r] = -INFINITY; l_w[r] = 0.f; }
  auto compute = [&](int grp, const Rows1& f, const Rows1& e, const float (&cv)[RB]) {
    const int pq = p0 + 4 * grp + qm;  // this lane group's position
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      float pd[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float cq = rdlane(cv[r], 16 * q);
        f32x2 d2 = f32x2{0.f, 0.f};
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
          const f32x2 y = fma2(bf2pair(f.x[q][jp]), splat2(K2LOG2E), fma2(w2[jp], splat2(cq), s2[r][jp]));
          d2 = fma2(v2[jp], rsig2(y), d2);
        }
        pd[q] = vsum - 2.0f * (d2.x + d2.y);  // the lane's share of e (bfly4 sums the lanes)
      }
      float eq = bfly4(pd, b5, b4);
      if (pq >= p1) eq = -INFINITY;
      if ((lane & 15) == 0 && pq < p1) {
        e_buf[(size_t)(r0 + r) * T + pq] = eq;
        if (gather && cov_keep) cov_keep[(size_t)(r0 + r) * T + pq] = cv[r];
      }
      const float e0 = rdlane(eq, 0), e1 = rdlane(eq, 16), e2 = rdlane(eq, 32), e3 = rdlane(eq, 48);
      const float mn = fmaxf(m_w[r], fmaxf(fmaxf(e0, e1), fmaxf(e2, e3)));  // e0 valid: p0 + 4 grp < p1
      const float sc = m_w[r] == -INFINITY ? 0.f : fexp(m_w[r] - mn);
      const float q0 = fexp(e0 - mn), q1 = fexp(e1 - mn), q2 = fexp(e2 - mn), q3 = fexp(e3 - mn);
      l_w[r] = l_w[r] * sc + ((q0 + q1) + (q2 + q3));
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        f32x2 a2 = acc[r][jp] * sc;
        a2 = fma2(bf2pair(e.x[0][jp]), splat2(q0), a2);
        a2 = fma2(bf2pair(e.x[1][jp]), splat2(q1), a2);
        a2 = fma2(bf2pair(e.x[2][jp]), splat2(q2), a2);
        acc[r][jp] = fma2(bf2pair(e.x[3][jp]), splat2(q3), a2);
      }
      m_w[r] = mn;
    }
  };
  for (int g = wid; g < ngrp;) {
    const int g1 = g + NW;
    if (g1 < ngrp) load(g1, fB, eB, cBv);
    compute(g, fA, eA, cA);
    if (g1 >= ngrp) break;
    const int g2 = g1 + NW;
    if (g2 < ngrp) load(g2, fA, eA, cA);
    compute(g1, fB, eB, cBv);
    g = g2;
  }
  // merge the waves' partials per hypothesis
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < RB; ++r) { wm[wid][r] = m_w[r]; wl[wid][r] = l_w[r]; }
  }
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int jp = 0; jp < 4; ++jp)
      *reinterpret_cast<float2*>(&part[wid][r][k0 + 2 * jp]) = make_float2(acc[r][jp].x, acc[r][jp].y);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    float m = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) m = fmaxf(m, wm[w][r]);
    float l = 0.f, wsc[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      wsc[w] = wm[w][r] == -INFINITY ? 0.f : fexp(wm[w][r] - m);
      l += wl[w][r] * wsc[w];
    }
    const size_t row = (size_t)(r0 + r) * S + c;
    if (tid == 0) {
      pm[row * 2] = m;
      pm[row * 2 + 1] = l;
    }
    for (int k = tid; k < A; k += NW * 64) {
      float x = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) x += part[w][r][k] * wsc[w];
      pctx[row * A + k] = x;
    }
  }
}

// grid R, 256 threads: combine the S chunk partials of hypothesis row b
__global__ __launch_bounds__(256) void attn_beam_merge_kernel(
    const float* __restrict__ e_buf, const float* __restrict__ pm, const float* __restrict__ pctx,
    const int* __restrict__ lens, float* __restrict__ a_out, float* __restrict__ ctx, bf16* __restrict__ ctx_bf,
    int T, int S, int rep) {
  constexpr int A = 512;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int len = (int)DCHECK_IDX(lens[b / rep], 1, T + 1, CHK_ATTN_LEN);
  const float* pmb = pm + (size_t)b * S * 2;
  float M = -INFINITY;
  for (int c = 0; c < S; ++c) M = fmaxf(M, pmb[2 * c]);
  float L = 0.f;
  for (int c = 0; c < S; ++c)
    if (pmb[2 * c] > -INFINITY) L += pmb[2 * c + 1] * fexp(pmb[2 * c] - M);
  const float invL = 1.0f / L;
  for (int k = tid; k < A; k += 256) {
    float x = 0.f;
    for (int c = 0; c < S; ++c)
      if (pmb[2 * c] > -INFINITY) x += pctx[((size_t)b * S + c) * A + k] * fexp(pmb[2 * c] - M);
    x *= invL;
    ctx[(size_t)b * A + k] = x;
    if (ctx_bf) ctx_bf[(size_t)b * A + k] = f2bf(x);
  }
  for (int i = tid; i < T; i += 256)
    a_out[(size_t)b * T + i] = i < len ? fexp(e_buf[(size_t)b * T + i] - M) * invL : 0.f;
}

bool attn_beam_supported(int A, int T, int rep) { return A == 512 && rep == kBeamRB && T >= 1 && T <= 4096; }

int attn_beam_chunks(int Na, int T) {
  // >= 512 workgroups (2 per CU), chunks of >= 32 positions
  int S = (512 + Na - 1) / max(1, Na);
  S = min(S, max(1, T / 32));
  return max(1, min(S, 64));
}

void launch_attn_beam(const bf16* F, const bf16* E, const float* s, const float* v, const float* wc, const float* cov,
                      const float* cov_src, const float* a_src, float* cov_keep, const int* cg, const int* lens,
                      float* e_buf, float* pm, float* pctx, float* a_out, float* ctx, bf16* ctx_bf, int R, int T,
                      int A, int rep, int S, hipStream_t st) {
  const int Na = R / rep;
  hipLaunchKernelGGL((attn_beam_part_kernel<kBeamNW, kBeamRB>), dim3(Na * S), dim3(kBeamNW * 64), 0, st, F, E, s, v,
                     wc, cov, cov_src, a_src, cov_keep, cg, lens, e_buf, pm, pctx, T, S);
  hipLaunchKernelGGL(attn_beam_merge_kernel, dim3(R), dim3(256), 0, st, e_buf, pm, pctx, lens, a_out, ctx, ctx_bf, T,
                     S, rep);
  (void)A;
}
