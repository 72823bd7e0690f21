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
#include <stdlib.h>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBeamRB = 4;     // hypotheses per article (rep)
constexpr int kBeamNW = 8;     // waves per workgroup (A = 512 = 8 waves x 64 features in phase B)
constexpr int kBeamCH = 512;   // max positions per chunk (LDS p table)

}  // namespace

// grid Na * S; block kBeamNW waves.  A = 512, RB = 4 hypotheses per article.
//   phase A (F): wave w scores the groups of 4 positions w, w + NW, ... for every hypothesis
//                (lanes over 8 features each, bfly4 over the wave); scores -> LDS (+ e_buf)
//   stats:       wave r: chunk max m_r, p_ri = e^(e_ri - m_r) (LDS, [position][hypothesis]),
//                l_r = sum_i p_ri -> pm
//   phase B (E): wave w owns features 64 w .. 64 w + 63; its lanes take 8 positions x 8
//                features per 16-byte load, so every E row of the chunk is read once and the
//                context partial sum_i p_ri E_i of all 4 hypotheses accumulates without a
//                cross-wave reduction (3 butterfly steps over the position lanes at the end)
template <int NW, int RB, int OCC, bool SLDS>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void attn_beam_part_kernel(
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
  static_assert(RB == 4 && NW * 64 == A, "layout: 4 hypotheses, one wave per 64 features in phase B");
  __shared__ float es[RB][kBeamCH];
  __shared__ __attribute__((aligned(16))) float4 pq[kBeamCH + 8];  // p of the chunk positions, [position][hypothesis]
  __shared__ __attribute__((aligned(16))) float s_l[SLDS ? RB : 1][SLDS ? A : 1];  // SLDS: pre-scaled queries
  const int a = blockIdx.x / S, c = blockIdx.x % S;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int len = (int)DCHECK_IDX(lens[a], 1, T + 1, CHK_ATTN_LEN);
  // chunk c of the article's len positions, in whole 4-position groups
  const int ng = (len + 3) >> 2, gpc = (ng + S - 1) / S;
  const int p0 = 4 * gpc * c, p1 = min(len, 4 * gpc * (c + 1));
  const int n = max(0, p1 - p0);
  const int ngrp = (n + 3) >> 2;
  const bf16* Fb = F + (size_t)a * T * A;
  const bf16* Eb = E + (size_t)a * T * A;
  const int r0 = a * RB;
  const bool gather = cg != nullptr;
  // ---------------------------------------------------------------- phase A: scores
  {
    const int qm = lane >> 4, b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1;
    size_t cb[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r)
      cb[r] = gather ? (size_t)DCHECK_IDX(cg[r0 + r], 0, (int)gridDim.x / S * RB, CHK_BEAM_PARENT) * T
                     : (size_t)(r0 + r) * T;
    u32x4 fA[4], fB[4];
    float cA[RB], cBv[RB];
    auto load = [&](int grp, u32x4 (&f)[4], float (&cv)[RB]) {
      const int q0 = p0 + 4 * grp;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        f[q] = __builtin_bit_cast(u32x4, ld8(Fb + (size_t)min(q0 + q, len - 1) * A + lane * 8));
      const int p = min(q0 + qm, len - 1);
#pragma unroll
      for (int r = 0; r < RB; ++r)
        cv[r] = gather ? cov_src[cb[r] + p] + a_src[cb[r] + p] : (cov ? cov[cb[r] + p] : 0.f);
    };
    if (wid < ngrp) load(wid, fA, cA);
    f32x2 w2[4], v2[4], s2[SLDS ? 1 : RB][4];
    float vsum = 0.f;
    const int k0 = lane * 8;
    if (SLDS) {  // the 4 queries (pre-scaled) in LDS, read per use: 32 registers less
      for (int i = tid; i < RB * A; i += NW * 64) s_l[i / A][i % A] = s[(size_t)r0 * A + i] * K2LOG2E;
      __syncthreads();
    }
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      const float2 vv = *reinterpret_cast<const float2*>(v + k0 + 2 * jp);
      const float2 wv = wc ? *reinterpret_cast<const float2*>(wc + k0 + 2 * jp) : make_float2(0.f, 0.f);
      w2[jp] = f32x2{wv.x, wv.y} * K2LOG2E;
      v2[jp] = f32x2{vv.x, vv.y};
      vsum += vv.x + vv.y;
      if (!SLDS) {
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const float2 sv = *reinterpret_cast<const float2*>(s + (size_t)(r0 + r) * A + k0 + 2 * jp);
          s2[r][jp] = f32x2{sv.x, sv.y} * K2LOG2E;
        }
      }
    }
    auto score = [&](int grp, const u32x4 (&f)[4], const float (&cv)[RB]) {
      const int pl = 4 * grp + qm;  // this lane group's position, chunk-local
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        f32x2 sr[4];
        if (SLDS) {
          const float4 x0 = *reinterpret_cast<const float4*>(&s_l[r][k0]);
          const float4 x1 = *reinterpret_cast<const float4*>(&s_l[r][k0 + 4]);
          sr[0] = f32x2{x0.x, x0.y}; sr[1] = f32x2{x0.z, x0.w}; sr[2] = f32x2{x1.x, x1.y}; sr[3] = f32x2{x1.z, x1.w};
        } else {
#pragma unroll
          for (int jp = 0; jp < 4; ++jp) sr[jp] = s2[SLDS ? 0 : r][jp];
        }
        float pd[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float cq = rdlane(cv[r], 16 * q);
          f32x2 d2 = f32x2{0.f, 0.f};
#pragma unroll
          for (int jp = 0; jp < 4; ++jp) {
            const f32x2 y = fma2(bf2pair(f[q][jp]), splat2(K2LOG2E), fma2(w2[jp], splat2(cq), sr[jp]));
            d2 = fma2(v2[jp], rsig2(y), d2);
          }
          pd[q] = vsum - 2.0f * (d2.x + d2.y);  // the lane's share of e (bfly4 sums the lanes)
        }
        const float eq = bfly4(pd, b5, b4);
        if ((lane & 15) == 0 && pl < n) {
          es[r][pl] = eq;
          e_buf[(size_t)(r0 + r) * T + p0 + pl] = eq;
          if (gather && cov_keep) cov_keep[(size_t)(r0 + r) * T + p0 + pl] = cv[r];
        }
      }
    };
    for (int g = wid; g < ngrp;) {
      const int g1 = g + NW;
      if (g1 < ngrp) load(g1, fB, cBv);
      score(g, fA, cA);
      if (g1 >= ngrp) break;
      const int g2 = g1 + NW;
      if (g2 < ngrp) load(g2, fA, cA);
      score(g1, fB, cBv);
      g = g2;
    }
  }
  __syncthreads();
  // ---------------------------------------------------------------- stats: wave r, hypothesis r
  if (wid < RB) {
    const int r = wid;
    float m = -INFINITY;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, es[r][i]);
    m = max_x32(max_x16(dpp_max16(m)));
    float l = 0.f;
    for (int i = lane; i < ((n + 7) & ~7); i += 64) {
      const float pv = i < n ? fexp(es[r][i] - m) : 0.f;
      reinterpret_cast<float*>(&pq[i])[r] = pv;
      l += pv;
    }
    l = sum_x32(sum_x16(dpp_sum16(l)));
    if (lane == 0) {
      const size_t row = (size_t)(r0 + r) * S + c;
      pm[row * 2] = n > 0 ? m : -INFINITY;
      pm[row * 2 + 1] = l;
    }
  }
  __syncthreads();
  // ---------------------------------------------------------------- phase B: context partials
  {
    const int f0 = 64 * wid + 8 * (lane & 7), ql = lane >> 3;  // 8 features, position ql of each 8
    f32x2 acc[RB][4];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) acc[r][jp] = f32x2{0.f, 0.f};
    const int nit = (n + 7) >> 3;
    constexpr int PF = 4;  // loads in flight per lane
    u32x4 eb[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u)
      if (u < nit) eb[u] = __builtin_bit_cast(u32x4, ld8(Eb + (size_t)min(p0 + 8 * u + ql, len - 1) * A + f0));
    for (int it = 0; it < nit; it += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        if (it + u >= nit) break;
        const u32x4 ev = eb[u];
        const int nx = it + u + PF;
        if (nx < nit) eb[u] = __builtin_bit_cast(u32x4, ld8(Eb + (size_t)min(p0 + 8 * nx + ql, len - 1) * A + f0));
        const float4 p4 = pq[8 * (it + u) + ql];  // 0 past the chunk
        const float pr[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
          for (int jp = 0; jp < 4; ++jp) acc[r][jp] = fma2(bf2pair(ev[jp]), splat2(pr[r]), acc[r][jp]);
      }
    }
    // sum over the 8 position lanes (l ^ 8, l ^ 16, l ^ 32): lanes 0-7 hold the totals
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        float x = acc[r][jp].x, y = acc[r][jp].y;
        x += dpp_f<DPP_ROR8>(x); y += dpp_f<DPP_ROR8>(y);
        x += xor16_f(x); y += xor16_f(y);
        x += xor32_f(x); y += xor32_f(y);
        acc[r][jp] = f32x2{x, y};
      }
    if (lane < 8) {
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        float* dst = pctx + ((size_t)(r0 + r) * S + c) * A + f0;
        *reinterpret_cast<float4*>(dst) = make_float4(acc[r][0].x, acc[r][0].y, acc[r][1].x, acc[r][1].y);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(acc[r][2].x, acc[r][2].y, acc[r][3].x, acc[r][3].y);
      }
    }
  }
}

// grid R, 256 threads: combine the S (<= 64) chunk partials of hypothesis row b.  The chunk
// weights e^(m_c - M) / L come from one wave's reduction (LDS), then every context element's S
// partial loads are issued together (unrolled), not one dependent load per chunk.
__global__ __launch_bounds__(256) void attn_beam_merge_kernel(
    const float* __restrict__ e_buf, const float* __restrict__ pm, const float* __restrict__ pctx,
    const int* __restrict__ lens, float* __restrict__ a_out, float* __restrict__ ctx, bf16* __restrict__ ctx_bf,
    int T, int S, int rep) {
  constexpr int A = 512;
  __shared__ float sc[64];
  __shared__ float sM, sInvL;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int len = (int)DCHECK_IDX(lens[b / rep], 1, T + 1, CHK_ATTN_LEN);
  const float* pmb = pm + (size_t)b * S * 2;
  if (tid < 64) {
    const float2 ml = tid < S ? *reinterpret_cast<const float2*>(pmb + 2 * tid) : make_float2(-INFINITY, 0.f);
    const float M = max_x32(max_x16(dpp_max16(ml.x)));
    const float w = ml.x > -INFINITY ? fexp(ml.x - M) : 0.f;
    const float L = sum_x32(sum_x16(dpp_sum16(ml.y * w)));
    sc[tid] = w / L;
    if (tid == 0) { sM = M; sInvL = 1.0f / L; }
  }
  __syncthreads();
  const float M = sM, invL = sInvL;
  const float* pb = pctx + (size_t)b * S * A;
  for (int k = tid; k < A; k += 256) {
    float x = 0.f;
    int c = 0;
    for (; c + 8 <= S; c += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = pb[(size_t)(c + u) * A + k];
#pragma unroll
      for (int u = 0; u < 8; ++u) x += v[u] * sc[c + u];
    }
    for (; c < S; ++c) x += pb[(size_t)c * A + k] * sc[c];
    ctx[(size_t)b * A + k] = x;
    if (ctx_bf) ctx_bf[(size_t)b * A + k] = f2bf(x);
  }
  for (int i = tid; i < T; i += 256)
    a_out[(size_t)b * T + i] = i < len ? fexp(e_buf[(size_t)b * T + i] - M) * invL : 0.f;
}

bool attn_beam_supported(int A, int T, int rep) { return A == 512 && rep == kBeamRB && T >= 1 && T <= 64 * kBeamCH; }

bool attn_beam_chunk_ok(int T, int S) { return S >= 1 && S <= 64 && 4 * (((T + 3) / 4 + S - 1) / S) <= kBeamCH; }

int attn_beam_chunks(int Na, int T) {
  // >= 512 workgroups (2 per CU), chunks of >= 32 and <= kBeamCH positions
  int S = (512 + Na - 1) / max(1, Na);
  S = min(S, max(1, T / 32));
  S = max(S, (T + kBeamCH - 1) / kBeamCH);
  return max(1, min(S, 64));
}

void launch_attn_beam(const bf16* F, const bf16* E, const float* s, const float* v, const float* wc, const float* cov,
                      const float* cov_src, const float* a_src, float* cov_keep, const int* cg, const int* lens,
                      float* e_buf, float* pm, float* pctx, float* a_out, float* ctx, bf16* ctx_bf, int R, int T,
                      int A, int rep, int S, hipStream_t st) {
  const int Na = R / rep;
  // A/B knob for the occupancy / query-placement variants (tools/decode_kernels_micro.py)
  static const int variant = getenv("TSAMD_ATTN_BEAM_VARIANT") ? atoi(getenv("TSAMD_ATTN_BEAM_VARIANT")) : 0;
#define LP(OCC, SL)                                                                                                 \
  hipLaunchKernelGGL((attn_beam_part_kernel<kBeamNW, kBeamRB, OCC, SL>), dim3(Na * S), dim3(kBeamNW * 64), 0, st, F, \
                     E, s, v, wc, cov, cov_src, a_src, cov_keep, cg, lens, e_buf, pm, pctx, T, S)
  if (variant == 1) LP(3, true);
  else if (variant == 2) LP(4, true);
  else LP(2, false);
#undef LP
  hipLaunchKernelGGL(attn_beam_merge_kernel, dim3(R), dim3(256), 0, st, e_buf, pm, pctx, lens, a_out, ctx, ctx_bf, T,
                     S, rep);
  (void)A;
}
