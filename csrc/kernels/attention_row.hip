// Row-resident Bahdanau attention with coverage: ONE workgroup per batch row (article) per
// decoder step (reference attention_decoder.py:79-129,
// model.py:463-480).  Same math as attention.hip, different decomposition:
//
//   * a workgroup of 8-16 waves (one workgroup per CU, row_waves()) owns row b
//     and streams its encoder rows F_i = (W_h enc_out)_i and E_i = enc_out_i (1 KB each at
//     A = 512) exactly once; at B = 256 the 256 rows are the 256 CUs, each pulling ~24 GB/s,
//     which is the HBM rate of the chip;
//   * the waves take groups of 4 positions round-robin (wave w: groups w, w + NW, ...); the
//     next group's rows are loaded before the current group is computed (double-buffered
//     registers), so 96-128 KB are in flight per CU;
//   * every row-level reduction (softmax statistics, S = sum_j a_j da_j, the 512-wide ds
//     and ctx vectors) stays inside the workgroup: no atomics, no partial buffers, no
//     pre-zeroed outputs, and one launch per step instead of two (score + softmax/context)
//     in the forward;
//   * lanes hold 8 features each (A = 512 * NK; NK = 1 at hidden 256, 2 at hidden 512), the
//     per-position dot products over the feature axis are reduced with the 4-position
//     butterfly (bfly4: the lanes of position q end up holding its total).
//
// forward (attn_fwd_row):  one pass with an online softmax per wave (running max m_w, sum
//   l_w and the rescaled context partial over the wave's positions, as in flash
//   attention): e_i = sum_k v_k tanh(F_ik + s_k + w_k cov_i) from F_i, then
//   ctx += exp(e_i - m) E_i from E_i in the same pass; the waves' partials are merged in LDS,
//   then a = softmax(e) (scores kept in LDS), cov' = cov + a, covloss = sum min(a, cov).
// backward (attn_bwd_row): da_i = r_i + dctx . E_i, de_i = a_i (da_i - S),
//   ds_k = sum_i de_i v_k sech2(u_ik), dcov_i = dcov_next_i + g [a_i > cov_i] +
//   de_i sum_k v_k w_k sech2(u_ik)  (S = sum_j a_j r_j + dctx . ctx, see attention.hip).
#include "attn_common.h"
#include <stdlib.h>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kRowMaxT = 2048;
// waves per workgroup: as many as the double-buffered rows leave registers for --
// forward at hidden 256: 16 (<= 128 VGPRs); backward at hidden 256: 12 (<= 168 VGPRs, the
// extra dctx / per-feature state); hidden 512 (16 features per lane): 8 (<= 256 VGPRs)
template <int NK, bool BWD>
constexpr int row_waves() { return NK == 1 ? (BWD ? 12 : 16) : 8; }

template <int NK>
struct Rows {
  u32x4 x[NK][4];  // 4 positions x NK 16-byte feature chunks of one tensor
};

template <int NK>
__device__ __forceinline__ void load_rows(Rows<NK>& r, const bf16* base, int p0, int len, int lane) {
  constexpr int A = 512 * NK;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = min(p0 + q, len - 1);
#pragma unroll
    for (int kb = 0; kb < NK; ++kb)
      r.x[kb][q] = __builtin_bit_cast(u32x4, ld8(base + (size_t)p * A + kb * 512 + lane * 8));
  }
}

}  // namespace

// ------------------------------------------------------------------------------ forward
// PROBE (attribution builds only, attn_fwd_row_probe): bit 0 no score arithmetic, bit 1 no context
// accumulation, bit 2 no E loads, bit 3 no F / E loads at all (results wrong by design)
template <int NK, int NW, int PROBE = 0>
__global__ __launch_bounds__(NW * 64) void attn_fwd_row_kernel(
    const bf16* __restrict__ F, const bf16* __restrict__ E, const float* __restrict__ s,
    const float* __restrict__ v, const float* __restrict__ wc, const float* __restrict__ cov,
    const int* __restrict__ lens, float* __restrict__ a_out, float* __restrict__ cov_out,
    float* __restrict__ covloss, float* __restrict__ ctx, bf16* __restrict__ ctx_bf, int T, int rep, int xper,
    const int* __restrict__ cg, const float* __restrict__ asrc, float* __restrict__ cov_keep) {
  const Dot2Sel dsel = dot2_sel();  // F pair selectors for fadd_bf2
  // cg set (beam decode): the coverage of hypothesis row b is its parent's coverage plus the
  // parent's last attention, cov = cov[g] + asrc[g] with g = cg[b] (the gather of the former
  // beam_gather kernel); cov_keep receives it for the next step
  constexpr int A = 512 * NK, NT = NW * 64;
  __shared__ float es[kRowMaxT];
  __shared__ float part[NW][A];
  __shared__ float wm[NW], wl[NW], red[NW];
  // xper > 0 (beam decode): workgroups are dispatched to the 8 XCDs round-robin, so workgroup
  // i runs on XCD i % 8; give XCD x the xper consecutive rows x * xper .. -- whole articles --
  // so the rep hypotheses of an article read its F / E rows through ONE XCD's L2
  const int b = xper ? (int)(blockIdx.x & 7) * xper + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  const int fr = b / rep;  // feature row: beam decode shares one encoder row between rep hypotheses
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int len = (int)DCHECK_IDX(lens[fr], 1, T + 1, CHK_ATTN_LEN);
  const size_t rb = (size_t)b * T;
  const size_t cb = cg ? (size_t)DCHECK_IDX(cg[b], 0, (int)gridDim.x, CHK_BEAM_PARENT) * T : rb;
  const bf16* Fb = F + (size_t)fr * T * A;
  const bf16* Eb = E + (size_t)fr * T * A;
  const int ngrp = (len + 3) >> 2;
  const int qm = lane >> 4;  // the position (within a group) whose total this lane's 16-lane group holds
  const int b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1;
  Rows<NK> fA, eA, fB, eB;
  if constexpr (PROBE & 12) {
#pragma unroll
    for (int kb = 0; kb < NK; ++kb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        fA.x[kb][q] = fB.x[kb][q] = u32x4{(unsigned)lane, 1u, 2u, 3u};
        eA.x[kb][q] = eB.x[kb][q] = u32x4{(unsigned)lane, 3u, 2u, 1u};
      }
  }
  float cA = 0.f, cB = 0.f;
  auto load = [&](int grp, Rows<NK>& f, Rows<NK>& e, float& c) {
    if constexpr (!(PROBE & 8)) load_rows<NK>(f, Fb, 4 * grp, len, lane);
    if constexpr (!(PROBE & 12)) load_rows<NK>(e, Eb, 4 * grp, len, lane);
    const int p = min(4 * grp + qm, len - 1);
    c = cov ? cov[cb + p] + (cg ? asrc[cb + p] : 0.f) : 0.f;
  };
  if (wid < ngrp) load(wid, fA, eA, cA);
  const float* srow = s + (size_t)b * A;
  // per-lane feature parameters, pre-scaled for the r-form (attn_common.h)
  f32x2 s2[NK][4], w2[NK][4], v2[NK][4], acc[NK][4];
  float vsum = 0.f;
#pragma unroll
  for (int kb = 0; kb < NK; ++kb) {
    const int k0 = kb * 512 + lane * 8;
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      const float2 sv = *reinterpret_cast<const float2*>(srow + k0 + 2 * jp);
      const float2 vv = *reinterpret_cast<const float2*>(v + k0 + 2 * jp);
      const float2 wv = wc ? *reinterpret_cast<const float2*>(wc + k0 + 2 * jp) : make_float2(0.f, 0.f);
      s2[kb][jp] = f32x2{sv.x, sv.y} * K2LOG2E;
      w2[kb][jp] = f32x2{wv.x, wv.y} * K2LOG2E;
      v2[kb][jp] = f32x2{vv.x, vv.y};
      acc[kb][jp] = f32x2{0.f, 0.f};
      vsum += vv.x + vv.y;
    }
  }
  float m_w = -INFINITY, l_w = 0.f;
  auto compute = [&](int grp, const Rows<NK>& f, const Rows<NK>& e, float c_l) {
    // scores of the group's 4 positions: e = sum_k v_k - 2 sum_k v_k r_k
    float pd[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float c = rdlane(c_l, 16 * q);
      f32x2 d2 = f32x2{0.f, 0.f};
      if constexpr (PROBE & 1) {
        d2.x = __uint_as_float(f.x[0][q][0] & 0x3fffffffu) + c;
      } else {
#pragma unroll
        for (int kb = 0; kb < NK; ++kb)
#pragma unroll
          for (int jp = 0; jp < 4; ++jp) {
            const f32x2 y = fadd_bf2(f.x[kb][q][jp], fma2(w2[kb][jp], splat2(c), s2[kb][jp]), dsel);
            d2 = fma2(v2[kb][jp], rsig2(y), d2);
          }
      }
      pd[q] = vsum - 2.0f * (d2.x + d2.y);
    }
    float eq = bfly4(pd, b5, b4);
    const int p = 4 * grp + qm;
    if (p >= len) eq = -INFINITY;
    if ((lane & 15) == 0 && p < len) es[p] = eq;
    const float e0 = rdlane(eq, 0), e1 = rdlane(eq, 16), e2 = rdlane(eq, 32), e3 = rdlane(eq, 48);
    const float mn = fmaxf(m_w, fmaxf(fmaxf(e0, e1), fmaxf(e2, e3)));  // e0 is always valid (p0 < len)
    const float sc = m_w == -INFINITY ? 0.f : fexp(m_w - mn);
    const float p0 = fexp(e0 - mn), p1 = fexp(e1 - mn), p2 = fexp(e2 - mn), p3 = fexp(e3 - mn);
    l_w = l_w * sc + ((p0 + p1) + (p2 + p3));
    if constexpr (PROBE & 2) {
      acc[0][0].x += __uint_as_float(e.x[0][0][0] & 0x3fffffffu) * p0;
    } else
#pragma unroll
    for (int kb = 0; kb < NK; ++kb)
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        f32x2 a2 = acc[kb][jp] * sc;
        a2 = fma2(bf2pair(e.x[kb][0][jp]), splat2(p0), a2);
        a2 = fma2(bf2pair(e.x[kb][1][jp]), splat2(p1), a2);
        a2 = fma2(bf2pair(e.x[kb][2][jp]), splat2(p2), a2);
        acc[kb][jp] = fma2(bf2pair(e.x[kb][3][jp]), splat2(p3), a2);
      }
    m_w = mn;
  };
  // double-buffered sweep: group g + NW's rows are in flight while group g is computed
  for (int g = wid; g < ngrp;) {
    const int g1 = g + NW;
    if (g1 < ngrp) load(g1, fB, eB, cB);
    compute(g, fA, eA, cA);
    if (g1 >= ngrp) break;
    const int g2 = g1 + NW;
    if (g2 < ngrp) load(g2, fA, eA, cA);
    compute(g1, fB, eB, cB);
    g = g2;
  }
  // merge the waves' online-softmax partials
  if (lane == 0) {
    wm[wid] = m_w;
    wl[wid] = l_w;
  }
#pragma unroll
  for (int kb = 0; kb < NK; ++kb)
#pragma unroll
    for (int jp = 0; jp < 4; ++jp)
      *reinterpret_cast<float2*>(&part[wid][kb * 512 + lane * 8 + 2 * jp]) =
          make_float2(acc[kb][jp].x, acc[kb][jp].y);
  __syncthreads();
  float m = -INFINITY;
#pragma unroll
  for (int w = 0; w < NW; ++w) m = fmaxf(m, wm[w]);
  float L = 0.f, wsc[NW];
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    wsc[w] = wm[w] == -INFINITY ? 0.f : fexp(wm[w] - m);
    L += wl[w] * wsc[w];
  }
  const float invL = 1.0f / L;
  for (int k = tid; k < A; k += NT) {
    float c = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) c += part[w][k] * wsc[w];
    c *= invL;
    ctx[(size_t)b * A + k] = c;
    if (ctx_bf) ctx_bf[(size_t)b * A + k] = f2bf(c);
  }
  float cl = 0.f;
  for (int i = tid; i < T; i += NT) {
    const float a = i < len ? fexp(es[i] - m) * invL : 0.f;
    a_out[rb + i] = a;
    if (cov_keep) cov_keep[rb + i] = cov[cb + i] + asrc[cb + i];
    if (cov_out) {
      const float c = cov ? cov[rb + i] : 0.f;
      cov_out[rb + i] = c + a;
      cl += fminf(a, c);
    }
  }
  if (covloss) {
    cl = block_sum<NT>(cl, red);
    if (tid == 0) covloss[b] = cl;
  }
}

// ------------------------------------------------------------------------------ backward
// The per-feature parameters (s, w, 4 v w, dctx: 32 NK floats per lane) live in LDS, not in
// registers: with them in registers the double-buffered rows spilled 65 VGPRs at A = 1024
// (tools/attn_micro_c5.py, 256 rows, T = 800: 323 -> 162 us; A = 512, T = 400: 51.0 -> 48.7 us).
// The parameter-major loop order (feature pair outer, position inner) reads each once per group.
template <int NK, int NW>
__global__ __launch_bounds__(NW * 64) void attn_bwd_row_kernel(
    const bf16* __restrict__ E, const bf16* __restrict__ F, const float* __restrict__ s,
    const float* __restrict__ v, const float* __restrict__ wc, const float* __restrict__ cov,
    const float* __restrict__ a, const float* __restrict__ dctx, const float* __restrict__ ctx,
    const float* __restrict__ Ga, const float* __restrict__ dcov_next, const float* __restrict__ gcl,
    const int* __restrict__ lens, float* __restrict__ de_out, float* __restrict__ ds,
    float* __restrict__ dcov_out, int T) {
  const Dot2Sel dsel = dot2_sel();  // F pair selectors for fadd_bf2
  constexpr int A = 512 * NK, NT = NW * 64;
  __shared__ float part[NW][A];
  __shared__ float red[NW];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int len = (int)DCHECK_IDX(lens[b], 1, T + 1, CHK_ATTN_LEN);
  const size_t rb = (size_t)b * T;
  const float g = gcl ? gcl[b] : 0.f;
  const bf16* Eb = E + (size_t)b * T * A;
  const bf16* Fb = F + (size_t)b * T * A;
  const int ngrp = (len + 3) >> 2;
  const int qm = lane >> 4;
  const int b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1;
  struct Scal {
    float a, r, c, dn;
  };
  Rows<NK> eA, fA, eB, fB;
  Scal xA{}, xB{};
  auto load = [&](int grp, Rows<NK>& e, Rows<NK>& f, Scal& x) {
    load_rows<NK>(e, Eb, 4 * grp, len, lane);
    load_rows<NK>(f, Fb, 4 * grp, len, lane);
    const int p = 4 * grp + qm;
    const size_t ix = rb + min(p, len - 1);
    x.a = a[ix];
    x.c = cov ? cov[ix] : 0.f;
    x.dn = dcov_next ? dcov_next[ix] : 0.f;
    x.r = (Ga ? Ga[ix] : 0.f) + x.dn + ((gcl && x.a <= x.c) ? g : 0.f);
  };
  if (wid < ngrp) load(wid, eA, fA, xA);
  // parameters in LDS [param][kb][jp][lane] (one copy: every wave has the same lane -> feature
  // map), written by wave 0 before the block_sum barrier below
  f32x2 acc[NK][4];
  __shared__ f32x2 prm[4 * NK * 4 * 64];
#pragma unroll
  for (int kb = 0; kb < NK; ++kb) {
    const int k0 = kb * 512 + lane * 8;
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      acc[kb][jp] = f32x2{0.f, 0.f};
      if (wid != 0) continue;
      const float2 sv = *reinterpret_cast<const float2*>(s + (size_t)b * A + k0 + 2 * jp);
      const float2 vv = *reinterpret_cast<const float2*>(v + k0 + 2 * jp);
      const float2 wv = wc ? *reinterpret_cast<const float2*>(wc + k0 + 2 * jp) : make_float2(0.f, 0.f);
      const float2 dv = *reinterpret_cast<const float2*>(dctx + (size_t)b * A + k0 + 2 * jp);
      const f32x2 ps = f32x2{sv.x, sv.y} * K2LOG2E, pw = f32x2{wv.x, wv.y} * K2LOG2E;
      const f32x2 pv = f32x2{4.f * vv.x * wv.x, 4.f * vv.y * wv.y}, pd = f32x2{dv.x, dv.y};
      prm[((0 * NK + kb) * 4 + jp) * 64 + lane] = ps;
      prm[((1 * NK + kb) * 4 + jp) * 64 + lane] = pw;
      prm[((2 * NK + kb) * 4 + jp) * 64 + lane] = pv;
      prm[((3 * NK + kb) * 4 + jp) * 64 + lane] = pd;
    }
  }
  auto par = [&](int which, int kb, int jp) -> f32x2 { return prm[((which * NK + kb) * 4 + jp) * 64 + lane]; };
  // S = sum_j a_j r_j + dctx . ctx  (the row's group-0 loads are already in flight)
  float S = 0.f;
  for (int i = tid; i < len; i += NT) {
    const size_t ix = rb + i;
    const float ai = a[ix];
    float r = (Ga ? Ga[ix] : 0.f) + (dcov_next ? dcov_next[ix] : 0.f);
    if (gcl && ai <= (cov ? cov[ix] : 0.f)) r += g;
    S += ai * r;
  }
  for (int k = tid; k < A; k += NT) S += dctx[(size_t)b * A + k] * ctx[(size_t)b * A + k];
  S = block_sum<NT>(S, red);
  auto compute = [&](int grp, const Rows<NK>& e, const Rows<NK>& f, const Scal& x) {
    f32x2 d2[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) d2[q] = f32x2{0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < NK; ++kb)
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        const f32x2 dk = par(3, kb, jp);
#pragma unroll
        for (int q = 0; q < 4; ++q) d2[q] = fma2(bf2pair(e.x[kb][q][jp]), dk, d2[q]);
      }
    float pd[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) pd[q] = d2[q].x + d2[q].y;
    const float dot = bfly4(pd, b5, b4);
    const int p = 4 * grp + qm;
    const float de_q = p < len ? x.a * (x.r + dot - S) : 0.f;
    float deq[4], cq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      deq[q] = rdlane(de_q, 16 * q);
      cq[q] = rdlane(x.c, 16 * q);
    }
    f32x2 dc2[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) dc2[q] = f32x2{0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < NK; ++kb)
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        const f32x2 ps = par(0, kb, jp), pw = par(1, kb, jp), pv = par(2, kb, jp);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x2 y = fadd_bf2(f.x[kb][q][jp], fma2(pw, splat2(cq[q]), ps), dsel);
          const f32x2 r = rsig2(y);
          const f32x2 qv = fma2(-r, r, r);
          acc[kb][jp] = fma2(qv, splat2(deq[q]), acc[kb][jp]);
          dc2[q] = fma2(qv, pv, dc2[q]);
        }
      }
    float dcv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) dcv[q] = dc2[q].x + dc2[q].y;
    const float hc = bfly4(dcv, b5, b4);
    if ((lane & 15) == 0 && p < T) {
      de_out[rb + p] = de_q;
      if (dcov_out) {
        float r = x.dn;
        if (p < len) {
          r += de_q * hc;
          if (gcl && x.a > x.c) r += g;
        } else {
          r = dcov_next ? dcov_next[rb + p] : 0.f;
        }
        dcov_out[rb + p] = r;
      }
    }
  };
  for (int gi = wid; gi < ngrp;) {
    const int g1 = gi + NW;
    if (g1 < ngrp) load(g1, eB, fB, xB);
    compute(gi, eA, fA, xA);
    if (g1 >= ngrp) break;
    const int g2 = g1 + NW;
    if (g2 < ngrp) load(g2, eA, fA, xA);
    compute(g1, eB, fB, xB);
    gi = g2;
  }
  // positions past the last group: de = 0, dcov passes through
  for (int p = 4 * ngrp + tid; p < T; p += NT) {
    de_out[rb + p] = 0.f;
    if (dcov_out) dcov_out[rb + p] = dcov_next ? dcov_next[rb + p] : 0.f;
  }
  // ds_k = 4 v_k sum_i de_i q_ik, summed over the waves in LDS: one plain store per feature
#pragma unroll
  for (int kb = 0; kb < NK; ++kb)
#pragma unroll
    for (int jp = 0; jp < 4; ++jp)
      *reinterpret_cast<float2*>(&part[wid][kb * 512 + lane * 8 + 2 * jp]) =
          make_float2(acc[kb][jp].x, acc[kb][jp].y);
  __syncthreads();
  for (int k = tid; k < A; k += NT) {
    float x = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) x += part[w][k];
    ds[(size_t)b * A + k] = 4.f * v[k] * x;
  }
}

// ------------------------------------------------------------------------------ projected context
// Training variant of the two kernels above that never reads E (reference
// attention_decoder.py:79-129,138-158).  Inside the decoder recurrence the context vector is only
// consumed through the input merge x_{t+1} = [emb, ctx_t] . W_in, so the loop needs
//   g_t = ctx_t . W_in[E:] = sum_i a_i G_i,   G = enc_out . W_in[E:]   ([T, EG], EG = emb_dim = 128)
// instead of ctx_t (A = 512 / 1024 features).  G is one GEMM before the loop; the full ctx_t of all
// steps (output projection, p_gen, weight gradients) is one batched GEMM a . enc_out after it.  The
// backward splits  da_i = dctx_t . E_i  into the part known before the loop (output projection and
// p_gen terms: one batched GEMM, folded into r_i = Ga_i) and the recurrent part
//   dctx_rec_t . E_i = (dx_{t+1} . W_in[E:]^T) . E_i = dx_{t+1} . G_i.
// Per (step, row, position) the loop then streams F_i (A features) and G_i (128) instead of F_i and
// E_i: 1.25 KB instead of 2 KB at A = 512, 2.25 KB instead of 4 KB at A = 1024 -- the row kernels run
// at the HBM rate, so the bytes are the time (profiles/r3/attention_analysis.md).
// Lane layout of G: a 4-position group is 4 x 128 bf16 = one 16-byte chunk per lane, lane l holding
// features (l & 15) * 8 .. + 8 of position l >> 4 -- the position whose score the lane holds after
// bfly4, so the context update needs no cross-lane traffic.
constexpr int kEG = 128;

template <int NK, int NW>
__global__ __launch_bounds__(NW * 64) void attn_fwd_rowp_kernel(
    const bf16* __restrict__ F, const bf16* __restrict__ G, const float* __restrict__ s,
    const float* __restrict__ v, const float* __restrict__ wc, const float* __restrict__ cov,
    const int* __restrict__ lens, float* __restrict__ a_out, float* __restrict__ cov_out,
    float* __restrict__ covloss, float* __restrict__ gx, bf16* __restrict__ gx_bf, int T,
    const int* __restrict__ dlen, int step, bf16* __restrict__ a_bf) {
  const Dot2Sel dsel = dot2_sel();  // F pair selectors for fadd_bf2
  constexpr int A = 512 * NK, NT = NW * 64;
  __shared__ float es[kRowMaxT];
  __shared__ float part[NW][4][kEG];
  __shared__ float wm[NW], wl[NW], red[NW];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int len = (int)DCHECK_IDX(lens[b], 1, T + 1, CHK_ATTN_LEN);
  const size_t rb = (size_t)b * T;
  if (dlen && step >= dlen[b]) {
    // a step past the row's last loss-weighted decoder step (block-uniform exit): nothing it
    // computes reaches the loss, so write zeros (a, g, coverage loss) and carry the coverage
    for (int i = tid; i < T; i += NT) {
      a_out[rb + i] = 0.f;
      if (a_bf) a_bf[rb + i] = f2bf(0.f);
      if (cov_out) cov_out[rb + i] = cov ? cov[rb + i] : 0.f;
    }
    for (int k = tid; k < kEG; k += NT) {
      gx[(size_t)b * kEG + k] = 0.f;
      gx_bf[(size_t)b * kEG + k] = f2bf(0.f);
    }
    if (covloss && tid == 0) covloss[b] = 0.f;
    return;
  }
  const bf16* Fb = F + (size_t)b * T * A;
  const bf16* Gb = G + (size_t)b * T * kEG + (lane & 15) * 8;
  const int ngrp = (len + 3) >> 2;
  const int qm = lane >> 4;
  const int b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1;
  Rows<NK> fA, fB;
  u32x4 gA, gB;
  float cA = 0.f, cB = 0.f;
  auto load = [&](int grp, Rows<NK>& f, u32x4& gq, float& c) {
    load_rows<NK>(f, Fb, 4 * grp, len, lane);
    const int p = min(4 * grp + qm, len - 1);
    gq = __builtin_bit_cast(u32x4, ld8(Gb + (size_t)p * kEG));
    c = cov ? cov[rb + p] : 0.f;
  };
  if (wid < ngrp) load(wid, fA, gA, cA);
  const float* srow = s + (size_t)b * A;
  f32x2 s2[NK][4], w2[NK][4], v2[NK][4], acc[4];
  float vsum = 0.f;
#pragma unroll
  for (int kb = 0; kb < NK; ++kb) {
    const int k0 = kb * 512 + lane * 8;
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      const float2 sv = *reinterpret_cast<const float2*>(srow + k0 + 2 * jp);
      const float2 vv = *reinterpret_cast<const float2*>(v + k0 + 2 * jp);
      const float2 wv = wc ? *reinterpret_cast<const float2*>(wc + k0 + 2 * jp) : make_float2(0.f, 0.f);
      s2[kb][jp] = f32x2{sv.x, sv.y} * K2LOG2E;
      w2[kb][jp] = f32x2{wv.x, wv.y} * K2LOG2E;
      v2[kb][jp] = f32x2{vv.x, vv.y};
      vsum += vv.x + vv.y;
    }
  }
#pragma unroll
  for (int jp = 0; jp < 4; ++jp) acc[jp] = f32x2{0.f, 0.f};
  // online softmax: m_w is wave-uniform, l_l is the lane's own position's share of the wave sum
  float m_w = -INFINITY, l_l = 0.f;
  auto compute = [&](int grp, const Rows<NK>& f, const u32x4& gq, float c_l) {
    float pd[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float c = rdlane(c_l, 16 * q);
      f32x2 d2 = f32x2{0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < NK; ++kb)
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
          const f32x2 y = fadd_bf2(f.x[kb][q][jp], fma2(w2[kb][jp], splat2(c), s2[kb][jp]), dsel);
          d2 = fma2(v2[kb][jp], rsig2(y), d2);
        }
      pd[q] = vsum - 2.0f * (d2.x + d2.y);
    }
    float eq = bfly4(pd, b5, b4);
    const int p = 4 * grp + qm;
    if (p >= len) eq = -INFINITY;
    if ((lane & 15) == 0 && p < len) es[p] = eq;
    const float e0 = rdlane(eq, 0), e1 = rdlane(eq, 16), e2 = rdlane(eq, 32), e3 = rdlane(eq, 48);
    const float mn = fmaxf(m_w, fmaxf(fmaxf(e0, e1), fmaxf(e2, e3)));  // e0 is always valid (p0 < len)
    const float sc = m_w == -INFINITY ? 0.f : fexp(m_w - mn);
    const float pq = fexp(eq - mn);
    l_l = fmaf(l_l, sc, pq);
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) acc[jp] = fma2(bf2pair(gq[jp]), splat2(pq), acc[jp] * sc);
    m_w = mn;
  };
  for (int g = wid; g < ngrp;) {
    const int g1 = g + NW;
    if (g1 < ngrp) load(g1, fB, gB, cB);
    compute(g, fA, gA, cA);
    if (g1 >= ngrp) break;
    const int g2 = g1 + NW;
    if (g2 < ngrp) load(g2, fA, gA, cA);
    compute(g1, fB, gB, cB);
    g = g2;
  }
  // merge: the 4 position quads of a wave hold the same features, then the waves
  const float lw = (rdlane(l_l, 0) + rdlane(l_l, 16)) + (rdlane(l_l, 32) + rdlane(l_l, 48));
  if (lane == 0) {
    wm[wid] = m_w;
    wl[wid] = lw;
  }
#pragma unroll
  for (int jp = 0; jp < 4; ++jp)
    *reinterpret_cast<float2*>(&part[wid][qm][(lane & 15) * 8 + 2 * jp]) = make_float2(acc[jp].x, acc[jp].y);
  __syncthreads();
  float m = -INFINITY;
#pragma unroll
  for (int w = 0; w < NW; ++w) m = fmaxf(m, wm[w]);
  float L = 0.f, wsc[NW];
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    wsc[w] = wm[w] == -INFINITY ? 0.f : fexp(wm[w] - m);
    L += wl[w] * wsc[w];
  }
  const float invL = 1.0f / L;
  for (int k = tid; k < kEG; k += NT) {
    float c = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) c += ((part[w][0][k] + part[w][1][k]) + (part[w][2][k] + part[w][3][k])) * wsc[w];
    c *= invL;
    gx[(size_t)b * kEG + k] = c;
    gx_bf[(size_t)b * kEG + k] = f2bf(c);
  }
  float cl = 0.f;
  for (int i = tid; i < T; i += NT) {
    const float a = i < len ? fexp(es[i] - m) * invL : 0.f;
    a_out[rb + i] = a;
    if (a_bf) a_bf[rb + i] = f2bf(a);  // the bf16 operand of the post-loop ctx GEMM (no cast pass)
    if (cov_out) {
      const float c = cov ? cov[rb + i] : 0.f;
      cov_out[rb + i] = c + a;
      cl += fminf(a, c);
    }
  }
  if (covloss) {
    cl = block_sum<NT>(cl, red);
    if (tid == 0) covloss[b] = cl;
  }
}

// backward: da_i = r_i + dx . G_i (r_i already holds the output-projection / p_gen part of
// dctx . E_i), S = sum_j a_j r_j + dx . g_t; the rest as attn_bwd_row.  dx == nullptr:
// last step.
template <int NK, int NW>
__global__ __launch_bounds__(NW * 64) void attn_bwd_rowp_kernel(
    const bf16* __restrict__ G, const bf16* __restrict__ F, const float* __restrict__ s,
    const float* __restrict__ v, const float* __restrict__ wc, const float* __restrict__ cov,
    const float* __restrict__ a, const float* __restrict__ dx, const float* __restrict__ gv,
    const float* __restrict__ Ga, const float* __restrict__ dcov_next, const float* __restrict__ gcl,
    const int* __restrict__ lens, float* __restrict__ de_out, float* __restrict__ ds,
    float* __restrict__ dcov_out, int T, const int* __restrict__ dlen, int step) {
  const Dot2Sel dsel = dot2_sel();  // F pair selectors for fadd_bf2
  constexpr int A = 512 * NK, NT = NW * 64;
  __shared__ float part[NW][A];
  __shared__ float red[NW];
  __shared__ f32x2 prm[3 * NK * 4 * 64];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int len = (int)DCHECK_IDX(lens[b], 1, T + 1, CHK_ATTN_LEN);
  const size_t rb = (size_t)b * T;
  if (dlen && step >= dlen[b]) {
    // past the row's last loss-weighted step every gradient is exactly zero (block-uniform exit)
    for (int i = tid; i < T; i += NT) {
      de_out[rb + i] = 0.f;
      if (dcov_out) dcov_out[rb + i] = 0.f;
    }
    for (int k = tid; k < A; k += NT) ds[(size_t)b * A + k] = 0.f;
    return;
  }
  const float g = gcl ? gcl[b] : 0.f;
  const bf16* Gb = G + (size_t)b * T * kEG + (lane & 15) * 8;
  const bf16* Fb = F + (size_t)b * T * A;
  const int ngrp = (len + 3) >> 2;
  const int qm = lane >> 4;
  const int b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1;
  struct Scal {
    float a, r, c, dn;
  };
  Rows<NK> fA, fB;
  u32x4 gA, gB;
  Scal xA{}, xB{};
  auto load = [&](int grp, Rows<NK>& f, u32x4& gq, Scal& x) {
    load_rows<NK>(f, Fb, 4 * grp, len, lane);
    const int p = 4 * grp + qm;
    const int pc = min(p, len - 1);
    gq = __builtin_bit_cast(u32x4, ld8(Gb + (size_t)pc * kEG));
    const size_t ix = rb + pc;
    x.a = a[ix];
    x.c = cov ? cov[ix] : 0.f;
    x.dn = dcov_next ? dcov_next[ix] : 0.f;
    x.r = (Ga ? Ga[ix] : 0.f) + x.dn + ((gcl && x.a <= x.c) ? g : 0.f);
  };
  if (wid < ngrp) load(wid, fA, gA, xA);
  f32x2 acc[NK][4];
#pragma unroll
  for (int kb = 0; kb < NK; ++kb) {
    const int k0 = kb * 512 + lane * 8;
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      acc[kb][jp] = f32x2{0.f, 0.f};
      if (wid != 0) continue;
      const float2 sv = *reinterpret_cast<const float2*>(s + (size_t)b * A + k0 + 2 * jp);
      const float2 vv = *reinterpret_cast<const float2*>(v + k0 + 2 * jp);
      const float2 wv = wc ? *reinterpret_cast<const float2*>(wc + k0 + 2 * jp) : make_float2(0.f, 0.f);
      prm[((0 * NK + kb) * 4 + jp) * 64 + lane] = f32x2{sv.x, sv.y} * K2LOG2E;
      prm[((1 * NK + kb) * 4 + jp) * 64 + lane] = f32x2{wv.x, wv.y} * K2LOG2E;
      prm[((2 * NK + kb) * 4 + jp) * 64 + lane] = f32x2{4.f * vv.x * wv.x, 4.f * vv.y * wv.y};
    }
  }
  auto par = [&](int which, int kb, int jp) -> f32x2 { return prm[((which * NK + kb) * 4 + jp) * 64 + lane]; };
  const float* dxp = dx ? dx + (size_t)b * kEG : nullptr;
  // dx (position-independent; lane l uses features (l & 15) * 8 .. + 8) in LDS, not in 8 VGPRs:
  // with it in registers the 16-wave kernel spilled 3 VGPRs inside the position loop (21.5 vs
  // 20.1 us per call at B = 256)
  __shared__ f32x2 dxl[4 * 16];
  if (tid < 64) {
    const int c = tid & 15, jp = tid >> 4;
    const float2 d = dxp ? *reinterpret_cast<const float2*>(dxp + c * 8 + 2 * jp) : make_float2(0.f, 0.f);
    dxl[jp * 16 + c] = f32x2{d.x, d.y};
  }
  float S = 0.f;
  for (int i = tid; i < len; i += NT) {
    const size_t ix = rb + i;
    const float ai = a[ix];
    float r = (Ga ? Ga[ix] : 0.f) + (dcov_next ? dcov_next[ix] : 0.f);
    if (gcl && ai <= (cov ? cov[ix] : 0.f)) r += g;
    S += ai * r;
  }
  if (dxp)
    for (int k = tid; k < kEG; k += NT) S += dxp[k] * gv[(size_t)b * kEG + k];
  S = block_sum<NT>(S, red);
  auto compute = [&](int grp, const Rows<NK>& f, const u32x4& gq, const Scal& x) {
    f32x2 d2 = f32x2{0.f, 0.f};
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) d2 = fma2(bf2pair(gq[jp]), dxl[jp * 16 + (lane & 15)], d2);
    const float dot = dpp_sum16(d2.x + d2.y);
    const int p = 4 * grp + qm;
    const float de_q = p < len ? x.a * (x.r + dot - S) : 0.f;
    float deq[4], cq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      deq[q] = rdlane(de_q, 16 * q);
      cq[q] = rdlane(x.c, 16 * q);
    }
    f32x2 dc2[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) dc2[q] = f32x2{0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < NK; ++kb)
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        const f32x2 ps = par(0, kb, jp), pw = par(1, kb, jp), pv = par(2, kb, jp);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x2 y = fadd_bf2(f.x[kb][q][jp], fma2(pw, splat2(cq[q]), ps), dsel);
          const f32x2 r = rsig2(y);
          const f32x2 qv = fma2(-r, r, r);
          acc[kb][jp] = fma2(qv, splat2(deq[q]), acc[kb][jp]);
          dc2[q] = fma2(qv, pv, dc2[q]);
        }
      }
    float dcv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) dcv[q] = dc2[q].x + dc2[q].y;
    const float hc = bfly4(dcv, b5, b4);
    if ((lane & 15) == 0 && p < T) {
      de_out[rb + p] = de_q;
      if (dcov_out) {
        float r = x.dn;
        if (p < len) {
          r += de_q * hc;
          if (gcl && x.a > x.c) r += g;
        } else {
          r = dcov_next ? dcov_next[rb + p] : 0.f;
        }
        dcov_out[rb + p] = r;
      }
    }
  };
  for (int gi = wid; gi < ngrp;) {
    const int g1 = gi + NW;
    if (g1 < ngrp) load(g1, fB, gB, xB);
    compute(gi, fA, gA, xA);
    if (g1 >= ngrp) break;
    const int g2 = g1 + NW;
    if (g2 < ngrp) load(g2, fA, gA, xA);
    compute(g1, fB, gB, xB);
    gi = g2;
  }
  for (int p = 4 * ngrp + tid; p < T; p += NT) {
    de_out[rb + p] = 0.f;
    if (dcov_out) dcov_out[rb + p] = dcov_next ? dcov_next[rb + p] : 0.f;
  }
#pragma unroll
  for (int kb = 0; kb < NK; ++kb)
#pragma unroll
    for (int jp = 0; jp < 4; ++jp)
      *reinterpret_cast<float2*>(&part[wid][kb * 512 + lane * 8 + 2 * jp]) =
          make_float2(acc[kb][jp].x, acc[kb][jp].y);
  __syncthreads();
  for (int k = tid; k < A; k += NT) {
    float x = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) x += part[w][k];
    ds[(size_t)b * A + k] = 4.f * v[k] * x;
  }
}

// ------------------------------------------------------------------------------ launchers
bool attn_row_supported(int A, int T) { return (A == 512 || A == 1024) && T >= 1 && T <= kRowMaxT; }
bool attn_rowp_supported(int A, int T, int EG) { return attn_row_supported(A, T) && EG == kEG; }

// waves per workgroup of the projected kernels: forward 16 / 8 (A = 512 / 1024) as row_waves();
// backward 16 at A = 512 (128 VGPRs, 2 spilled: B = 256 17.47-17.51 -> 17.22 ms per step against
// 12 waves, 17.75 with 8) and 8 at A = 1024 (4 equal, 12 spills 75; profiles/r3/ab/rowp_waves.txt)
template <int NK>
constexpr int rowp_bwd_waves() { return NK == 1 ? 16 : 8; }

void launch_attn_fwd_rowp(const bf16* F, const bf16* G, const float* s, const float* v, const float* wc,
                          const float* cov, const int* lens, float* a_out, float* cov_out, float* covloss, float* gx,
                          bf16* gx_bf, int B, int T, int A, const int* dlen, int step, hipStream_t st, bf16* a_bf) {
#define LF(NK)                                                                                            \
  hipLaunchKernelGGL((attn_fwd_rowp_kernel<NK, row_waves<NK, false>()>), dim3(B),                        \
                     dim3(row_waves<NK, false>() * 64), 0, st, F, G, s, v, wc, cov, lens, a_out, cov_out, covloss, \
                     gx, gx_bf, T, dlen, step, a_bf)
  if (A == 512) LF(1);
  else LF(2);
#undef LF
}

void launch_attn_bwd_rowp(const bf16* G, const bf16* F, const float* s, const float* v, const float* wc,
                          const float* cov, const float* a, const float* dx, const float* gv, const float* Ga,
                          const float* dcov_next, const float* gcl, const int* lens, float* de_out, float* ds,
                          float* dcov_out, int B, int T, int A, const int* dlen, int step, hipStream_t st) {
#define LB(NK)                                                                                            \
  hipLaunchKernelGGL((attn_bwd_rowp_kernel<NK, rowp_bwd_waves<NK>()>), dim3(B), dim3(rowp_bwd_waves<NK>() * 64), \
                     0, st, G, F, s, v, wc, cov, a, dx, gv, Ga, dcov_next, gcl, lens, de_out, ds, dcov_out, T, dlen, step)
  if (A == 512) LB(1);
  else LB(2);
#undef LB
}

void launch_attn_fwd_row(const bf16* F, const bf16* E, const float* s, const float* v, const float* wc,
                         const float* cov, const int* lens, float* a_out, float* cov_out, float* covloss, float* ctx,
                         bf16* ctx_bf, int B, int T, int A, int rep, hipStream_t st, const int* cg, const float* asrc,
                         float* cov_keep) {
  // beam decode: each XCD takes whole articles (their hypotheses share F / E rows in its L2)
  const int xper = (rep > 1 && B % 8 == 0 && (B / 8) % rep == 0) ? B / 8 : 0;
#define LF(NK)                                                                                                 \
  hipLaunchKernelGGL((attn_fwd_row_kernel<NK, row_waves<NK, false>()>), dim3(B), dim3(row_waves<NK, false>() * 64), \
                     0, st, F, E, s, v, wc, cov, lens, a_out, cov_out, covloss, ctx, ctx_bf, T, rep, xper, cg, asrc, cov_keep)
  // beam decode at A = 512: 12 waves per workgroup (bench_decode 6093 / 6137 vs 6061 / 6105 summaries/s with 16,
  // 5945 / 5984 with 8: profiles/r5/runs/r5aw)
  if (A == 512 && rep > 1)
    hipLaunchKernelGGL((attn_fwd_row_kernel<1, 12>), dim3(B), dim3(12 * 64), 0, st, F, E, s, v, wc, cov, lens, a_out,
                       cov_out, covloss, ctx, ctx_bf, T, rep, xper, cg, asrc, cov_keep);
  else if (A == 512) LF(1);
  else LF(2);
#undef LF
}

// attribution probe: the beam-decode forward (A = 512, 12 waves) with PROBE bits
void launch_attn_fwd_row_probe(const bf16* F, const bf16* E, const float* s, const float* v, const float* wc,
                               const float* cov, const int* lens, float* a_out, float* ctx, int B, int T, int rep,
                               int probe, hipStream_t st) {
  const int xper = (rep > 1 && B % 8 == 0 && (B / 8) % rep == 0) ? B / 8 : 0;
#define LP(PB)                                                                                                  \
  hipLaunchKernelGGL((attn_fwd_row_kernel<1, 12, PB>), dim3(B), dim3(12 * 64), 0, st, F, E, s, v, wc, cov, lens, a_out, \
                     nullptr, nullptr, ctx, nullptr, T, rep, xper, nullptr, nullptr, nullptr)
  switch (probe) {
    case 0: LP(0); break;
    case 1: LP(1); break;
    case 2: LP(2); break;
    case 3: LP(3); break;
    case 4: LP(4); break;
    case 8: LP(8); break;
    default: LP(11); break;
  }
#undef LP
}

void launch_attn_bwd_row(const bf16* E, const bf16* F, const float* s, const float* v, const float* wc,
                         const float* cov, const float* a, const float* dctx, const float* ctx, const float* Ga,
                         const float* dcov_next, const float* gcl, const int* lens, float* de_out, float* ds,
                         float* dcov_out, int B, int T, int A, hipStream_t st) {
#define LB(NK)                                                                                                \
  hipLaunchKernelGGL((attn_bwd_row_kernel<NK, row_waves<NK, true>()>), dim3(B), dim3(row_waves<NK, true>() * 64), \
                     0, st, E, F, s, v, wc, cov, a, dctx, ctx, Ga, dcov_next, gcl, lens, de_out, ds, dcov_out, T)
  if (A == 512) LB(1);
  else LB(2);
#undef LB
}
