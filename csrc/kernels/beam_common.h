// Beam bookkeeping shared by beam_step_kernel (beam.hip) and the vocab select kernel's fused
// per-article tail (vocab_topk.hip): extend each live hypothesis with its top-K candidates,
// rank by total log-prob, collect finished (STOP) hypotheses after min_dec steps, keep the
// best ``beam`` live ones (reference beam_search.py:110-156).
#pragma once
#include "common.h"
#include "launchers.h"

#define BEAM_CAND_MAX 16  // max beam (new hypotheses kept per step)

// ------------------------------------------------------------------ beam bookkeeping
__device__ __forceinline__ void beam_step_body(
    const int* __restrict__ top_ids, const float* __restrict__ top_lp, float* __restrict__ lp_sum,
    int* __restrict__ latest, int* __restrict__ gidx, int* __restrict__ tok_hist, int* __restrict__ par_hist,
    int* __restrict__ done, int* __restrict__ res_count, float* __restrict__ res_score, int* __restrict__ res_len,
    int* __restrict__ res_step, int* __restrict__ res_par, float* cval, int* cid, int* srt, int a, int lane, int t,
    int base, int beam, int K, int stop_id, int min_dec, float tot, int tid_cand, int nres0, int Na) {
  // tot / tid_cand / nres0: this lane's candidate and the result count, loaded by the caller
  // in the same memory round trip as the step counter and the done flag
  const int norig = t == 0 ? 1 : beam;
  const int ncand = norig * K;
  if (lane >= ncand) tot = -INFINITY;
  // stable rank: descending total, ties keep candidate order (readlane: a uniform lane index,
  // no LDS permute per candidate)
  int rank = 0;
  for (int q = 0; q < ncand; ++q) {
    const float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tot), q));
    if (v > tot || (v == tot && q < lane)) ++rank;
  }
  if (lane < ncand) {  // rank-ordered candidate table: value, token, parent
    cval[rank] = tot;
    cid[rank] = tid_cand;
    srt[rank] = lane / K;
  }
  __shared__ float nlp[BEAM_CAND_MAX];
  __shared__ int ntok[BEAM_CAND_MAX], npar[BEAM_CAND_MAX];
  __shared__ int nh_s, nres_s;
  __syncthreads();
  // The reference walks the ranked candidates in order: a STOP (from step min_dec on) becomes a
  // result, any other token a new hypothesis, until beam of either (beam_search.py:120-150).
  // Here every rank position decides at once: with the exclusive counts of results / hypotheses
  // ranked before it (ballot + popcount), position q is reached iff both counts are still below
  // beam, and its slot is that count.
  if (lane < 64) {
    const bool act = lane < ncand;
    const int tok = act ? cid[lane] : 0;
    const bool is_res = act && tok == stop_id && t >= min_dec;
    const bool is_hyp = act && tok != stop_id;
    const unsigned long long below = (1ull << lane) - 1ull;  // lanes < this one (lane <= 63)
    const unsigned long long mres = __ballot(is_res), mhyp = __ballot(is_hyp);
    const int ns = __popcll(mres & below), nn = __popcll(mhyp & below);
    const bool reached = act && nn < beam && nres0 + ns < beam;
    const float v = act ? cval[lane] : 0.f;
    const int par = act ? srt[lane] : 0;
    if (reached && is_res) {
      const int slot = a * beam + nres0 + ns;
      res_score[slot] = v / (float)(t + 2);
      res_len[slot] = t + 2;
      res_step[slot] = t;
      res_par[slot] = par;
    }
    if (reached && is_hyp) {
      nlp[nn] = v;
      ntok[nn] = tok;
      npar[nn] = par;
    }
    const unsigned long long mreach = __ballot(reached);
    if (lane == 0) {
      const int nres = nres0 + __popcll(mres & mreach);
      nh_s = __popcll(mhyp & mreach);
      nres_s = nres;
      res_count[a] = nres;
      if (nres >= beam) done[a] = 1;
    }
  }
  __syncthreads();
  if (lane < beam) {
    const int nh = nh_s, k = lane;
    const int kk = k < nh ? k : (nh > 0 ? nh - 1 : 0);
    const int par = nh > 0 ? npar[kk] : 0;
    lp_sum[base + k] = nh > 0 ? nlp[kk] : -INFINITY;
    latest[base + k] = nh > 0 ? ntok[kk] : stop_id;
    gidx[base + k] = base + par;
    tok_hist[(size_t)t * Na * beam + base + k] = nh > 0 ? ntok[kk] : stop_id;
    par_hist[(size_t)t * Na * beam + base + k] = par;
  }
  (void)nres_s;
}


// Beam bookkeeping of article a run by the LAST of its rows' workgroups in the vocab select
// kernel (vocab_topk.hip, BeamTail): the same steps as beam_step_kernel for one article, with
// t = *step - 1 (the step counter was advanced at the start of this decode step).  The rows'
// candidates arrive as tagged 64-bit granules {tag = step (15 bits) | id (17 bits), log-prob}
// written with relaxed agent-scope atomic stores by the rows' workgroups (possibly on other
// XCDs): the tail polls them until every tag is this step's -- no device-scope fence (on this
// GPU a release fence writes back the whole L2).  Every thread of the workgroup calls it (it
// contains block barriers); lanes < 64 do the work.  err: set when a poll times out.
__device__ __forceinline__ void beam_article_tail(const BeamTail& bt, int a, float* cval, int* cid, int* srt) {
  const int lane = threadIdx.x, beam = bt.beam, K = bt.K, base = a * beam;
  const size_t R = (size_t)bt.Na * beam;
  const int t = *bt.step - 1;
  const unsigned tag = (unsigned)(*bt.step) & 0x7fffu;
  const int is_done = bt.done[a], nres0 = bt.res_count[a];
  float tot = -INFINITY;
  int tid_cand = 0;
  if (lane < beam * K) {
    const int i = lane / K, j = lane % K;
    const unsigned long long* g = bt.gran + (size_t)(base + i) * K + j;
    unsigned long long x = 0;
    for (unsigned spins = 0;; ++spins) {
      x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((unsigned)(x >> 49) == tag) break;
      if (spins > (1u << 20)) {  // bounded: results garbage, error recorded, the grid drains
        __hip_atomic_store(bt.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    tid_cand = (int)((x >> 32) & 0x1ffffu);
    tot = bt.lp_sum[base + i] + __uint_as_float((unsigned)x);
  }
  if (bt.att_hist) {
    const size_t th = (size_t)min(t, bt.max_dec - 1);
    // (att was written by the previous launch; each row workgroup stores its own pg_hist entry)
    for (int i = lane; i < beam * bt.T; i += blockDim.x)
      bt.att_hist[(th * R + base) * bt.T + i] = bt.att[(size_t)base * bt.T + i];
  }
  if (is_done || t >= bt.max_dec) {
    if (lane < beam) bt.gidx[base + lane] = base + lane;
  } else {
    beam_step_body(nullptr, nullptr, bt.lp_sum, bt.latest, bt.gidx, bt.tok_hist, bt.par_hist, bt.done, bt.res_count,
                   bt.res_score, bt.res_len, bt.res_step, bt.res_par, cval, cid, srt, a, lane, t, base, beam, K,
                   bt.stop_id, bt.min_dec, tot, tid_cand, nres0, bt.Na);
  }
}
