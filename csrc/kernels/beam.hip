// Device-resident beam search for the pointer-generator decoder (SURVEY K17, K20, K26;
// reference model.py:146-183, 280-285 and beam_search.py:82-173).
//
// final_topk: one block per hypothesis row.  The extended-vocab final distribution
//   P(w) = p_gen * softmax(z)[w] * [w < V] + (1 - p_gen) * sum_i a_i [ext_i == w]
// is never materialised: the exact top-2k is the top-2k of the union of
//   (a) the plain top-2k of z over the vocabulary (monotone in P for words NOT copied), and
//   (b) every distinct copied id with its combined value,
// because a non-copied word outside the plain top-2k is beaten by >= 2k words whose true
// value is at least their plain value.  Ties break to the lower id (tf.nn.top_k).
//
// beam_step: one wave per article.  Candidates (hyp i, rank j) for i < (t == 0 ? 1 : beam)
// are ranked by total log-prob (all have the same length, so this is the reference's
// avg_log_prob order) with Python's stable tie order (i-major, j-minor); lane 0 then walks
// the ranking exactly like beam_search.py:144-154: [STOP] goes to results only when
// t >= min_dec_steps, otherwise it is dropped; stop at beam live hyps or beam results.
// Parents / tokens / scores of the new hyps are written for the next step's gather, plus
// the (token, parent) history used to backtrack the final sequences on the host.
#include "common.h"

#define TOPK_MAX 16
#define TOPK_THREADS 256

struct Cand {
  float v;
  int id;
};
__device__ __forceinline__ bool better(float v1, int i1, float v2, int i2) { return v1 > v2 || (v1 == v2 && i1 < i2); }

// Branch-light insertion into a register-resident sorted list (compile-time indices only,
// so the list stays in VGPRs): the new candidate bubbles down through the 16 slots.
__device__ __forceinline__ void cand_insert(Cand (&c)[TOPK_MAX], float v, int id) {
  if (!better(v, id, c[TOPK_MAX - 1].v, c[TOPK_MAX - 1].id)) return;
  Cand x{v, id};
#pragma unroll
  for (int p = 0; p < TOPK_MAX; ++p) {
    if (better(x.v, x.id, c[p].v, c[p].id)) {
      const Cand y = c[p];
      c[p] = x;
      x = y;
    }
  }
}

__global__ __launch_bounds__(TOPK_THREADS) void final_topk_kernel(
    const float* __restrict__ logits, const float* __restrict__ bias, const float* __restrict__ pgen,
    const float* __restrict__ attn, const int* __restrict__ ext, const int* __restrict__ lens,
    int* __restrict__ out_ids, float* __restrict__ out_lp, int V, int T, int K, int beam) {
  __shared__ float red[8];
  __shared__ float sv[TOPK_THREADS * TOPK_MAX];
  __shared__ int si[TOPK_THREADS * TOPK_MAX];
  __shared__ float sa[2048];
  __shared__ int se[2048];
  __shared__ float cv[2 * TOPK_MAX];
  __shared__ int ci[2 * TOPK_MAX];
  __shared__ int ncopy;
  const int r = blockIdx.x, tid = threadIdx.x;
  const int art = r / beam;
  const float* z = logits + (size_t)r * V;
  // ---- pass 1: LSE and per-thread plain top-K
  Cand c[TOPK_MAX];
#pragma unroll
  for (int k = 0; k < TOPK_MAX; ++k) c[k] = Cand{-INFINITY, 0x7fffffff};
  float m = -INFINITY, s = 0.f;
  for (int k = tid; k < V; k += TOPK_THREADS) {
    const float x = z[k] + bias[k];
    if (x > m) { s *= fexp(m - x); m = x; }
    s += fexp(x - m);
    cand_insert(c, x, k);
  }
  const float M = block_max<TOPK_THREADS>(m, red);
  const float S = block_sum<TOPK_THREADS>(m == -INFINITY ? 0.f : s * fexp(m - M), red);
  const float lse = M + __logf(S);
#pragma unroll
  for (int k = 0; k < TOPK_MAX; ++k) {
    if (k < K) {
      sv[tid * K + k] = c[k].v;
      si[tid * K + k] = c[k].id;
    }
  }
  const float pg = pgen ? pgen[r] : 1.0f;
  const int len = pgen ? lens[art] : 0;
  for (int i = tid; i < len; i += TOPK_THREADS) {
    sa[i] = attn[(size_t)r * T + i];
    se[i] = ext[(size_t)art * T + i];
  }
  if (tid == 0) ncopy = 0;
  __syncthreads();
  // ---- block merge of the plain candidates: K rounds of arg-max by wave 0
  if (tid < 64) {
    for (int round = 0; round < K; ++round) {
      float bv = -INFINITY;
      int bi = 0x7fffffff, bs = -1;
      for (int q = tid; q < TOPK_THREADS * K; q += 64) {
        if (better(sv[q], si[q], bv, bi)) { bv = sv[q]; bi = si[q]; bs = q; }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64), os = __shfl_xor(bs, o, 64);
        if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; bs = os; }
      }
      if (tid == 0) {
        // plain value -> final-dist probability
        cv[round] = pg * fexp(bv - lse);
        ci[round] = bi;
        if (bs >= 0) sv[bs] = -INFINITY;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
  }
  __syncthreads();
  // ---- copy distribution: representatives (first occurrence of each id) with combined value
  // candidates from the copy set are appended after the K plain ones (dedup below)
  for (int i = tid; i < len; i += TOPK_THREADS) {
    const int w = se[i];
    bool rep = true;
    float mass = 0.f;
    for (int j = 0; j < len; ++j) {
      if (se[j] == w) {
        if (j < i) { rep = false; break; }
        mass += sa[j];
      }
    }
    if (!rep) continue;
    const float pv = w < V ? fexp(z[w] + bias[w] - lse) : 0.f;
    const float val = pg * pv + (1.0f - pg) * mass;
    // keep the K best copy candidates in a small LDS list guarded by an atomic counter
    // (len <= T distinct ids; we only need the best K, so store all reps in sv/si scratch)
    const int slot = atomicAdd(&ncopy, 1);
    sv[slot] = val;
    si[slot] = w;
  }
  __syncthreads();
  if (tid < 64) {
    const int nc = ncopy;
    // drop plain candidates whose id is in the copy set (the copy entry carries the true value)
    for (int k = tid; k < K; k += 64) {
      const int w = ci[k];
      bool incopy = false;
      for (int q = 0; q < nc; ++q)
        if (si[q] == w) { incopy = true; break; }
      if (incopy) cv[k] = -INFINITY;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    // final K rounds over plain (K) + copy (nc) candidates
    for (int round = 0; round < K; ++round) {
      float bv = -INFINITY;
      int bi = 0x7fffffff, bs = -1;
      for (int q = tid; q < K + nc; q += 64) {
        const float v = q < K ? cv[q] : sv[q - K];
        const int id = q < K ? ci[q] : si[q - K];
        if (better(v, id, bv, bi)) { bv = v; bi = id; bs = q; }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64), os = __shfl_xor(bs, o, 64);
        if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; bs = os; }
      }
      if (tid == 0) {
        out_ids[(size_t)r * K + round] = bi;
        out_lp[(size_t)r * K + round] = __logf(bv);
        if (bs >= 0) {
          if (bs < K) cv[bs] = -INFINITY;
          else sv[bs - K] = -INFINITY;
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
  }
}

// ------------------------------------------------------------------ beam bookkeeping
__global__ __launch_bounds__(64) void beam_step_kernel(
    const int* __restrict__ top_ids, const float* __restrict__ top_lp,  // [R][K]
    float* __restrict__ lp_sum,        // [R] in: per live hyp; out: per new hyp
    int* __restrict__ latest,          // [R] out: token of each new hyp
    int* __restrict__ gidx,            // [R] out: global row of each new hyp's parent
    int* __restrict__ tok_hist, int* __restrict__ par_hist,  // [maxD][R]
    int* __restrict__ done, int* __restrict__ res_count,    // [Na]
    float* __restrict__ res_score, int* __restrict__ res_len, int* __restrict__ res_step,
    int* __restrict__ res_par,         // [Na][beam]
    const int* __restrict__ step, int beam, int K, int stop_id, int min_dec, int max_dec) {
  __shared__ float cval[64];
  __shared__ int cid[64];
  __shared__ int srt[64];
  const int a = blockIdx.x, lane = threadIdx.x;
  const int t = *step;
  const int base = a * beam;
  if (done[a] || t >= max_dec) {
    if (lane < beam) gidx[base + lane] = base + lane;
    return;
  }
  const int norig = t == 0 ? 1 : beam;
  const int ncand = norig * K;
  float tot = -INFINITY;
  if (lane < ncand) {
    const int i = lane / K, j = lane % K;
    tot = lp_sum[base + i] + top_lp[(size_t)(base + i) * K + j];
    cval[lane] = tot;
    cid[lane] = top_ids[(size_t)(base + i) * K + j];
  }
  // stable rank: descending total, ties keep candidate order
  int rank = 0;
  for (int q = 0; q < ncand; ++q) {
    const float v = __shfl(tot, q, 64);
    if (v > tot || (v == tot && q < lane)) ++rank;
  }
  if (lane < ncand) srt[rank] = lane;
  __syncthreads();
  if (lane == 0) {
    int nres = res_count[a], nh = 0;
    float new_lp[TOPK_MAX];
    int new_tok[TOPK_MAX], new_par[TOPK_MAX];
    for (int q = 0; q < ncand; ++q) {
      const int cnd = srt[q];
      const int i = cnd / K, tok = cid[cnd];
      const float v = cval[cnd];
      if (tok == stop_id) {
        if (t >= min_dec && nres < beam) {
          res_score[a * beam + nres] = v / (float)(t + 2);
          res_len[a * beam + nres] = t + 2;
          res_step[a * beam + nres] = t;
          res_par[a * beam + nres] = i;
          ++nres;
        }
      } else if (nh < beam) {
        new_lp[nh] = v;
        new_tok[nh] = tok;
        new_par[nh] = i;
        ++nh;
      }
      if (nh == beam || nres == beam) break;
    }
    res_count[a] = nres;
    if (nres >= beam) done[a] = 1;
    for (int k = 0; k < beam; ++k) {
      const int kk = k < nh ? k : (nh > 0 ? nh - 1 : 0);
      const int par = nh > 0 ? new_par[kk] : 0;
      lp_sum[base + k] = nh > 0 ? new_lp[kk] : -INFINITY;
      latest[base + k] = nh > 0 ? new_tok[kk] : stop_id;
      gidx[base + k] = base + par;
      tok_hist[(size_t)t * gridDim.x * beam + base + k] = nh > 0 ? new_tok[kk] : stop_id;
      par_hist[(size_t)t * gridDim.x * beam + base + k] = par;
    }
  }
}

void launch_final_topk(const float* logits, const float* bias, const float* pgen, const float* attn, const int* ext,
                       const int* lens, int* out_ids, float* out_lp, int R, int V, int T, int K, int beam,
                       hipStream_t st) {
  hipLaunchKernelGGL(final_topk_kernel, dim3(R), dim3(TOPK_THREADS), 0, st, logits, bias, pgen, attn, ext, lens,
                     out_ids, out_lp, V, T, K, beam);
}

void launch_beam_step(const int* top_ids, const float* top_lp, float* lp_sum, int* latest, int* gidx, int* tok_hist,
                      int* par_hist, int* done, int* res_count, float* res_score, int* res_len, int* res_step,
                      int* res_par, const int* step, int Na, int beam, int K, int stop_id, int min_dec, int max_dec,
                      hipStream_t st) {
  hipLaunchKernelGGL(beam_step_kernel, dim3(Na), dim3(64), 0, st, top_ids, top_lp, lp_sum, latest, gidx, tok_hist,
                     par_hist, done, res_count, res_score, res_len, res_step, res_par, step, beam, K, stop_id, min_dec,
                     max_dec);
}
