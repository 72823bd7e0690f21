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
#include "beam_common.h"

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

#define MAX_SPLIT 64  // blocks per row in the vocab pass: ceil(V / (256*32)), V <= 524288
#define HASH_SIZE 2048

// Block-wide selection of the best K (value, id) pairs from n LDS entries by wave 0:
// K rounds of wave arg-max, selected entries knocked out.  Writes out_v / out_i.
__device__ __forceinline__ void wave_select(float* v, int* id, int n, int K, float* out_v, int* out_i) {
  const int lane = threadIdx.x & 63;
  for (int round = 0; round < K; ++round) {
    float bv = -INFINITY;
    int bi = 0x7fffffff, bs = -1;
    for (int q = lane; q < n; q += 64) {
      const float x = v[q];
      const int xi = id[q];
      if (better(x, xi, bv, bi)) { bv = x; bi = xi; bs = q; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64), os = __shfl_xor(bs, o, 64);
      if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; bs = os; }
    }
    if (lane == 0) {
      out_v[round] = bv;
      out_i[round] = bi;
      if (bs >= 0) v[bs] = -INFINITY;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  }
}

// Pass 1, grid (nsplit, R): each block owns <= 256*32 logits of one row, held in
// registers (32 per thread, 4 vector batches issued together).  One read gives the online
// (max, sumexp) and the per-thread maximum; tau = K-th largest per-thread maximum is a
// lower bound of the true K-th largest value (the top-K thread maxima are K distinct
// elements), so every top-K element satisfies x >= tau.  Survivors are appended to LDS
// and the block's top-K selected from them.  Pathological ties (> FILTER_CAP survivors,
// e.g. all-equal logits) fall back to a register bubble-insert top-K.
#define PER_THREAD 32
#define FILTER_CAP 2048
__global__ __launch_bounds__(TOPK_THREADS) void final_topk_partial_kernel(
    const float* __restrict__ logits, const float* __restrict__ bias, float* __restrict__ part_ms,
    float* __restrict__ part_v, int* __restrict__ part_i, int V, int K, int per) {
  __shared__ float red[8];
  __shared__ float sv[FILTER_CAP];
  __shared__ int si[FILTER_CAP];
  __shared__ float tmax_v[TOPK_THREADS];
  __shared__ int tmax_i[TOPK_THREADS];
  __shared__ float selv[TOPK_MAX];
  __shared__ int seli[TOPK_MAX];
  __shared__ int cnt;
  const int r = blockIdx.y, sp = blockIdx.x, tid = threadIdx.x;
  const int lo = sp * per, hi = min(V, lo + per);
  const float* z = logits + (size_t)r * V;
  float x[PER_THREAD];
  const bool vec = (V % 8 == 0) && (per % 8 == 0);
#pragma unroll
  for (int bt = 0; bt < PER_THREAD / 8; ++bt) {
    const int k0 = lo + (bt * TOPK_THREADS + tid) * 8;
    if (vec && k0 + 8 <= hi) {
      const float4 a0 = *reinterpret_cast<const float4*>(z + k0), a1 = *reinterpret_cast<const float4*>(z + k0 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(bias + k0), b1 = *reinterpret_cast<const float4*>(bias + k0 + 4);
      x[bt * 8 + 0] = a0.x + b0.x; x[bt * 8 + 1] = a0.y + b0.y; x[bt * 8 + 2] = a0.z + b0.z; x[bt * 8 + 3] = a0.w + b0.w;
      x[bt * 8 + 4] = a1.x + b1.x; x[bt * 8 + 5] = a1.y + b1.y; x[bt * 8 + 6] = a1.z + b1.z; x[bt * 8 + 7] = a1.w + b1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[bt * 8 + j] = (k0 + j < hi) ? z[k0 + j] + bias[k0 + j] : -INFINITY;
    }
  }
  float m = -INFINITY;
  int mi = 0x7fffffff;
#pragma unroll
  for (int q = 0; q < PER_THREAD; ++q) {
    const int id = lo + ((q >> 3) * TOPK_THREADS + tid) * 8 + (q & 7);
    if (better(x[q], id, m, mi)) { m = x[q]; mi = id; }
  }
  float s = 0.f;
  if (m > -INFINITY) {
#pragma unroll
    for (int q = 0; q < PER_THREAD; ++q) s += fexp(x[q] - m);
  }
  const float M = block_max<TOPK_THREADS>(m, red);
  const float S = block_sum<TOPK_THREADS>(m == -INFINITY ? 0.f : s * fexp(m - M), red);
  tmax_v[tid] = m;
  tmax_i[tid] = mi;
  if (tid == 0) cnt = 0;
  __syncthreads();
  if (tid < 64) wave_select(tmax_v, tmax_i, TOPK_THREADS, K, selv, seli);
  __syncthreads();
  const float tau = selv[K - 1];
#pragma unroll
  for (int q = 0; q < PER_THREAD; ++q) {
    if (x[q] >= tau && x[q] > -INFINITY) {
      const int slot = atomicAdd(&cnt, 1);
      if (slot < FILTER_CAP) {
        sv[slot] = x[q];
        si[slot] = lo + ((q >> 3) * TOPK_THREADS + tid) * 8 + (q & 7);
      }
    }
  }
  __syncthreads();
  const int n = cnt;
  const size_t o = ((size_t)r * gridDim.x + sp) * K;
  if (n <= FILTER_CAP) {
    if (tid < 64) wave_select(sv, si, n, K, part_v + o, part_i + o);
  } else {  // tie-heavy fallback: exact per-thread insertion then block selection
    Cand c[TOPK_MAX];
#pragma unroll
    for (int k = 0; k < TOPK_MAX; ++k) c[k] = Cand{-INFINITY, 0x7fffffff};
#pragma unroll
    for (int q = 0; q < PER_THREAD; ++q) cand_insert(c, x[q], lo + ((q >> 3) * TOPK_THREADS + tid) * 8 + (q & 7));
    __syncthreads();
#pragma unroll
    for (int k = 0; k < TOPK_MAX; ++k) {
      if (k < K && tid * K + k < FILTER_CAP) {
        sv[tid * K + k] = c[k].v;
        si[tid * K + k] = c[k].id;
      }
    }
    __syncthreads();
    if (tid < 64) wave_select(sv, si, min(TOPK_THREADS * K, FILTER_CAP), K, part_v + o, part_i + o);
  }
  if (tid == 0) {
    part_ms[((size_t)r * gridDim.x + sp) * 2] = M;
    part_ms[((size_t)r * gridDim.x + sp) * 2 + 1] = S;
  }
}

__device__ __forceinline__ int hslot(int w) { return (int)(((unsigned)w * 2654435761u) >> 21) & (HASH_SIZE - 1); }

// Pass 2, grid R: merge the TOPK_SPLIT partials (LSE + plain top-K), build the copy
// distribution with an LDS hash table (one atomicCAS/atomicAdd per source position),
// replace copied ids' plain values by their combined value, take the final top-K.
__global__ __launch_bounds__(TOPK_THREADS) void final_topk_merge_kernel(
    const float* __restrict__ part_ms, const float* __restrict__ part_v, const int* __restrict__ part_i,
    const float* __restrict__ logits, const float* __restrict__ bias, const float* __restrict__ pgen,
    const float* __restrict__ attn, const int* __restrict__ ext, const int* __restrict__ lens,
    int* __restrict__ out_ids, float* __restrict__ out_lp, int V, int T, int K, int beam, int nsplit) {
  __shared__ int hkey[HASH_SIZE];
  __shared__ float hmass[HASH_SIZE];
  __shared__ float cvv[MAX_SPLIT * TOPK_MAX + HASH_SIZE];
  __shared__ int cii[MAX_SPLIT * TOPK_MAX + HASH_SIZE];
  __shared__ float plain_v[TOPK_MAX];
  __shared__ int plain_i[TOPK_MAX];
  __shared__ int ncopy;
  __shared__ float s_lse;
  const int r = blockIdx.x, tid = threadIdx.x;
  const int art = r / beam;
  for (int i = tid; i < HASH_SIZE; i += TOPK_THREADS) { hkey[i] = -1; hmass[i] = 0.f; }
  if (tid == 0) {
    float M = -INFINITY;
    for (int q = 0; q < nsplit; ++q) M = fmaxf(M, part_ms[((size_t)r * nsplit + q) * 2]);
    float S = 0.f;
    for (int q = 0; q < nsplit; ++q) {
      const float mq = part_ms[((size_t)r * nsplit + q) * 2];
      if (mq > -INFINITY) S += part_ms[((size_t)r * nsplit + q) * 2 + 1] * fexp(mq - M);
    }
    s_lse = M + __logf(S);
    ncopy = 0;
  }
  for (int q = tid; q < nsplit * K; q += TOPK_THREADS) {
    cvv[q] = part_v[(size_t)r * nsplit * K + q];
    cii[q] = part_i[(size_t)r * nsplit * K + q];
  }
  __syncthreads();
  const float lse = s_lse;
  const float pg = pgen ? pgen[r] : 1.0f;
  const int len = pgen ? (int)DCHECK_IDX(lens[art], 0, T + 1, CHK_LOSS_LEN) : 0;
  // copy mass per distinct id
  for (int i = tid; i < len; i += TOPK_THREADS) {
    const int w = ext[(size_t)art * T + i];
    const float a = attn[(size_t)r * T + i];
    int h = hslot(w);
    for (int probe = 0; probe < HASH_SIZE; ++probe) {
      const int prev = atomicCAS(&hkey[h], -1, w);
      if (prev == -1 || prev == w) {
        atomicAdd(&hmass[h], a);
        break;
      }
      h = (h + 1) & (HASH_SIZE - 1);
    }
  }
  __syncthreads();
  // plain top-K over the split winners (logit values)
  if (tid < 64) wave_select(cvv, cii, nsplit * K, K, plain_v, plain_i);
  __syncthreads();
  // candidates: plain ids not in the copy set (value p_gen*pv) + every copied id (combined)
  if (tid < K) {
    const int w = plain_i[tid];
    bool incopy = false;
    if (len > 0) {
      int h = hslot(w);
      for (int probe = 0; probe < HASH_SIZE; ++probe) {
        const int kk = hkey[h];
        if (kk == -1) break;
        if (kk == w) { incopy = true; break; }
        h = (h + 1) & (HASH_SIZE - 1);
      }
    }
    cvv[tid] = incopy ? -INFINITY : pg * fexp(plain_v[tid] - lse);
    cii[tid] = w;
  }
  __syncthreads();
  for (int hsl = tid; hsl < HASH_SIZE; hsl += TOPK_THREADS) {
    const int w = hkey[hsl];
    if (w < 0) continue;
    const float pv = w < V ? fexp(logits[(size_t)r * V + w] + bias[w] - lse) : 0.f;
    const int slot = atomicAdd(&ncopy, 1);
    cvv[K + slot] = pg * pv + (1.0f - pg) * hmass[hsl];
    cii[K + slot] = w;
  }
  __syncthreads();
  if (tid < 64) {
    wave_select(cvv, cii, K + ncopy, K, plain_v, plain_i);
    if (tid < K) {
      out_ids[(size_t)r * K + tid] = plain_i[tid];
      out_lp[(size_t)r * K + tid] = __logf(plain_v[tid]);
    }
  }
}

__global__ __launch_bounds__(64) void beam_step_kernel(
    const int* __restrict__ top_ids, const float* __restrict__ top_lp,  // [R][K]
    float* __restrict__ lp_sum,        // [R] in: per live hyp; out: per new hyp
    int* __restrict__ latest,          // [R] out: token of each new hyp
    int* __restrict__ gidx,            // [R] out: global row of each new hyp's parent
    int* __restrict__ tok_hist, int* __restrict__ par_hist,  // [maxD][R]
    int* __restrict__ done, int* __restrict__ res_count,    // [Na]
    float* __restrict__ res_score, int* __restrict__ res_len, int* __restrict__ res_step,
    int* __restrict__ res_par,         // [Na][beam]
    int* __restrict__ step, unsigned* __restrict__ ctr,  // step advanced by the last block to finish
    const float* __restrict__ att, float* __restrict__ att_hist,  // optional: [R][T] -> [maxD][R][T]
    const float* __restrict__ pg, float* __restrict__ pg_hist,    // optional: [R] -> [maxD][R]
    int T, int beam, int K, int stop_id, int min_dec, int max_dec) {
  __shared__ float cval[64];
  __shared__ int cid[64];
  __shared__ int srt[64];
  const int a = blockIdx.x, lane = threadIdx.x;
  const int base = a * beam;
  const size_t R = (size_t)gridDim.x * beam;
  // one memory round trip for everything the bookkeeping reads: the step counter, the done
  // flag, the result count and this lane's candidate (rows of step t > 0; at t == 0 only row
  // base's K candidates are used and the others are masked in the body)
  // ctr == nullptr: beam_gather advanced the counter at the start of this decode step
  const int t = ctr ? *step : *step - 1;
  const int is_done = done[a], nres0 = res_count[a];
  float tot = -INFINITY;
  int tid_cand = 0;
  if (lane < beam * K) {
    const int i = lane / K, j = lane % K;
    tot = lp_sum[base + i] + top_lp[(size_t)(base + i) * K + j];
    tid_cand = top_ids[(size_t)(base + i) * K + j];
  }
  if (att_hist) {  // attention / p_gen history for the visualiser, row t (clamped)
    const size_t th = (size_t)min(t, max_dec - 1);
    for (int i = lane; i < beam * T; i += 64) att_hist[(th * R + base) * T + i] = att[(size_t)base * T + i];
    if (pg_hist && lane < beam) pg_hist[th * R + base + lane] = pg[base + lane];
  }
  if (is_done || t >= max_dec) {
    if (lane < beam) gidx[base + lane] = base + lane;
  } else {
    beam_step_body(top_ids, top_lp, lp_sum, latest, gidx, tok_hist, par_hist, done, res_count, res_score, res_len,
                   res_step, res_par, cval, cid, srt, a, lane, t, base, beam, K, stop_id, min_dec, tot, tid_cand,
                   nres0, (int)gridDim.x);
  }
  // grid-wide step advance (standalone use): every block read *step above; the last one to
  // arrive bumps it -- a fence plus one same-address atomic per article (64 serialised L2
  // atomics at 64 articles), which the decoder avoids by letting beam_gather advance it
  if (ctr && lane == 0) {
    __threadfence();
    if (atomicAdd(ctr, 1u) == gridDim.x - 1) {
      *step = t + 1;
      *ctr = 0u;
    }
  }
}

// ------------------------------------------------------------------ state gather
// One block per hypothesis row r with parent g = gidx[r]: copies the parent's decoder
// state (c fp32, h bf16, post-cell ctx fp32 -> fp32 + bf16), advances coverage
// cov'[r] = cov_src[g] + a[g] (coverage on), and gathers the per-token input tables
// (XG = (emb.W_in + b).W_cell[:E] + b_cell, x0 = emb.W_in + b) for the hypothesis's
// latest token (in-article OOV ids -> [UNK]).  Replaces ~10 tiny gather / elementwise
// launches per decode step.
__global__ __launch_bounds__(256) void beam_gather_kernel(
    const int* __restrict__ gidx, const int* __restrict__ latest,
    const float* __restrict__ c_src, const bf16* __restrict__ h_src, const float* __restrict__ ctx_src,
    const float* __restrict__ a_src, const float* __restrict__ cov_src,
    const float* __restrict__ XGtab, const float* __restrict__ Xtab,
    float* __restrict__ c_out, bf16* __restrict__ h_out, float* __restrict__ ctx_out, bf16* __restrict__ ctxb_out,
    float* __restrict__ cov_out, float* __restrict__ XG_out, float* __restrict__ x_out,
    int H, int A, int T, int E, int V, int unk, int* __restrict__ step) {
  const int r = blockIdx.x, tid = threadIdx.x;
  // step (optional): the decode-step counter, advanced here -- one plain store by one thread,
  // the kernel boundary orders it before this step's beam_step (which then reads t = step - 1)
  if (step && r == 0 && tid == 0) *step += 1;
  const int g = (int)DCHECK_IDX(gidx[r], 0, (int)gridDim.x, CHK_BEAM_PARENT);
  int tok = (int)DCHECK_IDX(latest[r], 0, 0x7fffffff, CHK_BEAM_TOKEN);
  tok = tok < V ? tok : unk;
  for (int i = tid; i < H; i += 256) {
    c_out[(size_t)r * H + i] = c_src[(size_t)g * H + i];
    h_out[(size_t)r * H + i] = h_src[(size_t)g * H + i];
  }
  for (int i = tid; i < A; i += 256) {
    const float v = ctx_src[(size_t)g * A + i];
    ctx_out[(size_t)r * A + i] = v;
    ctxb_out[(size_t)r * A + i] = f2bf(v);
  }
  if (cov_out)
    for (int i = tid; i < T; i += 256) cov_out[(size_t)r * T + i] = cov_src[(size_t)g * T + i] + a_src[(size_t)g * T + i];
  for (int i = tid; i < 4 * H; i += 256) XG_out[(size_t)r * 4 * H + i] = XGtab[(size_t)tok * 4 * H + i];
  for (int i = tid; i < E; i += 256) x_out[(size_t)r * E + i] = Xtab[(size_t)tok * E + i];
}

void launch_beam_gather(const int* gidx, const int* latest, const float* c_src, const bf16* h_src,
                        const float* ctx_src, const float* a_src, const float* cov_src, const float* XGtab,
                        const float* Xtab, float* c_out, bf16* h_out, float* ctx_out, bf16* ctxb_out, float* cov_out,
                        float* XG_out, float* x_out, int R, int H, int A, int T, int E, int V, int unk,
                        int* step, hipStream_t st) {
  hipLaunchKernelGGL(beam_gather_kernel, dim3(R), dim3(256), 0, st, gidx, latest, c_src, h_src, ctx_src, a_src,
                     cov_src, XGtab, Xtab, c_out, h_out, ctx_out, ctxb_out, cov_out, XG_out, x_out, H, A, T, E, V,
                     unk, step);
}

int topk_split(int V) { return (V + TOPK_THREADS * PER_THREAD - 1) / (TOPK_THREADS * PER_THREAD); }

void launch_final_topk(const float* logits, const float* bias, const float* pgen, const float* attn, const int* ext,
                       const int* lens, int* out_ids, float* out_lp, float* part_ms, float* part_v, int* part_i, int R,
                       int V, int T, int K, int beam, hipStream_t st) {
  const int ns = topk_split(V);
  const int per = ((V + ns - 1) / ns + 7) / 8 * 8;
  hipLaunchKernelGGL(final_topk_partial_kernel, dim3(ns, R), dim3(TOPK_THREADS), 0, st, logits, bias, part_ms, part_v,
                     part_i, V, K, per);
  hipLaunchKernelGGL(final_topk_merge_kernel, dim3(R), dim3(TOPK_THREADS), 0, st, part_ms, part_v, part_i, logits, bias,
                     pgen, attn, ext, lens, out_ids, out_lp, V, T, K, beam, ns);
}

void launch_beam_step(const int* top_ids, const float* top_lp, float* lp_sum, int* latest, int* gidx, int* tok_hist,
                      int* par_hist, int* done, int* res_count, float* res_score, int* res_len, int* res_step,
                      int* res_par, int* step, unsigned* ctr, const float* att, float* att_hist, const float* pg,
                      float* pg_hist, int T, int Na, int beam, int K, int stop_id, int min_dec, int max_dec,
                      hipStream_t st) {
  hipLaunchKernelGGL(beam_step_kernel, dim3(Na), dim3(64), 0, st, top_ids, top_lp, lp_sum, latest, gidx, tok_hist,
                     par_hist, done, res_count, res_score, res_len, res_step, res_par, step, ctr, att, att_hist, pg,
                     pg_hist, T, beam, K, stop_id, min_dec, max_dec);
}
