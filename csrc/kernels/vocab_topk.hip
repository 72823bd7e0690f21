// Decode vocab head for the device beam search (reference
// model.py:229-243, 146-183, 280-285).
//
//   vocab_logits_kernel grid (ceil(R/64), ceil(V/256)), 4 waves: a 64-row x 256-column tile of
//                       logits = X . W_out + b by MFMA (K = H), stored fp32 straight from the
//                       accumulators, plus the tile's per-row (max, sum exp) partials;
//   vocab_select_kernel grid R: log-sum-exp from the partials; tau = K-th largest TILE max is a
//                       lower bound of the row's K-th largest logit (tile maxima are distinct
//                       elements), so one scan keeps only x >= tau (a handful) for the plain
//                       top-K; then the pointer copy mass (LDS hash) and the exact top-K of the
//                       extended-vocab final distribution (same argument as final_topk in
//                       beam.hip: plain top-K union copied ids).
// Replaces a library GEMM + a separate per-element top-k pass over the logits.
#include "common.h"

#define VT_COLS 256   // vocab columns per workgroup
#define VT_ROWS 64    // rows per workgroup
#define VT_K 8        // max K (= 2 * beam, beam <= 4)
#define VM_CAND 4096  // max nt * K candidates in the merge
#define VM_HASH 2048
#define VT_HMAX 256   // hidden size limit of the logits kernel (X tile staged in LDS)

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

__global__ __launch_bounds__(256) void vocab_logits_kernel(
    const bf16* __restrict__ X,     // [R][H]  output-projection activations (bf16)
    const bf16* __restrict__ WT,    // [V][H]  output_projection/w transposed ("Bt")
    const float* __restrict__ bias, // [V]
    float* __restrict__ logits,     // [R][V]  fp32 (bias added)
    float* __restrict__ part_ms,    // [R][nt][2]  per tile (max, sum exp)
    int R, int V, int H) {
  __shared__ float Pm[4][VT_ROWS], Ps[4][VT_ROWS];
  __shared__ float St[4][16][68];  // per wave: one 16 x 64 row tile, staged for full-line stores
  __shared__ __attribute__((aligned(16))) bf16 Xs[VT_ROWS * (VT_HMAX + 8)];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // XCD-aware order: the RB row blocks of one vocab tile get block ids equal mod 8 (one XCD
  // under round-robin dealing), so the tile's W^T columns come from HBM once and are then
  // served from that XCD's L2 to the other row blocks
  const int RB = (R + VT_ROWS - 1) / VT_ROWS, nt = (V + VT_COLS - 1) / VT_COLS;
  const int slot = blockIdx.x >> 3, vt = (slot / RB) * 8 + (blockIdx.x & 7);
  if (vt >= nt) return;
  const int rb = (slot % RB) * VT_ROWS;
  const int cw = vt * VT_COLS + 64 * wid;  // this wave's first column
  // X rows of this block -> LDS once (shared by the 4 waves); every B fragment of the wave
  // (4 column tiles x H/32 k-steps) is issued before the first MFMA: one memory round trip.
  const int kof = 8 * (lane >> 4);
  for (int c = threadIdx.x; c < VT_ROWS * (H / 8); c += 256) {
    const int rr = c / (H / 8), k8 = (c % (H / 8)) * 8;
    *reinterpret_cast<bf16x8*>(&Xs[rr * (H + 8) + k8]) = ld8(X + (size_t)min(rb + rr, R - 1) * H + k8);
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  const bf16* brow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) brow[j] = WT + (size_t)min(cw + 16 * j + (lane & 15), V - 1) * H + kof;
  __syncthreads();
  for (int k0 = 0; k0 < H; k0 += 256) {  // H <= 256 in one pass (128 VGPRs of B fragments)
    bf16x8 b[8][4];
#pragma unroll
    for (int h = 0; h < 8; ++h)
#pragma unroll
      for (int j = 0; j < 4; ++j) b[h][j] = ld8(brow[j] + min(k0 + 32 * h, H - 32));
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      if (k0 + 32 * h >= H) break;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&Xs[(16 * i + (lane & 15)) * (H + 8) + k0 + 32 * h + kof]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a, b[h][j], acc[i][j]);
      }
    }
  }
  // ---- epilogue: + bias, store fp32, per-row (max, sum exp) over this wave's 64 columns.
  // Accumulator (i, j, r) holds row 16i + 4(lane>>4) + r, column 16j + (lane&15).
  float bj[4];
  bool cok[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = cw + 16 * j + (lane & 15);
    cok[j] = col < V;
    bj[j] = cok[j] ? bias[col] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = rb + 16 * i + 4 * (lane >> 4) + r;
      float x[4], m = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[j] = cok[j] ? acc[i][j][r] + bj[j] : -INFINITY;
        m = fmaxf(m, x[j]);
        St[wid][4 * (lane >> 4) + r][16 * j + (lane & 15)] = x[j];
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      float sm = 0.f;
      if (m > -INFINITY) {
#pragma unroll
        for (int j = 0; j < 4; ++j) sm += fexp(x[j] - m);  // exp(-inf) = 0 for padded columns
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) sm += __shfl_xor(sm, o, 64);
      if ((lane & 15) == 0) {
        Pm[wid][16 * i + 4 * (lane >> 4) + r] = m;
        Ps[wid][16 * i + 4 * (lane >> 4) + r] = sm;
      }
      if (r == 3) {
        // the 16-row tile i is staged: store it as 4 rows x 256 B per instruction
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const bool vec = (V % 4 == 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int tr = 4 * q + (lane >> 4), row2 = rb + 16 * i + tr, c4 = 4 * (lane & 15);
          const int col = cw + c4;
          if (row2 < R) {
            float* dst = logits + (size_t)row2 * V + col;
            if (vec && col + 4 <= V) {
              *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(&St[wid][tr][c4]);
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (col + e < V) dst[e] = St[wid][tr][c4 + e];
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      }
    }
  __syncthreads();
  if (wid == 0) {
    const int rr = lane, row = rb + rr;
    float m = Pm[0][rr], sm = Ps[0][rr];
#pragma unroll
    for (int w = 1; w < 4; ++w) ms_combine(m, sm, Pm[w][rr], Ps[w][rr]);
    if (row < R) {
      part_ms[((size_t)row * nt + vt) * 2] = m;
      part_ms[((size_t)row * nt + vt) * 2 + 1] = sm;
    }
  }
}

namespace {
__device__ __forceinline__ int vhslot(int w) { return (int)(((unsigned)w * 2654435761u) >> 21) & (VM_HASH - 1); }

// K rounds of wave arg-max over n LDS entries (selected entries knocked out)
__device__ __forceinline__ void vselect(float* v, int* id, int n, int K, float* out_v, int* out_i) {
  const int lane = threadIdx.x & 63;
  for (int round = 0; round < K; ++round) {
    float bv = -INFINITY;
    int bi = 0x7fffffff, bs = -1;
    for (int q = lane; q < n; q += 64) {
      const float x = v[q];
      const int xi = id[q];
      if (vbetter(x, xi, bv, bi)) { bv = x; bi = xi; bs = q; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64), os = __shfl_xor(bs, o, 64);
      if (vbetter(ov, oi, bv, bi)) { bv = ov; bi = oi; bs = os; }
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
}  // namespace

#define VS_THREADS 1024
__global__ __launch_bounds__(VS_THREADS) void vocab_select_kernel(
    const float* __restrict__ logits, const float* __restrict__ part_ms, const float* __restrict__ pgen,
    const float* __restrict__ attn, const int* __restrict__ ext, const int* __restrict__ lens,
    int* __restrict__ out_ids, float* __restrict__ out_lp, int V, int T, int K, int beam, int nt) {
  __shared__ int hkey[VM_HASH];
  __shared__ float hmass[VM_HASH];
  __shared__ float cv[VM_CAND];
  __shared__ int ci[VM_CAND];
  __shared__ float red[16];
  __shared__ float pv_s[VT_K];
  __shared__ int pi_s[VT_K];
  __shared__ int ncand, ncopy;
  const int r = blockIdx.x, tid = threadIdx.x;
  const int art = r / beam;
  const float* z = logits + (size_t)r * V;
  for (int i = tid; i < VM_HASH; i += VS_THREADS) { hkey[i] = -1; hmass[i] = 0.f; }
  // tile maxima -> LDS (for tau) and the log-sum-exp
  float m = -INFINITY;
  for (int q = tid; q < nt; q += VS_THREADS) {
    const float mq = part_ms[((size_t)r * nt + q) * 2];
    cv[q] = mq;
    ci[q] = q;
    m = fmaxf(m, mq);
  }
  const float M = block_max<VS_THREADS>(m, red);
  float s = 0.f;
  for (int q = tid; q < nt; q += VS_THREADS) {
    const float mq = part_ms[((size_t)r * nt + q) * 2];
    if (mq > -INFINITY) s += part_ms[((size_t)r * nt + q) * 2 + 1] * fexp(mq - M);
  }
  const float lse = M + __logf(block_sum<VS_THREADS>(s, red));
  if (tid < 64) vselect(cv, ci, nt, K, pv_s, pi_s);  // K-th largest tile max
  if (tid == 0) { ncand = 0; ncopy = 0; }
  __syncthreads();
  const float tau = pv_s[K - 1];
  __syncthreads();
  // survivors x >= tau of the row (a handful); vectorised scan
  const int V4 = V & ~3;
  constexpr int UNR = 16;  // 16 independent 16-B loads in flight per thread (V <= 64k: one pass)
  for (int c0 = tid * 4; c0 < V4; c0 += VS_THREADS * 4 * UNR) {
    float4 x[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int c = c0 + u * VS_THREADS * 4;
      x[u] = c < V4 ? *reinterpret_cast<const float4*>(z + c) : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const float xs[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (xs[j] >= tau) {
          const int slot = atomicAdd(&ncand, 1);
          if (slot < VM_CAND) { cv[slot] = xs[j]; ci[slot] = c0 + u * VS_THREADS * 4 + j; }
        }
    }
  }
  for (int c = V4 + tid; c < V; c += VS_THREADS)
    if (z[c] >= tau) {
      const int slot = atomicAdd(&ncand, 1);
      if (slot < VM_CAND) { cv[slot] = z[c]; ci[slot] = c; }
    }
  const float pg = pgen ? pgen[r] : 1.0f;
  const int len = pgen ? lens[art] : 0;
  for (int i = tid; i < len; i += VS_THREADS) {
    const int w = ext[(size_t)art * T + i];
    const float a = attn[(size_t)r * T + i];
    int h = vhslot(w);
    for (int probe = 0; probe < VM_HASH; ++probe) {
      const int prev = atomicCAS(&hkey[h], -1, w);
      if (prev == -1 || prev == w) {
        atomicAdd(&hmass[h], a);
        break;
      }
      h = (h + 1) & (VM_HASH - 1);
    }
  }
  __syncthreads();
  const int nc = ncand;
  if (nc > VM_CAND) {  // pathological ties: exact fallback by K-round full scans (wave 0)
    if (tid < 64) {
      for (int round = 0; round < K; ++round) {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
        for (int c = tid; c < V; c += 64) {
          const float x = z[c];
          bool taken = false;
          for (int p = 0; p < round; ++p) taken |= (pi_s[p] == c);
          if (!taken && vbetter(x, c, bv, bi)) { bv = x; bi = c; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const float ov = __shfl_xor(bv, o, 64);
          const int oi = __shfl_xor(bi, o, 64);
          if (vbetter(ov, oi, bv, bi)) { bv = ov; bi = oi; }
        }
        if (tid == 0) { pv_s[round] = bv; pi_s[round] = bi; }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      }
    }
  } else if (tid < 64) {
    vselect(cv, ci, nc, K, pv_s, pi_s);
  }
  __syncthreads();
  if (tid < K) {
    const int w = pi_s[tid];
    bool incopy = false;
    if (len > 0) {
      int h = vhslot(w);
      for (int probe = 0; probe < VM_HASH; ++probe) {
        const int kk = hkey[h];
        if (kk == -1) break;
        if (kk == w) { incopy = true; break; }
        h = (h + 1) & (VM_HASH - 1);
      }
    }
    cv[tid] = incopy ? -INFINITY : pg * fexp(pv_s[tid] - lse);
    ci[tid] = w;
  }
  __syncthreads();
  {
    // all of this thread's hash slots' logit loads in flight at once (one round trip)
    constexpr int SPT = VM_HASH / VS_THREADS;
    int wk[SPT];
    float zk[SPT];
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      wk[u] = hkey[tid + VS_THREADS * u];
      zk[u] = (wk[u] >= 0 && wk[u] < V) ? z[wk[u]] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      if (wk[u] < 0) continue;
      const float pv = wk[u] < V ? fexp(zk[u] - lse) : 0.f;
      const int slot = atomicAdd(&ncopy, 1);
      cv[K + slot] = pg * pv + (1.0f - pg) * hmass[tid + VS_THREADS * u];
      ci[K + slot] = wk[u];
    }
  }
  __syncthreads();
  if (tid < 64) {
    vselect(cv, ci, K + ncopy, K, pv_s, pi_s);
    if (tid < K) {
      out_ids[(size_t)r * K + tid] = pi_s[tid];
      out_lp[(size_t)r * K + tid] = __logf(pv_s[tid]);
    }
  }
}

int vocab_topk_tiles(int V) { return (V + VT_COLS - 1) / VT_COLS; }

void launch_vocab_topk(const bf16* X, const bf16* WT, const float* bias, const float* pgen, const float* attn,
                       const int* ext, const int* lens, int* out_ids, float* out_lp, float* logits, float* part_ms,
                       int R, int V, int H, int T, int K, int beam, hipStream_t st) {
  const int nt = vocab_topk_tiles(V);
  const int RB = (R + VT_ROWS - 1) / VT_ROWS;
  hipLaunchKernelGGL(vocab_logits_kernel, dim3(8 * RB * ((nt + 7) / 8)), dim3(256), 0, st, X, WT, bias, logits,
                     part_ms, R, V, H);
  hipLaunchKernelGGL(vocab_select_kernel, dim3(R), dim3(VS_THREADS), 0, st, logits, part_ms, pgen, attn, ext, lens, out_ids,
                     out_lp, V, T, K, beam, nt);
}
