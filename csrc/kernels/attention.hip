// Bahdanau attention with coverage, one decoder step per launch pair
// (reference attention_decoder.py:79-129, model.py:463-480).
//
//   e_i   = sum_k v_k tanh(F[i,k] + s[k] + w_c[k] * cov_i)      (F = W_h enc_out, s = W_s[c;h] + b)
//   a     = masked softmax(e)                                    (== softmax*mask renormalised)
//   cov'  = cov + a           covloss = sum_i min(a_i, cov_i)
//   ctx   = sum_i a_i E[i,:]
//
// Score kernels map lanes to the feature axis (8 contiguous bf16 per lane = one
// 16-byte load of a [B][T][A] row) and waves to positions, so every F/E byte is read
// once per step with full-width loads; the per-position dot product is a 6-step DPP
// reduction.  The weight gradients of v, w_c and the [B,T,A] gradient of F are NOT
// accumulated per step: the backward step stores de_t and a post-loop kernel
// (attn_bwd_feat) recomputes tanh once over all steps, so the recurrent critical path
// only carries what the recurrence needs (ds_t, dcov_t).
#include "common.h"

#define POS_PER_WAVE 16
#define POS_PER_BLOCK 64

// ---------------------------------------------------------------- forward: scores
__global__ __launch_bounds__(256) void attn_score_kernel(
    const bf16* __restrict__ F, const float* __restrict__ s, const float* __restrict__ v,
    const float* __restrict__ wc, const float* __restrict__ cov, const int* __restrict__ lens,
    float* __restrict__ e, int T, int A) {
  const int b = blockIdx.y;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int len = lens[b];
  const int p0 = blockIdx.x * POS_PER_BLOCK + wid * POS_PER_WAVE;
  if (p0 >= len) return;  // masked positions are never read by the softmax
  const int NK = (A + 511) / 512;  // k-blocks of 512 per lane-slice
  float sk[2][8], vk[2][8], wk[2][8];
  for (int kb = 0; kb < NK; ++kb) {
    const int k0 = kb * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = k0 + j < A;
      sk[kb][j] = ok ? s[(size_t)b * A + k0 + j] : 0.f;
      vk[kb][j] = ok ? v[k0 + j] : 0.f;
      wk[kb][j] = (ok && wc) ? wc[k0 + j] : 0.f;
    }
  }
  const bf16* Fb = F + (size_t)b * T * A;
#pragma unroll 4
  for (int q = 0; q < POS_PER_WAVE; ++q) {
    const int p = p0 + q;
    if (p >= len) break;
    const float c = cov ? cov[(size_t)b * T + p] : 0.f;
    float acc = 0.f;
    for (int kb = 0; kb < NK; ++kb) {
      const int k0 = kb * 512 + lane * 8;
      if (k0 < A) {
        bf16x8 f = ld8(Fb + (size_t)p * A + k0);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += vk[kb][j] * ftanh(bf2f(f[j]) + sk[kb][j] + wk[kb][j] * c);
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) e[(size_t)b * T + p] = acc;
  }
}

// ------------------------------------------------- forward: softmax, coverage, context
// grid (A/64 feature chunks, B).  Every block recomputes the row softmax (T floats);
// block x==0 also publishes a_t, cov_{t+1} and the coverage loss of this step.
#define MAXT 2048
__global__ __launch_bounds__(256) void attn_softmax_ctx_kernel(
    const float* __restrict__ e, const bf16* __restrict__ E, const int* __restrict__ lens,
    const float* __restrict__ cov, float* __restrict__ a_out, float* __restrict__ cov_out,
    float* __restrict__ covloss, float* __restrict__ ctx, bf16* __restrict__ ctx_bf, int T, int A) {
  __shared__ float sa[MAXT];
  __shared__ float red[8];
  __shared__ float part[4][64];
  const int b = blockIdx.y;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int len = lens[b];
  const float* er = e + (size_t)b * T;
  float m = -INFINITY;
  for (int i = tid; i < len; i += 256) m = fmaxf(m, er[i]);
  m = block_max<256>(m, red);
  float sum = 0.f;
  for (int i = tid; i < len; i += 256) {
    float x = fexp(er[i] - m);
    sa[i] = x;
    sum += x;
  }
  sum = block_sum<256>(sum, red);
  const float inv = 1.0f / sum;
  for (int i = tid; i < len; i += 256) sa[i] *= inv;
  __syncthreads();
  if (blockIdx.x == 0) {
    float cl = 0.f;
    for (int i = tid; i < T; i += 256) {
      const float a = i < len ? sa[i] : 0.f;
      a_out[(size_t)b * T + i] = a;
      if (cov_out) {
        const float c = cov ? cov[(size_t)b * T + i] : 0.f;
        cov_out[(size_t)b * T + i] = c + a;
        cl += fminf(a, c);
      }
    }
    if (covloss) {
      cl = block_sum<256>(cl, red);
      if (tid == 0) covloss[b] = cl;
    }
  }
  // context: 64 features per block; lane = (pos sub-index 0..7, feature group 0..7)
  const int f0 = blockIdx.x * 64;
  const int ps = lane >> 3, fg = lane & 7;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bf16* Eb = E + (size_t)b * T * A + f0 + fg * 8;
  for (int i = wid * 8 + ps; i < len; i += 32) {
    const float a = sa[i];
    bf16x8 x = ld8(Eb + (size_t)i * A);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += a * bf2f(x[j]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float x = acc[j];
    x += __shfl_xor(x, 8, 64);
    x += __shfl_xor(x, 16, 64);
    x += __shfl_xor(x, 32, 64);
    acc[j] = x;
  }
  if (ps == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) part[wid][fg * 8 + j] = acc[j];
  }
  __syncthreads();
  if (tid < 64) {
    const float c = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid];
    ctx[(size_t)b * A + f0 + tid] = c;
    if (ctx_bf) ctx_bf[(size_t)b * A + f0 + tid] = f2bf(c);
  }
}

// ------------------------------------------------------------- backward step: da
//   da_i = Ga_i + dcov_next_i + g_cl*[a_i <= cov_i] + dctx . E[i,:]
__global__ __launch_bounds__(256) void attn_bwd_da_kernel(
    const bf16* __restrict__ E, const float* __restrict__ dctx, const float* __restrict__ Ga,
    const float* __restrict__ dcov_next, const float* __restrict__ a, const float* __restrict__ cov,
    const float* __restrict__ gcl, const int* __restrict__ lens, float* __restrict__ da, int T, int A) {
  const int b = blockIdx.y;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int len = lens[b];
  const int p0 = blockIdx.x * POS_PER_BLOCK + wid * POS_PER_WAVE;
  if (p0 >= len) return;
  const int NK = (A + 511) / 512;
  float dk[2][8];
  for (int kb = 0; kb < NK; ++kb) {
    const int k0 = kb * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) dk[kb][j] = k0 + j < A ? dctx[(size_t)b * A + k0 + j] : 0.f;
  }
  const float g = gcl ? gcl[b] : 0.f;
  const bf16* Eb = E + (size_t)b * T * A;
#pragma unroll 4
  for (int q = 0; q < POS_PER_WAVE; ++q) {
    const int p = p0 + q;
    if (p >= len) break;
    float acc = 0.f;
    for (int kb = 0; kb < NK; ++kb) {
      const int k0 = kb * 512 + lane * 8;
      if (k0 < A) {
        bf16x8 x = ld8(Eb + (size_t)p * A + k0);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += dk[kb][j] * bf2f(x[j]);
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) {
      const size_t ix = (size_t)b * T + p;
      float r = acc;
      if (Ga) r += Ga[ix];
      if (dcov_next) r += dcov_next[ix];
      if (gcl && a[ix] <= (cov ? cov[ix] : 0.f)) r += g;
      da[ix] = r;
    }
  }
}

// ----------------------------------------------------- backward step: de, ds, dcov
// de_i = a_i (da_i - sum_j a_j da_j);  ds_k = sum_i de_i v_k sech2(u_ik) (partial per
// 64-position chunk: dsp[b][chunk][A]);  dcov_i = dcov_next_i + g_cl*[a_i > cov_i]
//   + de_i sum_k v_k w_c_k sech2(u_ik).
__global__ __launch_bounds__(256) void attn_bwd_tanh_kernel(
    const bf16* __restrict__ F, const float* __restrict__ s, const float* __restrict__ v,
    const float* __restrict__ wc, const float* __restrict__ cov, const float* __restrict__ a,
    const float* __restrict__ da, const float* __restrict__ dcov_next, const float* __restrict__ gcl,
    const int* __restrict__ lens, float* __restrict__ de_out, float* __restrict__ dsp,
    float* __restrict__ dcov_out, int T, int A) {
  __shared__ float red[8];
  __shared__ float part[4][1024];
  const int b = blockIdx.y;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int len = lens[b];
  const size_t rb = (size_t)b * T;
  float S = 0.f;
  for (int i = tid; i < len; i += 256) S += a[rb + i] * da[rb + i];
  S = block_sum<256>(S, red);
  const int NK = (A + 511) / 512;
  const int p0 = blockIdx.x * POS_PER_BLOCK + wid * POS_PER_WAVE;
  const float g = gcl ? gcl[b] : 0.f;
  float sk[2][8], vk[2][8], wk[2][8], acc[2][8];
  for (int kb = 0; kb < NK; ++kb) {
    const int k0 = kb * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = k0 + j < A;
      sk[kb][j] = ok ? s[(size_t)b * A + k0 + j] : 0.f;
      vk[kb][j] = ok ? v[k0 + j] : 0.f;
      wk[kb][j] = (ok && wc) ? wc[k0 + j] : 0.f;
      acc[kb][j] = 0.f;
    }
  }
  const bf16* Fb = F + (size_t)b * T * A;
  for (int q = 0; q < POS_PER_WAVE; ++q) {
    const int p = p0 + q;
    if (p >= T) break;
    const size_t ix = rb + p;
    if (p >= len) {
      if (lane == 0) {
        de_out[ix] = 0.f;
        if (dcov_out) dcov_out[ix] = dcov_next ? dcov_next[ix] : 0.f;
      }
      continue;
    }
    const float ap = a[ix];
    const float de = ap * (da[ix] - S);
    const float c = cov ? cov[ix] : 0.f;
    float dcv = 0.f;
    for (int kb = 0; kb < NK; ++kb) {
      const int k0 = kb * 512 + lane * 8;
      if (k0 < A) {
        bf16x8 f = ld8(Fb + (size_t)p * A + k0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float th = ftanh(bf2f(f[j]) + sk[kb][j] + wk[kb][j] * c);
          const float gs = de * vk[kb][j] * (1.0f - th * th);
          acc[kb][j] += gs;
          dcv += gs * wk[kb][j];
        }
      }
    }
    if (dcov_out) dcv = wave_sum(dcv);
    if (lane == 0) {
      de_out[ix] = de;
      if (dcov_out) {
        float r = dcv + (dcov_next ? dcov_next[ix] : 0.f);
        if (gcl && ap > c) r += g;
        dcov_out[ix] = r;
      }
    }
  }
  for (int kb = 0; kb < NK; ++kb) {
    const int k0 = kb * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (k0 + j < A) part[wid][k0 + j] = acc[kb][j];
  }
  __syncthreads();
  float* out = dsp + ((size_t)b * gridDim.x + blockIdx.x) * A;
  for (int k = tid; k < A; k += 256) out[k] = part[0][k] + part[1][k] + part[2][k] + part[3][k];
}

// ------------------------------------------------------ post-loop: dF, dv, dw_c
// dF[b,i,k] = sum_t de[t,b,i] v_k sech2(u_tik); dv_k = sum de tanh(u); dwc_k = sum de v_k sech2 cov.
// Each wave keeps 8 positions x 8 features of dF in registers across all D steps.
__global__ __launch_bounds__(256) void attn_bwd_feat_kernel(
    const bf16* __restrict__ F, const float* __restrict__ S_all, const float* __restrict__ v,
    const float* __restrict__ wc, const float* __restrict__ cov_all, const float* __restrict__ de_all,
    const int* __restrict__ lens, float* __restrict__ dF, float* __restrict__ dv, float* __restrict__ dwc,
    int D, int B, int T, int A) {
  __shared__ float pv[4][512];
  __shared__ float pw[4][512];
  const int b = blockIdx.y;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int len = lens[b];
  const int kbase = blockIdx.z * 512;
  const int k0 = kbase + lane * 8;
  const bool kok = k0 < A;
  const int p0 = blockIdx.x * 32 + wid * 8;
  float vk[8], wk[8], adv[8], adw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool ok = kok && k0 + j < A;
    vk[j] = ok ? v[k0 + j] : 0.f;
    wk[j] = (ok && wc) ? wc[k0 + j] : 0.f;
    adv[j] = 0.f;
    adw[j] = 0.f;
  }
  if (p0 < len && kok) {
    const int np = min(8, len - p0);
    float f[8][8], acc[8][8];
    for (int q = 0; q < 8; ++q) {
      const int p = min(p0 + q, T - 1);
      bf16x8 x = ld8(F + ((size_t)b * T + p) * A + k0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f[q][j] = bf2f(x[j]);
        acc[q][j] = 0.f;
      }
    }
    for (int t = 0; t < D; ++t) {
      const float* st = S_all + ((size_t)t * B + b) * A + k0;
      float sk[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) sk[j] = st[j];
      const size_t rb = ((size_t)t * B + b) * T + p0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (q < np) {
          const float de = de_all[rb + q];
          const float c = cov_all ? cov_all[rb + q] : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float th = ftanh(f[q][j] + sk[j] + wk[j] * c);
            const float g = de * (1.0f - th * th);
            acc[q][j] += g * vk[j];
            adv[j] += de * th;
            adw[j] += g * vk[j] * c;
          }
        }
      }
    }
    for (int q = 0; q < np; ++q) {
      float* o = dF + ((size_t)b * T + p0 + q) * A + k0;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (k0 + j < A) o[j] = acc[q][j];
    }
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
      if (x != 0.f) atomicAdd(dv + kk, x);
      if (dwc && y != 0.f) atomicAdd(dwc + kk, y);
    }
  }
}

void launch_attn_score(const bf16* F, const float* s, const float* v, const float* wc, const float* cov,
                       const int* lens, float* e, int B, int T, int A, hipStream_t st) {
  dim3 grid((T + POS_PER_BLOCK - 1) / POS_PER_BLOCK, B);
  hipLaunchKernelGGL(attn_score_kernel, grid, dim3(256), 0, st, F, s, v, wc, cov, lens, e, T, A);
}
void launch_attn_softmax_ctx(const float* e, const bf16* E, const int* lens, const float* cov, float* a_out,
                             float* cov_out, float* covloss, float* ctx, bf16* ctx_bf, int B, int T, int A,
                             hipStream_t st) {
  dim3 grid(A / 64, B);
  hipLaunchKernelGGL(attn_softmax_ctx_kernel, grid, dim3(256), 0, st, e, E, lens, cov, a_out, cov_out, covloss, ctx,
                     ctx_bf, T, A);
}
void launch_attn_bwd_da(const bf16* E, const float* dctx, const float* Ga, const float* dcov_next, const float* a,
                        const float* cov, const float* gcl, const int* lens, float* da, int B, int T, int A,
                        hipStream_t st) {
  dim3 grid((T + POS_PER_BLOCK - 1) / POS_PER_BLOCK, B);
  hipLaunchKernelGGL(attn_bwd_da_kernel, grid, dim3(256), 0, st, E, dctx, Ga, dcov_next, a, cov, gcl, lens, da, T,
                     A);
}
int attn_nchunk(int T) { return (T + POS_PER_BLOCK - 1) / POS_PER_BLOCK; }
void launch_attn_bwd_tanh(const bf16* F, const float* s, const float* v, const float* wc, const float* cov,
                          const float* a, const float* da, const float* dcov_next, const float* gcl, const int* lens,
                          float* de_out, float* dsp, float* dcov_out, int B, int T, int A, hipStream_t st) {
  dim3 grid(attn_nchunk(T), B);
  hipLaunchKernelGGL(attn_bwd_tanh_kernel, grid, dim3(256), 0, st, F, s, v, wc, cov, a, da, dcov_next, gcl, lens,
                     de_out, dsp, dcov_out, T, A);
}
void launch_attn_bwd_feat(const bf16* F, const float* S_all, const float* v, const float* wc, const float* cov_all,
                          const float* de_all, const int* lens, float* dF, float* dv, float* dwc, int D, int B, int T,
                          int A, hipStream_t st) {
  dim3 grid((T + 31) / 32, B, (A + 511) / 512);
  hipLaunchKernelGGL(attn_bwd_feat_kernel, grid, dim3(256), 0, st, F, S_all, v, wc, cov_all, de_all, lens, dF, dv,
                     dwc, D, B, T, A);
}
