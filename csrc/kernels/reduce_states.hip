// reduce_states: the encoder's final fw/bw LSTM states -> the decoder's initial state
// (reference model.py:96-120):
//   c0 = relu([c_fw, c_bw] . W_reduce_c + b_c),   h0 = relu([h_fw, h_bw] . W_reduce_h + b_h).
// Forward: ONE launch for both problems (blockIdx.z), reading the final states straight from
// the encoder's step-frame state buffers (no concat, no casts) and writing the decoder's
// initial state buffers (fp32 c, bf16 c and h) plus the pre-activations (backward mask) and
// bf16 copies of the concatenated inputs (operands of the weight-gradient GEMMs).
// Backward: ONE launch: dp = g * [pre > 0] -> bf16 dp (weight-gradient GEMM operand), the
// bias gradient (column sums of dp, one atomic per column per workgroup) and
// d_old = dp . W^T written directly into the encoder BPTT's step-frame seeds (dc_carry /
// dh_fin halves [fw; bw]).  Replaces ~25 small torch launches per training step.
#include "common.h"

namespace {

// A fragment of [x_fw, x_bw] row ar at absolute k (8 consecutive columns never straddle
// the fw/bw boundary: H % 32 == 0)
template <typename TX>
__device__ __forceinline__ bf16x8 ld_state(const TX* x0, size_t dstride, int ar, int H, int k);
template <>
__device__ __forceinline__ bf16x8 ld_state<float>(const float* x0, size_t dstride, int ar, int H, int k) {
  const int d = k >= H;
  return ld8f(x0 + d * dstride + (size_t)ar * H + (k - d * H));
}
template <>
__device__ __forceinline__ bf16x8 ld_state<bf16>(const bf16* x0, size_t dstride, int ar, int H, int k) {
  const int d = k >= H;
  return ld8(x0 + d * dstride + (size_t)ar * H + (k - d * H));
}

template <typename TX>
__device__ __forceinline__ void rs_fwd_body(const TX* x0, size_t dstride, const bf16* WT, const float* bias,
                                            float* pre, float* out_f, bf16* out_b, bf16* xcat, int B, int H,
                                            float* red) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = blockIdx.x * 16, r0 = blockIdx.y * 16;
  const int ar = min(r0 + (lane & 15), B - 1), kof = 8 * (lane >> 4), K = 2 * H;
  const bf16* brow = WT + (size_t)(n0 + (lane & 15)) * K + kof;
  const int nst = K / 32;
  const int k0 = (wid * nst / 4) * 32, k1 = ((wid + 1) * nst / 4) * 32;
  f32x4 acc[1] = {f32x4{0, 0, 0, 0}};
  kslice_mma<1>([&](int k) { return ld_state<TX>(x0, dstride, ar, H, k + kof); },
                [&](int, int k) { return ld8(brow + k); }, k0, k1, acc);
  float o[1];
  ksplit_reduce<1>(acc, red, o);
  const int r = r0 + (lane >> 4) * 4 + wid, n = n0 + (lane & 15);
  if (r < B) {
    const size_t ix = (size_t)r * H + n;
    const float v = o[0] + bias[n];
    pre[ix] = v;
    const float y = fmaxf(v, 0.f);
    if (out_f) out_f[ix] = y;
    out_b[ix] = f2bf(y);
  }
  // bf16 copy of the concatenated input rows (column tile 0 only: each row once)
  if (blockIdx.x == 0 && xcat) {
    for (int idx = threadIdx.x; idx < 16 * K; idx += 256) {
      const int rr = r0 + idx / K, k = idx % K;
      if (rr < B) {
        const int d = k >= H;
        xcat[(size_t)rr * K + k] = f2bf((float)x0[d * dstride + (size_t)rr * H + (k - d * H)]);
      }
    }
  }
}

}  // namespace

// grid (H/16, ceil(B/16), 2): z = 0 the c problem (fp32 states), z = 1 the h problem (bf16).
__global__ __launch_bounds__(256) void rs_fwd_kernel(
    const float* __restrict__ c_fw, const bf16* __restrict__ h_fw, size_t dstride,  // state rows [B][H]; bw at +dstride
    const bf16* __restrict__ RCt, const bf16* __restrict__ RHt,                   // [H][2H] (W^T, "Bt")
    const float* __restrict__ bc, const float* __restrict__ bh,
    float* __restrict__ pre_c, float* __restrict__ pre_h,                           // [B][H]
    float* __restrict__ c0, bf16* __restrict__ c0b, bf16* __restrict__ h0b,        // [B][H]
    bf16* __restrict__ cat_c, bf16* __restrict__ cat_h,                             // [B][2H] (nullable)
    int B, int H) {
  __shared__ float red[4 * 256];
  if (blockIdx.z == 0) rs_fwd_body<float>(c_fw, dstride, RCt, bc, pre_c, c0, c0b, cat_c, B, H, red);
  else rs_fwd_body<bf16>(h_fw, dstride, RHt, bh, pre_h, nullptr, h0b, cat_h, B, H, red);
}

// grid (ceil(B/16), 2): one workgroup per (16-row tile, problem); wave w computes column
// tiles w, w + 4, ... of d_old = dp . W^T (K = H), dp built on the fly from g and pre.
// grid (row tiles of 16, 2 problems, H / 32 column groups): each workgroup recomputes its 16 dp
// rows (16 x H, cheap) and its 4 waves each own one 16-column tile of d_old (2H / 16 tiles over
// the H / 32 groups), the W rows' fragments loaded up front -- 256 workgroups at B = 256 instead
// of 32 with 8 dependent tiles per wave (85 -> see profiles/r6/rs_bwd.md).  Group 0 alone writes
// the bf16 dp rows and the bias-gradient atomics.
__global__ __launch_bounds__(256) void rs_bwd_kernel(
    const float* __restrict__ gc, const float* __restrict__ gh,        // dL/dc0, dL/dh0 [B][H]
    const float* __restrict__ pre_c, const float* __restrict__ pre_h,  // [B][H]
    const bf16* __restrict__ RC, const bf16* __restrict__ RH,          // [2H][H] (TF layout = "Bt" for d_old)
    bf16* __restrict__ dpc, bf16* __restrict__ dph,                    // [B][H] bf16 dp (wgrad operands)
    float* __restrict__ gbc, float* __restrict__ gbh,                  // [H] bias gradients (+=)
    float* __restrict__ dold_c, float* __restrict__ dold_h, size_t dstride,  // fw rows [B][H]; bw at +dstride
    int B, int H) {
  __shared__ __attribute__((aligned(16))) bf16 Ds[16][512 + 8];  // dp rows of the tile (H <= 512)
  const int prob = blockIdx.y, grp = blockIdx.z;
  const float* g = prob ? gh : gc;
  const float* pre = prob ? pre_h : pre_c;
  const bf16* R = prob ? RH : RC;
  bf16* dpo = prob ? dph : dpc;
  float* gb = prob ? gbh : gbc;
  float* dold = prob ? dold_h : dold_c;
  const int r0 = blockIdx.x * 16;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // this wave's d_old column tile and its W rows' fragments, loaded before the dp pass
  const int kof = 8 * (lane >> 4), j0 = (4 * grp + wid) * 16;
  const bf16* brow = R + (size_t)(j0 + (lane & 15)) * H + kof;
  bf16x8 bw[16];
#pragma unroll
  for (int kk = 0; kk < 16; ++kk)
    if (32 * kk < H) bw[kk] = ld8(brow + 32 * kk);
  // dp tile -> LDS (and, group 0, the bf16 dp rows and the bias-gradient column partials)
  for (int col = threadIdx.x; col < H; col += 256) {
    float cs = 0.f;
    for (int rr = 0; rr < 16; ++rr) {
      const int r = r0 + rr;
      float v = 0.f;
      if (r < B) {
        const size_t ix = (size_t)r * H + col;
        v = pre[ix] > 0.f ? g[ix] : 0.f;
        if (grp == 0) dpo[ix] = f2bf(v);
      }
      cs += v;
      Ds[rr][col] = f2bf(v);
    }
    if (gb && grp == 0) atomicAdd(gb + col, cs);
  }
  __syncthreads();
  // d_old[r][j] = sum_u dp[r][u] R[j][u], j < 2H: MFMA A = dp rows (LDS), B = R rows
  f32x4 acc = f32x4{0, 0, 0, 0};
#pragma unroll
  for (int kk = 0; kk < 16; ++kk)
    if (32 * kk < H) acc = mfma16(*reinterpret_cast<const bf16x8*>(&Ds[lane & 15][32 * kk + kof]), bw[kk], acc);
  const int j = j0 + (lane & 15), d = j >= H;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + (lane >> 4) * 4 + i;
    if (r < B) dold[d * dstride + (size_t)r * H + (j - d * H)] = acc[i];
  }
}

void launch_rs_fwd(const float* c_fw, const bf16* h_fw, size_t dstride, const bf16* RCt, const bf16* RHt,
                   const float* bc, const float* bh, float* pre_c, float* pre_h, float* c0, bf16* c0b, bf16* h0b,
                   bf16* cat_c, bf16* cat_h, int B, int H, hipStream_t st) {
  hipLaunchKernelGGL(rs_fwd_kernel, dim3(H / 16, (B + 15) / 16, 2), dim3(256), 0, st, c_fw, h_fw, dstride, RCt, RHt,
                     bc, bh, pre_c, pre_h, c0, c0b, h0b, cat_c, cat_h, B, H);
}

void launch_rs_bwd(const float* gc, const float* gh, const float* pre_c, const float* pre_h, const bf16* RC,
                   const bf16* RH, bf16* dpc, bf16* dph, float* gbc, float* gbh, float* dold_c, float* dold_h,
                   size_t dstride, int B, int H, hipStream_t st) {
  hipLaunchKernelGGL(rs_bwd_kernel, dim3((B + 15) / 16, 2, H / 32), dim3(256), 0, st, gc, gh, pre_c, pre_h, RC, RH, dpc,
                     dph, gbc, gbh, dold_c, dold_h, dstride, B, H);
}
