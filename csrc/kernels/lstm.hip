// Bidirectional LSTM encoder recurrence (reference model.py:76-94, TF LSTMCell).
//
// One launch per time step runs BOTH directions (blockIdx.z = direction); the launches
// are captured into one hipGraph by the caller, so a step costs the dependent-kernel
// boundary (~1.5 us, MI355X_MICROARCH "boundary") plus one L2 round trip: each block
// owns a 16-row x 16-unit tile of all four gates, its 4 waves split the K = H reduction
// (all fragment loads issued up front, kslice_mma), and the partial tiles are summed in
// LDS.  The input projection x.W_x + b for all T steps is hoisted out of the recurrence
// into one big GEMM (gx), as is every weight gradient.
//
// Layout ("step frame"): the bw direction consumes x reversed within each sequence
// length (TF ReverseSequence), so step s of direction d reads gx[d][s] for every row,
// and writes its output h to enc_out[r][t][d*H+u] with t = s (fw) or len_r-1-s (bw).
// Rows with s >= len_r are frozen: state copied through, output left zero (dynamic_rnn
// with sequence_length), so the final state of both directions sits at step index T.
//
// Gate order i, j, f, o (TF LSTMCell), forget_bias = 1.0 added at runtime.
#include "common.h"

__global__ __launch_bounds__(256) void lstm_enc_fwd_step_kernel(
    const float* __restrict__ gx,     // [2][T][B][H][4]  x.W_x, gate-interleaved (step frame, bias-free GEMM)
    const float* __restrict__ bias,   // [2][4H]        gate biases b
    const bf16* __restrict__ Wt,      // [2][4H][H]     W_hh^T
    bf16* __restrict__ hs,            // [2][T+1][B][H] h entering step s (bf16)
    float* __restrict__ cs,           // [2][T+1][B][H] c entering step s
    float* __restrict__ acts,         // [2][T][B][H][4]  (sig(i), tanh(j), sig(f+1), sig(o)) per unit
    bf16* __restrict__ out,           // [B][T][2H]
    const int* __restrict__ lens, int s, int T, int B, int H) {
  __shared__ float red[4 * 4 * 256];
  const int d = blockIdx.z;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int u0 = blockIdx.x * 16, r0 = blockIdx.y * 16;
  const size_t BH = (size_t)B * H, G = 4 * (size_t)H;
  // ---- prefetch this lane's epilogue operands (independent of the GEMM)
  const int r = r0 + (lane >> 4) * 4 + wid, u = u0 + (lane & 15);
  const bool rok = r < B;
  const int len = rok ? lens[r] : 0;
  const bool active = s < len;
  const float4 gq = *reinterpret_cast<const float4*>(gx + ((((size_t)d * T + s) * B + (rok ? r : 0)) * H + u) * 4);
  const float gxv[4] = {gq.x, gq.y, gq.z, gq.w};
  const bf16* hprev = hs + ((size_t)d * (T + 1) + s) * BH;
  const float* cprev = cs + ((size_t)d * (T + 1) + s) * BH;
  const size_t ri = (size_t)(rok ? r : 0) * H + u;
  float gz[4], cp;  // unconditional: no lens -> address dependence on the critical path
#pragma unroll
  for (int g = 0; g < 4; ++g) gz[g] = gxv[g] + bias[(size_t)d * G + g * H + u];
  cp = cprev[ri];
  // ---- h_{s-1} . W_hh, K split over the 4 waves
  const int ar = min(r0 + (lane & 15), B - 1);
  const int kof = 8 * (lane >> 4);
  const bf16* arow = hprev + (size_t)ar * H + kof;
  const bf16* W = Wt + (size_t)d * G * H + (size_t)(u0 + (lane & 15)) * H + kof;
  const int nst = H / 32;
  const int k0 = (wid * nst / 4) * 32, k1 = ((wid + 1) * nst / 4) * 32;
  f32x4 acc[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) acc[g] = f32x4{0, 0, 0, 0};
  kslice_mma<4>([&](int k) { return ld8(arow + k); }, [&](int g, int k) { return ld8(W + (size_t)g * H * H + k); },
                k0, k1, acc);
  float z[4];
  ksplit_reduce<4>(acc, red, z);
  if (!rok) return;
  float* cnext = cs + ((size_t)d * (T + 1) + s + 1) * BH;
  bf16* hnext = hs + ((size_t)d * (T + 1) + s + 1) * BH;
  if (active) {
    const float ig = fsigmoid(z[0] + gz[0]), jg = ftanh(z[1] + gz[1]);
    const float fg = fsigmoid(z[2] + gz[2] + 1.0f), og = fsigmoid(z[3] + gz[3]);
    const float c = fg * cp + ig * jg;
    const float h = og * ftanh(c);
    cnext[ri] = c;
    hnext[ri] = f2bf(h);
    *reinterpret_cast<float4*>(acts + ((((size_t)d * T + s) * B + r) * H + u) * 4) = make_float4(ig, jg, fg, og);
    const int t = d == 0 ? s : len - 1 - s;
    out[((size_t)r * T + t) * 2 * H + d * H + u] = f2bf(h);
  } else {
    cnext[ri] = cp;
    hnext[ri] = hprev[ri];
  }
}

// BPTT step s (launched for s = T-1 ... 0).  dh entering the cell at step s is
//   dz_{s+1} . W_hh^T  (recurrent, all gate columns of step s+1)  + dOut (step frame)
//   + dh_fin for the last active step (s+1 == len_r; frozen steps pass it through).
// dc is carried per unit in dc_carry (initialised to dc_fin by the caller).
// dz is written in bf16 for the step-frame weight-gradient GEMMs done after the loop;
// inactive rows write zeros so the next step's GEMM sees no contribution.
__global__ __launch_bounds__(256) void lstm_enc_bwd_step_kernel(
    bf16* __restrict__ dz,            // [2][T][B][4H]
    const bf16* __restrict__ Wn,      // [2][H][4H]  W_hh (rows = input unit)
    const float* __restrict__ dout,   // [2][T][B][H]  dL/dh_out in step frame
    const float* __restrict__ dh_fin, // [2][B][H]
    float* __restrict__ dc_carry,     // [2][B][H]
    const float* __restrict__ acts, const float* __restrict__ cs,
    const int* __restrict__ lens, int s, int T, int B, int H) {
  __shared__ float red[4 * 256];
  const int d = blockIdx.z;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int u0 = blockIdx.x * 16, r0 = blockIdx.y * 16;
  const size_t BH = (size_t)B * H, G = 4 * (size_t)H;
  // ---- prefetch epilogue operands
  const int r = r0 + (lane >> 4) * 4 + wid, u = u0 + (lane & 15);
  const bool rok = r < B;
  const int len = rok ? lens[r] : 0;
  const bool active = s < len;
  const size_t ri = (size_t)(rok ? r : 0) * H + u;
  // all epilogue operands loaded unconditionally (addresses independent of len)
  float a4[4];
  const float dho = dout[((size_t)d * T + s) * BH + ri];
  const float dhf = dh_fin[(size_t)d * BH + ri];
  {
    const float4 q = *reinterpret_cast<const float4*>(acts + ((((size_t)d * T + s) * B + (rok ? r : 0)) * H + u) * 4);
    a4[0] = q.x; a4[1] = q.y; a4[2] = q.z; a4[3] = q.w;
  }
  const float cn = cs[((size_t)d * (T + 1) + s + 1) * BH + ri];
  const float cpv = cs[((size_t)d * (T + 1) + s) * BH + ri];
  const float dcin = dc_carry[(size_t)d * BH + ri];
  // ---- dz_{s+1} . W_hh^T, K = 4H split over the 4 waves
  f32x4 acc[1] = {f32x4{0, 0, 0, 0}};
  if (s + 1 < T) {
    const int ar = min(r0 + (lane & 15), B - 1);
    const int kof = 8 * (lane >> 4);
    const bf16* arow = dz + (((size_t)d * T + s + 1) * B + ar) * G + kof;
    const bf16* brow = Wn + ((size_t)d * H + u0 + (lane & 15)) * G + kof;
    const int nst = (int)(G / 32);
    const int k0 = (wid * nst / 4) * 32, k1 = ((wid + 1) * nst / 4) * 32;
    kslice_mma<1>([&](int k) { return ld8(arow + k); }, [&](int, int k) { return ld8(brow + k); }, k0, k1, acc);
  }
  float rec[1];
  ksplit_reduce<1>(acc, red, rec);
  if (!rok) return;
  bf16* dzr = dz + (((size_t)d * T + s) * B + r) * G;
  if (active) {
    const float dh = rec[0] + dho + (s + 1 >= len ? dhf : 0.f);
    const float ig = a4[0], jg = a4[1], fg = a4[2], og = a4[3];
    const float tc = ftanh(cn);
    const float dc = dcin + dh * og * (1.0f - tc * tc);
    const float dzo = dh * tc * og * (1.0f - og);
    const float dzi = dc * jg * ig * (1.0f - ig);
    const float dzj = dc * ig * (1.0f - jg * jg);
    const float dzf = dc * cpv * fg * (1.0f - fg);
    dc_carry[(size_t)d * BH + ri] = dc * fg;
    dzr[u] = f2bf(dzi); dzr[H + u] = f2bf(dzj); dzr[2 * H + u] = f2bf(dzf); dzr[3 * H + u] = f2bf(dzo);
  } else {
    const bf16 zz = f2bf(0.f);
    dzr[u] = zz; dzr[H + u] = zz; dzr[2 * H + u] = zz; dzr[3 * H + u] = zz;
  }
}

void launch_lstm_enc_fwd_step(const float* gx, const float* bias, const bf16* Wt, bf16* hs, float* cs, float* acts, bf16* out,
                              const int* lens, int s, int T, int B, int H, hipStream_t st) {
  dim3 grid(H / 16, (B + 15) / 16, 2);
  hipLaunchKernelGGL(lstm_enc_fwd_step_kernel, grid, dim3(256), 0, st, gx, bias, Wt, hs, cs, acts, out, lens, s, T, B,
                     H);
}

void launch_lstm_enc_bwd_step(bf16* dz, const bf16* Wn, const float* dout, const float* dh_fin, float* dc_carry,
                              const float* acts, const float* cs, const int* lens, int s, int T, int B, int H,
                              hipStream_t st) {
  dim3 grid(H / 16, (B + 15) / 16, 2);
  hipLaunchKernelGGL(lstm_enc_bwd_step_kernel, grid, dim3(256), 0, st, dz, Wn, dout, dh_fin, dc_carry, acts, cs,
                     lens, s, T, B, H);
}
