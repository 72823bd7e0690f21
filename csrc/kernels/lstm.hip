// Bidirectional LSTM encoder recurrence (reference model.py:76-94, TF LSTMCell).
//
// One launch per time step runs BOTH directions (fw on blockIdx.z==0, bw on 1); the
// launches are captured into one hipGraph by the caller, so the per-step cost is the
// dependent-kernel boundary (~1.5 us, MI355X_MICROARCH "boundary") plus one small MFMA
// GEMM: h_{s-1}[B,H] x W_hh[H,4H].  The input projection x.W_x + b for all T steps is
// hoisted out of the recurrence into one big GEMM (gx), as is every weight gradient.
//
// Layout ("step frame"): the bw direction consumes x reversed within each sequence
// length (TF ReverseSequence), so step s of direction d reads gx[d][s] for every row,
// and writes its output h to enc_out[r][t][d*H+u] with t = s (fw) or len_r-1-s (bw).
// Rows with s >= len_r are frozen: state copied through, output left zero (dynamic_rnn
// with sequence_length), so the final state of both directions sits at step index T.
//
// Gate order i, j, f, o (TF LSTMCell), forget_bias = 1.0 added at runtime.
#include "common.h"

// Each wave owns a 16-row x 16-unit tile and computes the 4 gate tiles of those units,
// so the whole cell update stays in registers.  Block = 4 waves = 64 units.
__global__ __launch_bounds__(256) void lstm_enc_fwd_step_kernel(
    const float* __restrict__ gx,     // [2][T][B][4H]  x.W_x + b (step frame)
    const bf16* __restrict__ Wt,      // [2][4H][H]     W_hh^T
    bf16* __restrict__ hs,            // [2][T+1][B][H] h entering step s (bf16)
    float* __restrict__ cs,           // [2][T+1][B][H] c entering step s
    float* __restrict__ acts,         // [2][T][B][4H]  sig(i) tanh(j) sig(f+1) sig(o)
    bf16* __restrict__ out,           // [B][T][2H]
    const int* __restrict__ lens, int s, int T, int B, int H) {
  const int d = blockIdx.z;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int u0 = (blockIdx.x * 4 + wid) * 16;
  const int r0 = blockIdx.y * 16;
  if (u0 >= H) return;
  const size_t BH = (size_t)B * H, G = 4 * (size_t)H;
  const int ar = min(r0 + (lane & 15), B - 1);
  const int kof = 8 * (lane >> 4);
  const bf16* hprev = hs + ((size_t)d * (T + 1) + s) * BH;
  const bf16* arow = hprev + (size_t)ar * H + kof;
  const bf16* W = Wt + (size_t)d * G * H;
  f32x4 acc[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) acc[g] = f32x4{0, 0, 0, 0};
  for (int k = 0; k < H; k += 32) {
    bf16x8 a = ld8(arow + k);
#pragma unroll
    for (int g = 0; g < 4; ++g)
      acc[g] = mfma16(a, ld8(W + ((size_t)g * H + u0 + (lane & 15)) * H + kof + k), acc[g]);
  }
  const int u = u0 + (lane & 15);
  const float* gxs = gx + ((size_t)d * T + s) * B * G;
  const float* cprev = cs + ((size_t)d * (T + 1) + s) * BH;
  float* cnext = cs + ((size_t)d * (T + 1) + s + 1) * BH;
  bf16* hnext = hs + ((size_t)d * (T + 1) + s + 1) * BH;
  float* act = acts + ((size_t)d * T + s) * B * G;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = r0 + (lane >> 4) * 4 + j;
    if (r >= B) continue;
    const int len = lens[r];
    const size_t ri = (size_t)r * H + u;
    if (s < len) {
      const float* gr = gxs + (size_t)r * G;
      float zi = acc[0][j] + gr[u], zj = acc[1][j] + gr[H + u];
      float zf = acc[2][j] + gr[2 * H + u], zo = acc[3][j] + gr[3 * H + u];
      float ig = fsigmoid(zi), jg = ftanh(zj), fg = fsigmoid(zf + 1.0f), og = fsigmoid(zo);
      float c = fg * cprev[ri] + ig * jg;
      float h = og * ftanh(c);
      cnext[ri] = c;
      hnext[ri] = f2bf(h);
      float* ar4 = act + (size_t)r * G;
      ar4[u] = ig; ar4[H + u] = jg; ar4[2 * H + u] = fg; ar4[3 * H + u] = og;
      const int t = d == 0 ? s : len - 1 - s;
      out[((size_t)r * T + t) * 2 * H + d * H + u] = f2bf(h);
    } else {
      cnext[ri] = cprev[ri];
      hnext[ri] = hprev[ri];
    }
  }
}

// BPTT step s (launched for s = T-1 ... 0).  dh entering the cell at step s is
//   dz_{s+1} . W_hh^T  (recurrent, all gate columns of step s+1)  + dOut[r][t]
//   + dh_fin for the last active step (s+1 == len_r; frozen steps pass it through).
// dc is carried per unit in dc_carry (initialised to dc_fin by the caller).
// dz is written in bf16 for the step-frame weight-gradient GEMMs done after the loop;
// inactive rows write zeros so the next step's GEMM sees no contribution.
__global__ __launch_bounds__(256) void lstm_enc_bwd_step_kernel(
    bf16* __restrict__ dz,            // [2][T][B][4H]
    const bf16* __restrict__ Wn,      // [2][H][4H]  W_hh (rows = input unit)
    const float* __restrict__ dout,   // [B][T][2H]
    const float* __restrict__ dh_fin, // [2][B][H]
    float* __restrict__ dc_carry,     // [2][B][H]
    const float* __restrict__ acts, const float* __restrict__ cs,
    const int* __restrict__ lens, int s, int T, int B, int H) {
  const int d = blockIdx.z;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int u0 = (blockIdx.x * 4 + wid) * 16;
  const int r0 = blockIdx.y * 16;
  if (u0 >= H) return;
  const size_t BH = (size_t)B * H, G = 4 * (size_t)H;
  f32x4 acc = {0, 0, 0, 0};
  if (s + 1 < T) {
    const int ar = min(r0 + (lane & 15), B - 1);
    const int kof = 8 * (lane >> 4);
    const bf16* arow = dz + (((size_t)d * T + s + 1) * B + ar) * G + kof;
    const bf16* brow = Wn + ((size_t)d * H + u0 + (lane & 15)) * G + kof;
    acc = mfma_k(arow, brow, (int)G, acc);
  }
  const int u = u0 + (lane & 15);
  const float* act = acts + ((size_t)d * T + s) * B * G;
  const float* cprev = cs + ((size_t)d * (T + 1) + s) * BH;
  const float* cnow = cs + ((size_t)d * (T + 1) + s + 1) * BH;
  bf16* dzs = dz + ((size_t)d * T + s) * B * G;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = r0 + (lane >> 4) * 4 + j;
    if (r >= B) continue;
    const int len = lens[r];
    const size_t ri = (size_t)r * H + u;
    bf16* dzr = dzs + (size_t)r * G;
    if (s < len) {
      const int t = d == 0 ? s : len - 1 - s;
      float dh = acc[j] + dout[((size_t)r * T + t) * 2 * H + d * H + u];
      if (s + 1 >= len) dh += dh_fin[(size_t)d * BH + ri];
      const float* a4 = act + (size_t)r * G;
      const float ig = a4[u], jg = a4[H + u], fg = a4[2 * H + u], og = a4[3 * H + u];
      const float c = cnow[ri];
      const float tc = ftanh(c);
      float dc = dc_carry[(size_t)d * BH + ri] + dh * og * (1.0f - tc * tc);
      const float dzo = dh * tc * og * (1.0f - og);
      const float dzi = dc * jg * ig * (1.0f - ig);
      const float dzj = dc * ig * (1.0f - jg * jg);
      const float dzf = dc * cprev[ri] * fg * (1.0f - fg);
      dc_carry[(size_t)d * BH + ri] = dc * fg;
      dzr[u] = f2bf(dzi); dzr[H + u] = f2bf(dzj); dzr[2 * H + u] = f2bf(dzf); dzr[3 * H + u] = f2bf(dzo);
    } else {
      const bf16 z = f2bf(0.f);
      dzr[u] = z; dzr[H + u] = z; dzr[2 * H + u] = z; dzr[3 * H + u] = z;
    }
  }
}

void launch_lstm_enc_fwd_step(const float* gx, const bf16* Wt, bf16* hs, float* cs, float* acts, bf16* out,
                              const int* lens, int s, int T, int B, int H, hipStream_t st) {
  dim3 grid((H + 63) / 64, (B + 15) / 16, 2);
  hipLaunchKernelGGL(lstm_enc_fwd_step_kernel, grid, dim3(256), 0, st, gx, Wt, hs, cs, acts, out, lens, s, T, B, H);
}

void launch_lstm_enc_bwd_step(bf16* dz, const bf16* Wn, const float* dout, const float* dh_fin, float* dc_carry,
                              const float* acts, const float* cs, const int* lens, int s, int T, int B, int H,
                              hipStream_t st) {
  dim3 grid((H + 63) / 64, (B + 15) / 16, 2);
  hipLaunchKernelGGL(lstm_enc_bwd_step_kernel, grid, dim3(256), 0, st, dz, Wn, dout, dh_fin, dc_carry, acts, cs,
                     lens, s, T, B, H);
}
