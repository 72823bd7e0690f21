// Layout kernels of the encoder: batch frame [B][T][*] <-> step frame [2][T][B][*] (the bw
// direction reversed within each sequence length), and the W_h feature transpose.
//
// The reference runs tf.nn.bidirectional_dynamic_rnn (model.py:89-93), whose bw pass is
// ReverseSequence -> LSTM -> ReverseSequence.  Here both directions run in one persistent
// kernel over step-frame inputs, so the frames are rebuilt around it; each of these replaces
// a chain of torch gather / transpose / copy / scatter_add launches (one 16-byte chunk per
// thread, ~2x the bytes moved, no temporaries).
#include "common.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// out[d][t][b][0:W] = src[row(b, tt)][off_d + 0:W], tt = t (d = 0) or rev[b][t] (d = 1),
// row(b, tt) = ids ? ids[b*T + tt] : b*T + tt; off_d = d * doff.  ES = element bytes.
template <int ES>
__global__ __launch_bounds__(256) void to_step_frame_kernel(const char* __restrict__ src, const int64_t* __restrict__ ids,
                                                            const int64_t* __restrict__ rev, char* __restrict__ out,
                                                            int B, int T, int W, int S, int doff, long nsrc) {
  const int cpr = W * ES / 16;  // 16-byte chunks per row
  const long n = 2L * T * B * cpr;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % cpr);
    const long rowo = i / cpr;  // (d, t, b)
    const int b = (int)(rowo % B);
    const int t = (int)((rowo / B) % T);
    const int d = (int)(rowo / ((long)B * T));
    const int tt = d == 0 ? t : (int)DCHECK_IDX(rev[(size_t)b * T + t], 0, T, CHK_FRAME_REV);
    const long srow = ids ? DCHECK_IDX(ids[(size_t)b * T + tt], 0, nsrc, CHK_FRAME_ID) : (long)b * T + tt;
    const u32x4 v = *reinterpret_cast<const u32x4*>(src + ((size_t)srow * S + (size_t)d * doff) * ES + (size_t)c * 16);
    *reinterpret_cast<u32x4*>(out + (size_t)rowo * W * ES + (size_t)c * 16) = v;
  }
}

// fp32: out[b][t][0:W] = in[0][t][b][:] + in[1][rev[b][t]][b][:]   (rev is an involution)
__global__ __launch_bounds__(256) void from_step_frame_kernel(const float* __restrict__ in, const int64_t* __restrict__ rev,
                                                              float* __restrict__ out, int B, int T, int W) {
  const int cpr = W / 4;
  const long n = (long)B * T * cpr;
  const size_t plane = (size_t)T * B * W;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % cpr);
    const long bt = i / cpr;
    const int t = (int)(bt % T), b = (int)(bt / T);
    const int rt = (int)DCHECK_IDX(rev[(size_t)b * T + t], 0, T, CHK_FRAME_REV);
    const float4 x = *reinterpret_cast<const float4*>(in + ((size_t)t * B + b) * W + 4 * c);
    const float4 y = *reinterpret_cast<const float4*>(in + plane + ((size_t)rt * B + b) * W + 4 * c);
    *reinterpret_cast<float4*>(out + (size_t)bt * W + 4 * c) = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
  }
}

// Between two stacked encoder layers in the BPTT: the upper layer's input gradients (step frame,
// in[dir][t][b][2H]) straight into the lower layer's output-gradient step frame out[d][t][b][H] --
// from_step_frame then to_step_frame (doff = H) in one pass, without the batch-frame dx between
// them (2 x T x B x 2H fp32 of traffic less per layer boundary; the same two fp32 operands added):
//   out[0][t][b] = in[0][t][b][0:H]    + in[1][rev(b,t)][b][0:H]
//   out[1][t][b] = in[0][rev(b,t)][b][H:2H] + in[1][t][b][H:2H]        (rev is an involution)
__global__ __launch_bounds__(256) void step_frame_hop_kernel(const float* __restrict__ in, const int64_t* __restrict__ rev,
                                                             float* __restrict__ out, int B, int T, int H) {
  const int cpr = H / 4;
  const long n = 2L * T * B * cpr;
  const size_t plane = (size_t)T * B * 2 * H;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % cpr);
    const long row = i / cpr;  // (d, t, b)
    const int b = (int)(row % B);
    const int t = (int)((row / B) % T);
    const int d = (int)(row / ((long)B * T));
    const int rt = (int)DCHECK_IDX(rev[(size_t)b * T + t], 0, T, CHK_FRAME_REV);
    const int t0 = d == 0 ? t : rt, t1 = d == 0 ? rt : t;
    const size_t col = (size_t)d * H + 4 * c;
    const float4 x = *reinterpret_cast<const float4*>(in + ((size_t)t0 * B + b) * 2 * H + col);
    const float4 y = *reinterpret_cast<const float4*>(in + plane + ((size_t)t1 * B + b) * 2 * H + col);
    *reinterpret_cast<float4*>(out + (size_t)row * H + 4 * c) = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
  }
}

// fp32 [P][Q][R] -> [Q][P][R] (out, nullable; acc: added to it) and its bf16 twin (outb, nullable)
// in one pass: the step-major ctx of all decoder steps from the batched a . enc_out GEMM
// ([B][D][A]), and the attention-weight gradient's dctx . E_i part added into dA ([B][D][T]),
// which took strided torch copies / adds plus a bf16 cast before
__global__ __launch_bounds__(256) void tr01_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                   bf16* __restrict__ outb, int P, int Q, int R4, bool acc) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;  // float4 index in the OUTPUT [Q][P][R4]
  if (i >= (size_t)P * Q * R4) return;
  const int r = (int)(i % R4);
  const size_t qp = i / R4;
  const int pp = (int)(qp % P), q = (int)(qp / P);
  const f32x4 x = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in) + ((size_t)pp * Q + q) * R4 + r);
  if (out) {
    f32x4 y = x;
    if (acc) y += reinterpret_cast<const f32x4*>(out)[i];
    reinterpret_cast<f32x4*>(out)[i] = y;
  }
  if (outb) {
    bf16 o[4] = {f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
    *reinterpret_cast<uint2*>(outb + 4 * i) = *reinterpret_cast<const uint2*>(o);
  }
}

// bf16 [B][T][A] -> [B][A][T] through a 64 x 64 LDS tile (8-byte loads and stores)
__global__ __launch_bounds__(256) void transpose_bta_kernel(const bf16* __restrict__ in, bf16* __restrict__ out, int T,
                                                            int A) {
  __shared__ bf16 tile[64][64 + 4];
  const int b = blockIdx.z, t0 = blockIdx.y * 64, a0 = blockIdx.x * 64;
  const int tid = threadIdx.x, q = (tid & 15) * 4;
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  for (int r = tid >> 4; r < 64; r += 16) {
    const int t = t0 + r;
    bf16x4 v = bf16x4{(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
    if (t < T) v = *reinterpret_cast<const bf16x4*>(in + ((size_t)b * T + t) * A + a0 + q);
#pragma unroll
    for (int j = 0; j < 4; ++j) tile[r][q + j] = v[j];
  }
  __syncthreads();
  for (int r = tid >> 4; r < 64; r += 16) {  // r: feature within the tile, q: 4 positions
    const int t = t0 + q;
    bf16x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = tile[q + j][r];
    bf16* dst = out + ((size_t)b * A + a0 + r) * T + t;
    if (t + 4 <= T && (T & 3) == 0) {
      *reinterpret_cast<bf16x4*>(dst) = v;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (t + j < T) dst[j] = v[j];
    }
  }
}

static int grid_for(long n) {
  const long g = (n + 255) / 256;
  return (int)(g < 8192 ? g : 8192);
}

void launch_to_step_frame(const void* src, int es, const int64_t* ids, const int64_t* rev, void* out, int B, int T,
                          int W, int S, int doff, long nsrc, hipStream_t st) {
  const long n = 2L * T * B * (W * es / 16);
  if (es == 2)
    hipLaunchKernelGGL(to_step_frame_kernel<2>, dim3(grid_for(n)), dim3(256), 0, st, (const char*)src, ids, rev,
                       (char*)out, B, T, W, S, doff, nsrc);
  else
    hipLaunchKernelGGL(to_step_frame_kernel<4>, dim3(grid_for(n)), dim3(256), 0, st, (const char*)src, ids, rev,
                       (char*)out, B, T, W, S, doff, nsrc);
}

void launch_from_step_frame(const float* in, const int64_t* rev, float* out, int B, int T, int W, hipStream_t st) {
  const long n = (long)B * T * (W / 4);
  hipLaunchKernelGGL(from_step_frame_kernel, dim3(grid_for(n)), dim3(256), 0, st, in, rev, out, B, T, W);
}

void launch_step_frame_hop(const float* in, const int64_t* rev, float* out, int B, int T, int H, hipStream_t st) {
  const long n = 2L * T * B * (H / 4);
  hipLaunchKernelGGL(step_frame_hop_kernel, dim3(grid_for(n)), dim3(256), 0, st, in, rev, out, B, T, H);
}

void launch_transpose_bta(const bf16* in, bf16* out, int B, int T, int A, hipStream_t st) {
  hipLaunchKernelGGL(transpose_bta_kernel, dim3(A / 64, (T + 63) / 64, B), dim3(256), 0, st, in, out, T, A);
}

// xb = bf16(x) and colsum[c] += sum_n x[n][c] in one read of x [N][C] fp32 (C % 4 == 0,
// C / 4 divides 256).  Replaces a cast plus a torch column reduction (a tall [N, C] sum(0)
// runs at ~0.6 TB/s).  Each thread owns 4 columns of every (256 / (C/4))-th row; the block's
// row groups meet in LDS and the block writes its partial row part[blockIdx][C]; a second
// one-block-per-256-columns kernel adds the G partials into colsum.  (Atomics straight into
// colsum serialise at L2 on the same C addresses: ~107 us at 1024 blocks, ~38 us at 128.)
__global__ __launch_bounds__(256) void cast_colsum_kernel(const float* __restrict__ x, bf16* __restrict__ xb,
                                                          float* __restrict__ part, int N, int C) {
  __shared__ float4 ps[256];
  const int C4 = C / 4, rpb = 256 / C4;  // rows per block pass
  const int cu = threadIdx.x % C4, rg = threadIdx.x / C4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (long r = (long)blockIdx.x * rpb + rg; r < N; r += (long)gridDim.x * rpb) {
    const float4 v = *reinterpret_cast<const float4*>(x + r * C + 4 * cu);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    bf16 o[4] = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
    *reinterpret_cast<uint2*>(xb + r * C + 4 * cu) = *reinterpret_cast<const uint2*>(o);
  }
  ps[threadIdx.x] = s;
  __syncthreads();
  if (rg == 0) {
    for (int g = 1; g < rpb; ++g) {
      const float4 p = ps[g * C4 + cu];
      s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
    }
    *reinterpret_cast<float4*>(part + (size_t)blockIdx.x * C + 4 * cu) = s;
  }
}

// colsum[c] += sum_g part[g][c]: 16 columns x 16 partial-row lanes per block, every lane's
// G/16 loads independent (one round trip), then an LDS reduce over the 16 lanes
__global__ __launch_bounds__(256) void colsum_finish_kernel(const float* __restrict__ part, float* __restrict__ colsum,
                                                            int G, int C) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, gl = threadIdx.x >> 4, c = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (c < C) {
#pragma unroll 16
    for (int g = gl; g < G; g += 16) s += part[(size_t)g * C + c];
  }
  red[gl][cl] = s;
  __syncthreads();
  if (gl == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][cl];
    colsum[c] += t;
  }
}

int cast_colsum_blocks(int N, int C) {
  const int rpb = 256 / (C / 4);
  const int g = (N + rpb - 1) / rpb;
  return g < 256 ? (g > 0 ? g : 1) : 256;
}

void launch_cast_colsum(const float* x, bf16* xb, float* part, float* colsum, int N, int C, hipStream_t st) {
  const int G = cast_colsum_blocks(N, C);
  hipLaunchKernelGGL(cast_colsum_kernel, dim3(G), dim3(256), 0, st, x, xb, part, N, C);
  hipLaunchKernelGGL(colsum_finish_kernel, dim3((C + 15) / 16), dim3(256), 0, st, part, colsum, G, C);
}

// Deterministic column sums out[c] (=, or += with acc) of a tall x [N][C] (fp32 or bf16):
// the tall reductions of the backward (bias gradients: sum over tokens / decoder rows).
// A torch sum(0) over ~10^5 rows splits each column over several workgroups and merges their
// partials through a semaphore; on this device its results were not reproducible run to run
// (profiles/r4/det_streams.md: the encoder LSTM bias gradient differed between two identical
// deterministic-mode trainings while every weight gradient matched).  Here the order is fixed
// by (N, C) alone: grid (column tiles of 256, G row chunks); wave w of a block sums rows
// r0 + w, r0 + w + 4, ... of its chunk for 4 columns per lane, the 4 waves meet in LDS in wave
// order, part[g][c] is stored, and colsum_det_finish adds the G partials in a fixed order.
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void colsum_det_part_kernel(const T* __restrict__ x, float* __restrict__ part,
                                                              int N, int C, int rpc) {
  __shared__ float4 ps[4][64];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c0 = blockIdx.x * 256 + lane * 4;
  const int r0 = blockIdx.y * rpc, r1 = min(N, r0 + rpc);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (c0 < C) {
    for (int r = r0 + wid; r < r1; r += 4) {
      const T* p = x + (size_t)r * C + c0;
      if constexpr (VEC) {  // C % 4 == 0: the lane's 4 columns in one load
        if constexpr (sizeof(T) == 4) {
          const float4 v = *reinterpret_cast<const float4*>(p);
          s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
        } else {
          const uint2 v = *reinterpret_cast<const uint2*>(p);
          s[0] += __uint_as_float(v.x << 16); s[1] += __uint_as_float(v.x & 0xffff0000u);
          s[2] += __uint_as_float(v.y << 16); s[3] += __uint_as_float(v.y & 0xffff0000u);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (c0 + j < C) s[j] += (float)p[j];
      }
    }
  }
  ps[wid][lane] = make_float4(s[0], s[1], s[2], s[3]);
  __syncthreads();
  if (wid == 0 && c0 < C) {
    float4 t = ps[0][lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 q = ps[w][lane];
      t.x += q.x; t.y += q.y; t.z += q.z; t.w += q.w;
    }
    const float tv[4] = {t.x, t.y, t.z, t.w};
    float* dst = part + (size_t)blockIdx.y * C + c0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (c0 + j < C) dst[j] = tv[j];
  }
}

// out[c] (= or += acc) of the G partial rows: CPB columns x (256 / CPB) partial-row lanes per
// block, every lane's loads independent (one round trip), then the lanes of a column summed in
// lane order through LDS -- a fixed order for a given (G, C)
template <int CPB>
__global__ __launch_bounds__(256) void colsum_det_finish_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                                int G, int C, int acc) {
  constexpr int GL = 256 / CPB;
  __shared__ float red[GL][CPB + 1];
  const int cl = threadIdx.x % CPB, gl = threadIdx.x / CPB, c = blockIdx.x * CPB + cl;
  float s = 0.f;
  if (c < C) {
#pragma unroll 8
    for (int g = gl; g < G; g += GL) s += part[(size_t)g * C + c];
  }
  red[gl][cl] = s;
  __syncthreads();
  if (gl == 0 && c < C) {
    float t = 0.f;
    for (int i = 0; i < GL; ++i) t += red[i][cl];
    out[c] = acc ? out[c] + t : t;
  }
}

// row chunks: about 2048 workgroups over the column tiles, at least 64 rows per chunk
int colsum_det_chunks(int N, int C) {
  const int nct = (C + 255) / 256;
  int G = (2048 + nct - 1) / nct;
  G = min(G, max(1, N / 64));
  return max(1, G);
}

void launch_colsum_det(const void* x, bool bf, float* part, float* out, int N, int C, bool acc, hipStream_t st) {
  if (N <= 0 || C <= 0) return;
  const int G = colsum_det_chunks(N, C), rpc = (N + G - 1) / G;
  const dim3 grid((C + 255) / 256, G);
  const bool vec = C % 4 == 0;
  if (bf) {
    if (vec) hipLaunchKernelGGL((colsum_det_part_kernel<bf16, true>), grid, dim3(256), 0, st, (const bf16*)x, part, N, C, rpc);
    else hipLaunchKernelGGL((colsum_det_part_kernel<bf16, false>), grid, dim3(256), 0, st, (const bf16*)x, part, N, C, rpc);
  } else {
    if (vec) hipLaunchKernelGGL((colsum_det_part_kernel<float, true>), grid, dim3(256), 0, st, (const float*)x, part, N, C, rpc);
    else hipLaunchKernelGGL((colsum_det_part_kernel<float, false>), grid, dim3(256), 0, st, (const float*)x, part, N, C, rpc);
  }
  if (C >= 64)
    hipLaunchKernelGGL(colsum_det_finish_kernel<16>, dim3((C + 15) / 16), dim3(256), 0, st, part, out, G, C, acc ? 1 : 0);
  else
    hipLaunchKernelGGL(colsum_det_finish_kernel<1>, dim3(C), dim3(256), 0, st, part, out, G, C, acc ? 1 : 0);
}

void launch_tr01(const float* in, float* out, bf16* outb, int P, int Q, int R, bool acc, hipStream_t st) {
  const size_t n = (size_t)P * Q * (R / 4);
  if (n == 0) return;
  hipLaunchKernelGGL(tr01_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, out, outb, P, Q, R / 4,
                     acc);
}
