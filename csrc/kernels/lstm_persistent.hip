// Persistent, weight-resident bidirectional LSTM recurrence (hard part 7.5-1;
// reference model.py:76-94 / TF LSTMCell semantics exactly as lstm.hip).
//
// Why: the per-step kernels of lstm.hip pay a dependent-kernel boundary (~1.5 us) plus an
// L2 round trip for W_hh every step, 2 x T = 800 times per training step.  Here ONE launch
// runs all T steps.  Work split:
//   * a TEAM = NC = H/64 workgroups owns one (direction, 16-row batch tile);
//   * workgroup c of a team owns hidden units [64c, 64c+64); its wave w owns 16 units and
//     computes all four gates for them, so the cell update needs no cross-wave reduction;
//   * W_hh for those gate columns lives in REGISTERS for the whole launch (H/2 VGPRs per
//     lane: 128 at H = 256) -- the B operand of every MFMA is already in place;
//   * the only per-step traffic between workgroups is h (forward) / dz (backward) of the
//     16-row tile, handed over as 8-byte {value, tag} granules written with ONE agent-scope
//     (sc1) store each and polled with sc1 loads until the tag matches (recipe R2 of the HIP
//     guide, Guideline 16; tags = step index + 1, the granule buffer is zeroed before every
//     launch).  Team members are placed on one XCD (blocks b, b+8, ...), so the hand-off stays
//     in that XCD's L2;
//   * the hand-off buffer is double-buffered by step parity; a member can only overwrite a
//     slot after every member has consumed it (it needed their next-step granules first);
//   * cell state c (forward) / dc (backward) never leaves registers.
// Every spin is bounded: on timeout the workgroup records a code in *err and stops waiting
// (results are then garbage, but the grid always drains).
//
// Layouts are those of lstm.hip (step frame; gx and acts [2][T][B][H][4 gates], hs/cs [2][T+1][B][H],
// out [B][T][2H], dz [2][T][B][4H]), so the two implementations are interchangeable.
#include "common.h"
#include <stdlib.h>

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;
#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

namespace {

constexpr unsigned kSpinLimit = 1u << 21;  // x s_sleep(1): ~0.1-1 s before giving up

__device__ __forceinline__ unsigned pack_bf2(float lo, float hi) {
  const unsigned a = __builtin_bit_cast(unsigned short, f2bf(lo));
  const unsigned b = __builtin_bit_cast(unsigned short, f2bf(hi));
  return a | (b << 16);
}

__device__ __forceinline__ void store_granule(gu64* g, unsigned tag, unsigned v) {
  __hip_atomic_store(g, ((unsigned long long)tag << 32) | v, RLX_AGENT);
}

// One wave reads NPL granules per lane (indices first + j*64 + lane) until every tag
// matches; a pass re-reads only the granules that were not ready yet.
template <int NPL>
__device__ __forceinline__ void sweep(const gu64* g, int first, unsigned tag, unsigned (&v)[NPL], bool& dead,
                                      gu32* err, unsigned code, int lane) {
  static_assert(NPL <= 32, "ready mask is 32 bits");
  constexpr unsigned all = NPL == 32 ? 0xffffffffu : ((1u << NPL) - 1);
  unsigned ready = 0;
  unsigned long long x[NPL];
  for (unsigned spins = 0;;) {
    // issue every outstanding load first (one round trip per pass), then check them
#pragma unroll
    for (int j = 0; j < NPL; ++j)
      if (!((ready >> j) & 1)) x[j] = __hip_atomic_load(g + first + j * 64 + lane, RLX_AGENT);
#pragma unroll
    for (int j = 0; j < NPL; ++j)
      if (!((ready >> j) & 1) && (unsigned)(x[j] >> 32) == tag) {
        v[j] = (unsigned)x[j];
        ready |= 1u << j;
      }
    if (__all(ready == all) || dead) return;
    if (++spins > kSpinLimit / 4) {  // the longer sleep below: about the same wall-time bound
      if (lane == 0) __hip_atomic_store(err, code, RLX_AGENT);
      dead = true;
      return;
    }
    // s_sleep(24) (~1500 clocks) between passes: the polls of 32 teams are a large share of
    // the L2 traffic, and fewer of them lower every team's hand-off latency (tools/lstm_micro.py,
    // per step: H = 512, B = 256: 6.82 us with s_sleep(1), 6.65 with 8, 6.28 with 24, 6.27 with
    // 48; H = 256, B = 256: 3.01 / 2.97 / 2.97 / 3.46).  Spinning on one granule per lane first
    // and sweeping once it is ready costs one more L2 round trip: 6.8 -> 8.3 us.
    __builtin_amdgcn_s_sleep(24);
  }
}

// Streaming activation traffic (gx / dout / acts / cs reads, acts / out / cs / hs / dz writes:
// ~10 MB per step at H = 512, B = 256, each byte touched once per launch).  nt = 1 issues it
// non-temporal so it does not evict the hand-off granules and W-side lines from L2 (the
// per-step hand-off latency grows from 4.2 us with 2 teams to 7.1 us with 32 at H = 512).
__device__ __forceinline__ void st_f4(float* p, float a, float b, float c, float d, bool nt) {
  if (nt) __builtin_nontemporal_store(f32x4{a, b, c, d}, reinterpret_cast<f32x4*>(p));
  else *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
__device__ __forceinline__ void st_f(float* p, float v, bool nt) {
  if (nt) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ void st_b(bf16* p, bf16 v, bool nt) {
  if (nt) __builtin_nontemporal_store(__builtin_bit_cast(unsigned short, v), reinterpret_cast<unsigned short*>(p));
  else *p = v;
}
// dL/dh_out of (direction d, step s, row r of length len, unit u) in the BATCH frame: the
// encoder-output gradient [B][T][2H] itself, read at position s (fw) or len - 1 - s (bw; steps past
// the length are dead and read position s) -- no to_step_frame pass before the top layer's BPTT
__device__ __forceinline__ size_t dout_bf_idx(int d, int s, int r, int len, int u, int T, int H) {
  const int t = (d == 0 || s >= len) ? s : len - 1 - s;
  return ((size_t)r * T + t) * 2 * H + (size_t)d * H + u;
}
__device__ __forceinline__ f32x4 ld_f4(const float* p, bool nt) {
  if (nt) return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return *reinterpret_cast<const f32x4*>(p);
}
__device__ __forceinline__ float ld_f(const float* p, bool nt) { return nt ? __builtin_nontemporal_load(p) : *p; }
// the BPTT's dL/dh_out element idx: DBF 0 / 1 fp32 (step / batch frame), DBF 2 bf16 (batch frame:
// the encoder-output gradient dE kept in bf16, profiles/r6/de_bf16.md)
template <int DBF>
__device__ __forceinline__ float ld_dout(const float* dout, size_t idx, bool nt) {
  if constexpr (DBF == 2) {
    const unsigned short* p = reinterpret_cast<const unsigned short*>(dout) + idx;
    return __uint_as_float((unsigned)(nt ? __builtin_nontemporal_load(p) : *p) << 16);
  } else {
    return ld_f(dout + idx, nt);
  }
}

// LDS tile [16 rows][RS] bf16 with the 16-byte chunk index XOR-swizzled by row (no padding:
// the backward tile is exactly 2 x 32 KB at H = 256).
template <int RS>
__device__ __forceinline__ int swz(int row, int col) {
  return row * RS + ((((col >> 3) ^ (row & 7))) << 3) + (col & 7);
}

// block -> (team, slice): team members share blockIdx % 8 (same XCD under round-robin dealing)
__device__ __forceinline__ bool team_of(int NC, int nteams, int& team, int& c) {
  const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
  team = (q / NC) * 8 + xcd;
  c = q % NC;
  return team < nteams;
}

}  // namespace

// RT row tiles per team (RT = 2 at H = 512: a team owns 32 rows, so a batch of 1024 runs in
// 2 launches instead of 4).  At H = 512 the 4 waves x 16 units x 4 gates need 256 VGPRs of
// W_hh B fragments per lane: launch bounds (256, 1) leave one wave per SIMD and the 512
// unified registers (arch + acc) for them.
//
// FX (layer 0, E = 128): the input projection x.W_x is computed HERE instead of by a GEMM
// writing gx (fp32 [2][T][B][4H]: 13.4 GB per direction at config #5 batch 2048, 420 MB at
// the bench shape).  The step-frame inputs xsf [2][T][B][128] (bf16, one gather launch) are
// read a step ahead; the x MFMAs of step s run before the step's hand-off sweep, i.e. in the
// shadow of the wait for the team's h_s, not on the recurrence's critical path.  W_x
// fragments: registers at RT = 1 (64 VGPRs), LDS at RT = 2 (64 KB; registers are full), where
// x is staged into LDS by global_load_lds (XOR-swizzled 16-byte chunks) and the x part of
// the gates waits in Gsh (the slots the cell update overwrites with the activations) --
// Ash is single-buffered there to make room: a wave only rewrites Ash after its sweep saw
// h_{s+1} of every wave of the team, each published after that wave's MFMAs read Ash.
template <int H, bool NT, int RT = 1, bool FX = false>
__global__ __launch_bounds__(256, 1) void lstm_fwd_persistent_kernel(
    const float* __restrict__ gx, const float* __restrict__ bias, const bf16* __restrict__ Wt,
    bf16* __restrict__ hs, float* __restrict__ cs, float* __restrict__ acts, bf16* __restrict__ out,
    const int* __restrict__ lens, gu64* xbuf, gu32* err, int T, int B, int ntile, int tile0, int ntile_l,
    const bf16* __restrict__ xsf, const bf16* __restrict__ Wx0, const bf16* __restrict__ Wx1) {
  constexpr int KS = H / 32, NC = H / 64, HP = H / 2, R = 16 * RT, G = R * HP, NPL = G / 256;
  constexpr int CH = NPL < 8 ? NPL : 8;  // granules per lane per sweep (chunks keep x[] at 16 VGPRs)
  constexpr int NR = 4 * RT;             // rows per lane
  constexpr int KE = 128, KSX = KE / 32; // FX: input width, its 32-deep MFMA steps
  constexpr bool FXL = FX && RT > 1;     // FX with W_x / x in LDS
  static_assert(NPL % CH == 0, "sweep chunks");
  __shared__ __attribute__((aligned(16))) bf16 Ash[FXL ? 1 : 2][R * H];
  // RT = 2: the step's gate activations wait here (not in registers) until the hand-off is out
  __shared__ __attribute__((aligned(16))) float Gsh[RT > 1 ? 256 * NR * 4 : 4];
  // FXL: x rows of steps s / s + 1 [2][R][128] and this workgroup's W_x fragments [wave][gate][kk][lane]
  __shared__ __attribute__((aligned(16))) bf16 Xsh[FXL ? 2 * R * KE : 8];
  __shared__ __attribute__((aligned(16))) bf16x8 Wxs[FXL ? 4 * 4 * KSX * 64 : 1];
  int lt, c;
  if (!team_of(NC, 2 * ntile_l, lt, c)) return;
  const int d = lt / ntile_l, tile = tile0 + lt % ntile_l, r0 = tile * R, team = d * ntile + tile;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int u = c * 64 + wid * 16 + (lane & 15);
  const size_t G4 = 4 * (size_t)H, BH = (size_t)B * H;
  bf16x8 Wf[4][KS];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) Wf[g][kk] = ld8(Wt + ((size_t)d * G4 + g * H + u) * H + kk * 32 + 8 * (lane >> 4));
  // gate biases of this lane's unit (gx = x.W_x comes from a bias-free GEMM)
  float gb[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) gb[g] = bias[(size_t)d * G4 + g * H + u];
  // lane rows: tile-local row rt * 16 + (lane >> 4) * 4 + i  (index j = rt * 4 + i)
  // rc / ln: recomputed / read from LDS (lnsh) rather than held in 2 x NR registers
  __shared__ int lnsh[R];
  if (threadIdx.x < R) lnsh[threadIdx.x] = r0 + (int)threadIdx.x < B ? lens[r0 + threadIdx.x] : 0;
  auto rowof = [&](int j) { return r0 + (j >> 2) * 16 + (lane >> 4) * 4 + (j & 3); };
  float creg[NR], hreg[NR];
  const bf16* hs0 = hs + (size_t)d * (T + 1) * BH;
  const float* cs0 = cs + (size_t)d * (T + 1) * BH;
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int r = rowof(j);
    const int rr = r < B ? r : B - 1;
    creg[j] = cs0[(size_t)rr * H + u];
    hreg[j] = bf2f(hs0[(size_t)rr * H + u]);
  }
  gu64* xb = xbuf + (size_t)team * 2 * G;
  bool dead = false;
  // FX: W_x B fragments of this lane's unit (row u * 4 + g of W_x^T [4H][128])
  bf16x8 Wxf[FX && !FXL ? 4 : 1][FX && !FXL ? KSX : 1];
  if constexpr (FX) {
    const bf16* Wx = d ? Wx1 : Wx0;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int kk = 0; kk < KSX; ++kk) {
        const bf16x8 wv = ld8(Wx + (size_t)(u * 4 + g) * KE + kk * 32 + 8 * (lane >> 4));
        if constexpr (FXL) Wxs[((wid * 4 + g) * KSX + kk) * 64 + lane] = wv;  // read back by this wave only
        else Wxf[g][kk] = wv;
      }
  }
  // FX: x rows of step st (tile rows, clamped to the batch) -- RT = 1 as A fragments in
  // registers (xan), RT = 2 into Xsh[st & 1] (wave w stages rows 8w .. 8w + 7, 1 KB per instruction)
  bf16x8 xan[FX && !FXL ? KSX : 1];
  auto load_x = [&](int st) {
    if constexpr (FXL) {
      int ln = lane;
      asm volatile("" : "+v"(ln));
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int row = (wid * 2 + q) * 4 + (ln >> 4), cg = (ln & 15) ^ (row & 7);
        const bf16* src = xsf + (((size_t)d * T + st) * B + min(r0 + row, B - 1)) * KE + cg * 8;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)&Xsh[(st & 1) * R * KE + (wid * 2 + q) * 512],
                                         16, 0, 0);
      }
    } else {
      const bf16* src = xsf + (((size_t)d * T + st) * B + min(r0 + (lane & 15), B - 1)) * KE + 8 * (lane >> 4);
#pragma unroll
      for (int kk = 0; kk < KSX; ++kk) xan[kk] = ld8(src + kk * 32);
    }
  };
  // gate pre-activations x.W_x of step s + 1 are loaded during step s (off the recurrence's
  // critical path: an HBM round trip per step otherwise)
  // RT = 1: in registers (gzn); RT = 2: straight into LDS (Gxsh, one global_load_lds_dwordx4
  // per row and lane: lane-linear 1 KB per wave instruction), no VGPRs
  float gzn[RT > 1 || FX ? 1 : NR][4];
  __shared__ __attribute__((aligned(16))) float Gxsh[RT > 1 && !FX ? 4 * NR * 64 * 4 : 4];
  auto load_gz = [&](int st) {
    const float* gxs = gx + ((size_t)d * T + st) * B * G4;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const float* src = gxs + ((size_t)min(rowof(j), B - 1) * H + u) * 4;
      if constexpr (RT > 1) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)&Gxsh[(wid * NR + j) * 256], 16, 0, 0);
      } else {
        const f32x4 q = ld_f4(src, NT);
        gzn[j][0] = q[0]; gzn[j][1] = q[1]; gzn[j][2] = q[2]; gzn[j][3] = q[3];
      }
    }
  };
  if constexpr (FX) load_x(0);
  else load_gz(0);
  for (int s = 0; s < T; ++s) {
    const int buf = FXL ? 0 : s & 1;
    f32x4 acc[RT][4];
    // FX: the x part of the gates, before the sweep (the wait for h_s hides it)
    if constexpr (FX && !FXL) {
      bf16x8 xa[KSX];
#pragma unroll
      for (int kk = 0; kk < KSX; ++kk) xa[kk] = xan[kk];
      if (s + 1 < T) load_x(s + 1);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        acc[0][g] = f32x4{0, 0, 0, 0};
#pragma unroll
        for (int kk = 0; kk < KSX; ++kk) acc[0][g] = mfma16(xa[kk], Wxf[g][kk], acc[0][g]);
      }
    } else if constexpr (FXL) {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's Xsh pieces of step s landed
      __syncthreads();                      // ... and every wave's
      const bf16* xs = &Xsh[(s & 1) * R * KE];
      // opaque per step: keeps the loop-invariant W_x fragment reads in the loop (hoisted, they
      // would hold 64 VGPRs for the whole launch and spill)
      // (and the lane's Xsh offsets: recomputed per step, not held)
      int wb = wid * 4 * KSX * 64 + lane, ln = lane;
      asm volatile("" : "+v"(wb), "+v"(ln));
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int row = rt * 16 + (ln & 15);
        bf16x8 xa[KSX];
#pragma unroll
        for (int kk = 0; kk < KSX; ++kk)
          xa[kk] = *reinterpret_cast<const bf16x8*>(&xs[row * KE + (((kk * 4 + (ln >> 4)) ^ (row & 7)) << 3)]);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 xz = f32x4{0, 0, 0, 0};
#pragma unroll
          for (int kk = 0; kk < KSX; ++kk) xz = mfma16(xa[kk], Wxs[wb + (g * KSX + kk) * 64], xz);
#pragma unroll
          for (int i = 0; i < 4; ++i) Gsh[((rt * 4 + i) * 256 + threadIdx.x) * 4 + g] = xz[i];
        }
      }
    }
    // RT = 1: the next step's x.W_x is requested now and the current one kept in gz; RT = 2
    // (no registers for two copies): requested after this step's cell update consumed gzn
    float gz[RT > 1 || FX ? 1 : NR][4];
    if constexpr (RT == 1 && !FX) {
#pragma unroll
      for (int j = 0; j < NR; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) gz[j][g] = gzn[j][g];
      if (s + 1 < T) load_gz(s + 1);
    }
    // ---- h_s of the whole R-row tile -> LDS
    if (s == 0) {
      for (int idx = threadIdx.x; idx < G; idx += 256) {
        const int row = idx / HP, p = idx % HP;
        const int rr = min(r0 + row, B - 1);
        *reinterpret_cast<unsigned*>(&Ash[0][swz<H>(row, 2 * p)]) =
            *reinterpret_cast<const unsigned*>(hs0 + (size_t)rr * H + 2 * p);
      }
    } else {
#pragma unroll
      for (int ch = 0; ch < NPL / CH; ++ch) {
        unsigned v[CH];
        const int first = wid * (G / 4) + ch * CH * 64;
        sweep<CH>(xb + (size_t)(s & 1) * G, first, (unsigned)s, v, dead, err, 1u, lane);
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          const int idx = first + j * 64 + lane;
          *reinterpret_cast<unsigned*>(&Ash[buf][swz<H>(idx / HP, 2 * (idx % HP))]) = v[j];
        }
      }
    }
    __syncthreads();
    if constexpr (RT > 1 && !FX) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this step's Gxsh landed
    // ---- z = h_s . W_hh for this wave's 16 units x 4 gates (B operands in registers)
    if constexpr (!(FX && !FXL)) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[rt][g] = f32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const bf16x8 a =
            *reinterpret_cast<const bf16x8*>(&Ash[buf][swz<H>(rt * 16 + (lane & 15), kk * 32 + 8 * (lane >> 4))]);
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[rt][g] = mfma16(a, Wf[g][kk], acc[rt][g]);
      }
    }
    // ---- cell update, NR rows x 1 unit per lane (gates kept in registers: stored after the
    // hand-off below, so the granule stores are not queued behind ~6 MB of activation stores
    // per step -- that ordering cost ~4 us per step at H = 512, B = 256)
    float ga[RT > 1 ? 1 : NR][4];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int rt = j >> 2, i = j & 3;
      if (s < lnsh[rowof(j) - r0]) {
        float* z = ga[RT > 1 ? 0 : j];
        float xv[4];
        if constexpr (FX && !FXL) {
          xv[0] = xv[1] = xv[2] = xv[3] = 0.f;  // already in acc
        } else if constexpr (FXL) {
          const float4 q = *reinterpret_cast<const float4*>(&Gsh[(j * 256 + threadIdx.x) * 4]);
          xv[0] = q.x; xv[1] = q.y; xv[2] = q.z; xv[3] = q.w;
        } else if constexpr (RT > 1) {
          const float4 q = *reinterpret_cast<const float4*>(&Gxsh[((wid * NR + j) * 64 + lane) * 4]);
          xv[0] = q.x; xv[1] = q.y; xv[2] = q.z; xv[3] = q.w;
        } else {
#pragma unroll
          for (int g = 0; g < 4; ++g) xv[g] = gz[RT > 1 ? 0 : j][g];
        }
        const float* x = xv;
        z[0] = fsigmoid(acc[rt][0][i] + x[0] + gb[0]);
        z[1] = ftanh(acc[rt][1][i] + x[1] + gb[1]);
        z[2] = fsigmoid(acc[rt][2][i] + x[2] + gb[2] + 1.0f);
        z[3] = fsigmoid(acc[rt][3][i] + x[3] + gb[3]);
        const float cc = z[2] * creg[j] + z[0] * z[1];
        creg[j] = cc;
        hreg[j] = bf2f(f2bf(z[3] * ftanh(cc)));
        if constexpr (RT > 1)
          *reinterpret_cast<float4*>(&Gsh[(j * 256 + threadIdx.x) * 4]) = make_float4(z[0], z[1], z[2], z[3]);
      }
    }
    if constexpr (FXL) {
      if (s + 1 < T) load_x(s + 1);
    } else if constexpr (RT > 1 && !FX) {
      if (s + 1 < T) load_gz(s + 1);
    }
    // ---- publish h_{s+1}: unit pairs (u, u+1) of adjacent lanes -> one granule
    if (s + 1 < T) {
      gu64* dst = xb + (size_t)((s + 1) & 1) * G;
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        const float hn = __shfl_xor(hreg[j], 1, 64);
        if (!(lane & 1))
          store_granule(dst + ((j >> 2) * 16 + (lane >> 4) * 4 + (j & 3)) * HP + u / 2, (unsigned)(s + 1),
                        pack_bf2(hreg[j], hn));
      }
    }
    float* cnext = cs + ((size_t)d * (T + 1) + s + 1) * BH;
    bf16* hnext = hs + ((size_t)d * (T + 1) + s + 1) * BH;
    // FXL: the rows' store addresses recomputed per step from an opaque lane (held for the
    // launch they spill, and the reloads wait behind the step's outstanding stores)
    int sl = lane;
    if constexpr (FXL) asm volatile("" : "+v"(sl));
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int r = r0 + (j >> 2) * 16 + (sl >> 4) * 4 + (j & 3), lj = lnsh[r - r0];
      if (s < lj) {
        if constexpr (RT > 1) {
          const float4 z = *reinterpret_cast<const float4*>(&Gsh[(j * 256 + threadIdx.x) * 4]);
          st_f4(acts + ((((size_t)d * T + s) * B + r) * H + u) * 4, z.x, z.y, z.z, z.w, NT);
        } else {
          st_f4(acts + ((((size_t)d * T + s) * B + r) * H + u) * 4, ga[j][0], ga[j][1], ga[j][2], ga[j][3],
                NT);  // one 16-byte store per (row, unit)
        }
      }
      if (r < B) {  // h at its position; positions past the length get zeros (no fill of out)
        const bool live = s < lj;
        const int t = (d == 0 || !live) ? s : lj - 1 - s;
        st_b(out + ((size_t)r * T + t) * 2 * H + d * H + u, f2bf(live ? hreg[j] : 0.f), NT);
      }
      if (r < B) {
        st_f(cnext + (size_t)r * H + u, creg[j], NT);
        st_b(hnext + (size_t)r * H + u, f2bf(hreg[j]), NT);
      }
    }
  }
}

// Forward with 8 waves per workgroup (H = 512; any H % 64 == 0).  Four waves x 16 units x 4
// gates would need H = 512 k-rows of W_hh per gate column: 256 VGPRs of B fragments per lane.
// Here wave w owns 8 units (c*64 + 8w .. +7) and two 16-column MFMA tiles: tile t, column n
// holds gate 2t + (n >> 3) of unit n & 7, so W_hh stays register-resident at H = 512 with
// 2 x KS x 4 = 128 VGPRs.  After the MFMAs lane n (< 8) has gates i, f and lane n ^ 8 has
// j, o of the same unit for the same 4 rows; four row_ror:8 DPP moves swap half of them, and
// each lane then updates the cell for 2 of the 4 rows (lanes n < 8: rows 0-1, n >= 8: 2-3).
// Hand-off, layouts and tags are the 4-wave kernel's.
template <int H, bool NT>
__global__ __launch_bounds__(512, 1) void lstm_fwd_persistent8_kernel(
    const float* __restrict__ gx, const float* __restrict__ bias, const bf16* __restrict__ Wt,
    bf16* __restrict__ hs, float* __restrict__ cs, float* __restrict__ acts, bf16* __restrict__ out,
    const int* __restrict__ lens, gu64* xbuf, gu32* err, int T, int B, int ntile, int tile0, int ntile_l) {
  constexpr int KS = H / 32, NC = H / 64, HP = H / 2, G = 16 * HP, NPL = G / 512;
  static_assert(H % 64 == 0 && G % 512 == 0, "8-wave LSTM layout");
  __shared__ __attribute__((aligned(16))) bf16 Ash[2][16 * H];
  int lt, c;
  if (!team_of(NC, 2 * ntile_l, lt, c)) return;
  const int d = lt / ntile_l, tile = tile0 + lt % ntile_l, r0 = tile * 16, team = d * ntile + tile;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = lane & 15, half = n >> 3;
  const int u = c * 64 + wid * 8 + (n & 7);
  const size_t G4 = 4 * (size_t)H, BH = (size_t)B * H;
  bf16x8 Wf[2][KS];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
      Wf[t][kk] = ld8(Wt + ((size_t)d * G4 + (2 * t + half) * H + u) * H + kk * 32 + 8 * (lane >> 4));
  float gb[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) gb[g] = bias[(size_t)d * G4 + g * H + u];
  // this lane's rows within the tile: 4 (lane >> 4) + 2 half + i
  int rc[2], ln[2], rt[2];
  bool rok[2];
  float creg[2], hreg[2];
  const bf16* hs0 = hs + (size_t)d * (T + 1) * BH;
  const float* cs0 = cs + (size_t)d * (T + 1) * BH;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rt[i] = (lane >> 4) * 4 + 2 * half + i;
    const int r = r0 + rt[i];
    rok[i] = r < B;
    rc[i] = rok[i] ? r : B - 1;
    ln[i] = rok[i] ? lens[r] : 0;
    creg[i] = cs0[(size_t)rc[i] * H + u];
    hreg[i] = bf2f(hs0[(size_t)rc[i] * H + u]);
  }
  gu64* xb = xbuf + (size_t)team * 2 * G;
  bool dead = false;
  float gzn[2][4];  // x.W_x of the next step, prefetched as in the 4-wave kernel
  auto load_gz = [&](int st) {
    const float* gxs = gx + ((size_t)d * T + st) * B * G4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 q = ld_f4(gxs + ((size_t)rc[i] * H + u) * 4, NT);
      gzn[i][0] = q[0]; gzn[i][1] = q[1]; gzn[i][2] = q[2]; gzn[i][3] = q[3];
    }
  };
  // Step outputs (gates, h, c) are stored one step late: issued right after the next step's
  // hand-off arrived, they drain during its MFMAs and cell update.  gfx9's vmcnt counts
  // stores too, so stores issued before a hand-off sweep made every poll wait for them
  // (H = 512, B = 256: 8.8 -> 7.0 us per step; the 4-wave H <= 256 kernel measured 3.3 ->
  // 3.5 us with the same change, so it keeps storing right after its own hand-off).
  float ga[2][4];
  auto store_step = [&](int ss) {
    float* cnext = cs + ((size_t)d * (T + 1) + ss + 1) * BH;
    bf16* hnext = hs + ((size_t)d * (T + 1) + ss + 1) * BH;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = rc[i];
      if (ss < ln[i]) {
        st_f4(acts + ((((size_t)d * T + ss) * B + r) * H + u) * 4, ga[i][0], ga[i][1], ga[i][2], ga[i][3], NT);
      }
      if (rok[i]) {  // h at its position; positions past the length get zeros (no fill of out)
        const bool live = ss < ln[i];
        const int t = (d == 0 || !live) ? ss : ln[i] - 1 - ss;
        st_b(out + ((size_t)r * T + t) * 2 * H + d * H + u, f2bf(live ? hreg[i] : 0.f), NT);
      }
      if (rok[i]) {
        st_f(cnext + (size_t)r * H + u, creg[i], NT);
        st_b(hnext + (size_t)r * H + u, f2bf(hreg[i]), NT);
      }
    }
  };
  load_gz(0);
  for (int s = 0; s < T; ++s) {
    const int buf = s & 1;
    float gz[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) gz[i][g] = gzn[i][g] + gb[g];
    if (s + 1 < T) load_gz(s + 1);
    if (s == 0) {
      for (int idx = threadIdx.x; idx < G; idx += 512) {
        const int row = idx / HP, p = idx % HP;
        const int rr = min(r0 + row, B - 1);
        *reinterpret_cast<unsigned*>(&Ash[0][swz<H>(row, 2 * p)]) =
            *reinterpret_cast<const unsigned*>(hs0 + (size_t)rr * H + 2 * p);
      }
    } else {
      unsigned v[NPL];
      sweep<NPL>(xb + (size_t)(s & 1) * G, wid * (G / 8), (unsigned)s, v, dead, err, 1u, lane);
#pragma unroll
      for (int j = 0; j < NPL; ++j) {
        const int idx = wid * (G / 8) + j * 64 + lane;
        *reinterpret_cast<unsigned*>(&Ash[buf][swz<H>(idx / HP, 2 * (idx % HP))]) = v[j];
      }
    }
    __syncthreads();
    if (s > 0) store_step(s - 1);
    f32x4 acc[2] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(&Ash[buf][swz<H>(lane & 15, kk * 32 + 8 * (lane >> 4))]);
      acc[0] = mfma16(a, Wf[0][kk], acc[0]);
      acc[1] = mfma16(a, Wf[1][kk], acc[1]);
    }
    // swap gate halves with the partner lane n ^ 8 (same rows): lanes n < 8 keep rows 0-1 and
    // receive j, o; lanes n >= 8 keep rows 2-3 and receive i, f
    float rcv[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      rcv[i] = dpp_f<DPP_ROR8>(half ? acc[0][i] : acc[0][2 + i]);
      rcv[2 + i] = dpp_f<DPP_ROR8>(half ? acc[1][i] : acc[1][2 + i]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (s < ln[i]) {
        const float zi = half ? rcv[i] : acc[0][i], zj = half ? acc[0][2 + i] : rcv[i];
        const float zf = half ? rcv[2 + i] : acc[1][i], zo = half ? acc[1][2 + i] : rcv[2 + i];
        ga[i][0] = fsigmoid(zi + gz[i][0]);
        ga[i][1] = ftanh(zj + gz[i][1]);
        ga[i][2] = fsigmoid(zf + gz[i][2] + 1.0f);
        ga[i][3] = fsigmoid(zo + gz[i][3]);
        const float cc = ga[i][2] * creg[i] + ga[i][0] * ga[i][1];
        creg[i] = cc;
        hreg[i] = bf2f(f2bf(ga[i][3] * ftanh(cc)));
      }
    }
    if (s + 1 < T) {
      gu64* dst = xb + (size_t)((s + 1) & 1) * G;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float hn = dpp_f<DPP_XOR1>(hreg[i]);  // unit u + 1 (lane n ^ 1, same half)
        if (!(lane & 1)) store_granule(dst + rt[i] * HP + u / 2, (unsigned)(s + 1), pack_bf2(hreg[i], hn));
      }
    }
  }
  store_step(T - 1);
}

// Backward.  Exchanging dz (4H gate columns) would cost 4x the forward's traffic, so the
// recurrent GEMM is split by K instead: workgroup c multiplies ITS dz slice (the 4 gates of
// its 64 units, 256 columns, written to LDS) by the matching W_hh rows and produces a
// PARTIAL dh for all H units; wave w's 64 output units are exactly slice w's, and go to
// workgroup (team, w) as fp32 granules.  Each workgroup sums NC partials for its own units
// (its own partial stays in LDS): per step a lane reads 4 x (NC-1) granules instead of 32.
// NW = 4 or 8 waves: the cell update covers the tile's 16 rows x 64 units with RPL = 16 / NW
// rows per lane (4 or 2); waves < NC run the partial GEMM (at H = 512, NC = 8: all 8 waves).
template <int H, int NW, bool NT, int DBF = 0>
__global__ __launch_bounds__(64 * NW, 1) void lstm_bwd_persistent_kernel(
    bf16* __restrict__ dz, const bf16* __restrict__ Wn, const float* __restrict__ dout,
    const float* __restrict__ dh_fin, float* __restrict__ dc_carry, const float* __restrict__ acts,
    const float* __restrict__ cs, const int* __restrict__ lens, gu64* xbuf, gu32* err,
    float* __restrict__ dbias,  // [2][4H] nullable: += sum over rows and steps of dz (gate-bias gradient)
    int T, int B, int ntile, int tile0, int ntile_l) {
  constexpr int G4 = 4 * H, NC = H / 64, KS = 256 / 32, SLOT = 16 * 64, TEAMX = 2 * NC * NC * SLOT;
  constexpr int RPL = 16 / NW;  // rows per lane in the cell update
  static_assert((NW == 4 || NW == 8) && NC <= NW && RPL * NC <= 32, "bwd layout");
  __shared__ __attribute__((aligned(16))) bf16 Ash[16 * 256];   // dz slice [16 rows][4 gates x 64 units]
  __shared__ float Pown[16 * 64];                                // own partial dh [16 rows][64 units]
  int lt, c;
  if (!team_of(NC, 2 * ntile_l, lt, c)) return;
  const int d = lt / ntile_l, tile = tile0 + lt % ntile_l, r0 = tile * 16, team = d * ntile + tile;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ul = (wid & 3) * 16 + (lane & 15);  // this lane's unit within the slice (cell update)
  const int row0 = (wid >> 2) * (4 * RPL) + (lane >> 4) * RPL;  // its first row within the tile
  const int u = c * 64 + ul;
  const size_t BH = (size_t)B * H;
  // B operand of the partial GEMM: B[k][n] = W_hh[v][gate col(k)], k = g*64 + unit-in-slice,
  // n = output unit v = 64*wid + 16*t + (lane&15)
  bf16x8 Wp[4][KS];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int k0 = kk * 32 + 8 * (lane >> 4), g = k0 / 64, ul0 = k0 % 64;
      const int v = min(64 * wid + 16 * t + (lane & 15), H - 1);  // waves >= NC own no output units
      Wp[t][kk] = ld8(Wn + ((size_t)d * H + v) * G4 + g * H + 64 * c + ul0);
    }
  int rc[RPL], ln[RPL];
  bool rok[RPL];
  float dcreg[RPL];
#pragma unroll
  for (int i = 0; i < RPL; ++i) {
    const int r = r0 + row0 + i;
    rok[i] = r < B;
    rc[i] = rok[i] ? r : B - 1;
    ln[i] = rok[i] ? lens[r] : 0;
    dcreg[i] = dc_carry[(size_t)d * BH + (size_t)rc[i] * H + u];
  }
  gu64* xb = xbuf + (size_t)team * TEAMX;  // [parity][dest][src][16][64]
  bool dead = false;
  // gate-bias gradient of (unit u, gate g): the lane's rows summed over all steps in
  // registers (fp32, off the recurrence's critical path), reduced over the wave's 4 row
  // groups and added once per team at the end -- replaces a 2 x 210 MB column reduction
  float bacc[4] = {0.f, 0.f, 0.f, 0.f};
  // dh_fin is step-invariant; c_s of step s is c_{(s-1)+1} of the next (reverse) step
  float dhf[RPL], cn[RPL];
#pragma unroll
  for (int i = 0; i < RPL; ++i) {
    const size_t ri = (size_t)rc[i] * H + u;
    dhf[i] = dh_fin[(size_t)d * BH + ri];
    cn[i] = cs[((size_t)d * (T + 1) + T) * BH + ri];
  }
  for (int s = T - 1; s >= 0; --s) {
    // row0v = row0, opaque to the optimizer each step: otherwise every per-peer / per-row
    // granule address is hoisted out of the step loop as a 64-bit register pair
    int row0v = row0;
    asm volatile("" : "+v"(row0v));
    float dho[RPL], a4[RPL][4], cpv[RPL];
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      const size_t ri = (size_t)rc[i] * H + u;
      if constexpr (NT) {
        dho[i] = ld_dout<DBF>(dout, DBF ? dout_bf_idx(d, s, rc[i], ln[i], u, T, H) : ((size_t)d * T + s) * BH + ri, true);
        const f32x4 q = ld_f4(acts + ((((size_t)d * T + s) * B + rc[i]) * H + u) * 4, true);
        a4[i][0] = q[0]; a4[i][1] = q[1]; a4[i][2] = q[2]; a4[i][3] = q[3];
        cpv[i] = ld_f(cs + ((size_t)d * (T + 1) + s) * BH + ri, true);
      } else {
        dho[i] = ld_dout<DBF>(dout, DBF ? dout_bf_idx(d, s, rc[i], ln[i], u, T, H) : ((size_t)d * T + s) * BH + ri, false);
        const float4 q = *reinterpret_cast<const float4*>(acts + ((((size_t)d * T + s) * B + rc[i]) * H + u) * 4);
        a4[i][0] = q.x; a4[i][1] = q.y; a4[i][2] = q.z; a4[i][3] = q.w;
        cpv[i] = cs[((size_t)d * (T + 1) + s) * BH + ri];
      }
    }
    // dz rows of step `step` -> global from the LDS copy (own-lane values), issued after this step's
    // hand-off stores (as in the forward: the granules must not queue behind the activation
    // traffic).  Deferring them to the next step's polls with LDS-only barriers measured slower:
    // H = 256, B = 256: 4.57 vs 3.67 us per step (profiles/r6/lstm_bptt.md)
    auto store_dz = [&](int step) {
#pragma unroll
      for (int i = 0; i < RPL; ++i)
        if (rok[i]) {
          bf16* dzr = dz + (((size_t)d * T + step) * B + rc[i]) * G4;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            if constexpr (NT) st_b(dzr + g * H + u, Ash[swz<256>(row0 + i, g * 64 + ul)], true);
            else dzr[g * H + u] = Ash[swz<256>(row0 + i, g * 64 + ul)];
          }
        }
    };
    // ---- recurrent dh for this lane's rows: own partial (LDS) + the peers' (granules)
    float rec[RPL];
#pragma unroll
    for (int i = 0; i < RPL; ++i) rec[i] = 0.f;
    if (s + 1 < T) {
#pragma unroll
      for (int i = 0; i < RPL; ++i) rec[i] = Pown[(row0 + i) * 64 + ul];
      if constexpr (NC > 1) {
        // peers in chunks of PC (at H = 512 all 8 at once would hold 32 VGPRs of granules and
        // spill); each chunk's ready granules keep their value in x (not re-read)
        // (all 8 peers at once at H = 512 spills 19 VGPRs: 8.9 vs 7.4 us per step)
        constexpr int PC = NC < 4 ? NC : 4;
        const gu64* src = xb + (size_t)((s + 1) & 1) * NC * NC * SLOT + (size_t)c * NC * SLOT;
        const unsigned tag = (unsigned)(T - 1 - s);
#pragma unroll
        for (int p0 = 0; p0 < NC; p0 += PC) {
          unsigned ready = 0;
          unsigned long long x[PC][RPL];
          constexpr unsigned allm = RPL * PC >= 32 ? 0xffffffffu : ((1u << (RPL * PC % 32)) - 1);
          const unsigned need = (c >= p0 && c < p0 + PC) ? allm & ~(((1u << RPL) - 1) << (RPL * (c - p0))) : allm;
          for (unsigned spins = 0;;) {
#pragma unroll
            for (int q = 0; q < PC; ++q)
#pragma unroll
              for (int i = 0; i < RPL; ++i)
                if (p0 + q != c && !((ready >> (q * RPL + i)) & 1))
                  x[q][i] = __hip_atomic_load(src + (size_t)(p0 + q) * SLOT + (row0v + i) * 64 + ul, RLX_AGENT);
#pragma unroll
            for (int q = 0; q < PC; ++q)
#pragma unroll
              for (int i = 0; i < RPL; ++i) {
                const int bit = q * RPL + i;
                if (p0 + q != c && !((ready >> bit) & 1) && (unsigned)(x[q][i] >> 32) == tag) ready |= 1u << bit;
              }
            if (__all((ready & need) == need) || dead) break;
            if (++spins > kSpinLimit / 4) {
              if (lane == 0) __hip_atomic_store(err, 2u, RLX_AGENT);
              dead = true;
              break;
            }
            // see sweep(): BPTT per step at H = 512, B = 256: 8.22 us with s_sleep(1), 8.09
            // with 8, 8.14 with 24, 8.13 with 48, 7.52 with 96; H = 256, B = 256: 4.04 / 3.83 /
            // 3.63 / 3.64 / 4.94; B = 512: 5.52 / 5.26 / 4.90 / 4.57 / 5.38
            __builtin_amdgcn_s_sleep(H >= 512 ? 96 : 48);
          }
#pragma unroll
          for (int q = 0; q < PC; ++q)
#pragma unroll
            for (int i = 0; i < RPL; ++i)
              if (p0 + q != c) rec[i] += ((ready >> (q * RPL + i)) & 1) ? __uint_as_float((unsigned)x[q][i]) : 0.f;
        }
      }
    }
    // ---- cell backward -> dz (4 gates) for (the lane's rows, unit u)
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      float dzv[4];
      if (s < ln[i]) {
        const float dh = rec[i] + dho[i] + (s + 1 >= ln[i] ? dhf[i] : 0.f);
        const float ig = a4[i][0], jg = a4[i][1], fg = a4[i][2], og = a4[i][3];
        const float tc = ftanh(cn[i]);
        const float dc = dcreg[i] + dh * og * (1.0f - tc * tc);
        dzv[0] = dc * jg * ig * (1.0f - ig);
        dzv[1] = dc * ig * (1.0f - jg * jg);
        dzv[2] = dc * cpv[i] * fg * (1.0f - fg);
        dzv[3] = dh * tc * og * (1.0f - og);
        dcreg[i] = dc * fg;
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) dzv[g] = 0.f;
      }
      cn[i] = cpv[i];
      const int row = row0 + i;
#pragma unroll
      for (int g = 0; g < 4; ++g) bacc[g] += dzv[g];
#pragma unroll
      for (int g = 0; g < 4; ++g) Ash[swz<256>(row, g * 64 + ul)] = f2bf(dzv[g]);
    }
    if (s == 0) {
      store_dz(0);  // own-lane LDS values: no barrier needed
      break;
    }
    __syncthreads();  // dz slice complete in LDS (and every lane has read Pown)
    // ---- partial dh over this slice's gate columns, for units 64*wid .. +63
    if (wid < NC) {
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(&Ash[swz<256>(lane & 15, kk * 32 + 8 * (lane >> 4))]);
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = mfma16(a, Wp[t][kk], acc[t]);
    }
    // ---- publish: wave wid's units belong to slice wid
    if (wid == c) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) Pown[((lane >> 4) * 4 + r) * 64 + 16 * t + (lane & 15)] = acc[t][r];
    } else {
      gu64* dst = xb + (size_t)(s & 1) * NC * NC * SLOT + ((size_t)wid * NC + c) * SLOT;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          store_granule(dst + ((lane >> 4) * 4 + r) * 64 + 16 * t + (lane & 15), (unsigned)(T - s),
                        __float_as_uint(acc[t][r]));
    }
    }
    store_dz(s);
    __syncthreads();  // Pown visible before the next step reads it; Ash free for rewriting
  }
#pragma unroll
  for (int i = 0; i < RPL; ++i)
    if (rok[i]) dc_carry[(size_t)d * BH + (size_t)rc[i] * H + u] = dcreg[i];
  if (dbias) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float t = sum_x32(sum_x16(bacc[g]));  // lanes l, l^16, l^32, l^48: the 4 row groups
      if ((lane >> 4) == 0) atomicAdd(dbias + (size_t)d * G4 + g * H + u, t);
    }
  }
}

// Backward with 32-row teams at H = 512 (batch > 256: batch 1024 in 2 launches instead of 4).
// 16 waves per workgroup (4 per SIMD, 128 unified registers each).  Wave w produces the partial
// dh of output units 32w .. 32w+31 (destined for slice w / 2) for all 32 rows: 2 x 2 MFMA
// tiles.  Its W_hh B fragments are 2 column tiles x 8 k-chunks: tile 0 in registers (32 VGPRs),
// tile 1 in LDS (16 waves x 8 KB = 128 KB, lane-contiguous 16-byte reads).  The cell update
// covers 32 rows x 64 units at 2 rows per lane; hand-off protocol, tags and layouts are the
// 16-row kernel's with 32-row slots.  (The earlier 32-row attempt -- 4 waves, all of W_hh in
// registers -- spilled ~40 registers: profiles/r3/micro/lstm_rt2_bwd_rejected.log.)
// base + a 32-bit byte offset: with a uniform base the access uses SGPR-base addressing and
// one 32-bit offset register instead of a 64-bit address pair per access
template <typename TT>
__device__ __forceinline__ TT* boff(TT* p, unsigned bytes) {
  return reinterpret_cast<TT*>(reinterpret_cast<char*>(const_cast<void*>(static_cast<const void*>(p))) + bytes);
}
__device__ __forceinline__ gu64* gboff(gu64* p, unsigned bytes) {
  return reinterpret_cast<gu64*>(reinterpret_cast<__attribute__((address_space(1))) char*>(p) + bytes);
}
__device__ __forceinline__ const gu64* gboff(const gu64* p, unsigned bytes) {
  return reinterpret_cast<const gu64*>(reinterpret_cast<const __attribute__((address_space(1))) char*>(p) + bytes);
}

// attribution builds (tools/lstm_bptt_stamps.py): thread 0 of every workgroup sums s_memtime
// deltas per step phase over the recurrence and stores the 8 sums at lb_stamps[(team NC + c) 8]
// (a buffer only the tool reads; STAMP = false compiles none of it)
__device__ unsigned long long* lb_stamps = nullptr;
static bool lb_stamps_on = false;
void set_lstm_bwd_stamps(unsigned long long* buf) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(lb_stamps), &buf, sizeof(buf));
  lb_stamps_on = buf != nullptr;
}

// PC: peers polled per chunk (4: 8 registers spill); SL: s_sleep between poll passes.
// Measured and not kept (profiles/r6/lstm_bptt.md): the step's dz stores issued after the NEXT
// step's hand-off poll with LDS-only barriers -- the stamps moved 1.7k of the 7.4k "dz stores +
// barrier 2" cycles, the BPTT micro -2.5 % at batch 2048, config #5 per step unchanged
// (356.3 / 356.9 vs 357.0 / 356.2 ms).
template <bool NT, int PC = 2, int SL = 96, int DBF = 0, bool STAMP = false>
__global__ __launch_bounds__(1024, 1) void lstm_bwd_persistent32_kernel(
    bf16* __restrict__ dz, const bf16* __restrict__ Wn, const float* __restrict__ dout,
    const float* __restrict__ dh_fin, float* __restrict__ dc_carry, const float* __restrict__ acts,
    const float* __restrict__ cs, const int* __restrict__ lens, gu64* xbuf, gu32* err,
    float* __restrict__ dbias, int T, int B, int ntile, int tile0, int ntile_l) {
  constexpr int H = 512, G4 = 4 * H, NC = H / 64, KS = 256 / 32, RT = 32, SLOT = RT * 64;
  constexpr int TEAMX = 2 * NC * NC * SLOT, RPL = 2;
  __shared__ __attribute__((aligned(16))) bf16x8 Wl[16 * KS * 64];  // [wave][kk][lane]
  __shared__ __attribute__((aligned(16))) bf16 Ash[RT * 256];      // dz slice [32 rows][4 gates x 64 units]
  __shared__ float Pown[RT * 64];                                  // own partial dh [32 rows][64 units]
  int lt, c;
  if (!team_of(NC, 2 * ntile_l, lt, c)) return;
  const int d = lt / ntile_l, tile = tile0 + lt % ntile_l, r0 = tile * RT, team = d * ntile + tile;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ul = (wid & 3) * 16 + (lane & 15);             // this lane's unit within the slice
  const int row0 = (wid >> 2) * 8 + (lane >> 4) * RPL;     // its first row within the tile
  const int u = c * 64 + ul;
  const size_t BH = (size_t)B * H;
  // B[k][n] = W_hh[v][gate col(k)], k = g*64 + unit-in-slice, n = output unit v = 32 wid + 16 t + (lane & 15)
  bf16x8 Wr[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const int k0 = kk * 32 + 8 * (lane >> 4), g = k0 / 64, ul0 = k0 % 64;
    const int v = 32 * wid + (lane & 15);
    Wr[kk] = ld8(Wn + ((size_t)d * H + v) * G4 + g * H + 64 * c + ul0);
    Wl[(wid * KS + kk) * 64 + lane] = ld8(Wn + ((size_t)d * H + v + 16) * G4 + g * H + 64 * c + ul0);
  }
  int rc[RPL], ln[RPL];
  bool rok[RPL];
  float dcreg[RPL], dhf[RPL], cn[RPL];
#pragma unroll
  for (int i = 0; i < RPL; ++i) {
    const int r = r0 + row0 + i;
    rok[i] = r < B;
    rc[i] = rok[i] ? r : B - 1;
    ln[i] = rok[i] ? lens[r] : 0;
    const size_t ri = (size_t)rc[i] * H + u;
    dcreg[i] = dc_carry[(size_t)d * BH + ri];
    dhf[i] = dh_fin[(size_t)d * BH + ri];
    cn[i] = cs[((size_t)d * (T + 1) + T) * BH + ri];
  }
  gu64* xb = xbuf + (size_t)team * TEAMX;  // [parity][dest][src][32][64]
  bool dead = false;
  float bacc[4] = {0.f, 0.f, 0.f, 0.f};
  // STAMP: phase sums (0 loads issued, 1 hand-off wait, 2 cell backward, 3 barrier 1, 4 MFMA,
  // 5 publish, 6 dz stores + barrier 2, 7 steps)
  unsigned long long st_last = 0;
  unsigned st_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0};

  auto stamp = [&](int ph) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (ph >= 0) st_sum[ph] += (unsigned)(t - st_last);
      st_last = t;
    }
  };
  for (int s = T - 1; s >= 0; --s) {
    stamp(-1);
    if constexpr (STAMP) st_sum[7] += 1;
    int row0v = row0;
    asm volatile("" : "+v"(row0v));
    // uniform step bases + 32-bit per-lane byte offsets (saddr addressing: no 64-bit address
    // pairs per row held across the step)
    // (DBF: the batch-frame gradient's direction half; rows and positions per lane below)
    const float* dout_s = DBF == 1 ? dout + d * H : dout + ((size_t)d * T + s) * BH;
    const bf16* doutb_s = reinterpret_cast<const bf16*>(dout) + d * H;  // (DBF 2)
    const float* acts_s = acts + ((size_t)d * T + s) * BH * 4;
    const float* cs_s = cs + ((size_t)d * (T + 1) + s) * BH;
    float dho[RPL], a4[RPL][4], cpv[RPL];
    unsigned rio[RPL];  // rc * H + u, opaque per step (no loop-strength-reduced 64-bit pointers)
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      rio[i] = (unsigned)(rc[i] * H + u);
      asm volatile("" : "+v"(rio[i]));
    }
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      const unsigned ri = rio[i];
      if constexpr (DBF) {  // batch-frame row (rc * T + position), opaque: no hoisted 64-bit offsets
        // (the row from the opaque rio = rc * H + u: no extra live register per row)
        const unsigned rt = (ri / H) * (unsigned)T + (unsigned)((d == 0 || s >= ln[i]) ? s : ln[i] - 1 - s);
        if constexpr (DBF == 2)
          dho[i] = ld_dout<2>(reinterpret_cast<const float*>(boff(doutb_s, (unsigned)u * 2u)), (size_t)rt * (2 * H), NT);
        else
          dho[i] = ld_f(boff(dout_s, (unsigned)u * 4u) + (size_t)rt * (2 * H), NT);
      } else {
        dho[i] = ld_f(boff(dout_s, ri * 4u), NT);
      }
      const f32x4 q = ld_f4(boff(acts_s, ri * 16u), NT);
      a4[i][0] = q[0]; a4[i][1] = q[1]; a4[i][2] = q[2]; a4[i][3] = q[3];
      cpv[i] = ld_f(boff(cs_s, ri * 4u), NT);
    }
    auto store_dz = [&](int step) {
#pragma unroll
      for (int i = 0; i < RPL; ++i)
        if (rok[i]) {
          bf16* dz_s = dz + ((size_t)d * T + step) * B * G4;
          const int sb = swz<256>(row0 + i, ul);
          const unsigned o = (rio[i] + (unsigned)(rc[i] * 3 * H)) * 2u;
#pragma unroll
          for (int g = 0; g < 4; ++g) st_b(boff(dz_s, o + g * H * 2u), Ash[sb + g * 64], NT);
        }
    };
    float rec[RPL];
#pragma unroll
    for (int i = 0; i < RPL; ++i) rec[i] = 0.f;
    stamp(0);
    if (s + 1 < T) {
#pragma unroll
      for (int i = 0; i < RPL; ++i) rec[i] = Pown[(row0 + i) * 64 + ul];
      const gu64* src = xb + (size_t)((s + 1) & 1) * NC * NC * SLOT + (size_t)c * NC * SLOT;
      const unsigned tag = (unsigned)(T - 1 - s);
#pragma unroll
      for (int p0 = 0; p0 < NC; p0 += PC) {
        unsigned ready = 0;
        unsigned long long x[PC][RPL];
        constexpr unsigned allm = (1u << (RPL * PC)) - 1;
        const unsigned need = (c >= p0 && c < p0 + PC) ? allm & ~(((1u << RPL) - 1) << (RPL * (c - p0))) : allm;
        for (unsigned spins = 0;;) {
          unsigned lo = (unsigned)(row0v * 64 + ul) * 8u;  // opaque per pass: not hoisted as address pairs
          asm volatile("" : "+v"(lo));
#pragma unroll
          for (int q = 0; q < PC; ++q)
#pragma unroll
            for (int i = 0; i < RPL; ++i)
              if (p0 + q != c && !((ready >> (q * RPL + i)) & 1))
                x[q][i] = __hip_atomic_load(gboff(src + (p0 + q) * SLOT, lo + i * 512u), RLX_AGENT);
#pragma unroll
          for (int q = 0; q < PC; ++q)
#pragma unroll
            for (int i = 0; i < RPL; ++i) {
              const int bit = q * RPL + i;
              if (p0 + q != c && !((ready >> bit) & 1) && (unsigned)(x[q][i] >> 32) == tag) ready |= 1u << bit;
            }
          if (__all((ready & need) == need) || dead) break;
          if (++spins > kSpinLimit / 4) {
            if (lane == 0) __hip_atomic_store(err, 2u, RLX_AGENT);
            dead = true;
            break;
          }
          __builtin_amdgcn_s_sleep(SL);
        }
#pragma unroll
        for (int q = 0; q < PC; ++q)
#pragma unroll
          for (int i = 0; i < RPL; ++i)
            if (p0 + q != c) rec[i] += ((ready >> (q * RPL + i)) & 1) ? __uint_as_float((unsigned)x[q][i]) : 0.f;
      }
    }
    stamp(1);
    // ---- cell backward -> dz (4 gates) for (the lane's rows, unit u)
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      float dzv[4];
      if (s < ln[i]) {
        const float dh = rec[i] + dho[i] + (s + 1 >= ln[i] ? dhf[i] : 0.f);
        const float ig = a4[i][0], jg = a4[i][1], fg = a4[i][2], og = a4[i][3];
        const float tc = ftanh(cn[i]);
        const float dc = dcreg[i] + dh * og * (1.0f - tc * tc);
        dzv[0] = dc * jg * ig * (1.0f - ig);
        dzv[1] = dc * ig * (1.0f - jg * jg);
        dzv[2] = dc * cpv[i] * fg * (1.0f - fg);
        dzv[3] = dh * tc * og * (1.0f - og);
        dcreg[i] = dc * fg;
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) dzv[g] = 0.f;
      }
      cn[i] = cpv[i];
#pragma unroll
      for (int g = 0; g < 4; ++g) bacc[g] += dzv[g];
      const int sb = swz<256>(row0 + i, ul);  // = swz(row, g * 64 + ul) - g * 64
#pragma unroll
      for (int g = 0; g < 4; ++g) Ash[sb + g * 64] = f2bf(dzv[g]);
    }
    if constexpr (STAMP) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (stamp after the LDS writes)
    stamp(2);
    if (s == 0) {
      store_dz(0);
      break;
    }
    __syncthreads();  // dz slice complete in LDS (and every lane has read Pown)
    stamp(3);
    // ---- partial dh over this slice's gate columns, output units 32 wid .. +31, all 32 rows
    f32x4 acc[2][2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[rt][t] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const bf16x8 w1 = Wl[(wid * KS + kk) * 64 + lane];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&Ash[swz<256>(rt * 16 + (lane & 15), kk * 32 + 8 * (lane >> 4))]);
        acc[rt][0] = mfma16(a, Wr[kk], acc[rt][0]);
        acc[rt][1] = mfma16(a, w1, acc[rt][1]);
      }
    }
    if constexpr (STAMP) {  // (stamp once the accumulators are final)
      float sink = acc[0][0][0] + acc[1][1][3];
      asm volatile("" : "+v"(sink));
    }
    stamp(4);
    // ---- publish: units 32 wid .. +31 are units (wid & 1) * 32 .. +31 of slice wid / 2
    const int dw = wid >> 1, ub = (wid & 1) * 32 + (lane & 15);
    if (dw == c) {
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) Pown[(rt * 16 + (lane >> 4) * 4 + r) * 64 + ub + 16 * t] = acc[rt][t][r];
    } else {
      gu64* dst = xb + (size_t)(s & 1) * NC * NC * SLOT + ((size_t)dw * NC + c) * SLOT;
      unsigned lo = (unsigned)((lane >> 4) * 4 * 64 + ub) * 8u;
      asm volatile("" : "+v"(lo));
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            store_granule(gboff(dst, lo + (unsigned)((rt * 16 + r) * 64 + 16 * t) * 8u), (unsigned)(T - s),
                          __float_as_uint(acc[rt][t][r]));
    }
    stamp(5);
    store_dz(s);
    __syncthreads();  // Pown visible before the next step reads it; Ash free for rewriting
    stamp(6);
  }
  if constexpr (STAMP) {
    if (threadIdx.x == 0 && lb_stamps) {
#pragma unroll
      for (int ph = 0; ph < 8; ++ph) lb_stamps[((size_t)team * NC + c) * 8 + ph] = st_sum[ph];
    }
  }
#pragma unroll
  for (int i = 0; i < RPL; ++i)
    if (rok[i]) dc_carry[(size_t)d * BH + (size_t)rc[i] * H + u] = dcreg[i];
  if (dbias) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float t = sum_x32(sum_x16(bacc[g]));  // lanes l, l^16, l^32, l^48: the wave's 4 row pairs
      if ((lane >> 4) == 0) atomicAdd(dbias + (size_t)d * G4 + g * H + u, t);
    }
  }
}

// ---------------------------------------------------------------------- launchers
// Kernel variants (measured, tools/lstm_micro.py): the forward runs 4 waves per workgroup
// (16 units per wave) up to H = 256 and 8 waves (8 units per wave) at H = 512, where the
// 4-wave forward would need 256 VGPRs of W_hh per lane; the backward runs 8 waves (2 rows
// per lane in the cell update) at every H -- 4.0 vs 4.6 us per step for 4 waves at H = 256,
// B = 256.  Activation traffic is non-temporal in the forward (H = 512, B = 256: 7.06 -> 6.83
// us per step; H = 256: 3.14 -> 3.00) and cached in the BPTT (its NT variant spills: 8.22 ->
// 8.41).
static int lstm_nw(int H) { return H == 512 ? 8 : 4; }  // forward waves per workgroup

static bool lstm_h_ok(int H) { return H == 64 || H == 128 || H == 256 || H == 512; }

// Workgroups of the persistent kernels the current device keeps resident at once: one per
// CU (launch bounds (64 NW, 1); the occupancy query must admit at least that for every
// variant), times the CU count the runtime reports -- not an assumed 256, so a partitioned
// or smaller device shrinks the admissible grid instead of spinning into the hand-off timeout.
int lstm_persistent_capacity(int H) {
  static int cache[64][4] = {};  // [device][log2(H/64)] -> capacity + 1
  int dev = 0;
  if (!lstm_h_ok(H) || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  const int hi = H == 64 ? 0 : H == 128 ? 1 : H == 256 ? 2 : 3;
  if (cache[dev][hi]) return cache[dev][hi] - 1;
  int cus = 0, o[4] = {1, 1, 1, 1};
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
  bool ok = true;
#define OCC(HH)                                                                                                    \
  if (H == HH) {                                                                                                   \
    ok &= hipOccupancyMaxActiveBlocksPerMultiprocessor(&o[0], lstm_bwd_persistent_kernel<HH, 8, false>, 512, 0) == hipSuccess; \
    ok &= hipOccupancyMaxActiveBlocksPerMultiprocessor(&o[1], lstm_fwd_persistent8_kernel<HH, true>, 512, 0) == hipSuccess; \
    if (HH <= 256) {                                                                                               \
      ok &= hipOccupancyMaxActiveBlocksPerMultiprocessor(&o[3], lstm_fwd_persistent_kernel<(HH <= 256 ? HH : 256), true>, \
                                                         256, 0) == hipSuccess;                                    \
      int ofx = 0;                                                                                                 \
      ok &= hipOccupancyMaxActiveBlocksPerMultiprocessor(                                                          \
                &ofx, lstm_fwd_persistent_kernel<(HH <= 256 ? HH : 256), true, 1, true>, 256, 0) == hipSuccess;    \
      o[3] = min(o[3], ofx);                                                                                       \
    } else {                                                                                                       \
      ok &= hipOccupancyMaxActiveBlocksPerMultiprocessor(&o[2], lstm_fwd_persistent_kernel<512, true, 2>, 256, 0) == hipSuccess; \
      int ofx = 0;                                                                                                 \
      ok &= hipOccupancyMaxActiveBlocksPerMultiprocessor(&ofx, lstm_fwd_persistent_kernel<512, true, 2, true>, 256, 0) == hipSuccess; \
      o[2] = min(o[2], ofx);                                                                                       \
      int o32 = 0;                                                                                                 \
      ok &= hipOccupancyMaxActiveBlocksPerMultiprocessor(&o32, lstm_bwd_persistent32_kernel<false>, 1024, 0) == hipSuccess; \
      o[2] = min(o[2], o32);                                                                                      \
    }                                                                                                              \
  }
  OCC(64) OCC(128) OCC(256) OCC(512)
#undef OCC
  const int cap = (ok && o[0] >= 1 && o[1] >= 1 && o[2] >= 1 && o[3] >= 1) ? cus : 0;
  cache[dev][hi] = cap + 1;
  return cap;
}

// Rows per team: 16, or 32 for the H = 512 forward above batch 256 (the 4-wave RT = 2 kernel:
// batch 1024 in 2 launches instead of 4; tools/lstm_micro.py, T = 800: B = 1024 19.1 -> 12.7 ms,
// B = 512 9.7 -> 6.4 ms per launch sequence, 7.9 us per step vs 6.0 for 16-row teams).  The
// backward keeps 16: a 32-row BPTT (4 waves with two output slices each, 256 registers of W_hh,
// inputs staged through LDS) still spilled ~40 registers and ran 36 us per step against 7.6 --
// B = 1024: 29.1 vs 24.4 ms.
// The backward runs 32-row teams at H = 512 above batch 256 too, with the 16-wave kernel
// (lstm_bwd_persistent32_kernel; TSAMD_LSTM_BWD32=0 restores the 16-row BPTT).
static bool lstm_bwd32() {
  static const int on = [] {
    const char* e = getenv("TSAMD_LSTM_BWD32");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return on;
}
static int lstm_rows(int H, int B, bool bwd) {
  return (H == 512 && B > 256 && (!bwd || lstm_bwd32())) ? 32 : 16;
}

// Row tiles per launch: the most whose grid (NC workgroups per (direction, tile) team,
// teams dealt 8 at a time so members share an XCD) fits the resident capacity.  Teams are
// independent, so a larger batch runs as consecutive launches over row-tile ranges.
static int lstm_tiles_per_launch(int H, int ntile) {
  const int NC = H / 64, cap = lstm_persistent_capacity(H);
  int nl = ntile;
  while (nl > 0 && 8 * NC * ((2 * nl + 7) / 8) > cap) --nl;
  return nl;
}

int lstm_persistent_grid(int H, int B) {
  if (!lstm_h_ok(H) || B < 1) return 0;
  int grid = 0;
  for (int bwd = 0; bwd < 2; ++bwd) {
    const int R = lstm_rows(H, B, bwd), NC = H / 64, nl = lstm_tiles_per_launch(H, (B + R - 1) / R);
    if (nl <= 0) return 0;
    grid = max(grid, 8 * NC * ((2 * nl + 7) / 8));  // grid of the largest launch
  }
  return grid;
}

int lstm_persistent_launches(int H, int B) {
  int n = 0;
  for (int bwd = 0; bwd < 2; ++bwd) {
    const int R = lstm_rows(H, B, bwd), ntile = (B + R - 1) / R, nl = lstm_tiles_per_launch(H, ntile);
    if (nl <= 0) return 0;
    n = max(n, (ntile + nl - 1) / nl);
  }
  return n;
}

size_t lstm_persistent_xbuf_elems(int H, int B, bool bwd) {
  const int R = lstm_rows(H, B, bwd), ntile = (B + R - 1) / R, NC = H / 64;
  // fwd: [team][parity][R rows][H/2 unit pairs]; bwd: [team][parity][dest][src][R][64]
  return (size_t)2 * ntile * 2 * (bwd ? (size_t)NC * NC * R * 64 : (size_t)R * (H / 2));
}

// FX (the input projection inside the recurrence, E = 128): the 4-wave kernels only -- the
// 8-wave H = 512 kernel (batch <= 256) has no registers or LDS left for W_x
bool lstm_persistent_fx_ok(int H, int B, int E) {
  return E == 128 && lstm_persistent_grid(H, B) > 0 && (lstm_rows(H, B, false) == 32 || lstm_nw(H) == 4);
}

void launch_lstm_fwd_persistent(const float* gx, const float* bias, const bf16* Wt, bf16* hs, float* cs, float* acts,
                                bf16* out, const int* lens, unsigned long long* xbuf, unsigned* err, int T, int B,
                                int H, hipStream_t st, const bf16* xsf, const bf16* Wx0, const bf16* Wx1) {
  const int R = lstm_rows(H, B, false), ntile = (B + R - 1) / R, nl = lstm_tiles_per_launch(H, ntile), NC = H / 64;
  const int nw = R == 32 ? 4 : lstm_nw(H);
  if (nl <= 0) return;
  const bool fx = xsf != nullptr;
  if (fx && nw != 4) return;  // the binding checks lstm_persistent_fx_ok first
  gu64* xb = (gu64*)xbuf;
  gu32* e = (gu32*)err;
  for (int t0 = 0; t0 < ntile; t0 += nl) {
    const int n = min(nl, ntile - t0), grid = 8 * NC * ((2 * n + 7) / 8);
#define ARGS gx, bias, Wt, hs, cs, acts, out, lens, xb, e, T, B, ntile, t0, n, xsf, Wx0, Wx1
#define LAUNCH_F(HH, NTV)                                                                                            \
  if (fx && R == 32)                                                                                            \
    hipLaunchKernelGGL((lstm_fwd_persistent_kernel<512, NTV, 2, true>), dim3(grid), dim3(256), 0, st, ARGS);    \
  else if (fx)                                                                                                  \
    hipLaunchKernelGGL((lstm_fwd_persistent_kernel<(HH <= 256 ? HH : 256), NTV, 1, true>), dim3(grid), dim3(256), \
                       0, st, ARGS);                                                                            \
  else if (nw == 8)                                                                                             \
    hipLaunchKernelGGL((lstm_fwd_persistent8_kernel<HH, NTV>), dim3(grid), dim3(512), 0, st, gx, bias, Wt, hs, cs, \
                       acts, out, lens, xb, e, T, B, ntile, t0, n);                                             \
  else if (R == 32)                                                                                             \
    hipLaunchKernelGGL((lstm_fwd_persistent_kernel<512, NTV, 2>), dim3(grid), dim3(256), 0, st, ARGS);          \
  else                                                                                                          \
    hipLaunchKernelGGL((lstm_fwd_persistent_kernel<(HH <= 256 ? HH : 256), NTV>), dim3(grid), dim3(256), 0, st, ARGS)
    if (H == 64) LAUNCH_F(64, true);
    else if (H == 128) LAUNCH_F(128, true);
    else if (H == 256) LAUNCH_F(256, true);
    else LAUNCH_F(512, true);
#undef LAUNCH_F
#undef ARGS
  }
}

void launch_lstm_bwd_persistent(bf16* dz, const bf16* Wn, const float* dout, const float* dh_fin, float* dc_carry,
                                const float* acts, const float* cs, const int* lens, unsigned long long* xbuf,
                                unsigned* err, float* dbias, int T, int B, int H, bool dout_bf, hipStream_t st,
                                bool dout_bf16) {
  const int R = lstm_rows(H, B, true), ntile = (B + R - 1) / R, nl = lstm_tiles_per_launch(H, ntile), NC = H / 64;
  if (nl <= 0) return;
  gu64* xb = (gu64*)xbuf;
  gu32* e = (gu32*)err;
  for (int t0 = 0; t0 < ntile; t0 += nl) {
    const int n = min(nl, ntile - t0), grid = 8 * NC * ((2 * n + 7) / 8);
    if (R == 32) {
#define LB32(PC, SL, DB, STP) hipLaunchKernelGGL((lstm_bwd_persistent32_kernel<false, PC, SL, DB, STP>), dim3(grid), \
                                                 dim3(1024), 0, st, dz, Wn, dout, dh_fin, dc_carry, acts, cs, lens, xb, e, \
                                                 dbias, T, B, ntile, t0, n)
      // poll 2 peers per pass, s_sleep(96): profiles/r4/ab/bptt32.md
      const int dbf = dout_bf ? (dout_bf16 ? 2 : 1) : 0;
      if (lb_stamps_on) {
        if (dbf == 2) LB32(2, 96, 2, true);
        else if (dbf == 1) LB32(2, 96, 1, true);
        else LB32(2, 96, 0, true);
      } else if (dbf == 2) LB32(2, 96, 2, false);
      else if (dbf == 1) LB32(2, 96, 1, false);
      else LB32(2, 96, 0, false);
#undef LB32
      continue;
    }
#define LB16(HH, NTV, DB) hipLaunchKernelGGL((lstm_bwd_persistent_kernel<HH, 8, NTV, DB>), dim3(grid), dim3(512), 0, st, \
                                           dz, Wn, dout, dh_fin, dc_carry, acts, cs, lens, xb, e, dbias, T, B, ntile, t0, n)
#define LAUNCH_B(HH, NTV)                          \
  if (dout_bf && dout_bf16) LB16(HH, NTV, 2);      \
  else if (dout_bf) LB16(HH, NTV, 1);              \
  else LB16(HH, NTV, 0)
    if (H == 64) LAUNCH_B(64, false);
    else if (H == 128) LAUNCH_B(128, false);
    else if (H == 256) LAUNCH_B(256, false);
    else LAUNCH_B(512, false);
#undef LAUNCH_B
#undef LB16
  }
}
