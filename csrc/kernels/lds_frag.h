// LDS-DMA staging and transposed-read fragments shared by the split-K weight-gradient GEMM
// (wgrad.hip) and the batched attention-context GEMMs (ctx_bmm.hip).
//
// Half image: 64 (or more) rows of 256 bytes (128 bf16 columns), the 16-byte chunk ch of row r at
// ch ^ tt_sw(r) (cdna_hip_programming.md T10 (b)): the two 4-row blocks a 32-lane half reads, 8
// rows apart in the same columns, hit distinct banks.  The XOR is applied to the per-lane GLOBAL
// source address, so the LDS-DMA image stays lane-linear.
#pragma once
#include "common.h"

namespace {
typedef __attribute__((address_space(3))) void* tt_lds_t;
typedef const __attribute__((address_space(1))) void* tt_gbl_t;

__device__ __forceinline__ int tt_sw(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// global_load_lds_dwordx4 hidden from hipcc's wait bookkeeping (cdna_hip_programming.md s5.7):
// with the builtin, hipcc cannot tell the in-flight DMA of the NEXT stage from the one being read
// and waits vmcnt(0) before the first ds_read of every K step -- the staging then never overlaps
// the MFMAs.  The kernel counts these loads itself (vmcnt(0) + barrier at the end of the step).
__device__ __forceinline__ void glds16_asm(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

// one operand fragment (16 columns c0.. of a half image, k rows kb + 8 (l >> 4) .. + 7) by two
// transposed reads: lane 4q + p of each 16-lane group addresses row (.. + 4 half + q), columns
// c0 + 4 p .. + 3
__device__ __forceinline__ bf16x8 tt_frag(const char* img, int kb, int c0, int lane) {
  typedef short v4i16 __attribute__((ext_vector_type(4)));
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const int q = (lane >> 2) & 3, p = lane & 3, g = lane >> 4;
  v4i16 h[2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const int r = kb + 8 * g + 4 * hf + q, ch = (c0 >> 3) + (p >> 1);
    const char* a = img + r * 256 + 16 * (ch ^ tt_sw(r)) + 8 * (p & 1);
    h[hf] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(const_cast<char*>(a)));
  }
  return __builtin_bit_cast(bf16x8, v8i16{h[0][0], h[0][1], h[0][2], h[0][3], h[1][0], h[1][1], h[1][2], h[1][3]});
}
}  // namespace
