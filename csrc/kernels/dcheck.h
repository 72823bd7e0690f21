// Bounds checks of data-dependent indices (token ids, sequence lengths, beam back-pointers)
// for the debug build of the kernel library (_C_debug.so: -DTSAMD_DEBUG, relocatable device
// code; `python -m textsummarization_on_flink_amd._build --debug`, selected at load time by
// TSAMD_KERNEL_DEBUG=1).  A failed check records (check id, block, thread, offending value) in
// one device word block -- the first failure wins -- and the kernel carries on with the index
// clamped into range, so a debug run reports the bad input (ops.debug_check()) instead of
// faulting the GPU.  The release build compiles every check away (DCHECK_IDX(x, ...) is x).
#pragma once

// check ids (textsummarization_on_flink_amd/ops/__init__.py DEBUG_CHECKS names them)
#define CHK_FRAME_ID 1     // to_step_frame: gathered row id in [0, table rows)
#define CHK_FRAME_REV 2    // to_step_frame / from_step_frame: reversal index in [0, T)
#define CHK_EMB_ID 3       // embedding gradient: token id in [0, V)
#define CHK_ATTN_LEN 4     // attention kernels: encoder length in [1, T]
#define CHK_LOSS_LEN 5     // pointer loss / row finalise: encoder length in [0, T]
#define CHK_BEAM_PARENT 6  // beam gather: parent row in [0, R)
#define CHK_BEAM_TOKEN 7   // beam gather: latest token id >= 0

#ifdef TSAMD_DEBUG
extern __device__ unsigned tsamd_dbg[4];

__device__ __forceinline__ long dcheck_idx(long x, long lo, long hi, unsigned id) {
  if (x < lo || x >= hi) {
    if (atomicCAS(&tsamd_dbg[0], 0u, id) == 0u) {
      tsamd_dbg[1] = blockIdx.x;
      tsamd_dbg[2] = threadIdx.x;
      tsamd_dbg[3] = (unsigned)x;
    }
    x = x < lo ? lo : hi - 1;
  }
  return x;
}
#define DCHECK_IDX(x, lo, hi, id) dcheck_idx((x), (lo), (hi), (id))
#define DCHECK_IN(x, lo, hi, id) ((void)dcheck_idx((x), (lo), (hi), (id)))  // record only
#else
#define DCHECK_IDX(x, lo, hi, id) (x)
#define DCHECK_IN(x, lo, hi, id) ((void)0)
#endif
