// Host access to the debug build's check record (dcheck.h).  In the release build the
// record does not exist: tsamd_debug_enabled() is 0 and the status reads as all zeros.
#include <hip/hip_runtime.h>
#include <string.h>

#include "dcheck.h"

#ifdef TSAMD_DEBUG
__device__ unsigned tsamd_dbg[4];

int tsamd_debug_enabled() { return 1; }

void tsamd_debug_read(unsigned* out4) {
  if (hipMemcpyFromSymbol(out4, HIP_SYMBOL(tsamd_dbg), 4 * sizeof(unsigned), 0, hipMemcpyDeviceToHost) != hipSuccess)
    memset(out4, 0xff, 4 * sizeof(unsigned));
}

void tsamd_debug_clear() {
  const unsigned z[4] = {0, 0, 0, 0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(tsamd_dbg), z, sizeof(z), 0, hipMemcpyHostToDevice);
}
#else
int tsamd_debug_enabled() { return 0; }
void tsamd_debug_read(unsigned* out4) { memset(out4, 0, 4 * sizeof(unsigned)); }
void tsamd_debug_clear() {}
#endif
