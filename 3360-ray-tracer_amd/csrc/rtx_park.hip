// PARK instantiations of the persistent kernel (k_persistent<STACK, true, COUNT, SCATTER,
// PARK = 1 or 2>), compiled apart from rtx_capi.hip so this translation unit can have its own
// per-TU choices (RTX_PARK_TU: see the top of rtx_device.h) and scheduler options (Makefile
// PARKFLAGS).  k_persistent refuses to be instantiated with PARK > 0 anywhere else.
#define RTX_PARK_TU 1
#include <hip/hip_runtime.h>

#include "rtx.h"
#include "rtx_kernels.h"

namespace rtxd {
#define RTX_PARK_DEFINE(ST, CO, SC, MP, PK)                                                                     \
  template __global__ void k_persistent<ST, true, CO, SC, PK, -1, false, false, false, MP>(RenderArgs,          \
                                                                                          unsigned long long*);
RTX_PARK_INSTANCES(RTX_PARK_DEFINE)
#undef RTX_PARK_DEFINE
#define RTX_PARK_TRI_DEFINE(ST, MP, PK)                                                                              \
  template __global__ void k_persistent<ST, true, false, false, PK, RTX_PRIM_TRIANGLE, false, false, false, MP>(    \
      RenderArgs, unsigned long long*);                                                                              \
  template __global__ void k_persistent<ST, true, false, false, PK, RTX_PRIM_TRIANGLE, true, false, false, MP>(     \
      RenderArgs, unsigned long long*);                                                                              \
  template __global__ void k_persistent<ST, true, false, false, PK, RTX_PRIM_TRIANGLE, true, true, false, MP>(      \
      RenderArgs, unsigned long long*);
RTX_PARK_TRI_INSTANCES(RTX_PARK_TRI_DEFINE)
#undef RTX_PARK_TRI_DEFINE
}  // namespace rtxd
