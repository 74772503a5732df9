// PARK instantiations of the persistent kernel (k_persistent<STACK, true, COUNT, SCATTER,
// PARK = 1 or 2>), compiled apart from rtx_capi.hip so this translation unit can have its own macro
// defaults (below) and scheduler options (see the Makefile and rtx_kernels.h).
#define RTX_PERSISTENT_ONLY 1
// the library cos()/sin() here: with the small-argument form the bunny's triangle-tree
// Lambertian build spills (0 -> 56 B per lane), see rtx_device.h
#ifndef RTX_SINCOS_SMALL
#define RTX_SINCOS_SMALL 0
#endif
// ... and the triangle test without early exits (bunny +3.8 %; the plain kernel's builds are
// slower with it)
#ifndef RTX_TRI_BRANCHLESS
#define RTX_TRI_BRANCHLESS 1
#endif
// ... and the leaf tests spread over the walk's iterations, one per lane and iteration
// (trace4_run_step: bunny +2.8 %; the plain kernel's sphere-tree builds are slower with it)
#ifndef RTX_LEAF_STEP
#define RTX_LEAF_STEP 1
#endif
// ... and the texture lookup where the reference does it: the early lookup makes the generic
// (textured) PARK build spill more (80 -> 128 B per lane)
#ifndef RTX_EARLY_TEX
#define RTX_EARLY_TEX 0
#endif
// ... and 512 slots per uniform-group chunk (bunny C3 +0.7 %; the plain kernel's C2 -0.4 % with
// it, profiles/r04/ab_chunk_map0_r6e_*.txt)
#ifndef RTX_CHUNK
#define RTX_CHUNK 512
#endif
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
