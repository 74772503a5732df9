// rtx_scan.h — the device-wide exclusive prefix sum (rocPRIM) of the adaptive sampler's slot
// layout (rtx_frame_kernels.h k_adapt_expand).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace rtxscan {

// Temporary storage exclusive_scan_u32 needs for n elements.
size_t temp_bytes(int64_t n);

// out[i] = in[0] + ... + in[i - 1] (out[0] = 0), enqueued on s; tmp holds temp_bytes(n).
hipError_t exclusive_scan_u32(const uint32_t* in, uint32_t* out, int64_t n, void* tmp, size_t tmp_bytes,
                              hipStream_t s);

}  // namespace rtxscan
