// rtx_scan.h — the device-wide exclusive prefix sum (rocPRIM) of the adaptive sampler's slot
// layout and pixel lists (rtx_frame_kernels.h k_adapt_expand).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace rtxscan {

// The adaptive phases' packed scan: out[i] = sum over j < i of (k[j] << 32 | (k[j] != 0)), i.e. the
// high word the slot offset of entry i, the low word its index among the nonzero entries
// (the sums stay below 2^32: the host bounds a phase's slots).  temp_bytes_packed(n) of tmp.
size_t temp_bytes_packed(int64_t n);
hipError_t exclusive_scan_packed(const uint32_t* k, uint64_t* out, int64_t n, void* tmp, size_t tmp_bytes,
                                 hipStream_t s);

}  // namespace rtxscan
