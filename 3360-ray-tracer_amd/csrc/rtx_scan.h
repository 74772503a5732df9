// rtx_scan.h — device-wide primitives (rocPRIM) for the adaptive sampler: the exclusive prefix
// sum of the slot layout (rtx_kernels.h k_adapt_expand, k_tile_compact) and the radix sort of
// the tile schedule's claim order (k_tile_keys).
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

// Temporary storage sort_pairs_u32 needs for n pairs.
size_t sort_temp_bytes(int64_t n);

// (keys, vals) sorted by key, ascending (stable), into (keys_out, vals_out); enqueued on s.
hipError_t sort_pairs_u32(const uint32_t* keys, uint32_t* keys_out, const uint32_t* vals, uint32_t* vals_out,
                          int64_t n, void* tmp, size_t tmp_bytes, hipStream_t s);

}  // namespace rtxscan
