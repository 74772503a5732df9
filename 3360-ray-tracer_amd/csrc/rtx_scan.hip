// rtx_scan.hip — see rtx_scan.h.
#include "rtx_scan.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

namespace rtxscan {

size_t temp_bytes(int64_t n) {
  size_t bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)n,
                                rocprim::plus<uint32_t>());
  return bytes;
}

hipError_t exclusive_scan_u32(const uint32_t* in, uint32_t* out, int64_t n, void* tmp, size_t tmp_bytes,
                              hipStream_t s) {
  if (n <= 0) return hipSuccess;
  return rocprim::exclusive_scan(tmp, tmp_bytes, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(), s);
}

size_t sort_temp_bytes(int64_t n) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n);
  return bytes;
}

hipError_t sort_pairs_u32(const uint32_t* keys, uint32_t* keys_out, const uint32_t* vals, uint32_t* vals_out,
                          int64_t n, void* tmp, size_t tmp_bytes, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  return rocprim::radix_sort_pairs(tmp, tmp_bytes, keys, keys_out, vals, vals_out, (size_t)n, 0u,
                                   8u * (unsigned)sizeof(uint32_t), s);
}

}  // namespace rtxscan
