// rtx_scan.hip — see rtx_scan.h.
#include "rtx_scan.h"

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

}  // namespace rtxscan
