// rtx_scan.hip — see rtx_scan.h.
#include "rtx_scan.h"

#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

namespace rtxscan {

namespace {
struct Pack {
  __host__ __device__ uint64_t operator()(uint32_t k) const { return ((uint64_t)k << 32) | (uint64_t)(k != 0u); }
};
}  // namespace

size_t temp_bytes_packed(int64_t n) {
  size_t bytes = 0;
  auto it = rocprim::make_transform_iterator((const uint32_t*)nullptr, Pack());
  (void)rocprim::exclusive_scan(nullptr, bytes, it, (uint64_t*)nullptr, (uint64_t)0, (size_t)n,
                                rocprim::plus<uint64_t>());
  return bytes;
}

hipError_t exclusive_scan_packed(const uint32_t* k, uint64_t* out, int64_t n, void* tmp, size_t tmp_bytes,
                                 hipStream_t s) {
  if (n <= 0) return hipSuccess;
  auto it = rocprim::make_transform_iterator(k, Pack());
  return rocprim::exclusive_scan(tmp, tmp_bytes, it, out, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), s);
}

}  // namespace rtxscan
