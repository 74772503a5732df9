// rtx_p3.hip — device-side P3 PPM encoding; see rtx_p3.h.
#include "rtx_p3.h"

#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

namespace rtxp3 {
namespace {

constexpr int kBlock = 256;

// write_color (core/color.h:10-33) for one channel
__device__ __forceinline__ uint32_t channel_byte(double x) {
  x = x > 0 ? sqrt(x) : 0.0;                  // linear_to_gamma (NaN -> 0)
  x = x < 0.0 ? 0.0 : (x > 0.999 ? 0.999 : x);  // Interval(0, 0.999).Clamp
  return (uint32_t)(int)(256 * x);
}
__device__ __forceinline__ uint32_t digits(uint32_t v) { return 1u + (v >= 10u) + (v >= 100u); }

// packed = r | g << 8 | b << 16 | line length << 24
__global__ __launch_bounds__(kBlock) void k_p3_pack(const double* __restrict__ rgb, int64_t n,
                                                    uint32_t* __restrict__ packed) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = channel_byte(rgb[3 * i]), g = channel_byte(rgb[3 * i + 1]), b = channel_byte(rgb[3 * i + 2]);
  const uint32_t len = digits(r) + digits(g) + digits(b) + 3u;
  packed[i] = r | (g << 8) | (b << 16) | (len << 24);
}

struct LineLength {
  __device__ __host__ uint32_t operator()(uint32_t p) const { return p >> 24; }
};

__device__ __forceinline__ char* put(char* o, uint32_t v) {
  if (v >= 100u) *o++ = (char)('0' + v / 100u);
  if (v >= 10u) *o++ = (char)('0' + (v / 10u) % 10u);
  *o++ = (char)('0' + v % 10u);
  return o;
}

__global__ __launch_bounds__(kBlock) void k_p3_write(const uint32_t* __restrict__ packed,
                                                     const uint32_t* __restrict__ off, int64_t n,
                                                     char* __restrict__ body, unsigned long long* total) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = packed[i];
  char* o = body + off[i];
  o = put(o, p & 0xffu);
  *o++ = ' ';
  o = put(o, (p >> 8) & 0xffu);
  *o++ = ' ';
  o = put(o, (p >> 16) & 0xffu);
  *o = '\n';
  if (i == n - 1) *total = (unsigned long long)off[i] + (p >> 24);
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t scan_temp(int64_t n) {
  size_t bytes = 0;
  auto in = rocprim::make_transform_iterator((const uint32_t*)nullptr, LineLength());
  (void)rocprim::exclusive_scan(nullptr, bytes, in, (uint32_t*)nullptr, 0u, (size_t)n, rocprim::plus<uint32_t>());
  return bytes;
}

}  // namespace

size_t scratch_bytes(int64_t n) {
  return align256(n * sizeof(uint32_t)) * 2 + align256(scan_temp(n)) + 256;
}

hipError_t encode_body(const double* d_rgb, int64_t n, void* d_scratch, char* d_body, size_t* len, hipStream_t s) {
  *len = 0;
  if (n <= 0) return hipSuccess;
  char* base = (char*)d_scratch;
  uint32_t* packed = (uint32_t*)base;
  uint32_t* off = (uint32_t*)(base + align256(n * sizeof(uint32_t)));
  void* tmp = base + 2 * align256(n * sizeof(uint32_t));
  size_t tmp_bytes = scan_temp(n);
  unsigned long long* total = (unsigned long long*)((char*)tmp + align256(tmp_bytes));
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_p3_pack, dim3(grid), dim3(kBlock), 0, s, d_rgb, n, packed);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  auto in = rocprim::make_transform_iterator((const uint32_t*)packed, LineLength());
  e = rocprim::exclusive_scan(tmp, tmp_bytes, in, off, 0u, (size_t)n, rocprim::plus<uint32_t>(), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_p3_write, dim3(grid), dim3(kBlock), 0, s, packed, off, n, d_body, total);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  unsigned long long h = 0;
  if ((e = hipMemcpyAsync(&h, total, sizeof h, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  *len = (size_t)h;
  return hipSuccess;
}

}  // namespace rtxp3
