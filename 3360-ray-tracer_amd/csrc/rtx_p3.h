// rtx_p3.h — device-side P3 PPM encoding (SURVEY §8f "on-GPU resolve + PPM output").
//
// The reference writes its image as ASCII P3 text, one `write_color` line per pixel
// (core/color.h:18-33, wavefront.cc:238-241): gamma = sqrt for x > 0 else 0, clamp to
// [0, 0.999], int(256 x), then "r g b\n".  At 4K that is 8.3M formatted lines on one CPU
// thread.  Here the bytes are produced on the GPU: one pass packs the three byte values and
// the line length per pixel, a device-wide exclusive scan (rocPRIM) turns lengths into
// offsets, and one pass writes every line at its offset.  HBM-bound: 24 B read + 4 B packed
// + 4 B offset + <= 12 B text per pixel.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace rtxp3 {

constexpr size_t kMaxLine = 12;  // "255 255 255\n"

// Scratch needed for npix pixels: packed values, offsets, scan temporaries, total length.
size_t scratch_bytes(int64_t npix);

// Encodes the P3 body (no header) of d_rgb (npix x 3 doubles, linear) into d_body, which must
// hold npix * kMaxLine bytes; d_scratch: scratch_bytes(npix) bytes.  Enqueues on `s`, then
// waits for the body length and returns it in *len.
hipError_t encode_body(const double* d_rgb, int64_t npix, void* d_scratch, char* d_body, size_t* len,
                       hipStream_t s);

}  // namespace rtxp3
