// rt/image.h — image decode behind Image::Load (the reference's scene/image.cc:16-73 reads
// textures with stb_image's stbi_loadf): 8-bit decode of JPEG (sequential / progressive) and
// binary PNM, then stb's gamma-2.2 float conversion and Image::FloatToByte.  See
// host/src/image_decode.cc for what is restated from stb_image v2.30 and how it is pinned.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace rt::scene {

// 8-bit RGB (3 bytes per pixel, rows top-down) as stbi_load(..., 3) returns it.
bool DecodeJpeg(const uint8_t* data, size_t n, int& width, int& height, std::vector<uint8_t>& rgb,
                std::string& err);
bool DecodeImage8(const std::vector<uint8_t>& file, int& width, int& height, std::vector<uint8_t>& rgb,
                  std::string& err);
// The texel byte an 8-bit sample becomes: FloatToByte((float)(pow(b / 255.0f, 2.2f))).
uint8_t TexelFromByte(uint8_t b);
// File -> texels (linear8: the 8-bit decode itself, without the gamma / FloatToByte step).
bool LoadTexels(const std::string& path, int& width, int& height, std::vector<uint8_t>& texels, std::string& err,
                bool linear8 = false);

}  // namespace rt::scene
