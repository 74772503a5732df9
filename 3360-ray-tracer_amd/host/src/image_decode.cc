// image_decode.cc — the image decode behind the reference's Image::Load (scene/image.cc:16-73),
// which reads textures through stb_image v2.30's stbi_loadf (vendored in the reference at
// src/third-party/stb/stb_image.h): 8-bit decode, then stbi__ldr_to_hdr (gamma 2.2) and
// Image::FloatToByte.  Formats: JPEG (baseline / extended sequential Huffman and progressive,
// 8-bit, 1/3/4 components with stb's colour handling) and binary PNM (P5 / P6, maxval <= 255).
//
// The pixels must be the bytes stb produces, so the arithmetic follows stb's published
// algorithm, restated here: canonical Huffman decoding with stb's end-of-data behaviour (zero
// bits after a marker), coefficients dequantised into 16-bit `short` (stb_image.h:2210-2262),
// the jidctint-derived integer IDCT with stb's 12-bit constants and rounding
// (stb_image.h:2426-2524; the SSE2 kernel the x86-64 reference runs is documented there as
// bit-identical to it), stb's "fancy" upsampling for 2x1 / 1x2 / 2x2 chroma and nearest
// neighbour otherwise (stb_image.h:3465-3657), and the reduced-precision fixed-point
// YCbCr -> RGB of stbi__YCbCr_to_RGB_row (stb_image.h:3659-3683; the SIMD kernel only covers
// 4-channel output, the reference asks for 3).  Pinned by tests/test_image_decode.py against
// the reference's own stb decode of generated JPEG / PNM fixtures and of earthmap.jpg.
#include <algorithm>
#include <cctype>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "rt/image.h"

namespace rt::scene {

namespace {

// ---- entropy-coded data ---------------------------------------------------------------
constexpr int kNoMarker = 0xff;

const uint8_t kDezigzag[64 + 15] = {  // zigzag position -> natural index; corrupt input lands on 63
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct Huffman {
  uint8_t values[256] = {};
  uint8_t size[257] = {};
  uint16_t code[256] = {};
  uint32_t maxcode[18] = {};  // largest code + 1 per length, left-aligned to 16 bits
  int delta[17] = {};         // symbol index = code + delta[length]
  int count = 0;
  bool build(const int lengths[16]) {
    int k = 0;
    for (int i = 0; i < 16; i++)
      for (int j = 0; j < lengths[i]; j++) {
        if (k >= 256) return false;
        size[k++] = (uint8_t)(i + 1);
      }
    size[k] = 0;
    count = k;
    uint32_t c = 0;
    k = 0;
    int j;
    for (j = 1; j <= 16; j++) {
      delta[j] = k - (int)c;
      if (size[k] == j) {
        while (size[k] == j) code[k++] = (uint16_t)(c++);
        if (c - 1 >= (1u << j)) return false;  // code lengths over-subscribed
      }
      maxcode[j] = c << (16 - j);
      c <<= 1;
    }
    maxcode[j] = 0xffffffffu;
    return true;
  }
};

struct Component {
  int id = 0, h = 1, v = 1, tq = 0, hd = 0, ha = 0;
  int dc_pred = 0;
  int x = 0, y = 0, w2 = 0, h2 = 0;  // effective size; padded plane size
  std::vector<uint8_t> data;          // w2 x h2 samples
  std::vector<int16_t> coeff;         // progressive: w2/8 x h2/8 blocks of 64
  int coeff_w = 0;
};

class Jpeg {
 public:
  Jpeg(const uint8_t* p, size_t n) : p_(p), end_(p + n) {}
  bool decode(int& w, int& h, std::vector<uint8_t>& rgb, std::string& err);

 private:
  const uint8_t* p_;
  const uint8_t* end_;
  std::string err_;
  bool fail(const char* m) {
    if (err_.empty()) err_ = m;
    return false;
  }
  // byte source: 0 past the end, like stb's get8
  int get8() { return p_ < end_ ? *p_++ : 0; }
  int get16() {
    const int a = get8();
    return (a << 8) | get8();
  }
  bool at_eof() const { return p_ >= end_; }
  void skip(int n) { p_ = (n < 0 || n > end_ - p_) ? end_ : p_ + n; }

  // bit reader (stbi__grow_buffer_unsafe semantics: a marker stops input, zeros follow)
  uint32_t buf_ = 0;
  int bits_ = 0;
  bool nomore_ = false;
  int marker_ = kNoMarker;
  void grow() {
    do {
      uint32_t b = nomore_ ? 0u : (uint32_t)get8();
      if (b == 0xff) {
        int c = get8();
        while (c == 0xff) c = get8();
        if (c != 0) {
          marker_ = c;
          nomore_ = true;
          return;
        }
      }
      buf_ |= b << (24 - bits_);
      bits_ += 8;
    } while (bits_ <= 24);
  }
  int huff_decode(const Huffman& hf) {
    if (bits_ < 16) grow();
    const uint32_t top = buf_ >> 16;
    int k;
    for (k = 1; k <= 16; k++)
      if (top < hf.maxcode[k]) break;
    if (k == 17) {
      bits_ -= 16;
      return -1;
    }
    if (k > bits_) return -1;
    const int c = (int)((buf_ >> (32 - k)) & ((1u << k) - 1u)) + hf.delta[k];
    if (c < 0 || c >= 256) return -1;
    bits_ -= k;
    buf_ <<= k;
    return hf.values[c];
  }
  int receive_extend(int n) {  // JPEG RECEIVE + EXTEND
    if (bits_ < n) grow();
    if (bits_ < n) return 0;
    const int sgn = (int)(buf_ >> 31);
    const uint32_t rot = (buf_ << n) | (buf_ >> ((32 - n) & 31));
    const uint32_t mask = (1u << n) - 1u;
    buf_ = rot & ~mask;
    const uint32_t k = rot & mask;
    bits_ -= n;
    const int bias = n ? -(1 << n) + 1 : 0;
    return (int)k + (bias & (sgn - 1));
  }
  int get_bits(int n) {
    if (bits_ < n) grow();
    if (bits_ < n) return 0;
    const uint32_t rot = (buf_ << n) | (buf_ >> ((32 - n) & 31));
    const uint32_t mask = (1u << n) - 1u;
    buf_ = rot & ~mask;
    bits_ -= n;
    return (int)(rot & mask);
  }
  bool get_bit() {
    if (bits_ < 1) grow();
    if (bits_ < 1) return false;
    const uint32_t k = buf_;
    buf_ <<= 1;
    bits_--;
    return (k & 0x80000000u) != 0;
  }
  int get_marker() {
    if (marker_ != kNoMarker) {
      const int x = marker_;
      marker_ = kNoMarker;
      return x;
    }
    int x = get8();
    if (x != 0xff) return kNoMarker;
    while (x == 0xff) x = get8();
    return x;
  }

  // stream state
  Huffman hdc_[4], hac_[4];
  uint16_t dequant_[4][64] = {};
  Component comp_[4];
  int n_ = 0, width_ = 0, height_ = 0;
  int hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
  bool progressive_ = false, jfif_ = false;
  int rgb_ids_ = 0, app14_ = -1;
  int restart_interval_ = 0, todo_ = 0, eob_run_ = 0;
  int scan_n_ = 0, order_[4] = {};
  int spec_start_ = 0, spec_end_ = 0, succ_high_ = 0, succ_low_ = 0;

  void reset() {
    bits_ = 0, buf_ = 0, nomore_ = false;
    for (auto& c : comp_) c.dc_pred = 0;
    marker_ = kNoMarker;
    todo_ = restart_interval_ ? restart_interval_ : 0x7fffffff;
    eob_run_ = 0;
  }
  static bool add_ok(int a, int b) {
    if ((a >= 0) != (b >= 0)) return true;
    if (a < 0 && b < 0) return a >= INT_MIN - b;
    return a <= INT_MAX - b;
  }
  static bool mul_short_ok(int a, int b) {  // a * b fits in a short
    if (b == 0 || b == -1) return true;
    if ((a >= 0) == (b >= 0)) return a <= SHRT_MAX / b;
    if (b < 0) return a <= SHRT_MIN / b;
    return a >= SHRT_MIN / b;
  }

  bool process_marker(int m);
  bool frame_header();
  bool scan_header();
  bool entropy_data();
  bool block_baseline(int16_t* data, const Component& c, int b);
  bool block_prog_dc(int16_t* data, int b);
  bool block_prog_ac(int16_t* data, const Huffman& hac);
  bool restart_countdown(bool& stop) {
    stop = false;
    if (--todo_ <= 0) {
      if (bits_ < 24) grow();
      if (!(marker_ >= 0xd0 && marker_ <= 0xd7)) {
        stop = true;
        return true;
      }
      reset();
    }
    return true;
  }
  int skip_junk_at_end();
  void idct(uint8_t* out, int stride, const int16_t* data);
};

bool Jpeg::process_marker(int m) {
  if (m == kNoMarker) return fail("expected marker");
  if (m == 0xdd) {  // DRI
    if (get16() != 4) return fail("bad DRI len");
    restart_interval_ = get16();
    return true;
  }
  if (m == 0xdb) {  // DQT
    int L = get16() - 2;
    while (L > 0) {
      const int q = get8(), p = q >> 4, t = q & 15;
      if (p != 0 && p != 1) return fail("bad DQT type");
      if (t > 3) return fail("bad DQT table");
      for (int i = 0; i < 64; i++) dequant_[t][kDezigzag[i]] = (uint16_t)(p ? get16() : get8());
      L -= p ? 129 : 65;
    }
    return L == 0 || fail("bad DQT len");
  }
  if (m == 0xc4) {  // DHT
    int L = get16() - 2;
    while (L > 0) {
      const int q = get8(), tc = q >> 4, th = q & 15;
      if (tc > 1 || th > 3) return fail("bad DHT header");
      int lengths[16], total = 0;
      for (int i = 0; i < 16; i++) lengths[i] = get8(), total += lengths[i];
      if (total > 256) return fail("bad DHT header");
      L -= 17;
      Huffman& hf = tc == 0 ? hdc_[th] : hac_[th];
      if (!hf.build(lengths)) return fail("bad code lengths");
      for (int i = 0; i < total; i++) hf.values[i] = (uint8_t)get8();
      L -= total;
    }
    return L == 0 || fail("bad DHT len");
  }
  if ((m >= 0xe0 && m <= 0xef) || m == 0xfe) {  // APPn / COM
    int L = get16();
    if (L < 2) return fail(m == 0xfe ? "bad COM len" : "bad APP len");
    L -= 2;
    if (m == 0xe0 && L >= 5) {  // JFIF
      static const uint8_t tag[5] = {'J', 'F', 'I', 'F', 0};
      bool ok = true;
      for (int i = 0; i < 5; i++) ok = (get8() == tag[i]) && ok;
      L -= 5;
      if (ok) jfif_ = true;
    } else if (m == 0xee && L >= 12) {  // Adobe APP14: colour transform
      static const uint8_t tag[6] = {'A', 'd', 'o', 'b', 'e', 0};
      bool ok = true;
      for (int i = 0; i < 6; i++) ok = (get8() == tag[i]) && ok;
      L -= 6;
      if (ok) {
        get8(), get16(), get16();
        app14_ = get8();
        L -= 6;
      }
    }
    skip(L);
    return true;
  }
  return fail("unknown marker");
}

bool Jpeg::frame_header() {
  const int Lf = get16();
  if (Lf < 11) return fail("bad SOF len");
  if (get8() != 8) return fail("only 8-bit JPEG");
  height_ = get16();
  if (height_ == 0) return fail("no header height");
  width_ = get16();
  if (width_ == 0) return fail("0 width");
  if (width_ > (1 << 24) || height_ > (1 << 24)) return fail("too large");
  n_ = get8();
  if (n_ != 1 && n_ != 3 && n_ != 4) return fail("bad component count");
  if (Lf != 8 + 3 * n_) return fail("bad SOF len");
  rgb_ids_ = 0;
  for (int i = 0; i < n_; i++) {
    static const uint8_t rgb[3] = {'R', 'G', 'B'};
    Component& c = comp_[i];
    c.id = get8();
    if (n_ == 3 && c.id == rgb[i]) rgb_ids_++;
    const int q = get8();
    c.h = q >> 4, c.v = q & 15;
    if (!c.h || c.h > 4) return fail("bad H");
    if (!c.v || c.v > 4) return fail("bad V");
    c.tq = get8();
    if (c.tq > 3) return fail("bad TQ");
  }
  if ((int64_t)width_ * height_ * n_ > INT_MAX) return fail("image too large");
  for (int i = 0; i < n_; i++) hmax_ = std::max(hmax_, comp_[i].h), vmax_ = std::max(vmax_, comp_[i].v);
  for (int i = 0; i < n_; i++)
    if (hmax_ % comp_[i].h || vmax_ % comp_[i].v) return fail("bad H/V");
  mcux_ = (width_ + hmax_ * 8 - 1) / (hmax_ * 8);
  mcuy_ = (height_ + vmax_ * 8 - 1) / (vmax_ * 8);
  for (int i = 0; i < n_; i++) {
    Component& c = comp_[i];
    c.x = (width_ * c.h + hmax_ - 1) / hmax_;
    c.y = (height_ * c.v + vmax_ - 1) / vmax_;
    c.w2 = mcux_ * c.h * 8;
    c.h2 = mcuy_ * c.v * 8;
    c.data.assign((size_t)c.w2 * c.h2, 0);
    if (progressive_) {
      c.coeff_w = c.w2 / 8;
      c.coeff.assign((size_t)c.w2 * c.h2, 0);
    }
  }
  return true;
}

bool Jpeg::scan_header() {
  const int Ls = get16();
  scan_n_ = get8();
  if (scan_n_ < 1 || scan_n_ > 4 || scan_n_ > n_) return fail("bad SOS component count");
  if (Ls != 6 + 2 * scan_n_) return fail("bad SOS len");
  for (int i = 0; i < scan_n_; i++) {
    const int id = get8(), q = get8();
    int which = 0;
    while (which < n_ && comp_[which].id != id) which++;
    if (which == n_) return fail("bad SOS component id");
    comp_[which].hd = q >> 4;
    comp_[which].ha = q & 15;
    if (comp_[which].hd > 3 || comp_[which].ha > 3) return fail("bad Huffman table id");
    order_[i] = which;
  }
  spec_start_ = get8();
  spec_end_ = get8();
  const int aa = get8();
  succ_high_ = aa >> 4, succ_low_ = aa & 15;
  if (progressive_) {
    if (spec_start_ > 63 || spec_end_ > 63 || spec_start_ > spec_end_ || succ_high_ > 13 || succ_low_ > 13)
      return fail("bad SOS");
  } else {
    if (spec_start_ != 0 || succ_high_ != 0 || succ_low_ != 0) return fail("bad SOS");
    spec_end_ = 63;
  }
  return true;
}

bool Jpeg::block_baseline(int16_t* data, const Component& c, int b) {
  const int t = huff_decode(hdc_[c.hd]);
  if (t < 0 || t > 15) return fail("bad huffman code");
  std::memset(data, 0, 64 * sizeof(int16_t));
  const int diff = t ? receive_extend(t) : 0;
  if (!add_ok(comp_[b].dc_pred, diff)) return fail("bad delta");
  const int dc = comp_[b].dc_pred + diff;
  comp_[b].dc_pred = dc;
  const uint16_t* dq = dequant_[c.tq];
  if (!mul_short_ok(dc, dq[0])) return fail("can't merge dc and ac");
  data[0] = (int16_t)(dc * dq[0]);
  int k = 1;
  do {
    const int rs = huff_decode(hac_[c.ha]);
    if (rs < 0) return fail("bad huffman code");
    const int s = rs & 15, r = rs >> 4;
    if (s == 0) {
      if (rs != 0xf0) break;  // end of block
      k += 16;
    } else {
      k += r;
      const int zig = kDezigzag[k++];
      data[zig] = (int16_t)(receive_extend(s) * dq[zig]);
    }
  } while (k < 64);
  return true;
}

bool Jpeg::block_prog_dc(int16_t* data, int b) {
  if (spec_end_ != 0) return fail("can't merge dc and ac");
  if (succ_high_ == 0) {
    std::memset(data, 0, 64 * sizeof(int16_t));
    const int t = huff_decode(hdc_[comp_[b].hd]);
    if (t < 0 || t > 15) return fail("can't merge dc and ac");
    const int diff = t ? receive_extend(t) : 0;
    if (!add_ok(comp_[b].dc_pred, diff)) return fail("bad delta");
    const int dc = comp_[b].dc_pred + diff;
    comp_[b].dc_pred = dc;
    if (!mul_short_ok(dc, 1 << succ_low_)) return fail("can't merge dc and ac");
    data[0] = (int16_t)(dc * (1 << succ_low_));
  } else if (get_bit()) {
    data[0] = (int16_t)(data[0] + (1 << succ_low_));
  }
  return true;
}

bool Jpeg::block_prog_ac(int16_t* data, const Huffman& hac) {
  if (spec_start_ == 0) return fail("can't merge dc and ac");
  if (succ_high_ == 0) {  // first pass of these coefficients
    if (eob_run_) {
      --eob_run_;
      return true;
    }
    int k = spec_start_;
    do {
      const int rs = huff_decode(hac);
      if (rs < 0) return fail("bad huffman code");
      const int s = rs & 15, r = rs >> 4;
      if (s == 0) {
        if (r < 15) {
          eob_run_ = 1 << r;
          if (r) eob_run_ += get_bits(r);
          --eob_run_;
          break;
        }
        k += 16;
      } else {
        k += r;
        const int zig = kDezigzag[k++];
        data[zig] = (int16_t)(receive_extend(s) * (1 << succ_low_));
      }
    } while (k <= spec_end_);
    return true;
  }
  // refinement pass
  const int16_t bit = (int16_t)(1 << succ_low_);
  auto refine = [&](int16_t* p) {
    if (get_bit() && (*p & bit) == 0) *p = (int16_t)(*p > 0 ? *p + bit : *p - bit);
  };
  if (eob_run_) {
    --eob_run_;
    for (int k = spec_start_; k <= spec_end_; ++k) {
      int16_t* p = &data[kDezigzag[k]];
      if (*p != 0) refine(p);
    }
    return true;
  }
  int k = spec_start_;
  do {
    const int rs = huff_decode(hac);
    if (rs < 0) return fail("bad huffman code");
    int s = rs & 15, r = rs >> 4;
    if (s == 0) {
      if (r < 15) {
        eob_run_ = (1 << r) - 1;
        if (r) eob_run_ += get_bits(r);
        r = 64;  // force end of block
      }
      // r = 15, s = 0: a run of 15 zero coefficients, then a zero
    } else {
      if (s != 1) return fail("bad huffman code");
      s = get_bit() ? bit : -bit;
    }
    while (k <= spec_end_) {
      int16_t* p = &data[kDezigzag[k++]];
      if (*p != 0) {
        refine(p);
      } else {
        if (r == 0) {
          *p = (int16_t)s;
          break;
        }
        --r;
      }
    }
  } while (k <= spec_end_);
  return true;
}

bool Jpeg::entropy_data() {
  reset();
  int16_t data[64];
  bool stop = false;
  if (scan_n_ == 1) {  // non-interleaved: blocks in raster order over the component's own size
    const int n = order_[0];
    Component& c = comp_[n];
    const int w = (c.x + 7) >> 3, h = (c.y + 7) >> 3;
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) {
        if (!progressive_) {
          if (!block_baseline(data, c, n)) return false;
          idct(c.data.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2, data);
        } else {
          int16_t* blk = c.coeff.data() + 64 * ((size_t)i + (size_t)j * c.coeff_w);
          if (spec_start_ == 0) {
            if (!block_prog_dc(blk, n)) return false;
          } else if (!block_prog_ac(blk, hac_[c.ha])) {
            return false;
          }
        }
        restart_countdown(stop);
        if (stop) return true;
      }
    return true;
  }
  for (int j = 0; j < mcuy_; ++j)  // interleaved MCUs
    for (int i = 0; i < mcux_; ++i) {
      for (int k = 0; k < scan_n_; ++k) {
        const int n = order_[k];
        Component& c = comp_[n];
        for (int y = 0; y < c.v; ++y)
          for (int x = 0; x < c.h; ++x) {
            const int bx = i * c.h + x, by = j * c.v + y;
            if (!progressive_) {
              if (!block_baseline(data, c, n)) return false;
              idct(c.data.data() + (size_t)c.w2 * by * 8 + bx * 8, c.w2, data);
            } else if (!block_prog_dc(c.coeff.data() + 64 * ((size_t)bx + (size_t)by * c.coeff_w), n)) {
              return false;
            }
          }
      }
      restart_countdown(stop);
      if (stop) return true;
    }
  return true;
}

int Jpeg::skip_junk_at_end() {
  while (!at_eof()) {
    int x = get8();
    while (x == 0xff) {
      if (at_eof()) return kNoMarker;
      x = get8();
      if (x != 0x00 && x != 0xff) return x;
    }
  }
  return kNoMarker;
}

// ---- integer IDCT (jidctint ISLOW with stb's 12-bit constants and rounding) -------------
// f2f(x) = (int)(x * 4096 + 0.5) with x a float literal, exactly as the reference evaluates it
#define RTX_F2F(x) ((int)(((x) * 4096 + 0.5)))
struct Idct1d {
  int t0, t1, t2, t3, x0, x1, x2, x3;
  Idct1d(int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7) {
    int p2 = s2, p3 = s6;
    int p1 = (p2 + p3) * RTX_F2F(0.5411961f);
    t2 = p1 + p3 * RTX_F2F(-1.847759065f);
    t3 = p1 + p2 * RTX_F2F(0.765366865f);
    p2 = s0, p3 = s4;
    t0 = (p2 + p3) * 4096;
    t1 = (p2 - p3) * 4096;
    x0 = t0 + t3, x3 = t0 - t3, x1 = t1 + t2, x2 = t1 - t2;
    t0 = s7, t1 = s5, t2 = s3, t3 = s1;
    p3 = t0 + t2;
    int p4 = t1 + t3;
    p1 = t0 + t3;
    p2 = t1 + t2;
    const int p5 = (p3 + p4) * RTX_F2F(1.175875602f);
    t0 = t0 * RTX_F2F(0.298631336f);
    t1 = t1 * RTX_F2F(2.053119869f);
    t2 = t2 * RTX_F2F(3.072711026f);
    t3 = t3 * RTX_F2F(1.501321110f);
    p1 = p5 + p1 * RTX_F2F(-0.899976223f);
    p2 = p5 + p2 * RTX_F2F(-2.562915447f);
    p3 = p3 * RTX_F2F(-1.961570560f);
    p4 = p4 * RTX_F2F(-0.390180644f);
    t3 += p1 + p4;
    t2 += p2 + p3;
    t1 += p2 + p4;
    t0 += p1 + p3;
  }
};
#undef RTX_F2F

inline uint8_t clamp255(int x) { return (uint8_t)(x < 0 ? 0 : (x > 255 ? 255 : x)); }

void Jpeg::idct(uint8_t* out, int stride, const int16_t* d) {
  int v[64];
  for (int i = 0; i < 8; ++i) {  // columns (a zero AC column is the same as the full transform)
    const int16_t* c = d + i;
    if (!c[8] && !c[16] && !c[24] && !c[32] && !c[40] && !c[48] && !c[56]) {
      const int dc = c[0] * 4;
      for (int r = 0; r < 8; r++) v[i + 8 * r] = dc;
      continue;
    }
    Idct1d t(c[0], c[8], c[16], c[24], c[32], c[40], c[48], c[56]);
    t.x0 += 512, t.x1 += 512, t.x2 += 512, t.x3 += 512;
    v[i + 0] = (t.x0 + t.t3) >> 10;
    v[i + 56] = (t.x0 - t.t3) >> 10;
    v[i + 8] = (t.x1 + t.t2) >> 10;
    v[i + 48] = (t.x1 - t.t2) >> 10;
    v[i + 16] = (t.x2 + t.t1) >> 10;
    v[i + 40] = (t.x2 - t.t1) >> 10;
    v[i + 24] = (t.x3 + t.t0) >> 10;
    v[i + 32] = (t.x3 - t.t0) >> 10;
  }
  for (int r = 0; r < 8; ++r) {  // rows: remove 1 << 17, round, and bias by 128
    const int* w = v + 8 * r;
    Idct1d t(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]);
    const int bias = 65536 + (128 << 17);
    t.x0 += bias, t.x1 += bias, t.x2 += bias, t.x3 += bias;
    uint8_t* o = out + (size_t)r * stride;
    o[0] = clamp255((t.x0 + t.t3) >> 17);
    o[7] = clamp255((t.x0 - t.t3) >> 17);
    o[1] = clamp255((t.x1 + t.t2) >> 17);
    o[6] = clamp255((t.x1 - t.t2) >> 17);
    o[2] = clamp255((t.x2 + t.t1) >> 17);
    o[5] = clamp255((t.x2 - t.t1) >> 17);
    o[3] = clamp255((t.x3 + t.t0) >> 17);
    o[4] = clamp255((t.x3 - t.t0) >> 17);
  }
}

// ---- upsampling and colour ---------------------------------------------------------------
using Resample = const uint8_t* (*)(uint8_t* out, const uint8_t* near, const uint8_t* far, int w, int hs);

const uint8_t* resample_1(uint8_t*, const uint8_t* near, const uint8_t*, int, int) { return near; }
const uint8_t* resample_v2(uint8_t* out, const uint8_t* near, const uint8_t* far, int w, int) {
  for (int i = 0; i < w; ++i) out[i] = (uint8_t)((3 * near[i] + far[i] + 2) >> 2);
  return out;
}
const uint8_t* resample_h2(uint8_t* out, const uint8_t* in, const uint8_t*, int w, int) {
  if (w == 1) {
    out[0] = out[1] = in[0];
    return out;
  }
  out[0] = in[0];
  out[1] = (uint8_t)((in[0] * 3 + in[1] + 2) >> 2);
  int i;
  for (i = 1; i < w - 1; ++i) {
    const int n = 3 * in[i] + 2;
    out[i * 2 + 0] = (uint8_t)((n + in[i - 1]) >> 2);
    out[i * 2 + 1] = (uint8_t)((n + in[i + 1]) >> 2);
  }
  out[i * 2 + 0] = (uint8_t)((in[w - 2] * 3 + in[w - 1] + 2) >> 2);
  out[i * 2 + 1] = in[w - 1];
  return out;
}
const uint8_t* resample_hv2(uint8_t* out, const uint8_t* near, const uint8_t* far, int w, int) {
  if (w == 1) {
    out[0] = out[1] = (uint8_t)((3 * near[0] + far[0] + 2) >> 2);
    return out;
  }
  int t1 = 3 * near[0] + far[0], t0;
  out[0] = (uint8_t)((t1 + 2) >> 2);
  for (int i = 1; i < w; ++i) {
    t0 = t1;
    t1 = 3 * near[i] + far[i];
    out[i * 2 - 1] = (uint8_t)((3 * t0 + t1 + 8) >> 4);
    out[i * 2] = (uint8_t)((3 * t1 + t0 + 8) >> 4);
  }
  out[w * 2 - 1] = (uint8_t)((t1 + 2) >> 2);
  return out;
}
const uint8_t* resample_nearest(uint8_t* out, const uint8_t* near, const uint8_t*, int w, int hs) {
  for (int i = 0; i < w; ++i)
    for (int j = 0; j < hs; ++j) out[i * hs + j] = near[i];
  return out;
}

// stbi__YCbCr_to_RGB_row: 20-bit fixed point, the cb term of g truncated to 16 fractional bits
#define RTX_FIX(x) (((int)((x) * 4096.0f + 0.5f)) << 8)
void ycbcr_to_rgb(uint8_t* out, const uint8_t* y, const uint8_t* cb, const uint8_t* cr, int count) {
  for (int i = 0; i < count; ++i, out += 3) {
    const int yf = (y[i] << 20) + (1 << 19);
    const int crv = cr[i] - 128, cbv = cb[i] - 128;
    int r = yf + crv * RTX_FIX(1.40200f);
    int g = yf + (crv * -RTX_FIX(0.71414f)) + ((cbv * -RTX_FIX(0.34414f)) & (int)0xffff0000);
    int b = yf + cbv * RTX_FIX(1.77200f);
    r >>= 20, g >>= 20, b >>= 20;
    out[0] = clamp255(r), out[1] = clamp255(g), out[2] = clamp255(b);
  }
}
#undef RTX_FIX

inline uint8_t blinn_8x8(uint8_t x, uint8_t y) {  // x * y / 255, rounded
  const unsigned t = (unsigned)x * y + 128u;
  return (uint8_t)((t + (t >> 8)) >> 8);
}

bool Jpeg::decode(int& w, int& h, std::vector<uint8_t>& rgb, std::string& err) {
  auto bail = [&]() {
    err = "JPEG: " + (err_.empty() ? std::string("corrupt") : err_);
    return false;
  };
  // header: SOI, markers up to SOF (stbi__decode_jpeg_header)
  marker_ = kNoMarker;
  if (get_marker() != 0xd8) return fail("no SOI"), bail();
  int m = get_marker();
  while (!(m == 0xc0 || m == 0xc1 || m == 0xc2)) {
    if (!process_marker(m)) return bail();
    m = get_marker();
    while (m == kNoMarker) {
      if (at_eof()) return fail("no SOF"), bail();
      m = get_marker();
    }
  }
  progressive_ = m == 0xc2;
  if (!frame_header()) return bail();
  // scans (stbi__decode_jpeg_image)
  m = get_marker();
  while (m != 0xd9) {
    if (m == 0xda) {
      if (!scan_header() || !entropy_data()) return bail();
      if (marker_ == kNoMarker) marker_ = skip_junk_at_end();
      m = get_marker();
      if (m >= 0xd0 && m <= 0xd7) m = get_marker();
    } else if (m == 0xdc) {  // DNL
      const int Ld = get16();
      const int NL = get16();
      if (Ld != 4) return fail("bad DNL len"), bail();
      if (NL != height_) return fail("bad DNL height"), bail();
      m = get_marker();
    } else {
      if (!process_marker(m)) break;  // stb stops here and keeps what it decoded (also at a missing EOI)
      m = get_marker();
    }
  }
  if (progressive_) {  // dequantise (16-bit) and transform (stbi__jpeg_finish)
    for (int n = 0; n < n_; ++n) {
      Component& c = comp_[n];
      const int bw = (c.x + 7) >> 3, bh = (c.y + 7) >> 3;
      for (int j = 0; j < bh; ++j)
        for (int i = 0; i < bw; ++i) {
          int16_t* blk = c.coeff.data() + 64 * ((size_t)i + (size_t)j * c.coeff_w);
          for (int k = 0; k < 64; ++k) blk[k] = (int16_t)(blk[k] * dequant_[c.tq][k]);
          idct(c.data.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2, blk);
        }
    }
  }
  // resample and colour-convert to 3 channels (load_jpeg_image with req_comp = 3)
  const bool is_rgb = n_ == 3 && (rgb_ids_ == 3 || (app14_ == 0 && !jfif_));
  struct Res {
    Resample fn;
    const uint8_t *line0, *line1;
    int hs, vs, w_lores, ystep, ypos;
    std::vector<uint8_t> linebuf;
  } res[4];
  for (int k = 0; k < n_; ++k) {
    Res& r = res[k];
    r.linebuf.assign((size_t)width_ + 3, 0);
    r.hs = hmax_ / comp_[k].h;
    r.vs = vmax_ / comp_[k].v;
    r.ystep = r.vs >> 1;
    r.w_lores = (width_ + r.hs - 1) / r.hs;
    r.ypos = 0;
    r.line0 = r.line1 = comp_[k].data.data();
    if (r.hs == 1 && r.vs == 1) r.fn = resample_1;
    else if (r.hs == 1 && r.vs == 2) r.fn = resample_v2;
    else if (r.hs == 2 && r.vs == 1) r.fn = resample_h2;
    else if (r.hs == 2 && r.vs == 2) r.fn = resample_hv2;
    else r.fn = resample_nearest;
  }
  rgb.assign((size_t)width_ * height_ * 3, 0);
  const uint8_t* co[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int j = 0; j < height_; ++j) {
    uint8_t* out = rgb.data() + (size_t)3 * width_ * j;
    for (int k = 0; k < n_; ++k) {
      Res& r = res[k];
      const bool y_bot = r.ystep >= (r.vs >> 1);
      co[k] = r.fn(r.linebuf.data(), y_bot ? r.line1 : r.line0, y_bot ? r.line0 : r.line1, r.w_lores, r.hs);
      if (++r.ystep >= r.vs) {
        r.ystep = 0;
        r.line0 = r.line1;
        if (++r.ypos < comp_[k].y) r.line1 += comp_[k].w2;
      }
    }
    if (n_ == 3) {
      if (is_rgb) {
        for (int i = 0; i < width_; ++i) out[3 * i] = co[0][i], out[3 * i + 1] = co[1][i], out[3 * i + 2] = co[2][i];
      } else {
        ycbcr_to_rgb(out, co[0], co[1], co[2], width_);
      }
    } else if (n_ == 4) {
      if (app14_ == 0) {  // CMYK
        for (int i = 0; i < width_; ++i) {
          const uint8_t k = co[3][i];
          out[3 * i] = blinn_8x8(co[0][i], k), out[3 * i + 1] = blinn_8x8(co[1][i], k);
          out[3 * i + 2] = blinn_8x8(co[2][i], k);
        }
      } else if (app14_ == 2) {  // YCCK
        ycbcr_to_rgb(out, co[0], co[1], co[2], width_);
        for (int i = 0; i < width_; ++i) {
          const uint8_t k = co[3][i];
          for (int c = 0; c < 3; c++) out[3 * i + c] = blinn_8x8((uint8_t)(255 - out[3 * i + c]), k);
        }
      } else {  // YCbCr + a fourth channel, ignored
        ycbcr_to_rgb(out, co[0], co[1], co[2], width_);
      }
    } else {
      for (int i = 0; i < width_; ++i) out[3 * i] = out[3 * i + 1] = out[3 * i + 2] = co[0][i];
    }
  }
  w = width_, h = height_;
  return true;
}

// ---- binary PNM (stbi__pnm_load: P5 / P6) ---------------------------------------------------
bool decode_pnm(const uint8_t* p, size_t n, int& w, int& h, std::vector<uint8_t>& rgb, std::string& err) {
  size_t i = 2;
  const int comps = p[1] == '5' ? 1 : 3;
  auto skip_ws = [&]() {
    while (i < n && (std::isspace(p[i]) || p[i] == '#')) {
      if (p[i] == '#')
        while (i < n && p[i] != '\n' && p[i] != '\r') i++;
      else
        i++;
    }
  };
  auto number = [&](int& v) {
    skip_ws();
    if (i >= n || !std::isdigit(p[i])) return false;
    long long x = 0;
    while (i < n && std::isdigit(p[i])) {
      x = x * 10 + (p[i++] - '0');
      if (x > INT_MAX) return false;
    }
    v = (int)x;
    return true;
  };
  int maxv = 0;
  if (!number(w) || !number(h) || !number(maxv)) return err = "PNM: bad header", false;
  if (w <= 0 || h <= 0) return err = "PNM: zero size", false;
  if (maxv > 255) return err = "PNM: 16-bit samples not supported", false;
  i++;  // the single whitespace after maxval
  const size_t need = (size_t)w * h * comps;
  if (i + need > n) return err = "PNM: truncated", false;
  rgb.resize((size_t)w * h * 3);
  for (size_t k = 0; k < (size_t)w * h; k++)
    for (int c = 0; c < 3; c++) rgb[3 * k + c] = p[i + k * comps + (comps == 3 ? c : 0)];
  return true;
}

}  // namespace

bool DecodeJpeg(const uint8_t* data, size_t n, int& w, int& h, std::vector<uint8_t>& rgb, std::string& err) {
  Jpeg j(data, n);
  return j.decode(w, h, rgb, err);
}

bool DecodeImage8(const std::vector<uint8_t>& file, int& w, int& h, std::vector<uint8_t>& rgb, std::string& err) {
  const uint8_t* p = file.data();
  const size_t n = file.size();
  if (n >= 2 && p[0] == 0xff && p[1] == 0xd8) return DecodeJpeg(p, n, w, h, rgb, err);
  if (n >= 2 && p[0] == 'P' && (p[1] == '5' || p[1] == '6')) return decode_pnm(p, n, w, h, rgb, err);
  err = "unknown image type (JPEG and binary PNM are supported)";
  return false;
}

uint8_t TexelFromByte(uint8_t b) {
  // stbi__ldr_to_hdr: (float)(pow(b / 255.0f, 2.2f) * 1.0f) with pow's float overload, then
  // Image::FloatToByte (image.cc:69-73)
  const float f = (float)(std::pow(b / 255.0f, 2.2f) * 1.0f);
  if (f <= 0.0f) return 0;
  if (f >= 1.0f) return 255;
  return (uint8_t)(f * 255.999f);
}

bool LoadTexels(const std::string& path, int& w, int& h, std::vector<uint8_t>& texels, std::string& err,
                bool linear8) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return err = "cannot open " + path, false;
  std::vector<uint8_t> file((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  if (!DecodeImage8(file, w, h, texels, err)) return false;
  if (!linear8) {
    uint8_t lut[256];
    for (int i = 0; i < 256; i++) lut[i] = TexelFromByte((uint8_t)i);
    for (uint8_t& b : texels) b = lut[b];
  }
  return true;
}

}  // namespace rt::scene
