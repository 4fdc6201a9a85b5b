// Baseline / extended-sequential Huffman JPEG decoder (8-bit, 1 or 3 components, any
// sampling factors up to 4x4, restart markers).  Used by the Tiny-ImageNet loader in place of
// the reference's vendored stb_image (src/data_loading/stb_image_impl.cpp:11).  Progressive and
// arithmetic-coded files are rejected with an error.
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "native.h"

namespace dcnn_native {
namespace {

const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                         41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                         30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
  // canonical code tables: for each length l, codes [mincode[l], maxcode[l]] map to vals[valptr[l] + c - mincode[l]]
  int mincode[17], maxcode[18], valptr[17];
  unsigned char vals[256];
  // 9-bit lookup: (len << 8) | value, 0 if longer
  unsigned short fast[512];
  bool present = false;
};

struct Comp {
  int id, h, v, tq, td = 0, ta = 0;
  int bw, bh;  // blocks per line / column in the component plane
  std::vector<unsigned char> plane;
  int dc_pred = 0;
};

class Decoder {
 public:
  Decoder(const unsigned char* p, size_t n) : p_(p), end_(p + n) {}
  void decode(std::vector<unsigned char>& out, int& W, int& H, int& C);

 private:
  const unsigned char* p_;
  const unsigned char* end_;
  unsigned short qt_[4][64];
  Huff hdc_[4], hac_[4];
  std::vector<Comp> comps_;
  int width_ = 0, height_ = 0, hmax_ = 1, vmax_ = 1, restart_ = 0;
  // bit reader
  unsigned bitbuf_ = 0;
  int bitcnt_ = 0;
  bool hit_marker_ = false;

  int u8() {
    if (p_ >= end_) throw std::runtime_error("jpeg: unexpected end of data");
    return *p_++;
  }
  int u16() {
    int a = u8();
    return (a << 8) | u8();
  }
  void build_huff(Huff& h, const unsigned char* counts, const unsigned char* vals, int nvals);
  void read_sof();
  void read_dht(int len);
  void read_dqt(int len);
  void read_sos();
  void fill_bits();
  int get_bits(int n);
  int decode_huff(const Huff& h);
  void reset_bits() {
    bitbuf_ = 0;
    bitcnt_ = 0;
    hit_marker_ = false;
  }
  void decode_block(Comp& c, short* blk);
};

void Decoder::build_huff(Huff& h, const unsigned char* counts, const unsigned char* vals, int nvals) {
  std::memcpy(h.vals, vals, nvals);
  int code = 0, k = 0;
  std::memset(h.fast, 0, sizeof(h.fast));
  for (int l = 1; l <= 16; ++l) {
    h.valptr[l] = k;
    h.mincode[l] = code;
    code += counts[l - 1];
    k += counts[l - 1];
    h.maxcode[l] = counts[l - 1] ? code - 1 : -1;
    code <<= 1;
  }
  h.maxcode[17] = 0x7fffffff;
  // fast table for codes of length <= 9
  for (int l = 1; l <= 9; ++l) {
    if (h.maxcode[l] < 0) continue;
    for (int c = h.mincode[l]; c <= h.maxcode[l]; ++c) {
      const int v = h.vals[h.valptr[l] + c - h.mincode[l]];
      const int shift = 9 - l;
      for (int f = 0; f < (1 << shift); ++f) h.fast[(c << shift) | f] = static_cast<unsigned short>((l << 8) | v);
    }
  }
  h.present = true;
}

void Decoder::read_sof() {
  const int len = u16();
  const int prec = u8();
  if (prec != 8) throw std::runtime_error("jpeg: only 8-bit precision supported");
  height_ = u16();
  width_ = u16();
  const int nc = u8();
  if (len != 8 + 3 * nc || (nc != 1 && nc != 3)) throw std::runtime_error("jpeg: unsupported component count");
  if (width_ <= 0 || height_ <= 0 || width_ > 16384 || height_ > 16384) throw std::runtime_error("jpeg: bad size");
  comps_.resize(nc);
  for (auto& c : comps_) {
    c.id = u8();
    const int hv = u8();
    c.h = hv >> 4;
    c.v = hv & 15;
    c.tq = u8() & 3;
    if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4) throw std::runtime_error("jpeg: bad sampling factor");
    hmax_ = std::max(hmax_, c.h);
    vmax_ = std::max(vmax_, c.v);
  }
}

void Decoder::read_dht(int len) {
  len -= 2;
  while (len > 0) {
    const int tc_th = u8();
    unsigned char counts[16], vals[256];
    int total = 0;
    for (int i = 0; i < 16; ++i) {
      counts[i] = static_cast<unsigned char>(u8());
      total += counts[i];
    }
    if (total > 256) throw std::runtime_error("jpeg: bad huffman table");
    for (int i = 0; i < total; ++i) vals[i] = static_cast<unsigned char>(u8());
    Huff& h = (tc_th >> 4) ? hac_[tc_th & 3] : hdc_[tc_th & 3];
    build_huff(h, counts, vals, total);
    len -= 17 + total;
  }
}

void Decoder::read_dqt(int len) {
  len -= 2;
  while (len > 0) {
    const int pq_tq = u8();
    const int t = pq_tq & 3;
    const bool wide = (pq_tq >> 4) != 0;
    for (int i = 0; i < 64; ++i) qt_[t][kZigzag[i]] = static_cast<unsigned short>(wide ? u16() : u8());
    len -= 1 + (wide ? 128 : 64);
  }
}

void Decoder::fill_bits() {
  while (bitcnt_ <= 24) {
    int b = 0;
    if (!hit_marker_ && p_ < end_) {
      b = *p_;
      if (b == 0xFF) {
        const int nxt = (p_ + 1 < end_) ? p_[1] : 0;
        if (nxt == 0x00) {
          p_ += 2;
        } else {
          hit_marker_ = true;  // marker: feed zeros, leave p_ at the marker
          b = 0;
        }
      } else {
        ++p_;
      }
    }
    bitbuf_ |= static_cast<unsigned>(b) << (24 - bitcnt_);
    bitcnt_ += 8;
  }
}

int Decoder::get_bits(int n) {
  if (n == 0) return 0;
  fill_bits();
  const unsigned v = bitbuf_ >> (32 - n);
  bitbuf_ <<= n;
  bitcnt_ -= n;
  return static_cast<int>(v);
}

int Decoder::decode_huff(const Huff& h) {
  if (!h.present) throw std::runtime_error("jpeg: missing huffman table");
  fill_bits();
  const unsigned short f = h.fast[bitbuf_ >> 23];
  if (f) {
    const int l = f >> 8;
    bitbuf_ <<= l;
    bitcnt_ -= l;
    return f & 0xFF;
  }
  int code = 0;
  for (int l = 1; l <= 16; ++l) {
    code = (code << 1) | static_cast<int>(bitbuf_ >> 31);
    bitbuf_ <<= 1;
    --bitcnt_;
    if (h.maxcode[l] >= 0 && code <= h.maxcode[l] && code >= h.mincode[l])
      return h.vals[h.valptr[l] + code - h.mincode[l]];
  }
  throw std::runtime_error("jpeg: bad huffman code");
}

inline int extend(int v, int n) { return (n && v < (1 << (n - 1))) ? v - (1 << n) + 1 : v; }

void Decoder::decode_block(Comp& c, short* blk) {
  std::memset(blk, 0, 64 * sizeof(short));
  const unsigned short* q = qt_[c.tq];
  const int t = decode_huff(hdc_[c.td]);
  const int diff = t ? extend(get_bits(t), t) : 0;
  c.dc_pred += diff;
  blk[0] = static_cast<short>(c.dc_pred * q[0]);
  for (int k = 1; k < 64;) {
    const int rs = decode_huff(hac_[c.ta]);
    const int r = rs >> 4, s = rs & 15;
    if (s == 0) {
      if (r != 15) break;  // EOB
      k += 16;
      continue;
    }
    k += r;
    if (k > 63) throw std::runtime_error("jpeg: AC index overflow");
    const int z = kZigzag[k];
    blk[z] = static_cast<short>(extend(get_bits(s), s) * q[z]);
    ++k;
  }
}

// separable float IDCT (accurate; images here are small)
void idct8x8(const short* in, unsigned char* out, int stride) {
  static float cosT[8][8];
  static bool init = false;
  if (!init) {
    for (int x = 0; x < 8; ++x)
      for (int u = 0; u < 8; ++u)
        cosT[x][u] = (u == 0 ? std::sqrt(0.125f) : 0.5f) * std::cos((2 * x + 1) * u * 3.14159265358979f / 16.0f);
    init = true;
  }
  float tmp[64];
  for (int y = 0; y < 8; ++y)  // rows: over u
    for (int x = 0; x < 8; ++x) {
      float s = 0;
      for (int u = 0; u < 8; ++u) s += cosT[x][u] * in[y * 8 + u];
      tmp[y * 8 + x] = s;
    }
  for (int x = 0; x < 8; ++x)
    for (int y = 0; y < 8; ++y) {
      float s = 0;
      for (int v = 0; v < 8; ++v) s += cosT[y][v] * tmp[v * 8 + x];
      int iv = static_cast<int>(std::lround(s + 128.0f));
      out[y * stride + x] = static_cast<unsigned char>(iv < 0 ? 0 : (iv > 255 ? 255 : iv));
    }
}

void Decoder::read_sos() {
  const int len = u16();
  const int ns = u8();
  if (ns != static_cast<int>(comps_.size()) || len != 6 + 2 * ns)
    throw std::runtime_error("jpeg: only interleaved single-scan images supported");
  for (int i = 0; i < ns; ++i) {
    const int cid = u8();
    const int t = u8();
    bool found = false;
    for (auto& c : comps_)
      if (c.id == cid) {
        c.td = t >> 4;
        c.ta = t & 15;
        found = true;
      }
    if (!found) throw std::runtime_error("jpeg: unknown component in scan");
  }
  u8();
  u8();
  u8();  // Ss, Se, Ah/Al (baseline: 0, 63, 0)
  const int mcux = (width_ + 8 * hmax_ - 1) / (8 * hmax_);
  const int mcuy = (height_ + 8 * vmax_ - 1) / (8 * vmax_);
  for (auto& c : comps_) {
    c.bw = mcux * c.h;
    c.bh = mcuy * c.v;
    c.plane.assign(static_cast<size_t>(c.bw) * 8 * c.bh * 8, 0);
    c.dc_pred = 0;
  }
  reset_bits();
  short blk[64];
  int mcus_left = restart_;
  for (int my = 0; my < mcuy; ++my)
    for (int mx = 0; mx < mcux; ++mx) {
      if (restart_ && mcus_left == 0) {
        // expect RSTn: skip to marker, consume it, reset predictors
        reset_bits();
        while (p_ + 1 < end_ && !(p_[0] == 0xFF && p_[1] >= 0xD0 && p_[1] <= 0xD7)) ++p_;
        if (p_ + 1 < end_) p_ += 2;
        for (auto& c : comps_) c.dc_pred = 0;
        mcus_left = restart_;
      }
      for (auto& c : comps_) {
        const int stride = c.bw * 8;
        for (int by = 0; by < c.v; ++by)
          for (int bx = 0; bx < c.h; ++bx) {
            decode_block(c, blk);
            const int px = (mx * c.h + bx) * 8, py = (my * c.v + by) * 8;
            idct8x8(blk, &c.plane[static_cast<size_t>(py) * stride + px], stride);
          }
      }
      if (restart_) --mcus_left;
    }
  // leave p_ at the next marker
  reset_bits();
  while (p_ + 1 < end_ && !(p_[0] == 0xFF && p_[1] != 0x00 && !(p_[1] >= 0xD0 && p_[1] <= 0xD7))) ++p_;
}

void Decoder::decode(std::vector<unsigned char>& out, int& W, int& H, int& C) {
  if (u8() != 0xFF || u8() != 0xD8) throw std::runtime_error("jpeg: missing SOI");
  bool have_frame = false, done = false;
  while (!done) {
    int m = u8();
    if (m != 0xFF) continue;
    while (m == 0xFF) m = u8();
    switch (m) {
      case 0xC0:
      case 0xC1: read_sof(); have_frame = true; break;
      case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB: case 0xCD:
      case 0xCE: case 0xCF:
        throw std::runtime_error("jpeg: progressive / lossless / arithmetic coding not supported");
      case 0xC4: read_dht(u16()); break;
      case 0xDB: read_dqt(u16()); break;
      case 0xDD:
        u16();
        restart_ = u16();
        break;
      case 0xDA:
        if (!have_frame) throw std::runtime_error("jpeg: SOS before SOF");
        read_sos();
        done = true;
        break;
      case 0xD9: done = true; break;
      default: {  // APPn, COM, ...
        const int len = u16();
        if (p_ + len - 2 > end_) throw std::runtime_error("jpeg: truncated segment");
        p_ += len - 2;
      }
    }
  }
  if (comps_.empty() || comps_[0].plane.empty()) throw std::runtime_error("jpeg: no image data");
  W = width_;
  H = height_;
  C = 3;
  out.assign(static_cast<size_t>(W) * H * 3, 0);
  if (comps_.size() == 1) {
    const Comp& c = comps_[0];
    const int stride = c.bw * 8;
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x) {
        const unsigned char g = c.plane[static_cast<size_t>(y) * stride + x];
        unsigned char* o = &out[(static_cast<size_t>(y) * W + x) * 3];
        o[0] = o[1] = o[2] = g;
      }
    return;
  }
  auto sample = [&](const Comp& c, int x, int y) -> float {
    const int stride = c.bw * 8;
    if (c.h == hmax_ && c.v == vmax_) return c.plane[static_cast<size_t>(y) * stride + x];
    // centred bilinear ("fancy") upsampling of subsampled chroma: 3/4-1/4 taps for 2x, as libjpeg
    const int cw = (W * c.h + hmax_ - 1) / hmax_, ch = (H * c.v + vmax_ - 1) / vmax_;
    const float sx = (x + 0.5f) * c.h / hmax_ - 0.5f, sy = (y + 0.5f) * c.v / vmax_ - 0.5f;
    int x0 = static_cast<int>(std::floor(sx)), y0 = static_cast<int>(std::floor(sy));
    const float fx = sx - x0, fy = sy - y0;
    auto at = [&](int yy, int xx) {
      xx = xx < 0 ? 0 : (xx >= cw ? cw - 1 : xx);
      yy = yy < 0 ? 0 : (yy >= ch ? ch - 1 : yy);
      return static_cast<float>(c.plane[static_cast<size_t>(yy) * stride + xx]);
    };
    return (1 - fy) * ((1 - fx) * at(y0, x0) + fx * at(y0, x0 + 1)) + fy * ((1 - fx) * at(y0 + 1, x0) + fx * at(y0 + 1, x0 + 1));
  };
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      const float Y = sample(comps_[0], x, y), Cb = sample(comps_[1], x, y) - 128.0f,
                  Cr = sample(comps_[2], x, y) - 128.0f;
      float rgb[3] = {Y + 1.402f * Cr, Y - 0.344136f * Cb - 0.714136f * Cr, Y + 1.772f * Cb};
      unsigned char* o = &out[(static_cast<size_t>(y) * W + x) * 3];
      for (int k = 0; k < 3; ++k) {
        const int v = static_cast<int>(std::lround(rgb[k]));
        o[k] = static_cast<unsigned char>(v < 0 ? 0 : (v > 255 ? 255 : v));
      }
    }
}

}  // namespace

bool decode_jpeg(const unsigned char* data, size_t n, std::vector<unsigned char>& rgb, int& w, int& h,
                 std::string* err) {
  try {
    int c = 0;
    Decoder d(data, n);
    d.decode(rgb, w, h, c);
    return true;
  } catch (const std::exception& e) {
    if (err) *err = e.what();
    return false;
  }
}

}  // namespace dcnn_native
