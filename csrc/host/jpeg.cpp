// Baseline JPEG codec (no external image library in this stack).
//
// Decoder: baseline / extended-sequential Huffman JPEG (SOF0/SOF1), 8-bit, 1 or 3 components,
// any h/v sampling up to 2x2, restart intervals.  It follows libjpeg's default decompression path
// (JDCT_ISLOW integer IDCT, "fancy" triangle upsampling, fixed-point YCbCr->RGB tables) so that
// decoded pixels match what cv::imread (libjpeg-turbo) gives the reference demos
// (RAFTStereo/test/main.cpp:13-14) on its test images.
// Encoder: baseline 4:2:0 (colour) / grey JPEG with the Annex K tables scaled by libjpeg's
// quality formula (cv::imwrite default quality 95), ISLOW forward DCT.
//
// Attribution: the integer IDCT / forward DCT follow the structure and fixed-point constants of the
// Independent JPEG Group's jidctint.c / jfdctint.c (libjpeg, Copyright (C) Thomas G. Lane et al.;
// "this software is based in part on the work of the Independent JPEG Group"), re-derived here so
// that decoded pixels are bit-exact with the libjpeg-backed cv::imread the reference uses.
// Every marker field is bounds-checked against its segment (malformed files fail, never overrun).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "sa/imgio.h"

namespace sa {
namespace {

const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                         41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                         30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

inline uint8_t clamp8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

// ---------------------------------------------------------------- ISLOW IDCT (jidctint.c)
constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                  F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
inline int32_t descale(int64_t x, int n) { return (int32_t)((x + ((int64_t)1 << (n - 1))) >> n); }

void idct_islow(const int32_t* in /*dequantised, natural order*/, uint8_t* out, int ostride) {
  int32_t ws[64];
  for (int c = 0; c < 8; ++c) {
    const int32_t* ip = in + c;
    int32_t* wp = ws + c;
    if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
      const int32_t dc = ip[0] * (1 << PASS1_BITS);
      for (int r = 0; r < 8; ++r) wp[8 * r] = dc;
      continue;
    }
    int64_t z2 = ip[16], z3 = ip[48];
    int64_t z1 = (z2 + z3) * F0541;
    int64_t tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
    z2 = ip[0];
    z3 = ip[32];
    int64_t tmp0 = (z2 + z3) * (1 << CONST_BITS), tmp1 = (z2 - z3) * (1 << CONST_BITS);
    const int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = ip[56];
    tmp1 = ip[40];
    tmp2 = ip[24];
    tmp3 = ip[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * F1175;
    tmp0 *= F0298;
    tmp1 *= F2053;
    tmp2 *= F3072;
    tmp3 *= F1501;
    z1 *= -F0899;
    z2 *= -F2562;
    z3 *= -F1961;
    z4 *= -F0390;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    const int sh = CONST_BITS - PASS1_BITS;
    wp[0] = descale(t10 + tmp3, sh);
    wp[56] = descale(t10 - tmp3, sh);
    wp[8] = descale(t11 + tmp2, sh);
    wp[48] = descale(t11 - tmp2, sh);
    wp[16] = descale(t12 + tmp1, sh);
    wp[40] = descale(t12 - tmp1, sh);
    wp[24] = descale(t13 + tmp0, sh);
    wp[32] = descale(t13 - tmp0, sh);
  }
  for (int r = 0; r < 8; ++r) {
    const int32_t* wp = ws + 8 * r;
    uint8_t* op = out + r * ostride;
    const int sh = CONST_BITS + PASS1_BITS + 3;
    if (!wp[1] && !wp[2] && !wp[3] && !wp[4] && !wp[5] && !wp[6] && !wp[7]) {
      const uint8_t v = clamp8(descale(wp[0], PASS1_BITS + 3) + 128);
      for (int c = 0; c < 8; ++c) op[c] = v;
      continue;
    }
    int64_t z2 = wp[2], z3 = wp[6];
    int64_t z1 = (z2 + z3) * F0541;
    int64_t tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
    int64_t tmp0 = ((int64_t)wp[0] + wp[4]) * (1 << CONST_BITS);
    int64_t tmp1 = ((int64_t)wp[0] - wp[4]) * (1 << CONST_BITS);
    const int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = wp[7];
    tmp1 = wp[5];
    tmp2 = wp[3];
    tmp3 = wp[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * F1175;
    tmp0 *= F0298;
    tmp1 *= F2053;
    tmp2 *= F3072;
    tmp3 *= F1501;
    z1 *= -F0899;
    z2 *= -F2562;
    z3 *= -F1961;
    z4 *= -F0390;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    op[0] = clamp8(descale(t10 + tmp3, sh) + 128);
    op[7] = clamp8(descale(t10 - tmp3, sh) + 128);
    op[1] = clamp8(descale(t11 + tmp2, sh) + 128);
    op[6] = clamp8(descale(t11 - tmp2, sh) + 128);
    op[2] = clamp8(descale(t12 + tmp1, sh) + 128);
    op[5] = clamp8(descale(t12 - tmp1, sh) + 128);
    op[3] = clamp8(descale(t13 + tmp0, sh) + 128);
    op[4] = clamp8(descale(t13 - tmp0, sh) + 128);
  }
}

// ---------------------------------------------------------------- Huffman decoding
struct Huff {
  uint8_t bits[17] = {};
  uint8_t vals[256] = {};
  int32_t maxcode[18] = {}, valptr[17] = {}, mincode[17] = {};
  bool present = false;
  void build() {
    int code = 0, k = 0;
    for (int l = 1; l <= 16; ++l) {
      valptr[l] = k;
      mincode[l] = code;
      code += bits[l];
      k += bits[l];
      maxcode[l] = bits[l] ? code - 1 : -1;
      code <<= 1;
    }
    maxcode[17] = 0x7fffffff;
    present = true;
  }
};

struct BitReader {
  const uint8_t* p;
  const uint8_t* end;
  uint32_t acc = 0;
  int n = 0;
  bool marker_hit = false;
  int fill_byte() {
    if (marker_hit || p >= end) return 0;
    uint8_t b = *p;
    if (b == 0xFF) {
      uint8_t nx = p + 1 < end ? p[1] : 0;
      if (nx == 0x00) {
        p += 2;
        return 0xFF;
      }
      marker_hit = true;  // RST/EOI: feed zeros
      return 0;
    }
    ++p;
    return b;
  }
  uint32_t peek(int k) {
    while (n < k) {
      acc = (acc << 8) | (uint32_t)fill_byte();
      n += 8;
    }
    return (acc >> (n - k)) & ((1u << k) - 1);
  }
  void skip(int k) { n -= k; }
  int bit() {
    uint32_t b = peek(1);
    skip(1);
    return (int)b;
  }
  int bits(int k) {
    if (k == 0) return 0;
    uint32_t b = peek(k);
    skip(k);
    return (int)b;
  }
  void reset() {
    acc = 0;
    n = 0;
    marker_hit = false;
  }
};

int decode_huff(BitReader& br, const Huff& h) {
  int code = br.bit();
  int l = 1;
  while (l <= 16 && code > h.maxcode[l]) {
    code = (code << 1) | br.bit();
    ++l;
  }
  if (l > 16) return 0;
  return h.vals[h.valptr[l] + code - h.mincode[l]];
}

inline int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }

struct Comp {
  int id, h, v, tq, td = 0, ta = 0;
  int bw, bh;  // blocks per line / column (padded to MCU)
  std::vector<uint8_t> plane;
  int pred = 0;
};

// libjpeg fixed-point YCbCr -> RGB tables (jdcolor.c)
struct YccTables {
  int cr_r[256], cb_b[256];
  int32_t cr_g[256], cb_g[256];
  YccTables() {
    const int SB = 16;
    const int32_t HALF = 1 << (SB - 1);
    auto FIX = [](double x) { return (int32_t)(x * (1 << 16) + 0.5); };
    for (int i = 0; i < 256; ++i) {
      const int x = i - 128;
      cr_r[i] = (int)((FIX(1.40200) * x + HALF) >> SB);
      cb_b[i] = (int)((FIX(1.77200) * x + HALF) >> SB);
      cr_g[i] = -FIX(0.71414) * x;
      cb_g[i] = -FIX(0.34414) * x + HALF;
    }
  }
};

// fancy upsampling of one component plane (cw x ch) to (W x H) for factors 1 or 2
void upsample(const Comp& c, int cw, int ch, int fx, int fy, int W, int H, std::vector<uint8_t>& out) {
  out.assign((size_t)W * H, 0);
  const int stride = c.bw * 8;
  auto in = [&](int y, int x) -> int {
    y = std::min(std::max(y, 0), ch - 1);
    x = std::min(std::max(x, 0), cw - 1);
    return c.plane[(size_t)y * stride + x];
  };
  if (fx == 1 && fy == 1) {
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x) out[(size_t)y * W + x] = (uint8_t)in(y, x);
    return;
  }
  if (fx == 2 && fy == 1) {  // h2v1_fancy_upsample
    for (int y = 0; y < H; ++y) {
      for (int x = 0; x < W; ++x) {
        const int sx = x >> 1;
        int v;
        if (cw == 1) v = in(y, 0);
        else if ((x & 1) == 0) v = sx == 0 ? in(y, 0) : (in(y, sx) * 3 + in(y, sx - 1) + 1) >> 2;
        else v = sx == cw - 1 ? in(y, cw - 1) : (in(y, sx) * 3 + in(y, sx + 1) + 2) >> 2;
        out[(size_t)y * W + x] = (uint8_t)v;
      }
    }
    return;
  }
  if (fx == 2 && fy == 2) {  // h2v2_fancy_upsample
    for (int y = 0; y < H; ++y) {
      const int sy = y >> 1;
      const int ny = (y & 1) ? sy + 1 : sy - 1;  // nearer neighbouring input row
      auto colsum = [&](int x) { return in(sy, x) * 3 + in(ny, x); };
      for (int x = 0; x < W; ++x) {
        const int sx = x >> 1;
        const int cs = colsum(sx);
        int v;
        if ((x & 1) == 0) v = sx == 0 ? (cs * 4 + 8) >> 4 : (cs * 3 + colsum(sx - 1) + 8) >> 4;
        else v = sx == cw - 1 ? (cs * 4 + 7) >> 4 : (cs * 3 + colsum(sx + 1) + 7) >> 4;
        out[(size_t)y * W + x] = (uint8_t)v;
      }
    }
    return;
  }
  // generic replication for other factors
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) out[(size_t)y * W + x] = (uint8_t)in(y / fy, x / fx);
}

}  // namespace

bool jpeg_decode(const uint8_t* data, size_t size, Image& img, std::string* err) {
  auto fail = [&](const char* m) {
    if (err) *err = m;
    return false;
  };
  if (size < 4 || data[0] != 0xFF || data[1] != 0xD8) return fail("not a JPEG");
  uint16_t qt[4][64] = {};
  Huff hdc[4], hac[4];
  std::vector<Comp> comps;
  int W = 0, H = 0, restart = 0, hmax = 1, vmax = 1;
  bool adobe_rgb = false;
  const uint8_t* p = data + 2;
  const uint8_t* end = data + size;
  auto u16 = [](const uint8_t* q) { return (q[0] << 8) | q[1]; };
  while (p + 4 <= end) {
    if (p[0] != 0xFF) {
      ++p;
      continue;
    }
    const uint8_t m = p[1];
    p += 2;
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01 || m == 0xFF) continue;
    if (m == 0xD9) break;
    const int len = u16(p);
    const uint8_t* seg = p + 2;
    // every field below is read from the file: bound each read by the segment it belongs to
    if (len < 2 || p + len > end) return fail("truncated segment");
    const uint8_t* sege = p + len;
    if (m == 0xDB) {
      const uint8_t* q = seg;
      while (q < sege) {
        const int pq = q[0] >> 4, tq = q[0] & 15;
        if (pq > 1 || tq > 3) return fail("bad DQT table");
        ++q;
        if (q + (pq ? 128 : 64) > sege) return fail("truncated DQT");
        for (int i = 0; i < 64; ++i) {
          qt[tq][kZigzag[i]] = pq ? (uint16_t)u16(q + 2 * i) : q[i];
        }
        q += pq ? 128 : 64;
      }
    } else if (m == 0xC4) {
      const uint8_t* q = seg;
      while (q < sege) {
        if (q + 17 > sege) return fail("truncated DHT");
        const int tc = q[0] >> 4, th = q[0] & 15;
        if (tc > 1 || th > 3) return fail("bad DHT table");
        Huff& h = tc ? hac[th] : hdc[th];
        int tot = 0;
        for (int i = 1; i <= 16; ++i) {
          h.bits[i] = q[i];
          tot += q[i];
        }
        if (tot > 256 || q + 17 + tot > sege) return fail("bad DHT code counts");
        std::memcpy(h.vals, q + 17, tot);
        h.build();
        q += 17 + tot;
      }
    } else if (m == 0xC0 || m == 0xC1) {
      if (len < 8) return fail("truncated SOF");
      if (seg[0] != 8) return fail("only 8-bit JPEG supported");
      H = u16(seg + 1);
      W = u16(seg + 3);
      const int nc = seg[5];
      if (H <= 0 || W <= 0) return fail("bad image size");
      if (nc != 1 && nc != 3) return fail("only 1- or 3-component JPEG supported");
      if (8 + 3 * nc > len) return fail("truncated SOF");
      comps.clear();
      hmax = vmax = 1;
      for (int i = 0; i < nc; ++i) {
        Comp c;
        c.id = seg[6 + 3 * i];
        c.h = seg[7 + 3 * i] >> 4;
        c.v = seg[7 + 3 * i] & 15;
        c.tq = seg[8 + 3 * i];
        if (c.h < 1 || c.h > 2 || c.v < 1 || c.v > 2) return fail("sampling factors above 2x2 not supported");
        if (c.tq > 3) return fail("bad quantisation table index");
        hmax = std::max(hmax, c.h);
        vmax = std::max(vmax, c.v);
        comps.push_back(c);
      }
    } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return fail("progressive / arithmetic / lossless JPEG not supported");
    } else if (m == 0xDD) {
      if (len < 4) return fail("truncated DRI");
      restart = u16(seg);
    } else if (m == 0xEE) {
      if (len >= 12 && std::memcmp(seg, "Adobe", 5) == 0) adobe_rgb = seg[11] == 0;
    } else if (m == 0xDA) {
      if (comps.empty()) return fail("SOS before SOF");
      if (len < 3) return fail("truncated SOS");
      const int ns = seg[0];
      if (ns < 1 || ns > (int)comps.size() || 3 + 2 * ns > len) return fail("bad SOS component count");
      std::vector<int> sc(ns, -1);
      for (int i = 0; i < ns; ++i) {
        const int cid = seg[1 + 2 * i];
        for (size_t k = 0; k < comps.size(); ++k)
          if (comps[k].id == cid) {
            sc[i] = (int)k;
            comps[k].td = seg[2 + 2 * i] >> 4;
            comps[k].ta = seg[2 + 2 * i] & 15;
            if (comps[k].td > 3 || comps[k].ta > 3) return fail("bad Huffman table index");
            if (!hdc[comps[k].td].present || !hac[comps[k].ta].present) return fail("undefined Huffman table");
          }
        if (sc[i] < 0) return fail("SOS names an unknown component");
      }
      const int mcux = (W + 8 * hmax - 1) / (8 * hmax), mcuy = (H + 8 * vmax - 1) / (8 * vmax);
      for (auto& c : comps) {
        c.bw = mcux * c.h;
        c.bh = mcuy * c.v;
        c.plane.assign((size_t)c.bw * 8 * c.bh * 8, 0);
        c.pred = 0;
      }
      const uint8_t* ep = p + len;
      BitReader br{ep, end};
      int32_t blk[64];
      int mcu_count = 0;
      const bool single = ns == 1;
      const int total_mcus = single ? ((W * comps[sc[0]].h / hmax + 7) / 8) * ((H * comps[sc[0]].v / vmax + 7) / 8)
                                    : mcux * mcuy;
      const int single_bw = single ? (W * comps[sc[0]].h / hmax + 7) / 8 : 0;
      for (int mcu = 0; mcu < total_mcus; ++mcu) {
        if (restart && mcu_count == restart) {
          // align to the RST marker
          br.reset();
          while (br.p + 1 < end && !(br.p[0] == 0xFF && br.p[1] >= 0xD0 && br.p[1] <= 0xD7)) ++br.p;
          if (br.p + 1 < end) br.p += 2;
          for (auto& c : comps) c.pred = 0;
          mcu_count = 0;
        }
        ++mcu_count;
        for (int s = 0; s < ns; ++s) {
          Comp& c = comps[sc[s]];
          const int nby = single ? 1 : c.v, nbx = single ? 1 : c.h;
          for (int by = 0; by < nby; ++by)
            for (int bx = 0; bx < nbx; ++bx) {
              std::fill(blk, blk + 64, 0);
              const int t = decode_huff(br, hdc[c.td]);
              if (t > 15) return fail("corrupt DC coefficient");
              const int diff = t ? extend(br.bits(t), t) : 0;
              c.pred += diff;
              blk[0] = c.pred * qt[c.tq][0];
              for (int k = 1; k < 64;) {
                const int rs = decode_huff(br, hac[c.ta]);
                const int r = rs >> 4, sz = rs & 15;
                if (sz == 0) {
                  if (r != 15) break;
                  k += 16;
                  continue;
                }
                k += r;
                if (k > 63) break;
                const int z = kZigzag[k];
                blk[z] = extend(br.bits(sz), sz) * qt[c.tq][z];
                ++k;
              }
              int row, col;
              if (single) {
                row = mcu / single_bw;
                col = mcu % single_bw;
              } else {
                row = (mcu / mcux) * c.v + by;
                col = (mcu % mcux) * c.h + bx;
              }
              idct_islow(blk, &c.plane[((size_t)row * 8) * c.bw * 8 + col * 8], c.bw * 8);
            }
        }
      }
      // continue scanning after the entropy-coded data
      p = br.p;
      while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) ++p;
      continue;
    }
    p += len;
  }
  if (W == 0 || comps.empty()) return fail("no image data");
  const int nc = (int)comps.size();
  img.width = W;
  img.height = H;
  img.channels = nc == 1 ? 1 : 3;
  img.data.assign((size_t)W * H * img.channels, 0);
  std::vector<std::vector<uint8_t>> full(nc);
  for (int k = 0; k < nc; ++k) {
    const Comp& c = comps[k];
    const int cw = (W * c.h + hmax - 1) / hmax, ch = (H * c.v + vmax - 1) / vmax;
    upsample(c, cw, ch, hmax / c.h, vmax / c.v, W, H, full[k]);
  }
  if (nc == 1) {
    img.data = full[0];
    return true;
  }
  static const YccTables T;
  for (size_t i = 0; i < (size_t)W * H; ++i) {
    const int y = full[0][i], cb = full[1][i], cr = full[2][i];
    uint8_t* o = &img.data[i * 3];
    if (adobe_rgb) {  // stored as RGB -> BGR
      o[0] = (uint8_t)cr;
      o[1] = (uint8_t)cb;
      o[2] = (uint8_t)y;
      continue;
    }
    // BGR order (cv::imread convention)
    o[2] = clamp8(y + T.cr_r[cr]);
    o[1] = clamp8(y + (int)((T.cb_g[cb] + T.cr_g[cr]) >> 16));
    o[0] = clamp8(y + T.cb_b[cb]);
  }
  return true;
}

// ================================================================ encoder
namespace {

const uint8_t kStdLumQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                              14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                              18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                              49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const uint8_t kStdChrQ[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99,
                              99, 99, 47, 66, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                              99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
const uint8_t kDcLumBits[17] = {0, 0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcLumVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kDcChrBits[17] = {0, 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcChrVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kAcLumBits[17] = {0, 0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kAcLumVal[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71, 0x14,
    0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09,
    0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a,
    0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65,
    0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88,
    0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9,
    0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea,
    0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t kAcChrBits[17] = {0, 0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kAcChrVal[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22, 0x32,
    0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16,
    0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39,
    0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86,
    0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8,
    0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9,
    0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

struct HuffEnc {
  uint16_t code[256] = {};
  uint8_t size[256] = {};
  void build(const uint8_t* bits, const uint8_t* vals) {
    int k = 0, c = 0;
    for (int l = 1; l <= 16; ++l) {
      for (int i = 0; i < bits[l]; ++i) {
        code[vals[k]] = (uint16_t)c++;
        size[vals[k]] = (uint8_t)l;
        ++k;
      }
      c <<= 1;
    }
  }
};

struct BitWriter {
  std::vector<uint8_t>& out;
  uint32_t acc = 0;
  int n = 0;
  void put(uint32_t v, int k) {
    acc = (acc << k) | (v & ((1u << k) - 1));
    n += k;
    while (n >= 8) {
      const uint8_t b = (uint8_t)(acc >> (n - 8));
      out.push_back(b);
      if (b == 0xFF) out.push_back(0);
      n -= 8;
    }
  }
  void flush() {
    if (n > 0) put(0x7F, 8 - n);  // pad with ones
  }
};

// ISLOW forward DCT (jfdctint.c); output scaled by 8
void fdct_islow(int32_t* d) {
  constexpr int CB = 13, P1 = 2;
  for (int r = 0; r < 8; ++r) {
    int32_t* p = d + 8 * r;
    int64_t tmp0 = p[0] + p[7], tmp7 = p[0] - p[7], tmp1 = p[1] + p[6], tmp6 = p[1] - p[6];
    int64_t tmp2 = p[2] + p[5], tmp5 = p[2] - p[5], tmp3 = p[3] + p[4], tmp4 = p[3] - p[4];
    int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    p[0] = (int32_t)((t10 + t11) * (1 << P1));
    p[4] = (int32_t)((t10 - t11) * (1 << P1));
    int64_t z1 = (t12 + t13) * F0541;
    p[2] = descale(z1 + t13 * F0765, CB - P1);
    p[6] = descale(z1 + t12 * -F1847, CB - P1);
    int64_t z1b = tmp4 + tmp7, z2 = tmp5 + tmp6, z3 = tmp4 + tmp6, z4 = tmp5 + tmp7;
    int64_t z5 = (z3 + z4) * F1175;
    tmp4 *= F0298;
    tmp5 *= F2053;
    tmp6 *= F3072;
    tmp7 *= F1501;
    z1b *= -F0899;
    z2 *= -F2562;
    z3 *= -F1961;
    z4 *= -F0390;
    z3 += z5;
    z4 += z5;
    p[7] = descale(tmp4 + z1b + z3, CB - P1);
    p[5] = descale(tmp5 + z2 + z4, CB - P1);
    p[3] = descale(tmp6 + z2 + z3, CB - P1);
    p[1] = descale(tmp7 + z1b + z4, CB - P1);
  }
  for (int c = 0; c < 8; ++c) {
    int32_t* p = d + c;
    int64_t tmp0 = p[0] + p[56], tmp7 = p[0] - p[56], tmp1 = p[8] + p[48], tmp6 = p[8] - p[48];
    int64_t tmp2 = p[16] + p[40], tmp5 = p[16] - p[40], tmp3 = p[24] + p[32], tmp4 = p[24] - p[32];
    int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    p[0] = descale(t10 + t11, P1);
    p[32] = descale(t10 - t11, P1);
    int64_t z1 = (t12 + t13) * F0541;
    p[16] = descale(z1 + t13 * F0765, CB + P1);
    p[48] = descale(z1 + t12 * -F1847, CB + P1);
    int64_t z1b = tmp4 + tmp7, z2 = tmp5 + tmp6, z3 = tmp4 + tmp6, z4 = tmp5 + tmp7;
    int64_t z5 = (z3 + z4) * F1175;
    tmp4 *= F0298;
    tmp5 *= F2053;
    tmp6 *= F3072;
    tmp7 *= F1501;
    z1b *= -F0899;
    z2 *= -F2562;
    z3 *= -F1961;
    z4 *= -F0390;
    z3 += z5;
    z4 += z5;
    p[56] = descale(tmp4 + z1b + z3, CB + P1);
    p[40] = descale(tmp5 + z2 + z4, CB + P1);
    p[24] = descale(tmp6 + z2 + z3, CB + P1);
    p[8] = descale(tmp7 + z1b + z4, CB + P1);
  }
}

void encode_block(BitWriter& bw, int32_t* blk, const uint16_t* q, int& pred, const HuffEnc& dc, const HuffEnc& ac) {
  fdct_islow(blk);
  int zz[64];
  for (int i = 0; i < 64; ++i) {
    const int32_t v = blk[kZigzag[i]];
    const int32_t d = q[kZigzag[i]] * 8;  // fdct output is scaled by 8
    zz[i] = v >= 0 ? (v + d / 2) / d : -((-v + d / 2) / d);
  }
  auto nbits = [](int v) {
    v = v < 0 ? -v : v;
    int n = 0;
    while (v) {
      ++n;
      v >>= 1;
    }
    return n;
  };
  int diff = zz[0] - pred;
  pred = zz[0];
  int n = nbits(diff);
  bw.put(dc.code[n], dc.size[n]);
  if (n) bw.put(diff < 0 ? diff - 1 : diff, n);
  int run = 0;
  for (int k = 1; k < 64; ++k) {
    if (zz[k] == 0) {
      ++run;
      continue;
    }
    while (run > 15) {
      bw.put(ac.code[0xF0], ac.size[0xF0]);
      run -= 16;
    }
    n = nbits(zz[k]);
    const int sym = (run << 4) | n;
    bw.put(ac.code[sym], ac.size[sym]);
    bw.put(zz[k] < 0 ? zz[k] - 1 : zz[k], n);
    run = 0;
  }
  if (run) bw.put(ac.code[0], ac.size[0]);
}

}  // namespace

bool jpeg_encode(const Image& img, int quality, std::vector<uint8_t>& out) {
  if (img.channels != 1 && img.channels != 3) return false;
  quality = std::min(100, std::max(1, quality));
  const int scale = quality < 50 ? 5000 / quality : 200 - quality * 2;
  uint16_t ql[64], qc[64];
  for (int i = 0; i < 64; ++i) {
    ql[i] = (uint16_t)std::min(255, std::max(1, (kStdLumQ[i] * scale + 50) / 100));
    qc[i] = (uint16_t)std::min(255, std::max(1, (kStdChrQ[i] * scale + 50) / 100));
  }
  const int W = img.width, H = img.height;
  const bool color = img.channels == 3;
  out.clear();
  auto put16 = [&](int v) {
    out.push_back((uint8_t)(v >> 8));
    out.push_back((uint8_t)v);
  };
  out.insert(out.end(), {0xFF, 0xD8, 0xFF, 0xE0});
  put16(16);
  out.insert(out.end(), {'J', 'F', 'I', 'F', 0, 1, 1, 0, 0, 1, 0, 1, 0, 0});
  auto dqt = [&](int id, const uint16_t* q) {
    out.insert(out.end(), {0xFF, 0xDB});
    put16(67);
    out.push_back((uint8_t)id);
    for (int i = 0; i < 64; ++i) out.push_back((uint8_t)q[kZigzag[i]]);
  };
  dqt(0, ql);
  if (color) dqt(1, qc);
  out.insert(out.end(), {0xFF, 0xC0});
  put16(color ? 17 : 11);
  out.push_back(8);
  put16(H);
  put16(W);
  out.push_back(color ? 3 : 1);
  out.insert(out.end(), {1, (uint8_t)(color ? 0x22 : 0x11), 0});
  if (color) out.insert(out.end(), {2, 0x11, 1, 3, 0x11, 1});
  auto dht = [&](int cls_id, const uint8_t* bits, const uint8_t* vals) {
    int tot = 0;
    for (int i = 1; i <= 16; ++i) tot += bits[i];
    out.insert(out.end(), {0xFF, 0xC4});
    put16(19 + tot);
    out.push_back((uint8_t)cls_id);
    for (int i = 1; i <= 16; ++i) out.push_back(bits[i]);
    out.insert(out.end(), vals, vals + tot);
  };
  dht(0x00, kDcLumBits, kDcLumVal);
  dht(0x10, kAcLumBits, kAcLumVal);
  if (color) {
    dht(0x01, kDcChrBits, kDcChrVal);
    dht(0x11, kAcChrBits, kAcChrVal);
  }
  out.insert(out.end(), {0xFF, 0xDA});
  put16(color ? 12 : 8);
  out.push_back(color ? 3 : 1);
  out.insert(out.end(), {1, 0x00});
  if (color) out.insert(out.end(), {2, 0x11, 3, 0x11});
  out.insert(out.end(), {0, 63, 0});

  HuffEnc dcl, acl, dcc, acc;
  dcl.build(kDcLumBits, kDcLumVal);
  acl.build(kAcLumBits, kAcLumVal);
  dcc.build(kDcChrBits, kDcChrVal);
  acc.build(kAcChrBits, kAcChrVal);
  BitWriter bw{out};
  // colour conversion (jccolor.c fixed point) with edge replication
  auto pix = [&](int y, int x, int c) -> int {
    y = std::min(y, H - 1);
    x = std::min(x, W - 1);
    return img.data[((size_t)y * W + x) * img.channels + c];
  };
  auto ycc = [&](int y, int x, int* Y, int* Cb, int* Cr) {
    if (!color) {
      *Y = pix(y, x, 0);
      return;
    }
    const int b = pix(y, x, 0), g = pix(y, x, 1), r = pix(y, x, 2);
    const int32_t S = 1 << 16, HALF = 1 << 15;
    auto F = [&](double v) { return (int32_t)(v * S + 0.5); };
    *Y = (int)((F(0.29900) * r + F(0.58700) * g + F(0.11400) * b + HALF) >> 16);
    *Cb = (int)((-F(0.16874) * r - F(0.33126) * g + F(0.5) * b + (128 << 16) + HALF - 1) >> 16);
    *Cr = (int)((F(0.5) * r - F(0.41869) * g - F(0.08131) * b + (128 << 16) + HALF - 1) >> 16);
  };
  int py = 0, pcb = 0, pcr = 0;
  const int mcu = color ? 16 : 8;
  int32_t blk[64];
  for (int my = 0; my < (H + mcu - 1) / mcu; ++my)
    for (int mx = 0; mx < (W + mcu - 1) / mcu; ++mx) {
      int Yb[16][16], Cbb[16][16], Crb[16][16];
      for (int y = 0; y < mcu; ++y)
        for (int x = 0; x < mcu; ++x) ycc(my * mcu + y, mx * mcu + x, &Yb[y][x], &Cbb[y][x], &Crb[y][x]);
      const int nb = color ? 2 : 1;
      for (int by = 0; by < nb; ++by)
        for (int bx = 0; bx < nb; ++bx) {
          for (int i = 0; i < 64; ++i) blk[i] = Yb[by * 8 + i / 8][bx * 8 + i % 8] - 128;
          encode_block(bw, blk, ql, py, dcl, acl);
        }
      if (color) {
        for (int c = 0; c < 2; ++c) {
          int (*src)[16] = c == 0 ? Cbb : Crb;
          for (int i = 0; i < 64; ++i) {
            const int y = (i / 8) * 2, x = (i % 8) * 2;
            const int bias = (i % 2) ? 2 : 1;  // jcsample.c h2v2 alternating bias
            blk[i] = ((src[y][x] + src[y][x + 1] + src[y + 1][x] + src[y + 1][x + 1] + bias) >> 2) - 128;
          }
          encode_block(bw, blk, qc, c == 0 ? pcb : pcr, dcc, acc);
        }
      }
    }
  bw.flush();
  out.insert(out.end(), {0xFF, 0xD9});
  return true;
}

}  // namespace sa
