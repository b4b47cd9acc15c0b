// PNG decode / encode on zlib (8/16-bit grey, grey+alpha, RGB, RGBA, palette; non-interlaced).
#include <zlib.h>

#include <cstring>
#include <string>
#include <vector>

#include "sa/imgio.h"

namespace sa {
namespace {
uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
void put32(std::vector<uint8_t>& o, uint32_t v) {
  o.push_back((uint8_t)(v >> 24));
  o.push_back((uint8_t)(v >> 16));
  o.push_back((uint8_t)(v >> 8));
  o.push_back((uint8_t)v);
}
int paeth(int a, int b, int c) {
  int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}
}  // namespace

bool png_decode(const uint8_t* d, size_t n, Image& img, std::string* err) {
  auto fail = [&](const char* m) {
    if (err) *err = m;
    return false;
  };
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (n < 8 || std::memcmp(d, sig, 8) != 0) return fail("not a PNG");
  size_t p = 8;
  uint32_t W = 0, H = 0;
  int depth = 0, ctype = 0, interlace = 0;
  std::vector<uint8_t> idat, palette;
  while (p + 8 <= n) {
    const uint32_t len = be32(d + p);
    const char* type = reinterpret_cast<const char*>(d + p + 4);
    const uint8_t* body = d + p + 8;
    if (p + 12 + len > n) return fail("truncated PNG");
    if (!std::memcmp(type, "IHDR", 4)) {
      if (len != 13) return fail("bad IHDR");
      W = be32(body);
      H = be32(body + 4);
      depth = body[8];
      ctype = body[9];
      interlace = body[12];
    } else if (!std::memcmp(type, "PLTE", 4)) {
      palette.assign(body, body + len);
    } else if (!std::memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), body, body + len);
    } else if (!std::memcmp(type, "IEND", 4)) {
      break;
    }
    p += 12 + len;
  }
  if (interlace) return fail("interlaced PNG not supported");
  // header fields come from the file: bound them before any size arithmetic
  constexpr uint32_t kMaxDim = 1u << 15;
  if (W == 0 || H == 0 || W > kMaxDim || H > kMaxDim) return fail("PNG dimensions out of range");
  if (ctype != 0 && ctype != 2 && ctype != 3 && ctype != 4 && ctype != 6) return fail("bad PNG colour type");
  const bool sub8 = depth == 1 || depth == 2 || depth == 4;
  if (sub8 ? (ctype != 0 && ctype != 3) : (depth != 8 && !(depth == 16 && ctype != 3)))
    return fail("unsupported PNG bit depth for this colour type");
  const int spp = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : 4;
  const int bpp = sub8 ? 1 : spp * depth / 8;  // filter unit (bytes), >= 1
  const size_t stride = sub8 ? ((size_t)W * depth + 7) / 8 : (size_t)W * bpp;  // <= 2^15 * 8 bytes
  std::vector<uint8_t> raw((stride + 1) * H);
  uLongf rl = (uLongf)raw.size();
  if (uncompress(raw.data(), &rl, idat.data(), (uLong)idat.size()) != Z_OK || rl != raw.size())
    return fail("PNG inflate failed");
  std::vector<uint8_t> px(stride * H);
  for (uint32_t y = 0; y < H; ++y) {
    const uint8_t f = raw[y * (stride + 1)];
    const uint8_t* s = &raw[y * (stride + 1) + 1];
    uint8_t* o = &px[y * stride];
    const uint8_t* up = y ? &px[(y - 1) * stride] : nullptr;
    for (size_t i = 0; i < stride; ++i) {
      const int a = i >= (size_t)bpp ? o[i - bpp] : 0, b = up ? up[i] : 0, c = (up && i >= (size_t)bpp) ? up[i - bpp] : 0;
      int v = s[i];
      switch (f) {
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: v += paeth(a, b, c); break;
        default: break;
      }
      o[i] = (uint8_t)v;
    }
  }
  img.width = (int)W;
  img.height = (int)H;
  const bool grey = ctype == 0 || ctype == 4;
  img.channels = grey ? 1 : 3;
  img.data.assign((size_t)W * H * img.channels, 0);
  const int bs = depth / 8;
  for (size_t i = 0; i < (size_t)W * H; ++i) {
    if (sub8) {  // packed 1/2/4-bit samples, MSB first, rows byte-aligned
      const size_t y = i / W, x = i % W;
      const size_t bit = x * depth;
      const int v = (px[y * stride + bit / 8] >> (8 - depth - (int)(bit % 8))) & ((1 << depth) - 1);
      if (ctype == 3) {
        for (int k = 0; k < 3; ++k)
          img.data[i * 3 + k] = palette.size() > (size_t)v * 3 + (2 - k) ? palette[v * 3 + (2 - k)] : 0;
      } else {
        img.data[i] = (uint8_t)(v * 255 / ((1 << depth) - 1));
      }
      continue;
    }
    const uint8_t* s = &px[i * bpp];
    auto sample = [&](int k) { return s[k * bs]; };  // 16-bit: keep the MSB (cv::imread 8-bit path)
    if (ctype == 3) {
      const int idx = s[0];
      img.data[i * 3 + 0] = palette.size() > (size_t)idx * 3 + 2 ? palette[idx * 3 + 2] : 0;
      img.data[i * 3 + 1] = palette.size() > (size_t)idx * 3 + 1 ? palette[idx * 3 + 1] : 0;
      img.data[i * 3 + 2] = palette.size() > (size_t)idx * 3 ? palette[idx * 3] : 0;
    } else if (grey) {
      img.data[i] = sample(0);
    } else {
      img.data[i * 3 + 0] = sample(2);
      img.data[i * 3 + 1] = sample(1);
      img.data[i * 3 + 2] = sample(0);
    }
  }
  return true;
}

bool png_encode(const Image& img, std::vector<uint8_t>& out) {
  const int cn = img.channels;
  if (cn != 1 && cn != 3) return false;
  const size_t stride = (size_t)img.width * cn;
  std::vector<uint8_t> raw((stride + 1) * img.height);
  for (int y = 0; y < img.height; ++y) {
    raw[y * (stride + 1)] = 1;  // Sub filter
    const uint8_t* s = &img.data[y * stride];
    uint8_t* o = &raw[y * (stride + 1) + 1];
    for (int x = 0; x < img.width; ++x)
      for (int c = 0; c < cn; ++c) {
        const int src_c = cn == 3 ? 2 - c : 0;  // BGR -> RGB
        const int v = s[x * cn + src_c];
        const int left = x ? s[(x - 1) * cn + src_c] : 0;
        o[x * cn + c] = (uint8_t)(v - left);
      }
  }
  uLongf cl = compressBound((uLong)raw.size());
  std::vector<uint8_t> comp(cl);
  if (compress2(comp.data(), &cl, raw.data(), (uLong)raw.size(), 3) != Z_OK) return false;
  comp.resize(cl);
  out.assign({137, 80, 78, 71, 13, 10, 26, 10});
  auto chunk = [&](const char* type, const std::vector<uint8_t>& body) {
    put32(out, (uint32_t)body.size());
    size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), body.begin(), body.end());
    put32(out, (uint32_t)crc32(0, out.data() + start, (uInt)(out.size() - start)));
  };
  std::vector<uint8_t> ihdr;
  put32(ihdr, (uint32_t)img.width);
  put32(ihdr, (uint32_t)img.height);
  ihdr.insert(ihdr.end(), {8, (uint8_t)(cn == 3 ? 2 : 0), 0, 0, 0});
  chunk("IHDR", ihdr);
  chunk("IDAT", comp);
  chunk("IEND", {});
  return true;
}

}  // namespace sa
