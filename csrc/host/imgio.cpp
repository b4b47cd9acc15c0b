// imread / imwrite / colour maps / point-cloud text output (see sa/imgio.h).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <iterator>

#include "sa/imgio.h"

namespace sa {

static std::string lower_ext(const std::string& path) {
  size_t d = path.find_last_of('.');
  std::string e = d == std::string::npos ? "" : path.substr(d + 1);
  for (auto& c : e) c = (char)std::tolower((unsigned char)c);
  return e;
}

static bool read_file(const std::string& path, std::vector<uint8_t>& buf) {
  std::ifstream f(path, std::ios::binary);
  if (!f.good()) return false;
  buf.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return true;
}

static bool pnm_decode(const std::vector<uint8_t>& b, Image& img) {
  if (b.size() < 3 || b[0] != 'P' || (b[1] != '5' && b[1] != '6')) return false;
  size_t p = 2;
  int vals[3], k = 0;
  while (k < 3 && p < b.size()) {
    while (p < b.size() && std::isspace(b[p])) ++p;
    if (p < b.size() && b[p] == '#') {
      while (p < b.size() && b[p] != '\n') ++p;
      continue;
    }
    int v = 0;
    while (p < b.size() && std::isdigit(b[p])) v = v * 10 + (b[p++] - '0');
    vals[k++] = v;
  }
  ++p;
  img.width = vals[0];
  img.height = vals[1];
  img.channels = b[1] == '6' ? 3 : 1;
  const size_t n = (size_t)img.width * img.height * img.channels;
  if (p + n > b.size()) return false;
  img.data.assign(b.begin() + p, b.begin() + p + n);
  if (img.channels == 3)
    for (size_t i = 0; i < n; i += 3) std::swap(img.data[i], img.data[i + 2]);  // RGB -> BGR
  return true;
}

Mat imread(const std::string& path, bool grayscale) {
  std::vector<uint8_t> buf;
  if (!read_file(path, buf)) return Mat();
  Image img;
  bool ok = false;
  if (buf.size() > 2 && buf[0] == 0xFF && buf[1] == 0xD8) ok = jpeg_decode(buf.data(), buf.size(), img);
  else if (buf.size() > 8 && buf[0] == 137 && buf[1] == 'P') ok = png_decode(buf.data(), buf.size(), img);
  else ok = pnm_decode(buf, img);
  if (!ok) return Mat();
  Mat m(img.height, img.width, img.channels == 3 ? SA_8UC3 : SA_8UC1);
  std::memcpy(m.data, img.data.data(), img.data.size());
  if (grayscale && img.channels == 3) return bgr2gray(m);
  if (!grayscale && img.channels == 1) {
    Mat c(img.height, img.width, SA_8UC3);
    for (size_t i = 0; i < m.total(); ++i) c.data[3 * i] = c.data[3 * i + 1] = c.data[3 * i + 2] = m.data[i];
    return c;
  }
  return m;
}

Mat to_u8(const Mat& src, double scale, double shift) {
  Mat out(src.rows, src.cols, sa_maketype(SA_8U, src.channels()));
  for (int r = 0; r < src.rows; ++r)
    for (int c = 0; c < src.cols * src.channels(); ++c) {
      double v;
      switch (src.depth()) {
        case SA_32F: v = src.ptr<float>(r)[c]; break;
        case SA_64F: v = src.ptr<double>(r)[c]; break;
        case SA_8U: v = src.ptr<uint8_t>(r)[c]; break;
        case SA_16S: v = src.ptr<int16_t>(r)[c]; break;
        case SA_32S: v = src.ptr<int32_t>(r)[c]; break;
        default: v = 0; break;
      }
      v = v * scale + shift;
      const double rv = std::nearbyint(v);
      out.ptr<uint8_t>(r)[c] = (uint8_t)(std::isnan(v) ? 0 : rv < 0 ? 0 : rv > 255 ? 255 : rv);
    }
  return out;
}

bool imwrite(const std::string& path, const Mat& m_in, int quality) {
  Mat m = m_in.depth() == SA_8U ? m_in : to_u8(m_in);
  if (m.channels() != 1 && m.channels() != 3) return false;
  Image img;
  img.width = m.cols;
  img.height = m.rows;
  img.channels = m.channels();
  img.data.resize((size_t)m.cols * m.rows * m.channels());
  for (int r = 0; r < m.rows; ++r)
    std::memcpy(&img.data[(size_t)r * m.cols * m.channels()], m.ptr<uint8_t>(r), (size_t)m.cols * m.channels());
  std::vector<uint8_t> out;
  const std::string e = lower_ext(path);
  bool ok;
  if (e == "jpg" || e == "jpeg") {
    ok = jpeg_encode(img, quality, out);
  } else if (e == "png") {
    ok = png_encode(img, out);
  } else if (e == "ppm" || e == "pgm" || e == "pnm") {
    std::string hdr = std::string(img.channels == 3 ? "P6" : "P5") + "\n" + std::to_string(img.width) + " " +
                      std::to_string(img.height) + "\n255\n";
    out.assign(hdr.begin(), hdr.end());
    size_t base = out.size();
    out.insert(out.end(), img.data.begin(), img.data.end());
    if (img.channels == 3)
      for (size_t i = base; i < out.size(); i += 3) std::swap(out[i], out[i + 2]);
    ok = true;
  } else {
    return false;
  }
  if (!ok) return false;
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char*>(out.data()), (std::streamsize)out.size());
  return f.good();
}

Mat bgr2gray(const Mat& bgr) {
  Mat g(bgr.rows, bgr.cols, SA_8UC1);
  for (int r = 0; r < bgr.rows; ++r) {
    const uint8_t* s = bgr.ptr<uint8_t>(r);
    uint8_t* o = g.ptr<uint8_t>(r);
    for (int c = 0; c < bgr.cols; ++c) o[c] = (uint8_t)((s[3 * c] * 1868 + s[3 * c + 1] * 9617 + s[3 * c + 2] * 4899 + (1 << 13)) >> 14);
  }
  return g;
}

// OpenCV colormap.cpp Jet: MATLAB jet(64) control points, linearly interpolated to 256 in float,
// converted with saturate_cast (round half to even) after *255.
static const std::vector<uint8_t>& jet_lut() {
  static std::vector<uint8_t> lut = [] {
    float r[64], g[64], b[64];
    const int m = 64, n = 16;
    float u[47];
    for (int i = 0; i < 47; ++i) u[i] = i < n ? (float)(i + 1) / n : (i < 2 * n - 1 ? 1.f : (float)(3 * n - 1 - i) / n);
    for (int i = 0; i < m; ++i) r[i] = g[i] = b[i] = 0.f;
    for (int i = 0; i < 47; ++i) {
      const int gi = 8 + i, ri = gi + n, bi = gi - n;  // 0-based of MATLAB's 9..55, 25..71, -7..39
      if (gi < m) g[gi] = u[i];
      if (ri < m) r[ri] = u[i];
      if (bi >= 0 && bi < m) b[bi] = u[i];
    }
    float X[64];
    const float step = 1.f / 63.f;
    for (int i = 0; i < 64; ++i) X[i] = 0.f + i * step;
    std::vector<uint8_t> out(256 * 3);
    const float step2 = 1.f / 255.f;
    for (int i = 0; i < 256; ++i) {
      const float xi = 0.f + i * step2;
      int low = 0, high = 63;
      if (xi < X[low]) high = 1;
      if (xi > X[high]) low = high - 1;
      while (high - low > 1) {
        const int c = low + ((high - low) >> 1);
        if (xi > X[c]) low = c;
        else high = c;
      }
      const float* ch[3] = {b, g, r};
      for (int k = 0; k < 3; ++k) {
        const float y = ch[k][low] + (xi - X[low]) * (ch[k][high] - ch[k][low]) / (X[high] - X[low]);
        const float v = y * 255.f;
        const float rv = std::nearbyint(v);
        out[i * 3 + k] = (uint8_t)(rv < 0 ? 0 : rv > 255 ? 255 : rv);
      }
    }
    return out;
  }();
  return lut;
}

Mat apply_colormap_jet(const Mat& u8) {
  const Mat g = u8.channels() == 3 ? bgr2gray(u8) : u8;
  const auto& lut = jet_lut();
  Mat out(g.rows, g.cols, SA_8UC3);
  for (int r = 0; r < g.rows; ++r)
    for (int c = 0; c < g.cols; ++c) std::memcpy(out.ptr<uint8_t>(r) + 3 * c, &lut[g.ptr<uint8_t>(r)[c] * 3], 3);
  return out;
}

Mat heatmap(const Mat& disp) {
  // (disparity - min) / ((max - min) / 255) in float, then convertScaleAbs and JET
  float mn = INFINITY, mx = -INFINITY;
  for (int r = 0; r < disp.rows; ++r)
    for (int c = 0; c < disp.cols; ++c) {
      const float v = disp.ptr<float>(r)[c];
      mn = std::min(mn, v);
      mx = std::max(mx, v);
    }
  const float sd = (float)(((double)mx - (double)mn) / 255);
  Mat a(disp.rows, disp.cols, SA_8UC1);
  for (int r = 0; r < disp.rows; ++r)
    for (int c = 0; c < disp.cols; ++c) {
      const float v = std::fabs((disp.ptr<float>(r)[c] - mn) / sd);
      const float rv = std::nearbyint(v);
      a.ptr<uint8_t>(r)[c] = (uint8_t)(std::isnan(v) ? 0 : rv > 255 ? 255 : rv);
    }
  return apply_colormap_jet(a);
}

bool write_pointcloud_txt(const std::string& path, const float* cloud, size_t points) {
  std::ofstream f(path);
  if (!f.good()) return false;
  for (size_t i = 0; i < points; ++i) {
    const float* p = cloud + i * 6;
    f << p[0] << " " << p[1] << " " << p[2] << " " << p[3] << " " << p[4] << " " << p[5] << std::endl;
  }
  return f.good();
}

}  // namespace sa
