// Camera / stereo geometry (OpenCV-equivalent math, no OpenCV): calibration YAML I/O, Rodrigues,
// undistortPoints, initUndistortRectifyMap, remap, stereoRectify (Bouguet), projectPoints,
// reprojectImageTo3D.  See sa/calib.h for the reference call sites each function replaces.
#include <algorithm>
#include <cfloat>
#include <cmath>

#include "sa/calib.h"
#include "sa/filestorage.h"

namespace sa {

// ------------------------------------------------------------------ small helpers
static Mat33 mat33(const Mat& m) {
  Mat33 r{1, 0, 0, 0, 1, 0, 0, 0, 1};
  if (m.empty()) return r;
  for (int i = 0; i < 9; ++i) r[i] = m.get(i);
  return r;
}
static Mat from33(const Mat33& a) {
  Mat m(3, 3, SA_64FC1);
  for (int i = 0; i < 9; ++i) m.ptr<double>(0)[i] = a[i];
  return m;
}
static Mat33 mul(const Mat33& a, const Mat33& b) {
  Mat33 c{};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0;
      for (int k = 0; k < 3; ++k) s += a[i * 3 + k] * b[k * 3 + j];
      c[i * 3 + j] = s;
    }
  return c;
}
static Mat33 transpose(const Mat33& a) {
  return {a[0], a[3], a[6], a[1], a[4], a[7], a[2], a[5], a[8]};
}
static Vec3 mulv(const Mat33& a, const Vec3& v) {
  return {a[0] * v[0] + a[1] * v[1] + a[2] * v[2], a[3] * v[0] + a[4] * v[1] + a[5] * v[2],
          a[6] * v[0] + a[7] * v[1] + a[8] * v[2]};
}
static Mat33 inv33(const Mat33& m) {
  const double a = m[0], b = m[1], c = m[2], d = m[3], e = m[4], f = m[5], g = m[6], h = m[7], i = m[8];
  const double A = e * i - f * h, B = -(d * i - f * g), C = d * h - e * g;
  const double det = a * A + b * B + c * C;
  const double id = 1.0 / det;
  return {A * id, -(b * i - c * h) * id, (b * f - c * e) * id, B * id, (a * i - c * g) * id,
          -(a * f - c * d) * id, C * id, -(a * h - b * g) * id, (a * e - b * d) * id};
}
static double norm3(const Vec3& v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

// ------------------------------------------------------------------ YAML
bool read_calibration(const std::string& path, CalibrationParam& p) {
  FileStorage fs(path, FileStorage::READ);
  if (!fs.isOpened()) return false;
  auto m = [&](const char* k) { return fs[k].mat; };
  p.intrinsic_left = m("intrinsic_left");
  p.distCoeffs_left = m("distCoeffs_left");
  p.intrinsic_right = m("intrinsic_right");
  p.distCoeffs_right = m("distCoeffs_right");
  p.R = m("R");
  p.T = m("T");
  p.R_L = m("R_L");
  p.R_R = m("R_R");
  p.P1 = m("P1");
  p.P2 = m("P2");
  p.Q = m("Q");
  auto roi = [&](const char* k, Rect& r) {
    auto v = fs[k].reals();
    if (v.size() == 4) {
      r = {(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
      return true;
    }
    return false;
  };
  p.has_roi = roi("validROIL", p.validROIL) & roi("validROIR", p.validROIR);
  // a file without any of the matrices is not a stereo calibration (OpenCV's FileStorage would already have
  // refused most such files; ours is lenient about the format)
  return !(p.Q.empty() && p.intrinsic_left.empty() && p.intrinsic_right.empty() && p.P1.empty() && p.P2.empty());
}

bool write_calibration(const std::string& path, const CalibrationParam& p) {
  // key order of Stereo_Calibration.cpp:165-179
  FileStorage fs(path, FileStorage::WRITE);
  if (!fs.isOpened()) return false;
  fs.write("intrinsic_left", p.intrinsic_left);
  fs.write("distCoeffs_left", p.distCoeffs_left);
  fs.write("intrinsic_right", p.intrinsic_right);
  fs.write("distCoeffs_right", p.distCoeffs_right);
  fs.write("R", p.R);
  fs.write("T", p.T);
  fs.write("R_L", p.R_L);
  fs.write("R_R", p.R_R);
  fs.write("P1", p.P1);
  fs.write("P2", p.P2);
  fs.write("Q", p.Q);
  if (p.has_roi) {
    fs.write_seq("validROIL", {p.validROIL.x, p.validROIL.y, p.validROIL.width, p.validROIL.height});
    fs.write_seq("validROIR", {p.validROIR.x, p.validROIR.y, p.validROIR.width, p.validROIR.height});
  }
  fs.release();
  return true;
}

// ------------------------------------------------------------------ Rodrigues
Mat33 rodrigues(const Vec3& r, double* jac) {
  const double theta = norm3(r);
  if (jac) std::fill(jac, jac + 27, 0.0);
  if (theta < DBL_EPSILON) {
    if (jac) {  // dR/dr at 0: skew generators
      jac[5] = jac[15] = jac[19] = -1;
      jac[7] = jac[11] = jac[21] = 1;
    }
    return {1, 0, 0, 0, 1, 0, 0, 0, 1};
  }
  const double c = std::cos(theta), s = std::sin(theta), c1 = 1. - c;
  const double it = 1. / theta;
  const double x = r[0] * it, y = r[1] * it, z = r[2] * it;
  const Mat33 rrt{x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
  const Mat33 rx{0, -z, y, z, 0, -x, -y, x, 0};
  Mat33 R;
  for (int k = 0; k < 9; ++k) R[k] = c * (k % 4 == 0 ? 1.0 : 0.0) + c1 * rrt[k] + s * rx[k];
  if (jac) {
    // OpenCV's analytic derivative (calibration.cpp cvRodrigues2)
    const Mat33 I{1, 0, 0, 0, 1, 0, 0, 0, 1};
    const double drrt[27] = {x + x, y, z, y, 0, 0, z, 0, 0, 0, x, 0, x, y + y, z, 0, z, 0,
                             0, 0, x, 0, 0, y, x, y, z + z};
    const double d_r_x_[27] = {0, 0, 0, 0, 0, -1, 0, 1, 0, 0, 0, 1, 0, 0, 0, -1, 0, 0,
                               0, -1, 0, 1, 0, 0, 0, 0, 0};
    const double rr[3] = {x, y, z};
    for (int i = 0; i < 3; ++i) {
      const double ri = rr[i];
      const double a0 = -s * ri, a1 = (s - 2 * c1 * it) * ri, a2 = c1 * it;
      const double a3 = (c - s * it) * ri, a4 = s * it;
      for (int k = 0; k < 9; ++k)
        jac[i * 9 + k] = a0 * I[k] + a1 * rrt[k] + a2 * drrt[i * 9 + k] + a3 * rx[k] + a4 * d_r_x_[i * 9 + k];
    }
    // OpenCV stores J as 3x9 (d R_k / d r_i) in row i; keep that layout
  }
  return R;
}

Vec3 rodrigues_inv(const Mat33& R) {
  double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
  const double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
  double c = (R[0] + R[4] + R[8] - 1) * 0.5;
  c = c > 1. ? 1. : c < -1. ? -1. : c;
  double theta = std::acos(c);
  if (s < 1e-5) {
    if (c > 0) return {0, 0, 0};
    double t = (R[0] + 1) * 0.5;
    rx = std::sqrt(std::max(t, 0.));
    t = (R[4] + 1) * 0.5;
    ry = std::sqrt(std::max(t, 0.)) * (R[1] < 0 ? -1. : 1.);
    t = (R[8] + 1) * 0.5;
    rz = std::sqrt(std::max(t, 0.)) * (R[2] < 0 ? -1. : 1.);
    if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
    theta /= std::sqrt(rx * rx + ry * ry + rz * rz);
    return {rx * theta, ry * theta, rz * theta};
  }
  const double vth = 1 / (2 * s) * theta;
  return {rx * vth, ry * vth, rz * vth};
}

std::array<double, 14> dist14(const Mat& D) {
  std::array<double, 14> k{};
  if (!D.empty())
    for (size_t i = 0; i < std::min<size_t>(14, D.total() * D.channels()); ++i) k[i] = D.get((int)i);
  return k;
}

// ------------------------------------------------------------------ undistortPoints
void undistort_points(const std::vector<std::array<double, 2>>& src, std::vector<std::array<double, 2>>& dst,
                      const Mat& Km, const Mat& D, const Mat& Rm, const Mat& Pm, int iters) {
  const Mat33 A = mat33(Km);
  const auto k = dist14(D);
  Mat33 RR = mat33(Rm);
  if (!Pm.empty()) {
    Mat33 PP{};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) PP[i * 3 + j] = Pm.get(i * Pm.cols + j);
    RR = mul(PP, RR);
  }
  const double fx = A[0], fy = A[4], ifx = 1. / fx, ify = 1. / fy, cx = A[2], cy = A[5];
  const bool has_dist = !D.empty();
  dst.resize(src.size());
  for (size_t i = 0; i < src.size(); ++i) {
    double x = src[i][0], y = src[i][1];
    const double u = x, v = y;
    x = (x - cx) * ifx;
    y = (y - cy) * ify;
    if (has_dist) {
      const double x0 = x, y0 = y;
      for (int j = 0; j < iters; ++j) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        if (icdist < 0) {
          x = (u - cx) * ifx;
          y = (v - cy) * ify;
          break;
        }
        const double dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        const double dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - dx) * icdist;
        y = (y0 - dy) * icdist;
      }
    }
    const double xx = RR[0] * x + RR[1] * y + RR[2];
    const double yy = RR[3] * x + RR[4] * y + RR[5];
    const double ww = 1. / (RR[6] * x + RR[7] * y + RR[8]);
    dst[i] = {xx * ww, yy * ww};
  }
}

// ------------------------------------------------------------------ rectification maps
void init_undistort_rectify_map(const Mat& Km, const Mat& D, const Mat& Rm, const Mat& Pm, int width, int height,
                                std::vector<float>& map, bool quantize) {
  const Mat33 A = mat33(Km);
  Mat33 Ar = A;
  if (!Pm.empty())
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Ar[i * 3 + j] = Pm.get(i * Pm.cols + j);
  const Mat33 iR = inv33(mul(Ar, mat33(Rm)));
  const double* ir = iR.data();
  const double u0 = A[2], v0 = A[5], fx = A[0], fy = A[4];
  const auto k = dist14(D);
  const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3], k3 = k[4], k4 = k[5], k5 = k[6], k6 = k[7];
  const double s1 = k[8], s2 = k[9], s3 = k[10], s4 = k[11];
  map.resize((size_t)width * height * 2);
  for (int i = 0; i < height; ++i) {
    double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
    for (int j = 0; j < width; ++j, _x += ir[0], _y += ir[3], _w += ir[6]) {
      const double w = 1. / _w, x = _x * w, y = _y * w;
      const double x2 = x * x, y2 = y * y;
      const double r2 = x2 + y2, _2xy = 2 * x * y;
      const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
      const double xd = x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2;
      const double yd = y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2;
      double u = fx * xd + u0, v = fy * yd + v0;
      float* o = &map[((size_t)i * width + j) * 2];
      if (quantize) {
        // CV_16SC2: saturate_cast<int>(u * INTER_TAB_SIZE) (round half to even), kept as k/32
        const double qu = std::nearbyint(u * 32.0), qv = std::nearbyint(v * 32.0);
        const double lim = 2147483647.0;
        o[0] = (float)(std::max(-lim, std::min(lim, qu)) / 32.0);
        o[1] = (float)(std::max(-lim, std::min(lim, qv)) / 32.0);
      } else {
        o[0] = (float)u;
        o[1] = (float)v;
      }
    }
  }
}

void remap_cpu(const Mat& src_in, Mat& dst, const std::vector<float>& map) {
  const Mat src = (src_in.data == dst.data) ? src_in.clone() : src_in;  // cv::remap clones in-place src
  const int H = (int)(map.size() / 2 / src.cols), W = src.cols;
  (void)H;
  const int oh = dst.empty() ? src.rows : dst.rows, ow = dst.empty() ? src.cols : dst.cols;
  if (dst.empty() || dst.type() != src.type()) dst.create(oh, ow, src.type());
  const int cn = src.channels();
  for (int y = 0; y < oh; ++y)
    for (int x = 0; x < ow; ++x) {
      const float* mp = &map[((size_t)y * ow + x) * 2];
      const int iu = (int)std::nearbyint(mp[0] * 32.0), iv = (int)std::nearbyint(mp[1] * 32.0);
      const int x0 = iu >> 5, y0 = iv >> 5;
      const float ax = (float)(iu & 31) / 32.f, ay = (float)(iv & 31) / 32.f;
      int w[4] = {(int)std::nearbyint((1.f - ax) * (1.f - ay) * 32768.f), (int)std::nearbyint(ax * (1.f - ay) * 32768.f),
                  (int)std::nearbyint((1.f - ax) * ay * 32768.f), (int)std::nearbyint(ax * ay * 32768.f)};
      const int diff = w[0] + w[1] + w[2] + w[3] - 32768;
      if (diff != 0) {
        int kk = 0;
        for (int j = 1; j < 4; ++j)
          if (diff < 0 ? (w[j] > w[kk]) : (w[j] < w[kk])) kk = j;
        w[kk] -= diff;
      }
      for (int c = 0; c < cn; ++c) {
        int acc = 0;
        for (int j = 0; j < 4; ++j) {
          const int xx = x0 + (j & 1), yy = y0 + (j >> 1);
          if (xx < 0 || xx >= src.cols || yy < 0 || yy >= src.rows) continue;
          acc += w[j] * src.ptr<uint8_t>(yy)[xx * cn + c];
        }
        const int v = (acc + (1 << 14)) >> 15;
        dst.ptr<uint8_t>(y)[x * cn + c] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
      }
    }
}

// ------------------------------------------------------------------ projectPoints
void project_points(const std::vector<std::array<double, 3>>& obj, const Vec3& rvec, const Vec3& tvec,
                    const Mat& Km, const Mat& D, std::vector<std::array<double, 2>>& img) {
  const Mat33 R = rodrigues(rvec);
  const Mat33 A = mat33(Km);
  const auto k = dist14(D);
  img.resize(obj.size());
  for (size_t i = 0; i < obj.size(); ++i) {
    const Vec3 X = mulv(R, {obj[i][0], obj[i][1], obj[i][2]});
    const double Z = X[2] + tvec[2];
    const double z = Z ? 1. / Z : 1.;
    const double x = (X[0] + tvec[0]) * z, y = (X[1] + tvec[1]) * z;
    const double r2 = x * x + y * y, r4 = r2 * r2, r6 = r4 * r2, a1 = 2 * x * y, a2 = r2 + 2 * x * x,
                 a3 = r2 + 2 * y * y;
    const double cdist = 1 + k[0] * r2 + k[1] * r4 + k[4] * r6;
    const double icdist2 = 1. / (1 + k[5] * r2 + k[6] * r4 + k[7] * r6);
    const double xd = x * cdist * icdist2 + k[2] * a1 + k[3] * a2 + k[8] * r2 + k[9] * r4;
    const double yd = y * cdist * icdist2 + k[2] * a3 + k[3] * a1 + k[10] * r2 + k[11] * r4;
    img[i] = {xd * A[0] + A[2], yd * A[4] + A[5]};
  }
}

// ------------------------------------------------------------------ stereoRectify
// cv::undistortPoints' default fixed-point iteration count (TermCriteria COUNT 5).  Image corners
// of strongly distorted lenses do not converge in 5 steps, so rectified f / c differ by up to ~0.1%
// between OpenCV builds; tests pin the reference file to that tolerance.
static const int g_rect_iters = 5;
static void get_rectangles(const Mat& K, const Mat& D, const Mat& R, const Mat& P, int W, int H, double inner[4],
                           double outer[4]) {
  const int N = 9;
  std::vector<std::array<double, 2>> pts;
  for (int y = 0; y < N; ++y)
    for (int x = 0; x < N; ++x) pts.push_back({(double)(float)((float)x * W / (N - 1)), (double)(float)((float)y * H / (N - 1))});
  undistort_points(pts, pts, K, D, R, P, g_rect_iters);
  float iX0 = -FLT_MAX, iX1 = FLT_MAX, iY0 = -FLT_MAX, iY1 = FLT_MAX;
  float oX0 = FLT_MAX, oX1 = -FLT_MAX, oY0 = FLT_MAX, oY1 = -FLT_MAX;
  for (int y = 0, k = 0; y < N; ++y)
    for (int x = 0; x < N; ++x) {
      const float px = (float)pts[k][0], py = (float)pts[k][1];
      ++k;
      oX0 = std::min(oX0, px);
      oX1 = std::max(oX1, px);
      oY0 = std::min(oY0, py);
      oY1 = std::max(oY1, py);
      if (x == 0) iX0 = std::max(iX0, px);
      if (x == N - 1) iX1 = std::min(iX1, px);
      if (y == 0) iY0 = std::max(iY0, py);
      if (y == N - 1) iY1 = std::min(iY1, py);
    }
  inner[0] = iX0;
  inner[1] = iY0;
  inner[2] = iX1 - iX0;
  inner[3] = iY1 - iY0;
  outer[0] = oX0;
  outer[1] = oY0;
  outer[2] = oX1 - oX0;
  outer[3] = oY1 - oY0;
}

void stereo_rectify(const Mat& K1, const Mat& D1, const Mat& K2, const Mat& D2, int W, int H, const Mat& Rm,
                    const Mat& Tm, Mat& R1, Mat& R2, Mat& P1, Mat& P2, Mat& Qm, bool zero_disparity, double alpha,
                    Rect* roi1, Rect* roi2) {
  const Mat33 R = mat33(Rm);
  const Vec3 T{Tm.get(0), Tm.get(1), Tm.get(2)};
  Vec3 om = rodrigues_inv(R);
  for (auto& v : om) v *= -0.5;  // average rotation
  const Mat33 r_r = rodrigues(om);
  Vec3 t = mulv(r_r, T);
  const int idx = std::fabs(t[0]) > std::fabs(t[1]) ? 0 : 1;
  const double c = t[idx], nt = norm3(t);
  Vec3 uu{0, 0, 0};
  uu[idx] = c > 0 ? 1 : -1;
  Vec3 ww{t[1] * uu[2] - t[2] * uu[1], t[2] * uu[0] - t[0] * uu[2], t[0] * uu[1] - t[1] * uu[0]};
  const double nw = norm3(ww);
  if (nw > 0.0) {
    const double sc = std::acos(std::fabs(c) / nt) / nw;
    for (auto& v : ww) v *= sc;
  }
  const Mat33 wR = rodrigues(ww);
  const Mat33 Ri1 = mul(wR, transpose(r_r));
  const Mat33 Ri2 = mul(wR, r_r);
  R1 = from33(Ri1);
  R2 = from33(Ri2);
  t = mulv(Ri2, T);

  const Mat33 A1 = mat33(K1), A2 = mat33(K2);
  double fc_new = (A1[(idx ^ 1) * 4] + A2[(idx ^ 1) * 4]) * 0.5;  // ratio = 1/2 for newImgSize = imageSize
  double ccx[2], ccy[2];
  for (int k = 0; k < 2; ++k) {
    std::vector<std::array<double, 2>> pts(4);
    for (int i = 0; i < 4; ++i) {
      const int j = i < 2 ? 0 : 1;
      pts[i] = {(double)(float)((i % 2) * (W - 1)), (double)(float)(j * (H - 1))};
    }
    undistort_points(pts, pts, k == 0 ? K1 : K2, k == 0 ? D1 : D2, Mat(), Mat(), g_rect_iters);
    // project (x, y, 1) with rotation R_k, zero translation, camera diag(fc_new, fc_new, 1)
    const Mat33& Rk = k == 0 ? Ri1 : Ri2;
    double sx = 0, sy = 0;
    for (int i = 0; i < 4; ++i) {
      // cvUndistortPoints writes CV_32FC2 in the reference: round-trip through float
      const Vec3 X = mulv(Rk, {(double)(float)pts[i][0], (double)(float)pts[i][1], 1.0});
      const double iz = 1. / X[2];
      sx += (float)(X[0] * iz * fc_new);
      sy += (float)(X[1] * iz * fc_new);
    }
    ccx[k] = (W - 1) / 2.0 - sx / 4;
    ccy[k] = (H - 1) / 2.0 - sy / 4;
  }
  if (zero_disparity) {
    ccx[0] = ccx[1] = (ccx[0] + ccx[1]) * 0.5;
    ccy[0] = ccy[1] = (ccy[0] + ccy[1]) * 0.5;
  } else if (idx == 0) {
    ccy[0] = ccy[1] = (ccy[0] + ccy[1]) * 0.5;
  } else {
    ccx[0] = ccx[1] = (ccx[0] + ccx[1]) * 0.5;
  }
  P1 = Mat(3, 4, SA_64FC1, 0.0);
  P2 = Mat(3, 4, SA_64FC1, 0.0);
  auto setP = [&](Mat& P, double f, double cx, double cy) {
    P.at<double>(0, 0) = P.at<double>(1, 1) = f;
    P.at<double>(0, 2) = cx;
    P.at<double>(1, 2) = cy;
    P.at<double>(2, 2) = 1;
  };
  setP(P1, fc_new, ccx[0], ccy[0]);
  setP(P2, fc_new, ccx[1], ccy[1]);
  P2.at<double>(idx, 3) = t[idx] * fc_new;

  alpha = std::min(alpha, 1.);
  double in1[4], out1[4], in2[4], out2[4];
  get_rectangles(K1, D1, R1, P1, W, H, in1, out1);
  get_rectangles(K2, D2, R2, P2, W, H, in2, out2);
  const double cx1_0 = ccx[0], cy1_0 = ccy[0], cx2_0 = ccx[1], cy2_0 = ccy[1];
  const double cx1 = cx1_0, cy1 = cy1_0, cx2 = cx2_0, cy2 = cy2_0;  // newImgSize == imageSize
  double s = 1.;
  if (alpha >= 0) {
    double s0 = std::max(std::max(std::max(cx1 / (cx1_0 - in1[0]), cy1 / (cy1_0 - in1[1])),
                                  (W - cx1) / (in1[0] + in1[2] - cx1_0)),
                         (H - cy1) / (in1[1] + in1[3] - cy1_0));
    s0 = std::max(std::max(std::max(std::max(cx2 / (cx2_0 - in2[0]), cy2 / (cy2_0 - in2[1])),
                                    (W - cx2) / (in2[0] + in2[2] - cx2_0)),
                           (H - cy2) / (in2[1] + in2[3] - cy2_0)),
                  s0);
    double s1 = std::min(std::min(std::min(cx1 / (cx1_0 - out1[0]), cy1 / (cy1_0 - out1[1])),
                                  (W - cx1) / (out1[0] + out1[2] - cx1_0)),
                         (H - cy1) / (out1[1] + out1[3] - cy1_0));
    s1 = std::min(std::min(std::min(std::min(cx2 / (cx2_0 - out2[0]), cy2 / (cy2_0 - out2[1])),
                                    (W - cx2) / (out2[0] + out2[2] - cx2_0)),
                           (H - cy2) / (out2[1] + out2[3] - cy2_0)),
                  s1);
    s = s0 * (1 - alpha) + s1 * alpha;
  }
  fc_new *= s;
  P1.at<double>(0, 0) = P1.at<double>(1, 1) = fc_new;
  P2.at<double>(0, 0) = P2.at<double>(1, 1) = fc_new;
  P2.at<double>(idx, 3) *= s;
  auto make_roi = [&](const double* in, double cx0, double cy0, double cx, double cy) {
    int x = (int)std::ceil((in[0] - cx0) * s + cx), y = (int)std::ceil((in[1] - cy0) * s + cy);
    int w = (int)std::floor(in[2] * s), h = (int)std::floor(in[3] * s);
    const int x1 = std::max(x, 0), y1 = std::max(y, 0);
    const int x2 = std::min(x + w, W), y2 = std::min(y + h, H);
    Rect r;
    if (x2 > x1 && y2 > y1) r = {x1, y1, x2 - x1, y2 - y1};
    return r;
  };
  if (roi1) *roi1 = make_roi(in1, cx1_0, cy1_0, cx1, cy1);
  if (roi2) *roi2 = make_roi(in2, cx2_0, cy2_0, cx2, cy2);
  Qm = Mat(4, 4, SA_64FC1, 0.0);
  double* q = Qm.ptr<double>(0);
  q[0] = 1;
  q[3] = -cx1;
  q[5] = 1;
  q[7] = -cy1;
  q[11] = fc_new;
  q[14] = -1. / t[idx];
  q[15] = (idx == 0 ? cx1 - cx2 : cy1 - cy2) / t[idx];
}

// ------------------------------------------------------------------ reprojection
void reproject_cpu(const float* disp, int H, int W, const double Q[16], float* xyz) {
  for (int r = 0; r < H; ++r)
    for (int c = 0; c < W; ++c) {
      const double d = disp[(size_t)r * W + c];
      const double X = Q[0] * c + Q[1] * r + Q[2] * d + Q[3];
      const double Y = Q[4] * c + Q[5] * r + Q[6] * d + Q[7];
      const double Z = Q[8] * c + Q[9] * r + Q[10] * d + Q[11];
      const double w = Q[12] * c + Q[13] * r + Q[14] * d + Q[15];
      float* o = xyz + ((size_t)r * W + c) * 3;
      o[0] = (float)(X / w);
      o[1] = (float)(Y / w);
      o[2] = (float)(Z / w);
    }
}

}  // namespace sa
