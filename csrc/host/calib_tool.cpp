// Chessboard stereo calibration pipeline (the reference's Stereo_Calibration tool,
// Stereo_Calibration/Stereo_Calibration.cpp:67-182), without OpenCV:
//
//   * find_chessboard_corners — X-junction (saddle) detector + lattice growth; an own algorithm, not
//     OpenCV's quad-linking.  Returns the cols x rows inner corners row-major from the top-left
//     (rows run along the `cols` axis, left to right, then downwards), the same physical ordering
//     for both cameras of a rig.
//   * corner_subpix          — cv::cornerSubPix's gradient-orthogonality iteration (Gaussian window
//     mask, bilinear patch, convergence / fallback rules of OpenCV's implementation)
//   * calibrate_camera       — principal point at the image centre + focal lengths from the
//     per-view homographies (the closed form of cvInitIntrinsicParams2D), homography extrinsics,
//     then Levenberg-Marquardt over (fx fy cx cy k1 k2 p1 p2 k3) + 6 per view
//   * stereo_calibrate       — CALIB_USE_INTRINSIC_GUESS: joint LM over both cameras' intrinsics and
//     distortion, the rig pose (R, T) and the left per-view poses (median initialisation of R, T)
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <queue>
#include <stdexcept>

#include "sa/calib.h"
#include "sa/imgio.h"

namespace sa {
namespace {

using Pt2 = std::array<double, 2>;
using Pt3 = std::array<double, 3>;

// ------------------------------------------------------------------ dense linear algebra
// Symmetric Jacobi eigen-decomposition; eigenvalues ascending, eigenvectors as columns of V.
void sym_eigen(std::vector<double> A, int n, std::vector<double>& w, std::vector<double>& V) {
  V.assign((size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i) V[i * n + i] = 1.0;
  for (int sweep = 0; sweep < 100; ++sweep) {
    double off = 0;
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j) off += A[i * n + j] * A[i * n + j];
    if (off < 1e-30) break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = A[p * n + q];
        if (std::fabs(apq) < 1e-300) continue;
        const double theta = (A[q * n + q] - A[p * n + p]) / (2 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
        const double c = 1 / std::sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < n; ++k) {  // A = J^T A J
          const double akp = A[k * n + p], akq = A[k * n + q];
          A[k * n + p] = c * akp - s * akq;
          A[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          const double apk = A[p * n + k], aqk = A[q * n + k];
          A[p * n + k] = c * apk - s * aqk;
          A[q * n + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k) {
          const double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = c * vkp - s * vkq;
          V[k * n + q] = s * vkp + c * vkq;
        }
      }
  }
  std::vector<int> idx(n);
  for (int i = 0; i < n; ++i) idx[i] = i;
  std::sort(idx.begin(), idx.end(), [&](int a, int b) { return A[a * n + a] < A[b * n + b]; });
  std::vector<double> V2((size_t)n * n);
  w.resize(n);
  for (int j = 0; j < n; ++j) {
    w[j] = A[idx[j] * n + idx[j]];
    for (int i = 0; i < n; ++i) V2[i * n + j] = V[i * n + idx[j]];
  }
  V.swap(V2);
}

// Solve the SPD system A x = b (Cholesky); false if not positive definite.
bool chol_solve(std::vector<double> A, std::vector<double> b, int n, std::vector<double>& x) {
  for (int j = 0; j < n; ++j) {
    double d = A[j * n + j];
    for (int k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
    if (d <= 0) return false;
    d = std::sqrt(d);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double s = A[i * n + j];
      for (int k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = s / d;
    }
  }
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= A[i * n + k] * b[k];
    b[i] = s / A[i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int k = i + 1; k < n; ++k) s -= A[k * n + i] * b[k];
    b[i] = s / A[i * n + i];
  }
  x = b;
  return true;
}

Mat33 mul33(const Mat33& a, const Mat33& b) {
  Mat33 c{};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      for (int k = 0; k < 3; ++k) c[i * 3 + j] += a[i * 3 + k] * b[k * 3 + j];
  return c;
}
Mat33 tr33(const Mat33& a) { return {a[0], a[3], a[6], a[1], a[4], a[7], a[2], a[5], a[8]}; }
Vec3 mv33(const Mat33& a, const Vec3& v) {
  return {a[0] * v[0] + a[1] * v[1] + a[2] * v[2], a[3] * v[0] + a[4] * v[1] + a[5] * v[2],
          a[6] * v[0] + a[7] * v[1] + a[8] * v[2]};
}

// nearest rotation (polar decomposition R = M (M^T M)^{-1/2})
Mat33 nearest_rotation(const Mat33& M) {
  std::vector<double> MtM(9), w, V;
  const Mat33 mm = mul33(tr33(M), M);
  for (int i = 0; i < 9; ++i) MtM[i] = mm[i];
  sym_eigen(MtM, 3, w, V);
  Mat33 isq{};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      for (int k = 0; k < 3; ++k) isq[i * 3 + j] += V[i * 3 + k] * V[j * 3 + k] / std::sqrt(std::max(w[k], 1e-300));
  return mul33(M, isq);
}

// Normalised DLT homography src (plane) -> dst, row-major 3x3 with H[8] = 1.
Mat33 homography(const std::vector<Pt2>& src, const std::vector<Pt2>& dst) {
  const size_t n = src.size();
  auto norm_t = [&](const std::vector<Pt2>& p, double T[3]) {  // similarity: (x - m) * s
    double mx = 0, my = 0;
    for (auto& q : p) mx += q[0], my += q[1];
    mx /= n, my /= n;
    double d = 0;
    for (auto& q : p) d += std::hypot(q[0] - mx, q[1] - my);
    d /= n;
    T[0] = d > 0 ? std::sqrt(2.0) / d : 1.0;
    T[1] = mx;
    T[2] = my;
  };
  double Ts[3], Td[3];
  norm_t(src, Ts);
  norm_t(dst, Td);
  std::vector<double> AtA(81, 0.0);
  for (size_t i = 0; i < n; ++i) {
    const double X = (src[i][0] - Ts[1]) * Ts[0], Y = (src[i][1] - Ts[2]) * Ts[0];
    const double u = (dst[i][0] - Td[1]) * Td[0], v = (dst[i][1] - Td[2]) * Td[0];
    const double r1[9] = {X, Y, 1, 0, 0, 0, -u * X, -u * Y, -u};
    const double r2[9] = {0, 0, 0, X, Y, 1, -v * X, -v * Y, -v};
    for (int a = 0; a < 9; ++a)
      for (int b = 0; b < 9; ++b) AtA[a * 9 + b] += r1[a] * r1[b] + r2[a] * r2[b];
  }
  std::vector<double> w, V;
  sym_eigen(AtA, 9, w, V);
  Mat33 Hn;
  for (int i = 0; i < 9; ++i) Hn[i] = V[i * 9 + 0];
  // H = Td^-1 Hn Ts
  const Mat33 S{Ts[0], 0, -Ts[0] * Ts[1], 0, Ts[0], -Ts[0] * Ts[2], 0, 0, 1};
  const Mat33 Di{1 / Td[0], 0, Td[1], 0, 1 / Td[0], Td[2], 0, 0, 1};
  Mat33 H = mul33(Di, mul33(Hn, S));
  const double s = H[8] != 0 ? 1.0 / H[8] : 1.0;
  for (auto& v : H) v *= s;
  return H;
}

// ------------------------------------------------------------------ projection model
// p: fx fy cx cy k1 k2 p1 p2 k3
inline Pt2 project(const double* in, const Mat33& R, const Vec3& t, const Pt3& X) {
  const double Xc = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + t[0];
  const double Yc = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + t[1];
  const double Zc = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + t[2];
  const double iz = Zc != 0 ? 1.0 / Zc : 1.0;
  const double x = Xc * iz, y = Yc * iz;
  const double r2 = x * x + y * y, r4 = r2 * r2, r6 = r4 * r2;
  const double rad = 1 + in[4] * r2 + in[5] * r4 + in[8] * r6;
  const double xd = x * rad + 2 * in[6] * x * y + in[7] * (r2 + 2 * x * x);
  const double yd = y * rad + in[6] * (r2 + 2 * y * y) + 2 * in[7] * x * y;
  return {in[0] * xd + in[2], in[1] * yd + in[3]};
}

// Generic Levenberg-Marquardt over blocks: residual groups g (views) depend on the shared params
// [0, nshared) and on their own block [nshared + 6g, nshared + 6g + 6) (+ optional extra shared).
struct LMProblem {
  int nparams = 0;
  int ngroups = 0;
  // residuals of group g for parameter vector x (appends to r)
  std::function<void(const std::vector<double>& x, int g, std::vector<double>& r)> residual;
  // parameters a group depends on
  std::function<void(int g, std::vector<int>& idx)> deps;
};

double lm_solve(const LMProblem& P, std::vector<double>& x, int max_iters, double eps) {
  const int n = P.nparams;
  auto total = [&](const std::vector<double>& xx, std::vector<std::vector<double>>* rs) {
    double s = 0;
    std::vector<double> r;
    for (int g = 0; g < P.ngroups; ++g) {
      r.clear();
      P.residual(xx, g, r);
      for (double v : r) s += v * v;
      if (rs) (*rs)[g] = r;
    }
    return s;
  };
  std::vector<std::vector<double>> res(P.ngroups);
  double cost = total(x, &res);
  double lambda = 1e-3;
  std::vector<int> dep;
  for (int it = 0; it < max_iters; ++it) {
    std::vector<double> JtJ((size_t)n * n, 0.0), Jtr(n, 0.0);
    for (int g = 0; g < P.ngroups; ++g) {
      P.deps(g, dep);
      const std::vector<double>& r0 = res[g];
      const size_t m = r0.size();
      std::vector<std::vector<double>> J(dep.size(), std::vector<double>(m));
      std::vector<double> xp = x, rp, rm;
      for (size_t k = 0; k < dep.size(); ++k) {
        const int j = dep[k];
        const double h = 1e-6 * std::max(1.0, std::fabs(x[j]));
        xp[j] = x[j] + h;
        rp.clear();
        P.residual(xp, g, rp);
        xp[j] = x[j] - h;
        rm.clear();
        P.residual(xp, g, rm);
        xp[j] = x[j];
        for (size_t i = 0; i < m; ++i) J[k][i] = (rp[i] - rm[i]) / (2 * h);
      }
      for (size_t a = 0; a < dep.size(); ++a) {
        double s = 0;
        for (size_t i = 0; i < m; ++i) s += J[a][i] * r0[i];
        Jtr[dep[a]] += s;
        for (size_t b = a; b < dep.size(); ++b) {
          double t = 0;
          for (size_t i = 0; i < m; ++i) t += J[a][i] * J[b][i];
          JtJ[(size_t)dep[a] * n + dep[b]] += t;
          if (a != b) JtJ[(size_t)dep[b] * n + dep[a]] += t;
        }
      }
    }
    bool improved = false;
    for (int tries = 0; tries < 12 && !improved; ++tries) {
      std::vector<double> A = JtJ, g(n), d;
      for (int i = 0; i < n; ++i) {
        A[(size_t)i * n + i] += lambda * std::max(JtJ[(size_t)i * n + i], 1e-12);
        g[i] = -Jtr[i];
      }
      if (!chol_solve(A, g, n, d)) {
        lambda *= 10;
        continue;
      }
      std::vector<double> xn(n);
      for (int i = 0; i < n; ++i) xn[i] = x[i] + d[i];
      std::vector<std::vector<double>> rn(P.ngroups);
      const double cn = total(xn, &rn);
      if (cn < cost) {
        double dn = 0, xnrm = 0;
        for (int i = 0; i < n; ++i) dn += d[i] * d[i], xnrm += x[i] * x[i];
        x.swap(xn);
        res.swap(rn);
        const double rel = (cost - cn) / std::max(cost, 1e-300);
        cost = cn;
        lambda = std::max(lambda / 10, 1e-12);
        improved = true;
        if (std::sqrt(dn) <= eps * (std::sqrt(xnrm) + eps) || rel < 1e-15) return cost;
      } else {
        lambda *= 10;
      }
    }
    if (!improved) break;
  }
  return cost;
}

// extrinsics of a planar view from its homography in normalised camera coordinates
void pose_from_homography(const Mat33& Hn, Vec3& rvec, Vec3& tvec) {
  Vec3 h1{Hn[0], Hn[3], Hn[6]}, h2{Hn[1], Hn[4], Hn[7]}, h3{Hn[2], Hn[5], Hn[8]};
  const double n1 = std::sqrt(h1[0] * h1[0] + h1[1] * h1[1] + h1[2] * h1[2]);
  const double n2 = std::sqrt(h2[0] * h2[0] + h2[1] * h2[1] + h2[2] * h2[2]);
  double lam = 2.0 / (n1 + n2);
  if (h3[2] * lam < 0) lam = -lam;  // board in front of the camera
  Vec3 r1{h1[0] * lam, h1[1] * lam, h1[2] * lam}, r2{h2[0] * lam, h2[1] * lam, h2[2] * lam};
  Vec3 r3{r1[1] * r2[2] - r1[2] * r2[1], r1[2] * r2[0] - r1[0] * r2[2], r1[0] * r2[1] - r1[1] * r2[0]};
  const Mat33 M{r1[0], r2[0], r3[0], r1[1], r2[1], r3[1], r1[2], r2[2], r3[2]};
  rvec = rodrigues_inv(nearest_rotation(M));
  tvec = {h3[0] * lam, h3[1] * lam, h3[2] * lam};
}

Mat mat_from(const double* v, int rows, int cols) {
  Mat m(rows, cols, SA_64FC1);
  for (int i = 0; i < rows * cols; ++i) m.ptr<double>(0)[i] = v[i];
  return m;
}

void intr_from(const CameraCalib& c, double* in) {
  const double* K = c.K.ptr<double>(0);
  in[0] = K[0];
  in[1] = K[4];
  in[2] = K[2];
  in[3] = K[5];
  for (int i = 0; i < 5; ++i) in[4 + i] = (!c.D.empty() && (int)c.D.total() > i) ? c.D.get(i) : 0.0;
}

void intr_to(const double* in, CameraCalib& c) {
  const double K[9] = {in[0], 0, in[2], 0, in[1], in[3], 0, 0, 1};
  c.K = mat_from(K, 3, 3);
  c.D = mat_from(in + 4, 1, 5);
}

// ------------------------------------------------------------------ image helpers
struct FImg {
  int w = 0, h = 0;
  std::vector<float> v;
  float at(int x, int y) const {
    x = std::min(std::max(x, 0), w - 1);
    y = std::min(std::max(y, 0), h - 1);
    return v[(size_t)y * w + x];
  }
  float bilinear(double x, double y) const {
    const int x0 = (int)std::floor(x), y0 = (int)std::floor(y);
    const float a = (float)(x - x0), b = (float)(y - y0);
    return (1 - b) * ((1 - a) * at(x0, y0) + a * at(x0 + 1, y0)) + b * ((1 - a) * at(x0, y0 + 1) + a * at(x0 + 1, y0 + 1));
  }
};

FImg to_float(const Mat& gray) {
  FImg f;
  f.w = gray.cols;
  f.h = gray.rows;
  f.v.resize((size_t)f.w * f.h);
  for (int y = 0; y < f.h; ++y)
    for (int x = 0; x < f.w; ++x) f.v[(size_t)y * f.w + x] = gray.ptr<uint8_t>(y)[x];
  return f;
}

FImg gaussian(const FImg& in, double sigma) {
  const int r = std::max(1, (int)std::ceil(3 * sigma));
  std::vector<float> k(2 * r + 1);
  double s = 0;
  for (int i = -r; i <= r; ++i) s += k[i + r] = (float)std::exp(-0.5 * i * i / (sigma * sigma));
  for (auto& v : k) v = (float)(v / s);
  FImg t = in, o = in;
  for (int y = 0; y < in.h; ++y)
    for (int x = 0; x < in.w; ++x) {
      float a = 0;
      for (int i = -r; i <= r; ++i) a += k[i + r] * in.at(x + i, y);
      t.v[(size_t)y * in.w + x] = a;
    }
  for (int y = 0; y < in.h; ++y)
    for (int x = 0; x < in.w; ++x) {
      float a = 0;
      for (int i = -r; i <= r; ++i) a += k[i + r] * t.at(x, y + i);
      o.v[(size_t)y * in.w + x] = a;
    }
  return o;
}

// X-junction test: around a chessboard corner the intensity on a circle alternates
// bright/dark/bright/dark (4 sign changes relative to the circle mean) with good contrast.
bool is_xcorner(const FImg& img, double cx, double cy, double rad) {
  const int S = 32;
  float v[S];
  float mn = 1e9f, mx = -1e9f, mean = 0;
  for (int i = 0; i < S; ++i) {
    const double a = 2 * M_PI * i / S;
    v[i] = img.bilinear(cx + rad * std::cos(a), cy + rad * std::sin(a));
    mn = std::min(mn, v[i]);
    mx = std::max(mx, v[i]);
    mean += v[i];
  }
  mean /= S;
  if (mx - mn < 25.f) return false;
  const float band = 0.15f * (mx - mn);
  int sgn[S];
  for (int i = 0; i < S; ++i) sgn[i] = v[i] > mean + band ? 1 : (v[i] < mean - band ? -1 : 0);
  // fill undecided samples from the previous decided one (cyclically)
  int start = -1;
  for (int i = 0; i < S; ++i)
    if (sgn[i]) {
      start = i;
      break;
    }
  if (start < 0) return false;
  int last = sgn[start], changes = 0, run = 0, minrun = S;
  for (int k = 1; k <= S; ++k) {
    const int i = (start + k) % S;
    ++run;
    if (sgn[i] && sgn[i] != last) {
      ++changes;
      minrun = std::min(minrun, run);
      run = 0;
      last = sgn[i];
    }
  }
  return changes == 4 && minrun >= 2;
}

}  // namespace

// ------------------------------------------------------------------ cornerSubPix
// Attribution: this follows OpenCV's cornerSubPix (modules/imgproc/src/cornersubpix.cpp, OpenCV, Apache-2.0 /
// BSD-3-Clause, Copyright (C) Intel Corporation, Willow Garage, OpenCV Foundation et al.): the same Gaussian window
// mask, the normal-equation accumulators (a, b, c, bb1, bb2), the stop rules and the fallback to the input corner
// when a refined position leaves the search window -- the reference tool calls cv::cornerSubPix
// (Stereo_Calibration/Stereo_Calibration.cpp:108-120) and the calibration tests compare against its behaviour.
void corner_subpix(const Mat& gray, std::vector<std::array<double, 2>>& corners, int win, int iters, double eps) {
  const FImg img = to_float(gray);
  const int ww = 2 * win + 1;
  std::vector<double> mask((size_t)ww * ww);
  std::vector<double> mx(ww);
  for (int i = 0; i < ww; ++i) {
    const double x = (double)(i - win) / win;
    mx[i] = std::exp(-x * x);
  }
  for (int i = 0; i < ww; ++i)
    for (int j = 0; j < ww; ++j) mask[i * ww + j] = mx[j] * mx[i];
  const double eps2 = eps * eps;
  std::vector<float> patch((size_t)(ww + 2) * (ww + 2));
  for (auto& c : corners) {
    const double x0 = c[0], y0 = c[1];
    double cx = x0, cy = y0;
    for (int it = 0; it < iters; ++it) {
      // bilinear patch of (ww+2)^2 centred at (cx, cy) (cv::getRectSubPix, replicated border)
      for (int i = 0; i < ww + 2; ++i)
        for (int j = 0; j < ww + 2; ++j)
          patch[(size_t)i * (ww + 2) + j] = img.bilinear(cx + j - win - 1, cy + i - win - 1);
      double a = 0, b = 0, cc = 0, bb1 = 0, bb2 = 0;
      for (int i = 0; i < ww; ++i) {
        const double py = i - win;
        for (int j = 0; j < ww; ++j) {
          const double m = mask[i * ww + j];
          const float* p = &patch[(size_t)(i + 1) * (ww + 2) + j + 1];
          const double gx = p[1] - p[-1], gy = p[ww + 2] - p[-(ww + 2)];
          const double gxx = gx * gx * m, gxy = gx * gy * m, gyy = gy * gy * m;
          const double px = j - win;
          a += gxx;
          b += gxy;
          cc += gyy;
          bb1 += gxx * px + gxy * py;
          bb2 += gxy * px + gyy * py;
        }
      }
      const double det = a * cc - b * b;
      if (std::fabs(det) <= DBL_EPSILON * DBL_EPSILON) break;
      const double s = 1.0 / det;
      const double nx = cx + cc * s * bb1 - b * s * bb2;
      const double ny = cy - b * s * bb1 + a * s * bb2;
      const double err = (nx - cx) * (nx - cx) + (ny - cy) * (ny - cy);
      cx = nx;
      cy = ny;
      if (cx < 0 || cx >= gray.cols || cy < 0 || cy >= gray.rows) break;
      if (err <= eps2) break;
    }
    if (std::fabs(cx - x0) > win || std::fabs(cy - y0) > win) cx = x0, cy = y0;
    c = {cx, cy};
  }
}

// ------------------------------------------------------------------ chessboard detection
bool find_chessboard_corners(const Mat& gray, int cols, int rows, std::vector<std::array<double, 2>>& corners) {
  corners.clear();
  if (gray.empty() || gray.channels() != 1) return false;
  const FImg raw = to_float(gray);
  const FImg bl = gaussian(raw, 1.5);
  const int W = bl.w, H = bl.h;
  // saddle response -det(Hessian)
  std::vector<float> sc((size_t)W * H, 0.f);
  float smax = 0;
  for (int y = 2; y < H - 2; ++y)
    for (int x = 2; x < W - 2; ++x) {
      const float c = bl.at(x, y);
      const float ixx = bl.at(x + 1, y) - 2 * c + bl.at(x - 1, y);
      const float iyy = bl.at(x, y + 1) - 2 * c + bl.at(x, y - 1);
      const float ixy = 0.25f * (bl.at(x + 1, y + 1) - bl.at(x - 1, y + 1) - bl.at(x + 1, y - 1) + bl.at(x - 1, y - 1));
      const float s = ixy * ixy - ixx * iyy;
      sc[(size_t)y * W + x] = s > 0 ? s : 0;
      smax = std::max(smax, sc[(size_t)y * W + x]);
    }
  if (smax <= 0) return false;
  std::vector<Pt2> cand;
  const int nms = 3;
  for (int y = 4; y < H - 4; ++y)
    for (int x = 4; x < W - 4; ++x) {
      const float s = sc[(size_t)y * W + x];
      if (s < 0.005f * smax) continue;
      bool peak = true;
      for (int dy = -nms; dy <= nms && peak; ++dy)
        for (int dx = -nms; dx <= nms; ++dx) {
          const float o = sc[(size_t)(y + dy) * W + x + dx];
          if (o > s || (o == s && (dy < 0 || (dy == 0 && dx < 0)))) {
            peak = false;
            break;
          }
        }
      if (!peak) continue;
      if (!is_xcorner(bl, x, y, 3.0) && !is_xcorner(bl, x, y, 4.5) && !is_xcorner(bl, x, y, 6.5)) continue;
      cand.push_back({(double)x, (double)y});
    }
  const bool dbg = std::getenv("SA_CB_DEBUG") != nullptr;
  if (dbg) std::fprintf(stderr, "chessboard: %zu candidates\n", cand.size());
  if ((int)cand.size() < cols * rows) return false;
  corner_subpix(gray, cand, 3, 20, 0.01);
  // merge duplicates after refinement
  std::vector<Pt2> pts;
  for (auto& p : cand) {
    bool dup = false;
    for (auto& q : pts)
      if (std::hypot(p[0] - q[0], p[1] - q[1]) < 2.0) dup = true;
    if (!dup) pts.push_back(p);
  }
  const int N = (int)pts.size();
  auto dist = [&](int a, int b) { return std::hypot(pts[a][0] - pts[b][0], pts[a][1] - pts[b][1]); };
  // candidate seeds: points whose 4 nearest neighbours form two opposite pairs
  std::vector<int> order(N);
  for (int i = 0; i < N; ++i) order[i] = i;
  double cxm = 0, cym = 0;
  for (auto& p : pts) cxm += p[0], cym += p[1];
  cxm /= N, cym /= N;
  std::sort(order.begin(), order.end(), [&](int a, int b) {
    return std::hypot(pts[a][0] - cxm, pts[a][1] - cym) < std::hypot(pts[b][0] - cxm, pts[b][1] - cym);
  });
  for (int si = 0; si < std::min(N, 40); ++si) {
    const int s = order[si];
    std::vector<std::pair<double, int>> nb;
    for (int j = 0; j < N; ++j)
      if (j != s) nb.push_back({dist(s, j), j});
    if (nb.size() < 4) continue;
    std::partial_sort(nb.begin(), nb.begin() + 4, nb.end());
    Pt2 v[4];
    for (int k = 0; k < 4; ++k) v[k] = {pts[nb[k].second][0] - pts[s][0], pts[nb[k].second][1] - pts[s][1]};
    const double avg = (nb[0].first + nb[1].first + nb[2].first + nb[3].first) / 4;
    if (nb[3].first > 1.5 * nb[0].first) continue;
    int pa = -1, pb = -1;
    for (int k = 1; k < 4; ++k)
      if (std::hypot(v[0][0] + v[k][0], v[0][1] + v[k][1]) < 0.3 * avg) pa = k;
    if (pa < 0) continue;
    int o1 = -1, o2 = -1;
    for (int k = 1; k < 4; ++k)
      if (k != pa) (o1 < 0 ? o1 : o2) = k;
    if (std::hypot(v[o1][0] + v[o2][0], v[o1][1] + v[o2][1]) >= 0.3 * avg) continue;
    pb = o1;
    const double cr = v[0][0] * v[pb][1] - v[0][1] * v[pb][0];
    if (std::fabs(cr) < 0.5 * nb[0].first * nb[0].first) continue;
    // lattice growth from the seed
    std::map<std::pair<int, int>, int> grid;
    std::vector<int> used(N, 0);
    struct Node {
      int i, j;
      Pt2 a, b;  // local lattice steps along i and j
    };
    std::queue<Node> q;
    grid[{0, 0}] = s;
    used[s] = 1;
    q.push({0, 0, v[0], v[pb]});
    while (!q.empty()) {
      const Node nd = q.front();
      q.pop();
      const Pt2 p = pts[grid[{nd.i, nd.j}]];
      const int di[4] = {1, -1, 0, 0}, dj[4] = {0, 0, 1, -1};
      for (int k = 0; k < 4; ++k) {
        const std::pair<int, int> key{nd.i + di[k], nd.j + dj[k]};
        if (grid.count(key)) continue;
        Pt2 step = {di[k] * nd.a[0] + dj[k] * nd.b[0], di[k] * nd.a[1] + dj[k] * nd.b[1]};
        const std::pair<int, int> back{nd.i - di[k], nd.j - dj[k]};
        if (grid.count(back)) {  // continue the local spacing (perspective-aware)
          const Pt2 pb2 = pts[grid[back]];
          step = {p[0] - pb2[0], p[1] - pb2[1]};
        }
        const Pt2 pred{p[0] + step[0], p[1] + step[1]};
        const double len = std::hypot(step[0], step[1]);
        int best = -1;
        double bd = 0.3 * len;
        for (int j = 0; j < N; ++j) {
          if (used[j]) continue;
          const double d = std::hypot(pts[j][0] - pred[0], pts[j][1] - pred[1]);
          if (d < bd) {
            bd = d;
            best = j;
          }
        }
        if (best < 0) continue;
        used[best] = 1;
        grid[key] = best;
        const Pt2 real{pts[best][0] - p[0], pts[best][1] - p[1]};
        Node nn{key.first, key.second, nd.a, nd.b};
        if (di[k]) nn.a = {real[0] * di[k], real[1] * di[k]};
        else nn.b = {real[0] * dj[k], real[1] * dj[k]};
        q.push(nn);
      }
    }
    int imin = 1 << 30, imax = -(1 << 30), jmin = 1 << 30, jmax = -(1 << 30);
    for (auto& kv : grid) {
      imin = std::min(imin, kv.first.first);
      imax = std::max(imax, kv.first.first);
      jmin = std::min(jmin, kv.first.second);
      jmax = std::max(jmax, kv.first.second);
    }
    const int ni = imax - imin + 1, nj = jmax - jmin + 1;
    if (dbg) std::fprintf(stderr, "  seed %d: grid %zu nodes, %d x %d\n", s, grid.size(), ni, nj);
    if ((int)grid.size() != cols * rows) continue;
    bool i_is_cols;
    if (ni == cols && nj == rows) i_is_cols = true;
    else if (ni == rows && nj == cols) i_is_cols = false;
    else continue;
    if (cols == rows) i_is_cols = true;
    auto at = [&](int c, int r) -> const Pt2& {  // c along the `cols` axis, r along `rows`
      return i_is_cols ? pts[grid[{imin + c, jmin + r}]] : pts[grid[{imin + r, jmin + c}]];
    };
    // orientation: the cols axis points right (or down if near vertical); rows axis completes a
    // right-handed frame in image coordinates (y down)
    const Pt2 &c0 = at(0, 0), &c1 = at(cols - 1, 0), &r1 = at(0, rows - 1);
    Pt2 u{c1[0] - c0[0], c1[1] - c0[1]}, w{r1[0] - c0[0], r1[1] - c0[1]};
    const bool flip_c = std::fabs(u[0]) >= std::fabs(u[1]) ? u[0] < 0 : u[1] < 0;
    if (flip_c) u = {-u[0], -u[1]};
    const bool flip_r_raw = (u[0] * w[1] - u[1] * w[0]) < 0;
    const bool flip_r = flip_r_raw;
    corners.resize((size_t)cols * rows);
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols; ++c) {
        const int cc = flip_c ? cols - 1 - c : c, rr = flip_r ? rows - 1 - r : r;
        corners[(size_t)r * cols + c] = at(cc, rr);
      }
    return true;
  }
  return false;
}

// ------------------------------------------------------------------ calibrateCamera
double calibrate_camera(const std::vector<std::vector<std::array<double, 3>>>& obj,
                        const std::vector<std::vector<std::array<double, 2>>>& img, int width, int height,
                        CameraCalib& out, int max_iters) {
  const int nv = (int)obj.size();
  if (nv == 0 || img.size() != obj.size()) throw std::invalid_argument("calibrate_camera: need matching non-empty view lists");
  // focal lengths with the principal point at the centre (cvInitIntrinsicParams2D)
  const double cx = (width - 1) * 0.5, cy = (height - 1) * 0.5;
  std::vector<Mat33> Hs(nv);
  std::vector<double> AtA(4, 0.0), Atb(2, 0.0);
  for (int v = 0; v < nv; ++v) {
    std::vector<Pt2> src(obj[v].size());
    for (size_t i = 0; i < obj[v].size(); ++i) src[i] = {obj[v][i][0], obj[v][i][1]};
    Mat33 H = homography(src, img[v]);
    Hs[v] = H;
    H[0] -= H[6] * cx, H[1] -= H[7] * cx, H[2] -= H[8] * cx;
    H[3] -= H[6] * cy, H[4] -= H[7] * cy, H[5] -= H[8] * cy;
    double h[3], vv[3], d1[3], d2[3], n[4] = {0, 0, 0, 0};
    for (int j = 0; j < 3; ++j) {
      const double t0 = H[j * 3], t1 = H[j * 3 + 1];
      h[j] = t0, vv[j] = t1, d1[j] = (t0 + t1) * 0.5, d2[j] = (t0 - t1) * 0.5;
      n[0] += t0 * t0, n[1] += t1 * t1, n[2] += d1[j] * d1[j], n[3] += d2[j] * d2[j];
    }
    for (double& x : n) x = 1.0 / std::sqrt(x);
    for (int j = 0; j < 3; ++j) h[j] *= n[0], vv[j] *= n[1], d1[j] *= n[2], d2[j] *= n[3];
    const double rowsA[2][2] = {{h[0] * vv[0], h[1] * vv[1]}, {d1[0] * d2[0], d1[1] * d2[1]}};
    const double bs[2] = {-h[2] * vv[2], -d1[2] * d2[2]};
    for (int r = 0; r < 2; ++r) {
      for (int a = 0; a < 2; ++a) {
        Atb[a] += rowsA[r][a] * bs[r];
        for (int b = 0; b < 2; ++b) AtA[a * 2 + b] += rowsA[r][a] * rowsA[r][b];
      }
    }
  }
  const double det = AtA[0] * AtA[3] - AtA[1] * AtA[2];
  const double f0 = (AtA[3] * Atb[0] - AtA[1] * Atb[1]) / det, f1 = (-AtA[2] * Atb[0] + AtA[0] * Atb[1]) / det;
  double intr[9] = {std::sqrt(std::fabs(1.0 / f0)), std::sqrt(std::fabs(1.0 / f1)), cx, cy, 0, 0, 0, 0, 0};
  // per-view extrinsics from homographies of normalised coordinates
  std::vector<double> x(9 + 6 * nv);
  for (int i = 0; i < 9; ++i) x[i] = intr[i];
  for (int v = 0; v < nv; ++v) {
    std::vector<Pt2> src(obj[v].size()), dst(obj[v].size());
    for (size_t i = 0; i < obj[v].size(); ++i) {
      src[i] = {obj[v][i][0], obj[v][i][1]};
      dst[i] = {(img[v][i][0] - cx) / intr[0], (img[v][i][1] - cy) / intr[1]};
    }
    Vec3 r, t;
    pose_from_homography(homography(src, dst), r, t);
    for (int k = 0; k < 3; ++k) x[9 + 6 * v + k] = r[k], x[9 + 6 * v + 3 + k] = t[k];
  }
  LMProblem P;
  P.nparams = (int)x.size();
  P.ngroups = nv;
  P.residual = [&](const std::vector<double>& p, int g, std::vector<double>& r) {
    const Mat33 R = rodrigues({p[9 + 6 * g], p[10 + 6 * g], p[11 + 6 * g]});
    const Vec3 t{p[12 + 6 * g], p[13 + 6 * g], p[14 + 6 * g]};
    for (size_t i = 0; i < obj[g].size(); ++i) {
      const Pt2 q = project(p.data(), R, t, obj[g][i]);
      r.push_back(q[0] - img[g][i][0]);
      r.push_back(q[1] - img[g][i][1]);
    }
  };
  P.deps = [&](int g, std::vector<int>& idx) {
    idx.clear();
    for (int i = 0; i < 9; ++i) idx.push_back(i);
    for (int i = 0; i < 6; ++i) idx.push_back(9 + 6 * g + i);
  };
  const double cost = lm_solve(P, x, max_iters, 1e-12);
  size_t npts = 0;
  for (auto& o : obj) npts += o.size();
  intr_to(x.data(), out);
  out.rvecs.resize(nv);
  out.tvecs.resize(nv);
  for (int v = 0; v < nv; ++v) {
    out.rvecs[v] = {x[9 + 6 * v], x[10 + 6 * v], x[11 + 6 * v]};
    out.tvecs[v] = {x[12 + 6 * v], x[13 + 6 * v], x[14 + 6 * v]};
  }
  out.rms = std::sqrt(cost / npts);
  return out.rms;
}

// ------------------------------------------------------------------ stereoCalibrate
double stereo_calibrate(const std::vector<std::vector<std::array<double, 3>>>& obj,
                        const std::vector<std::vector<std::array<double, 2>>>& img1,
                        const std::vector<std::vector<std::array<double, 2>>>& img2, CameraCalib& c1,
                        CameraCalib& c2, Mat& Rout, Mat& Tout, int max_iters, double eps) {
  const int nv = (int)obj.size();
  if (nv == 0 || (int)c1.rvecs.size() != nv || (int)c2.rvecs.size() != nv)
    throw std::invalid_argument("stereo_calibrate: run calibrate_camera on both cameras first");
  // R, T initialisation: per-view relative poses, component-wise median (as OpenCV)
  std::vector<double> om[3], tt[3];
  for (int v = 0; v < nv; ++v) {
    const Mat33 R1 = rodrigues(c1.rvecs[v]), R2 = rodrigues(c2.rvecs[v]);
    const Mat33 R = mul33(R2, tr33(R1));
    const Vec3 r = rodrigues_inv(R);
    const Vec3 Rt1 = mv33(R, c1.tvecs[v]);
    for (int k = 0; k < 3; ++k) {
      om[k].push_back(r[k]);
      tt[k].push_back(c2.tvecs[v][k] - Rt1[k]);
    }
  }
  auto median = [](std::vector<double> a) {
    std::nth_element(a.begin(), a.begin() + a.size() / 2, a.end());
    return a[a.size() / 2];
  };
  std::vector<double> x(18 + 6 + 6 * nv);
  intr_from(c1, &x[0]);
  intr_from(c2, &x[9]);
  for (int k = 0; k < 3; ++k) x[18 + k] = median(om[k]), x[21 + k] = median(tt[k]);
  for (int v = 0; v < nv; ++v)
    for (int k = 0; k < 3; ++k) x[24 + 6 * v + k] = c1.rvecs[v][k], x[27 + 6 * v + k] = c1.tvecs[v][k];
  LMProblem P;
  P.nparams = (int)x.size();
  P.ngroups = nv;
  P.residual = [&](const std::vector<double>& p, int g, std::vector<double>& r) {
    const Mat33 R1 = rodrigues({p[24 + 6 * g], p[25 + 6 * g], p[26 + 6 * g]});
    const Vec3 t1{p[27 + 6 * g], p[28 + 6 * g], p[29 + 6 * g]};
    const Mat33 Rr = rodrigues({p[18], p[19], p[20]});
    const Mat33 R2 = mul33(Rr, R1);
    const Vec3 Rt = mv33(Rr, t1);
    const Vec3 t2{Rt[0] + p[21], Rt[1] + p[22], Rt[2] + p[23]};
    for (size_t i = 0; i < obj[g].size(); ++i) {
      const Pt2 a = project(&p[0], R1, t1, obj[g][i]);
      const Pt2 b = project(&p[9], R2, t2, obj[g][i]);
      r.push_back(a[0] - img1[g][i][0]);
      r.push_back(a[1] - img1[g][i][1]);
      r.push_back(b[0] - img2[g][i][0]);
      r.push_back(b[1] - img2[g][i][1]);
    }
  };
  P.deps = [&](int g, std::vector<int>& idx) {
    idx.clear();
    for (int i = 0; i < 24; ++i) idx.push_back(i);
    for (int i = 0; i < 6; ++i) idx.push_back(24 + 6 * g + i);
  };
  const double cost = lm_solve(P, x, max_iters, eps);
  size_t npts = 0;
  for (auto& o : obj) npts += o.size();
  intr_to(&x[0], c1);
  intr_to(&x[9], c2);
  for (int v = 0; v < nv; ++v) {
    c1.rvecs[v] = {x[24 + 6 * v], x[25 + 6 * v], x[26 + 6 * v]};
    c1.tvecs[v] = {x[27 + 6 * v], x[28 + 6 * v], x[29 + 6 * v]};
  }
  const Mat33 R = rodrigues({x[18], x[19], x[20]});
  Rout = mat_from(R.data(), 3, 3);
  Tout = mat_from(&x[21], 3, 1);
  const double rms = std::sqrt(cost / (2.0 * npts));
  c1.rms = c2.rms = rms;
  return rms;
}

// ------------------------------------------------------------------ the tool's pipeline
// Stereo_Calibration.cpp:67-182: images alternate left/right; pairs where either board is not found
// are skipped; corners refined with cornerSubPix(5x5, 30 it / 1e-3) when `subpix`; both cameras
// calibrated independently, then stereoCalibrate (USE_INTRINSIC_GUESS, 100 it / 1e-5) and
// stereoRectify (CALIB_ZERO_DISPARITY, alpha 0) at the left image size.
bool run_stereo_calibration(const std::vector<std::string>& images, int cols, int rows, double square, bool subpix,
                            CalibrationParam& out, StereoCalibReport* rep) {
  if (images.size() % 2) throw std::invalid_argument("image list must alternate left/right (even length)");
  std::vector<std::array<double, 3>> board;
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j) board.push_back({j * square, i * square, 0.0});
  std::vector<std::vector<std::array<double, 3>>> obj;
  std::vector<std::vector<std::array<double, 2>>> il, ir;
  int width = 0, height = 0;
  StereoCalibReport r;
  for (size_t k = 0; k + 1 < images.size(); k += 2) {
    const Mat L = imread(images[k]), R = imread(images[k + 1]);
    if (L.empty() || R.empty()) {
      r.skipped.push_back(images[k]);
      continue;
    }
    width = L.cols;
    height = L.rows;
    const Mat gl = bgr2gray(L), gr = bgr2gray(R);
    std::vector<std::array<double, 2>> cl, cr;
    const bool okr = find_chessboard_corners(gr, cols, rows, cr);
    const bool okl = find_chessboard_corners(gl, cols, rows, cl);
    if (!okl || !okr) {
      r.skipped.push_back(images[k]);
      continue;
    }
    if (subpix) {
      corner_subpix(gl, cl, 5, 30, 1e-3);
      corner_subpix(gr, cr, 5, 30, 1e-3);
    }
    il.push_back(cl);
    ir.push_back(cr);
    obj.push_back(board);
    r.used.push_back(images[k]);
  }
  if (obj.size() < 3) {
    if (rep) *rep = r;
    return false;
  }
  CameraCalib c1, c2;
  r.rms_left = calibrate_camera(obj, il, width, height, c1);
  r.rms_right = calibrate_camera(obj, ir, width, height, c2);
  Mat Rm, Tm;
  r.rms_stereo = stereo_calibrate(obj, il, ir, c1, c2, Rm, Tm, 100, 1e-5);
  out.intrinsic_left = c1.K;
  out.distCoeffs_left = c1.D;
  out.intrinsic_right = c2.K;
  out.distCoeffs_right = c2.D;
  out.R = Rm;
  out.T = Tm;
  stereo_rectify(c1.K, c1.D, c2.K, c2.D, width, height, Rm, Tm, out.R_L, out.R_R, out.P1, out.P2, out.Q, true, 0.0,
                 &out.validROIL, &out.validROIR);
  out.has_roi = true;
  r.width = width;
  r.height = height;
  r.corners_left = il;
  r.corners_right = ir;
  if (rep) *rep = r;
  return true;
}

}  // namespace sa
