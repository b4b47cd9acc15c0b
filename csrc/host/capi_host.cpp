// Flat C API of libstereo_host.so (CPU only): image I/O, colour maps, calibration files,
// rectification math.  Consumed by the Python package (ctypes) and usable from any FFI.
#include <cstdlib>
#include <cstring>
#include <string>

#include "sa/calib.h"
#include "sa/filestorage.h"
#include "sa/imgio.h"

using namespace sa;

namespace {
Mat* slot(CalibrationParam& p, const std::string& k) {
  if (k == "intrinsic_left") return &p.intrinsic_left;
  if (k == "distCoeffs_left") return &p.distCoeffs_left;
  if (k == "intrinsic_right") return &p.intrinsic_right;
  if (k == "distCoeffs_right") return &p.distCoeffs_right;
  if (k == "R") return &p.R;
  if (k == "T") return &p.T;
  if (k == "R_L") return &p.R_L;
  if (k == "R_R") return &p.R_R;
  if (k == "P1") return &p.P1;
  if (k == "P2") return &p.P2;
  if (k == "Q") return &p.Q;
  return nullptr;
}
Mat from_doubles(const double* v, int rows, int cols) {
  Mat m(rows, cols, SA_64FC1);
  std::memcpy(m.data, v, sizeof(double) * rows * cols);
  return m;
}
}  // namespace

extern "C" {

const char* sa_host_version(void) { return "stereoalgorithms_amd host 0.1.0"; }
void sa_host_free(void* p) { std::free(p); }

// ---------------------------------------------------------------- images
void* sa_imread(const char* path, int gray, int* h, int* w, int* c) {
  Mat m = imread(path, gray != 0);
  if (m.empty()) return nullptr;
  *h = m.rows;
  *w = m.cols;
  *c = m.channels();
  const size_t n = m.total() * m.channels();
  void* out = std::malloc(n);
  for (int r = 0; r < m.rows; ++r) std::memcpy((uint8_t*)out + (size_t)r * m.cols * m.channels(), m.ptr<uint8_t>(r), (size_t)m.cols * m.channels());
  return out;
}

int sa_imwrite(const char* path, const void* data, int h, int w, int c, int depth, int quality) {
  Mat m(h, w, sa_maketype(depth, c), const_cast<void*>(data));
  return imwrite(path, m, quality) ? 0 : -1;
}

int sa_jpeg_decode(const uint8_t* buf, size_t n, uint8_t* out, int* h, int* w, int* c) {
  Image img;
  if (!jpeg_decode(buf, n, img)) return -1;
  *h = img.height;
  *w = img.width;
  *c = img.channels;
  if (out) std::memcpy(out, img.data.data(), img.data.size());
  return 0;
}

int sa_heatmap(const float* disp, int h, int w, uint8_t* out_bgr) {
  Mat d(h, w, SA_32FC1, const_cast<float*>(disp));
  Mat hm = heatmap(d);
  std::memcpy(out_bgr, hm.data, (size_t)h * w * 3);
  return 0;
}

int sa_colormap_jet(const uint8_t* in, int n, uint8_t* out_bgr) {
  Mat m(1, n, SA_8UC1, const_cast<uint8_t*>(in));
  Mat c = apply_colormap_jet(m);
  std::memcpy(out_bgr, c.data, (size_t)n * 3);
  return 0;
}

int sa_bgr2gray(const uint8_t* in, int h, int w, uint8_t* out) {
  Mat m(h, w, SA_8UC3, const_cast<uint8_t*>(in));
  Mat g = bgr2gray(m);
  std::memcpy(out, g.data, (size_t)h * w);
  return 0;
}

int sa_write_pointcloud(const char* path, const float* cloud, long points) {
  return write_pointcloud_txt(path, cloud, (size_t)points) ? 0 : -1;
}

// ---------------------------------------------------------------- calibration files
void* sa_calib_new(void) { return new CalibrationParam(); }
void* sa_calib_load(const char* path) {
  auto* p = new CalibrationParam();
  if (!read_calibration(path, *p)) {
    delete p;
    return nullptr;
  }
  return p;
}
void sa_calib_free(void* h) { delete static_cast<CalibrationParam*>(h); }
int sa_calib_save(void* h, const char* path) {
  return write_calibration(path, *static_cast<CalibrationParam*>(h)) ? 0 : -1;
}
// returns element count (0 = empty key), -1 = unknown key
int sa_calib_get(void* h, const char* key, double* out, int cap, int* rows, int* cols) {
  Mat* m = slot(*static_cast<CalibrationParam*>(h), key);
  if (!m) return -1;
  *rows = m->rows;
  *cols = m->cols;
  const int n = (int)(m->total() * m->channels());
  for (int i = 0; i < n && i < cap; ++i) out[i] = m->get(i);
  return n;
}
int sa_calib_set(void* h, const char* key, const double* v, int rows, int cols) {
  Mat* m = slot(*static_cast<CalibrationParam*>(h), key);
  if (!m) return -1;
  *m = from_doubles(v, rows, cols);
  return 0;
}
int sa_calib_get_roi(void* h, int* out8) {
  auto* p = static_cast<CalibrationParam*>(h);
  const Rect r[2] = {p->validROIL, p->validROIR};
  for (int i = 0; i < 2; ++i) {
    out8[4 * i] = r[i].x;
    out8[4 * i + 1] = r[i].y;
    out8[4 * i + 2] = r[i].width;
    out8[4 * i + 3] = r[i].height;
  }
  return p->has_roi ? 1 : 0;
}
int sa_calib_set_roi(void* h, const int* v8) {
  auto* p = static_cast<CalibrationParam*>(h);
  p->validROIL = {v8[0], v8[1], v8[2], v8[3]};
  p->validROIR = {v8[4], v8[5], v8[6], v8[7]};
  p->has_roi = true;
  return 0;
}
// rectification maps for both cameras (float [H][W][2], CV_16SC2-quantised when quantize)
int sa_calib_rectify_maps(void* h, int width, int height, float* map_l, float* map_r, int quantize) {
  auto* p = static_cast<CalibrationParam*>(h);
  if (p->intrinsic_left.empty() || p->intrinsic_right.empty()) return -1;
  std::vector<float> m;
  init_undistort_rectify_map(p->intrinsic_left, p->distCoeffs_left, p->R_L, p->P1, width, height, m, quantize != 0);
  std::memcpy(map_l, m.data(), m.size() * 4);
  init_undistort_rectify_map(p->intrinsic_right, p->distCoeffs_right, p->R_R, p->P2, width, height, m, quantize != 0);
  std::memcpy(map_r, m.data(), m.size() * 4);
  return 0;
}
// recompute R_L, R_R, P1, P2, Q and the valid ROIs from K/D/R/T (cv::stereoRectify)
int sa_calib_stereo_rectify(void* h, int width, int height, double alpha, int zero_disparity) {
  auto* p = static_cast<CalibrationParam*>(h);
  if (p->R.empty() || p->T.empty()) return -1;
  stereo_rectify(p->intrinsic_left, p->distCoeffs_left, p->intrinsic_right, p->distCoeffs_right, width, height,
                 p->R, p->T, p->R_L, p->R_R, p->P1, p->P2, p->Q, zero_disparity != 0, alpha, &p->validROIL,
                 &p->validROIR);
  p->has_roi = true;
  return 0;
}

// ---------------------------------------------------------------- geometry kernels (CPU)
int sa_undistort_points(const double* K9, const double* D, int nd, const double* R9, const double* P, int prows,
                        int pcols, const double* src, int n, double* dst) {
  Mat K = from_doubles(K9, 3, 3);
  Mat Dm = nd > 0 ? from_doubles(D, 1, nd) : Mat();
  Mat Rm = R9 ? from_doubles(R9, 3, 3) : Mat();
  Mat Pm = P ? from_doubles(P, prows, pcols) : Mat();
  std::vector<std::array<double, 2>> s(n), d;
  for (int i = 0; i < n; ++i) s[i] = {src[2 * i], src[2 * i + 1]};
  undistort_points(s, d, K, Dm, Rm, Pm);
  for (int i = 0; i < n; ++i) {
    dst[2 * i] = d[i][0];
    dst[2 * i + 1] = d[i][1];
  }
  return 0;
}

int sa_project_points(const double* obj, int n, const double* rvec, const double* tvec, const double* K9,
                      const double* D, int nd, double* out) {
  std::vector<std::array<double, 3>> o(n);
  for (int i = 0; i < n; ++i) o[i] = {obj[3 * i], obj[3 * i + 1], obj[3 * i + 2]};
  std::vector<std::array<double, 2>> img;
  project_points(o, {rvec[0], rvec[1], rvec[2]}, {tvec[0], tvec[1], tvec[2]}, from_doubles(K9, 3, 3),
                 nd > 0 ? from_doubles(D, 1, nd) : Mat(), img);
  for (int i = 0; i < n; ++i) {
    out[2 * i] = img[i][0];
    out[2 * i + 1] = img[i][1];
  }
  return 0;
}

int sa_rodrigues(const double* r3, double* R9) {
  Mat33 R = rodrigues({r3[0], r3[1], r3[2]});
  std::memcpy(R9, R.data(), 72);
  return 0;
}
int sa_rodrigues_inv(const double* R9, double* r3) {
  Mat33 R;
  std::memcpy(R.data(), R9, 72);
  Vec3 r = rodrigues_inv(R);
  std::memcpy(r3, r.data(), 24);
  return 0;
}

int sa_remap_u8_cpu(const uint8_t* src, int h, int w, int c, const float* map, uint8_t* dst) {
  Mat s(h, w, sa_maketype(SA_8U, c), const_cast<uint8_t*>(src));
  Mat d(h, w, sa_maketype(SA_8U, c), dst);
  std::vector<float> m(map, map + (size_t)h * w * 2);
  remap_cpu(s, d, m);
  return 0;
}

int sa_reproject_cpu(const float* disp, int h, int w, const double* Q16, float* xyz) {
  reproject_cpu(disp, h, w, Q16, xyz);
  return 0;
}

// ---------------------------------------------------------------- calibration tool
// gray u8 [h][w] -> corners [cols*rows][2] (row-major from the top-left); returns 1 if found
int sa_find_chessboard(const uint8_t* gray, int h, int w, int cols, int rows, int subpix, double* out) {
  Mat g(h, w, SA_8UC1, const_cast<uint8_t*>(gray));
  std::vector<std::array<double, 2>> c;
  if (!find_chessboard_corners(g, cols, rows, c)) return 0;
  if (subpix) corner_subpix(g, c, 5, 30, 1e-3);
  for (size_t i = 0; i < c.size(); ++i) out[2 * i] = c[i][0], out[2 * i + 1] = c[i][1];
  return 1;
}

// newline-separated alternating left/right image paths -> calibration handle filled in;
// rms[3] = left, right, stereo RMS; returns the number of pairs used (< 0 on failure)
int sa_stereo_calibrate_images(const char* paths, int cols, int rows, double square, int subpix, void* calib,
                               double* rms) {
  std::vector<std::string> list;
  std::string cur;
  for (const char* q = paths; ; ++q) {
    if (*q == '\n' || *q == 0) {
      if (!cur.empty()) list.push_back(cur);
      cur.clear();
      if (!*q) break;
    } else {
      cur += *q;
    }
  }
  try {
    StereoCalibReport rep;
    if (!run_stereo_calibration(list, cols, rows, square, subpix != 0, *static_cast<CalibrationParam*>(calib), &rep))
      return -1;
    if (rms) rms[0] = rep.rms_left, rms[1] = rep.rms_right, rms[2] = rep.rms_stereo;
    return (int)rep.used.size();
  } catch (const std::exception&) {
    return -2;
  }
}

}  // extern "C"
