// Stereo_Calibration — chessboard stereo calibration tool (reference: Stereo_Calibration/Stereo_Calibration.cpp,
// README.en.md:9 usage `./Stereo_Calibration 5 8 40 1`).
//
//   Stereo_Calibration [image_list.xml] [cols rows square_mm [subpix]] [-o StereoCalibration.yml] [-r rectified_dir]
//
// Defaults follow the reference's hard-coded values (:222-233): stereo_calib.xml, 11 x 8 inner
// corners, 25 mm squares, sub-pixel refinement on.  Pipeline (:67-182): corners on every left/right
// pair, per-camera calibration, stereo calibration, Bouguet rectification (alpha 0, zero disparity),
// StereoCalibration.yml (13 keys).  Then, like :236-289 but headless: every pair is remapped and
// written to <rectified_dir>/{left,right}<i>.jpg plus a side-by-side check image with the valid
// ROIs and green epipolar lines every 40 px (<rectified_dir>/rectified<i>.jpg).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "sa/calib.h"
#include "sa/imgio.h"

using namespace sa;

static bool read_image_list(const std::string& path, std::vector<std::string>& out) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  const size_t a = s.find("<imagelist>"), b = s.find("</imagelist>");
  if (a == std::string::npos || b == std::string::npos) return false;
  std::istringstream body(s.substr(a + 11, b - a - 11));
  std::string dir = path.substr(0, path.find_last_of('/') == std::string::npos ? 0 : path.find_last_of('/') + 1);
  std::string tok;
  while (body >> tok) {
    if (tok.size() >= 2 && tok.front() == '"' && tok.back() == '"') tok = tok.substr(1, tok.size() - 2);
    out.push_back(tok[0] == '/' ? tok : dir + tok);
  }
  return true;
}

static void put(Mat& img, int x, int y, uint8_t b, uint8_t g, uint8_t r) {
  if (x < 0 || y < 0 || x >= img.cols || y >= img.rows) return;
  uint8_t* p = img.ptr<uint8_t>(y) + 3 * x;
  p[0] = b, p[1] = g, p[2] = r;
}

int main(int argc, char** argv) {
  std::string list = "stereo_calib.xml", out = "StereoCalibration.yml", rect_dir;
  std::vector<std::string> pos;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "-o" && i + 1 < argc) out = argv[++i];
    else if (a == "-r" && i + 1 < argc) rect_dir = argv[++i];
    else if (a == "-h" || a == "--help") {
      std::printf("usage: %s [image_list.xml] [cols rows square_mm [subpix]] [-o out.yml] [-r rectified_dir]\n", argv[0]);
      return 0;
    } else pos.push_back(a);
  }
  size_t k = 0;
  if (k < pos.size() && pos[k].find(".xml") != std::string::npos) list = pos[k++];
  int cols = 11, rows = 8, subpix = 1;
  double square = 25.0;
  if (pos.size() >= k + 3) {
    cols = std::atoi(pos[k].c_str());
    rows = std::atoi(pos[k + 1].c_str());
    square = std::atof(pos[k + 2].c_str());
    if (pos.size() - k >= 4) subpix = std::atoi(pos[k + 3].c_str());
  }
  std::vector<std::string> images;
  if (!read_image_list(list, images)) {
    std::fprintf(stderr, "cannot read image list %s\n", list.c_str());
    return 1;
  }
  std::printf("%zu images, board %d x %d inner corners, %.3g mm squares\n", images.size(), cols, rows, square);
  CalibrationParam cal;
  StereoCalibReport rep;
  if (!run_stereo_calibration(images, cols, rows, square, subpix != 0, cal, &rep)) {
    std::fprintf(stderr, "calibration failed: %zu usable pairs\n", rep.used.size());
    return 2;
  }
  for (const auto& s : rep.skipped) std::printf("chessboard not found: %s (pair skipped)\n", s.c_str());
  std::printf("left RMS %.4f px, right RMS %.4f px\n", rep.rms_left, rep.rms_right);
  std::printf("Stereo Calibration done with RMS error = %.6f (%zu pairs)\n", rep.rms_stereo, rep.used.size());
  if (!write_calibration(out, cal)) {
    std::fprintf(stderr, "cannot write %s\n", out.c_str());
    return 3;
  }
  std::printf("Save Calibration to %s\n", out.c_str());
  if (rect_dir.empty()) return 0;
  CalibrationParam back;
  read_calibration(out, back);
  std::vector<float> ml, mr;
  init_undistort_rectify_map(back.intrinsic_left, back.distCoeffs_left, back.R_L, back.P1, rep.width, rep.height, ml);
  init_undistort_rectify_map(back.intrinsic_right, back.distCoeffs_right, back.R_R, back.P2, rep.width, rep.height, mr);
  for (size_t i = 0; i + 1 < images.size(); i += 2) {
    const Mat L = imread(images[i]), R = imread(images[i + 1]);
    if (L.empty() || R.empty()) continue;
    Mat rl, rr;
    remap_cpu(L, rl, ml);
    remap_cpu(R, rr, mr);
    const std::string idx = std::to_string(i / 2);
    imwrite(rect_dir + "/left" + idx + ".jpg", rl);
    imwrite(rect_dir + "/right" + idx + ".jpg", rr);
    Mat canvas(rl.rows, 2 * rl.cols, SA_8UC3);
    for (int y = 0; y < rl.rows; ++y) {
      std::memcpy(canvas.ptr<uint8_t>(y), rl.ptr<uint8_t>(y), (size_t)rl.cols * 3);
      std::memcpy(canvas.ptr<uint8_t>(y) + (size_t)rl.cols * 3, rr.ptr<uint8_t>(y), (size_t)rr.cols * 3);
    }
    const Rect rois[2] = {back.validROIL, back.validROIR};
    for (int s = 0; s < 2; ++s) {
      const Rect& r = rois[s];
      const int ox = s * rl.cols;
      for (int x = r.x; x < r.x + r.width; ++x) put(canvas, ox + x, r.y, 0, 0, 255), put(canvas, ox + x, r.y + r.height - 1, 0, 0, 255);
      for (int y = r.y; y < r.y + r.height; ++y) put(canvas, ox + r.x, y, 0, 0, 255), put(canvas, ox + r.x + r.width - 1, y, 0, 0, 255);
    }
    for (int y = 0; y < canvas.rows; y += 40)
      for (int x = 0; x < canvas.cols; ++x) put(canvas, x, y, 0, 255, 0);
    imwrite(rect_dir + "/rectified" + idx + ".jpg", canvas);
  }
  std::printf("rectified pairs written to %s\n", rect_dir.c_str());
  return 0;
}
