// Host-code sanitizer harness (ASan/UBSan for host code).  Built together with
// csrc/host/*.cpp under -fsanitize=address,undefined by tools/sanitize/run.sh (and
// tests/test_tools_cpu.py::test_host_sanitizers); exercises the CPU-only subsystems on the
// reference's own fixtures: calibration YAML read/write (5- and 8-coefficient files), rectification
// maps + CPU remap, stereoRectify, JPEG decode/encode, PNG round trip, JET heat-map, point-cloud
// writer, chessboard detection + sub-pixel refinement, and a short stereo calibration.
//
//   host_check <fixtures_dir> <scratch_dir>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "sa/calib.h"
#include "sa/imgio.h"

using namespace sa;

#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const std::string fx = argv[1], tmp = argv[2];
  // calibration YAML
  CalibrationParam c5, c8;
  CHECK(read_calibration(fx + "/StereoCalibration.yml", c5));
  CHECK(read_calibration(fx + "/StereoCalibration_new.yml", c8));
  CHECK(write_calibration(tmp + "/rt.yml", c5));
  CalibrationParam rt;
  CHECK(read_calibration(tmp + "/rt.yml", rt));
  CHECK(rt.Q.rows == 4 && rt.Q.cols == 4);
  // rectification maps (5 and 8 coefficients) + CPU remap of the reference pair
  Mat left = imread(fx + "/left0.jpg");
  CHECK(!left.empty() && left.rows == 480 && left.cols == 640);
  for (const CalibrationParam* c : {&c5, &c8}) {
    std::vector<float> map;
    init_undistort_rectify_map(c->intrinsic_left, c->distCoeffs_left, c->R_L, c->P1, 640, 480, map, true);
    CHECK(map.size() == 640u * 480u * 2u);
    Mat rect;
    remap_cpu(left, rect, map);
    CHECK(rect.rows == 480 && rect.cols == 640);
  }
  Mat R1, R2, P1, P2, Q;
  Rect roi1, roi2;
  stereo_rectify(c5.intrinsic_left, c5.distCoeffs_left, c5.intrinsic_right, c5.distCoeffs_right, 640, 480, c5.R, c5.T,
                 R1, R2, P1, P2, Q, true, 0.0, &roi1, &roi2);
  CHECK(Q.rows == 4);
  // image codecs + visualisation
  CHECK(imwrite(tmp + "/l.jpg", left));
  CHECK(imwrite(tmp + "/l.png", left));
  Mat png = imread(tmp + "/l.png");
  CHECK(png.rows == 480 && std::memcmp(png.data, left.data, (size_t)480 * 640 * 3) == 0);
  Mat disp(480, 640, SA_32FC1);
  for (int y = 0; y < 480; ++y)
    for (int x = 0; x < 640; ++x) disp.ptr<float>(y)[x] = (float)(x % 97) * 0.5f;
  Mat hm = heatmap(disp);
  CHECK(hm.rows == 480 && hm.channels() == 3);
  std::vector<float> cloud((size_t)16 * 6, 1.f);
  CHECK(write_pointcloud_txt(tmp + "/pc.txt", cloud.data(), 16));
  // chessboard + a small stereo calibration on the reference captures
  std::vector<std::string> imgs;
  for (int i : {1, 2, 3, 4}) {
    imgs.push_back(fx + "/calib/left_right_image/left" + std::to_string(i) + ".jpg");
    imgs.push_back(fx + "/calib/left_right_image/right" + std::to_string(i) + ".jpg");
  }
  Mat gray = bgr2gray(imread(imgs[0]));
  std::vector<std::array<double, 2>> corners;
  if (find_chessboard_corners(gray, 11, 8, corners)) corner_subpix(gray, corners);
  CalibrationParam out;
  StereoCalibReport rep;
  (void)run_stereo_calibration(imgs, 11, 8, 25.0, true, out, &rep);
  std::printf("host_check ok: %zu corners, %zu pairs used, rms %.3f\n", corners.size(), rep.used.size(),
              rep.rms_stereo);
  return 0;
}
