// Host-code sanitizer harness (ASan/UBSan for host code).  Built together with
// csrc/host/*.cpp under -fsanitize=address,undefined by tools/sanitize/run.sh (and
// tests/test_tools_cpu.py::test_host_sanitizers); exercises the CPU-only subsystems on the
// reference's own fixtures: calibration YAML read/write (5- and 8-coefficient files), rectification
// maps + CPU remap, stereoRectify, JPEG decode/encode, PNG round trip, JET heat-map, point-cloud
// writer, chessboard detection + sub-pixel refinement, and a short stereo calibration.
//
//   host_check <fixtures_dir> <scratch_dir>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <random>
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

static std::vector<uint8_t> slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}

// Malformed-input cases for the decoders: crafted headers that used to overrun fixed tables,
// truncations at every marker, and random byte mutations of the real fixtures.  Any decode result is fine;
// only out-of-bounds accesses / UB (caught by ASan/UBSan) are failures.
static int malformed_codecs(const std::string& fx, const std::string& tmp) {
  const std::vector<uint8_t> jpg = slurp(fx + "/left0.jpg");
  CHECK(jpg.size() > 1000);
  Image img;
  // DHT whose 16 code counts sum to 16 * 255 = 4080 (> the 256-entry value table)
  {
    std::vector<uint8_t> f = {0xFF, 0xD8, 0xFF, 0xC4};
    const int len = 2 + 17 + 64;
    f.push_back(len >> 8), f.push_back(len & 255), f.push_back(0x10);
    for (int i = 0; i < 16; ++i) f.push_back(255);
    for (int i = 0; i < 64; ++i) f.push_back(1);
    f.push_back(0xFF), f.push_back(0xD9);
    CHECK(!jpeg_decode(f.data(), f.size(), img));
  }
  // SOF naming quantisation table 200, sampling 15x15 and 200 components in a short segment
  {
    std::vector<uint8_t> f = {0xFF, 0xD8, 0xFF, 0xC0, 0x00, 0x11, 8, 0, 16, 0, 16, 3,
                              1, 0x11, 200, 2, 0xFF, 0, 3, 0x11, 0, 0xFF, 0xD9};
    CHECK(!jpeg_decode(f.data(), f.size(), img));
    f[11] = 200;
    CHECK(!jpeg_decode(f.data(), f.size(), img));
  }
  // SOS with table selectors 15/15 and more components than the frame declares
  {
    std::vector<uint8_t> f = {0xFF, 0xD8, 0xFF, 0xC0, 0x00, 0x0B, 8, 0, 8, 0, 8, 1, 1, 0x11, 0,
                              0xFF, 0xDA, 0x00, 0x08, 1, 1, 0xFF, 0, 63, 0, 0, 0, 0xFF, 0xD9};
    CHECK(!jpeg_decode(f.data(), f.size(), img));
    f[19] = 9;
    CHECK(!jpeg_decode(f.data(), f.size(), img));
  }
  // truncation at every 97th byte and 300 random 1-8 byte mutations of the real file
  for (size_t n = 0; n < jpg.size(); n += 97) (void)jpeg_decode(jpg.data(), n, img);
  std::mt19937 rng(1234);
  for (int t = 0; t < 300; ++t) {
    std::vector<uint8_t> f = jpg;
    const int k = 1 + (int)(rng() % 8);
    for (int i = 0; i < k; ++i) f[rng() % std::min<size_t>(f.size(), 700)] = (uint8_t)rng();  // header region
    (void)jpeg_decode(f.data(), f.size(), img);
  }
  // PNG: short IHDR, huge / zero dimensions, bad colour type; mutations of a real PNG
  Mat small(8, 8, SA_8UC3);
  for (int i = 0; i < 8 * 8 * 3; ++i) small.data[i] = (uint8_t)(i * 7);
  CHECK(imwrite(tmp + "/s.png", small));
  const std::vector<uint8_t> png = slurp(tmp + "/s.png");
  CHECK(png.size() > 33 && png_decode(png.data(), png.size(), img));
  {
    std::vector<uint8_t> f = png;
    f[11] = 5;  // IHDR length 5
    CHECK(!png_decode(f.data(), f.size(), img));
    f = png;
    f[16] = 0x7F, f[20] = 0x7F;  // 2^31-scale width and height
    CHECK(!png_decode(f.data(), f.size(), img));
    f = png;
    f[25] = 7;  // colour type 7
    CHECK(!png_decode(f.data(), f.size(), img));
  }
  for (size_t n = 0; n < png.size(); n += 5) (void)png_decode(png.data(), n, img);
  for (int t = 0; t < 300; ++t) {
    std::vector<uint8_t> f = png;
    f[rng() % f.size()] = (uint8_t)rng();
    (void)png_decode(f.data(), f.size(), img);
  }
  return 0;
}

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
  CHECK(malformed_codecs(fx, tmp) == 0);
  std::printf("host_check ok: %zu corners, %zu pairs used, rms %.3f\n", corners.size(), rep.used.size(),
              rep.rms_stereo);
  return 0;
}
