// Stereo camera model: calibration parameters, OpenCV-equivalent undistortion / rectification
// math, rectification maps, disparity reprojection and the chessboard calibration pipeline.
//
// Reference behaviour reproduced here (OpenCV is not part of this stack):
//   * CalibrationParam — the 11 matrices of RAFTStereo/include/TRTRAFTStereo.h:30-43 (+ ROIs of
//     Stereo_Calibration/Stereo_Calibration.cpp:11-25), read by ReadObjectYml
//     (RAFTStereo/src/RAFTStereoAlgorithm.cpp:79-95) and written at Stereo_Calibration.cpp:165-179;
//   * init_undistort_rectify_map — cv::initUndistortRectifyMap(..., CV_16SC2) as called per frame at
//     RAFTStereo/src/RAFTStereoAlgorithm.cpp:120-121 (here computed ONCE, then applied by the HIP
//     remap kernel or remap_cpu); 4/5/8/12/14-coefficient distortion;
//   * stereo_rectify — cv::stereoRectify (Bouguet, CALIB_ZERO_DISPARITY, alpha) of
//     Stereo_Calibration.cpp:162;
//   * calibrate_camera / stereo_calibrate / find_chessboard_corners / corner_subpix — the
//     calibration tool pipeline (Stereo_Calibration.cpp:67-182).
#pragma once
#include <array>
#include <string>
#include <vector>

#include "sa/mat.h"

namespace sa {

struct Rect {
  int x = 0, y = 0, width = 0, height = 0;
};

struct CalibrationParam {
  Mat intrinsic_left, distCoeffs_left, intrinsic_right, distCoeffs_right;
  Mat R, T, R_L, R_R, P1, P2, Q;
  Rect validROIL, validROIR;
  bool has_roi = false;
};

// YAML (OpenCV FileStorage) load/save.  Missing keys leave empty matrices (reference semantics).
bool read_calibration(const std::string& path, CalibrationParam& p);
bool write_calibration(const std::string& path, const CalibrationParam& p);

using Mat33 = std::array<double, 9>;
using Vec3 = std::array<double, 3>;

// Rodrigues rotation vector <-> matrix (with optional 3x9 Jacobian d R / d r, row-major)
Mat33 rodrigues(const Vec3& r, double* jac = nullptr);
Vec3 rodrigues_inv(const Mat33& R);

// Distortion vector padded to 14 coefficients (k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4 tx ty)
std::array<double, 14> dist14(const Mat& D);

// cv::undistortPoints(src, dst, K, D, R, P) with the default 5 fixed-point iterations.
// R / P may be empty (identity / normalised output).
void undistort_points(const std::vector<std::array<double, 2>>& src, std::vector<std::array<double, 2>>& dst,
                      const Mat& K, const Mat& D, const Mat& R, const Mat& P, int iters = 5);

// cv::initUndistortRectifyMap.  Float maps [H][W][2] (x, y) quantised exactly as the CV_16SC2 path
// (1/32 pixel) when `quantize` is set, so the GPU remap reproduces cv::remap(INTER_LINEAR)
// bit-exactly.
void init_undistort_rectify_map(const Mat& K, const Mat& D, const Mat& R, const Mat& P, int width,
                                int height, std::vector<float>& map_xy, bool quantize = true);

// cv::remap(src, dst, map, INTER_LINEAR, BORDER_CONSTANT 0) for u8 images, using OpenCV's 1/32
// fixed-point bilinear table (host reference for the HIP kernel; in-place safe).
void remap_cpu(const Mat& src, Mat& dst, const std::vector<float>& map_xy);

// cv::stereoRectify with CALIB_ZERO_DISPARITY when zero_disparity; alpha in [-1, 1] (-1 = default
// scaling, which OpenCV treats like 0 for this function).
void stereo_rectify(const Mat& K1, const Mat& D1, const Mat& K2, const Mat& D2, int width, int height,
                    const Mat& R, const Mat& T, Mat& R1, Mat& R2, Mat& P1, Mat& P2, Mat& Q,
                    bool zero_disparity = true, double alpha = -1, Rect* roi1 = nullptr, Rect* roi2 = nullptr);

// Project object points with pose (rvec, tvec), intrinsics and distortion (cv::projectPoints).
void project_points(const std::vector<std::array<double, 3>>& obj, const Vec3& rvec, const Vec3& tvec,
                    const Mat& K, const Mat& D, std::vector<std::array<double, 2>>& img);

// disparity -> XYZ (cv::reprojectImageTo3D semantics with the full 4x4 Q), CPU reference
void reproject_cpu(const float* disp, int H, int W, const double Q[16], float* xyz /*[H][W][3]*/);

// ------------------------------------------------------------------ calibration tool
// Chessboard detection on a grey u8 image; pattern = inner corners (cols, rows) as in
// cv::findChessboardCorners(Size(11, 8)).  Corners are ordered row-major from the top-left.
bool find_chessboard_corners(const Mat& gray, int pattern_cols, int pattern_rows,
                             std::vector<std::array<double, 2>>& corners);
// cv::cornerSubPix(win = (win,win), zeroZone (-1,-1), criteria iters/eps)
void corner_subpix(const Mat& gray, std::vector<std::array<double, 2>>& corners, int win = 5, int iters = 30,
                   double eps = 1e-3);

struct CameraCalib {
  Mat K, D;  // 3x3, 1x5
  std::vector<Vec3> rvecs, tvecs;
  double rms = 0;
};
// Zhang initialisation (homographies) + Levenberg-Marquardt over all views (cv::calibrateCamera,
// k1 k2 p1 p2 k3 model).
double calibrate_camera(const std::vector<std::vector<std::array<double, 3>>>& obj,
                        const std::vector<std::vector<std::array<double, 2>>>& img, int width, int height,
                        CameraCalib& out, int max_iters = 100);
// cv::stereoCalibrate with CALIB_USE_INTRINSIC_GUESS: joint LM over both cameras' intrinsics,
// the relative pose (R, T) and the per-view left poses.  Returns the RMS reprojection error.
double stereo_calibrate(const std::vector<std::vector<std::array<double, 3>>>& obj,
                        const std::vector<std::vector<std::array<double, 2>>>& img1,
                        const std::vector<std::vector<std::array<double, 2>>>& img2, CameraCalib& c1,
                        CameraCalib& c2, Mat& R, Mat& T, int max_iters = 100, double eps = 1e-5);

struct StereoCalibReport {
  std::vector<std::string> used, skipped;  // left image of each pair
  double rms_left = 0, rms_right = 0, rms_stereo = 0;
  int width = 0, height = 0;
  std::vector<std::vector<std::array<double, 2>>> corners_left, corners_right;
};
// The whole Stereo_Calibration pipeline over an alternating left/right image list
// (Stereo_Calibration.cpp:67-182).  Fills every CalibrationParam field incl. ROIs.
bool run_stereo_calibration(const std::vector<std::string>& images, int cols, int rows, double square, bool subpix,
                            CalibrationParam& out, StereoCalibReport* report = nullptr);

}  // namespace sa
