// Image / point-cloud I/O and visualisation used by the demos and the calibration tool.
//
// Replaces the OpenCV calls of the reference demos (RAFTStereo/test/main.cpp:13-39,
// CREStereo/test/main.cpp:7-24,55-69): cv::imread / cv::imwrite (JPEG via the in-tree baseline codec,
// PNG via zlib, PPM/PGM), the float->u8 saturation OpenCV applies when a CV_32FC1 disparity is
// written as JPEG, cv::applyColorMap(COLORMAP_JET) with OpenCV's exact 256-entry LUT, the demo
// `heatmap()` (min-max normalisation + convertScaleAbs + JET) and the `pointcloud.txt` writer
// (`x y z r g b` per line, iostream default precision).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "sa/mat.h"

namespace sa {

struct Image {
  int width = 0, height = 0, channels = 0;  // channels 1 (grey) or 3 (BGR)
  std::vector<uint8_t> data;
};

bool jpeg_decode(const uint8_t* data, size_t size, Image& img, std::string* err = nullptr);
bool jpeg_encode(const Image& img, int quality, std::vector<uint8_t>& out);
bool png_decode(const uint8_t* data, size_t size, Image& img, std::string* err = nullptr);
bool png_encode(const Image& img, std::vector<uint8_t>& out);

// cv::imread(path) (IMREAD_COLOR: 3-channel BGR; grey files are expanded) / IMREAD_GRAYSCALE
Mat imread(const std::string& path, bool grayscale = false);
// cv::imwrite: format from extension (.jpg/.jpeg q95, .png, .ppm/.pgm); CV_32F/64F input is
// saturated to u8 first (OpenCV's convertTo(CV_8U) fallback)
bool imwrite(const std::string& path, const Mat& m, int jpeg_quality = 95);

// BGR -> grey (cv::cvtColor COLOR_BGR2GRAY fixed-point coefficients)
Mat bgr2gray(const Mat& bgr);
// cv::applyColorMap(src u8, COLORMAP_JET) -> BGR
Mat apply_colormap_jet(const Mat& u8);
// reference demo heatmap() (CREStereo/test/main.cpp:7-24)
Mat heatmap(const Mat& disparity_f32);
// float -> u8 with OpenCV saturate_cast (round half to even, clamp)
Mat to_u8(const Mat& f32, double scale = 1.0, double shift = 0.0);

// pointcloud.txt (H*W lines "x y z r g b"), std::ostream default formatting
bool write_pointcloud_txt(const std::string& path, const float* cloud, size_t points);

}  // namespace sa
