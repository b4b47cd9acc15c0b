// Shared main() of the four demo executables (reference RAFTStereo/test/main.cpp, HitNet/test/main.cpp,
// CREStereo/test/main.cpp, FastACVNet_plus/test/main.cpp): load a stereo pair and the calibration,
// Initialize through the model's C ABI, run N frames on clones of the inputs (the reference loops
// 1000x, Fast-ACVNet+ 5x), then write disparity.jpg (CV_32FC1 saturated to u8 as cv::imwrite does),
// heatmap.jpg (CREStereo/test/main.cpp:7-24) and pointcloud.txt (x y z r g b per pixel).
// Unlike the reference, paths are flags (defaults = the reference's file names) and per-frame
// latency statistics are printed.
#pragma once
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sa/imgio.h"
#include "sa/mat.h"

typedef int (*sa_demo_run_fn)(void*, sa::Mat&, sa::Mat&, float*, sa::Mat&);

static int sa_demo_main(int argc, char** argv, const char* name, const char* default_model, int default_frames,
                        sa_demo_run_fn run, sa_demo_run_fn run_rectify) {
  std::string model = default_model, calib = "StereoCalibration.yml", left = "left0.jpg", right = "right0.jpg",
              out = ".";
  int frames = default_frames, gpu = 0;
  bool rectify = true;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--model") model = next();
    else if (a == "--calib") calib = next();
    else if (a == "--left") left = next();
    else if (a == "--right") right = next();
    else if (a == "--frames") frames = std::atoi(next().c_str());
    else if (a == "--gpu") gpu = std::atoi(next().c_str());
    else if (a == "--out") out = next();
    else if (a == "--no-rectify") rectify = false;
    else {
      std::printf("usage: %s [--model preset|weights.safetensors|preset@weights] [--calib StereoCalibration.yml]\n"
                  "          [--left left0.jpg] [--right right0.jpg] [--frames N] [--gpu ID] [--out DIR]%s\n",
                  name, run_rectify ? " [--no-rectify]" : "");
      return a == "--help" || a == "-h" ? 0 : 2;
    }
  }
  sa::Mat imageL = sa::imread(left), imageR = sa::imread(right);
  if (imageL.empty() || imageR.empty()) {
    std::fprintf(stderr, "cannot read %s / %s\n", left.c_str(), right.c_str());
    return 1;
  }
  void* h = Initialize(const_cast<char*>(model.c_str()), gpu, const_cast<char*>(calib.c_str()));
  if (!h) return 1;
  std::printf("%s: %s\n", name, Version(h));
  std::vector<float> pointcloud((size_t)imageL.cols * imageL.rows * 6);
  sa::Mat disparity, imageL1, imageR1;
  std::vector<double> ms;
  for (int i = 0; i < frames; ++i) {
    imageL1 = imageL.clone();
    imageR1 = imageR.clone();
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = (rectify || !run_rectify) ? (run_rectify ? run_rectify : run)(h, imageL1, imageR1, pointcloud.data(), disparity)
                                             : run(h, imageL1, imageR1, pointcloud.data(), disparity);
    ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    if (rc != 0) {
      std::fprintf(stderr, "run failed at frame %d\n", i);
      Release(h);
      return 1;
    }
  }
  std::vector<double> s = ms;
  std::sort(s.begin(), s.end());
  const size_t warm = std::min<size_t>(s.size() > 3 ? 3 : 0, s.size());
  double mean = 0;
  for (size_t i = warm; i < ms.size(); ++i) mean += ms[i];
  mean /= std::max<size_t>(1, ms.size() - warm);
  std::printf("frames %d  mean %.3f ms  p50 %.3f ms  p99 %.3f ms  (%.1f FPS)\n", frames, mean, s[s.size() / 2],
              s[std::min(s.size() - 1, (size_t)(s.size() * 0.99))], 1000.0 / mean);
  sa::imwrite(out + "/disparity.jpg", disparity);
  sa::imwrite(out + "/heatmap.jpg", sa::heatmap(disparity));
  sa::write_pointcloud_txt(out + "/pointcloud.txt", pointcloud.data(), (size_t)imageL.cols * imageL.rows);
  Release(h);
  return 0;
}
