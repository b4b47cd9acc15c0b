// Shared main() of the four demo executables (reference RAFTStereo/test/main.cpp, HitNet/test/main.cpp,
// CREStereo/test/main.cpp, FastACVNet_plus/test/main.cpp): load a stereo pair and the calibration,
// Initialize through the model's C ABI, run N frames on clones of the inputs (the reference loops
// 1000x, Fast-ACVNet+ 5x), then write disparity.jpg (CV_32FC1 saturated to u8 as cv::imwrite does),
// heatmap.jpg (CREStereo/test/main.cpp:7-24) and pointcloud.txt (x y z r g b per pixel).
// Unlike the reference, paths are flags (defaults = the reference's file names) and per-frame
// latency statistics are printed.  --list FILE streams many pairs ("left right" per line) through sa::FramePipeline
// (sa/pipeline.h): JPEG decode of pair i+1 and the disk writes of pair i-1 run on host threads while the GPU
// works on pair i; --save-all writes disparity_<i>.jpg per pair.
#pragma once
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <sstream>
#include <string>
#include <vector>

#include "sa/imgio.h"
#include "sa/mat.h"
#include "sa/pipeline.h"

typedef int (*sa_demo_run_fn)(void*, sa::Mat&, sa::Mat&, float*, sa::Mat&);

// --list mode: every "left right" line of `list` through the frame pipeline
static int sa_demo_stream(void* h, sa_demo_run_fn fn, const std::string& list, const std::string& out, bool save_all,
                          int depth) {
  std::ifstream in(list);
  if (!in) {
    std::fprintf(stderr, "cannot read %s\n", list.c_str());
    return 1;
  }
  std::vector<std::pair<std::string, std::string>> pairs;
  for (std::string line; std::getline(in, line);) {
    std::istringstream ls(line);
    std::string l, r;
    if (ls >> l >> r && l[0] != '#') pairs.emplace_back(l, r);
  }
  sa::Mat last_disp;
  std::vector<float> last_cloud;
  sa::FramePipeline pipe(depth);
  const sa::PipelineStats st = pipe.run(
      [&](sa::StereoFrame& f) {
        if (f.index >= (long)pairs.size()) return false;
        f.tag = pairs[f.index].first;
        f.left = sa::imread(pairs[f.index].first);
        f.right = sa::imread(pairs[f.index].second);
        if (f.left.empty() || f.right.empty()) throw std::runtime_error("cannot read " + f.tag);
        f.cloud.resize((size_t)f.left.rows * f.left.cols * 6);
        return true;
      },
      [&](sa::StereoFrame& f) { return fn(h, f.left, f.right, f.cloud.data(), f.disparity); },
      [&](sa::StereoFrame& f) {
        if (save_all) sa::imwrite(out + "/disparity_" + std::to_string(f.index) + ".jpg", f.disparity);
        if (f.index + 1 == (long)pairs.size()) {
          last_disp = f.disparity.clone();
          last_cloud = f.cloud;
        }
      });
  if (st.status != 0) {
    std::fprintf(stderr, "stream failed: %s\n", st.error.c_str());
    return 1;
  }
  std::printf("stream frames %ld  wall %.1f ms  %.1f FPS pipelined  run mean %.3f ms  p50 %.3f  p99 %.3f\n", st.frames,
              st.wall_ms, st.fps, st.infer_mean_ms, st.infer_p50_ms, st.infer_p99_ms);
  if (!last_disp.empty()) {
    sa::imwrite(out + "/disparity.jpg", last_disp);
    sa::imwrite(out + "/heatmap.jpg", sa::heatmap(last_disp));
    sa::write_pointcloud_txt(out + "/pointcloud.txt", last_cloud.data(), (size_t)last_disp.cols * last_disp.rows);
  }
  return 0;
}

static int sa_demo_main(int argc, char** argv, const char* name, const char* default_model, int default_frames,
                        sa_demo_run_fn run, sa_demo_run_fn run_rectify) {
  std::string model = default_model, calib = "StereoCalibration.yml", left = "left0.jpg", right = "right0.jpg",
              out = ".", list;
  int frames = default_frames, gpu = 0, depth = 2;
  bool rectify = true, save_all = false;
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
    else if (a == "--list") list = next();
    else if (a == "--save-all") save_all = true;
    else if (a == "--depth") depth = std::atoi(next().c_str());
    else {
      std::printf("usage: %s [--model preset|weights.safetensors|preset@weights] [--calib StereoCalibration.yml]\n"
                  "          [--left left0.jpg] [--right right0.jpg] [--frames N] [--gpu ID] [--out DIR]%s\n"
                  "          [--list pairs.txt [--save-all] [--depth 2]]\n",
                  name, run_rectify ? " [--no-rectify]" : "");
      return a == "--help" || a == "-h" ? 0 : 2;
    }
  }
  sa_demo_run_fn fn = (rectify || !run_rectify) ? (run_rectify ? run_rectify : run) : run;
  if (!list.empty()) {
    void* hs = Initialize(const_cast<char*>(model.c_str()), gpu, const_cast<char*>(calib.c_str()));
    if (!hs) return 1;
    std::printf("%s: %s\n", name, Version(hs));
    const int rc = sa_demo_stream(hs, fn, list, out, save_all, depth);
    Release(hs);
    return rc;
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
    const int rc = fn(h, imageL1, imageR1, pointcloud.data(), disparity);
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
