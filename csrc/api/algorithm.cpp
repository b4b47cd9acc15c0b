// StereoAlgorithm facade (see sa/algorithm.h).
#include "sa/algorithm.h"

#include <chrono>
#include <cstring>
#include <fstream>
#include <vector>

#include "sa/engine.h"

namespace sa {

static bool file_exists(const std::string& p) {
  std::ifstream f(p);
  return f.good();
}

static bool ends_with(const std::string& s, const std::string& suf) {
  return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

bool resolve_model_spec(const std::string& spec, const std::string& default_preset, std::string& preset,
                        std::string& weights, std::string& err) {
  preset.clear();
  weights.clear();
  const size_t at = spec.find('@');
  if (at != std::string::npos) {
    preset = spec.substr(0, at);
    weights = spec.substr(at + 1);
  } else if (ends_with(spec, ".safetensors")) {
    weights = spec;
  } else if (ends_with(spec, ".onnx") || ends_with(spec, ".engine") || ends_with(spec, ".trt")) {
    err = "ONNX/TensorRT model files are not supported: pass a .safetensors weights file or a preset name "
          "(e.g. \"raftstereo-realtime\")";
    return false;
  } else if (ends_with(spec, ".pth") || ends_with(spec, ".ckpt") || ends_with(spec, ".pt") || ends_with(spec, ".tar")) {
    err = "PyTorch checkpoints are not loaded natively (unpickling executes code): convert once with "
          "\"python -m stereoalgorithms_amd.utils.import_ckpt " + spec + " <out>.safetensors\" and pass the "
          ".safetensors file";
    return false;
  } else if (!spec.empty()) {
    preset = spec;
  } else {
    preset = default_preset;
  }
  if (!weights.empty() && !file_exists(weights)) {
    err = "weights file not found: " + weights;
    return false;
  }
  if (preset.empty() && weights.empty()) {
    err = "no model given";
    return false;
  }
  return true;
}

StereoAlgorithm::StereoAlgorithm() = default;
StereoAlgorithm::~StereoAlgorithm() { Release(); }

int StereoAlgorithm::Initialize(const std::string& model, int gpu_id, const std::string& calib_path,
                                const std::string& default_preset) {
  try {
    // reference: calibration file must exist (RAFTStereoAlgorithm.cpp:37-40)
    if (!file_exists(calib_path)) {
      err_ = "calibration file not found: " + calib_path;
      SA_LOGE("%s", err_.c_str());
      return -1;
    }
    if (!read_calibration(calib_path, calib_)) {
      err_ = "cannot parse calibration file " + calib_path;
      return -1;
    }
    std::string preset, weights;
    if (!resolve_model_spec(model, default_preset, preset, weights, err_)) {
      SA_LOGE("%s", err_.c_str());
      return -1;
    }
    EngineConfig cfg;
    cfg.model = preset;
    cfg.weights = weights;
    cfg.device = gpu_id;
    cfg.height = 480;  // reference input size (TRTRAFTStereo.cpp:13-14)
    cfg.width = 640;
    cfg.batch = 1;
    engine_ = StereoEngine::create(cfg);
    model_ = engine_->config().model;
    // Q for reprojection (Q.convertTo(CV_64F) -> float, TRTRAFTStereo.cpp:103-109)
    if (!calib_.Q.empty()) {
      float q[16];
      for (int i = 0; i < 16; ++i) q[i] = (float)calib_.Q.get(i);
      engine_->set_Q(q);
    }
    // rectification maps computed once, applied on the GPU per frame
    have_maps_ = false;
    if (!calib_.intrinsic_left.empty() && !calib_.intrinsic_right.empty() && !calib_.P1.empty() &&
        !calib_.P2.empty()) {
      std::vector<float> ml, mr;
      init_undistort_rectify_map(calib_.intrinsic_left, calib_.distCoeffs_left, calib_.R_L, calib_.P1, cfg.width,
                                 cfg.height, ml, true);
      init_undistort_rectify_map(calib_.intrinsic_right, calib_.distCoeffs_right, calib_.R_R, calib_.P2, cfg.width,
                                 cfg.height, mr, true);
      engine_->set_rectify_maps(ml.data(), mr.data());
      have_maps_ = true;
    }
    SA_LOGI("init successed! model %s on GPU %d", model_.c_str(), gpu_id);
    return 0;
  } catch (const std::exception& e) {
    err_ = e.what();
    SA_LOGE("Initialize failed: %s", e.what());
    engine_.reset();
    return -1;
  }
}

int StereoAlgorithm::Run(Mat& left, Mat& right, float* pointcloud, Mat& disparity, bool rectify) {
  if (!engine_) {
    err_ = "not initialized";
    SA_LOGE("%s", err_.c_str());
    return -1;
  }
  if (left.empty() || right.empty()) {
    err_ = "empty input image";
    SA_LOGE("%s", err_.c_str());
    return -1;
  }
  const int H = engine_->H(), W = engine_->W();
  if (left.rows != H || left.cols != W || right.rows != H || right.cols != W || left.type() != SA_8UC3 ||
      right.type() != SA_8UC3) {
    err_ = "inputs must be CV_8UC3 " + std::to_string(W) + "x" + std::to_string(H);
    SA_LOGE("%s", err_.c_str());
    return -1;
  }
  if (rectify && !have_maps_) {
    err_ = "rectification requested but the calibration lacks K/D/R_L/R_R/P1/P2";
    return -1;
  }
  try {
    // contiguous BGR views (copy only if the caller passed strided ROIs)
    Mat l = left.isContinuous() ? left : left.clone();
    Mat r = right.isContinuous() ? right : right.clone();
    disparity.create(H, W, SA_32FC1);
    const auto t0 = std::chrono::steady_clock::now();
    engine_->run_host(l.data, r.data, disparity.ptr<float>(), pointcloud, rectify);
    last_ms_ = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rectify) {  // rectified images back into the caller's matrices
      if (l.data != left.data) l.copyTo(left);
      if (r.data != right.data) r.copyTo(right);
    }
    SA_LOGI("inference time:%.3fms", last_ms_);
    return 0;
  } catch (const std::exception& e) {
    err_ = e.what();
    SA_LOGE("Run failed: %s", e.what());
    return -1;
  }
}

int StereoAlgorithm::height() const { return engine_ ? engine_->H() : 0; }
int StereoAlgorithm::width() const { return engine_ ? engine_->W() : 0; }

int StereoAlgorithm::Release() {
  engine_.reset();
  have_maps_ = false;
  return 0;
}

}  // namespace sa
