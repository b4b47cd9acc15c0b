// StereoAlgorithm: the per-model facade of the reference (RAFTStereo/src/RAFTStereoAlgorithm.cpp,
// HitNet/src/HitNetAlgorithm.cpp, CREStereo/src/CREStereoAlgorithm.cpp,
// FastACVNet_plus/src/FastACVNet_plus_Algorithm.cpp) as one class:
//
//   Initialize(model, gpu, calibration.yml) -> read the YAML (ReadObjectYml), build the engine,
//       compute the rectification maps ONCE (the reference recomputes them every frame,
//       RAFTStereoAlgorithm.cpp:120-121) and upload them with Q to the device;
//   Run(left, right, pointcloud, disparity, rectify) -> the reference timed region
//       (TRTRAFTStereo.cpp:119-146) with rectification moved onto the GPU: left/right are
//       overwritten with their rectified versions when rectify is set (reference semantics),
//       disparity receives a fresh CV_32FC1 H x W matrix, pointcloud H*W*6 floats (x y z r g b).
//
// `model` is a weights file (.safetensors written by stereoalgorithms_amd.utils.weights, preset in
// its metadata) or "<preset>" / "<preset>@<weights>" (preset alone = seeded random init).  ONNX /
// TensorRT engine files are not accepted: the network is this framework's own op graph.
#pragma once
#include <memory>
#include <string>

#include "sa/calib.h"
#include "sa/mat.h"

namespace sa {

class StereoEngine;

class StereoAlgorithm {
 public:
  StereoAlgorithm();
  ~StereoAlgorithm();
  // 0 on success, -1 on error (message via last_error())
  int Initialize(const std::string& model, int gpu_id, const std::string& calibration_path,
                 const std::string& default_preset = "");
  int Run(Mat& left, Mat& right, float* pointcloud, Mat& disparity, bool rectify);
  int Release();
  bool initialized() const { return engine_ != nullptr; }
  const std::string& last_error() const { return err_; }
  const CalibrationParam& calibration() const { return calib_; }
  float last_ms() const { return last_ms_; }
  // frame size of the engine (0 before Initialize)
  int height() const;
  int width() const;
  std::string model() const { return model_; }

 private:
  std::unique_ptr<StereoEngine> engine_;
  CalibrationParam calib_;
  std::string err_, model_;
  bool have_maps_ = false;
  float last_ms_ = 0.f;
};

// Resolve "<preset>", "<preset>@<weights>", "<weights>.safetensors" into (preset, weights).
bool resolve_model_spec(const std::string& spec, const std::string& default_preset, std::string& preset,
                        std::string& weights, std::string& err);

}  // namespace sa
