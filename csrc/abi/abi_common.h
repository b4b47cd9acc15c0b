// Shared body of the reference-compatible per-model C ABI (RAFTStereo/src/RAFTStereoAlgorithm.cpp:133-163
// and its three siblings).  Each model library (libRAFTStereo.so, libHitNet.so, libCREStereo.so,
// libFastACVNet_plus.so) exports the reference's exact symbol names: Initialize / Run<Model>
// [_RectifyImage] / Version / Release.  Documented deviations: Initialize
// returns NULL when initialisation fails, and Release deletes the handle.
#pragma once
#include <cstdio>

#include "sa/algorithm.h"

#define SA_ABI_EXPORT __attribute__((visibility("default")))

namespace sa_abi {

inline void* initialize(const char* model_path, int gpu_id, const char* calib, const char* default_preset) {
  auto* a = new sa::StereoAlgorithm();
  if (a->Initialize(model_path ? model_path : "", gpu_id, calib ? calib : "", default_preset) != 0) {
    std::fprintf(stderr, "Initialize failed: %s\n", a->last_error().c_str());
    delete a;
    return nullptr;
  }
  return a;
}

inline int run(void* p, sa::Mat& l, sa::Mat& r, float* pc, sa::Mat& d, bool rectify) {
  if (!p) return -1;
  return static_cast<sa::StereoAlgorithm*>(p)->Run(l, r, pc, d, rectify);
}

inline int release(void* p) {
  delete static_cast<sa::StereoAlgorithm*>(p);
  return 0;
}

}  // namespace sa_abi
