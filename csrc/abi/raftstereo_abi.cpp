// libRAFTStereo.so — reference C ABI of RAFTStereo/include/RAFTStereoAlgorithm.h:24-39.
// RunRAFTStereo always rectifies (RAFTStereoAlgorithm.cpp:57-72).
#include "abi/RAFTStereoAlgorithm.h"

#include "abi_common.h"

extern "C" {
SA_ABI_EXPORT void* Initialize(char* model_path, int gpu_id, char* calibration_path) {
  return sa_abi::initialize(model_path, gpu_id, calibration_path, "raftstereo-realtime");
}
SA_ABI_EXPORT int RunRAFTStereo(void* p, sa::Mat& left, sa::Mat& right, float* pointcloud, sa::Mat& disparity) {
  return sa_abi::run(p, left, right, pointcloud, disparity, true);
}
SA_ABI_EXPORT const char* Version(void*) { return "RAFTStereoAlgorithm_V1.0"; }
SA_ABI_EXPORT int Release(void* p) { return sa_abi::release(p); }
}
