// libFastACVNet_plus.so — reference C ABI of FastACVNet_plus/include/FastACVNet_plus_Algorithm.h:
// RunFastACVNet_plus (no rectification) / RunFastACVNet_plus_RectifyImage
// (FastACVNet_plus_Algorithm.cpp:59-91).
#include "abi/FastACVNet_plus_Algorithm.h"

#include "abi_common.h"

extern "C" {
SA_ABI_EXPORT void* Initialize(char* model_path, int gpu_id, char* calibration_path) {
  return sa_abi::initialize(model_path, gpu_id, calibration_path, "fastacvnet-plus");
}
SA_ABI_EXPORT int RunFastACVNet_plus(void* p, sa::Mat& left, sa::Mat& right, float* pointcloud,
                                     sa::Mat& disparity) {
  return sa_abi::run(p, left, right, pointcloud, disparity, false);
}
SA_ABI_EXPORT int RunFastACVNet_plus_RectifyImage(void* p, sa::Mat& left, sa::Mat& right, float* pointcloud,
                                                  sa::Mat& disparity) {
  return sa_abi::run(p, left, right, pointcloud, disparity, true);
}
SA_ABI_EXPORT const char* Version(void*) { return "FastACVNet_plus_Algorithm_V1.0"; }
SA_ABI_EXPORT int Release(void* p) { return sa_abi::release(p); }
}
