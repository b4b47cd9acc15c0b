// libHitNet.so — reference C ABI of HitNet/include/HitNetAlgorithm.h (RunHitNet rectifies,
// HitNetAlgorithm.cpp:47).
#include "abi/HitNetAlgorithm.h"

#include "abi_common.h"

extern "C" {
SA_ABI_EXPORT void* Initialize(char* model_path, int gpu_id, char* calibration_path) {
  return sa_abi::initialize(model_path, gpu_id, calibration_path, "hitnet-d400");
}
SA_ABI_EXPORT int RunHitNet(void* p, sa::Mat& left, sa::Mat& right, float* pointcloud, sa::Mat& disparity) {
  return sa_abi::run(p, left, right, pointcloud, disparity, true);
}
SA_ABI_EXPORT const char* Version(void*) { return "HitNetAlgorithm_V1.0"; }
SA_ABI_EXPORT int Release(void* p) { return sa_abi::release(p); }
}
