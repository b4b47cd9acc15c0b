// libCREStereo.so — reference C ABI of CREStereo/include/CREStereoAlgorithm.h:24-44: RunCREStereo does
// NOT rectify, RunCREStereo_RectifyImage does (CREStereoAlgorithm.cpp:59-91).
#include "abi/CREStereoAlgorithm.h"

#include "abi_common.h"

extern "C" {
SA_ABI_EXPORT void* Initialize(char* model_path, int gpu_id, char* calibration_path) {
  return sa_abi::initialize(model_path, gpu_id, calibration_path, "crestereo-iter5");
}
SA_ABI_EXPORT int RunCREStereo(void* p, sa::Mat& left, sa::Mat& right, float* pointcloud, sa::Mat& disparity) {
  return sa_abi::run(p, left, right, pointcloud, disparity, false);
}
SA_ABI_EXPORT int RunCREStereo_RectifyImage(void* p, sa::Mat& left, sa::Mat& right, float* pointcloud,
                                            sa::Mat& disparity) {
  return sa_abi::run(p, left, right, pointcloud, disparity, true);
}
SA_ABI_EXPORT const char* Version(void*) { return "CREStereoAlgorithm_V1.0"; }
SA_ABI_EXPORT int Release(void* p) { return sa_abi::release(p); }
}
