// Reference-compatible C ABI header (same file name and symbols as the reference's
// include/RAFTStereoAlgorithm.h); cv::Mat is replaced by sa::Mat (sa/mat.h: same rows/cols/data/type() and
// CV_8UC3 / CV_32FC1 type codes); with OpenCV on the include path, abi/cv_adapter.h adds the reference's
// cv::Mat& overloads.  Link with libRAFTStereo.so (see stereoalgorithms_amd/_build.py).
#pragma once
#include "sa/mat.h"
#define SA_ABI_RAFTSTEREO 1

extern "C" void* Initialize(char* model_path, int gpu_id, char* calibration_path);
extern "C" int RunRAFTStereo(void* p, sa::Mat& left_image, sa::Mat& right_image, float* pointcloud, sa::Mat& disparity);
extern "C" const char* Version(void* p);
extern "C" int Release(void* p);

#include "abi/cv_adapter.h"
