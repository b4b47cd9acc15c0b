// crestereo_demo (reference CREStereo/test/main.cpp): 1000 frames through RunCREStereo_RectifyImage.
#include "abi/CREStereoAlgorithm.h"
#include "demo_main.h"
int main(int argc, char** argv) {
  return sa_demo_main(argc, argv, "crestereo_demo", "crestereo-iter5", 1000, RunCREStereo, RunCREStereo_RectifyImage);
}
