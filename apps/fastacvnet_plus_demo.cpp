// fastacvnet_plus_demo (reference FastACVNet_plus/test/main.cpp): 5 frames through
// RunFastACVNet_plus_RectifyImage.
#include "abi/FastACVNet_plus_Algorithm.h"
#include "demo_main.h"
int main(int argc, char** argv) {
  return sa_demo_main(argc, argv, "fastacvnet_plus_demo", "fastacvnet-plus", 5, RunFastACVNet_plus,
                      RunFastACVNet_plus_RectifyImage);
}
