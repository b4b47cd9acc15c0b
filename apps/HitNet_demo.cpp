// HitNet_demo (reference HitNet/test/main.cpp): 1000 frames through RunHitNet (rectifying).
#include "abi/HitNetAlgorithm.h"
#include "demo_main.h"
int main(int argc, char** argv) {
  return sa_demo_main(argc, argv, "HitNet_demo", "hitnet-d400", 1000, RunHitNet, nullptr);
}
