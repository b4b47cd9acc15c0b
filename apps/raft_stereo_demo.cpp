// raft_stereo_demo (reference RAFTStereo/test/main.cpp): 1000 frames through RunRAFTStereo (rectifying).
#include "abi/RAFTStereoAlgorithm.h"
#include "demo_main.h"
int main(int argc, char** argv) {
  return sa_demo_main(argc, argv, "raft_stereo_demo", "raftstereo-realtime", 1000, RunRAFTStereo, nullptr);
}
