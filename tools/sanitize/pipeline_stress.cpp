// Stress test of sa::FramePipeline (csrc/host/pipeline.cpp) for ThreadSanitizer: many short pipelines with random
// stage delays; checks frame order and content through recycled buffers, and that a failing Infer, a throwing Source
// or Sink and a frame cap all end the run with every thread joined.
//   pipeline_stress [rounds]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <stdexcept>
#include <thread>

#include "sa/pipeline.h"

namespace {
thread_local std::mt19937 rng(12345);
void jitter() {
  const int us = (int)(rng() % 40);
  if (us > 30) std::this_thread::sleep_for(std::chrono::microseconds(us));
}
int fails = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "check failed line %d: %s\n", __LINE__, #c);  \
      ++fails;                                                           \
    }                                                                    \
  } while (0)
}  // namespace

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 300;
  for (int r = 0; r < rounds; ++r) {
    const int depth = 1 + r % 3;
    const long n = 5 + r % 17;
    const int mode = r % 5;  // 0 normal, 1 infer fails, 2 source throws, 3 sink throws, 4 frame cap
    const long bad = n / 2;
    long expect = 0;
    sa::FramePipeline pipe(depth);
    auto source = [&](sa::StereoFrame& f) {
      jitter();
      if (f.index >= n) return false;
      if (mode == 2 && f.index == bad) throw std::runtime_error("source broke");
      f.left.create(2, 3, sa::SA_8UC3);
      f.right.create(2, 3, sa::SA_8UC3);
      f.left.setTo((double)(f.index % 200));
      return true;
    };
    auto infer = [&](sa::StereoFrame& f) {
      jitter();
      if (mode == 1 && f.index == bad) return 7;
      f.disparity.create(2, 3, sa::SA_32FC1);
      f.disparity.setTo((double)f.left.at<unsigned char>(1, 2) + 0.5);
      return 0;
    };
    auto sink = [&](sa::StereoFrame& f) {
      jitter();
      CHECK(f.index == expect);
      CHECK(f.disparity.at<float>(1, 1) == (float)(f.index % 200) + 0.5f);
      ++expect;
      if (mode == 3 && f.index == bad) throw std::runtime_error("sink broke");
    };
    const sa::PipelineStats st = pipe.run(source, infer, sink, mode == 4 ? bad : -1);
    switch (mode) {
      case 0: CHECK(st.status == 0 && st.frames == n && expect == n); break;
      case 1: CHECK(st.status == 7 && st.frames == bad && expect <= bad); break;
      case 2: CHECK(st.status == -1 && st.frames <= bad && expect <= bad && st.error.find("source") == 0); break;
      case 3: CHECK(st.status == -1 && expect == bad + 1 && st.error.find("sink") == 0); break;
      case 4: CHECK(st.status == 0 && st.frames == bad && expect == bad); break;
    }
    if (fails) {
      std::fprintf(stderr, "round %d (mode %d depth %d n %ld): status %d frames %ld sunk %ld error '%s'\n", r, mode,
                   depth, n, st.status, st.frames, expect, st.error.c_str());
      return 1;
    }
  }
  std::printf("pipeline_stress: %d rounds ok\n", rounds);
  return 0;
}
