// Back-to-back HostCopyPool::run() calls with tiny tasks (the pattern of run_host: inputs, then outputs, every
// frame), built with ThreadSanitizer by tools/sanitize/hostcopy_tsan.sh.  Every run must copy every task; a lost
// task shows up as a hang (the caller's bounded wait below) or a wrong byte.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "sa/hostcopy.h"

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  const int workers = argc > 2 ? std::atoi(argv[2]) : 3;
  sa::HostCopyPool pool(workers);
  std::vector<unsigned char> src(64), dst(64);
  std::atomic<int> done{0};
  std::thread watchdog([&] {
    for (int s = 0; s < 600 && done.load() == 0; ++s) std::this_thread::sleep_for(std::chrono::milliseconds(100));
    if (done.load() == 0) {
      std::fprintf(stderr, "hostcopy_stress: run() hung\n");
      std::_Exit(3);
    }
  });
  for (int it = 0; it < iters; ++it) {
    const int n = 1 + it % 5;  // 1..5 tasks of 8 bytes
    for (int i = 0; i < 64; ++i) src[i] = (unsigned char)(it * 7 + i);
    std::vector<sa::HostCopyPool::Task> tasks;
    for (int i = 0; i < n; ++i) tasks.push_back({dst.data() + 8 * i, src.data() + 8 * i, 8, nullptr});
    pool.run(tasks);
    for (int i = 0; i < 8 * n; ++i) {
      if (dst[i] != src[i]) {
        std::fprintf(stderr, "hostcopy_stress: iteration %d byte %d not copied\n", it, i);
        return 2;
      }
    }
  }
  done = 1;
  watchdog.join();
  std::printf("hostcopy_stress: %d runs x %d workers ok\n", iters, workers);
  return 0;
}
