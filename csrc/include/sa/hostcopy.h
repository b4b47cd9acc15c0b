// Host-side copy pool for the engine's timed region (run_host): the point cloud / disparity D2H is split into
// chunks with one event each, and the copies from the pinned staging buffer into the caller's (pageable)
// arrays run on a few persistent threads as the chunks land, instead of one memcpy after the whole transfer.
// RAFT-Stereo realtime batch 1: the 7.4 MB cloud cost ~0.45 ms on one thread after a full sync
// (tools/diag/latency_parts.py).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <thread>
#include <vector>

namespace sa {

class HostCopyPool {
 public:
  struct Task {
    void* dst;
    const void* src;
    size_t bytes;
    hipEvent_t ready;  // waited on (hipEventSynchronize) before the copy; nullptr = ready now
  };
  explicit HostCopyPool(int workers);
  ~HostCopyPool();
  HostCopyPool(const HostCopyPool&) = delete;
  HostCopyPool& operator=(const HostCopyPool&) = delete;
  // runs every task on the workers and the calling thread; returns when all are done
  void run(const std::vector<Task>& tasks);

 private:
  void worker();
  void drain(const std::vector<Task>* tasks, int n, uint32_t gen);
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::vector<Task>* tasks_ = nullptr;
  int n_ = 0;
  std::atomic<uint64_t> claim_{0};  // (generation << 32) | next task index
  int remaining_ = 0, active_ = 0;
  uint32_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace sa
