#include "sa/hostcopy.h"

#include <cstring>

#include "sa/common.h"

namespace sa {

HostCopyPool::HostCopyPool(int workers) {
  for (int i = 0; i < workers; ++i) th_.emplace_back([this] { worker(); });
}

HostCopyPool::~HostCopyPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : th_) t.join();
}

// Claims are (generation << 32 | index) in one 64-bit word: a claim succeeds only while the word still carries
// the caller's generation, so a worker that woke late for run() N can never take an index of run() N + 1 (the
// round-2 version shared a bare index counter, and a stale fetch_add after run() N + 1's reset lost task 0 of that
// run, leaving remaining_ above zero forever).
void HostCopyPool::drain(const std::vector<Task>* tasks, int n, uint32_t gen) {
  for (;;) {
    uint64_t cur = claim_.load(std::memory_order_relaxed);
    int i;
    do {
      if ((uint32_t)(cur >> 32) != gen) return;
      i = (int)(uint32_t)cur;
      if (i >= n) return;
    } while (!claim_.compare_exchange_weak(cur, cur + 1, std::memory_order_acq_rel, std::memory_order_relaxed));
    const Task& t = (*tasks)[i];
    if (t.ready) HIP_CHECK(hipEventSynchronize(t.ready));
    std::memcpy(t.dst, t.src, t.bytes);
    std::lock_guard<std::mutex> lk(mu_);
    if (--remaining_ == 0) done_cv_.notify_all();
  }
}

void HostCopyPool::worker() {
  uint32_t seen = 0;
  for (;;) {
    const std::vector<Task>* tasks;
    int n;
    uint32_t gen;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen = gen_;
      tasks = tasks_;
      n = n_;
      if (!tasks || n == 0) continue;  // that run() already returned: nothing to take part in
      ++active_;  // run() returns only once every worker that joined this generation is done with it
    }
    drain(tasks, n, gen);
    std::lock_guard<std::mutex> lk(mu_);
    if (--active_ == 0) done_cv_.notify_all();
  }
}

void HostCopyPool::run(const std::vector<Task>& tasks) {
  if (tasks.empty()) return;
  uint32_t gen;
  {
    std::lock_guard<std::mutex> lk(mu_);
    tasks_ = &tasks;
    n_ = (int)tasks.size();
    remaining_ = n_;
    gen = ++gen_;
    claim_.store((uint64_t)gen << 32, std::memory_order_release);
  }
  cv_.notify_all();
  drain(&tasks, (int)tasks.size(), gen);
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return remaining_ == 0 && active_ == 0; });
  tasks_ = nullptr;
  n_ = 0;
}

}  // namespace sa
