#include "sa/hostcopy.h"

#include <cstring>

#include "sa/runtime.h"

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

void HostCopyPool::drain(const std::vector<Task>* tasks, int n) {
  int i;
  while ((i = next_.fetch_add(1)) < n) {
    const Task& t = (*tasks)[i];
    if (t.ready) HIP_CHECK(hipEventSynchronize(t.ready));
    std::memcpy(t.dst, t.src, t.bytes);
    std::lock_guard<std::mutex> lk(mu_);
    if (--remaining_ == 0) done_cv_.notify_all();
  }
}

void HostCopyPool::worker() {
  unsigned long seen = 0;
  for (;;) {
    const std::vector<Task>* tasks;
    int n;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      tasks = tasks_;
      n = n_;
      ++active_;  // run() returns only once every worker that woke for this generation is done with it
    }
    drain(tasks, n);
    std::lock_guard<std::mutex> lk(mu_);
    if (--active_ == 0) done_cv_.notify_all();
  }
}

void HostCopyPool::run(const std::vector<Task>& tasks) {
  if (tasks.empty()) return;
  {
    std::lock_guard<std::mutex> lk(mu_);
    tasks_ = &tasks;
    n_ = (int)tasks.size();
    next_.store(0);
    remaining_ = n_;
    ++gen_;
  }
  cv_.notify_all();
  drain(&tasks, (int)tasks.size());
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return remaining_ == 0 && active_ == 0; });
  tasks_ = nullptr;
  n_ = 0;
}

}  // namespace sa
