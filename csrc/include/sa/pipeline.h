// Host-side frame pipeline for streaming use of an engine (SURVEY.md §2.4 "intra-process threading": producer /
// consumer pipelining of frames).  The reference processes one frame at a time on one thread: imread, Run, write
// (RAFTStereo/test/main.cpp).  Here a loader thread decodes / captures frame i+1 and a writer thread consumes the
// results of frame i-1 while the calling thread keeps the GPU busy with frame i:
//
//   loader thread:  Source(frame)   -> ready queue
//   caller thread:  Infer(frame)    -> done queue      (the engine stays on the thread that created it)
//   writer thread:  Sink(frame)     -> free list       (results in frame order)
//
// Frames are recycled through a free list of depth + 2 buffers, so a steady stream allocates nothing once the
// Mats reach their size.  A non-zero Infer status, an exception in any stage or a Source returning false ends the
// run; every thread is joined before run() returns.  tools/sanitize/pipeline_stress.cpp runs it under TSan.
#pragma once
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "sa/mat.h"

namespace sa {

// Blocking bounded MPMC queue; close() wakes every waiter, pop() drains what is left before reporting the end.
template <class T>
class BoundedQueue {
 public:
  explicit BoundedQueue(size_t cap) : cap_(cap ? cap : 1) {}
  bool push(T v) {
    std::unique_lock<std::mutex> lk(mu_);
    not_full_.wait(lk, [&] { return q_.size() < cap_ || closed_; });
    if (closed_) return false;
    q_.push_back(std::move(v));
    not_empty_.notify_one();
    return true;
  }
  bool pop(T& out) {
    std::unique_lock<std::mutex> lk(mu_);
    not_empty_.wait(lk, [&] { return !q_.empty() || closed_; });
    if (q_.empty()) return false;
    out = std::move(q_.front());
    q_.pop_front();
    not_full_.notify_one();
    return true;
  }
  void close() {
    std::lock_guard<std::mutex> lk(mu_);
    closed_ = true;
    not_empty_.notify_all();
    not_full_.notify_all();
  }

 private:
  std::mutex mu_;
  std::condition_variable not_full_, not_empty_;
  std::deque<T> q_;
  size_t cap_;
  bool closed_ = false;
};

struct StereoFrame {
  long index = -1;
  std::string tag;  // free-form (e.g. the source file name)
  Mat left, right, disparity;
  std::vector<float> cloud;
  double infer_ms = 0.0;
  int status = 0;
};

struct PipelineStats {
  long frames = 0;       // frames that went through Infer successfully
  double wall_ms = 0.0;  // first Source call to the last Sink
  double infer_mean_ms = 0.0, infer_p50_ms = 0.0, infer_p99_ms = 0.0;
  double fps = 0.0;      // frames / wall time (the pipelined rate)
  int status = 0;        // 0, the failing Infer status, or -1 for an exception
  std::string error;     // exception text
};

class FramePipeline {
 public:
  using Source = std::function<bool(StereoFrame&)>;  // fill left / right (false = end of stream)
  using Infer = std::function<int(StereoFrame&)>;    // run the engine (non-zero status stops the run)
  using Sink = std::function<void(StereoFrame&)>;    // consume disparity / cloud

  explicit FramePipeline(int depth = 2) : depth_(depth < 1 ? 1 : depth) {}
  // max_frames < 0: until the Source ends
  PipelineStats run(const Source& source, const Infer& infer, const Sink& sink, long max_frames = -1);

 private:
  int depth_;
};

}  // namespace sa
