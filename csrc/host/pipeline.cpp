// FramePipeline (sa/pipeline.h): loader thread -> caller thread (engine) -> writer thread, recycled frames.
#include "sa/pipeline.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <exception>
#include <memory>
#include <thread>

namespace sa {

PipelineStats FramePipeline::run(const Source& source, const Infer& infer, const Sink& sink, long max_frames) {
  using clock = std::chrono::steady_clock;
  using FramePtr = std::unique_ptr<StereoFrame>;
  const size_t nbuf = (size_t)depth_ + 2;
  BoundedQueue<FramePtr> free_q(nbuf), ready_q(depth_), done_q(depth_);
  for (size_t i = 0; i < nbuf; ++i) free_q.push(std::make_unique<StereoFrame>());

  PipelineStats st;
  std::mutex err_mu;
  std::atomic<bool> stop{false};
  auto fail = [&](int status, const std::string& what) {
    {
      std::lock_guard<std::mutex> lk(err_mu);
      if (st.status == 0) {
        st.status = status;
        st.error = what;
      }
    }
    stop = true;
    // unblock every stage: queued frames are dropped, blocked pushes / pops return false
    free_q.close();
    ready_q.close();
    done_q.close();
  };

  const auto t0 = clock::now();
  std::thread loader([&] {
    try {
      for (long i = 0; (max_frames < 0 || i < max_frames) && !stop; ++i) {
        FramePtr f;
        if (!free_q.pop(f)) break;
        f->index = i;
        f->status = 0;
        f->infer_ms = 0.0;
        if (!source(*f)) break;
        if (!ready_q.push(std::move(f))) break;
      }
    } catch (const std::exception& e) {
      fail(-1, std::string("source: ") + e.what());
    } catch (...) {
      fail(-1, "source: unknown exception");
    }
    ready_q.close();  // end of stream for the inference stage
  });
  std::thread writer([&] {
    try {
      FramePtr f;
      while (done_q.pop(f)) {
        sink(*f);
        if (!free_q.push(std::move(f))) break;
      }
    } catch (const std::exception& e) {
      fail(-1, std::string("sink: ") + e.what());
    } catch (...) {
      fail(-1, "sink: unknown exception");
    }
  });

  std::vector<double> ms;
  try {
    FramePtr f;
    while (!stop && ready_q.pop(f)) {
      const auto a = clock::now();
      f->status = infer(*f);
      f->infer_ms = std::chrono::duration<double, std::milli>(clock::now() - a).count();
      if (f->status != 0) {
        fail(f->status, "infer failed at frame " + std::to_string(f->index));
        break;
      }
      ms.push_back(f->infer_ms);
      if (!done_q.push(std::move(f))) break;
    }
  } catch (const std::exception& e) {
    fail(-1, std::string("infer: ") + e.what());
  } catch (...) {
    fail(-1, "infer: unknown exception");
  }
  done_q.close();  // the writer drains what is queued, then ends
  writer.join();
  free_q.close();  // a loader blocked on a free buffer (after a failure) wakes up
  loader.join();

  st.wall_ms = std::chrono::duration<double, std::milli>(clock::now() - t0).count();
  st.frames = (long)ms.size();
  if (!ms.empty()) {
    double sum = 0.0;
    for (double v : ms) sum += v;
    st.infer_mean_ms = sum / (double)ms.size();
    std::vector<double> s = ms;
    std::sort(s.begin(), s.end());
    st.infer_p50_ms = s[s.size() / 2];
    st.infer_p99_ms = s[std::min(s.size() - 1, (size_t)((double)s.size() * 0.99))];
    st.fps = st.wall_ms > 0.0 ? 1000.0 * (double)st.frames / st.wall_ms : 0.0;
  }
  return st;
}

}  // namespace sa
