// Native multi-GPU data parallelism over RCCL (xGMI), for C++ users of the framework.
//
// The reference is single-GPU, batch 1 (RAFTStereo/include/TRTRAFTStereo.h:15);
// this is the C++ counterpart of stereoalgorithms_amd/parallel/dp.py: one process per GPU, each rank
// runs its contiguous shard of stereo pairs through its own hipGraph engine, and the disparity maps are
// all-gathered with ONE ncclAllGather per step on a dedicated comm stream, overlapped with the next
// step's frame graph (ping-pong send/recv slots; the compute stream waits only when it is about to
// overwrite a slot whose collective is still in flight).
//
// Bootstrap: torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT).  Rank 0 creates
// the ncclUniqueId and hands it to the other ranks over a TCP socket on MASTER_ADDR:MASTER_PORT.
// Failure detection: every host-side wait polls ncclCommGetAsyncError and a deadline
// (SA_DIST_TIMEOUT seconds, default 600); on error or timeout the communicator is aborted and an
// sa::Error is thrown, so a dead peer fails the job instead of hanging it.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>

namespace sa {
class StereoEngine;
namespace dist {

struct DistEnv {
  int rank = 0, world = 1, local_rank = 0;
  std::string master_addr = "127.0.0.1";
  int master_port = 29500;
  int timeout_s = 600;
};
DistEnv env_from_environment();

// Rank 0 sends `n` bytes of `buf` to every other rank, which receive them into `buf` (TCP star on
// addr:port).  Returns 0 on success, -1 on error / timeout.  GPU-free (unit-tested on CPU).
int exchange_blob(int rank, int world, const char* addr, int port, void* buf, size_t n, int timeout_ms);

// The deadline loop behind the non-blocking communicator's init and enqueues, over an arbitrary status source
// (ncclResult_t values): 0 once it reports ncclSuccess, 1 on any other non-InProgress status, -1 at the deadline.
// GPU-free (unit-tested on CPU through sa_dist_settle_probe).
int settle_probe_impl(const std::function<int()>& status, int timeout_ms);

// Contiguous shard [start, end) of `total` items for `rank` (remainders to low ranks), as dp.py.
void shard_range(long total, int world, int rank, long* start, long* end);

class Communicator {
 public:
  Communicator(const DistEnv& env, int device);
  ~Communicator();
  Communicator(const Communicator&) = delete;
  Communicator& operator=(const Communicator&) = delete;
  int rank() const { return env_.rank; }
  int world() const { return env_.world; }
  // recv = concat over ranks of `bytes` from each rank's send (rank-major), enqueued on `s`.
  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s);
  // max over ranks of a host double (blocking, bounded by the timeout)
  double allreduce_max(double v, hipStream_t s);
  // host bytes of rank `root` -> every rank's `data` (length first, then the bytes; two ncclBroadcasts on `s`,
  // blocking).  Used to hand rank 0's tuned tactic plan to every rank before they build their engines.
  void broadcast_bytes(std::string& data, int root, hipStream_t s);
  void barrier(hipStream_t s);
  // Host wait for `s` with async-error polling and the deadline; throws (after abort) on failure.
  void wait_stream(hipStream_t s);

 private:
  void check_async();
  void enqueue_ok(int r, const char* what);  // ncclResult_t of an enqueue; ncclInProgress settles under the deadline
  DistEnv env_;
  void* comm_ = nullptr;  // ncclComm_t
  double* scratch_ = nullptr;
  bool aborted_ = false;
};

// One rank of a DP stereo job: engine (batch = per-rank shard) + comm stream + ping-pong slots.
class DataParallelRunner {
 public:
  DataParallelRunner(StereoEngine* engine, Communicator* comm);
  ~DataParallelRunner();
  // left/right: this rank's u8 BGR [B][H][W][3] device buffers.  Enqueues the frame graph on the
  // engine's stream and the all-gather on the comm stream; returns the device pointer of the
  // gathered fp32 [world*B][H][W] disparity, valid after wait() or until the slot is reused two
  // steps later.
  // cloud (optional): this rank's fp32 XYZRGB [B][H][W][6] device buffer, reprojected in the frame graph (needs Q).
  const float* step(const uint8_t* left, const uint8_t* right, float* cloud = nullptr);
  // block until every outstanding collective and frame has finished (with failure detection)
  void wait();
  hipStream_t comm_stream() const { return comm_stream_; }

 private:
  StereoEngine* eng_;
  Communicator* comm_;
  hipStream_t comm_stream_ = nullptr;
  static constexpr int kSlots = 2;
  float* send_[kSlots] = {};
  float* recv_[kSlots] = {};
  hipEvent_t ev_done_[kSlots] = {};   // frame finished writing send_[slot]
  hipEvent_t ev_gather_[kSlots] = {}; // collective finished with slot
  bool pending_[kSlots] = {};
  long i_ = 0;
  size_t bytes_ = 0;
  bool force_gather_ = false;
};

}  // namespace dist
}  // namespace sa
