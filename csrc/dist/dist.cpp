// Native RCCL data parallelism (see sa/dist.h).  Python counterpart: stereoalgorithms_amd/parallel/dp.py.
#include "sa/dist.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <functional>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "sa/common.h"
#include "sa/engine.h"

namespace sa {
namespace dist {

namespace {
int env_int(const char* k, int def) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : def;
}
using Clock = std::chrono::steady_clock;

bool send_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

bool recv_all(int fd, char* p, size_t n, Clock::time_point deadline) {
  while (n) {
    int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count();
    if (left <= 0) return false;
    pollfd pf{fd, POLLIN, 0};
    if (::poll(&pf, 1, left) <= 0) return false;
    ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

#define NCCL_CHECK(expr)                                                                        \
  do {                                                                                          \
    ncclResult_t _r = (expr);                                                                   \
    if (_r != ncclSuccess) {                                                                    \
      ::sa::log_msg(::sa::LogLevel::kError, __FILE__, __LINE__, "RCCL error %s: %s", #expr,     \
                    ncclGetErrorString(_r));                                                    \
      throw ::sa::Error(std::string("RCCL: ") + ncclGetErrorString(_r));                        \
    }                                                                                           \
  } while (0)
// Poll `status` (ncclCommGetAsyncError of a non-blocking communicator) until it leaves ncclInProgress: 0 on
// ncclSuccess, 1 on an error (*last holds it), -1 once `deadline` passes
template <typename F>
int settle(F status, Clock::time_point deadline, ncclResult_t* last) {
  for (;;) {
    const ncclResult_t st = status();
    if (last) *last = st;
    if (st == ncclSuccess) return 0;
    if (st != ncclInProgress) return 1;
    if (Clock::now() > deadline) return -1;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}
}  // namespace

DistEnv env_from_environment() {
  DistEnv e;
  e.rank = env_int("RANK", 0);
  e.world = env_int("WORLD_SIZE", 1);
  e.local_rank = env_int("LOCAL_RANK", e.rank);
  if (const char* a = std::getenv("MASTER_ADDR")) e.master_addr = a;
  // +1: a torchrun launcher already owns MASTER_PORT for its own store
  e.master_port = env_int("SA_DIST_PORT", env_int("MASTER_PORT", 29500) + 1);
  e.timeout_s = env_int("SA_DIST_TIMEOUT", 600);
  return e;
}

void shard_range(long total, int world, int rank, long* start, long* end) {
  long base = total / world, rem = total % world;
  *start = rank * base + (rank < rem ? rank : rem);
  *end = *start + base + (rank < rem ? 1 : 0);
}

int exchange_blob(int rank, int world, const char* addr, int port, void* buf, size_t n, int timeout_ms) {
  if (world <= 1) return 0;
  const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
  // MASTER_ADDR may be a hostname (torchrun sets socket.getfqdn()) or a dotted literal: resolve it.
  // Rank 0 listens on every interface, so whichever address the name resolves to on a peer reaches it.
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  if (::inet_pton(AF_INET, addr, &sa.sin_addr) != 1) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (::getaddrinfo(addr, nullptr, &hints, &res) != 0 || !res) return -1;
    sa.sin_addr = ((sockaddr_in*)res->ai_addr)->sin_addr;
    ::freeaddrinfo(res);
  }
  if (rank == 0) {
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    int ls = ::socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) return -1;
    int one = 1;
    ::setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (::bind(ls, (sockaddr*)&sa, sizeof(sa)) != 0 || ::listen(ls, world) != 0) {
      ::close(ls);
      return -1;
    }
    int served = 0, rc = 0;
    while (served < world - 1) {
      int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count();
      pollfd pf{ls, POLLIN, 0};
      if (left <= 0 || ::poll(&pf, 1, left) <= 0) {
        rc = -1;
        break;
      }
      int c = ::accept(ls, nullptr, nullptr);
      if (c < 0) continue;
      uint64_t len = n;
      bool ok = send_all(c, (const char*)&len, sizeof(len)) && send_all(c, (const char*)buf, n);
      ::close(c);
      if (!ok) {
        rc = -1;
        break;
      }
      ++served;
    }
    ::close(ls);
    return rc;
  }
  while (Clock::now() < deadline) {  // peers retry until rank 0 listens
    int s = ::socket(AF_INET, SOCK_STREAM, 0);
    if (s < 0) return -1;
    if (::connect(s, (sockaddr*)&sa, sizeof(sa)) == 0) {
      uint64_t len = 0;
      bool ok = recv_all(s, (char*)&len, sizeof(len), deadline) && len == n &&
                recv_all(s, (char*)buf, n, deadline);
      ::close(s);
      return ok ? 0 : -1;
    }
    ::close(s);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  return -1;
}

// ------------------------------------------------------------------ Communicator
Communicator::Communicator(const DistEnv& env, int device) : env_(env) {
  HIP_CHECK(hipSetDevice(device));
  ncclUniqueId id{};
  if (env_.rank == 0) NCCL_CHECK(ncclGetUniqueId(&id));
  SA_REQUIRE(exchange_blob(env_.rank, env_.world, env_.master_addr.c_str(), env_.master_port, &id, sizeof(id),
                           env_.timeout_s * 1000) == 0,
             "rank %d: ncclUniqueId bootstrap over %s:%d failed", env_.rank, env_.master_addr.c_str(),
             env_.master_port);
  // Non-blocking init (blocking = 0), polled against the same SA_DIST_TIMEOUT deadline as the bootstrap: a peer
  // that dies or never reaches init can no longer hang every other rank inside ncclCommInitRank
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t c = nullptr;
  const ncclResult_t r0 = ncclCommInitRankConfig(&c, env_.world, id, env_.rank, &cfg);
  if (r0 != ncclSuccess && r0 != ncclInProgress) {
    SA_LOGE("rank %d: ncclCommInitRankConfig: %s", env_.rank, ncclGetErrorString(r0));
    throw Error(std::string("RCCL init: ") + ncclGetErrorString(r0));
  }
  ncclResult_t st = ncclSuccess;
  const int rc = settle(
      [&] {
        ncclResult_t x = ncclSuccess;
        ncclCommGetAsyncError(c, &x);
        return x;
      },
      Clock::now() + std::chrono::seconds(env_.timeout_s), &st);
  if (rc != 0) {
    if (c) ncclCommAbort(c);
    SA_LOGE("rank %d: RCCL communicator init %s", env_.rank, rc < 0 ? "timed out" : ncclGetErrorString(st));
    throw Error(rc < 0 ? "RCCL communicator init timed out (SA_DIST_TIMEOUT): a peer never completed init"
                       : std::string("RCCL init: ") + ncclGetErrorString(st));
  }
  comm_ = c;
  HIP_CHECK(hipMalloc(&scratch_, sizeof(double)));
  SA_LOGI("rank %d/%d: RCCL communicator up on device %d", env_.rank, env_.world, device);
}

Communicator::~Communicator() {
  if (comm_ && !aborted_) {
    ncclComm_t c = (ncclComm_t)comm_;
    // non-blocking communicator: finalize may return ncclInProgress; bounded wait, then destroy (or abort)
    const ncclResult_t r = ncclCommFinalize(c);
    const int rc = (r == ncclSuccess || r == ncclInProgress)
                       ? settle(
                             [&] {
                               ncclResult_t x = ncclSuccess;
                               ncclCommGetAsyncError(c, &x);
                               return x;
                             },
                             Clock::now() + std::chrono::seconds(env_.timeout_s), nullptr)
                       : 1;
    if (rc == 0) ncclCommDestroy(c);
    else ncclCommAbort(c);
  }
  if (scratch_) (void)hipFree(scratch_);
}

void Communicator::check_async() {
  ncclResult_t st = ncclSuccess;
  ncclCommGetAsyncError((ncclComm_t)comm_, &st);
  if (st != ncclSuccess && st != ncclInProgress) {
    ncclCommAbort((ncclComm_t)comm_);
    aborted_ = true;
    throw Error(std::string("RCCL async error: ") + ncclGetErrorString(st));
  }
}

// a call on the non-blocking communicator may return ncclInProgress: the next call must wait until it settled
void Communicator::enqueue_ok(int r, const char* what) {
  if (r == ncclSuccess) return;
  if (r == ncclInProgress) {
    ncclResult_t st = ncclSuccess;
    const int rc = settle(
        [&] {
          ncclResult_t x = ncclSuccess;
          ncclCommGetAsyncError((ncclComm_t)comm_, &x);
          return x;
        },
        Clock::now() + std::chrono::seconds(env_.timeout_s), &st);
    if (rc == 0) return;
    ncclCommAbort((ncclComm_t)comm_);
    aborted_ = true;
    throw Error(std::string(what) + (rc < 0 ? ": timed out (SA_DIST_TIMEOUT)" : ": ") +
                (rc < 0 ? "" : ncclGetErrorString(st)));
  }
  throw Error(std::string(what) + ": " + ncclGetErrorString((ncclResult_t)r));
}

void Communicator::all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) {
  enqueue_ok(ncclAllGather(send, recv, bytes, ncclChar, (ncclComm_t)comm_, s), "ncclAllGather");
}

void Communicator::barrier(hipStream_t s) {
  enqueue_ok(ncclAllReduce(scratch_, scratch_, 1, ncclDouble, ncclSum, (ncclComm_t)comm_, s), "barrier");
  wait_stream(s);
}

double Communicator::allreduce_max(double v, hipStream_t s) {
  HIP_CHECK(hipMemcpyAsync(scratch_, &v, sizeof(v), hipMemcpyHostToDevice, s));
  enqueue_ok(ncclAllReduce(scratch_, scratch_, 1, ncclDouble, ncclMax, (ncclComm_t)comm_, s), "allreduce");
  HIP_CHECK(hipMemcpyAsync(&v, scratch_, sizeof(v), hipMemcpyDeviceToHost, s));
  wait_stream(s);
  return v;
}

void Communicator::broadcast_bytes(std::string& data, int root, hipStream_t s) {
  double len = env_.rank == root ? (double)data.size() : 0.0;
  HIP_CHECK(hipMemcpyAsync(scratch_, &len, sizeof(len), hipMemcpyHostToDevice, s));
  enqueue_ok(ncclBroadcast(scratch_, scratch_, 1, ncclDouble, root, (ncclComm_t)comm_, s), "ncclBroadcast(len)");
  HIP_CHECK(hipMemcpyAsync(&len, scratch_, sizeof(len), hipMemcpyDeviceToHost, s));
  wait_stream(s);
  const size_t n = (size_t)len;
  if (n == 0) {
    data.clear();
    return;
  }
  char* buf = nullptr;
  HIP_CHECK(hipMalloc((void**)&buf, n));
  if (env_.rank == root) HIP_CHECK(hipMemcpyAsync(buf, data.data(), n, hipMemcpyHostToDevice, s));
  enqueue_ok(ncclBroadcast(buf, buf, n, ncclChar, root, (ncclComm_t)comm_, s), "ncclBroadcast(bytes)");
  data.resize(n);
  HIP_CHECK(hipMemcpyAsync(&data[0], buf, n, hipMemcpyDeviceToHost, s));
  wait_stream(s);
  HIP_CHECK(hipFree(buf));
}

void Communicator::wait_stream(hipStream_t s) {
  const auto deadline = Clock::now() + std::chrono::seconds(env_.timeout_s);
  for (;;) {
    hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) HIP_CHECK(q);
    check_async();
    if (Clock::now() > deadline) {
      ncclCommAbort((ncclComm_t)comm_);
      aborted_ = true;
      throw Error("RCCL collective timed out (SA_DIST_TIMEOUT)");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

int settle_probe_impl(const std::function<int()>& status, int timeout_ms) {
  return settle([&] { return (ncclResult_t)status(); }, Clock::now() + std::chrono::milliseconds(timeout_ms), nullptr);
}

// ------------------------------------------------------------------ DataParallelRunner
DataParallelRunner::DataParallelRunner(StereoEngine* engine, Communicator* comm) : eng_(engine), comm_(comm) {
  const size_t frame = (size_t)eng_->H() * eng_->W() * sizeof(float);
  bytes_ = frame * eng_->B();
  const char* fg = std::getenv("SA_DP_GATHER_WORLD1");
  force_gather_ = fg && fg[0] == '1';
  HIP_CHECK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking));
  for (int s = 0; s < kSlots; ++s) {
    HIP_CHECK(hipMalloc(&send_[s], bytes_));
    HIP_CHECK(hipMalloc(&recv_[s], bytes_ * comm_->world()));
    HIP_CHECK(hipEventCreateWithFlags(&ev_done_[s], hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_gather_[s], hipEventDisableTiming));
  }
}

DataParallelRunner::~DataParallelRunner() {
  (void)hipStreamSynchronize(comm_stream_);
  for (int s = 0; s < kSlots; ++s) {
    (void)hipFree(send_[s]);
    (void)hipFree(recv_[s]);
    (void)hipEventDestroy(ev_done_[s]);
    (void)hipEventDestroy(ev_gather_[s]);
  }
  (void)hipStreamDestroy(comm_stream_);
}

const float* DataParallelRunner::step(const uint8_t* left, const uint8_t* right, float* cloud) {
  const int slot = (int)(i_++ % kSlots);
  hipStream_t cs = eng_->stream();
  if (pending_[slot]) HIP_CHECK(hipStreamWaitEvent(cs, ev_gather_[slot], 0));  // WAR on the slot
  eng_->run_device(left, right, send_[slot], cloud, false, cs);
  // nothing to gather at world 1 (SA_DP_GATHER_WORLD1=1 still runs the collective path, for tests)
  if (comm_->world() == 1 && !force_gather_) return send_[slot];
  HIP_CHECK(hipEventRecord(ev_done_[slot], cs));
  HIP_CHECK(hipStreamWaitEvent(comm_stream_, ev_done_[slot], 0));
  comm_->all_gather(send_[slot], recv_[slot], bytes_, comm_stream_);
  HIP_CHECK(hipEventRecord(ev_gather_[slot], comm_stream_));
  pending_[slot] = true;
  return recv_[slot];
}

void DataParallelRunner::wait() {
  HIP_CHECK(hipStreamSynchronize(eng_->stream()));
  comm_->wait_stream(comm_stream_);
  for (bool& p : pending_) p = false;
}

}  // namespace dist
}  // namespace sa

// ------------------------------------------------------------------ flat C entry (ctypes tests)
// the init / enqueue deadline loop on the CPU (tests): a status source that reports ncclInProgress `in_progress`
// times, then `final_status`; returns settle()'s 0 / 1 / -1
extern "C" int sa_dist_settle_probe(int in_progress, int final_status, int timeout_ms) {
  int n = 0;
  return sa::dist::settle_probe_impl(
      [&] { return n++ < in_progress ? (int)ncclInProgress : final_status; }, timeout_ms);
}
extern "C" int sa_dist_exchange_blob(int rank, int world, const char* addr, int port, void* buf, size_t n,
                                     int timeout_ms) {
  return sa::dist::exchange_blob(rank, world, addr, port, buf, n, timeout_ms);
}
