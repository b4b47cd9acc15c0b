// Cross-queue dependency latency inside a captured hipGraph (what a fork / join edge costs on the critical chain).
//
//   xq_latency [--reps N]
//
// Every kernel is one workgroup that spins for a fixed time on s_memrealtime (100 MHz) and stamps its start / end
// into a device buffer with vector stores.  Per case, one graph is captured, replayed a few times, and the
// dispatch-to-dispatch gaps of the last replay are printed (median over --reps replays):
//   serial   A -> B -> C on one stream                            (gap of a same-queue edge)
//   forkjoin A (s0) -> B (s1) -> C (s0)                           (fork edge A->B and join edge B->C)
//   ready    A (s0) -> {B short on s1, D long on s0} -> C (s0)   (join on a side branch that finished long ago)
//   fanout   A (s0) -> {B (s1), D (s0)} both short -> C (s0)     (join where both branches end together)
//   busy     A (s0) -> {B short on s1, 20 chip-filling kernels on s0} -> C (s0): does the side queue's B start
//            promptly while the other queue keeps the chip full?  (A->B is the number to read)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      std::exit(2);                                                                               \
    }                                                                                             \
  } while (0)

__global__ void spin_kernel(unsigned long long* stamps, int slot, unsigned ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    // plain vector stores of the two stamps
    volatile unsigned long long* p = stamps + 2 * slot;
    p[0] = t0;
    p[1] = t;
  }
}

static void launch(hipStream_t s, unsigned long long* st, int slot, unsigned us, int blocks = 1, int threads = 64) {
  hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(threads), 0, s, st, slot, us * 100u);
}

struct Case {
  const char* name;
  int nk;  // kernels stamped
};

int main(int argc, char** argv) {
  int reps = 20;
  for (int i = 1; i < argc; ++i)
    if (!std::strcmp(argv[i], "--reps") && i + 1 < argc) reps = std::atoi(argv[++i]);
  hipStream_t s0, s1;
  CHECK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t ef, ej;
  CHECK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
  CHECK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
  unsigned long long* st;
  CHECK(hipMalloc(&st, 64 * sizeof(unsigned long long)));
  const char* names[] = {"serial", "forkjoin", "ready", "fanout", "busy"};
  for (int c = 0; c < 5; ++c) {
    hipGraph_t g;
    CHECK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
    launch(s0, st, 0, 20);  // A
    if (c == 0) {
      launch(s0, st, 1, 20);  // B
      launch(s0, st, 2, 20);  // C
    } else {
      CHECK(hipEventRecord(ef, s0));
      CHECK(hipStreamWaitEvent(s1, ef, 0));
      launch(s1, st, 1, c == 2 || c == 4 ? 5 : 20);  // B on the side stream
      if (c == 4)
        for (int k = 0; k < 20; ++k) launch(s0, st, 3, 20, 2048, 256);  // chip-filling kernels, D = the last one
      else if (c >= 2)
        launch(s0, st, 3, c == 2 ? 60 : 20);  // D on the main stream
      CHECK(hipEventRecord(ej, s1));
      CHECK(hipStreamWaitEvent(s0, ej, 0));
      launch(s0, st, 2, 20);  // C
    }
    CHECK(hipStreamEndCapture(s0, &g));
    hipGraphExec_t ge;
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    std::vector<double> ab, bc, dc, span;
    for (int r = 0; r < reps + 3; ++r) {
      CHECK(hipMemset(st, 0, 64 * sizeof(unsigned long long)));
      CHECK(hipGraphLaunch(ge, s0));
      CHECK(hipStreamSynchronize(s0));
      unsigned long long h[8];
      CHECK(hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
      if (r < 3) continue;
      auto us = [](unsigned long long a, unsigned long long b) { return ((double)b - (double)a) / 100.0; };
      ab.push_back(us(h[1], h[2]));  // A end -> B start
      bc.push_back(us(h[3], h[4]));  // B end -> C start
      if (c >= 2) dc.push_back(us(h[7], h[4]));  // D end -> C start
      span.push_back(us(h[0], h[5]));
    }
    auto med = [](std::vector<double> v) {
      if (v.empty()) return 0.0;
      std::sort(v.begin(), v.end());
      return v[v.size() / 2];
    };
    std::printf("%-9s A->B %6.2f us  B->C %6.2f us  D->C %6.2f us  span %7.2f us\n", names[c], med(ab), med(bc),
                med(dc), med(span));
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
  }
  // independent roots: s1's single kernel B forked before anything ran on s0, s0 then runs 20 x 40 us kernels
  // (case "roots_fill": chip-filling ones).  B's start relative to the first s0 kernel's start is the number.
  for (int fill = 0; fill < 2; ++fill) {
    hipGraph_t g;
    CHECK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
    CHECK(hipEventRecord(ef, s0));
    CHECK(hipStreamWaitEvent(s1, ef, 0));
    for (int k = 0; k < 20; ++k) launch(s0, st, k == 0 ? 0 : 3, 40, fill ? 2048 : 1, fill ? 256 : 64);
    launch(s1, st, 1, 5);
    CHECK(hipEventRecord(ej, s1));
    CHECK(hipStreamWaitEvent(s0, ej, 0));
    launch(s0, st, 2, 5);
    CHECK(hipStreamEndCapture(s0, &g));
    hipGraphExec_t ge;
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    std::vector<double> b0;
    for (int r = 0; r < reps + 3; ++r) {
      CHECK(hipMemset(st, 0, 64 * sizeof(unsigned long long)));
      CHECK(hipGraphLaunch(ge, s0));
      CHECK(hipStreamSynchronize(s0));
      unsigned long long h[8];
      CHECK(hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
      if (r < 3) continue;
      b0.push_back(((double)h[2] - (double)h[0]) / 100.0);  // B start - first s0 kernel start
    }
    std::sort(b0.begin(), b0.end());
    std::printf("%-9s B starts %7.2f us after the first s0 kernel (s0 chain 20 x 40 us)\n", fill ? "roots_fil" : "roots",
                b0[b0.size() / 2]);
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
  }
  // two graphs, one per stream, linked by an external event: graph A on s0 = A -> record(ev) -> D (60 us);
  // graph B on s1 = wait(ev) -> B.  A->B is the cross-graph edge (explicit queue placement instead of the executor's)
  {
    hipEvent_t ex;
    CHECK(hipEventCreateWithFlags(&ex, hipEventDisableTiming));
    hipGraph_t ga, gb;
    CHECK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
    launch(s0, st, 0, 20);
    CHECK(hipEventRecordWithFlags(ex, s0, hipEventRecordExternal));
    launch(s0, st, 3, 60);
    CHECK(hipStreamEndCapture(s0, &ga));
    CHECK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
    CHECK(hipStreamWaitEvent(s1, ex, hipEventWaitExternal));
    launch(s1, st, 1, 5);
    CHECK(hipStreamEndCapture(s1, &gb));
    hipGraphExec_t ea, eb;
    CHECK(hipGraphInstantiate(&ea, ga, nullptr, nullptr, 0));
    CHECK(hipGraphInstantiate(&eb, gb, nullptr, nullptr, 0));
    std::vector<double> ab, span;
    for (int r = 0; r < reps + 3; ++r) {
      CHECK(hipMemset(st, 0, 64 * sizeof(unsigned long long)));
      CHECK(hipDeviceSynchronize());
      CHECK(hipGraphLaunch(ea, s0));
      CHECK(hipGraphLaunch(eb, s1));
      CHECK(hipDeviceSynchronize());
      unsigned long long h[8];
      CHECK(hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
      if (r < 3) continue;
      ab.push_back(((double)h[2] - (double)h[1]) / 100.0);
      span.push_back(((double)h[7] - (double)h[0]) / 100.0);
    }
    std::sort(ab.begin(), ab.end());
    std::sort(span.begin(), span.end());
    std::printf("%-9s A->B %6.2f us  (two graphs, external event)  span(A..D) %7.2f us\n", "xgraph", ab[ab.size() / 2],
                span[span.size() / 2]);
    CHECK(hipGraphExecDestroy(ea));
    CHECK(hipGraphExecDestroy(eb));
    CHECK(hipGraphDestroy(ga));
    CHECK(hipGraphDestroy(gb));
    CHECK(hipEventDestroy(ex));
  }
  CHECK(hipFree(st));
  return 0;
}
