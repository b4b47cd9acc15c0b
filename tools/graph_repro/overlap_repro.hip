// overlap_repro — do consecutive kernels of one stream / one captured graph ever overlap, and is every
// kernel's output visible to the next one on every XCD?
//
// A chain of NK kernels, each a grid of G blocks that spin ~SPIN cycles:
//   * ordering: block start reads fin[k-1] (agent-scope atomic load); if the previous kernel has not
//     finished all G blocks the block counts a violation; block end does fin[k] += 1.
//   * visibility: kernel k writes buf[k & 1][i] = k for all i with plain stores; kernel k+1 checks that
//     buf[k & 1] holds k everywhere with plain loads (a stale L2 / scalar-cache line on another XCD
//     would show as a mismatch).
//   * memset ordering: every kernel adds 1 to each element of acc[]; a hipMemsetAsync node zeroes acc after
//     kernel NK/2, so at the end acc[i] == NK - 1 - NK/2 exactly when the memset ran between its neighbours.
// Run eagerly, then as a captured graph replayed R times with a null-stream D2D copy + event hand-off
// between replays (the engine's run_device pattern).  Prints a JSON line; exit 1 on any violation.
// --kernel-zero replaces the memset node with a zeroing kernel; --memset-bytes B --memset-offset O zero only
// bytes [O, O+B) of acc (4-byte multiples), e.g. the small / 8-byte-tail memsets the engine used to capture.
//   overlap_repro [--reps R] [--nonblocking] [--kernels NK] [--blocks G]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                              \
    }                                                                                            \
  } while (0)

constexpr int kSpin = 20000;  // ~10 us at ~2 GHz

__global__ __launch_bounds__(256) void k_chain(int k, unsigned* fin, unsigned* viol, unsigned* mism, int* buf0,
                                               int* buf1, int n, int G, int* acc, int nacc) {
  if (threadIdx.x == 0 && k > 0) {
    const unsigned prev = __hip_atomic_load(fin + (k - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev != (unsigned)G) atomicAdd(viol, 1u);
  }
  // check the previous kernel's output, write ours
  int* rd = (k & 1) ? buf0 : buf1;  // written by kernel k-1
  int* wr = (k & 1) ? buf1 : buf0;
  unsigned bad = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += G * 256) {
    if (k > 0 && rd[i] != k - 1) ++bad;
    wr[i] = k;
  }
  if (bad) atomicAdd(mism, bad);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nacc; i += G * 256) acc[i] += 1;
  const long long t0 = clock64();
  while (clock64() - t0 < kSpin) __builtin_amdgcn_s_sleep(2);
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    atomicAdd(fin + k, 1u);
  }
}

__global__ void k_zero(int* p, int n) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[i] = 0;
}

// elements [z0, z1) were zeroed after kernel NK/2 (want_in), the rest count every kernel (want_out)
__global__ void k_check_acc(const int* acc, int n, int z0, int z1, int want_in, int want_out, unsigned* bad) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
    if (acc[i] != ((i >= z0 && i < z1) ? want_in : want_out)) atomicAdd(bad, 1u);
}

int main(int argc, char** argv) {
  int reps = 100, NK = 200, G = 2048;
  bool nonblocking = false, kernel_zero = false;
  long zbytes = -1, zoff = 0;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--reps" && i + 1 < argc) reps = std::atoi(argv[++i]);
    else if (a == "--kernels" && i + 1 < argc) NK = std::atoi(argv[++i]);
    else if (a == "--blocks" && i + 1 < argc) G = std::atoi(argv[++i]);
    else if (a == "--nonblocking") nonblocking = true;
    else if (a == "--kernel-zero") kernel_zero = true;
    else if (a == "--memset-bytes" && i + 1 < argc) zbytes = std::atol(argv[++i]);
    else if (a == "--memset-offset" && i + 1 < argc) zoff = std::atol(argv[++i]);
  }
  const int n = 1 << 22;
  CK(hipSetDevice(0));
  unsigned *fin, *cnt;
  int *buf0, *buf1, *acc;
  const int nacc = 1 << 20;
  CK(hipMalloc(&acc, (size_t)nacc * 4));
  if (zbytes < 0) zbytes = (long)nacc * 4;
  if (zoff % 4 || zbytes % 4 || zoff + zbytes > (long)nacc * 4) {
    std::fprintf(stderr, "bad memset range\n");
    return 2;
  }
  const int z0 = (int)(zoff / 4), z1 = (int)((zoff + zbytes) / 4);
  char *src, *dst;
  CK(hipMalloc(&fin, NK * sizeof(unsigned)));
  CK(hipMalloc(&cnt, 3 * sizeof(unsigned)));
  CK(hipMalloc(&buf0, (size_t)n * 4));
  CK(hipMalloc(&buf1, (size_t)n * 4));
  CK(hipMalloc(&src, 1 << 20));
  CK(hipMalloc(&dst, 1 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, nonblocking ? hipStreamNonBlocking : hipStreamDefault));
  hipEvent_t ein, eout;
  CK(hipEventCreateWithFlags(&ein, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&eout, hipEventDisableTiming));
  auto body = [&](hipStream_t st) {
    CK(hipMemsetAsync(fin, 0, NK * sizeof(unsigned), st));
    hipLaunchKernelGGL(k_zero, dim3(1024), dim3(256), 0, st, acc, nacc);  // frame start: all of acc
    for (int k = 0; k < NK; ++k) {
      hipLaunchKernelGGL(k_chain, dim3(G), dim3(256), 0, st, k, fin, cnt, cnt + 1, buf0, buf1, n, G, acc, nacc);
      if (k == NK / 2) {
        if (kernel_zero) hipLaunchKernelGGL(k_zero, dim3(1024), dim3(256), 0, st, acc + z0, z1 - z0);
        else CK(hipMemsetAsync(acc + z0, 0, (size_t)zbytes, st));
      }
    }
    hipLaunchKernelGGL(k_check_acc, dim3(1024), dim3(256), 0, st, acc, nacc, z0, z1, NK - 1 - NK / 2, NK, cnt + 2);
  };
  unsigned h[3];
  // eager
  CK(hipMemset(cnt, 0, 12));
  body(s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(h, cnt, 12, hipMemcpyDeviceToHost));
  const unsigned eager_viol = h[0], eager_mism = h[1], eager_acc = h[2];
  // graph
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  body(s);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipMemset(cnt, 0, 12));
  CK(hipDeviceSynchronize());
  for (int r = 0; r < reps; ++r) {
    CK(hipMemcpyAsync(dst, src, 1 << 20, hipMemcpyDeviceToDevice, nullptr));  // caller-stream work
    CK(hipEventRecord(ein, nullptr));
    CK(hipStreamWaitEvent(s, ein, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(eout, s));
    CK(hipStreamWaitEvent(nullptr, eout, 0));
  }
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h, cnt, 12, hipMemcpyDeviceToHost));
  const char* pc = std::getenv("DEBUG_CLR_GRAPH_PACKET_CAPTURE");
  std::printf("{\"packet_capture_env\": \"%s\", \"nonblocking\": %s, \"kernels\": %d, \"blocks\": %d, \"reps\": %d, "
              "\"eager_order_violations\": %u, \"eager_stale_reads\": %u, \"graph_order_violations\": %u, "
              "\"graph_stale_reads\": %u, \"zero_node\": \"%s\", \"zero_off\": %ld, \"zero_bytes\": %ld, \"eager_acc_errors\": %u, \"graph_acc_errors\": %u}\n",
              pc ? pc : "(unset)", nonblocking ? "true" : "false", NK, G, reps, eager_viol, eager_mism, h[0], h[1],
              kernel_zero ? "kernel" : "memset", zoff, zbytes, eager_acc, h[2]);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return (eager_viol || eager_mism || eager_acc || h[0] || h[1] || h[2]) ? 1 : 0;
}
