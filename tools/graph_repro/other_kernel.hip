// Code object loaded at run time by graph_capture_repro (hipModuleLoad between graph replays, the way torch
// lazily loads kernels from its fat binaries).
#include <hip/hip_runtime.h>

extern "C" __global__ void other_kernel(float* x, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] * 0.25f + v;
}
