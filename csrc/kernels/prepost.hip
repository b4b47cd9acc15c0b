// Pre/post-processing kernels shared by every model:
//   * sa_preprocess  — one fused pass replacing the reference's four per-model preprocess kernels
//     (RAFTStereo/src/stereo_preprocess.cu:4-39, HitNet/src/HitNet_preprocess.cu:4-53,
//     CREStereo/src/CREStereo_preprocess.cu:4-39, FastACVNet_plus/src/FastACVNet_plus_preprocess.cu:4-39):
//     u8 BGR HWC -> fp16 NHWC RGB with the model's normalisation, written straight into the
//     network's padded input channels;
//   * sa_remap_bgr   — GPU stereo rectification (cv::remap INTER_LINEAR / BORDER_CONSTANT with
//     OpenCV's 1/32-pixel fixed-point interpolation table), replacing the per-frame CPU path of
//     RAFTStereo/src/RAFTStereoAlgorithm.cpp:113-126;
//   * sa_reproject   — disparity -> XYZRGB (cv::reprojectImageTo3D) replacing the four
//     reprojection kernels (e.g. RAFTStereo/src/stereo_preprocess.cu:41-68); `sign` covers
//     RAFT-Stereo's negative-flow output, and it runs on the caller's stream (the reference
//     launched it on the legacy default stream);
//   * sa_convex_upsample — RAFT-Stereo / CREStereo learned convex upsampling (softmax over the 3x3
//     neighbourhood, x factor^2 sub-pixels), output as signed fp32 disparity.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include "sa/kernels.h"

namespace {
typedef _Float16 f16;

__global__ void preprocess_kernel(const uint8_t* __restrict__ bgr, int total, int mode,
                                  f16* __restrict__ out, int ostride, int c_off, int zero_to) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const uint8_t* p = bgr + (long)i * 3;
  float rgb[3] = {(float)p[2], (float)p[1], (float)p[0]};
  const float mean[3] = {0.485f, 0.456f, 0.406f};
  const float stdv[3] = {0.229f, 0.224f, 0.225f};
  f16* o = out + (long)i * ostride;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float v = rgb[c];
    switch (mode) {
      case SA_PRE_UNIT: v = v / 255.f; break;
      case SA_PRE_IMAGENET: v = (v / 255.f - mean[c]) / stdv[c]; break;
      case SA_PRE_SIGNED: v = 2.f * (v / 255.f) - 1.f; break;
      default: break;
    }
    o[c_off + c] = (f16)v;
  }
  for (int c = c_off + 3; c < zero_to; ++c) o[c] = (f16)0.f;
}

// OpenCV remap with CV_16SC2 maps: coordinates quantised to 1/32 px (INTER_TAB_SIZE), weights
// in 1/32768 fixed point (INTER_REMAP_COEF_SCALE), rounding add 1<<14.
__global__ void remap_kernel(const uint8_t* __restrict__ src, int B, int Hs, int Ws,
                             const float* __restrict__ maps, int nmaps, int H, int W,
                             uint8_t* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = B * H * W;
  if (i >= total) return;
  const int b = i / (H * W);
  const int pix = i - b * H * W;
  const float* mp = maps + ((long)(b % nmaps) * H * W + pix) * 2;
  const int iu = __float2int_rn(mp[0] * 32.f);
  const int iv = __float2int_rn(mp[1] * 32.f);
  const int x0 = iu >> 5, y0 = iv >> 5;
  const float ax = (float)(iu & 31) / 32.f, ay = (float)(iv & 31) / 32.f;
  int w[4];
  w[0] = __float2int_rn((1.f - ax) * (1.f - ay) * 32768.f);
  w[1] = __float2int_rn(ax * (1.f - ay) * 32768.f);
  w[2] = __float2int_rn((1.f - ax) * ay * 32768.f);
  w[3] = __float2int_rn(ax * ay * 32768.f);
  int diff = w[0] + w[1] + w[2] + w[3] - 32768;
  if (diff != 0) {  // OpenCV corrects the largest (diff<0) / smallest (diff>0) coefficient
    int k = 0;
    for (int j = 1; j < 4; ++j)
      if (diff < 0 ? (w[j] > w[k]) : (w[j] < w[k])) k = j;
    w[k] -= diff;
  }
  const uint8_t* img = src + (long)b * Hs * Ws * 3;
  int acc[3] = {0, 0, 0};
  for (int j = 0; j < 4; ++j) {
    int xx = x0 + (j & 1), yy = y0 + (j >> 1);
    if (xx < 0 || xx >= Ws || yy < 0 || yy >= Hs) continue;
    const uint8_t* q = img + ((long)yy * Ws + xx) * 3;
    acc[0] += w[j] * q[0];
    acc[1] += w[j] * q[1];
    acc[2] += w[j] * q[2];
  }
  uint8_t* o = dst + (long)i * 3;
  for (int c = 0; c < 3; ++c) {
    int v = (acc[c] + (1 << 14)) >> 15;
    o[c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
}

struct Q16 {
  float q[16];
};

// One thread per pixel computes its XYZRGB; the workgroup's 256 x 6 floats are staged in LDS and leave as
// contiguous 16-B stores (the cloud and the disparity copy may live in pinned host memory: the engine's zero-copy
// run_host path writes them straight over PCIe, where 4-B stores with a 24-B stride would cost a bus transaction
// each).
__global__ __launch_bounds__(256) void reproject_kernel(const float* __restrict__ din, int dstride, float sign,
                                                        const uint8_t* __restrict__ left, int B, int H, int W, Q16 Q,
                                                        float* __restrict__ dout, float* __restrict__ cloud) {
  __shared__ __attribute__((aligned(16))) float st[256 * 6];
  __shared__ __attribute__((aligned(16))) float sd[256];
  const int total = B * H * W;
  const long base = (long)blockIdx.x * 256;
  const int i = (int)base + threadIdx.x;
  const bool ok = i < total;
  float d = 0.f;
  if (ok) {
    const int pix = i % (H * W);
    const int r = pix / W, c = pix - (pix / W) * W;
    d = sign * din[(long)i * dstride];
    const float* q = Q.q;
    const float X = q[0] * c + q[1] * r + q[2] * d + q[3];
    const float Y = q[4] * c + q[5] * r + q[6] * d + q[7];
    const float Z = q[8] * c + q[9] * r + q[10] * d + q[11];
    const float Wh = q[12] * c + q[13] * r + q[14] * d + q[15];
    float* o = st + threadIdx.x * 6;
    o[0] = X / Wh;
    o[1] = Y / Wh;
    o[2] = Z / Wh;
    const uint8_t* px = left + (long)i * 3;
    o[3] = (float)px[2];
    o[4] = (float)px[1];
    o[5] = (float)px[0];
  }
  sd[threadIdx.x] = d;
  __syncthreads();
  const int n = total - (int)base < 256 ? total - (int)base : 256;  // pixels of this workgroup
  if (cloud) {
    float* cb = cloud + base * 6;
    if (n == 256 && (((uintptr_t)cb) & 15) == 0) {
      for (int k = threadIdx.x; k < 384; k += 256)
        reinterpret_cast<float4*>(cb)[k] = reinterpret_cast<const float4*>(st)[k];
    } else {
      for (int k = threadIdx.x; k < n * 6; k += 256) cb[k] = st[k];
    }
  }
  if (dout) {
    float* db = dout + base;
    if (n == 256 && (((uintptr_t)db) & 15) == 0) {
      if (threadIdx.x < 64) reinterpret_cast<float4*>(db)[threadIdx.x] = reinterpret_cast<const float4*>(sd)[threadIdx.x];
    } else if (threadIdx.x < n) {
      db[threadIdx.x] = sd[threadIdx.x];
    }
  }
}

__global__ void convex_upsample_kernel(const f16* __restrict__ mask, int mstride,
                                       const float* __restrict__ flow, int B, int H, int W, int f,
                                       float sign, float* __restrict__ out) {
  const int Ho = H * f, Wo = W * f;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * Ho * Wo) return;
  const int b = i / (Ho * Wo);
  const int p = i - b * Ho * Wo;
  const int oy = p / Wo, ox = p - (p / Wo) * Wo;
  const int h = oy / f, w = ox / f, fy = oy - h * f, fx = ox - w * f;
  const long lp = (long)(b * H + h) * W + w;
  const f16* m = mask + lp * mstride + fy * f + fx;
  float mv[9], mx = -1e30f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    mv[k] = (float)m[k * f * f];
    mx = fmaxf(mx, mv[k]);
  }
  float den = 0.f, num = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = h + k / 3 - 1, xx = w + k % 3 - 1;
    const float e = __expf(mv[k] - mx);
    den += e;
    const float fv = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? flow[(long)(b * H + yy) * W + xx] : 0.f;
    num += e * fv;
  }
  out[i] = sign * (float)f * num / den;
}

// multi-channel convex upsampling (CREStereo flow has x and y)
__global__ void convex_upsample_c_kernel(const f16* __restrict__ mask, int mstride, const float* __restrict__ flow,
                                         int fc, int B, int H, int W, int f, float sign, float* __restrict__ out,
                                         int oc) {
  const int Ho = H * f, Wo = W * f;
  const long total = (long)B * Ho * Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / ((long)Ho * Wo));
    const long p = i - (long)b * Ho * Wo;
    const int oy = (int)(p / Wo), ox = (int)(p % Wo);
    const int h = oy / f, w = ox / f, fy = oy - h * f, fx = ox - w * f;
    const long lp = ((long)b * H + h) * W + w;
    const f16* m = mask + lp * mstride + fy * f + fx;
    float mv[9], mx = -1e30f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      mv[k] = (float)m[k * f * f];
      mx = fmaxf(mx, mv[k]);
    }
    float den = 0.f, num[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int yy = h + k / 3 - 1, xx = w + k % 3 - 1;
      const float e = __expf(mv[k] - mx);
      den += e;
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        const float* fv = flow + (((long)b * H + yy) * W + xx) * fc;
        for (int c = 0; c < oc; ++c) num[c] += e * fv[c];
      }
    }
    for (int c = 0; c < oc; ++c) out[i * oc + c] = sign * (float)f * num[c] / den;
  }
}

}  // namespace

extern "C" int sa_convex_upsample_c(const void* mask, int mask_stride, const float* flow, int fc, int B, int H,
                                    int W, int factor, float sign, float* out, int oc, hipStream_t stream) {
  if (oc < 1 || oc > 4 || oc > fc) return -2;
  const long total = (long)B * H * W * factor * factor;
  long g = (total + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(convex_upsample_c_kernel, dim3((unsigned)g), dim3(256), 0, stream, (const f16*)mask,
                     mask_stride, flow, fc, B, H, W, factor, sign, out, oc);
  return (int)hipGetLastError();
}

extern "C" int sa_preprocess(const uint8_t* bgr, int B, int H, int W, int mode, void* out,
                             int out_stride, int c_off, int zero_to, hipStream_t stream) {
  int total = B * H * W;
  hipLaunchKernelGGL(preprocess_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, bgr, total,
                     mode, (f16*)out, out_stride, c_off, zero_to);
  return (int)hipGetLastError();
}

extern "C" int sa_remap_bgr(const uint8_t* src, int B, int Hs, int Ws, const float* maps,
                            int nmaps, int H, int W, uint8_t* dst, hipStream_t stream) {
  int total = B * H * W;
  hipLaunchKernelGGL(remap_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, src, B, Hs, Ws,
                     maps, nmaps, H, W, dst);
  return (int)hipGetLastError();
}

extern "C" int sa_reproject(const float* disp_in, int disp_stride, float sign,
                            const uint8_t* left_bgr, int B, int H, int W, const float* Q16p,
                            float* disp_out, float* cloud, hipStream_t stream) {
  Q16 q;
  for (int i = 0; i < 16; ++i) q.q[i] = Q16p[i];
  int total = B * H * W;
  hipLaunchKernelGGL(reproject_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, disp_in,
                     disp_stride, sign, left_bgr, B, H, W, q, disp_out, cloud);
  return (int)hipGetLastError();
}

// Re-point the output arguments of a reprojection kernel node of an instantiated graph (the node captured from
// sa_reproject; everything but disp_out / cloud must be what it was captured with).  The engine's host-output frame
// graphs write straight into host memory -- its own pinned buffers or mapped caller buffers -- and a different
// caller buffer only changes these two arguments: one node update instead of a re-capture, nothing per frame.
extern "C" int sa_reproject_update_node(hipGraphExec_t exec, hipGraphNode_t node, const float* disp_in,
                                        int disp_stride, float sign, const uint8_t* left_bgr, int B, int H, int W,
                                        const float* Q16p, float* disp_out, float* cloud) {
  hipKernelNodeParams p{};
  hipError_t e = hipGraphKernelNodeGetParams(node, &p);
  if (e != hipSuccess) return (int)e;
  if (p.func != reinterpret_cast<void*>(reproject_kernel)) return -2;
  Q16 q;
  for (int i = 0; i < 16; ++i) q.q[i] = Q16p[i];
  void* args[] = {(void*)&disp_in, (void*)&disp_stride, (void*)&sign, (void*)&left_bgr, (void*)&B, (void*)&H,
                  (void*)&W, (void*)&q, (void*)&disp_out, (void*)&cloud};
  p.kernelParams = args;
  p.extra = nullptr;
  return (int)hipGraphExecKernelNodeSetParams(exec, node, &p);
}

// Frame inputs straight from mapped host memory (run_host's zero-copy input path): one launch copies both images of
// the frame from the caller's registered arrays or the engine's pinned staging into device memory -- PCIe reads
// issued by the CUs, replacing two host-enqueued DMA copies ahead of the graph.  16 B per lane; bytes % 16 == 0.
__global__ __launch_bounds__(256) void copy_frames_kernel(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                          uint4* __restrict__ da, uint4* __restrict__ db, long n16) {
  const uint4* src = blockIdx.y ? b : a;
  uint4* dst = blockIdx.y ? db : da;
  constexpr int U = 4;
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * U; i < n16; i += (long)gridDim.x * 256 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u < n16) v[u] = src[i + u];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u < n16) dst[i + u] = v[u];
  }
}

static dim3 copy_frames_grid(long n16) {
  long g = (n16 + 1023) / 1024;
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  return dim3((unsigned)g, 2);
}

extern "C" int sa_copy_frames(const void* a, const void* b, void* da, void* db, long bytes, hipStream_t stream) {
  if (bytes <= 0 || bytes % 16 || ((uintptr_t)a | (uintptr_t)b | (uintptr_t)da | (uintptr_t)db) % 16) return -2;
  const long n16 = bytes / 16;
  hipLaunchKernelGGL(copy_frames_kernel, copy_frames_grid(n16), dim3(256), 0, stream, (const uint4*)a, (const uint4*)b,
                     (uint4*)da, (uint4*)db, n16);
  return (int)hipGetLastError();
}

// re-point the sources of a captured sa_copy_frames node (destinations / size unchanged)
extern "C" int sa_copy_frames_update_node(hipGraphExec_t exec, hipGraphNode_t node, const void* a, const void* b,
                                          void* da, void* db, long bytes) {
  if (bytes <= 0 || bytes % 16 || ((uintptr_t)a | (uintptr_t)b) % 16) return -2;
  hipKernelNodeParams p{};
  hipError_t e = hipGraphKernelNodeGetParams(node, &p);
  if (e != hipSuccess) return (int)e;
  if (p.func != reinterpret_cast<void*>(copy_frames_kernel)) return -2;
  const long n16 = bytes / 16;
  const uint4 *sa = (const uint4*)a, *sb = (const uint4*)b;
  uint4 *sda = (uint4*)da, *sdb = (uint4*)db;
  void* args[] = {(void*)&sa, (void*)&sb, (void*)&sda, (void*)&sdb, (void*)&n16};
  p.kernelParams = args;
  p.extra = nullptr;
  return (int)hipGraphExecKernelNodeSetParams(exec, node, &p);
}

extern "C" int sa_convex_upsample(const void* mask, int mask_stride, const float* flow, int B,
                                  int H, int W, int factor, float sign, float* out,
                                  hipStream_t stream) {
  int total = B * H * W * factor * factor;
  hipLaunchKernelGGL(convex_upsample_kernel, dim3((total + 255) / 256), dim3(256), 0, stream,
                     (const f16*)mask, mask_stride, flow, B, H, W, factor, sign, out);
  return (int)hipGetLastError();
}

// ---- stage timestamps: one wave writes the GPU's constant-rate wall clock (a kernel node of the
// frame graph, so it runs after everything queued before it on the stream)
namespace {
__global__ void stamp_kernel(unsigned long long* buf, int idx) {
  if (threadIdx.x == 0) buf[idx] = wall_clock64();
}
}  // namespace

extern "C" int sa_stamp(unsigned long long* buf, int idx, hipStream_t stream) {
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, stream, buf, idx);
  return (int)hipGetLastError();
}
