// Memory-bound NHWC fp16 kernels: instance-norm apply (+residual), 3x3/s2 and kxk average
// pooling, bilinear resize.  Every thread moves 8 channels (16 B) per access (CDNA4 guide,
// Guideline 13) and the kernels read/write channel slices of wider buffers so that
// torch.cat-style concatenations in the upstream networks are free.
//
// Upstream ops mirrored: nn.InstanceNorm2d (RAFT-Stereo fnet, CREStereo fnet),
// pool2x = F.avg_pool2d(x, 3, 2, 1) and interp = F.interpolate(bilinear, align_corners=True)
// between the multi-level ConvGRUs of RAFT-Stereo.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <hip/hip_fp16.h>

#include "sa/kernels.h"

namespace {

// zero fill with 16-B vector stores (a captured hipMemsetAsync of a few MB becomes a chain of small
// runtime fill kernels: ~20 us each, 18 per RAFT-SF b8 frame for the instance-norm statistics pool)
__global__ __launch_bounds__(256) void zero16_kernel(uint4* __restrict__ p, long n16) {
  const uint4 z = {0u, 0u, 0u, 0u};
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) p[i] = z;
}
__global__ __launch_bounds__(256) void zero4_kernel(unsigned* __restrict__ p, long n4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) p[i] = 0u;
}
typedef _Float16 f16;
typedef f16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float act_apply(float v, int act, float alpha) {
  switch (act) {
    case SA_ACT_RELU: return v > 0.f ? v : 0.f;
    case SA_ACT_LEAKY: return v > 0.f ? v : v * alpha;
    case SA_ACT_TANH: return tanhf(v);
    case SA_ACT_SIGMOID: return 1.f / (1.f + __expf(-v));
    default: return v;
  }
}

__device__ __forceinline__ void ld8(const f16* p, float* v) {
  half8 h = *reinterpret_cast<const half8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)h[j];
}
__device__ __forceinline__ void st8(f16* p, const float* v) {
  half8 h;
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = (f16)v[j];
  *reinterpret_cast<half8*>(p) = h;
}

// Per-(image, channel) mean and rstd of the block's image into LDS once per block: the fixed-point sums of the
// stat_slots copies are added in integer (bitwise the sum sa_stats_reduce would leave in copy 0), so no separate
// fold launch precedes the apply (round 4: one 1-2 workgroup launch + edge per instance norm on the critical chain).
// lds: [mean C][rstd C][rmean C][rrstd C] floats.
__device__ __forceinline__ void norm_lds(const sa_stat_t* st, int slots, int N, int C, int n, long HW, float eps,
                                         float* mean, float* rstd) {
  const double inv = 1.0 / ((double)HW * SA_STAT_SCALE);
  const long slot = (long)N * C * 2;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const sa_stat_t* s = st + ((long)n * C + c) * 2;
    // every slot's pair loaded before the adds (integer sums: any order is bitwise the same).  A plain r-loop kept
    // one L2 round trip per slot in flight: 16 serial loads at the start of every apply block (12-24 us per
    // CREStereo / RAFT encoder apply at 600 workgroups)
    typedef long long ll2 __attribute__((ext_vector_type(2)));
    long long s0 = 0, s1 = 0;
    int r = 0;
    for (; r + 8 <= slots; r += 8) {
      ll2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const ll2*>(s + (r + u) * slot);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s0 += v[u][0];
        s1 += v[u][1];
      }
    }
    for (; r < slots; ++r) {
      s0 += s[r * slot];
      s1 += s[r * slot + 1];
    }
    const double m = (double)s0 * inv;
    const double var = (double)s1 * inv - m * m;
    mean[c] = (float)m;
    rstd[c] = rsqrtf((float)(var > 0.0 ? var : 0.0) + eps);
  }
}

// grid: (pixel chunks, N); a block's threads tile (pixels x channel groups) of one image, each thread
// keeps one channel group and walks pixels
__global__ __launch_bounds__(256) void instnorm_apply_kernel(const SaNormArgs a, int pix_per_block) {
  extern __shared__ float nlds[];
  const int C8 = a.C >> 3;
  const int n = blockIdx.y;
  const int tid = threadIdx.x;
  const int slots = a.stat_slots > 1 ? a.stat_slots : 1;
  const bool rs = a.res && a.res_stats;
  norm_lds(a.stats, slots, a.N, a.C, n, a.HW, a.eps, nlds, nlds + a.C);
  if (rs) norm_lds(a.res_stats, slots, a.N, a.C, n, a.HW, a.eps, nlds + 2 * a.C, nlds + 3 * a.C);
  __syncthreads();
  const int c8 = tid % C8;
  const int lanes_per_c = 256 / C8;  // threads sharing a channel group
  if (tid >= lanes_per_c * C8) return;
  const int c = c8 * 8;
  float mean[8], rstd[8], rmean[8], rrstd[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mean[j] = nlds[c + j];
    rstd[j] = nlds[a.C + c + j];
    rmean[j] = rs ? nlds[2 * a.C + c + j] : 0.f;
    rrstd[j] = rs ? nlds[3 * a.C + c + j] : 1.f;
  }
  const long p0 = (long)blockIdx.x * pix_per_block;
  const long p1 = p0 + pix_per_block < a.HW ? p0 + pix_per_block : a.HW;
  // 4 pixels per step, every load issued before the first store (out may alias x: the compiler would
  // otherwise keep one 16-B load in flight per thread)
  constexpr int U = 4;
  const f16* xb = reinterpret_cast<const f16*>(a.x);
  const f16* rb = reinterpret_cast<const f16*>(a.res);
  f16* ob = reinterpret_cast<f16*>(a.out);
  for (long pb = p0 + tid / C8; pb < p1; pb += (long)U * lanes_per_c) {
    half8 hx[U], hr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long p = pb + (long)u * lanes_per_c;
      if (p < p1) {
        const long pix = (long)n * a.HW + p;
        hx[u] = *reinterpret_cast<const half8*>(xb + pix * a.x_stride + c);
        if (rb) hr[u] = *reinterpret_cast<const half8*>(rb + pix * a.res_stride + c);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long p = pb + (long)u * lanes_per_c;
      if (p >= p1) break;
      const long pix = (long)n * a.HW + p;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = act_apply(((float)hx[u][j] - mean[j]) * rstd[j], a.act, a.alpha);
      if (rb) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float r = rs ? act_apply(((float)hr[u][j] - rmean[j]) * rrstd[j], a.res_act, a.alpha) : (float)hr[u][j];
          v[j] = act_apply(v[j] + r, a.act2, a.alpha);
        }
      }
      st8(ob + pix * a.out_stride + c, v);
    }
  }
}

__global__ void stats_reduce_kernel(sa_stat_t* stats, int slots, long count) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < count; i += (long)gridDim.x * blockDim.x) {
    sa_stat_t acc = 0;
    for (int r = 0; r < slots; ++r) {
      acc += stats[(size_t)r * count + i];
      if (r > 0) stats[(size_t)r * count + i] = 0;
    }
    stats[i] = acc;
  }
}

struct PoolJob {
  const f16* x;
  int xs;
  f16* out;
  int os, N, H, W, C, Ho, Wo;
};
struct InterpJob {
  const f16* x;
  int xs;
  f16* out;
  int os, N, H, W, C, Ho, Wo, ac;
  float mul;
};

// 3x3 / stride 2 / pad 1 average (count_include_pad), elements i0, i0 + step, ...
__device__ __forceinline__ void avgpool3s2_body(const PoolJob& j, long i0, long step) {
  const f16* __restrict__ x = j.x;
  const int C8 = j.C >> 3, H = j.H, W = j.W, Ho = j.Ho, Wo = j.Wo;
  const long total = (long)j.N * Ho * Wo * C8;
  for (long i = i0; i < total; i += step) {
    // 32-bit index decomposition (total < 2^31, host-checked): 64-bit div/mod is a long emulated
    // sequence per element that outweighed the 8-channel arithmetic
    const unsigned ii = (unsigned)i;
    const int c = (int)(ii % (unsigned)C8) * 8;
    unsigned p = ii / (unsigned)C8;
    const int ow = (int)(p % (unsigned)Wo);
    p /= (unsigned)Wo;
    const int oh = (int)(p % (unsigned)Ho);
    const int n = (int)(p / (unsigned)Ho);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int dy = -1; dy <= 1; ++dy) {
      int ih = oh * 2 + dy;
      if (ih < 0 || ih >= H) continue;
      for (int dx = -1; dx <= 1; ++dx) {
        int iw = ow * 2 + dx;
        if (iw < 0 || iw >= W) continue;
        float v[8];
        ld8(x + ((long)(n * H + ih) * W + iw) * j.xs + c, v);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += v[q];
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] *= (1.f / 9.f);
    st8(j.out + ((long)(n * Ho + oh) * Wo + ow) * j.os + c, acc);
  }
}

__global__ void avgpool3s2_kernel(const PoolJob j) {
  avgpool3s2_body(j, blockIdx.x * (long)blockDim.x + threadIdx.x, (long)gridDim.x * blockDim.x);
}

__global__ void avgpoolk_kernel(const f16* __restrict__ x, int xs, f16* __restrict__ out, int os,
                                int N, int H, int W, int C, int Ho, int Wo, int k) {
  const int C8 = C >> 3;
  const long total = (long)N * Ho * Wo * C8;
  const float inv = 1.f / (float)(k * k);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    // 32-bit index decomposition (total < 2^31, host-checked): 64-bit div/mod is a long emulated
    // sequence per element that outweighed the 8-channel arithmetic
    const unsigned ii = (unsigned)i;
    const int c = (int)(ii % (unsigned)C8) * 8;
    unsigned p = ii / (unsigned)C8;
    const int ow = (int)(p % (unsigned)Wo);
    p /= (unsigned)Wo;
    const int oh = (int)(p % (unsigned)Ho);
    const int n = (int)(p / (unsigned)Ho);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int dy = 0; dy < k; ++dy)
      for (int dx = 0; dx < k; ++dx) {
        float v[8];
        ld8(x + ((long)(n * H + oh * k + dy) * W + ow * k + dx) * xs + c, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j];
      }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= inv;
    st8(out + ((long)(n * Ho + oh) * Wo + ow) * os + c, acc);
  }
}

__device__ __forceinline__ float src_index(int dst, int in_size, int out_size, int ac) {
  if (ac) return out_size > 1 ? (float)dst * (float)(in_size - 1) / (float)(out_size - 1) : 0.f;
  float s = ((float)dst + 0.5f) * (float)in_size / (float)out_size - 0.5f;
  return s < 0.f ? 0.f : s;
}

// bilinear resize (align_corners = ac) times mul, elements i0, i0 + step, ...
__device__ __forceinline__ void interp_body(const InterpJob& j, long i0, long step) {
  const f16* __restrict__ x = j.x;
  const int C8 = j.C >> 3, H = j.H, W = j.W, Ho = j.Ho, Wo = j.Wo;
  const long total = (long)j.N * Ho * Wo * C8;
  for (long i = i0; i < total; i += step) {
    // 32-bit index decomposition (total < 2^31, host-checked)
    const unsigned ii = (unsigned)i;
    const int c = (int)(ii % (unsigned)C8) * 8;
    unsigned p = ii / (unsigned)C8;
    const int ow = (int)(p % (unsigned)Wo);
    p /= (unsigned)Wo;
    const int oh = (int)(p % (unsigned)Ho);
    const int n = (int)(p / (unsigned)Ho);
    float sy = src_index(oh, H, Ho, j.ac), sx = src_index(ow, W, Wo, j.ac);
    int y0 = (int)floorf(sy), x0 = (int)floorf(sx);
    y0 = y0 > H - 1 ? H - 1 : y0;
    x0 = x0 > W - 1 ? W - 1 : x0;
    int y1 = y0 + 1 < H ? y0 + 1 : H - 1;
    int x1 = x0 + 1 < W ? x0 + 1 : W - 1;
    float ly = sy - y0, lx = sx - x0;
    float v00[8], v01[8], v10[8], v11[8];
    ld8(x + ((long)(n * H + y0) * W + x0) * j.xs + c, v00);
    ld8(x + ((long)(n * H + y0) * W + x1) * j.xs + c, v01);
    ld8(x + ((long)(n * H + y1) * W + x0) * j.xs + c, v10);
    ld8(x + ((long)(n * H + y1) * W + x1) * j.xs + c, v11);
    float r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      r[q] = j.mul * ((1.f - ly) * ((1.f - lx) * v00[q] + lx * v01[q]) + ly * ((1.f - lx) * v10[q] + lx * v11[q]));
    st8(j.out + ((long)(n * Ho + oh) * Wo + ow) * j.os + c, r);
  }
}

__global__ void interp_kernel(const InterpJob j) {
  interp_body(j, blockIdx.x * (long)blockDim.x + threadIdx.x, (long)gridDim.x * blockDim.x);
}

// a pool job and an interp job of one GRU level's inputs in one launch: blocks [0, gp) pool, the rest interp
// (same per-element arithmetic as the two kernels, so the results are bitwise those of two launches)
__global__ void pool_interp_kernel(const PoolJob pj, const InterpJob ij, int gp) {
  if ((int)blockIdx.x < gp) avgpool3s2_body(pj, blockIdx.x * (long)blockDim.x + threadIdx.x, (long)gp * blockDim.x);
  else interp_body(ij, (blockIdx.x - gp) * (long)blockDim.x + threadIdx.x, (long)(gridDim.x - gp) * blockDim.x);
}

// max |a - b| and max |b| over n elements (fp16 or fp32), as float bits in res[0] / res[1] (non-negative
// floats order like their unsigned bit patterns, so a vector atomicMax merges blocks).  A NaN / inf
// difference counts as +inf.  Used by the conv tactic tuner to reject a candidate whose output disagrees
// with the reference candidate's.
__global__ void absdiff_max_kernel(const void* __restrict__ a, const void* __restrict__ b, long n, int f32,
                                   unsigned* __restrict__ res) {
  float md = 0.f, mb = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float x = f32 ? ((const float*)a)[i] : (float)((const f16*)a)[i];
    const float y = f32 ? ((const float*)b)[i] : (float)((const f16*)b)[i];
    float d = fabsf(x - y);
    if (!(d <= 3.0e38f)) d = INFINITY;  // NaN or inf
    md = fmaxf(md, d);
    const float ay = fabsf(y);
    if (ay <= 3.0e38f) mb = fmaxf(mb, ay);
  }
  for (int o = 32; o > 0; o >>= 1) {
    md = fmaxf(md, __shfl_xor(md, o));
    mb = fmaxf(mb, __shfl_xor(mb, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(res, __float_as_uint(md));
    atomicMax(res + 1, __float_as_uint(mb));
  }
}

inline int grid_for(long work) {
  long g = (work + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" int sa_zero(void* p, size_t bytes, hipStream_t stream) {
  if (((uintptr_t)p & 3) || (bytes & 3)) return -2;
  if (((uintptr_t)p & 15) || (bytes & 15)) {  // 4-byte granularity (fp32 / int buffers of any length)
    const long n4 = (long)(bytes >> 2);
    if (n4 == 0) return 0;
    long blocks = (n4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(zero4_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (unsigned*)p, n4);
    return (int)hipGetLastError();
  }
  const long n16 = (long)(bytes >> 4);
  if (n16 == 0) return 0;
  long blocks = (n16 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(zero16_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (uint4*)p, n16);
  return (int)hipGetLastError();
}

extern "C" int sa_instnorm_apply(const SaNormArgs* a, hipStream_t stream) {
  if (a->C % 8) return -2;
  if (a->C > 8 * 256) return -3;
  // ~8 pixels per thread: enough reuse of the per-thread statistics, enough blocks to fill the chip
  const int lanes_per_c = 256 / (a->C / 8);
  const int ppb = lanes_per_c * 8;
  const long chunks = (a->HW + ppb - 1) / ppb;
  if (chunks > 2147483647L || a->N > 65535) return -3;
  const size_t lds = (size_t)a->C * 4 * sizeof(float);
  hipLaunchKernelGGL(instnorm_apply_kernel, dim3((unsigned)chunks, a->N), dim3(256), lds, stream, *a, ppb);
  return (int)hipGetLastError();
}

extern "C" int sa_avgpool3s2(const void* x, int xs, void* out, int os, int N, int H, int W, int C,
                             hipStream_t stream) {
  if (C % 8) return -2;
  int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  long work = (long)N * Ho * Wo * (C / 8);
  if (work >= (1L << 31)) return -2;  // 32-bit index math in the kernel
  hipLaunchKernelGGL(avgpool3s2_kernel, dim3(grid_for(work)), dim3(256), 0, stream,
                     PoolJob{(const f16*)x, xs, (f16*)out, os, N, H, W, C, Ho, Wo});
  return (int)hipGetLastError();
}

extern "C" int sa_avgpool_k(const void* x, int xs, void* out, int os, int N, int H, int W, int C,
                            int k, hipStream_t stream) {
  if (C % 8) return -2;
  int Ho = H / k, Wo = W / k;
  long work = (long)N * Ho * Wo * (C / 8);
  if (work >= (1L << 31)) return -2;  // 32-bit index math in the kernel
  hipLaunchKernelGGL(avgpoolk_kernel, dim3(grid_for(work)), dim3(256), 0, stream, (const f16*)x,
                     xs, (f16*)out, os, N, H, W, C, Ho, Wo, k);
  return (int)hipGetLastError();
}

extern "C" int sa_interp_bilinear(const void* x, int xs, void* out, int os, int N, int H, int W,
                                  int C, int Ho, int Wo, int ac, float mul, hipStream_t stream) {
  if (C % 8) return -2;
  long work = (long)N * Ho * Wo * (C / 8);
  if (work >= (1L << 31)) return -2;  // 32-bit index math in the kernel
  hipLaunchKernelGGL(interp_kernel, dim3(grid_for(work)), dim3(256), 0, stream,
                     InterpJob{(const f16*)x, xs, (f16*)out, os, N, H, W, C, Ho, Wo, ac, mul});
  return (int)hipGetLastError();
}

extern "C" int sa_pool_interp(const void* px, int pxs, void* pout, int pos, int pN, int pH, int pW, int pC,
                              const void* ix, int ixs, void* iout, int ios, int iN, int iH, int iW, int iC, int iHo,
                              int iWo, int ac, float mul, hipStream_t stream) {
  if (pC % 8 || iC % 8) return -2;
  const int pHo = (pH - 1) / 2 + 1, pWo = (pW - 1) / 2 + 1;
  const long pwork = (long)pN * pHo * pWo * (pC / 8), iwork = (long)iN * iHo * iWo * (iC / 8);
  if (pwork >= (1L << 31) || iwork >= (1L << 31)) return -2;
  const int gp = grid_for(pwork), gi = grid_for(iwork);
  hipLaunchKernelGGL(pool_interp_kernel, dim3(gp + gi), dim3(256), 0, stream,
                     PoolJob{(const f16*)px, pxs, (f16*)pout, pos, pN, pH, pW, pC, pHo, pWo},
                     InterpJob{(const f16*)ix, ixs, (f16*)iout, ios, iN, iH, iW, iC, iHo, iWo, ac, mul}, gp);
  return (int)hipGetLastError();
}

extern "C" int sa_absdiff_max(const void* a, const void* b, long n, int f32, unsigned* res, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(absdiff_max_kernel, dim3(grid_for(n)), dim3(256), 0, stream, a, b, n, f32, res);
  return (int)hipGetLastError();
}

extern "C" int sa_stats_reduce(sa_stat_t* stats, int slots, long count, hipStream_t stream) {
  if (slots <= 1) return 0;
  if (count <= 0) return -2;
  long g = (count + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(stats_reduce_kernel, dim3((unsigned)g), dim3(256), 0, stream, stats, slots, count);
  return (int)hipGetLastError();
}
