// RAFT-Stereo 1-D all-pairs correlation pyramid and its per-iteration lookup.
//
// corr[b,h,w1,w2] = <fmap1[b,h,w1,:], fmap2[b,h,w2,:]> / sqrt(C) is a batch of per-row GEMMs
// (W1 x W2 x C).  One workgroup owns one image row: the NHWC feature rows are contiguous
// [W][C] panels, so MFMA fragments are loaded straight from L2 with 16-B loads, the 32-row
// result slab is staged in LDS (fp32) and the whole avg-pool pyramid along w2 is written from
// that slab in the same kernel (no second pass over the volume).
//
// Lookup = CorrBlock1D.__call__ of upstream RAFT-Stereo (grid_sample bilinear, align_corners,
// zero padding, 2r+1 taps per level): all taps of a level share one fractional weight, so a
// thread gathers 2r+2 consecutive values per level.  It also emits the [flow_x, 0] features
// the motion encoder consumes, so the update step needs no separate flow-to-fp16 pass.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>
#include <cstdlib>

#include "sa/kernels.h"

namespace {
typedef _Float16 f16;
typedef f16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int CORR_ROWS = 32;  // w1 rows per LDS slab

// one bilinear tap of the lookup, in one fixed rounding order (every lookup kernel -- standalone, fused head,
// fused encoder -- uses this, so they agree bit for bit whatever the compiler contracts elsewhere)
__device__ __forceinline__ float lerp_tap(float v0, float v1, float a) { return __fmaf_rn(a, v1, __fmul_rn(1.f - a, v0)); }

__global__ __launch_bounds__(256) void corr_pyramid_kernel(const f16* __restrict__ f1,
                                                           const f16* __restrict__ f2, int stride,
                                                           int H, int W1, int W2, int C,
                                                           int levels, long lvl_off1,
                                                           long lvl_off2, long lvl_off3,
                                                           float* __restrict__ pyr) {
  extern __shared__ __attribute__((aligned(16))) float slab[];  // [CORR_ROWS][W2+1]
  const int bh = blockIdx.x;  // b*H + h
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int SW = W2 + 1;
  const f16* r1 = f1 + (long)bh * W1 * stride;
  const f16* r2 = f2 + (long)bh * W2 * stride;
  const float inv = rsqrtf((float)C);
  const int nct = (W2 + 15) / 16;
  const half8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
  long lvl_off[4] = {0, lvl_off1, lvl_off2, lvl_off3};

  // slabs of this row: blockIdx.y, +gridDim.y, ... (small frames split a row's slabs over workgroups)
  for (int w1b = blockIdx.y * CORR_ROWS; w1b < W1; w1b += gridDim.y * CORR_ROWS) {
    const int ntiles = (CORR_ROWS / 16) * nct;
    for (int t = wave; t < ntiles; t += 4) {
      const int tr = t / nct, tc = t % nct;
      const int a_row = w1b + tr * 16 + (lane & 15);
      const int b_row = tc * 16 + (lane & 15);
      const int kofs = (lane >> 4) * 8;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < C; k += 32) {
        half8 a = a_row < W1 ? *reinterpret_cast<const half8*>(r1 + (long)a_row * stride + k + kofs)
                             : zero8;
        half8 b = b_row < W2 ? *reinterpret_cast<const half8*>(r2 + (long)b_row * stride + k + kofs)
                             : zero8;
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = tr * 16 + (lane >> 4) * 4 + r;
        int col = tc * 16 + (lane & 15);
        if (col < W2) slab[row * SW + col] = acc[r] * inv;
      }
    }
    __syncthreads();
    // write level 0 and pooled levels for rows of this slab
    const int rows = min(CORR_ROWS, W1 - w1b);
    int Wl = W2;
    for (int l = 0; l < levels; ++l) {
      const int f = 1 << l;
      float* dst = pyr + lvl_off[l] + ((long)bh * W1 + w1b) * Wl;
      const float invf = 1.f / (float)f;
      for (int i = threadIdx.x; i < rows * Wl; i += 256) {
        int r = i / Wl, j = i - r * Wl;
        const float* s = slab + r * SW + j * f;
        float acc = 0.f;
        for (int t = 0; t < f; ++t) acc += s[t];
        dst[(long)r * Wl + j] = acc * invf;
      }
      Wl >>= 1;
    }
    __syncthreads();
  }
}

__global__ void corr_lookup_kernel(const float* __restrict__ pyr, const float* __restrict__ flow,
                                   int total, int W1, int W2, int levels, int radius,
                                   long lvl_off1, long lvl_off2, long lvl_off3,
                                   f16* __restrict__ out, int out_stride, int out_channels,
                                   f16* __restrict__ fout, int fstride, int fch,
                                   f16* __restrict__ fout2, int fstride2) {
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= total) return;
  const int w1 = pix % W1;
  const float fx = flow[pix];
  const float x = (float)w1 + fx;
  const int ntap = 2 * radius + 1;
  long lvl_off[4] = {0, lvl_off1, lvl_off2, lvl_off3};
  float vals[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) vals[i] = 0.f;
  int Wl = W2;
  for (int l = 0; l < levels; ++l) {
    const float* row = pyr + lvl_off[l] + (long)pix * Wl;
    const float xl = x / (float)(1 << l) - (float)radius;
    const float x0f = floorf(xl);
    const float a = xl - x0f;
    const int x0 = (int)x0f;
    float prev = (x0 >= 0 && x0 < Wl) ? row[x0] : 0.f;
    for (int k = 0; k < ntap; ++k) {
      int xi = x0 + k + 1;
      float nxt = (xi >= 0 && xi < Wl) ? row[xi] : 0.f;
      vals[l * ntap + k] = lerp_tap(prev, nxt, a);
      prev = nxt;
    }
    Wl >>= 1;
  }
  f16* op = out + (long)pix * out_stride;
  for (int c = 0; c < out_channels; c += 8) {
    half8 h;
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] = (f16)((c + j) < 64 ? vals[(c + j) & 63] : 0.f);
    *reinterpret_cast<half8*>(op + c) = h;
  }
  if (fout) {
    f16* fp = fout + (long)pix * fstride;
    for (int c = 0; c < fch; c += 8) {
      half8 h = {0, 0, 0, 0, 0, 0, 0, 0};
      if (c == 0) h[0] = (f16)fx;
      *reinterpret_cast<half8*>(fp + c) = h;
    }
  }
  if (fout2) {
    f16* fp = fout2 + (long)pix * fstride2;
    fp[0] = (f16)fx;
    fp[1] = (f16)0.f;
  }
}

// RAFT-Stereo motion-encoder head fused with the correlation lookup (SURVEY.md §7.2 "corr-lookup +
// convc1"): for 64 pixels per block, wave l computes pyramid level l's 2r+1 bilinear taps into LDS,
// then wave q produces output channels [16q, 16q+16) of
//   cor1 = relu(convc1(corr))      (1x1, levels*(2r+1) -> 64)
//   flo1 = relu(convf1(flow))      (7x7, 2 -> 64; the y flow is identically 0 in RAFT-Stereo, so only
//                                   the x-channel taps are applied)
// and wave 0 also writes the [flow_x, 0] tail of the motion features.  Weights are fp32 [k][64]
// (k-major, so a wave's 16 outputs of one k are one scalar load); the corr features never leave
// the chip and three launches per GRU iteration become one.
// MFMA form: the block's 64 pixels become a [64 x 96] fp16 A tile in LDS (k < nc:
// the bilinear correlation taps, wave l gathering level l; nc <= k < nc + 49: the 7x7 flow_x taps, 13
// per wave; rest zero) and both 1x1 / 7x7 convs are ONE GEMM against a block-diagonal [96 x 128]
// B (cols 0-63 convc1 on the corr rows, 64-127 convf1 on the flow rows), 6 fp16 B fragments per wave
// built from the fp32 weights, 24 v_mfma_f32_16x16x32_f16 per wave.  The relu'd fp16 outputs are
// staged through LDS for 16-B coalesced stores.  Operands are fp16 like every other conv input.
__global__ __launch_bounds__(256) void raft_motion_head_mfma_kernel(
    const float* __restrict__ pyr, const float* __restrict__ flow, int total, int H, int W1, int W2,
    int levels, int radius, long lvl_off1, long lvl_off2, long lvl_off3, const float* __restrict__ wc,
    const float* __restrict__ bc, const float* __restrict__ wf, const float* __restrict__ bf,
    f16* __restrict__ cor, int cstride, f16* __restrict__ flo, int fstride, f16* __restrict__ fcopy,
    int fcstride) {
  constexpr int KP = 96, AS = KP + 8, CS = 128 + 8;
  __shared__ __attribute__((aligned(16))) f16 a_s[64 * AS];
  __shared__ __attribute__((aligned(16))) f16 c_s[64 * CS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pixi = blockIdx.x * 64 + lane;
  const long pix = pixi;
  const bool ok = pixi < total;
  const int ntap = 2 * radius + 1, nc = levels * ntap;
  const int w1 = ok ? pixi % W1 : 0;
  const int y = ok ? (pixi / W1) % H : 0;
  const float fx = ok ? flow[pix] : 0.f;
  f16* arow = a_s + lane * AS;
  if (q < levels) {
    const long off = q == 0 ? 0 : (q == 1 ? lvl_off1 : (q == 2 ? lvl_off2 : lvl_off3));
    const int Wl = W2 >> q;
    const float* row = pyr + off + pix * Wl;
    const float xl = ((float)w1 + fx) / (float)(1 << q) - (float)radius;
    const float x0f = floorf(xl);
    const float a = xl - x0f;
    const int x0 = (int)x0f;
    float prev = (ok && x0 >= 0 && x0 < Wl) ? row[x0] : 0.f;
    for (int k = 0; k < ntap; ++k) {
      const int xi = x0 + k + 1;
      const float nxt = (ok && xi >= 0 && xi < Wl) ? row[xi] : 0.f;
      arow[q * ntap + k] = (f16)lerp_tap(prev, nxt, a);
      prev = nxt;
    }
  }
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const int t = q * 13 + i;
    if (t < 49) {
      const int ky = t / 7, kx = t - ky * 7;
      const bool tok = ok && (unsigned)(y + ky - 3) < (unsigned)H && (unsigned)(w1 + kx - 3) < (unsigned)W1;
      arow[nc + t] = (f16)(tok ? flow[pix + (long)(ky - 3) * W1 + (kx - 3)] : 0.f);
    }
  }
  if (q == 3)
    for (int k = nc + 49; k < KP; ++k) arow[k] = (f16)0.f;
  __syncthreads();

  const int r16 = lane & 15, kofs = (lane >> 4) * 8;
  half8 bfr[2][3];
  float bias[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = 32 * q + 16 * j + r16;
    bias[j] = n < 64 ? bc[n] : bf[n - 64];
#pragma unroll
    for (int ks = 0; ks < 3; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = ks * 32 + kofs + e;
        float v = 0.f;
        if (n < 64) {
          if (k < nc) v = wc[k * 64 + n];
        } else if (k >= nc && k < nc + 49) {
          v = wf[(k - nc) * 64 + (n - 64)];
        }
        bfr[j][ks][e] = (f16)v;
      }
  }
  floatx4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 3; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const half8 a = *reinterpret_cast<const half8*>(a_s + (16 * i + r16) * AS + ks * 32 + kofs);
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bfr[j][ks], acc[i][j], 0, 0, 0);
    }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * i + (lane >> 4) * 4 + r;
        const int col = 32 * q + 16 * j + r16;
        c_s[row * CS + col] = (f16)fmaxf(acc[i][j][r] + bias[j], 0.f);
      }
  __syncthreads();
  for (int c = tid; c < 64 * 16; c += 256) {
    const int row = c >> 4, ch = (c & 15) * 8;
    const int p = blockIdx.x * 64 + row;
    if (p < total) {
      const half8 v = *reinterpret_cast<const half8*>(c_s + row * CS + ch);
      if (ch < 64) *reinterpret_cast<half8*>(cor + (long)p * cstride + ch) = v;
      else *reinterpret_cast<half8*>(flo + (long)p * fstride + (ch - 64)) = v;
    }
  }
  if (q == 0 && ok && fcopy) {
    fcopy[pix * fcstride] = (f16)fx;
    fcopy[pix * fcstride + 1] = (f16)0.f;
  }
}

}  // namespace

extern "C" int sa_corr1d_pyramid(const void* f1, const void* f2, int stride, int B, int H, int W1,
                                 int W2, int C, int levels, float* pyr, hipStream_t stream) {
  if (C % 32 || levels < 1 || levels > 4) return -2;
  long off[4] = {0, 0, 0, 0};
  long acc = 0;
  int Wl = W2;
  for (int l = 0; l < levels; ++l) {
    off[l] = acc;
    acc += (long)B * H * W1 * Wl;
    Wl >>= 1;
  }
  size_t smem = (size_t)CORR_ROWS * (W2 + 1) * sizeof(float);
  if (smem > 160 * 1024) return -3;
  // one workgroup per image row fills the chip at batch 8 (960 rows); at batch 1 (120 rows) the row's 32-row
  // slabs go to separate workgroups (each re-reads the row's right features from L2)
  const int nslab = (W1 + CORR_ROWS - 1) / CORR_ROWS;
  const int split = B * H >= 512 ? 1 : nslab;
  hipLaunchKernelGGL(corr_pyramid_kernel, dim3(B * H, split), dim3(256), smem, stream, (const f16*)f1,
                     (const f16*)f2, stride, H, W1, W2, C, levels, off[1], off[2], off[3], pyr);
  return (int)hipGetLastError();
}

extern "C" int sa_corr1d_lookup(const float* pyr, const float* flow, int B, int H, int W1, int W2,
                                int levels, int radius, void* out, int out_stride,
                                int out_channels, void* flow_out, int flow_stride,
                                int flow_channels, void* flow_out2, int flow_stride2,
                                hipStream_t stream) {
  if (levels < 1 || levels > 4 || levels * (2 * radius + 1) > 64 || out_channels % 8 ||
      out_channels < levels * (2 * radius + 1))
    return -2;
  long off[4] = {0, 0, 0, 0};
  long acc = 0;
  int Wl = W2;
  for (int l = 0; l < levels; ++l) {
    off[l] = acc;
    acc += (long)B * H * W1 * Wl;
    Wl >>= 1;
  }
  int total = B * H * W1;
  hipLaunchKernelGGL(corr_lookup_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, pyr, flow,
                     total, W1, W2, levels, radius, off[1], off[2], off[3], (f16*)out, out_stride,
                     out_channels, (f16*)flow_out, flow_stride, flow_channels, (f16*)flow_out2,
                     flow_stride2);
  return (int)hipGetLastError();
}

extern "C" int sa_raft_motion_head(const float* pyr, const float* flow, int B, int H, int W1, int W2, int levels,
                                   int radius, const float* wc, const float* bc, const float* wf, const float* bf,
                                   void* cor, int cstride, void* flo, int fstride, void* fcopy, int fcstride,
                                   hipStream_t stream) {
  if (levels < 1 || levels > 4 || levels * (2 * radius + 1) > 36 || cstride % 8 || fstride % 8) return -2;
  long off[4] = {0, 0, 0, 0};
  long acc = 0;
  int Wl = W2;
  for (int l = 0; l < levels; ++l) {
    off[l] = acc;
    acc += (long)B * H * W1 * Wl;
    Wl >>= 1;
  }
  if ((long)B * H * W1 >= (1L << 31) - 64) return -2;
  const int total = B * H * W1;
  if (((uintptr_t)cor | (uintptr_t)flo) & 15) return -2;
  hipLaunchKernelGGL(raft_motion_head_mfma_kernel, dim3((total + 63) / 64),
                     dim3(256), 0, stream, pyr, flow, total, H, W1, W2, levels, radius, off[1], off[2], off[3], wc,
                     bc, wf, bf, (f16*)cor, cstride, (f16*)flo, fstride, (f16*)fcopy, fcstride);
  return (int)hipGetLastError();
}
