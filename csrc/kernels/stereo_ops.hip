// Model-specific stereo kernels for CREStereo / Fast-ACVNet+ / HITNet (NHWC; fp16 features, fp32
// flow / disparity state).
//
//   * sa_agcl_corr        — CREStereo Adaptive Group Correlation (4 channel groups x 9 taps, 1x9 or
//                           3x3 window; "iter" mode warps the right features by the flow and takes
//                           the window with replicate padding, "offset" mode samples the right
//                           features at flow + window + learned offset with zero padding)
//   * sa_linear_attention — LoFTR linear attention (ELU+1 kernel, fp32 math): per-64-token-chunk partial
//                           KV / Ksum, then per-64-token-tile outputs summing the partials in order
//   * sa_layernorm        — row LayerNorm with optional residual add
//   * sa_ew               — elementwise activation / scale / add of channel slices (+ broadcast
//                           addend, e.g. a positional encoding)
//   * sa_flow_features    — fp32 flow -> fp16 motion-encoder inputs (concat-free)
//   * sa_interp_flow      — fp32 multi-channel bilinear resize (align_corners) with scale
// Upstream ops: SURVEY.md §2.6 (grid_sample / local group correlation / linear attention rows).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <hip/hip_fp16.h>

#include "sa/kernels.h"

namespace {
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

inline int grid_for(long work, int block = 256) {
  long g = (work + block - 1) / block;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  return (int)g;
}

// ------------------------------------------------------------------ AGCL correlation
// one thread per (pixel, group, tap); the 64 channels of the group are read as 8 half8 vectors
__global__ void agcl_kernel(const SaAgclArgs a) {
  const int ntap = 9, G = 4;
  const long total = (long)a.N * a.H * a.W * G * ntap;
  const int Cg = a.C / G;
  const int px = a.small_patch ? 3 : 9, py = a.small_patch ? 3 : 1;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    // 32-bit index decomposition (total < 2^31, host-checked): the 64-bit div / mod chain is an emulated
    // sequence per element
    const unsigned ii = (unsigned)i;
    const int k = (int)(ii % (unsigned)ntap);
    const unsigned q = ii / (unsigned)ntap;
    const int g = (int)(q % (unsigned)G);
    const unsigned pixu = q / (unsigned)G;
    const long pix = (long)pixu;
    const int w = (int)(pixu % (unsigned)a.W);
    const unsigned hw = pixu / (unsigned)a.W;
    const int h = (int)(hw % (unsigned)a.H);
    const int n = (int)(hw / (unsigned)a.H);
    const int dx = k % px - px / 2, dy = k / px - py / 2;
    float sx, sy;
    if (a.iter_mode) {
      int hh = h + dy, ww = w + dx;
      hh = hh < 0 ? 0 : (hh >= a.H ? a.H - 1 : hh);
      ww = ww < 0 ? 0 : (ww >= a.W ? a.W - 1 : ww);
      const float* f = a.flow + (((long)n * a.H + hh) * a.W + ww) * 2;
      sx = (float)ww + f[0];
      sy = (float)hh + f[1];
    } else {
      const float* f = a.flow + pix * 2;
      sx = (float)w + f[0] + (float)dx;
      sy = (float)h + f[1] + (float)dy;
      if (a.offset) {
        const f16* o = reinterpret_cast<const f16*>(a.offset) + pix * a.offset_stride + k * 2;
        sx += (float)o[0];
        sy += (float)o[1];
      }
    }
    const float x0f = floorf(sx), y0f = floorf(sy);
    const int x0 = (int)x0f, y0 = (int)y0f;
    const float ax = sx - x0f, ay = sy - y0f;
    const f16* lp = reinterpret_cast<const f16*>(a.f1) + pix * a.f1_stride + g * Cg;
    float acc = 0.f;
    const float wts[4] = {(1.f - ax) * (1.f - ay), ax * (1.f - ay), (1.f - ax) * ay, ax * ay};
    const bool finite = isfinite(sx) && isfinite(sy);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int xx = x0 + (t & 1), yy = y0 + (t >> 1);
      if (!finite || xx < 0 || xx >= a.W || yy < 0 || yy >= a.H || wts[t] == 0.f) continue;
      const f16* rp = reinterpret_cast<const f16*>(a.f2) + (((long)n * a.H + yy) * a.W + xx) * a.f2_stride + g * Cg;
      float s = 0.f;
      for (int c = 0; c < Cg; c += 8) {
        const half8 l8 = *reinterpret_cast<const half8*>(lp + c);
        const half8 r8 = *reinterpret_cast<const half8*>(rp + c);
        typedef _Float16 half2v __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int j = 0; j < 8; j += 2)  // fp16 pairs, fp32 accumulation (v_dot2_f32_f16)
          s = __builtin_amdgcn_fdot2(half2v{l8[j], l8[j + 1]}, half2v{r8[j], r8[j + 1]}, s, false);
      }
      acc += wts[t] * s;
    }
    reinterpret_cast<f16*>(a.out)[pix * a.out_stride + g * ntap + k] = (f16)(acc / (float)Cg);
  }
}

// Same op, 8 lanes per (pixel, group, tap): lane c8 owns channels 8*c8 .. +8 of the group's 64, so the left chunk
// and each bilinear corner's right chunk are one contiguous 128-B line per 8 lanes (the one-thread-per-tap kernel
// above issues 8 scattered 16-B loads per line and per thread); the 8 partial dot products are summed with DPP.
// Needs C / 4 == 64 channels per group (CREStereo: C = 256 at every level).
__global__ void agcl8_kernel(const SaAgclArgs a) {
  constexpr int ntap = 9, G = 4, CG = 64;
  const unsigned total = (unsigned)a.N * a.H * a.W * G * ntap;
  const int px = a.small_patch ? 3 : 9, py = a.small_patch ? 3 : 1;
  const int c8 = threadIdx.x & 7;
  typedef _Float16 half2v __attribute__((ext_vector_type(2)));
  for (unsigned ii = (blockIdx.x * (unsigned)blockDim.x + threadIdx.x) >> 3; ii < total;
       ii += (gridDim.x * (unsigned)blockDim.x) >> 3) {
    const int k = (int)(ii % (unsigned)ntap);
    const unsigned q = ii / (unsigned)ntap;
    const int g = (int)(q % (unsigned)G);
    const unsigned pixu = q / (unsigned)G;
    const long pix = (long)pixu;
    const int w = (int)(pixu % (unsigned)a.W);
    const unsigned hw = pixu / (unsigned)a.W;
    const int h = (int)(hw % (unsigned)a.H);
    const int n = (int)(hw / (unsigned)a.H);
    const int dx = k % px - px / 2, dy = k / px - py / 2;
    float sx, sy;
    if (a.iter_mode) {
      int hh = h + dy, ww = w + dx;
      hh = hh < 0 ? 0 : (hh >= a.H ? a.H - 1 : hh);
      ww = ww < 0 ? 0 : (ww >= a.W ? a.W - 1 : ww);
      const float* f = a.flow + (((long)n * a.H + hh) * a.W + ww) * 2;
      sx = (float)ww + f[0];
      sy = (float)hh + f[1];
    } else {
      const float* f = a.flow + pix * 2;
      sx = (float)w + f[0] + (float)dx;
      sy = (float)h + f[1] + (float)dy;
      if (a.offset) {
        const f16* o = reinterpret_cast<const f16*>(a.offset) + pix * a.offset_stride + k * 2;
        sx += (float)o[0];
        sy += (float)o[1];
      }
    }
    const float x0f = floorf(sx), y0f = floorf(sy);
    const int x0 = (int)x0f, y0 = (int)y0f;
    const float ax = sx - x0f, ay = sy - y0f;
    const half8 l8 = *reinterpret_cast<const half8*>(reinterpret_cast<const f16*>(a.f1) + pix * a.f1_stride + g * CG +
                                                     c8 * 8);
    float acc = 0.f;
    const float wts[4] = {(1.f - ax) * (1.f - ay), ax * (1.f - ay), (1.f - ax) * ay, ax * ay};
    const bool finite = isfinite(sx) && isfinite(sy);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int xx = x0 + (t & 1), yy = y0 + (t >> 1);
      if (!finite || xx < 0 || xx >= a.W || yy < 0 || yy >= a.H || wts[t] == 0.f) continue;
      const half8 r8 = *reinterpret_cast<const half8*>(reinterpret_cast<const f16*>(a.f2) +
                                                       (((long)n * a.H + yy) * a.W + xx) * a.f2_stride + g * CG + c8 * 8);
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; j += 2)
        s = __builtin_amdgcn_fdot2(half2v{l8[j], l8[j + 1]}, half2v{r8[j], r8[j + 1]}, s, false);
      acc += wts[t] * s;
    }
    // sum over the 8 lanes of this tap (quad_perm xor 1, xor 2, then row_ror 4 within the 8-lane half-row)
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    if (c8 == 0) reinterpret_cast<f16*>(a.out)[pix * a.out_stride + g * ntap + k] = (f16)(acc / (float)CG);
  }
}

// Same op, one wave per pixel: lane l holds channels 4l .. 4l+3 of the 256 (group l >> 4), so the left features are
// read once per pixel (agcl8 re-reads them for each of the 9 taps) and every corner of a tap is one coalesced 512-B
// row of the right features.  In the plain window modes (no learned offsets, not iter mode) the 9 taps share their
// bilinear corners -- a 1x9 window touches 2 rows x 10 columns, a 3x3 one 4 x 4 -- so those are loaded once into
// registers and reused (36 corner rows -> 20 / 16).  Per-tap group sums: xor shuffles inside the 16 lanes of a
// group; lane 16g + k stores tap k of group g.
// SPX: 0 = per-tap corners (offset / iter modes), 9 = shared 1 x 9 window, 3 = shared 3 x 3 window
template <int SPX>
__global__ __launch_bounds__(256) void agclw_kernel(const SaAgclArgs a) {
  constexpr bool SHARED = SPX != 0;
  constexpr int ntap = 9;
  typedef _Float16 half4 __attribute__((ext_vector_type(4)));
  typedef _Float16 half2v __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long P = (long)a.N * a.H * a.W;
  const long pix = (long)blockIdx.x * 4 + wave;
  if (pix >= P) return;
  const int w = (int)(pix % a.W);
  const long hw = pix / a.W;
  const int h = (int)(hw % a.H);
  const int n = (int)(hw / a.H);
  const int px = SHARED ? SPX : (a.small_patch ? 3 : 9), py = SHARED ? (SPX == 3 ? 3 : 1) : (a.small_patch ? 3 : 1);
  const half4 l4 = *reinterpret_cast<const half4*>(reinterpret_cast<const f16*>(a.f1) + pix * a.f1_stride + lane * 4);
  const f16* f2 = reinterpret_cast<const f16*>(a.f2) + (long)n * a.H * a.W * a.f2_stride + lane * 4;
  auto dot4 = [&](const half4 r) {
    float s = __builtin_amdgcn_fdot2(half2v{l4[0], l4[1]}, half2v{r[0], r[1]}, 0.f, false);
    return __builtin_amdgcn_fdot2(half2v{l4[2], l4[3]}, half2v{r[2], r[3]}, s, false);
  };
  auto corner = [&](int xx, int yy) -> float {  // zero padding outside the image
    if (xx < 0 || xx >= a.W || yy < 0 || yy >= a.H) return 0.f;
    return dot4(*reinterpret_cast<const half4*>(f2 + ((long)yy * a.W + xx) * a.f2_stride));
  };
  float res = 0.f;  // lane 16 g + k keeps tap k of group g
  auto emit = [&](int k, float v) {
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    if ((lane & 15) == k) res = v;
  };
  if constexpr (SHARED) {
    // sample (w + f + dx, h + f + dy): one fractional part for every tap
    const float* f = a.flow + pix * 2;
    const float sx0 = (float)w + f[0] - (float)(px / 2), sy0 = (float)h + f[1] - (float)(py / 2);
    const bool finite = isfinite(sx0) && isfinite(sy0);
    const float x0f = finite ? floorf(sx0) : 0.f, y0f = finite ? floorf(sy0) : 0.f;
    const int x0 = (int)x0f, y0 = (int)y0f;
    const float ax = sx0 - x0f, ay = sy0 - y0f;
    // corner dot products of the (py + 1) x (px + 1) patch, row by row (each row's px + 1 corners once)
    constexpr int PX = SPX, PY = SPX == 3 ? 3 : 1;
    float prev[PX + 1];
#pragma unroll
    for (int r = 0; r <= PY; ++r) {
      float cur[PX + 1];
#pragma unroll
      for (int c = 0; c <= PX; ++c) cur[c] = finite ? corner(x0 + c, y0 + r) : 0.f;
      if (r > 0) {
#pragma unroll
        for (int c = 0; c < PX; ++c) {
          const float v = (1.f - ay) * ((1.f - ax) * prev[c] + ax * prev[c + 1]) + ay * ((1.f - ax) * cur[c] + ax * cur[c + 1]);
          emit((r - 1) * PX + c, v);
        }
      }
#pragma unroll
      for (int c = 0; c <= PX; ++c) prev[c] = cur[c];
    }
  } else {
#pragma unroll
    for (int k = 0; k < ntap; ++k) {
      const int dx = k % px - px / 2, dy = k / px - py / 2;
      float sx, sy;
      if (a.iter_mode) {
        int hh = h + dy, ww = w + dx;
        hh = hh < 0 ? 0 : (hh >= a.H ? a.H - 1 : hh);
        ww = ww < 0 ? 0 : (ww >= a.W ? a.W - 1 : ww);
        const float* f = a.flow + (((long)n * a.H + hh) * a.W + ww) * 2;
        sx = (float)ww + f[0];
        sy = (float)hh + f[1];
      } else {
        const float* f = a.flow + pix * 2;
        sx = (float)w + f[0] + (float)dx;
        sy = (float)h + f[1] + (float)dy;
        if (a.offset) {
          const f16* o = reinterpret_cast<const f16*>(a.offset) + pix * a.offset_stride + k * 2;
          sx += (float)o[0];
          sy += (float)o[1];
        }
      }
      float v = 0.f;
      if (isfinite(sx) && isfinite(sy)) {
        const float x0f = floorf(sx), y0f = floorf(sy);
        const int x0 = (int)x0f, y0 = (int)y0f;
        const float ax = sx - x0f, ay = sy - y0f;
        v = (1.f - ay) * ((1.f - ax) * corner(x0, y0) + ax * corner(x0 + 1, y0)) +
            ay * ((1.f - ax) * corner(x0, y0 + 1) + ax * corner(x0 + 1, y0 + 1));
      }
      emit(k, v);
    }
  }
  if ((lane & 15) < ntap)
    reinterpret_cast<f16*>(a.out)[pix * a.out_stride + (lane >> 4) * ntap + (lane & 15)] = (f16)(res * (1.f / 64.f));
}

// Iter mode, tiled (the CREStereo refinement hot path: agcl8 above spends 43 us per 1/4-scale b1 iteration because
// every one of the 9 taps recomputes the flow lookup and the 4 bilinear corners of its neighbour, i.e. each warped
// right pixel is rebuilt 9 times).  Here one workgroup owns a TH x TW output tile and one 64-channel group
// (blockIdx.y): phase 1 warps the tile plus its window halo once into LDS in fp32 (halo positions clamped to the
// image = the replicate padding of the warped map; zero outside the right image, non-finite samples give zero),
// phase 2 takes the 9 window dot products per output pixel from LDS.  8 lanes per pixel own 8 channels each; the
// 16-B chunk j of LDS pixel p is stored at chunk j ^ (p & 1), so the 16-lane groups of a ds_read_b128 (4 pixels of
// alternating parity) hit 16 distinct 16-B bank slots.  The 9 per-lane partial sums are reduce-scattered across the 8
// lanes (7 + 3 shuffles instead of 27): lane c8 ends with tap c8, lane 0 also with tap 8.
// RX, RY: window half-widths (1x9: 4, 0; 3x3: 1, 1).
template <int RX, int RY>
__global__ __launch_bounds__(256) void agcl_iter_tile_kernel(const SaAgclArgs a) {
  constexpr int TW = 32, TH = 4, HWX = TW + 2 * RX, HP = HWX * (TH + 2 * RY);
  constexpr int PX = 2 * RX + 1;
  static_assert(PX * (2 * RY + 1) == 9, "9-tap window");
  __shared__ float4 warped[HP][16];
  const int tid = threadIdx.x, c8 = tid & 7, slot = tid >> 3;
  const int g = blockIdx.y;
  const int tiles_x = (a.W + TW - 1) / TW, tiles_y = (a.H + TH - 1) / TH;
  const int bt = blockIdx.x;
  const int tx = bt % tiles_x, ty = (bt / tiles_x) % tiles_y, n = bt / (tiles_x * tiles_y);
  const int x0 = tx * TW - RX, y0 = ty * TH - RY;
  const long img = (long)n * a.H * a.W;
  const f16* f2 = reinterpret_cast<const f16*>(a.f2) + img * a.f2_stride + g * 64 + c8 * 8;
  // Everything is issued before anything is consumed (the kernel is latency-bound: one flow load -> four dependent
  // corner loads per pixel, a few pixels per lane): the flows of all this lane's halo pixels and the left chunks of
  // its phase-2 pixels first, then the corners four pixels (16 loads) at a time.
  constexpr int NPI = (HP + 31) / 32, NQ = TH * TW / 32;
  float2 fl[NPI];
  int hw_[NPI];
#pragma unroll
  for (int i = 0; i < NPI; ++i) {
    const int p = slot + 32 * i < HP ? slot + 32 * i : HP - 1;
    int hh = y0 + p / HWX, ww = x0 + p % HWX;
    hh = hh < 0 ? 0 : (hh >= a.H ? a.H - 1 : hh);
    ww = ww < 0 ? 0 : (ww >= a.W ? a.W - 1 : ww);
    hw_[i] = (hh << 16) | ww;
    fl[i] = *reinterpret_cast<const float2*>(a.flow + (img + (long)hh * a.W + ww) * 2);
  }
  half8 lf[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = slot + 32 * i;
    const int h = ty * TH + q / TW, w = tx * TW + q % TW;
    if (h < a.H && w < a.W)
      lf[i] = *reinterpret_cast<const half8*>(reinterpret_cast<const f16*>(a.f1) + (img + (long)h * a.W + w) * a.f1_stride +
                                              g * 64 + c8 * 8);
    else
      lf[i] = half8{};
  }
#pragma unroll
  for (int i0 = 0; i0 < NPI; i0 += 4) {
    constexpr int CH = 4;
    half8 rv[CH][4];
    float wv[CH][4];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if (i0 + j >= NPI) break;
      const int i = i0 + j;
      const float sx = (float)(hw_[i] & 0xffff) + fl[i].x, sy = (float)(hw_[i] >> 16) + fl[i].y;
      const bool fin = isfinite(sx) && isfinite(sy);
      const float xf = fin ? floorf(sx) : 0.f, yf = fin ? floorf(sy) : 0.f;
      const int xi = (int)xf, yi = (int)yf;
      const float ax = sx - xf, ay = sy - yf;
      const float wts[4] = {(1.f - ax) * (1.f - ay), ax * (1.f - ay), (1.f - ax) * ay, ax * ay};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int xx = xi + (t & 1), yy = yi + (t >> 1);
        const bool ok = fin && xx >= 0 && xx < a.W && yy >= 0 && yy < a.H && wts[t] != 0.f;
        wv[j][t] = ok ? wts[t] : 0.f;
        if (ok) rv[j][t] = *reinterpret_cast<const half8*>(f2 + ((long)yy * a.W + xx) * a.f2_stride);
        else rv[j][t] = half8{};
      }
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if (i0 + j >= NPI) break;
      const int p = slot + 32 * (i0 + j);
      float acc[8];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        acc[e] = wv[j][0] * (float)rv[j][0][e] + wv[j][1] * (float)rv[j][1][e] + wv[j][2] * (float)rv[j][2][e] +
                 wv[j][3] * (float)rv[j][3][e];
      if (p < HP) {
        const int s = p & 1;
        warped[p][(2 * c8) ^ s] = float4{acc[0], acc[1], acc[2], acc[3]};
        warped[p][(2 * c8 + 1) ^ s] = float4{acc[4], acc[5], acc[6], acc[7]};
      }
    }
  }
  __syncthreads();
  const bool b2 = c8 & 4, b1 = c8 & 2, b0 = c8 & 1;
#pragma unroll
  for (int iq = 0; iq < NQ; ++iq) {
    const int q = slot + 32 * iq;
    const int oy = q / TW, ox = q % TW;
    const int h = ty * TH + oy, w = tx * TW + ox;
    if (h >= a.H || w >= a.W) continue;  // uniform over the pixel's 8 lanes (the shuffles stay inside them)
    const long pix = img + (long)h * a.W + w;
    const half8 l8 = lf[iq];
    float l[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) l[j] = (float)l8[j];
    float r[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int dx = k % PX - RX, dy = k / PX - RY;
      const int p = (oy + RY + dy) * HWX + ox + RX + dx;
      const int s = p & 1;
      const float4 u = warped[p][(2 * c8) ^ s], v = warped[p][(2 * c8 + 1) ^ s];
      r[k] = l[0] * u.x + l[1] * u.y + l[2] * u.z + l[3] * u.w + l[4] * v.x + l[5] * v.y + l[6] * v.z + l[7] * v.w;
    }
    // reduce-scatter taps 0..7 over the 8 lanes: after the xor-4 / xor-2 / xor-1 steps lane c8 holds tap c8
    float r4[4], r2[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) r4[i] = (b2 ? r[i + 4] : r[i]) + __shfl_xor(b2 ? r[i] : r[i + 4], 4);
#pragma unroll
    for (int i = 0; i < 2; ++i) r2[i] = (b1 ? r4[i + 2] : r4[i]) + __shfl_xor(b1 ? r4[i] : r4[i + 2], 2);
    const float mine = (b0 ? r2[1] : r2[0]) + __shfl_xor(b0 ? r2[0] : r2[1], 1);
    float t8 = r[8];
    t8 += __shfl_xor(t8, 4);
    t8 += __shfl_xor(t8, 2);
    t8 += __shfl_xor(t8, 1);
    f16* o = reinterpret_cast<f16*>(a.out) + pix * a.out_stride + g * 9;
    o[c8] = (f16)(mine * (1.f / 64.f));
    if (c8 == 0) o[8] = (f16)(t8 * (1.f / 64.f));
  }
}

// Iter-mode AGCL fused with the motion encoder's convc1 (1x1, 36 -> 256, bias, relu): the CREStereo 1/4-scale
// chain ran AGCL (15-25 us) then a K = 36 GEMM whose tile prologue / epilogue cost 15-30 us for 0.4 GFLOP.  One
// workgroup (8 waves) owns a 2 x 32 pixel tile and all four channel groups:
//   phase 1  warps the tile + window halo once for all 256 channels into LDS as fp16 (32 lanes per pixel, lane cc
//            owns 16-B chunk cc; the halo replicate padding / zero outside / non-finite rules of the kernel above);
//   phase 2  lane (g, c8) of a pixel's 32 takes the 9 window dot products of group g over its 8 channels
//            (fp16 pairs, fp32 sums), reduce-scatters them over the group's 8 lanes and writes the fp16-rounded
//            correlation (the value the unfused path stores) into an LDS [64 px][36 + pad] A tile;
//   GEMM     [64 x 64] x [64 x 256] with v_mfma_f32_16x16x32_f16 (wave w: columns 32w..32w+31, weights as B
//            fragments straight from global memory), bias + relu, staged through LDS for 16-B stores.
// FL: the flow branch's first conv rides along -- convf1 (7x7, 2 -> 128, pad 3, bias, relu) over the fp16 flow of an
// 8 x 38 halo tile staged in LDS, as a second [64 x 128(98 taps)] x [128 x 128] MFMA GEMM, plus the fp16 copy of the
// flow the GRU input carries (xin[254:256]); the flow branch then needs no launch of its own before convf2.
// w16: [256][64] fp16 (k >= 36 zero), bias fp32 [256]; wf16: [128][128] fp16, k = c * 49 + ky * 7 + kx (k >= 98 zero).
// PRE: the correlation was computed by sa_agcl_corr (offset mode, the coarse levels) and is read from a.out
// (a.out_stride per pixel, 36 channels) instead of phases 1 / 2.
template <int RX, int RY, bool FL, bool PRE = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void agcl_iter_c1_kernel(
    const SaAgclArgs a, const SaCreHeadArgs hd) {
  const f16* __restrict__ w16 = reinterpret_cast<const f16*>(hd.w16);
  const float* __restrict__ bias = hd.bias;
  f16* __restrict__ out = reinterpret_cast<f16*>(hd.cor);
  const int out_stride = hd.cor_stride;
  constexpr int TW = 32, TH = 2, HWX = TW + 2 * RX, HP = HWX * (TH + 2 * RY), NPX = TH * TW;
  constexpr int PX = 2 * RX + 1;
  static_assert(PX * (2 * RY + 1) == 9, "9-tap window");
  constexpr int CRS = 72, OS = 256 + 8;
  constexpr int AFS = 136, FHW = TW + 6, FHP = (TH + 6) * FHW;  // convf1 A-tile row stride, flow halo width / size
  constexpr int WP_BYTES = PRE ? 0 : HP * 512, OST_BYTES = NPX * OS * 2, AF_BYTES = FL ? NPX * AFS * 2 : 0;
  constexpr int SMEM = WP_BYTES > OST_BYTES + AF_BYTES ? WP_BYTES : OST_BYTES + AF_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  __shared__ f16 fh[FL ? FHP * 2 : 2];
  __shared__ __attribute__((aligned(16))) f16 cr[NPX * CRS];
  __shared__ float2 spos[PRE ? 1 : HP];
  half8* wp = reinterpret_cast<half8*>(smem);  // [HP][32] 16-B chunks
  typedef _Float16 half2v __attribute__((ext_vector_type(2)));
  typedef float floatx4 __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, cc = tid & 31, ps = tid >> 5, c8 = tid & 7, g = (tid >> 3) & 3;
  const int tiles_x = (a.W + TW - 1) / TW, tiles_y = (a.H + TH - 1) / TH;
  const int bt = blockIdx.x;
  const int tx = bt % tiles_x, ty = (bt / tiles_x) % tiles_y, n = bt / (tiles_x * tiles_y);
  const int x0 = tx * TW - RX, y0 = ty * TH - RY;
  const long img = (long)n * a.H * a.W;
  const f16* f2 = reinterpret_cast<const f16*>(a.f2) + img * a.f2_stride + cc * 8;
  constexpr int NPI = (HP + 15) / 16, NQ = NPX / 16;
  // the halo's sample positions go through LDS (one flow load per halo pixel instead of one per lane and pixel)
  for (int p = tid; p < (PRE ? 0 : HP); p += 512) {
    int hh = y0 + p / HWX, ww = x0 + p % HWX;
    hh = hh < 0 ? 0 : (hh >= a.H ? a.H - 1 : hh);
    ww = ww < 0 ? 0 : (ww >= a.W ? a.W - 1 : ww);
    const float2 f = *reinterpret_cast<const float2*>(a.flow + (img + (long)hh * a.W + ww) * 2);
    spos[p] = float2{(float)ww + f.x, (float)hh + f.y};
  }
  if constexpr (FL) {
    // zero-padded fp16 flow around the tile for convf1, and the tile's own flow into the GRU input slice
    for (int p = tid; p < FHP; p += 512) {
      const int hh = ty * TH - 3 + p / FHW, ww = tx * TW - 3 + p % FHW;
      float2 f = float2{0.f, 0.f};
      if (hh >= 0 && hh < a.H && ww >= 0 && ww < a.W)
        f = *reinterpret_cast<const float2*>(a.flow + (img + (long)hh * a.W + ww) * 2);
      fh[2 * p] = (f16)f.x;
      fh[2 * p + 1] = (f16)f.y;
      const int r = p / FHW - 3, c = p % FHW - 3;
      if (r >= 0 && r < TH && c >= 0 && c < TW && hh < a.H && ww < a.W) {
        f16* fc = reinterpret_cast<f16*>(hd.fcopy) + (img + (long)hh * a.W + ww) * hd.fcopy_stride;
        fc[0] = (f16)f.x;
        fc[1] = (f16)f.y;
      }
    }
  }
  half8 lf[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    if constexpr (PRE) break;
    const int q = ps + 16 * i;
    const int h = ty * TH + q / TW, w = tx * TW + q % TW;
    if (h < a.H && w < a.W)
      lf[i] = *reinterpret_cast<const half8*>(reinterpret_cast<const f16*>(a.f1) + (img + (long)h * a.W + w) * a.f1_stride +
                                              cc * 8);
    else
      lf[i] = half8{};
  }
  for (int e = tid; e < NPX * (CRS - 36); e += 512) cr[(e / (CRS - 36)) * CRS + 36 + e % (CRS - 36)] = (f16)0.f;
  if constexpr (PRE) {
    for (int e = tid; e < NPX * 36; e += 512) {
      const int m = e / 36, kk = e - 36 * m;
      const int h = ty * TH + m / TW, w = tx * TW + m % TW;
      cr[m * CRS + kk] = h < a.H && w < a.W
                             ? reinterpret_cast<const f16*>(a.out)[(img + (long)h * a.W + w) * a.out_stride + kk]
                             : (f16)0.f;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i0 = 0; i0 < (PRE ? 0 : NPI); i0 += 4) {
    constexpr int CH = 4;
    half8 rv[CH][4];
    float wv[CH][4];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if (i0 + j >= NPI) break;
      const int i = i0 + j;
      const float2 sp = spos[ps + 16 * i < HP ? ps + 16 * i : HP - 1];
      const float sx = sp.x, sy = sp.y;
      const bool fin = isfinite(sx) && isfinite(sy);
      const float xf = fin ? floorf(sx) : 0.f, yf = fin ? floorf(sy) : 0.f;
      const int xi = (int)xf, yi = (int)yf;
      const float ax = sx - xf, ay = sy - yf;
      const float wts[4] = {(1.f - ax) * (1.f - ay), ax * (1.f - ay), (1.f - ax) * ay, ax * ay};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int xx = xi + (t & 1), yy = yi + (t >> 1);
        const bool ok = fin && xx >= 0 && xx < a.W && yy >= 0 && yy < a.H && wts[t] != 0.f;
        wv[j][t] = ok ? wts[t] : 0.f;
        if (ok) rv[j][t] = *reinterpret_cast<const half8*>(f2 + ((long)yy * a.W + xx) * a.f2_stride);
        else rv[j][t] = half8{};
      }
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if (i0 + j >= NPI) break;
      const int p = ps + 16 * (i0 + j);
      half8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        o[e] = (f16)(wv[j][0] * (float)rv[j][0][e] + wv[j][1] * (float)rv[j][1][e] + wv[j][2] * (float)rv[j][2][e] +
                     wv[j][3] * (float)rv[j][3][e]);
      if (p < HP) wp[p * 32 + cc] = o;
    }
  }
  __syncthreads();
  const bool b2 = c8 & 4, b1 = c8 & 2, b0 = c8 & 1;
#pragma unroll
  for (int iq = 0; iq < NQ; ++iq) {
    if constexpr (PRE) break;
    const int q = ps + 16 * iq;
    const int oy = q / TW, ox = q % TW;
    const half8 l8 = lf[iq];
    float r[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int dx = k % PX - RX, dy = k / PX - RY;
      const half8 v = wp[((oy + RY + dy) * HWX + ox + RX + dx) * 32 + cc];
      float acc = 0.f;
#pragma unroll
      for (int e = 0; e < 8; e += 2)
        acc = __builtin_amdgcn_fdot2(half2v{l8[e], l8[e + 1]}, half2v{v[e], v[e + 1]}, acc, false);
      r[k] = acc;
    }
    float r4[4], r2[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) r4[i] = (b2 ? r[i + 4] : r[i]) + __shfl_xor(b2 ? r[i] : r[i + 4], 4);
#pragma unroll
    for (int i = 0; i < 2; ++i) r2[i] = (b1 ? r4[i + 2] : r4[i]) + __shfl_xor(b1 ? r4[i] : r4[i + 2], 2);
    const float mine = (b0 ? r2[1] : r2[0]) + __shfl_xor(b0 ? r2[0] : r2[1], 1);
    float t8 = r[8];
    t8 += __shfl_xor(t8, 4);
    t8 += __shfl_xor(t8, 2);
    t8 += __shfl_xor(t8, 1);
    cr[q * CRS + g * 9 + c8] = (f16)(mine * (1.f / 64.f));
    if (c8 == 0) cr[q * CRS + g * 9 + 8] = (f16)(t8 * (1.f / 64.f));
  }
  __syncthreads();
  f16* af = reinterpret_cast<f16*>(smem + OST_BYTES);  // convf1 A tile [64 px][AFS] (the warped image is dead now)
  if constexpr (FL) {
#pragma unroll
    for (int j = 0; j < NPX * 128 / 512; ++j) {
      const int e = tid + 512 * j, m = e >> 7, kk = e & 127;
      f16 v = (f16)0.f;
      if (kk < 98) {
        const int c = kk >= 49, t = kk - 49 * c, ky = t / 7, kx = t - 7 * ky;
        v = fh[2 * ((m / TW + ky) * FHW + m % TW + kx) + c];
      }
      af[m * AFS + kk] = v;
    }
  }
  const int lane = tid & 63, wv = tid >> 6, r16 = lane & 15, kofs = (lane >> 4) * 8;
  half8 bfr[2][2];
  float bj[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nn = wv * 32 + 16 * j + r16;
    bj[j] = bias[nn];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) bfr[j][ks] = *reinterpret_cast<const half8*>(w16 + nn * 64 + ks * 32 + kofs);
  }
  floatx4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const half8 av = *reinterpret_cast<const half8*>(cr + (16 * i + r16) * CRS + ks * 32 + kofs);
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bfr[j][ks], acc[i][j], 0, 0, 0);
    }
  f16* ost = reinterpret_cast<f16*>(smem);  // phase 2's reads of wp all happened before the barrier above
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        ost[(16 * i + (lane >> 4) * 4 + rr) * OS + wv * 32 + 16 * j + r16] = (f16)fmaxf(acc[i][j][rr] + bj[j], 0.f);
  __syncthreads();
#pragma unroll
  for (int c = tid; c < NPX * 32; c += 512) {
    const int row = c >> 5, ch = (c & 31) * 8;
    const int h = ty * TH + row / TW, w = tx * TW + row % TW;
    if (h < a.H && w < a.W)
      *reinterpret_cast<half8*>(out + (img + (long)h * a.W + w) * out_stride + ch) =
          *reinterpret_cast<const half8*>(ost + row * OS + ch);
  }
  if constexpr (FL) {
    // convf1: wave w -> output columns 16w .. 16w + 15, all 64 rows, 4 k-steps over the 98 (128) taps
    const f16* wf = reinterpret_cast<const f16*>(hd.wf16);
    half8 bf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) bf[ks] = *reinterpret_cast<const half8*>(wf + (16 * wv + r16) * 128 + ks * 32 + kofs);
    const float fb = hd.fbias[16 * wv + r16];
    floatx4 a2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a2[i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const half8 av = *reinterpret_cast<const half8*>(af + (16 * i + r16) * AFS + ks * 32 + kofs);
        a2[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bf[ks], a2[i], 0, 0, 0);
      }
    f16* flo = reinterpret_cast<f16*>(hd.flo);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = 16 * i + (lane >> 4) * 4 + rr;
        const int h = ty * TH + row / TW, w = tx * TW + row % TW;
        if (h < a.H && w < a.W)
          flo[(img + (long)h * a.W + w) * hd.flo_stride + 16 * wv + r16] = (f16)fmaxf(a2[i][rr] + fb, 0.f);
      }
  }
}

__global__ void zero_tail_kernel(f16* out, int stride, long P, int c0, int c1) {
  const int n = c1 - c0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < P * n; i += (long)gridDim.x * blockDim.x)
    out[(i / n) * stride + c0 + (int)(i % n)] = (f16)0.f;
}

// ------------------------------------------------------------------ linear attention
// out[l][v] = sum_d phi(Q)[l][d] KV[d][v] / (sum_d phi(Q)[l][d] Ksum[d] + eps), KV[d][v] = sum_s phi(K)[s][d] V[s][v],
// Ksum[d] = sum_s phi(K)[s][d], phi = elu + 1, per (image, head) with head dim D.
// Two kernels over many workgroups (round 1 ran one workgroup per (image, head): 8-16 workgroups on 256 CUs,
// 0.6 ms per call): (1) one 64-token chunk of K / V per workgroup -> partial [KV | Ksum] into the workspace;
// (2) one 64-token tile of Q per workgroup sums the partials in chunk order (deterministic) and writes its
// outputs, phi(Q) computed once per element and staged in LDS.
constexpr int LA_CHUNK = 64;

template <int D>
__global__ __launch_bounds__(256) void linear_attn_kv_kernel(const f16* __restrict__ k, int ks, const f16* __restrict__ v,
                                                             int vs, int S, int heads, float* __restrict__ ws) {
  __shared__ float kt[LA_CHUNK][D + 1];
  __shared__ float vt[LA_CHUNK][D + 1];
  const int c = blockIdx.x, h = blockIdx.y, n = blockIdx.z, tid = threadIdx.x;
  const int nch = gridDim.x;
  const int s0 = c * LA_CHUNK, hoff = h * D;
  for (int e = tid; e < LA_CHUNK * D; e += 256) {
    const int s = e / D, d = e % D;
    float kk = 0.f, vv = 0.f;
    if (s0 + s < S) {
      const long row = (long)n * S + s0 + s;
      kk = (float)k[row * ks + hoff + d];
      kk = kk > 0.f ? kk + 1.f : __expf(kk);  // elu(x) + 1
      vv = (float)v[row * vs + hoff + d];
    }
    kt[s][d] = kk;
    vt[s][d] = vv;
  }
  __syncthreads();
  float* dst = ws + (((size_t)n * heads + h) * nch + c) * (D * D + D);
  for (int pidx = tid; pidx < D * D; pidx += 256) {
    const int d = pidx / D, vv = pidx % D;
    float a = 0.f;
#pragma unroll 8
    for (int s = 0; s < LA_CHUNK; ++s) a += kt[s][d] * vt[s][vv];
    dst[pidx] = a;
  }
  if (tid < D) {
    float a = 0.f;
    for (int s = 0; s < LA_CHUNK; ++s) a += kt[s][tid];
    dst[D * D + tid] = a;
  }
}

template <int D>
__global__ __launch_bounds__(256) void linear_attn_out_kernel(const f16* __restrict__ q, int qs, const float* __restrict__ ws,
                                                              int nch, int heads, f16* __restrict__ out, int os, int L,
                                                              float eps) {
  __shared__ float kv[D][D + 1];
  __shared__ float ksum[D];
  __shared__ float qt[LA_CHUNK][D + 1];
  const int t = blockIdx.x, h = blockIdx.y, n = blockIdx.z, tid = threadIdx.x;
  const int l0 = t * LA_CHUNK, hoff = h * D;
  const float* src = ws + ((size_t)n * heads + h) * nch * (D * D + D);
  // sum of the chunk partials, every load of a chunk issued before the adds (a serial c-loop left one L2 round
  // trip per chunk exposed: 28 us per call at the CREStereo 1/16 size, 19 chunks)
  constexpr int E = D * D + D, NE = (E + 255) / 256;
  float part[NE];
#pragma unroll
  for (int j = 0; j < NE; ++j) part[j] = 0.f;
  int c = 0;
  for (; c + 4 <= nch; c += 4) {
    float v[4][NE];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < NE; ++j) {
        const int e = tid + 256 * j;
        v[u][j] = e < E ? src[(size_t)(c + u) * E + e] : 0.f;
      }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < NE; ++j) part[j] += v[u][j];
  }
  for (; c < nch; ++c)
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int e = tid + 256 * j;
      part[j] += e < E ? src[(size_t)c * E + e] : 0.f;
    }
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const int e = tid + 256 * j;
    if (e < D * D) kv[e / D][e % D] = part[j];
    else if (e < E) ksum[e - D * D] = part[j];
  }
  for (int e = tid; e < LA_CHUNK * D; e += 256) {
    const int l = e / D, d = e % D;
    float qq = 0.f;
    if (l0 + l < L) {
      qq = (float)q[((long)n * L + l0 + l) * qs + hoff + d];
      qq = qq > 0.f ? qq + 1.f : __expf(qq);
    }
    qt[l][d] = qq;
  }
  __syncthreads();
  // thread -> token tid / 4, 8 consecutive output channels (tid % 4) * 8 (D = 32)
  constexpr int VPT = D / 4;
  const int l = tid >> 2, vb = (tid & 3) * VPT;
  if (l0 + l >= L) return;
  float num[VPT], den = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) num[j] = 0.f;
  for (int d = 0; d < D; ++d) {
    const float qq = qt[l][d];
    den += qq * ksum[d];
#pragma unroll
    for (int j = 0; j < VPT; ++j) num[j] += qq * kv[d][vb + j];
  }
  const float inv = 1.f / (den + eps);
  f16* op = out + ((long)n * L + l0 + l) * os + hoff + vb;
#pragma unroll
  for (int j = 0; j < VPT; ++j) op[j] = (f16)(num[j] * inv);
}

// ------------------------------------------------------------------ layer norm (+ residual)
// one wave per row (C <= 512), fp32 statistics
__global__ void layernorm_kernel(const f16* __restrict__ x, int xs, const float* __restrict__ gamma,
                                 const float* __restrict__ beta, const f16* __restrict__ res, int rs,
                                 f16* __restrict__ out, int os, long rows, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = blockIdx.x * (long)(blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const f16* xp = x + row * xs;
  float v[8];
  int nv = 0;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) {
    v[nv] = (float)xp[c];
    s += v[nv++];
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / C;
  float q = 0.f;
  for (int j = 0; j < nv; ++j) q += (v[j] - mean) * (v[j] - mean);
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  const float rstd = rsqrtf(q / C + eps);
  int j = 0;
  for (int c = lane; c < C; c += 64, ++j) {
    float y = (v[j] - mean) * rstd * gamma[c] + beta[c];
    if (res) y += (float)res[row * rs + c];
    out[row * os + c] = (f16)y;
  }
}

// ------------------------------------------------------------------ elementwise
__global__ void ew_kernel(const SaEwArgs a) {
  const long total = a.P * a.C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / a.C;
    const int c = (int)(i % a.C);
    float v = (float)reinterpret_cast<const f16*>(a.x)[p * a.x_stride + c] * a.scale;
    if (a.add) v += (float)reinterpret_cast<const f16*>(a.add)[p * a.add_stride + c];
    if (a.bcast) v += a.bcast[(p % a.bcast_period) * a.C + c];
    v = act_apply(v, a.act, 0.01f);
    reinterpret_cast<f16*>(a.out)[p * a.out_stride + c] = (f16)v;
  }
}

__global__ void flow_features_kernel(const float* __restrict__ flow, int fc, long P, f16* o1, int s1, int c1,
                                     f16* o2, int s2) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < P; p += (long)gridDim.x * blockDim.x) {
    const float fx = flow[p * fc], fy = fc > 1 ? flow[p * fc + 1] : 0.f;
    if (o1) {
      f16* d = o1 + p * s1;
      d[0] = (f16)fx;
      d[1] = (f16)fy;
      for (int c = 2; c < c1; ++c) d[c] = (f16)0.f;
    }
    if (o2) {
      f16* d = o2 + p * s2;
      d[0] = (f16)fx;
      d[1] = (f16)fy;
    }
  }
}

__global__ void interp_flow_kernel(const float* __restrict__ x, float* __restrict__ out, int N, int H, int W,
                                   int C, int Ho, int Wo, float mul) {
  const long total = (long)N * Ho * Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ow = (int)(i % Wo);
    const int oh = (int)((i / Wo) % Ho);
    const int n = (int)(i / ((long)Wo * Ho));
    const float sy = Ho > 1 ? (float)oh * (float)(H - 1) / (float)(Ho - 1) : 0.f;
    const float sx = Wo > 1 ? (float)ow * (float)(W - 1) / (float)(Wo - 1) : 0.f;
    int y0 = (int)floorf(sy), x0 = (int)floorf(sx);
    y0 = y0 > H - 1 ? H - 1 : y0;
    x0 = x0 > W - 1 ? W - 1 : x0;
    const int y1 = y0 + 1 < H ? y0 + 1 : H - 1, x1 = x0 + 1 < W ? x0 + 1 : W - 1;
    const float ly = sy - y0, lx = sx - x0;
    for (int c = 0; c < C; ++c) {
      auto at = [&](int y, int xx) { return x[(((long)n * H + y) * W + xx) * C + c]; };
      const float v = (1.f - ly) * ((1.f - lx) * at(y0, x0) + lx * at(y0, x1)) + ly * ((1.f - lx) * at(y1, x0) + lx * at(y1, x1));
      out[i * C + c] = mul * v;
    }
  }
}

}  // namespace

extern "C" int sa_agcl_corr(const SaAgclArgs* a, hipStream_t stream) {
  if (a->C % 32 || a->out_channels < 36) return -2;
  const long total = (long)a->N * a->H * a->W * 36;
  if (total >= (1L << 31)) return -2;  // 32-bit index math in the kernel
  // 256-channel CREStereo features: 8 lanes per (pixel, group, tap); SA_AGCL_KERNEL=w: one wave per pixel (same-process
  // A/B on CREStereo iter10 b1: 6.423 ms with the 8-lane kernel, 6.528 with the wave kernel -- a quarter of the
  // threads, each walking 9 dependent flow -> corner loads); one thread per tap otherwise
  const char* ak = std::getenv("SA_AGCL_KERNEL");  // per launch (captured once per graph): in-process A/B knob
  const bool wave = ak && ak[0] == 'w';
  const long P = (long)a->N * a->H * a->W;
  const char* at = std::getenv("SA_AGCL_TILE");  // 0: iter mode falls back to the per-tap kernels (A/B knob)
  const long tiles = (long)a->N * ((a->H + 3) / 4) * ((a->W + 31) / 32);
  if (a->C == 256 && a->iter_mode && !wave && !(at && at[0] == '0') && tiles < (1L << 31)) {
    const dim3 g((unsigned)tiles, 4);
    if (a->small_patch) hipLaunchKernelGGL((agcl_iter_tile_kernel<1, 1>), g, dim3(256), 0, stream, *a);
    else hipLaunchKernelGGL((agcl_iter_tile_kernel<4, 0>), g, dim3(256), 0, stream, *a);
  } else if (a->C == 256 && wave && (P + 3) / 4 < (1L << 31)) {
    const dim3 g((unsigned)((P + 3) / 4));
    if (a->iter_mode || a->offset) hipLaunchKernelGGL(agclw_kernel<0>, g, dim3(256), 0, stream, *a);
    else if (a->small_patch) hipLaunchKernelGGL(agclw_kernel<3>, g, dim3(256), 0, stream, *a);
    else hipLaunchKernelGGL(agclw_kernel<9>, g, dim3(256), 0, stream, *a);
  } else if (a->C == 256 && total * 8 < (1L << 31))
    hipLaunchKernelGGL(agcl8_kernel, dim3(grid_for(total * 8)), dim3(256), 0, stream, *a);
  else
    hipLaunchKernelGGL(agcl_kernel, dim3(grid_for(total)), dim3(256), 0, stream, *a);
  if (a->out_channels > 36) {
    hipLaunchKernelGGL(zero_tail_kernel, dim3(grid_for(P * (a->out_channels - 36))), dim3(256), 0, stream,
                       (f16*)a->out, a->out_stride, P, 36, a->out_channels);
  }
  return (int)hipGetLastError();
}

extern "C" int sa_cre_motion_head(const SaAgclArgs* a, const SaCreHeadArgs* h, hipStream_t stream) {
  const bool fl = h->wf16 != nullptr;
  if (!a->iter_mode || a->C != 256 || !h->w16 || !h->bias || !h->cor || h->cor_stride < 256 || h->cor_stride % 8 ||
      a->f1_stride % 8 || a->f2_stride % 8 ||
      ((uintptr_t)h->cor | (uintptr_t)h->w16 | (uintptr_t)a->f1 | (uintptr_t)a->f2) % 16 || (uintptr_t)a->flow % 8 ||
      a->H >= 65536 || a->W >= 65536)
    return -2;
  if (fl && (!h->fbias || !h->flo || h->flo_stride < 128 || !h->fcopy || h->fcopy_stride < 2 || (uintptr_t)h->wf16 % 16))
    return -2;
  const long tiles = (long)a->N * ((a->H + 1) / 2) * ((a->W + 31) / 32);
  if (tiles >= (1L << 31)) return -2;
  const dim3 g((unsigned)tiles);
  if (a->small_patch) {
    if (fl) hipLaunchKernelGGL((agcl_iter_c1_kernel<1, 1, true>), g, dim3(512), 0, stream, *a, *h);
    else hipLaunchKernelGGL((agcl_iter_c1_kernel<1, 1, false>), g, dim3(512), 0, stream, *a, *h);
  } else {
    if (fl) hipLaunchKernelGGL((agcl_iter_c1_kernel<4, 0, true>), g, dim3(512), 0, stream, *a, *h);
    else hipLaunchKernelGGL((agcl_iter_c1_kernel<4, 0, false>), g, dim3(512), 0, stream, *a, *h);
  }
  return (int)hipGetLastError();
}

extern "C" int sa_cre_motion_head_pre(const SaAgclArgs* a, const SaCreHeadArgs* h, hipStream_t stream) {
  if (!a->out || a->out_stride < 36 || !h->w16 || !h->bias || !h->cor || h->cor_stride < 256 || h->cor_stride % 8 ||
      ((uintptr_t)h->cor | (uintptr_t)h->w16) % 16 || (uintptr_t)a->flow % 8 || !h->wf16 || !h->fbias || !h->flo ||
      h->flo_stride < 128 || !h->fcopy || h->fcopy_stride < 2 || (uintptr_t)h->wf16 % 16)
    return -2;
  const long tiles = (long)a->N * ((a->H + 1) / 2) * ((a->W + 31) / 32);
  if (tiles >= (1L << 31)) return -2;
  hipLaunchKernelGGL((agcl_iter_c1_kernel<4, 0, true, true>), dim3((unsigned)tiles), dim3(512), 0, stream, *a, *h);
  return (int)hipGetLastError();
}

extern "C" int sa_agcl_conv1x1(const SaAgclArgs* a, const void* w16, const float* bias, int cout, void* out,
                               int out_stride, hipStream_t stream) {
  if (cout != 256) return -2;
  SaCreHeadArgs h{};
  h.w16 = w16;
  h.bias = bias;
  h.cor = out;
  h.cor_stride = out_stride;
  return sa_cre_motion_head(a, &h, stream);
}

extern "C" long sa_linear_attention_ws_floats(int N, int S, int heads, int dim) {
  return (long)N * heads * ((S + LA_CHUNK - 1) / LA_CHUNK) * (dim * dim + dim);
}

extern "C" int sa_linear_attention(const void* q, int qs, const void* k, int ks, const void* v, int vs, void* out,
                                   int os, int N, int L, int S, int heads, int dim, float eps, float* ws,
                                   hipStream_t stream) {
  if (dim != 32 || !ws || N < 1 || L < 1 || S < 1 || heads < 1 || N > 65535 || heads > 65535) return -2;
  const int nch = (S + LA_CHUNK - 1) / LA_CHUNK;
  hipLaunchKernelGGL(linear_attn_kv_kernel<32>, dim3(nch, heads, N), dim3(256), 0, stream, (const f16*)k, ks,
                     (const f16*)v, vs, S, heads, ws);
  hipLaunchKernelGGL(linear_attn_out_kernel<32>, dim3((L + LA_CHUNK - 1) / LA_CHUNK, heads, N), dim3(256), 0, stream,
                     (const f16*)q, qs, ws, nch, heads, (f16*)out, os, L, eps);
  return (int)hipGetLastError();
}

extern "C" int sa_layernorm(const void* x, int xs, const float* gamma, const float* beta, const void* res, int rs,
                            void* out, int os, long rows, int C, float eps, hipStream_t stream) {
  if (C > 512) return -2;
  const long blocks = (rows + 3) / 4;
  hipLaunchKernelGGL(layernorm_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (const f16*)x, xs, gamma, beta,
                     (const f16*)res, rs, (f16*)out, os, rows, C, eps);
  return (int)hipGetLastError();
}

extern "C" int sa_ew(const SaEwArgs* a, hipStream_t stream) {
  hipLaunchKernelGGL(ew_kernel, dim3(grid_for(a->P * a->C)), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

extern "C" int sa_flow_features(const float* flow, int fc, long P, void* out1, int s1, int c1, void* out2, int s2,
                                hipStream_t stream) {
  hipLaunchKernelGGL(flow_features_kernel, dim3(grid_for(P)), dim3(256), 0, stream, flow, fc, P, (f16*)out1, s1, c1,
                     (f16*)out2, s2);
  return (int)hipGetLastError();
}

extern "C" int sa_interp_flow(const float* x, float* out, int N, int H, int W, int C, int Ho, int Wo, float mul,
                              hipStream_t stream) {
  hipLaunchKernelGGL(interp_flow_kernel, dim3(grid_for((long)N * Ho * Wo)), dim3(256), 0, stream, x, out, N, H, W, C,
                     Ho, Wo, mul);
  return (int)hipGetLastError();
}
