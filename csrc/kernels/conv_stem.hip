// 7x7 stem convolution of the RAFT-Stereo / CREStereo encoders (conv1: 3 -> 64 channels, stride 1 or 2,
// pad 3) on MFMA, persistent tiles (gfx950).
//
// The implicit-GEMM kernels (conv2d.hip) see this layer as K = 49 taps x 8 padded channels = 392 with
// five of every eight k values multiplying zero weights, and gather one 16-B chunk per tap: 0.08-0.23
// PFLOP/s at 480x640 (profiles/r02_sf_b8_serial_kernels.txt).  Here the channels are compacted to 4
// (3 real + a zero lane) and K is ordered (kh, kw, c) with kw padded 7 -> 8, so one 32-deep MFMA k-step
// is exactly one filter row: 8 input pixels x 4 channels = 64 contiguous bytes of the staged input row.
// 7 k-steps instead of 13, and every A/B fragment is a 16-B read of LDS.
//
//   * the output tile is 4 rows x 32 columns; one wave per row, 2 pixel fragments of 16 columns;
//   * roles are swapped (C^T = W * X^T): the weights are the MFMA A operand, held in registers for the
//     whole kernel (7 k-steps x 4 fragments), and the input pixels are the B operand, read from LDS;
//   * the weight rows of fragment j are permuted so that lane (frow, kq) of v_mfma_f32_16x16x32_f16
//     ends up holding channels kq*16 .. kq*16+15 of one pixel: the epilogue is two 16-B global stores
//     per pixel fragment straight from the accumulators (no LDS staging of the C tile);
//   * the next tile's input pixels are prefetched into registers under the current tile's MFMAs;
//   * optional instance-norm statistics (per-lane running sums, reduced and flushed with slotted
//     fixed-point atomics when the image changes, same layout as the conv2d.hip epilogue).
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <type_traits>

#include "sa/kernels.h"

namespace {

typedef _Float16 f16;
typedef f16 half4 __attribute__((ext_vector_type(4)));
typedef f16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int TR = 4, TC = 32;  // output tile (one wave per row)
constexpr int PF = TC / 16;      // pixel fragments per wave
constexpr int KSTEPS = 7;       // one per filter row

template <int S>
struct StemGeom {
  static constexpr int IR = (TR - 1) * S + 7;             // input rows of a tile
  static constexpr int IC = ((TC - 1) * S + 8 + 1) & ~1;  // input cols (kw padded to 8), even
  static constexpr int PIX = IR * IC;
  static constexpr int PER_THREAD = (PIX + 255) / 256;
};

__device__ __forceinline__ float act_apply(float v, int act, float alpha) {
  switch (act) {
    case SA_ACT_RELU: return v > 0.f ? v : 0.f;
    case SA_ACT_LEAKY: return v > 0.f ? v : v * alpha;
    case SA_ACT_TANH: {
      float e = __expf(-2.f * fabsf(v));
      float t = (1.f - e) / (1.f + e);
      return v < 0.f ? -t : t;
    }
    case SA_ACT_SIGMOID: return 1.f / (1.f + __expf(-v));
    case SA_ACT_RELU6: return v < 0.f ? 0.f : (v > 6.f ? 6.f : v);
    default: return v;
  }
}

struct StemArgs {
  const f16* x;
  int xs;     // input pixel stride (elements)
  int creal;  // real input channels (1..4); the rest of the 4 staged lanes is zero
  const f16* w;  // packed [>=64][kpad], K ordered (kh, kw, ci) with ci padded to cpad
  int kpad, cpad;
  const float* bias;
  f16* out;
  int os;
  int N, H, W, Ho, Wo;
  float alpha;
  sa_stat_t* stats;
  int slots;
};

// output-channel permutation: row rr (0..15) of fragment j holds channel (rr >> 2) * 16 + j * 4 + (rr & 3)
__device__ __forceinline__ int stem_channel(int j, int rr) { return (rr >> 2) * 16 + j * 4 + (rr & 3); }

template <int S, int ACT, bool STATS>
__global__ __launch_bounds__(256, 2) void conv7x7_stem_kernel(const StemArgs p) {
  using G = StemGeom<S>;
  __shared__ __attribute__((aligned(16))) half4 tile[G::PIX];
  __shared__ float red[STATS ? 4 * 64 * 2 : 1];  // flush: per-wave channel totals [wave][64][sum, sumsq]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, kq = lane >> 4;
  const int tiles_x = (p.Wo + TC - 1) / TC, tiles_y = (p.Ho + TR - 1) / TR;
  const int tiles_img = tiles_x * tiles_y;
  const int ntiles = p.N * tiles_img;

  // stationary weight fragments (MFMA A operand): row frow of fragment j = output channel
  // stem_channel(j, frow); k values kq*8 .. kq*8+7 of filter row kh = pixels kw = 2kq, 2kq+1 x 4 channels
  half8 wa[KSTEPS][4];
#pragma unroll
  for (int kh = 0; kh < KSTEPS; ++kh)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f16* wr = p.w + (size_t)stem_channel(j, frow) * p.kpad;
      half8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int kw = 2 * kq + (e >> 2), c = e & 3;
        v[e] = (kw < 7 && c < p.creal) ? wr[(kh * 7 + kw) * p.cpad + c] : (f16)0.f;
      }
      wa[kh][j] = v;
    }
  // bias of this lane's 16 output channels kq*16 .. +15 (accumulator element (j, r) = channel kq*16 + 4j + r)
  float bias16[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) bias16[e] = p.bias ? p.bias[kq * 16 + e] : 0.f;

  float ssum[16], ssq[16];
  if constexpr (STATS) {
#pragma unroll
    for (int e = 0; e < 16; ++e) ssum[e] = ssq[e] = 0.f;
  }
  int stat_img = -1;
  auto flush_stats = [&]() {
    if constexpr (STATS) {
      // lanes sharing kq hold the same 16 channels: reduce over frow (lane bits 0..3)
#pragma unroll
      for (int off = 1; off < 16; off <<= 1)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          ssum[e] += __shfl_xor(ssum[e], off);
          ssq[e] += __shfl_xor(ssq[e], off);
        }
      // the 4 waves' totals summed in LDS in a fixed order, then one wave issues the atomics (a quarter of
      // them; the flush is block-uniform)
      if (frow == 0)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          red[(wave * 64 + kq * 16 + e) * 2] = ssum[e];
          red[(wave * 64 + kq * 16 + e) * 2 + 1] = ssq[e];
        }
      __syncthreads();
      if (wave == 0 && stat_img >= 0) {
        sa_stat_t* st = p.stats + (size_t)(blockIdx.x % (p.slots > 1 ? p.slots : 1)) * p.N * 64 * 2;
        const int c = lane;  // one channel per lane
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) a0 += red[(w * 64 + c) * 2], a1 += red[(w * 64 + c) * 2 + 1];
        unsigned long long* sp = reinterpret_cast<unsigned long long*>(st) + ((size_t)stat_img * 64 + c) * 2;
        atomicAdd(sp, (unsigned long long)__double2ll_rn((double)a0 * SA_STAT_SCALE));
        atomicAdd(sp + 1, (unsigned long long)__double2ll_rn((double)a1 * SA_STAT_SCALE));
      }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 16; ++e) ssum[e] = ssq[e] = 0.f;
    }
  };

  // input staging: thread tid owns staged pixels tid + 256 * i (row-major over IR x IC), 4 channels each
  half4 pre[G::PER_THREAD];
  auto fetch = [&](int t) {
    const int n = t / tiles_img, r = t - n * tiles_img;
    const int ty = r / tiles_x, tx = r - ty * tiles_x;
    const int y0 = ty * TR * S - 3, x0 = tx * TC * S - 3;
#pragma unroll
    for (int i = 0; i < G::PER_THREAD; ++i) {
      const int q = tid + 256 * i;
      const int iy = y0 + q / G::IC, ix = x0 + q % G::IC;
      half4 v = {0, 0, 0, 0};
      if (q < G::PIX && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W) {
        v = *reinterpret_cast<const half4*>(p.x + ((size_t)((size_t)n * p.H + iy) * p.W + ix) * p.xs);
        if (p.creal < 4) v[3] = 0;
        if (p.creal < 3) v[2] = 0;
        if (p.creal < 2) v[1] = 0;
      }
      pre[i] = v;
    }
  };

  // contiguous run of tiles per workgroup: image boundaries (statistics flushes) are crossed once or twice
  // per workgroup instead of in lockstep by all of them
  const int per = (ntiles + gridDim.x - 1) / gridDim.x;
  const int tb = blockIdx.x * per;
  const int te = tb + per < ntiles ? tb + per : ntiles;
  int t = tb;
  if (t < te) fetch(t);
  for (; t < te; ++t) {
#pragma unroll
    for (int i = 0; i < G::PER_THREAD; ++i) {
      const int q = tid + 256 * i;
      if (q < G::PIX) tile[q] = pre[i];
    }
    __syncthreads();
    if (t + 1 < te) fetch(t + 1);  // next tile's pixels in flight under the MFMAs

    floatx4 acc[PF][4];
#pragma unroll
    for (int i = 0; i < PF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < KSTEPS; ++kh) {
      half8 b[PF];
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        // output column 16 i + frow of row `wave`: staged pixels (wave*S + kh, (16i + frow)*S + 2kq .. +1)
        const half4* src = tile + (wave * S + kh) * G::IC + (16 * i + frow) * S + 2 * kq;
        const half4 lo = src[0], hi = src[1];
        b[i] = half8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < PF; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[kh][j], b[i], acc[i][j], 0, 0, 0);
    }

    const int n = t / tiles_img, rr = t - n * tiles_img;
    const int ty = rr / tiles_x, tx = rr - ty * tiles_x;
    if constexpr (STATS) {
      if (n != stat_img) {
        if (stat_img >= 0) flush_stats();
        stat_img = n;
      }
    }
    const int oy = ty * TR + wave;
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int ox = tx * TC + 16 * i + frow;
      if (oy < p.Ho && ox < p.Wo) {
        half8 h0, h1;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int e = 4 * j + r;
            const float v = act_apply(acc[i][j][r] + bias16[e], ACT, p.alpha);
            if (e < 8) h0[e] = (f16)v;
            else h1[e - 8] = (f16)v;
            if constexpr (STATS) {
              ssum[e] += v;
              ssq[e] += v * v;
            }
          }
        f16* o = p.out + ((size_t)((size_t)n * p.Ho + oy) * p.Wo + ox) * p.os + kq * 16;
        *reinterpret_cast<half8*>(o) = h0;
        *reinterpret_cast<half8*>(o + 8) = h1;
      }
    }
    __syncthreads();  // every wave done reading the staged tile before it is overwritten
  }
  if constexpr (STATS) {
    if (stat_img >= 0) flush_stats();
  }
}

template <int S, bool STATS>
void launch_stem(const StemArgs& a, int act, dim3 g, hipStream_t s) {
  switch (act) {
    case SA_ACT_RELU: hipLaunchKernelGGL((conv7x7_stem_kernel<S, SA_ACT_RELU, STATS>), g, dim3(256), 0, s, a); break;
    case SA_ACT_LEAKY: hipLaunchKernelGGL((conv7x7_stem_kernel<S, SA_ACT_LEAKY, STATS>), g, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL((conv7x7_stem_kernel<S, SA_ACT_NONE, STATS>), g, dim3(256), 0, s, a); break;
  }
}

}  // namespace

extern "C" int sa_conv7x7_stem(const void* x, int xs, int creal, const void* w, int kpad, int cpad,
                               const float* bias, void* out, int os, int N, int H, int W, int stride, int act,
                               float alpha, sa_stat_t* stats, int slots, hipStream_t stream) {
  if (creal < 1 || creal > 4 || cpad < 4 || kpad < 49 * cpad || xs < 4 || xs % 4 || os < 64 || os % 8 ||
      (stride != 1 && stride != 2) || (act != SA_ACT_NONE && act != SA_ACT_RELU && act != SA_ACT_LEAKY))
    return -2;
  const int Ho = (H + 6 - 7) / stride + 1, Wo = (W + 6 - 7) / stride + 1;
  StemArgs a{(const f16*)x, xs, creal, (const f16*)w, kpad, cpad, bias, (f16*)out, os, N, H, W, Ho, Wo, alpha,
             stats, slots};
  const long ntiles = (long)N * ((Ho + TR - 1) / TR) * ((Wo + TC - 1) / TC);
  if (ntiles < 1) return 0;
  // persistent: two blocks per CU (256 CUs), each walks tiles blockIdx, +grid, ...
  const long g = ntiles < 512 ? ntiles : 512;
  const dim3 grid((unsigned)g);
  if (stride == 1) {
    if (stats) launch_stem<1, true>(a, act, grid, stream);
    else launch_stem<1, false>(a, act, grid, stream);
  } else {
    if (stats) launch_stem<2, true>(a, act, grid, stream);
    else launch_stem<2, false>(a, act, grid, stream);
  }
  return (int)hipGetLastError();
}
