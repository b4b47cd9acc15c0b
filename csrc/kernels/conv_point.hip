// Strided 1x1 convolution (the residual-block downsample of the RAFT-Stereo / CREStereo encoders: 64 -> 96 and
// 96 -> 128 at stride 2), tile_cfg 25.
//
// As an implicit GEMM this is K = 64 / 96: one or two k-steps per tile prologue and epilogue, 0.1 PFLOP/s and far
// from the HBM roofline (285 us for 1.23 M output pixels at RAFT-SF b8, where ~75 us moves its bytes).  Here the
// whole weight matrix stays in registers as the MFMA A operand (COUT / 16 fragments x CIN / 32 k-steps), every
// lane loads its pixel's 16-B channel chunks straight from global memory into B fragments (no LDS), and
// C^T = W * X^T leaves each lane with 8 consecutive output channels of one pixel per fragment pair: one 16-B
// store each.  Each wave walks a contiguous run of 16-pixel fragments, the next fragment's loads in flight under
// the current MFMAs; optional instance-norm statistics (per-lane running sums, DPP row reduction, slotted
// fixed-point atomics when the image changes) or bias / activation only.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include "sa/kernels.h"

namespace {

typedef _Float16 f16;
typedef f16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float act_apply(float v, int act, float alpha) {
  switch (act) {
    case SA_ACT_RELU: return v > 0.f ? v : 0.f;
    case SA_ACT_LEAKY: return v > 0.f ? v : v * alpha;
    default: return v;
  }
}

__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
  return v;
}

struct PointArgs {
  const f16* x;
  int xs;
  const f16* w;
  int kpad;
  const float* bias;
  f16* out;
  int os;
  int N, H, W, Ho, Wo, stride;
  int act;
  float alpha;
  sa_stat_t* stats;
  int slots;
};

// output channel of accumulator row rr of fragment j: fragment pair (j >> 1) covers 32 channels, lane kq of the
// pair gets 8 consecutive ones (4 from each fragment)
__device__ __forceinline__ int point_channel(int j, int rr) { return (j >> 1) * 32 + (rr >> 2) * 8 + (j & 1) * 4 + (rr & 3); }

template <int CIN, int COUT, bool STATS>
__global__ __launch_bounds__(256, 2) void conv1x1_point_kernel(const PointArgs p) {
  constexpr int NJ = COUT / 16, KS = CIN / 32;
  const int lane = threadIdx.x & 63;
  const int frow = lane & 15, kq = lane >> 4;
  half8 wa[KS][NJ];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      wa[ks][j] = *reinterpret_cast<const half8*>(p.w + (size_t)point_channel(j, frow) * p.kpad + ks * 32 + kq * 8);
  float ssum[NJ / 2][8], ssq[NJ / 2][8];
#pragma unroll
  for (int jp = 0; jp < NJ / 2; ++jp)
#pragma unroll
    for (int e = 0; e < 8; ++e) ssum[jp][e] = ssq[jp][e] = 0.f;
  int stat_img = -1;
  auto flush = [&]() {
    if constexpr (STATS) {
#pragma unroll
      for (int jp = 0; jp < NJ / 2; ++jp)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float s0 = row16_sum(ssum[jp][e]), s1 = row16_sum(ssq[jp][e]);
          ssum[jp][e] = ssq[jp][e] = 0.f;
          if (frow == 0) {
            sa_stat_t* st = p.stats + (size_t)(blockIdx.x % (p.slots > 1 ? p.slots : 1)) * p.N * COUT * 2;
            unsigned long long* sp =
                reinterpret_cast<unsigned long long*>(st) + ((size_t)stat_img * COUT + jp * 32 + kq * 8 + e) * 2;
            atomicAdd(sp, (unsigned long long)__double2ll_rn((double)s0 * SA_STAT_SCALE));
            atomicAdd(sp + 1, (unsigned long long)__double2ll_rn((double)s1 * SA_STAT_SCALE));
          }
        }
    }
  };

  const long M = (long)p.N * p.Ho * p.Wo;
  const long nfrag = (M + 15) / 16;
  const long waves = (long)gridDim.x * (blockDim.x >> 6);
  const long wid = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long per = (nfrag + waves - 1) / waves;
  const long f0 = wid * per, f1 = f0 + per < nfrag ? f0 + per : nfrag;
  const int HWo = p.Ho * p.Wo;
  auto fetch = [&](long f, half8* b) {
    const long m = f * 16 + frow;
    if (m < M) {
      const int n = (int)(m / HWo), r = (int)(m - (long)n * HWo);
      const int oy = r / p.Wo, ox = r - oy * p.Wo;
      const f16* src = p.x + ((size_t)((size_t)n * p.H + oy * p.stride) * p.W + ox * p.stride) * p.xs + kq * 8;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) b[ks] = *reinterpret_cast<const half8*>(src + ks * 32);
    } else {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) b[ks] = half8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  half8 bcur[KS], bnext[KS];
  if (f0 < f1) fetch(f0, bcur);
  for (long f = f0; f < f1; ++f) {
    if (f + 1 < f1) fetch(f + 1, bnext);
    floatx4 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[ks][j], bcur[ks], acc[j], 0, 0, 0);
    const long m = f * 16 + frow;
    const bool ok = m < M;
    if constexpr (STATS) {
      // every fragment lies in one image (host guarantees Ho * Wo % 16 == 0): flush when the wave's image changes
      const int n0 = (int)((f * 16) / HWo);
      if (n0 != stat_img) {
        if (stat_img >= 0) flush();
        stat_img = n0;
      }
    }
#pragma unroll
    for (int jp = 0; jp < NJ / 2; ++jp) {
      float bias8[8];  // re-read per fragment (L1 hits): registers go to the weights and statistics
      if (p.bias) {
        const floatx4 b0 = *reinterpret_cast<const floatx4*>(p.bias + jp * 32 + kq * 8);
        const floatx4 b1 = *reinterpret_cast<const floatx4*>(p.bias + jp * 32 + kq * 8 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) bias8[e] = b0[e], bias8[e + 4] = b1[e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) bias8[e] = 0.f;
      }
      half8 h;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int j = jp * 2 + (e >> 2), r = e & 3;
        const float v = act_apply(acc[j][r] + bias8[e], p.act, p.alpha);
        h[e] = (f16)v;
        if constexpr (STATS) {
          const float vm = ok ? v : 0.f;
          ssum[jp][e] += vm;
          ssq[jp][e] = fmaf(vm, vm, ssq[jp][e]);
        }
      }
      if (ok) *reinterpret_cast<half8*>(p.out + (size_t)m * p.os + jp * 32 + kq * 8) = h;
    }
    if (f + 1 < f1) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) bcur[ks] = bnext[ks];
    }
  }
  if constexpr (STATS) {
    if (stat_img >= 0) flush();
  }
}

template <int CIN, int COUT>
void launch_point(const PointArgs& a, unsigned g, hipStream_t s) {
  if (a.stats) hipLaunchKernelGGL((conv1x1_point_kernel<CIN, COUT, true>), dim3(g), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((conv1x1_point_kernel<CIN, COUT, false>), dim3(g), dim3(256), 0, s, a);
}

}  // namespace

extern "C" int sa_conv1x1_point(const void* x, int xs, int cin, const void* w, int kpad, const float* bias, void* out,
                                int os, int cout, int N, int H, int W, int stride, int act, float alpha,
                                sa_stat_t* stats, int slots, hipStream_t stream) {
  if (!((cin == 64 && cout == 96) || (cin == 96 && cout == 128))) return -5;
  if (kpad < cin || xs < cin || xs % 8 || os < cout || os % 8 || stride < 1 ||
      (act != SA_ACT_NONE && act != SA_ACT_RELU && act != SA_ACT_LEAKY))
    return -2;
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  if (stats && ((long)Ho * Wo) % 16) return -5;  // a 16-pixel fragment must not straddle two images
  PointArgs a{(const f16*)x, xs, (const f16*)w, kpad, bias, (f16*)out, os, N, H, W, Ho, Wo, stride, act, alpha, stats,
              slots};
  const long nfrag = ((long)N * Ho * Wo + 15) / 16;
  long g = (nfrag + 3) / 4;
  // 4 blocks of 4 waves per CU, each wave a contiguous run of fragments.  With statistics every wave flushes its
  // per-image sums with atomics: for 96 -> 128 (64 sums per lane) one block per CU wins (tools/conv_bench.py
  // ds38 --stats: 75 vs 143 us), for 64 -> 96 the memory parallelism of four (ds8: 173 vs 206 us)
  const long gmax = stats && cin == 96 ? 256 : 1024;
  if (g > gmax) g = gmax;
  if (g < 1) return 0;
  if (cin == 64) launch_point<64, 96>(a, (unsigned)g, stream);
  else launch_point<96, 128>(a, (unsigned)g, stream);
  return (int)hipGetLastError();
}
