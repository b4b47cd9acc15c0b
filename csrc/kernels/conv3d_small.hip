// Direct 3x3x3 convolution for the small-channel cost volumes of Fast-ACVNet+ (tactic 34): stride
// 1, or 2 for 8 / 16 input channels (the hourglasses' downsampling convs).
//
// Fast-ACVNet+'s correlation stem (1 real -> 8 channels over [48, 120, 160]) and concatenation stem (32 -> 16 over
// [24, 120, 160]) and the hourglasses' stride-1 convs (8-32 channels) ran as implicit GEMMs on 256 x 16 register
// tiles: N = 8-16 output columns leave most of every MFMA idle and the im2col gather re-reads each input voxel 27
// times from L2 (/root/reference/README_en.md:293-295 times the whole network at 12 ms on an RTX 3090;
// profiles/timeline_r5_facv.txt: 547 us of the 1 848 us frame chain in those tiles).
//
// Here one workgroup (4 waves) owns a 2 x 4 x 32 (D x H x W) output block = 16 row fragments of 16 voxels.  Its input
// patch (4 x 6 x 34 voxels x Cin channels, <= 52 KB) is loaded into LDS ONCE and every one of the 27 taps reads its
// fragments there at a shifted voxel offset.  K runs in the packed weights' (kd, kh, kw, ci) order, 32 per
// v_mfma_f32_16x16x32_f16: a lane's 8 k-values are one 8-channel chunk of one tap of one voxel, i.e. one 16-B LDS
// read (1, 2 or 4 taps per k-step for Cin = 32 / 16 / 8).  The product is transposed (weights are the A operand), so
// a lane ends with 4 consecutive output channels of one voxel: one 8-B store per fragment and column tile.  Weight
// fragments come straight from global memory (L2 / L1 resident: <= 57 KB shared by every workgroup), one k-step
// ahead.  LDS rows are 16 B x Cin/8 per voxel with the chunk XOR'd by (voxel >> log2(16 / (Cin / 8))), so the 16
// lanes of a fragment read (16 consecutive voxels, one chunk) hit 16 distinct 16-B bank groups.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>

#include "sa/kernels.h"

namespace {

typedef _Float16 f16;
typedef f16 half8 __attribute__((ext_vector_type(8)));
typedef f16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int DT = 2, HT = 4, WT = 32;  // output block
// input patch of a stride-ST block: 4 x 6 x 34 (ST 1), 5 x 9 x 65 (ST 2)
template <int ST>
struct Patch {
  static constexpr int PD = (DT - 1) * ST + 3, PH = (HT - 1) * ST + 3, PW = (WT - 1) * ST + 3;
  static constexpr int PVOX = PD * PH * PW;
};

struct Conv3dArgs {
  const f16* x;
  int xs;  // pixel stride (elements)
  const f16* w;  // packed [Cout_pad][Kpad], K = (kd, kh, kw, ci)
  int Kpad;
  const float* bias;
  f16* out;
  int os;
  int N, D, H, W, Cout;  // input dims
  int Do, Ho, Wo;        // output dims (stride 1: the input's)
  int act;
  float alpha, scale;
  const f16* gate;  // [N][H][W][gs] (broadcast over depth) or null
  int gs;
  int out_f32;    // fp32 output (SA_EPI_STORE_F32)
  int cout_real;  // > 0: Cout = 8 parity classes of cout_real channels scattered to the 2x output volume (a k4 / s2
                  // transposed conv3d as a 3x3x3 conv): class pi -> depth parity pi >> 2, row (pi >> 1) & 1, column pi & 1
};

__device__ __forceinline__ float act_apply(float v, int act, float alpha) {
  switch (act) {
    case SA_ACT_RELU: return v > 0.f ? v : 0.f;
    case SA_ACT_LEAKY: return v > 0.f ? v : v * alpha;
    case SA_ACT_SIGMOID: return 1.f / (1.f + __expf(-v));
    case SA_ACT_RELU6: return v < 0.f ? 0.f : (v > 6.f ? 6.f : v);
    case SA_ACT_TANH: {
      const float e = __expf(-2.f * fabsf(v));
      const float t = (1.f - e) / (1.f + e);
      return v < 0.f ? -t : t;
    }
    default: return v;
  }
}

template <int NCH>
__device__ __forceinline__ int pslot(int vox, int chunk) {
  constexpr int SH = NCH == 1 ? 4 : (NCH == 2 ? 3 : 2);  // log2(16 / NCH)
  return (vox * NCH + (chunk ^ ((vox >> SH) & (NCH - 1)))) << 4;
}

// NCH = Cin / 8 (1, 2, 4); NCT = output column tiles of 16 (1 or 2); ST = stride (1, or 2 for NCH <= 2)
template <int NCH, int NCT, int ST = 1>
__global__ __launch_bounds__(256) void conv3d_small_kernel(const Conv3dArgs p) {
  constexpr int CIN = 8 * NCH;
  constexpr int PH = Patch<ST>::PH, PW = Patch<ST>::PW, PVOX = Patch<ST>::PVOX;
  __shared__ __attribute__((aligned(16))) char patch[PVOX * NCH * 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int tw = (p.Wo + WT - 1) / WT, th = (p.Ho + HT - 1) / HT, td = (p.Do + DT - 1) / DT;
  int b = blockIdx.x;
  const int bx = b % tw;
  b /= tw;
  const int by = b % th;
  b /= th;
  const int bz = b % td;
  const int n = b / td;
  const int x0 = bx * WT, y0 = by * HT, z0 = bz * DT;

  // ---- input patch -> LDS (zero padding outside the volume): a thread's loads issued in batches of up to 13 before
  // their stores ----
  constexpr int NLD = (PVOX * NCH + 255) / 256;
  constexpr int LB = NLD < 13 ? NLD : 13;
#pragma unroll
  for (int k0 = 0; k0 < NLD; k0 += LB) {
    half8 pv[LB];
#pragma unroll
    for (int k = 0; k < LB; ++k) {
      const int i = tid + 256 * (k0 + k);
      const int vox = i / NCH, c = i - vox * NCH;
      const int pz = vox / (PH * PW), rem = vox - pz * (PH * PW);
      const int py = rem / PW, px = rem - py * PW;
      const int z = z0 * ST - 1 + pz, y = y0 * ST - 1 + py, x = x0 * ST - 1 + px;
#pragma unroll
      for (int j = 0; j < 8; ++j) pv[k][j] = (f16)0.f;
      if (k0 + k < NLD && i < PVOX * NCH && (unsigned)z < (unsigned)p.D && (unsigned)y < (unsigned)p.H &&
          (unsigned)x < (unsigned)p.W)
        pv[k] = *reinterpret_cast<const half8*>(p.x + ((((long)n * p.D + z) * p.H + y) * p.W + x) * p.xs + 8 * c);
    }
#pragma unroll
    for (int k = 0; k < LB; ++k) {
      const int i = tid + 256 * (k0 + k);
      if (k0 + k < NLD && i < PVOX * NCH) *reinterpret_cast<half8*>(patch + pslot<NCH>(i / NCH, i % NCH)) = pv[k];
    }
  }
  __syncthreads();

  // ---- K loop: wave w owns fragments 4w .. 4w + 3 (fragment f: dz = f / 8, hy = (f / 2) % 4, wx0 = 16 (f % 2)) ----
  int fbase[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int f = 4 * wave + i;
    fbase[i] = (((f / 8) * PH + (f / 2) % 4) * PW + (f % 2) * 16 + r16) * ST;
  }
  floatx4 acc[4][NCT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NCT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  constexpr int NK = (27 * CIN + 31) / 32;  // k-steps holding real taps (the packed K padding beyond is zero)
  const f16* wrow[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j) wrow[j] = p.w + (size_t)(16 * j + r16) * p.Kpad + 8 * g;
  half8 wcur[NCT], wnext[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j) wcur[j] = *reinterpret_cast<const half8*>(wrow[j]);
#pragma unroll
  for (int ks = 0; ks < NK; ++ks) {
    if (ks + 1 < NK) {
#pragma unroll
      for (int j = 0; j < NCT; ++j) wnext[j] = *reinterpret_cast<const half8*>(wrow[j] + 32 * (ks + 1));
    }
    // this lane's 8 k-values: chunk u = 4 ks + g of the (tap, chunk) sequence
    const int u = 4 * ks + g;
    const int tap = u / NCH, c = u - tap * NCH;
    const bool live = tap < 27;
    const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
    const int toff = (kd * PH + kh) * PW + kw;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      half8 a;
      if (live) {
        a = *reinterpret_cast<const half8*>(patch + pslot<NCH>(fbase[i] + toff, c));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = (f16)0.f;
      }
#pragma unroll
      for (int j = 0; j < NCT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wcur[j], a, acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NCT; ++j) wcur[j] = wnext[j];
  }

  // ---- epilogue: lane (r16, g) holds output channels 16 j + 4 g .. + 3 of voxel r16 of each fragment ----
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int f = 4 * wave + i;
    const int z = z0 + f / 8, y = y0 + (f / 2) % 4, x = x0 + (f % 2) * 16 + r16;
    if (z >= p.Do || y >= p.Ho || x >= p.Wo) continue;
    const long vox = (((long)n * p.Do + z) * p.Ho + y) * p.Wo + x;
#pragma unroll
    for (int j = 0; j < NCT; ++j) {
      const int co = 16 * j + 4 * g;
      if (co >= p.Cout) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cc = co + r;
        v[r] = acc[i][j][r] * p.scale + (p.bias && cc < p.Cout ? p.bias[cc] : 0.f);
        v[r] = act_apply(v[r], p.act, p.alpha);
        if (p.gate && cc < p.Cout) v[r] *= (float)p.gate[(((long)n * p.Ho + y) * p.Wo + x) * p.gs + cc];
      }
      if (p.cout_real > 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int cj = co + r;
          if (cj >= p.Cout) break;
          const int pi = cj / p.cout_real, c = cj - pi * p.cout_real;
          const long ovox = ((((long)n * 2 * p.Do + 2 * z + (pi >> 2)) * 2 * p.Ho + 2 * y + ((pi >> 1) & 1)) * 2 * p.Wo +
                             2 * x + (pi & 1));
          if (p.out_f32) reinterpret_cast<float*>(p.out)[ovox * p.os + c] = v[r];
          else p.out[ovox * p.os + c] = (f16)v[r];
        }
        continue;
      }
      if (p.out_f32) {
        float* op = reinterpret_cast<float*>(p.out) + vox * p.os + co;
        for (int r = 0; r < 4 && co + r < p.Cout; ++r) op[r] = v[r];
        continue;
      }
      f16* op = p.out + vox * p.os + co;
      if (co + 4 <= p.Cout) {
        half4 h;
#pragma unroll
        for (int r = 0; r < 4; ++r) h[r] = (f16)v[r];
        *reinterpret_cast<half4*>(op) = h;
      } else {
        for (int r = 0; co + r < p.Cout; ++r) op[r] = (f16)v[r];
      }
    }
  }
}

}  // namespace

extern "C" int sa_conv3d_small(const void* x, int xs, int Cin, const void* w, int Kpad, const float* bias, void* out,
                               int os, int N, int D, int H, int W, int Cout, int act, float alpha, float scale,
                               const void* gate, int gs, int out_f32, int cout_real, int stride, hipStream_t stream) {
  if (!(Cin == 8 || Cin == 16 || Cin == 32) || Cout < 1 || Cout > 32 || Kpad % 32 || Kpad < 27 * Cin) return -2;
  if (!(stride == 1 || (stride == 2 && Cin <= 16 && !cout_real))) return -2;  // stride 2: the 5 x 9 x 65 patch
  if (cout_real > 0 && (gate || Cout != 8 * cout_real)) return -2;
  const bool scatter_or_f32 = cout_real > 0 || out_f32;  // element stores
  if (xs % 8 || (!scatter_or_f32 && os % 4) || ((uintptr_t)x & 15) || (!scatter_or_f32 && ((uintptr_t)out & 7)) ||
      ((uintptr_t)w & 15))
    return -2;
  if (N < 1 || D < 1 || H < 1 || W < 1) return -2;
  const int Do = (D - 1) / stride + 1, Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  Conv3dArgs a{(const f16*)x, xs, (const f16*)w, Kpad, bias, (f16*)out, os, N, D, H, W, Cout, Do, Ho, Wo, act, alpha,
               scale, (const f16*)gate, gs, out_f32, cout_real};
  const long blocks = (long)N * ((Do + DT - 1) / DT) * ((Ho + HT - 1) / HT) * ((Wo + WT - 1) / WT);
  if (blocks > 0x7fffffffL) return -2;
  const dim3 grid((unsigned)blocks), blk(256);
  const bool two = Cout > 16;
  if (stride == 2) {
    if (Cin == 8) {
      if (two) hipLaunchKernelGGL((conv3d_small_kernel<1, 2, 2>), grid, blk, 0, stream, a);
      else hipLaunchKernelGGL((conv3d_small_kernel<1, 1, 2>), grid, blk, 0, stream, a);
    } else {
      if (two) hipLaunchKernelGGL((conv3d_small_kernel<2, 2, 2>), grid, blk, 0, stream, a);
      else hipLaunchKernelGGL((conv3d_small_kernel<2, 1, 2>), grid, blk, 0, stream, a);
    }
  } else if (Cin == 8) {
    if (two) hipLaunchKernelGGL((conv3d_small_kernel<1, 2>), grid, blk, 0, stream, a);
    else hipLaunchKernelGGL((conv3d_small_kernel<1, 1>), grid, blk, 0, stream, a);
  } else if (Cin == 16) {
    if (two) hipLaunchKernelGGL((conv3d_small_kernel<2, 2>), grid, blk, 0, stream, a);
    else hipLaunchKernelGGL((conv3d_small_kernel<2, 1>), grid, blk, 0, stream, a);
  } else {
    if (two) hipLaunchKernelGGL((conv3d_small_kernel<4, 2>), grid, blk, 0, stream, a);
    else hipLaunchKernelGGL((conv3d_small_kernel<4, 1>), grid, blk, 0, stream, a);
  }
  return (int)hipGetLastError();
}
