// Direct 3x3 / stride 1 or 2 convolution for small channel counts (tactic 36): Cin in {8, 16, 32, 48, 64, 96} from one or two
// channel-concatenated sources, Cout <= 64, dilation 1, 2 or 4 ("same" padding), fp16 or fp32 output, optionally the
// parity scatter of a k4 / s2 transposed conv.
//
// Fast-ACVNet+'s feature upsampling / refinement convs (32 -> 32 at 240 x 320, 48 -> 48 and [24|24] -> 48 at
// 120 x 160, the spx branch's [32|32] -> 64 at full resolution) and HITNet's feature extractor run 3x3 convs whose
// N = 16-64 output columns leave the implicit GEMM's 128-wide tiles mostly idle while its im2col gather re-reads every
// input pixel 9 times (e.g. 2 x 240 x 320, 32 -> 32: 39 us at 73 TFLOP/s for 20 MB that HBM moves in 4 us,
// profiles/round6_notes.md).  The 3-D twin of this kernel is conv3d_small.hip (tactic 34).
//
// One workgroup (4 waves) owns an 8 x 32 output block = 16 row fragments of 16 pixels.  Its (8 + 2d) x (32 + 2d) input
// patch x Cin channels (<= 80 KB at dilation 4) is loaded into LDS ONCE and every one of the 9 taps reads its fragments
// there at a shifted pixel offset (HITNet's tile-update residual blocks are dilated 1 / 2 / 4).  K runs in the packed
// weights' (kh, kw, ci) order, 32 per v_mfma_f32_16x16x32_f16: a lane's 8 k-values are one 8-channel chunk of one tap
// of one pixel, one 16-B LDS read.  The product is transposed (weights
// are the A operand, from L1 one k-step ahead), so a lane ends with 4 consecutive output channels of one pixel: one
// 8-B store per fragment and column tile.  Power-of-two chunk counts XOR-swizzle the chunk by the pixel index so the
// 16 lanes of a fragment read hit distinct 16-B bank groups.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>

#include "sa/kernels.h"

namespace {

typedef _Float16 f16;
typedef f16 half8 __attribute__((ext_vector_type(8)));
typedef f16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int HT = 8, WT = 32;  // output block; input patch (HT + 2 dil) x (WT + 2 dil)

struct C2Args {
  const f16* x0;  // source 0: c0 channels at pixel stride xs0
  int xs0, c0;
  const f16* x1;  // source 1 (or null): the remaining Cin - c0 channels at stride xs1
  int xs1;
  const f16* w;  // packed [Cout_pad][Kpad], K = (kh, kw, ci)
  int Kpad;
  const float* bias;
  f16* out;
  int os;
  int N, H, W, Cout;
  int act;
  float alpha, scale;
  const f16* res;
  int rs, act2;
  int dil;        // dilation = padding (1, 2, 4)
  int out_f32;    // fp32 output (SA_EPI_STORE_F32)
  int stride;     // 1 or 2 (input H x W -> output Ho x Wo)
  int Ho, Wo;
  int cout_real;  // > 0: Cout = 4 parity classes of cout_real channels scattered to the 2x output (a k4 / s2 / p1
                  // transposed conv as a 3x3 conv, ops.deconv_as_conv_weight): class pi -> row parity pi >> 1,
                  // column parity pi & 1
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
__device__ __forceinline__ int pslot(int pix, int chunk) {
  if constexpr ((NCH & (NCH - 1)) == 0) {
    constexpr int SH = NCH == 1 ? 4 : (NCH == 2 ? 3 : (NCH == 4 ? 2 : 1));  // log2(16 / NCH)
    return (pix * NCH + (chunk ^ ((pix >> SH) & (NCH - 1)))) << 4;
  } else {
    return (pix * NCH + chunk) << 4;
  }
}

// NCH = Cin / 8 (1, 2, 4, 6, 8, 12); NCT = 16-column output tiles (1..4)
template <int NCH, int NCT>
__global__ __launch_bounds__(256) void conv2d_small_kernel(const C2Args p) {
  constexpr int CIN = 8 * NCH;
  extern __shared__ __attribute__((aligned(16))) char patch[];  // [PH * PW pixels][NCH chunks] (pslot)
  const int d = p.dil, st = p.stride;
  const int PH = (HT - 1) * st + 1 + 2 * d, PW = (WT - 1) * st + 1 + 2 * d, PPIX = PH * PW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int tw = (p.Wo + WT - 1) / WT, th = (p.Ho + HT - 1) / HT;
  int b = blockIdx.x;
  const int bx = b % tw;
  b /= tw;
  const int by = b % th;
  const int n = b / th;
  const int x0 = bx * WT, y0 = by * HT;
  const int nch0 = p.c0 >> 3;

  // ---- input patch -> LDS (zero padding outside the image), 8 loads of a thread in flight before their stores ----
  constexpr int LB = 8;
  const int npiece = PPIX * NCH;
  for (int k0 = 0; k0 < npiece; k0 += 256 * LB) {
    half8 pv[LB];
#pragma unroll
    for (int k = 0; k < LB; ++k) {
      const int i = k0 + tid + 256 * k;
      const int pix = i / NCH, c = i - pix * NCH;
      const int py = pix / PW, px = pix - py * PW;
      const int y = y0 * st - d + py, x = x0 * st - d + px;
#pragma unroll
      for (int j = 0; j < 8; ++j) pv[k][j] = (f16)0.f;
      if (i < npiece && (unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W) {
        const long q = ((long)n * p.H + y) * p.W + x;
        pv[k] = c < nch0 ? *reinterpret_cast<const half8*>(p.x0 + q * p.xs0 + 8 * c)
                         : *reinterpret_cast<const half8*>(p.x1 + q * p.xs1 + 8 * (c - nch0));
      }
    }
#pragma unroll
    for (int k = 0; k < LB; ++k) {
      const int i = k0 + tid + 256 * k;
      if (i < npiece) *reinterpret_cast<half8*>(patch + pslot<NCH>(i / NCH, i % NCH)) = pv[k];
    }
  }
  __syncthreads();

  // ---- K loop: wave w owns fragments 4w .. 4w + 3 (fragment f: output row f / 2, columns 16 (f % 2) .. + 15) ----
  int fbase[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int f = 4 * wave + i;
    fbase[i] = ((f / 2) * PW + (f % 2) * 16 + r16) * st;
  }
  floatx4 acc[4][NCT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NCT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  constexpr int NK = (9 * CIN + 31) / 32;  // k-steps holding real taps (the packed K padding beyond is zero)
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
    const int u = 4 * ks + g;  // this lane's chunk of the (tap, chunk) sequence
    const int tap = u / NCH, c = u - tap * NCH;
    const bool live = tap < 9;
    const int toff = ((tap / 3) * PW + tap % 3) * d;
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

  // ---- epilogue: lane (r16, g) holds output channels 16 j + 4 g .. + 3 of pixel r16 of each fragment ----
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int f = 4 * wave + i;
    const int y = y0 + f / 2, x = x0 + (f % 2) * 16 + r16;
    if (y >= p.Ho || x >= p.Wo) continue;
    const long pix = ((long)n * p.Ho + y) * p.Wo + x;
#pragma unroll
    for (int j = 0; j < NCT; ++j) {
      const int co = 16 * j + 4 * g;
      if (co >= p.Cout) continue;
      const bool full = co + 4 <= p.Cout;
      half4 r4;
      if (p.res && full) r4 = *reinterpret_cast<const half4*>(p.res + pix * p.rs + co);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cc = co + r;
        v[r] = act_apply(acc[i][j][r] * p.scale + (p.bias && cc < p.Cout ? p.bias[cc] : 0.f), p.act, p.alpha);
        if (p.res && cc < p.Cout) v[r] = act_apply(v[r] + (float)(full ? r4[r] : p.res[pix * p.rs + cc]), p.act2, p.alpha);
      }
      if (p.cout_real > 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int cj = co + r;
          if (cj >= p.Cout) break;
          const int pi = cj / p.cout_real, c = cj - pi * p.cout_real;
          const long opix = ((long)n * 2 * p.Ho + 2 * y + ((pi >> 1) & 1)) * 2 * p.Wo + 2 * x + (pi & 1);
          if (p.out_f32) reinterpret_cast<float*>(p.out)[opix * p.os + c] = v[r];
          else p.out[opix * p.os + c] = (f16)v[r];
        }
      } else if (p.out_f32) {
        float* op = reinterpret_cast<float*>(p.out) + pix * p.os + co;
        typedef float floatx2 __attribute__((ext_vector_type(2)));
        if (full) {  // two 8-B stores: fp32 rows of an even (not necessarily 4-aligned) width, e.g. HITNet's 34
          reinterpret_cast<floatx2*>(op)[0] = floatx2{v[0], v[1]};
          reinterpret_cast<floatx2*>(op)[1] = floatx2{v[2], v[3]};
        } else
          for (int r = 0; co + r < p.Cout; ++r) op[r] = v[r];
      } else {
        f16* op = p.out + pix * p.os + co;
        if (full) {
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
}

template <int NCH>
int launch_nct(const C2Args& a, dim3 grid, hipStream_t s) {
  const unsigned lds = (unsigned)(((HT - 1) * a.stride + 1 + 2 * a.dil) * ((WT - 1) * a.stride + 1 + 2 * a.dil) * NCH * 16);
  if (lds > 102400) return -2;  // stride 2 with many channels: the 17 x 65 patch
  switch ((a.Cout + 15) / 16) {
    case 1: hipLaunchKernelGGL((conv2d_small_kernel<NCH, 1>), grid, dim3(256), lds, s, a); break;
    case 2: hipLaunchKernelGGL((conv2d_small_kernel<NCH, 2>), grid, dim3(256), lds, s, a); break;
    case 3: hipLaunchKernelGGL((conv2d_small_kernel<NCH, 3>), grid, dim3(256), lds, s, a); break;
    default: hipLaunchKernelGGL((conv2d_small_kernel<NCH, 4>), grid, dim3(256), lds, s, a); break;
  }
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int sa_conv2d_small(const void* x0, int xs0, int c0, const void* x1, int xs1, int Cin, const void* w,
                               int Kpad, const float* bias, void* out, int os, int N, int H, int W, int Cout, int act,
                               float alpha, float scale, const void* res, int rs, int act2, int dil, int out_f32,
                               int cout_real, int stride, hipStream_t stream) {
  if (!(stride == 1 || (stride == 2 && dil == 1 && !cout_real))) return -2;
  if (!(dil == 1 || dil == 2 || dil == 4) || (out_f32 && !cout_real && (res || os % 2))) return -2;
  if (cout_real > 0 && (res || Cout != 4 * cout_real)) return -2;
  if (!(Cin == 8 || Cin == 16 || Cin == 32 || Cin == 48 || Cin == 64 || Cin == 96) || Cout < 1 || Cout > 64 ||
      Kpad % 32 ||
      Kpad < 9 * Cin)
    return -2;
  if (c0 < 8 || c0 % 8 || c0 > Cin || (c0 < Cin && !x1)) return -2;
  if (xs0 % 8 || ((uintptr_t)x0 & 15) || (x1 && (xs1 % 8 || ((uintptr_t)x1 & 15))) ||
      (!out_f32 && !cout_real && os % 4) || (!cout_real && ((uintptr_t)out & 7)) ||
      ((uintptr_t)w & 15) || (res && (rs % 4 || ((uintptr_t)res & 7))))
    return -2;
  if (N < 1 || H < 1 || W < 1) return -2;
  C2Args a{(const f16*)x0, xs0, c0, (const f16*)x1, xs1, (const f16*)w, Kpad, bias, (f16*)out, os, N, H, W, Cout,
           act, alpha, scale, (const f16*)res, rs, act2, dil, out_f32, stride, (H - 1) / stride + 1,
           (W - 1) / stride + 1, cout_real};
  const long blocks = (long)N * ((a.Ho + HT - 1) / HT) * ((a.Wo + WT - 1) / WT);
  if (blocks > 0x7fffffffL) return -2;
  const dim3 grid((unsigned)blocks);
  switch (Cin / 8) {
    case 1: return launch_nct<1>(a, grid, stream);
    case 2: return launch_nct<2>(a, grid, stream);
    case 4: return launch_nct<4>(a, grid, stream);
    case 6: return launch_nct<6>(a, grid, stream);
    case 8: return launch_nct<8>(a, grid, stream);
    default: return launch_nct<12>(a, grid, stream);
  }
}
