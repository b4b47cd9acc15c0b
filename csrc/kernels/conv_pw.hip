// Pointwise (1x1, stride 1) convolution for narrow GEMMs (tactic 35): Cin <= 256 from one or two channel-concatenated
// sources, Cout <= 256; also the k = 2 / s = 2 transposed conv as a 1x1 conv with the parity scatter (HITNet's
// upsampling).
//
// Fast-ACVNet+'s MobileNetV2 feature extractor expands 16 -> 96, 24 -> 144, 32 -> 192 channels and projects back
// 144 -> 24, 192 -> 32 with 1x1 convs (/root/reference/README_en.md:293-295 times the whole network at 12 ms on an
// RTX 3090).  As implicit GEMMs those are K = 16-32 or N = 24-32 problems on 128-wide tiles: the expand at 1/2
// resolution (153600 pixels, 16 -> 96) took 47 us for 34 MB of traffic that HBM moves in 7 (profiles/round6_notes.md).
//
// Here one wave owns 16 pixels and ALL (<= 256) Cout columns: the product is transposed (C^T = W X^T), so the weights are the
// MFMA A operand, the pixels' 8-channel chunks the B operand (one 16-B load per lane per k-step straight from the
// NHWC input), and a lane ends with 4 consecutive output channels of one pixel per 16-column tile: one 8-B store
// each, the 4 lane groups of a pixel writing 64 contiguous bytes.  Weight fragments come from global memory (<= 96 KB,
// L1 / L2 resident) and are issued for the whole k-step before its MFMAs.  Epilogue: bias, activation, optional
// residual add (+ second activation).
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>

#include "sa/kernels.h"

namespace {

typedef _Float16 f16;
typedef f16 half8 __attribute__((ext_vector_type(8)));
typedef f16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

struct PwArgs {
  const f16* x;
  int xs;       // input pixel stride (elements)
  int c0;       // channels of x (the rest, Cin - c0, come from x1)
  const f16* x1;
  int xs1;
  int Cin;      // input channels (multiple of 8)
  const f16* w;  // packed [Cout_pad][Kpad]
  int Kpad;
  const float* bias;
  f16* out;
  int os;
  long M;  // pixels
  int Cout;
  int act;
  float alpha, scale;
  const f16* res;
  int rs;
  int act2;
  int H, W;       // the M pixels are N x H x W (up: output H, W doubled)
  int cout_real;  // up == 2: Cout = 4 parity classes of cout_real channels, scattered to the 2x output (ConvTranspose
                  // k = 2, s = 2 as a 1x1 conv; class pi -> row parity pi >> 1, column parity pi & 1)
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

// NN = 16-column output tiles (Cout <= 16 NN)
template <int NN>
__global__ __launch_bounds__(256) void conv_pw_kernel(const PwArgs p) {
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15, g = lane >> 4;
  const long tile = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long px0 = tile * 16;
  if (px0 >= p.M) return;  // wave-uniform
  const long px = px0 + r16;
  const bool pv = px < p.M;
  const f16* xrow = p.x + (pv ? px : 0) * p.xs;
  floatx4 acc[NN];
#pragma unroll
  for (int j = 0; j < NN; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nk = (p.Cin + 31) / 32;
  for (int kt = 0; kt < nk; ++kt) {
    const int c = kt * 32 + g * 8;  // this lane's 8 k-values: channels c .. c + 7 of pixel px
    half8 b;
    if (pv && c < p.c0) {
      b = *reinterpret_cast<const half8*>(xrow + c);
    } else if (pv && c < p.Cin) {
      b = *reinterpret_cast<const half8*>(p.x1 + px * p.xs1 + (c - p.c0));
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) b[e] = (f16)0.f;
    }
    half8 a[NN];
#pragma unroll
    for (int j = 0; j < NN; ++j)  // weight rows 16 j + r16 (zero-padded to 128), k-values kt * 32 + 8 g
      a[j] = *reinterpret_cast<const half8*>(p.w + (size_t)(16 * j + r16) * p.Kpad + kt * 32 + g * 8);
#pragma unroll
    for (int j = 0; j < NN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[j], b, acc[j], 0, 0, 0);
  }
  // lane (r16, g) holds output channels 16 j + 4 g .. + 3 of pixel px0 + r16
  if (!pv) return;
  if (p.cout_real > 0) {  // transposed 1x1: channel cj -> parity class cj / cout_real of the 2x output
    const long hw = (long)p.H * p.W;
    const long nimg = px / hw, r = px - nimg * hw;
    const int oh = (int)(r / p.W), ow = (int)(r - (long)oh * p.W);
#pragma unroll
    for (int j = 0; j < NN; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int cj = 16 * j + 4 * g + i;
        if (cj >= p.Cout) continue;
        const int pi = cj / p.cout_real, c = cj - pi * p.cout_real;
        const long opix = (nimg * 2 * p.H + 2 * oh + ((pi >> 1) & 1)) * 2 * p.W + 2 * ow + (pi & 1);
        const float v = act_apply(acc[j][i] * p.scale + (p.bias ? p.bias[cj] : 0.f), p.act, p.alpha);
        p.out[opix * p.os + c] = (f16)v;
      }
    return;
  }
  f16* orow = p.out + px * p.os;
  const f16* rrow = p.res ? p.res + px * p.rs : nullptr;
#pragma unroll
  for (int j = 0; j < NN; ++j) {
    const int co = 16 * j + 4 * g;
    if (co >= p.Cout) continue;
    float v[4];
    half4 r4;
    if (rrow && co + 4 <= p.Cout) r4 = *reinterpret_cast<const half4*>(rrow + co);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cc = co + i;
      v[i] = act_apply(acc[j][i] * p.scale + (p.bias && cc < p.Cout ? p.bias[cc] : 0.f), p.act, p.alpha);
      if (rrow && cc < p.Cout)
        v[i] = act_apply(v[i] + (float)(co + 4 <= p.Cout ? r4[i] : rrow[cc]), p.act2, p.alpha);
    }
    if (co + 4 <= p.Cout) {
      half4 h;
#pragma unroll
      for (int i = 0; i < 4; ++i) h[i] = (f16)v[i];
      *reinterpret_cast<half4*>(orow + co) = h;
    } else {
      for (int i = 0; co + i < p.Cout; ++i) orow[co + i] = (f16)v[i];
    }
  }
}

template <int NN>
void launch_pw(const PwArgs& a, hipStream_t s) {
  const long tiles = (a.M + 15) / 16;
  hipLaunchKernelGGL((conv_pw_kernel<NN>), dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, s, a);
}

}  // namespace

extern "C" int sa_conv_pw(const void* x, int xs, int c0, const void* x1, int xs1, int Cin, const void* w, int Kpad,
                          const float* bias, void* out, int os, int N, int H, int W, int Cout, int act, float alpha,
                          float scale, const void* res, int rs, int act2, int cout_real, hipStream_t stream) {
  const long M = (long)N * H * W;
  if (Cin < 8 || Cin % 8 || Cin > 256 || Kpad < (Cin + 31) / 32 * 32 || Kpad % 32 || Cout < 1 || Cout > 256) return -2;
  if (c0 < 8 || c0 % 8 || c0 > Cin || (c0 < Cin && (!x1 || xs1 % 8 || ((uintptr_t)x1 & 15)))) return -2;
  if (cout_real > 0 && (res || Cout != 4 * cout_real)) return -2;
  if (xs % 8 || (cout_real == 0 && os % 4) || (res && rs % 4) || ((uintptr_t)x & 15) ||
      (cout_real == 0 && ((uintptr_t)out & 7)) || ((uintptr_t)w & 15) || (res && ((uintptr_t)res & 7)) || M < 1)
    return -2;
  if ((M + 63) / 64 > 0x7fffffffL) return -2;
  PwArgs a{(const f16*)x, xs, c0, (const f16*)x1, xs1, Cin, (const f16*)w, Kpad, bias, (f16*)out, os, M, Cout, act,
           alpha, scale, (const f16*)res, rs, act2, H, W, cout_real};
  switch ((Cout + 15) / 16) {
    case 1: launch_pw<1>(a, stream); break;
    case 2: launch_pw<2>(a, stream); break;
    case 3: launch_pw<3>(a, stream); break;
    case 4: launch_pw<4>(a, stream); break;
    case 5: launch_pw<5>(a, stream); break;
    case 6: launch_pw<6>(a, stream); break;
    case 7: launch_pw<7>(a, stream); break;
    case 8: launch_pw<8>(a, stream); break;
    case 9: launch_pw<9>(a, stream); break;
    case 10: launch_pw<10>(a, stream); break;
    case 11: launch_pw<11>(a, stream); break;
    case 12: launch_pw<12>(a, stream); break;
    case 13: launch_pw<13>(a, stream); break;
    case 14: launch_pw<14>(a, stream); break;
    case 15: launch_pw<15>(a, stream); break;
    default: launch_pw<16>(a, stream); break;
  }
  return (int)hipGetLastError();
}
