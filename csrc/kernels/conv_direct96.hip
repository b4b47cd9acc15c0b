// Direct 3x3 convolution to 96 channels, pad 1 (tile_cfg 24): 96 -> 96 at stride 1, the 1/2-resolution layer2
// convs of the RAFT-Stereo / CREStereo encoders (three per trunk), and 64 -> 96 at stride 2 (layer2.0.conv1).  The implicit GEMM runs them at ~0.3 PFLOP/s at
// RAFT-SF b8 (682 us per call, profiles/r02_sf_b8_serial_kernels.txt): K = 864 is only 14 64-deep k-steps per
// tile epilogue and N = 96 leaves a quarter of every 128-wide tile idle.  Same scheme as the 64-channel direct
// conv v2 (conv_direct.hip):
//   * persistent workgroups (one per CU), each walking a contiguous run of 2 x 32-pixel output tiles whose
//     input (4 x 34 pixels x 192 B) is DMA'd global->LDS (global_load_lds_dwordx4) into a 4-deep ring with an
//     exact counted vmcnt (every wave issues the same vector-memory ops per tile: out-of-range stores are
//     dropped by the buffer descriptor's range check);
//   * 12 waves (3 per SIMD): wave w owns pixel row w / 6 of the tile (2 pixel fragments of 16) x output
//     channels (w % 6) * 16 .. +16, whose 27 k-steps of weights stay in registers as the MFMA A operand
//     (C^T = W * X^T), so each lane ends with 4 consecutive channels of one pixel: one 8-B store per fragment;
//   * 192-B pixel rows, 16-B chunk c stored at c ^ ((pixel >> 2) & 3): the 16 lanes of a ds_read_b128 phase
//     (16 consecutive pixels, one chunk) cover all 64 banks;
//   * optional instance-norm statistics (per-lane running sums in LDS, DPP row reduction, the two pixel rows
//     of a channel group summed in LDS before the slotted fixed-point atomics, once per image change) or a
//     residual epilogue y = act2(act(acc + b) + res).
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdlib>

#include "sa/kernels.h"

namespace {

typedef _Float16 f16;
typedef f16 half4 __attribute__((ext_vector_type(4)));
typedef f16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned uint2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int C = 96;                          // output channels
constexpr int TR = 2, TC = 32;                 // output tile
constexpr int NW = 12;
constexpr int PF = TC / 16;                    // 2 pixel fragments per wave

// staged-input geometry for CIN input channels at stride S (96 / 1: the layer2 convs; 64 / 2: layer2.0.conv1)
template <int CIN, int S>
struct Geo {
  static constexpr int IR = (TR - 1) * S + 3, IC = (TC - 1) * S + 3;  // input tile with halo (4 x 34 / 5 x 65)
  static constexpr int PB = CIN * 2;                                  // bytes per staged pixel
  static constexpr int CH = CIN / 8;                                  // 16-B chunks per pixel
  static constexpr int PIECES = IR * IC * CH;                         // 1632 / 2600
  static constexpr int INSTR = (PIECES + 63) / 64;                    // DMA wave-instructions per tile (26 / 41)
  static constexpr int BUF = INSTR * 1024;                            // the last instruction's spare lanes: pad
  static constexpr int PER_WAVE = (INSTR + NW - 1) / NW;              // 3 / 4
  static constexpr int KS = 9 * CIN / 32;                             // k-steps (27 / 18)
  static constexpr int NB = S == 1 ? 4 : 3;                           // ring depth
  static constexpr int DUMMY = NB * BUF;
  static constexpr int BIAS = DUMMY + 1024;
  static constexpr int ST = BIAS + C * 4;                             // per-lane IN sums [sum 4 | sumsq 4][768]
  static constexpr int RED = ST + NW * 64 * 32;                       // flush: [12 waves][4 kq][8]
  static constexpr int SMEM = RED + NW * 4 * 8 * 4;
  static_assert(SMEM <= 163840, "LDS budget");
  // 16-B chunk swizzle.  96 channels (12 chunks, 192-B rows), stride 1: c ^ ((pixel >> 2) & 3) keeps a chunk in
  // its aligned group of 4 and spreads 16 consecutive pixels over all 64 banks.  64 channels (128-B rows),
  // stride 2: the 16 lanes read every other pixel, c ^ ((pixel >> 1) & 7) leaves a 2-way conflict (8 chunk
  // slots per half of the banks, 16 lanes)
  static __device__ __forceinline__ int swz(int pp) { return CIN == 96 ? (pp >> 2) & 3 : (pp >> 1) & 7; }
};

__device__ __attribute__((aligned(16))) const unsigned char g_zero16c[64] = {0};

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

__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
#define SA_VM(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    SA_VM(0) SA_VM(1) SA_VM(2) SA_VM(3) SA_VM(4) SA_VM(5) SA_VM(6) SA_VM(7) SA_VM(8) SA_VM(9) SA_VM(10)
    SA_VM(11) SA_VM(12) SA_VM(13) SA_VM(14) SA_VM(15) SA_VM(16) SA_VM(17) SA_VM(18) SA_VM(19) SA_VM(20)
    SA_VM(21) SA_VM(22) SA_VM(23) SA_VM(24)
#undef SA_VM
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

struct D96Args {
  const f16* x;
  int xs;
  const f16* w;
  int kpad;
  const float* bias;
  f16* out;
  int os;
  unsigned out_bytes, res_bytes;
  int N, H, W, Ho, Wo;
  int act;
  float alpha;
  sa_stat_t* stats;
  int slots;
  const f16* res;
  int rs;
  int act2;
};

template <int CIN, int S, bool STATS, bool RES>
__global__ __launch_bounds__(768, 1) void conv3x3_c96_direct_kernel(const D96Args p) {
  using Gm = Geo<CIN, S>;
  constexpr int IC = Gm::IC, CH = Gm::CH, PIECES = Gm::PIECES, INSTR = Gm::INSTR, BUF = Gm::BUF;
  constexpr int PER_WAVE = Gm::PER_WAVE, KS = Gm::KS, NB = Gm::NB, PB = Gm::PB;
  constexpr int DUMMY = Gm::DUMMY, BIAS = Gm::BIAS, ST = Gm::ST, RED = Gm::RED;
  __shared__ __attribute__((aligned(16))) char smem[Gm::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, kq = lane >> 4;
  const int tiles_x = (p.Wo + TC - 1) / TC, tiles_y = (p.Ho + TR - 1) / TR;
  const int tiles_img = tiles_x * tiles_y;
  const int ntiles = p.N * tiles_img;
  const void* zero = g_zero16c;

  auto issue_tile = [&](int t, int buf) {
    const int n = t / tiles_img, r = t - n * tiles_img;
    const int ty = r / tiles_x, tx = r - ty * tiles_x;
    const int y0 = ty * TR * S - 1, x0 = tx * TC * S - 1;
    char* ib = smem + buf * BUF;
    int ln = lane;
    asm volatile("" : "+v"(ln));  // no hoisting of the tile-invariant piece decomposition (see conv_direct.hip)
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int ins = i * NW + wave;
      const void* src = zero;
      char* dst = smem + DUMMY;
      if (ins < INSTR) {
        const int g = ins * 64 + ln;
        const int pp = g / CH, sl = g - pp * CH;
        const int q = sl ^ Gm::swz(pp);
        const int iy = y0 + pp / IC, ix = x0 + pp % IC;
        if (g < PIECES && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W)
          src = p.x + ((size_t)((size_t)n * p.H + iy) * p.W + ix) * p.xs + q * 8;
        dst = ib + ins * 1024;
      }
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)dst, 16, 0, 0);
    }
  };

  const int prow = wave / 6, cg = wave - prow * 6;
  half8 wa[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    wa[ks] = *reinterpret_cast<const half8*>(p.w + (size_t)(cg * 16 + frow) * p.kpad + ks * 32 + kq * 8);
  const int c0 = cg * 16 + kq * 4;  // this lane's 4 output channels
  float* bias_lds = reinterpret_cast<float*>(smem + BIAS);
  if (tid < C) bias_lds[tid] = p.bias ? p.bias[tid] : 0.f;

  // [sum 0-3 | sq 0-3][768 lanes]: contiguous 16-B accesses per wave (the lane-major [768][2] layout put lanes 8
  // apart on the same banks: 2-way on every statistics ds_read / ds_write_b128)
  struct StLane {
    floatx4* b;
    __device__ floatx4& operator[](int v) const { return b[v * 768]; }
  } st_lane{reinterpret_cast<floatx4*>(smem + ST) + tid};
  if constexpr (STATS) st_lane[0] = st_lane[1] = floatx4{0.f, 0.f, 0.f, 0.f};
  int stat_img = -1;
  auto flush_stats = [&]() {
    if constexpr (STATS) {
      float f[8];
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const floatx4 x4 = st_lane[v];
        st_lane[v] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 4; ++u) f[v * 4 + u] = row16_sum(x4[u]);
      }
      float* red = reinterpret_cast<float*>(smem + RED);
      if (frow == 0)
#pragma unroll
        for (int e = 0; e < 8; ++e) red[(wave * 4 + kq) * 8 + e] = f[e];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (prow == 0 && frow == 0 && stat_img >= 0) {
        sa_stat_t* st = p.stats + (size_t)(blockIdx.x % (p.slots > 1 ? p.slots : 1)) * p.N * C * 2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float s0 = red[(wave * 4 + kq) * 8 + e] + red[((wave + 6) * 4 + kq) * 8 + e];
          const float s1 = red[(wave * 4 + kq) * 8 + 4 + e] + red[((wave + 6) * 4 + kq) * 8 + 4 + e];
          unsigned long long* sp = reinterpret_cast<unsigned long long*>(st) + ((size_t)stat_img * C + c0 + e) * 2;
          atomicAdd(sp, (unsigned long long)__double2ll_rn((double)s0 * SA_STAT_SCALE));
          atomicAdd(sp + 1, (unsigned long long)__double2ll_rn((double)s1 * SA_STAT_SCALE));
        }
      }
    }
  };
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(p.out, 0, p.out_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rrsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(p.res), 0, RES ? p.res_bytes : 0, 0x00020000);

  const int G = gridDim.x;
  const int per = (ntiles + G - 1) / G;
  const int t0 = blockIdx.x * per;
  const int kb = t0 < ntiles ? (ntiles - t0 < per ? ntiles - t0 : per) : 0;
#pragma unroll
  for (int k = 0; k < NB - 1; ++k)
    if (k < kb) issue_tile(t0 + k, k);

  for (int k = 0; k < kb; ++k) {
    const int t = t0 + k;
    const int cur = k % NB;
    const int ahead = (kb - 1 - k) < NB - 2 ? (kb - 1 - k) : NB - 2;
    constexpr int kOps = RES ? 2 * PF : PF;  // stores (+ residual loads) per tile, never skipped
    wait_vmcnt(ahead * PER_WAVE + (k < NB - 1 ? k : NB - 1) * kOps);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int n = t / tiles_img, rr = t - n * tiles_img;
    const int ty = rr / tiles_x, tx = rr - ty * tiles_x;
    const int oy = ty * TR + prow;
    half4 rv[PF];  // (residual pixels are output pixels)
    if constexpr (RES) {
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const int ox = tx * TC + i * 16 + frow;
        const bool ok = oy < p.Ho && ox < p.Wo;
        const size_t pix = ((size_t)n * p.Ho + oy) * p.Wo + ox;
        const unsigned roff = ok ? (unsigned)(pix * p.rs + c0) * 2u : 0xFFFFFFF0u;
        rv[i] = __builtin_bit_cast(half4, __builtin_amdgcn_raw_buffer_load_b64(rrsrc, roff, 0, 0));
      }
    }
    if (k + NB - 1 < kb) issue_tile(t + NB - 1, (k + NB - 1) % NB);
    const char* ib = smem + cur * BUF;

    floatx4 acc[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    // laundered per tile: the 54 fragment addresses are tile-invariant and the compiler would otherwise keep
    // them all live across the tile loop (spilling the weights)
    int fr = frow, kql = kq;
    asm volatile("" : "+v"(fr), "+v"(kql));
    auto load = [&](int ks, half8* bf) {
      constexpr int KPT = CIN / 32;  // k-steps per tap
      const int tap = ks / KPT, kh = tap / 3, kw = tap - kh * 3;
      const int q = (ks - tap * KPT) * 4 + kql;
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const int pp = (prow * S + kh) * IC + (i * 16 + fr) * S + kw;
        bf[i] = *reinterpret_cast<const half8*>(ib + pp * PB + ((q ^ Gm::swz(pp)) << 4));
      }
    };
    // one k-step of fragments in flight under the MFMAs of the previous one; the memory clobber per k-step keeps
    // the compiler from hoisting all 27 k-steps' LDS reads (the register file is 168 VGPRs at 3 waves per SIMD,
    // 108 of them the stationary weights)
    half8 b0[PF], b1[PF];
    load(0, b0);
#pragma unroll
    for (int ks = 0; ks < KS; ks += 2) {
      if (ks + 1 < KS) load(ks + 1, b1);
#pragma unroll
      for (int i = 0; i < PF; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[ks], b0[i], acc[i], 0, 0, 0);
      asm volatile("" ::: "memory");
      if (ks + 1 < KS) {
        if (ks + 2 < KS) load(ks + 2, b0);
#pragma unroll
        for (int i = 0; i < PF; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[ks + 1], b1[i], acc[i], 0, 0, 0);
        asm volatile("" ::: "memory");
      }
    }

    if constexpr (STATS) {
      if (n != stat_img) {
        if (stat_img >= 0) flush_stats();
        stat_img = n;
      }
    }
    const floatx4 bias4 = *reinterpret_cast<const floatx4*>(bias_lds + c0);
    float tsum[4] = {0.f, 0.f, 0.f, 0.f}, tsq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int ox = tx * TC + i * 16 + frow;
      const bool ok = oy < p.Ho && ox < p.Wo;
      const size_t pix = ((size_t)n * p.Ho + oy) * p.Wo + ox;
      half4 h;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = act_apply(acc[i][r] + bias4[r], p.act, p.alpha);
        if constexpr (RES) v = p.act2 == SA_ACT_RELU ? fmaxf(v + (float)rv[i][r], 0.f) : v + (float)rv[i][r];
        h[r] = (f16)v;
        if constexpr (STATS) {
          const float vm = ok ? v : 0.f;
          tsum[r] += vm;
          tsq[r] = fmaf(vm, vm, tsq[r]);
        }
      }
      const unsigned off = ok ? (unsigned)(pix * p.os + c0) * 2u : 0xFFFFFFF0u;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, h), orsrc, off, 0, 0);
    }
    if constexpr (STATS) {
      st_lane[0] += floatx4{tsum[0], tsum[1], tsum[2], tsum[3]};
      st_lane[1] += floatx4{tsq[0], tsq[1], tsq[2], tsq[3]};
    }
  }
  if constexpr (STATS) {
    if (stat_img >= 0) flush_stats();
  }
}

}  // namespace

extern "C" int sa_conv3x3_c96_direct(const void* x, int xs, int cin, int stride, const void* w, int kpad,
                                     const float* bias, void* out, int os, int N, int H, int W, int act, float alpha,
                                     sa_stat_t* stats, int slots, const void* res, int rs, int act2,
                                     hipStream_t stream) {
  if (!((cin == 96 && stride == 1) || (cin == 64 && stride == 2))) return -5;
  if (kpad < 9 * cin || xs < cin || os < C || xs % 8 || os % 4 ||
      (act != SA_ACT_NONE && act != SA_ACT_RELU && act != SA_ACT_LEAKY))
    return -2;
  if (res && (stats || rs < C || rs % 4 || (act2 != SA_ACT_NONE && act2 != SA_ACT_RELU))) return -5;
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const size_t last = ((size_t)N * Ho - 1) * Wo + (Wo - 1);
  const size_t span = last * (size_t)os * 2 + 2 * C, rspan = res ? last * (size_t)rs * 2 + 2 * C : 0;
  if (span >= 0xFFFFFF00ull || rspan >= 0xFFFFFF00ull) return -5;
  D96Args a{(const f16*)x, xs, (const f16*)w, kpad, bias, (f16*)out, os, (unsigned)span, (unsigned)rspan, N, H, W, Ho,
            Wo, act, alpha, stats, slots, (const f16*)res, rs, act2};
  const long ntiles = (long)N * ((Ho + TR - 1) / TR) * ((Wo + TC - 1) / TC);
  long g = 256;
  if (g > ntiles) g = ntiles;
  if (g < 1) return 0;
  const dim3 grid((unsigned)g), block(768);
  if (cin == 96) {
    if (stats) hipLaunchKernelGGL((conv3x3_c96_direct_kernel<96, 1, true, false>), grid, block, 0, stream, a);
    else if (res) hipLaunchKernelGGL((conv3x3_c96_direct_kernel<96, 1, false, true>), grid, block, 0, stream, a);
    else hipLaunchKernelGGL((conv3x3_c96_direct_kernel<96, 1, false, false>), grid, block, 0, stream, a);
  } else {
    if (stats) hipLaunchKernelGGL((conv3x3_c96_direct_kernel<64, 2, true, false>), grid, block, 0, stream, a);
    else if (res) hipLaunchKernelGGL((conv3x3_c96_direct_kernel<64, 2, false, true>), grid, block, 0, stream, a);
    else hipLaunchKernelGGL((conv3x3_c96_direct_kernel<64, 2, false, false>), grid, block, 0, stream, a);
  }
  return (int)hipGetLastError();
}
