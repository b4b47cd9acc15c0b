// Direct 3x3 convolution, 64 -> 64 channels, stride 1, pad 1, weight-stationary with persistent output tiles
// (gfx950; tile_cfg 23).
//
// The implicit-GEMM kernels (conv2d.hip) gather every im2col row from L2 once per tap: for the
// full-resolution 64-channel layers of the RAFT-Stereo / CREStereo feature encoders (K = 576, only 9
// 64-deep k-steps) that is 9 reads of every input pixel per conv and the per-block prologue / epilogue
// dominate.  Here one persistent workgroup per CU holds the whole 64 x 576 weight matrix as MFMA fragments in
// VGPRs (loaded once) and walks output tiles of 2 rows x 64 columns: the input tile with its halo (4 x 66
// pixels x 64 channels) is DMA'd global->LDS (global_load_lds_dwordx4) into a ring several tiles ahead, and
// every tap's fragment is read from that tile (each input pixel crosses L2 ~2x instead of 9x).
//
// A first version ran one wave per SIMD (4 waves, 288 weight VGPRs each, LDS-staged epilogue); its ablations on
// the RAFT-SF b8 full-resolution layer put the MFMA + LDS-read loop alone at 0.83 PFLOP/s and the whole kernel
// at 0.40 (profiles/direct_conv_r02.txt): one wave per SIMD exposes every DMA wait, barrier and the epilogue.
// The kernel below replaced it.

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>


#include "sa/kernels.h"

namespace {

typedef _Float16 f16;
typedef f16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int TR = 2, TC = 64;                // output tile rows x cols
constexpr int IR = TR + 2, IC = TC + 2;       // input tile with halo
constexpr int KTOT = 576;                     // 3 * 3 * 64
constexpr int IN_BYTES = IR * IC * 128;       // 33792
constexpr int IN_PIECES = IR * IC * 8;        // 16-B pieces per input tile (2112)
constexpr int IN_INSTR = (IN_PIECES + 63) / 64;  // wave-instructions per tile (33)

__device__ __attribute__((aligned(16))) const unsigned char g_zero16d[64] = {0};
// padding source of the folded input norm (NIN): -65504 in fp16, which relu(IN(.)) maps to +0 for any statistics,
// i.e. the zero padding of the normalised input without a per-piece bounds test in the transform
__device__ __attribute__((aligned(16))) const unsigned short g_negmax16d[8] = {0xFBFF, 0xFBFF, 0xFBFF, 0xFBFF,
                                                                              0xFBFF, 0xFBFF, 0xFBFF, 0xFBFF};

// workgroup barrier that orders LDS only: __syncthreads() would also wait vmcnt(0), i.e. for the
// in-flight input DMA of the next tiles and for this tile's global stores to be acknowledged
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

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

// ---------------------------------------------------------------------------------------------------
// Two waves per SIMD:
//   * 8 waves per workgroup, one workgroup per CU: wave w owns 32 pixels (pixel group w & 3 of the
//     2 x 64 tile) x 32 output channels (half w >> 2), so the stationary weights are 144 VGPRs and two
//     waves share each SIMD (one computes while the other waits or stores);
//   * roles swapped (C^T = W * X^T): weights are the MFMA A operand, the staged input pixels the B
//     operand; the weight rows are permuted so that each lane ends up with 8 consecutive output
//     channels of one pixel -> one 16-B store per pixel fragment straight from the accumulators;
//   * stores are buffer stores (out-of-range pixels dropped by the descriptor's range check), so every
//     wave issues exactly the same vector-memory ops per tile and the counted vmcnt of the DMA ring is
//     exact (the wait above also counted the epilogue stores as ring pieces);
//   * LDS chunk swizzle by (pixel >> 1) & 7: the 16 lanes of one ds_read_b128 phase (16 consecutive
//     pixels, one 16-B chunk each) cover all 64 banks;
//   * one barrier per tile: DMA of tile t + 3 is issued right after the barrier that also retires the
//     reads of tile t - 1's buffer.
constexpr int V2_WAVES = 8;
constexpr int V2_PIECES = IN_INSTR;                                    // 33 DMA wave-instructions per tile
constexpr int V2_PER_WAVE = (V2_PIECES + V2_WAVES - 1) / V2_WAVES;     // 5 (waves 1..7: one dummy)
// LDS layout: NB ring buffers | 1 KB sink for the dummy pieces | 64 fp32 biases | (STATS) per-lane running
// IN sums [512 lanes][sum 8 | sumsq 8] -- in LDS, not VGPRs: 16 more live registers next to the 144 of the
// stationary weights made the compiler drop the fragment prefetch (a lgkmcnt(0) after every ds_read) |
// (NIN) the folded input norm's mean / rstd, [2 image slots][mean 64 | rstd 64] fp32
template <bool STATS, bool NIN = false>
struct V2Lds {
  static constexpr int NB = STATS ? 3 : 4;  // ring depth (3 leaves room for the statistics)
  static constexpr int DUMMY = NB * IN_BYTES;
  static constexpr int BIAS = DUMMY + 1024;
  static constexpr int ST = BIAS + 256;
  static constexpr int RED = ST + (STATS ? 512 * 64 : 0);  // flush: [8 waves][4 kq][16] wave totals
  static constexpr int NRM = RED + (STATS ? 8 * 4 * 16 * 4 : 0);
  static constexpr int SMEM = NRM + (NIN ? 2 * 128 * 4 : 0);
};

// sum over the 16 lanes of a DPP row (every lane gets the row total)
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
  return v;
}

__device__ __forceinline__ int v2_swz(int pp) { return (pp >> 1) & 7; }

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (0..31)
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
#define SA_VM(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    SA_VM(0) SA_VM(1) SA_VM(2) SA_VM(3) SA_VM(4) SA_VM(5) SA_VM(6) SA_VM(7) SA_VM(8) SA_VM(9) SA_VM(10)
    SA_VM(11) SA_VM(12) SA_VM(13) SA_VM(14) SA_VM(15) SA_VM(16) SA_VM(17) SA_VM(18) SA_VM(19) SA_VM(20)
#undef SA_VM
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

struct DirectArgs2 {
  const f16* x;
  int xs;
  const f16* w;
  int kpad;
  const float* bias;
  f16* out;
  int os;
  unsigned out_bytes;  // buffer-store range of `out`
  unsigned res_bytes;  // buffer-load range of `res`
  int N, H, W;
  float alpha;
  sa_stat_t* stats;
  int slots;
  const f16* res;  // optional residual (RES): y = act2(act(acc + bias) + res)
  int rs;
  int act2;
  // NIN: x is a conv's raw output with these slotted statistics ([in_slots][N][64][2]); the conv reads relu(IN(x))
  const sa_stat_t* in_stats;
  int in_slots;
  float in_eps;
  double in_inv;  // 1 / (H W SA_STAT_SCALE), from the host: a kernel argument (SGPRs), not a hoisted VGPR pair
};

// NIN (input instance norm folded in): the instance-norm residual blocks' conv2 reads conv1's
// RAW output and normalises it in LDS instead of a separate relu(IN(.)) pass over the full-resolution tensor (one
// HBM read + write of it).  Each wave transforms the 16-B pieces it DMA'd itself -- landed per its own vmcnt, no
// extra barrier -- for tile k+1 at the end of tile k (after the epilogue: the fragment and accumulator registers
// are free there, and the DMA of tile k+2 stays in flight); the loop-top barrier of tile k+1 publishes it.  The
// arithmetic is instnorm_apply's ((x - mean) * rstd, relu, round to fp16), so the conv sees bitwise the same input.
// Round 2 measured a transform phase of the round-2 kernel between two extra barriers as neutral
// (profiles/fused_input_norm_r02.txt).
template <int ACT, bool STATS, bool RES, bool NIN = false>
__global__ __launch_bounds__(512, 1) void conv3x3_c64_direct2_kernel(const DirectArgs2 p) {
  using L = V2Lds<STATS, NIN>;
  constexpr int NB = L::NB;
  __shared__ __attribute__((aligned(16))) char smem[L::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, kq = lane >> 4;
  const int tiles_x = (p.W + TC - 1) / TC, tiles_y = (p.H + TR - 1) / TR;
  const int tiles_img = tiles_x * tiles_y;
  const int ntiles = p.N * tiles_img;
  const void* zero = NIN ? (const void*)g_negmax16d : (const void*)g_zero16d;

  auto issue_tile = [&](int t, int buf) {
    const int n = t / tiles_img, r = t - n * tiles_img;
    const int ty = r / tiles_x, tx = r - ty * tiles_x;
    const int y0 = ty * TR - 1, x0 = tx * TC - 1;
    char* ib = smem + buf * IN_BYTES;
    // laundered lane index: keeps the compiler from hoisting the tile-invariant piece decomposition out of
    // the tile loop into ~20 long-lived VGPRs (which spilled, and a spill reload waits on the whole ring)
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < V2_PER_WAVE; ++i) {
      const int ins = i * V2_WAVES + wave;
      const void* src = zero;
      char* dst = smem + L::DUMMY;
      if (ins < V2_PIECES) {
        const int g = ins * 64 + ln;
        const int pp = g >> 3, s = g & 7;
        const int q = s ^ v2_swz(pp);
        const int iy = y0 + pp / IC, ix = x0 + pp % IC;
        if (g < IN_PIECES && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W)
          src = p.x + ((size_t)((size_t)n * p.H + iy) * p.W + ix) * p.xs + q * 8;
        dst = ib + ins * 1024;
      }
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)dst, 16, 0, 0);
    }
  };

  // wave roles: pixel group pg (row pg >> 1 of the tile, columns (pg & 1) * 32 .. +32), channel half hc
  const int pg = wave & 3, hc = wave >> 2;
  const int prow = pg >> 1, pcol = (pg & 1) * 32;
  // A fragments: row rr of fragment j = output channel hc*32 + (rr >> 2) * 8 + j * 4 + (rr & 3)
  half8 wa[KTOT / 32][2];
#pragma unroll
  for (int ks = 0; ks < KTOT / 32; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = hc * 32 + (frow >> 2) * 8 + j * 4 + (frow & 3);
      wa[ks][j] = *reinterpret_cast<const half8*>(p.w + (size_t)co * p.kpad + ks * 32 + kq * 8);
    }
  // this lane's 8 output channels: hc*32 + kq*8 + e, e = 4 j + r
  const int c0 = hc * 32 + kq * 8;
  // instance-norm statistics: per-lane running sums of the lane's 8 channels over its pixels, across tiles
  // of one image; row-reduced with DPP and flushed to the slotted fixed-point atomics when the image changes
  // [sum 0-3 | sum 4-7 | sq 0-3 | sq 4-7][512 lanes]: a wave's 16-B accesses are contiguous (conflict-free); the
  // lane-major [512][4] layout put lanes 4 apart on the same banks (4-way on every ds_read / ds_write_b128):
  // fr8 with statistics 552.7 -> 545.6 us, l1b8 139.9 -> 138.7 us (conv_bench, profiles/round6_notes.md)
  struct StLane {
    floatx4* b;
    __device__ floatx4& operator[](int v) const { return b[v * 512]; }
  } st_lane{reinterpret_cast<floatx4*>(smem + L::ST) + tid};
  if constexpr (STATS) {
#pragma unroll
    for (int v = 0; v < 4; ++v) st_lane[v] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  int stat_img = -1;
  auto flush_stats = [&]() {
    if constexpr (STATS) {
      float f[16];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const floatx4 x4 = st_lane[v];
        st_lane[v] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 4; ++u) f[v * 4 + u] = row16_sum(x4[u]);
      }
      // the four waves of a channel half (pixel groups 0..3) are summed in LDS in a fixed order: a quarter of
      // the atomics (block-uniform: every wave flushes at the same tile)
      float* red = reinterpret_cast<float*>(smem + L::RED);
      if (frow == 0)
#pragma unroll
        for (int e = 0; e < 16; ++e) red[(wave * 4 + kq) * 16 + e] = f[e];
      lds_barrier();
      if (pg == 0 && frow == 0 && stat_img >= 0) {
#pragma unroll
        for (int e = 0; e < 16; ++e)
          f[e] = red[((wave + 0) * 4 + kq) * 16 + e] + red[((wave + 1) * 4 + kq) * 16 + e] +
                 red[((wave + 2) * 4 + kq) * 16 + e] + red[((wave + 3) * 4 + kq) * 16 + e];
        sa_stat_t* st = p.stats + (size_t)(blockIdx.x % (p.slots > 1 ? p.slots : 1)) * p.N * 64 * 2;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          unsigned long long* sp = reinterpret_cast<unsigned long long*>(st) + ((size_t)stat_img * 64 + c0 + e) * 2;
          atomicAdd(sp, (unsigned long long)__double2ll_rn((double)f[e] * SA_STAT_SCALE));
          atomicAdd(sp + 1, (unsigned long long)__double2ll_rn((double)f[8 + e] * SA_STAT_SCALE));
        }
      }
    }
  };
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(p.out, 0, p.out_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rrsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(p.res), 0, RES ? p.res_bytes : 0, 0x00020000);
  // biases staged in LDS: an epilogue global load would make the compiler wait for the whole DMA ring
  // (vmcnt counts in issue order); the first loop barrier publishes them
  float* bias_lds = reinterpret_cast<float*>(smem + L::BIAS);
  if (tid < 64) bias_lds[tid] = p.bias ? p.bias[tid] : 0.f;

  // each workgroup walks a contiguous run of tiles (row-major within an image): an image boundary is crossed
  // at most once or twice per workgroup, so the statistics flushes (whose atomics, when every workgroup
  // crossed images in lockstep under a grid stride, cost 150 us of 800 at RAFT-SF b8) are rare and spread out,
  // and vertically adjacent tiles (10 apart) reuse their halo rows from the same XCD's L2
  const int G = gridDim.x;
  const int per = (ntiles + G - 1) / G;
  const int t0 = blockIdx.x * per;
  const int kb = t0 < ntiles ? (ntiles - t0 < per ? ntiles - t0 : per) : 0;  // tiles of this workgroup
#pragma unroll
  for (int k = 0; k < NB - 1; ++k)
    if (k < kb) issue_tile(t0 + k, k);

  // NIN: per-image mean / rstd into LDS slot (n & 1) (the arithmetic of elementwise.hip norm_lds: integer sums over
  // the slots, then double), block-uniform call
  float* nrm = reinterpret_cast<float*>(smem + L::NRM);
  int nrm_img = -1;
  auto nrm_load = [&](int n) {
    if constexpr (NIN) {
      if (tid < 64) {
        const double inv = p.in_inv;
        const long slot = (long)p.N * 64 * 2;
        const sa_stat_t* sp = p.in_stats + ((long)n * 64 + tid) * 2;
        long long s0 = 0, s1 = 0;
        for (int r = 0; r < p.in_slots; ++r) {
          s0 += sp[r * slot];
          s1 += sp[r * slot + 1];
        }
        const double m = (double)s0 * inv;
        const double var = (double)s1 * inv - m * m;
        nrm[(n & 1) * 128 + tid] = (float)m;
        nrm[(n & 1) * 128 + 64 + tid] = rsqrtf((float)(var > 0.0 ? var : 0.0) + p.in_eps);
      }
      lds_barrier();
      nrm_img = n;
    }
  };
  // NIN: this wave's own (landed) pieces of tile t0 + kk -> relu(IN(.)) in place; the image's mean / rstd must be in
  // its LDS slot already (nrm_load has a barrier: called by all waves at the same point)
  auto fold_tile = [&](int kk) {
    if constexpr (NIN) {
      const int n1 = (t0 + kk) / tiles_img;
      char* ib = smem + (kk % NB) * IN_BYTES;
      // laundered lane index and a rolled loop: the tile-invariant piece decomposition is not hoisted into
      // long-lived VGPRs next to the stationary weights (the STATS variant spilled 36 of them)
      int ln = lane;
      asm volatile("" : "+v"(ln));
      // a lane's channel chunk is the same in all its pieces: piece g = (i * 8 + wave) * 64 + ln holds chunk
      // (g & 7) ^ v2_swz(g >> 3) = (ln & 7) ^ (4 (wave & 1) + (ln >> 4)) for every i, so its 8 means / rstds
      // are read once per tile
      const int q = (ln & 7) ^ (4 * (wave & 1) + (ln >> 4));
      const float* d = nrm + (n1 & 1) * 128 + q * 8;
      const floatx4 m0 = *reinterpret_cast<const floatx4*>(d), m1 = *reinterpret_cast<const floatx4*>(d + 4);
      const floatx4 r0 = *reinterpret_cast<const floatx4*>(d + 64), r1 = *reinterpret_cast<const floatx4*>(d + 68);
#pragma unroll 1
      for (int i = 0; i < V2_PER_WAVE; ++i) {
        const int ins = i * V2_WAVES + wave;
        if (ins < V2_PIECES) {
          const int g = ins * 64 + ln;
          half8 h = *reinterpret_cast<const half8*>(ib + g * 16);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = ((float)h[e] - (e < 4 ? m0[e & 3] : m1[e & 3])) * (e < 4 ? r0[e & 3] : r1[e & 3]);
            h[e] = (f16)(v > 0.f ? v : 0.f);
          }
          *reinterpret_cast<half8*>(ib + g * 16) = h;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // complete before the loop-top barrier publishes the tile
    }
  };
  constexpr int kOpsPerTile = RES ? 4 : 2;  // buffer stores (+ residual buffer loads), range-checked, never skipped
  if constexpr (NIN) {
    if (kb > 0) {
      nrm_load(t0 / tiles_img);
      wait_vmcnt((kb - 1 < NB - 2 ? kb - 1 : NB - 2) * V2_PER_WAVE);  // tile 0's pieces (later tiles in flight)
      fold_tile(0);
    }
  }

  for (int k = 0; k < kb; ++k) {
    const int t = t0 + k;
    const int cur = k % NB;
    // ops this wave issued after tile t's DMA: the ring pieces of tiles k+1, k+2 and the stores of the
    // (at most 3) tiles computed since
    const int ahead = (kb - 1 - k) < NB - 2 ? (kb - 1 - k) : NB - 2;
    wait_vmcnt(ahead * V2_PER_WAVE + (k < NB - 1 ? k : NB - 1) * kOpsPerTile);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int n = t / tiles_img, rr = t - n * tiles_img;
    const int ty = rr / tiles_x, tx = rr - ty * tiles_x;
    const int oy = ty * TR + prow;
    // residual of this tile's pixels, issued before the next DMA so the epilogue's wait for it leaves the
    // ring pieces of tile k+3 in flight
    half8 rv[2];
    if constexpr (RES) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ox = tx * TC + pcol + i * 16 + frow;
        const bool ok = oy < p.H && ox < p.W;
        const size_t pix = ((size_t)n * p.H + oy) * p.W + ox;
        const unsigned roff = ok ? (unsigned)(pix * p.rs + c0) * 2u : 0xFFFFFFF0u;
        typedef unsigned uint4v __attribute__((ext_vector_type(4)));
        rv[i] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rrsrc, roff, 0, 0));
      }
    }
    // every wave is past tile k-1: its buffer takes tile k+NB-1
    if (k + NB - 1 < kb) issue_tile(t + NB - 1, (k + NB - 1) % NB);
    if constexpr (NIN) {
      // tile k+1's pieces are normalised by the waves of channel half 1 HERE, before their MFMA loop, and by those
      // of half 0 after their epilogue: the two waves sharing a SIMD (w, w + 4) fold while the other computes
      if (k + 1 < kb) {
        const int n1 = (t + 1) / tiles_img;
        if (n1 != nrm_img) nrm_load(n1);  // block-uniform (every wave, same k)
        if (hc == 1) {
          // ops issued after tile k+1's DMA: tile k+2's (.. k+NB-2's) pieces and the stores of tiles since
          const int a2 = (kb - 2 - k) < NB - 2 ? (kb - 2 - k) : NB - 2;
          wait_vmcnt(a2 * V2_PER_WAVE + (k < NB - 2 ? k : NB - 2) * kOpsPerTile);
          fold_tile(k + 1);
        }
      }
    }
    const char* ib = smem + cur * IN_BYTES;
    floatx4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    int fr = frow, kql = kq;
    if constexpr (NIN) {
      // laundered per tile: the fragment addresses are recomputed here instead of living across the whole tile
      // loop (with the fold's temporaries they spilled, and a scratch reload inside the MFMA loop waits vmcnt(0))
      asm volatile("" : "+v"(fr), "+v"(kql));
    }
    auto load = [&](int ks, half8* bf) {
      const int tap = ks >> 1, kh = tap / 3, kw = tap - kh * 3;
      const int q = (ks & 1) * 4 + kql;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int pp = (prow + kh) * IC + pcol + i * 16 + fr + kw;
        bf[i] = *reinterpret_cast<const half8*>(ib + pp * 128 + ((q ^ v2_swz(pp)) << 4));
      }
    };
    half8 b0[2], b1[2];
    load(0, b0);
#pragma unroll
    for (int ks = 0; ks < KTOT / 32; ks += 2) {
      load(ks + 1, b1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[ks][j], b0[i], acc[i][j], 0, 0, 0);
      if (ks + 2 < KTOT / 32) load(ks + 2, b0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[ks + 1][j], b1[i], acc[i][j], 0, 0, 0);
    }

    if constexpr (STATS) {
      if (n != stat_img) {
        if (stat_img >= 0) flush_stats();
        stat_img = n;
      }
    }
    // bias re-read per tile from LDS: 8 VGPRs fewer across the main loop
    float tsum[8], tsq[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) tsum[e] = tsq[e] = 0.f;
    float bias8[8];
    {
      const floatx4 b0v = *reinterpret_cast<const floatx4*>(bias_lds + c0);
      const floatx4 b1v = *reinterpret_cast<const floatx4*>(bias_lds + c0 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) bias8[e] = b0v[e], bias8[e + 4] = b1v[e];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ox = tx * TC + pcol + i * 16 + frow;
      const bool ok = oy < p.H && ox < p.W;
      const size_t pix = ((size_t)n * p.H + oy) * p.W + ox;
      half8 h;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = 4 * j + r;
          float v = act_apply(acc[i][j][r] + bias8[e], ACT, p.alpha);
          if constexpr (RES) v = p.act2 == SA_ACT_RELU ? fmaxf(v + (float)rv[i][e], 0.f) : v + (float)rv[i][e];
          h[e] = (f16)v;
          if constexpr (STATS) {
            const float vm = ok ? v : 0.f;
            tsum[e] += vm;
            tsq[e] = fmaf(vm, vm, tsq[e]);
          }
        }
      const unsigned off = ok ? (unsigned)(pix * p.os + c0) * 2u : 0xFFFFFFF0u;
      typedef unsigned uint4v __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, h), orsrc, off, 0, 0);
    }
    if constexpr (STATS) {
      st_lane[0] += floatx4{tsum[0], tsum[1], tsum[2], tsum[3]};
      st_lane[1] += floatx4{tsum[4], tsum[5], tsum[6], tsum[7]};
      st_lane[2] += floatx4{tsq[0], tsq[1], tsq[2], tsq[3]};
      st_lane[3] += floatx4{tsq[4], tsq[5], tsq[6], tsq[7]};
    }
    if constexpr (NIN) {
      if (k + 1 < kb && hc == 0) {
        // ops this wave issued after tile k+1's DMA: tile k+2's (.. k+NB-2's) pieces and the stores of the tiles
        // computed since (this one included)
        const int a2 = (kb - 2 - k) < NB - 2 ? (kb - 2 - k) : NB - 2;
        wait_vmcnt(a2 * V2_PER_WAVE + (k + 1 < NB - 1 ? k + 1 : NB - 1) * kOpsPerTile);
        fold_tile(k + 1);
      }
    }
  }
  if constexpr (STATS) {
    if (stat_img >= 0) flush_stats();
  }
}

template <bool STATS, bool RES, bool NIN = false>
void launch_direct2(const DirectArgs2& a, int act, unsigned g, hipStream_t s) {
  switch (act) {
    case SA_ACT_RELU:
      hipLaunchKernelGGL((conv3x3_c64_direct2_kernel<SA_ACT_RELU, STATS, RES, NIN>), dim3(g), dim3(512), 0, s, a);
      break;
    case SA_ACT_LEAKY:
      hipLaunchKernelGGL((conv3x3_c64_direct2_kernel<SA_ACT_LEAKY, STATS, RES, NIN>), dim3(g), dim3(512), 0, s, a);
      break;
    default:
      hipLaunchKernelGGL((conv3x3_c64_direct2_kernel<SA_ACT_NONE, STATS, RES, NIN>), dim3(g), dim3(512), 0, s, a);
      break;
  }
}

}  // namespace

extern "C" int sa_conv3x3_c64_direct2(const void* x, int xs, const void* w, int kpad, const float* bias, void* out,
                                      int os, int N, int H, int W, int act, float alpha, sa_stat_t* stats, int slots,
                                      const void* res, int rs, int act2, const sa_stat_t* in_stats, int in_slots,
                                      float in_eps, int max_blocks, hipStream_t stream) {
  if (kpad < KTOT || xs < 64 || os < 64 || xs % 8 || os % 8 ||
      (act != SA_ACT_NONE && act != SA_ACT_RELU && act != SA_ACT_LEAKY))
    return -2;
  if (res && (stats || rs < 64 || rs % 8 || (act2 != SA_ACT_NONE && act2 != SA_ACT_RELU))) return -5;
  if (in_stats && res) return -5;  // the folded input norm is the instance-norm blocks' conv2: no residual
  const size_t span = (((size_t)N * H - 1) * W + (W - 1)) * (size_t)os * 2 + 128;  // last pixel's 64 channels
  const size_t rspan = res ? (((size_t)N * H - 1) * W + (W - 1)) * (size_t)rs * 2 + 128 : 0;
  if (span >= 0xFFFFFF00ull || rspan >= 0xFFFFFF00ull) return -5;  // 32-bit buffer offsets
  DirectArgs2 a{(const f16*)x, xs, (const f16*)w, kpad, bias, (f16*)out, os, (unsigned)span, (unsigned)rspan, N, H, W,
                alpha, stats, slots, (const f16*)res, rs, act2, in_stats, in_slots > 1 ? in_slots : 1, in_eps,
                1.0 / ((double)H * W * SA_STAT_SCALE)};
  const long ntiles = (long)N * ((H + TR - 1) / TR) * ((W + TC - 1) / TC);
  long g = max_blocks > 0 ? max_blocks : 256;
  if (g > ntiles) g = ntiles;
  if (g < 1) return 0;
  if (in_stats) {
    if (stats) launch_direct2<true, false, true>(a, act, (unsigned)g, stream);
    else launch_direct2<false, false, true>(a, act, (unsigned)g, stream);
  } else if (stats) launch_direct2<true, false>(a, act, (unsigned)g, stream);
  else if (res) launch_direct2<false, true>(a, act, (unsigned)g, stream);
  else launch_direct2<false, false>(a, act, (unsigned)g, stream);
  return (int)hipGetLastError();
}
