// RAFT-Stereo motion encoder in one kernel (upstream core/update.py BasicMotionEncoder):
//   cor1 = relu(convc1(lookup))      1x1, L*(2r+1) -> 64
//   flo1 = relu(convf1([fx, 0]))     7x7, 2 -> 64 (the y flow is identically 0: only the x taps count)
//   cor2 = relu(convc2(cor1))        3x3, 64 -> 64
//   flo2 = relu(convf2(flo1))        3x3, 64 -> 64
//   out  = relu(conv([cor2, flo2]))  3x3, 128 -> 126, then the [fx, 0] tail -> 128 channels
//
// Unfused, this is the lookup/head kernel plus three implicit GEMMs with N = 64 / 64 / 128 per GRU
// iteration: at N = 64 every im2col row fetched into LDS feeds only 64 MACs per k (0.25 PFLOP/s at batch 8),
// the 3x3 halos re-read cor1 / flo1 / the concat nine times from L2, and at batch 1 the four dependent
// launches sit on the iteration's critical path.  Here one workgroup (4 waves) owns an 8 x 16 output tile
// and keeps every intermediate in LDS:
//   stage 0  the fp32 flow patch the 7x7 taps need (18 x 26 around the tile)
//   stage 1  for the 12 x 20 pixels the two 3x3 convs need, the lookup taps + flow taps as a [240 x 96]
//            fp16 operand, then one MFMA GEMM against the block-diagonal [convc1 | convf1] (packed once at
//            engine build) -> S1 = [cor1 | flo1] (zero outside the image, which is the next conv's zero
//            padding)
//   stage 2  convc2 / convf2 over the 10 x 18 pixels of the last conv's halo, A fragments read straight
//            from S1 at the nine tap offsets (each S1 pixel crosses LDS nine times, HBM / L2 zero times),
//            waves 0-1 cor2, waves 2-3 flo2 -> S2
//   stage 3  conv over the 8 x 16 tile from S2, K = 9 x 128; bias + relu, [fx, 0] tail, staged through LDS
//            for 16-B coalesced stores of all 128 channels
// All GEMMs are v_mfma_f32_16x16x32_f16; the stage 2 / 3 weights (packed [n][K] fp16 like every conv, L2
// resident, shared by all workgroups) stream through per-wave global->LDS DMA rings in whichever LDS area
// the stage has finished with (5 / 11 k-steps ahead, counted vmcnt, no barriers).
// LDS rows are 256 B (128 channels) with the 16-B chunk XOR'd by the pixel index, so the 16 lanes of a
// fragment read (16 consecutive pixels, same chunk) hit 16 different bank groups.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>
#include <cstdlib>

#include "sa/kernels.h"

namespace {
typedef _Float16 f16;
typedef f16 half8 __attribute__((ext_vector_type(8)));
typedef f16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int TH = 8, TW = 16;                 // output tile
constexpr int R2H = TH + 2, R2W = TW + 2;      // S2 region (convc2 / convf2 outputs): 10 x 18
constexpr int R1H = TH + 4, R1W = TW + 4;      // S1 region (cor1 / flo1): 12 x 20
constexpr int FH = R1H + 6, FW = R1W + 6;      // flow patch for the 7x7 taps: 18 x 26
constexpr int P1 = R1H * R1W, P2 = R2H * R2W;  // 240, 180
constexpr int KP = 96, AS = 104;               // stage-1 K (padded) and operand row stride (halfs)
constexpr int S1_OFF = 0, S2_OFF = S1_OFF + P1 * 256, A1_OFF = S2_OFF + P2 * 256, FL_OFF = A1_OFF + P1 * AS * 2;
constexpr int SMEM = FL_OFF + FH * FW * 4;     // 159312 B
static_assert(SMEM <= 163840, "LDS budget");

struct MotionEncArgs {
  const float* pyr;
  long lvl_off1, lvl_off2, lvl_off3;
  const float* flow;  // fp32 [B][H][W] (x flow)
  int B, H, W, W2, levels, radius;
  const f16* w1;    // stage-1 block-diagonal B, fp16 [128][96] (n-major: convc1 rows 0-63 on k < nc, convf1
                    // rows 64-127 on nc <= k < nc + 49)
  const float* b1;  // [128] = [bc | bf]
  const f16* w2c;  // convc2 packed [>=64][576]
  const float* b2c;
  const f16* w2f;  // convf2 packed [>=64][576]
  const float* b2f;
  const f16* w3;  // conv packed [>=128][1152]
  const float* b3;  // [126]
  f16* out;  // [B][H][W][os], channels 0..127
  int os;
  unsigned long long* stamps;  // diagnostics (sa_raft_motion_encoder_stamps): [block][8 marks][64 lanes] or null
  // fused flow-head stencil (null: off): the previous flow head's tap projections P [B][H][W][2][9] fp32
  // (SA_EPI_TAPPROJ) are applied while the flow patch is loaded -- flow(p) = flow_in(p) + bias + sum over the 3x3
  // taps of both n-tile partials, in sa_tapproj_stencil's order (bitwise the same flow) -- and the tile's own pixels
  // of the updated flow are written to flow_out (a different buffer: neighbouring tiles still read flow_in)
  const float* proj;
  const float* proj_bias;
  float* flow_out;
};

// stage 0 of both variants: the fp32 flow patch (image rows ty0-5 .., cols tx0-5 ..), zero outside.  With p.proj
// the previous flow head's stencil is applied on the way: the projections of the 20 x 28 pixels the patch's 3x3
// stencils touch are first copied into LDS scratch `pl` (8-B loads, each image row's 28 x 18 floats contiguous; 40 KB
// of an area the later stages have not written yet), then each patch pixel sums its nine taps there, in
// sa_tapproj_stencil's order (bitwise the same flow)
constexpr int PLH = FH + 2, PLW = FW + 2;  // 20 x 28 projection pixels
constexpr int PL_BYTES = PLH * PLW * 18 * 4;  // 40320
__device__ __forceinline__ void menc_flow_patch(const MotionEncArgs& p, long img_base, int ty0, int tx0, float* fl,
                                                float* pl, int tid, int nt) {
  if (p.proj) {
    // row r of the scratch = image row ty0 - 6 + r, columns tx0 - 6 .. tx0 + 21 (9 float2 per pixel)
    for (int i = tid; i < PLH * PLW * 9; i += nt) {
      const int r = i / (PLW * 9), rem = i - r * (PLW * 9);
      const int c = rem / 9, k = rem - c * 9;
      const int y = ty0 - 6 + r, x = tx0 - 6 + c;
      float2 v = make_float2(0.f, 0.f);
      if ((unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W)
        v = reinterpret_cast<const float2*>(p.proj + (img_base + (long)y * p.W + x) * 18)[k];
      reinterpret_cast<float2*>(pl)[i] = v;
    }
    __syncthreads();
  }
  for (int i = tid; i < FH * FW; i += nt) {
    const int r = i / FW, c = i - r * FW;
    const int y = ty0 - 5 + r, x = tx0 - 5 + c;
    float v = 0.f;
    if ((unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W) {
      const long px = img_base + (long)y * p.W + x;
      v = p.flow[px];
      if (p.proj) {
        float s = p.proj_bias ? p.proj_bias[0] : 0.f;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int yy = y + ky - 1, xx = x + kx - 1;
            if (yy < 0 || yy >= p.H || xx < 0 || xx >= p.W) continue;
            const float* q = pl + ((r + ky) * PLW + (c + kx)) * 18 + (ky * 3 + kx);
            s += q[0] + q[9];
          }
        v += s;
        if (y >= ty0 && y < ty0 + 8 && x >= tx0 && x < tx0 + 16) p.flow_out[px] = v;
      }
    }
    fl[i] = v;
  }
}

typedef __attribute__((address_space(3))) void lds_void_t;

// s_waitcnt vmcnt(N) through the intrinsic (gfx9 encoding: vmcnt bits [3:0] + [15:14], expcnt [6:4] and lgkmcnt
// [11:8] left at their maxima): unlike an inline-asm wait, the compiler's own waitcnt pass sees it and does not
// drain every counter in front of it, so LDS prefetch reads stay in flight
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
// vmcnt <= s * PER for a wave-uniform s in [0, K]
template <int PER, int K>
__device__ __forceinline__ void wait_vm_le(int s) {
  if constexpr (K <= 0) {
    wait_vm<0>();
  } else {
    if (s >= K) wait_vm<K * PER>();
    else wait_vm_le<PER, K - 1>(s);
  }
}

// weight-ring row swizzle: row r's 16-B slot = chunk ^ bs(r >> 2); bs = identity (v1) or 0, 2, 3, 1 (conflict-free
// under the same lane groups: the row quads a group touches at its two chunks land on four distinct slot columns)
template <bool CF>
__device__ __forceinline__ int bswz(int quad) {
  if constexpr (CF) return (0x78 >> (2 * quad)) & 3;
  else return quad & 3;
}

// Per-wave B ring for a conv stage: the wave's 16 * JN weight rows (KROW halfs each) stream through RING LDS
// slots of [16 JN rows][64 B] (one 32-deep k-step) via global->LDS DMA, RING - 1 steps ahead; the 16-B chunk
// of row r sits at slot chunk c ^ ((r >> 2) & 3) so a fragment read (16 rows, one chunk) is conflict-free.
// Only the issuing wave reads its ring, so its own vmcnt is the only ordering needed.
template <int JN, int RING, int KROW, bool CF = false>
struct BRing {
  static constexpr int SLOT = JN * 1024;
  char* base;        // this wave's ring (LDS)
  const f16* src[JN];  // per DMA instruction: this lane's row / chunk source at k = 0
  __device__ __forceinline__ void init(char* ring, const f16* w, int row0, int lane) {
    base = ring;
#pragma unroll
    for (int i = 0; i < JN; ++i) {
      const int r = 16 * i + (lane >> 2), c = lane & 3;
      src[i] = w + (size_t)(row0 + r) * KROW + ((c ^ bswz<CF>((r >> 2) & 3)) << 3);
    }
  }
  __device__ __forceinline__ void issue(int step) {
    char* dst = base + (step % RING) * SLOT;
#pragma unroll
    for (int i = 0; i < JN; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + step * 32), (lds_void_t*)(dst + i * 1024), 16, 0, 0);
  }
  // B fragment of column tile j for k-step `step` (lane: row 16 j + (lane & 15), k chunk lane >> 4)
  __device__ __forceinline__ half8 frag(int step, int j, int lane) const {
    const int r = 16 * j + (lane & 15);
    return *reinterpret_cast<const half8*>(base + (step % RING) * SLOT + r * 64 +
                                           ((((lane >> 4) ^ bswz<CF>((r >> 2) & 3))) << 4));
  }
};

// byte offset of (pixel, 16-B chunk) in a 256-B-per-pixel LDS image
__device__ __forceinline__ int sw(int pix, int chunk) { return pix * 256 + ((chunk ^ (pix & 15)) << 4); }

// Conflict-free variant (round 6).  ds_read_b128 serves a wave in four lane groups that are NOT 16 contiguous lanes
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63}, MI355X_MICROARCH.md "LDS"):
// with fragment row r16 = lane & 15 reading pixel p0 + r16 and k-chunk c0 + (lane >> 4), sw()'s chunk ^ (pix & 15)
// puts 2-4 lanes of a group on one bank set (model: 1.3 extra cycles per stage-3 read, 3.2 per stage-2 read, PMC:
// SQ_LDS_BANK_CONFLICT 2.6x SQ_INSTS_LDS).  Fix: fragment row r16 reads pixel p0 + perm16(r16) -- the rows of the
// groups' chunk-c0 halves get the even offsets, the chunk-c0^1 halves the odd ones -- and the chunk is XOR'd with
// T[pix & 15], a permutation for which k -> T[(p0 + k) & 15] ^ (k & 1) is one-to-one for EVERY start p0 (found by
// search; packed 4 bits per entry), so every group covers 16 distinct 16-B bank slots at any tap shift.
__device__ __forceinline__ int perm16(int r) { return r < 4 ? 2 * r : (r < 12 ? 2 * r - 7 : 2 * r - 16); }
__device__ __forceinline__ int swc(int pix, int chunk) {
  const int t = (int)((0xc2d3958e17bf06a4ull >> (4 * (pix & 15))) & 15);
  return pix * 256 + ((chunk ^ t) << 4);
}
template <bool CF>
__device__ __forceinline__ int swt(int pix, int chunk) {
  if constexpr (CF) return swc(pix, chunk);
  else return sw(pix, chunk);
}

// NW waves per workgroup (4: one per SIMD, 2 x 16 output channels per wave in stages 2 / 3; 8: two per SIMD,
// one 16-channel column tile per wave)
// VEC: every pyramid row length is a multiple of 4 floats (W2 % 32 == 0), so each level's 10 taps come from four
// aligned 16-B loads (one cache line per lane instead of ten scalar loads that each touch 64 lines per wave)
template <int NW, bool VEC, bool CF = false>
__global__ __launch_bounds__(64 * NW) void raft_motion_encoder_kernel(const MotionEncArgs p) {
  constexpr int NT = 64 * NW, JN = 8 / NW;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  char* s1 = smem + S1_OFF;
  char* s2 = smem + S2_OFF;
  f16* a1 = reinterpret_cast<f16*>(smem + A1_OFF);
  float* fl = reinterpret_cast<float*>(smem + FL_OFF);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kofs = (lane >> 4) * 8;
  const int tiles_x = (p.W + TW - 1) / TW, tiles_y = (p.H + TH - 1) / TH;
  const int bimg = blockIdx.x / (tiles_x * tiles_y);
  const int trem = blockIdx.x - bimg * tiles_x * tiles_y;
  const int ty0 = (trem / tiles_x) * TH, tx0 = (trem % tiles_x) * TW;
  const long img_base = (long)bimg * p.H * p.W;
  // stage timestamps of wave 0 (diagnostics only; every lane stores its own slot: plain vector stores)
  auto stamp = [&](int mark) {
    if (p.stamps && wave == 0) p.stamps[((size_t)blockIdx.x * 8 + mark) * 64 + lane] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  // ---------------- stage 0: flow patch (image rows ty0-5 .., cols tx0-5 ..), zero outside ----------------
  static_assert(PL_BYTES <= P2 * 256, "projection scratch fits the S2 area");
  menc_flow_patch(p, img_base, ty0, tx0, fl, reinterpret_cast<float*>(s2), tid, NT);
  __syncthreads();

  stamp(1);
  // ---------------- stage 1a: the [240 x 96] operand ----------------
  // one S1 pixel per thread: its 4 levels x 10 pyramid values are loaded before any is used (one global
  // latency), the 9 bilinear taps per level (the arithmetic of sa_corr1d_lookup), its 49 flow taps from the
  // patch and the zero tail are assembled in registers and stored as 12 16-B LDS writes.
  // K layout: [0, 36) lookup (level-major), [36, 85) flow taps ky * 7 + kx, [85, 96) zero.
  if (tid < P1) {
    const int pix = tid;
    const int r = pix / R1W, c = pix - r * R1W;
    const int y = ty0 - 2 + r, x = tx0 - 2 + c;
    const bool in = (unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W;
    const float fx = fl[(r + 3) * FW + (c + 3)];
    half8 hv[12];
    if constexpr (VEC) {
      // level q: the 16 floats of row[b .. b + 16), b = x0 rounded down to a multiple of 4 (chunks lie wholly inside
      // or wholly outside the row, so the zero padding is per chunk); tap k = lerp(x0 - b + k)
      floatx4 f[4][4];
      float wa[4];
      int d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const long off = q == 0 ? 0 : (q == 1 ? p.lvl_off1 : (q == 2 ? p.lvl_off2 : p.lvl_off3));
        const int Wl = p.W2 >> q;
        const float* row = p.pyr + off + (img_base + (long)(in ? y : 0) * p.W + (in ? x : 0)) * Wl;
        const float xl = ((float)x + fx) / (float)(1 << q) - 4.f;
        const float x0f = floorf(xl);
        wa[q] = xl - x0f;
        const int x0 = (int)x0f;
        const int b = x0 & ~3;
        d[q] = x0 - b;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int c = b + 4 * t;
          f[q][t] = (in && c >= 0 && c < Wl) ? *reinterpret_cast<const floatx4*>(row + c) : floatx4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float g[13];
#pragma unroll
        for (int sidx = 0; sidx < 13; ++sidx)  // = lerp_tap (corr.hip) at offset sidx
          g[sidx] = __fmaf_rn(wa[q], f[q][(sidx + 1) >> 2][(sidx + 1) & 3], __fmul_rn(1.f - wa[q], f[q][sidx >> 2][sidx & 3]));
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const int kk = 9 * q + k;
          const float t = d[q] == 0 ? g[k] : (d[q] == 1 ? g[k + 1] : (d[q] == 2 ? g[k + 2] : g[k + 3]));
          hv[kk >> 3][kk & 7] = (f16)t;
        }
      }
    } else {
      float v[4][10], wa[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const long off = q == 0 ? 0 : (q == 1 ? p.lvl_off1 : (q == 2 ? p.lvl_off2 : p.lvl_off3));
        const int Wl = p.W2 >> q;
        const float* row = p.pyr + off + (img_base + (long)(in ? y : 0) * p.W + (in ? x : 0)) * Wl;
        const float xl = ((float)x + fx) / (float)(1 << q) - 4.f;
        const float x0f = floorf(xl);
        wa[q] = xl - x0f;
        const int x0 = (int)x0f;
#pragma unroll
        for (int k = 0; k < 10; ++k) {
          const int xi = x0 + k;
          v[q][k] = (in && xi >= 0 && xi < Wl) ? row[xi] : 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const int kk = 9 * q + k;
          hv[kk >> 3][kk & 7] = (f16)__fmaf_rn(wa[q], v[q][k + 1], __fmul_rn(1.f - wa[q], v[q][k]));  // = lerp_tap (corr.hip)
        }
    }
#pragma unroll
    for (int t = 0; t < 49; ++t) {
      const int kk = 36 + t, ky = t / 7, kx = t % 7;
      hv[kk >> 3][kk & 7] = (f16)fl[(r + ky) * FW + (c + kx)];
    }
#pragma unroll
    for (int kk = 85; kk < 96; ++kk) hv[kk >> 3][kk & 7] = (f16)0.f;
#pragma unroll
    for (int i = 0; i < 12; ++i) *reinterpret_cast<half8*>(a1 + pix * AS + 8 * i) = hv[i];
  }
  __syncthreads();

  stamp(2);
  // ---------------- stage 1b: S1 = relu([lookup | flow taps] x blockdiag(convc1, convf1)) ----------------
  // wave w: column tiles w * JN .. w * JN + JN - 1 of all 15 row tiles
  {
    constexpr int NT1 = P1 / 16;  // 15
    half8 bfr[JN][3];
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int n = 16 * (wave * JN + j) + r16;
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) bfr[j][ks] = *reinterpret_cast<const half8*>(p.w1 + n * KP + ks * 32 + kofs);
    }
    // transposed product (weights as the A operand): lane (r16, g) holds output channels 4 g .. 4 g + 3 of pixel
    // 16 i + r16, stored as one 8-byte LDS write instead of four 2-byte ones
    floatx4 acc[NT1][JN];
#pragma unroll
    for (int i = 0; i < NT1; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 3; ++ks)
#pragma unroll
      for (int i = 0; i < NT1; ++i) {
        const half8 a = *reinterpret_cast<const half8*>(a1 + (16 * i + r16) * AS + ks * 32 + kofs);
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bfr[j][ks], a, acc[i][j], 0, 0, 0);
      }
    float bias4[JN][4];
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) bias4[j][rr] = p.b1[16 * (wave * JN + j) + 4 * (lane >> 4) + rr];
#pragma unroll
    for (int i = 0; i < NT1; ++i) {
      const int pix = 16 * i + r16;
      const int r = pix / R1W, c = pix - r * R1W;
      const bool in = (unsigned)(ty0 - 2 + r) < (unsigned)p.H && (unsigned)(tx0 - 2 + c) < (unsigned)p.W;
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const int col = 16 * (wave * JN + j) + 4 * (lane >> 4);
        half4 h;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) h[rr] = (f16)(in ? fmaxf(acc[i][j][rr] + bias4[j][rr], 0.f) : 0.f);
        *reinterpret_cast<half4*>(s1 + swt<CF>(pix, col >> 3) + (col & 7) * 2) = h;
      }
    }
  }
  __syncthreads();

  stamp(3);
  // ---------------- stage 2: S2 = [relu(convc2(cor1)) | relu(convf2(flo1))] over the 10 x 18 region -------------
  {
    constexpr int NT2 = (P2 + 15) / 16;  // 12 row tiles (192 rows, 180 valid)
    constexpr int NS2 = 18;              // 9 taps x 2 k32 halves of 64 channels
    const int ct0 = wave * JN;            // first of this wave's JN 16-channel column tiles (0-3 cor2, 4-7 flo2)
    const int cb = ct0 < 4 ? 0 : 64;      // source / destination channel base (cor | flo)
    const f16* wsrc = ct0 < 4 ? p.w2c : p.w2f;
    const float* bsrc = ct0 < 4 ? p.b2c : p.b2f;
    const int nb = (16 * ct0) & 63;       // first output channel within the conv
    int base[NT2];                        // S1 pixel of tap (0, 0) for this lane's row of each tile
    // CF: tile i < 10 is S2 row i, columns perm16(r16) (16 consecutive S1 pixels per tap: the shift-proof layout
    // holds); tiles 10 / 11 hold the rows' last two columns (k = 2 row + col - 16, k < 20)
    auto s2q = [&](int i) -> int {
      if constexpr (CF) {
        const int o = perm16(r16);
        if (i < R2H) return i * R2W + o;
        const int k = (i - R2H) * 16 + o;
        return k < 2 * R2H ? (k >> 1) * R2W + 16 + (k & 1) : -1;
      } else {
        const int q = 16 * i + r16;
        return q < P2 ? q : -1;
      }
    };
#pragma unroll
    for (int i = 0; i < NT2; ++i) {
      int q = s2q(i);
      q = q < 0 ? (CF ? 0 : P2 - 1) : q;
      base[i] = (q / R2W) * R1W + (q % R2W);
    }
    floatx4 acc[NT2][JN];
#pragma unroll
    for (int i = 0; i < NT2; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // weights through a per-wave DMA ring in the (finished) stage-1 operand area
    constexpr int RING = 6;
    static_assert(NW * RING * JN * 1024 <= P1 * AS * 2, "stage-2 B rings fit the A1 area");
    BRing<JN, RING, 576, CF> br;
    br.init(smem + A1_OFF + wave * RING * JN * 1024, wsrc, nb, lane);
    // software pipeline: the A / B fragments of step st + 1 are read while step st's MFMAs run
    auto readA = [&](int st, half8* a) {
      const int tap = st >> 1, ky = tap / 3, kx = tap - ky * 3;
      const int toff = ky * R1W + kx;
      const int chunk = (cb + 32 * (st & 1) + kofs) >> 3;
#pragma unroll
      for (int i = 0; i < NT2; ++i) a[i] = *reinterpret_cast<const half8*>(s1 + swt<CF>(base[i] + toff, chunk));
    };
    auto readB = [&](int st, half8* b) {
#pragma unroll
      for (int j = 0; j < JN; ++j) b[j] = br.frag(st, j, lane);
    };
    // One k-step: refill the ring slot freed by step st - 1 (the DMA goes first: the compiler drains lgkmcnt
    // around it, which must not catch the prefetch reads), wait for step st + 1's weights, read step st + 1's
    // A / B fragments, then step st's MFMAs.  Fully unrolled straight-line code (constant vmcnt), so the
    // compiler's lgkmcnt tracking keeps the prefetch reads in flight under the MFMAs (a loop back-edge made it
    // drain them before every step).
    auto step = [&](int st, bool issue, bool prefetch, int ahead, const half8* ac, const half8* bc, half8* an,
                    half8* bn) {
      __builtin_amdgcn_sched_barrier(0);
      if (issue) br.issue(st + RING - 1);
      if (prefetch) {
        wait_vm_le<JN, RING - 2>(ahead);
        readB(st + 1, bn);
        readA(st + 1, an);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this step's MFMAs
#pragma unroll
      for (int i = 0; i < NT2; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bc[j], ac[i], acc[i][j], 0, 0, 0);
    };
#pragma unroll
    for (int st = 0; st < RING - 1; ++st) br.issue(st);
    half8 a0[NT2], a1v[NT2], b0[JN], b1v[JN];
    wait_vm_le<JN, RING - 2>(RING - 2);
    readB(0, b0);
    readA(0, a0);
    constexpr int MAIN = ((NS2 - RING + 1) / 2) * 2;  // steps with both a refill and a prefetch, in pairs
#pragma unroll
    for (int st = 0; st < MAIN; st += 2) {
      step(st, true, true, RING - 2, a0, b0, a1v, b1v);
      step(st + 1, true, true, RING - 2, a1v, b1v, a0, b0);
    }
#pragma unroll
    for (int st = MAIN; st < NS2; ++st) {
      const int ahead = NS2 - 2 - st < RING - 2 ? NS2 - 2 - st : RING - 2;
      if ((st - MAIN) % 2 == 0) step(st, st + RING - 1 < NS2, st + 1 < NS2, ahead, a0, b0, a1v, b1v);
      else step(st, st + RING - 1 < NS2, st + 1 < NS2, ahead, a1v, b1v, a0, b0);
    }
    // transposed product: lane (r16, g) holds channels 4 g .. 4 g + 3 of S2 pixel 16 i + r16 (one 8-byte write)
    float bias4[JN][4];
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) bias4[j][rr] = bsrc[nb + 16 * j + 4 * (lane >> 4) + rr];
#pragma unroll
    for (int i = 0; i < NT2; ++i) {
      const int q = s2q(i);
      if (q < 0) continue;
      const int r = q / R2W, c = q - r * R2W;
      const bool in = (unsigned)(ty0 - 1 + r) < (unsigned)p.H && (unsigned)(tx0 - 1 + c) < (unsigned)p.W;
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const int col = cb + nb + 16 * j + 4 * (lane >> 4);
        half4 h;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) h[rr] = (f16)(in ? fmaxf(acc[i][j][rr] + bias4[j][rr], 0.f) : 0.f);
        *reinterpret_cast<half4*>(s2 + swt<CF>(q, col >> 3) + (col & 7) * 2) = h;
      }
    }
  }
  __syncthreads();

  stamp(4);
  // ---------------- stage 3: out = relu(conv([cor2 | flo2])) over the 8 x 16 tile, K = 9 x 128 ----------------
  {
    constexpr int NT3 = TH * TW / 16;  // 8 row tiles
    constexpr int NS3 = 36;            // 9 taps x 4 k32 quarters of 128 channels
    const int nb = wave * JN * 16;     // this wave's first output channel
    int base[NT3];
    const int o3 = CF ? perm16(r16) : r16;  // output row i, column o3 (TW = 16)
#pragma unroll
    for (int i = 0; i < NT3; ++i) {
      const int q = 16 * i + o3;
      base[i] = (q / TW) * R2W + (q % TW);
    }
    floatx4 acc[NT3][JN];
#pragma unroll
    for (int i = 0; i < NT3; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // weights through per-wave DMA rings in the S1 and A1 areas (both finished): half the waves each
    constexpr int RING = 12;
    static_assert((NW / 2) * RING * JN * 1024 <= P1 * AS * 2 && (NW / 2) * RING * JN * 1024 <= P1 * 256,
                  "stage-3 B rings fit the S1 / A1 areas");
    BRing<JN, RING, 1152, CF> br;
    br.init(smem + (wave < NW / 2 ? S1_OFF : A1_OFF) + (wave % (NW / 2)) * RING * JN * 1024, p.w3, nb, lane);
    auto readA = [&](int st, half8* a) {
      const int tap = st >> 2, ky = tap / 3, kx = tap - ky * 3;
      const int toff = ky * R2W + kx;
      const int chunk = (32 * (st & 3) + kofs) >> 3;
#pragma unroll
      for (int i = 0; i < NT3; ++i) a[i] = *reinterpret_cast<const half8*>(s2 + swt<CF>(base[i] + toff, chunk));
    };
    auto readB = [&](int st, half8* b) {
#pragma unroll
      for (int j = 0; j < JN; ++j) b[j] = br.frag(st, j, lane);
    };
    // One k-step: refill the ring slot freed by step st - 1 (the DMA goes first: the compiler drains lgkmcnt
    // around it, which must not catch the prefetch reads), wait for step st + 1's weights, read step st + 1's
    // A / B fragments, then step st's MFMAs.  Fully unrolled straight-line code (constant vmcnt), so the
    // compiler's lgkmcnt tracking keeps the prefetch reads in flight under the MFMAs (a loop back-edge made it
    // drain them before every step).
    auto step = [&](int st, bool issue, bool prefetch, int ahead, const half8* ac, const half8* bc, half8* an,
                    half8* bn) {
      __builtin_amdgcn_sched_barrier(0);
      if (issue) br.issue(st + RING - 1);
      if (prefetch) {
        wait_vm_le<JN, RING - 2>(ahead);
        readB(st + 1, bn);
        readA(st + 1, an);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this step's MFMAs
#pragma unroll
      for (int i = 0; i < NT3; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bc[j], ac[i], acc[i][j], 0, 0, 0);
    };
#pragma unroll
    for (int st = 0; st < RING - 1; ++st) br.issue(st);
    half8 a0[NT3], a1v[NT3], b0[JN], b1v[JN];
    wait_vm_le<JN, RING - 2>(RING - 2);
    readB(0, b0);
    readA(0, a0);
    constexpr int MAIN = ((NS3 - RING + 1) / 2) * 2;  // steps with both a refill and a prefetch, in pairs
#pragma unroll
    for (int st = 0; st < MAIN; st += 2) {
      step(st, true, true, RING - 2, a0, b0, a1v, b1v);
      step(st + 1, true, true, RING - 2, a1v, b1v, a0, b0);
    }
#pragma unroll
    for (int st = MAIN; st < NS3; ++st) {
      const int ahead = NS3 - 2 - st < RING - 2 ? NS3 - 2 - st : RING - 2;
      if ((st - MAIN) % 2 == 0) step(st, st + RING - 1 < NS3, st + 1 < NS3, ahead, a0, b0, a1v, b1v);
      else step(st, st + RING - 1 < NS3, st + 1 < NS3, ahead, a1v, b1v, a0, b0);
    }
    stamp(5);
    __syncthreads();  // every wave is done with its ring before the S1 area takes the output tile
    // bias + relu (channels < 126), [fx, 0] tail, staged in the (finished) S1 area
    // transposed product: lane (r16, g) holds channels 4 g .. 4 g + 3 of output pixel 16 i + r16
    char* so = s1;
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int col0 = nb + 16 * j + 4 * (lane >> 4);
      float bj[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) bj[rr] = col0 + rr < 126 ? p.b3[col0 + rr] : 0.f;
#pragma unroll
      for (int i = 0; i < NT3; ++i) {
        const int q = 16 * i + o3;
        const float fx = fl[((q / TW) + 5) * FW + (q % TW) + 5];
        half4 h;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int col = col0 + rr;
          h[rr] = (f16)(col < 126 ? fmaxf(acc[i][j][rr] + bj[rr], 0.f) : (col == 126 ? fx : 0.f));
        }
        *reinterpret_cast<half4*>(so + swt<CF>(q, col0 >> 3) + (col0 & 7) * 2) = h;
      }
    }
    __syncthreads();
    for (int i = tid; i < TH * TW * 16; i += NT) {
      const int q = i >> 4, ch = i & 15;
      const int y = ty0 + q / TW, x = tx0 + q % TW;
      if (y < p.H && x < p.W)
        *reinterpret_cast<half8*>(p.out + (img_base + (long)y * p.W + x) * p.os + ch * 8) =
            *reinterpret_cast<const half8*>(so + swt<CF>(q, ch));
    }
  }
  stamp(6);
}

// ---------------------------------------------------------------------------------------------------------------
// v2: the same 8 x 16 tile and arithmetic in 63 KB of LDS, so TWO workgroups share a CU (8 waves, 2 per SIMD):
// one workgroup's latency-bound phases (the pyramid gather of stage 1a, barriers, epilogue stores) run under the
// other's MFMA stages.  v1 holds A1, S1 and S2 at once (159 KB, one workgroup per CU, MFMA busy 0.22 at batch 8).
// Here one 61 440-B region R = 240 pixels x 256 B carries them in turn -- A1 (the stage-1 operand, 96 of 128 chunk
// slots used), then S1, then S2, then the output tile -- each overwrite after a barrier that ends the previous
// stage's reads (the stage's accumulators wait in registers across it).  Weights no longer stream through LDS
// rings: each wave reads only its own 16 JN output-channel rows, so its B fragments are plain 16-B global loads
// (L2 resident, shared by every workgroup) issued DEPTH k-steps ahead into registers.
constexpr int R_BYTES = P1 * 256;               // 61440
constexpr int SMEM2 = R_BYTES + FH * FW * 4;    // 63312
static_assert(2 * SMEM2 <= 163840, "two workgroups per CU");
#ifndef MENC2_D3
#define MENC2_D3 3  // k-steps of stage-3 weights in flight
#endif

// one conv stage of v2: acc[NTI][JN] += A (LDS image `src`, per-row-tile tap-0 pixel base[i], tap offsets via
// `tapoff(st)` / chunk via `chunk(st)`) x B (global rows w[n0 + 16 j + r16][KROW], k-step st = 32 halfs)
template <int NTI, int JN, int NS, int DEPTH, int KROW, typename TapOff, typename Chunk>
__device__ __forceinline__ void menc2_stage(floatx4 (&acc)[NTI][JN], const char* src, const int (&base)[NTI],
                                            const f16* w, int n0, int lane, TapOff tapoff, Chunk chunk) {
  const int r16 = lane & 15, kofs = (lane >> 4) * 8;
  const f16* wrow[JN];
#pragma unroll
  for (int j = 0; j < JN; ++j) wrow[j] = w + (size_t)(n0 + 16 * j + r16) * KROW + kofs;
  half8 bq[NS][JN];
  half8 aq[2][NTI];
#pragma unroll
  for (int st = 0; st < DEPTH && st < NS; ++st)
#pragma unroll
    for (int j = 0; j < JN; ++j) bq[st][j] = *reinterpret_cast<const half8*>(wrow[j] + st * 32);
  auto readA = [&](int st, half8* a) {
    const int toff = tapoff(st), c = chunk(st);
#pragma unroll
    for (int i = 0; i < NTI; ++i) a[i] = *reinterpret_cast<const half8*>(src + sw(base[i] + toff, c));
  };
  readA(0, aq[0]);
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    __builtin_amdgcn_sched_barrier(0);
    if (st + DEPTH < NS) {
#pragma unroll
      for (int j = 0; j < JN; ++j) bq[st + DEPTH][j] = *reinterpret_cast<const half8*>(wrow[j] + (st + DEPTH) * 32);
    }
    if (st + 1 < NS) readA(st + 1, aq[(st + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < NTI; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bq[st][j], aq[st & 1][i], acc[i][j], 0, 0, 0);
  }
}

template <bool VEC>
__global__ __launch_bounds__(256, 2) void raft_motion_encoder_v2_kernel(const MotionEncArgs p) {
  constexpr int NT = 256, NW = 4, JN = 2;
  __shared__ __attribute__((aligned(16))) char smem[SMEM2];
  char* R = smem;
  float* fl = reinterpret_cast<float*>(smem + R_BYTES);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kofs = (lane >> 4) * 8;
  const int tiles_x = (p.W + TW - 1) / TW, tiles_y = (p.H + TH - 1) / TH;
  const int bimg = blockIdx.x / (tiles_x * tiles_y);
  const int trem = blockIdx.x - bimg * tiles_x * tiles_y;
  const int ty0 = (trem / tiles_x) * TH, tx0 = (trem % tiles_x) * TW;
  const long img_base = (long)bimg * p.H * p.W;
  auto stamp = [&](int mark) {
    if (p.stamps && wave == 0) p.stamps[((size_t)blockIdx.x * 8 + mark) * 64 + lane] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  // ---------------- stage 0: flow patch ----------------
  static_assert(PL_BYTES <= R_BYTES, "projection scratch fits R");
  menc_flow_patch(p, img_base, ty0, tx0, fl, reinterpret_cast<float*>(R), tid, NT);
  __syncthreads();
  stamp(1);

  // ---------------- stage 1a: the [240 x 96] operand into R (v1's arithmetic, chunk slots swizzled as S1) --------
  if (tid < P1) {
    const int pix = tid;
    const int r = pix / R1W, c = pix - r * R1W;
    const int y = ty0 - 2 + r, x = tx0 - 2 + c;
    const bool in = (unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W;
    const float fx = fl[(r + 3) * FW + (c + 3)];
    half8 hv[12];
    if constexpr (VEC) {
      floatx4 f[4][4];
      float wa[4];
      int d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const long off = q == 0 ? 0 : (q == 1 ? p.lvl_off1 : (q == 2 ? p.lvl_off2 : p.lvl_off3));
        const int Wl = p.W2 >> q;
        const float* row = p.pyr + off + (img_base + (long)(in ? y : 0) * p.W + (in ? x : 0)) * Wl;
        const float xl = ((float)x + fx) / (float)(1 << q) - 4.f;
        const float x0f = floorf(xl);
        wa[q] = xl - x0f;
        const int x0 = (int)x0f;
        const int b = x0 & ~3;
        d[q] = x0 - b;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int cc = b + 4 * t;
          f[q][t] = (in && cc >= 0 && cc < Wl) ? *reinterpret_cast<const floatx4*>(row + cc) : floatx4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float g[13];
#pragma unroll
        for (int sidx = 0; sidx < 13; ++sidx)
          g[sidx] = __fmaf_rn(wa[q], f[q][(sidx + 1) >> 2][(sidx + 1) & 3], __fmul_rn(1.f - wa[q], f[q][sidx >> 2][sidx & 3]));
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const int kk = 9 * q + k;
          const float t = d[q] == 0 ? g[k] : (d[q] == 1 ? g[k + 1] : (d[q] == 2 ? g[k + 2] : g[k + 3]));
          hv[kk >> 3][kk & 7] = (f16)t;
        }
      }
    } else {
      float v[4][10], wa[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const long off = q == 0 ? 0 : (q == 1 ? p.lvl_off1 : (q == 2 ? p.lvl_off2 : p.lvl_off3));
        const int Wl = p.W2 >> q;
        const float* row = p.pyr + off + (img_base + (long)(in ? y : 0) * p.W + (in ? x : 0)) * Wl;
        const float xl = ((float)x + fx) / (float)(1 << q) - 4.f;
        const float x0f = floorf(xl);
        wa[q] = xl - x0f;
        const int x0 = (int)x0f;
#pragma unroll
        for (int k = 0; k < 10; ++k) {
          const int xi = x0 + k;
          v[q][k] = (in && xi >= 0 && xi < Wl) ? row[xi] : 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const int kk = 9 * q + k;
          hv[kk >> 3][kk & 7] = (f16)__fmaf_rn(wa[q], v[q][k + 1], __fmul_rn(1.f - wa[q], v[q][k]));
        }
    }
#pragma unroll
    for (int t = 0; t < 49; ++t) {
      const int kk = 36 + t, ky = t / 7, kx = t % 7;
      hv[kk >> 3][kk & 7] = (f16)fl[(r + ky) * FW + (c + kx)];
    }
#pragma unroll
    for (int kk = 85; kk < 96; ++kk) hv[kk >> 3][kk & 7] = (f16)0.f;
#pragma unroll
    for (int i = 0; i < 12; ++i) *reinterpret_cast<half8*>(R + sw(pix, i)) = hv[i];
  }
  __syncthreads();
  stamp(2);

  // ---------------- stage 1b: S1 = relu(A1 x blockdiag(convc1, convf1)), written over A1 ----------------
  {
    constexpr int NT1 = P1 / 16;  // 15
    half8 bfr[JN][3];
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int n = 16 * (wave * JN + j) + r16;
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) bfr[j][ks] = *reinterpret_cast<const half8*>(p.w1 + n * KP + ks * 32 + kofs);
    }
    floatx4 acc[NT1][JN];
#pragma unroll
    for (int i = 0; i < NT1; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 3; ++ks)
#pragma unroll
      for (int i = 0; i < NT1; ++i) {
        const half8 a = *reinterpret_cast<const half8*>(R + sw(16 * i + r16, ks * 4 + (lane >> 4)));
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bfr[j][ks], a, acc[i][j], 0, 0, 0);
      }
    float bias4[JN][4];
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) bias4[j][rr] = p.b1[16 * (wave * JN + j) + 4 * (lane >> 4) + rr];
    __syncthreads();  // every wave has read A1
#pragma unroll
    for (int i = 0; i < NT1; ++i) {
      const int pix = 16 * i + r16;
      const int r = pix / R1W, c = pix - r * R1W;
      const bool in = (unsigned)(ty0 - 2 + r) < (unsigned)p.H && (unsigned)(tx0 - 2 + c) < (unsigned)p.W;
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const int col = 16 * (wave * JN + j) + 4 * (lane >> 4);
        half4 h;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) h[rr] = (f16)(in ? fmaxf(acc[i][j][rr] + bias4[j][rr], 0.f) : 0.f);
        *reinterpret_cast<half4*>(R + sw(pix, col >> 3) + (col & 7) * 2) = h;
      }
    }
  }
  __syncthreads();
  stamp(3);

  // ---------------- stage 2: S2 = [relu(convc2(cor1)) | relu(convf2(flo1))] over 10 x 18, written over S1 ---------
  // wave w: row tiles 6 (w & 1) .. + 5 of the 12 (192 rows, 180 valid) x all four 16-channel column tiles of convc2
  // (w < 2) or convf2 (w >= 2): 6 A + 4 B fragments per 24 MFMAs
  {
    constexpr int NTW = 6, JN2 = 4;
    const int i0 = (wave & 1) * NTW;
    const int cb = wave < 2 ? 0 : 64;
    const f16* wsrc = wave < 2 ? p.w2c : p.w2f;
    const float* bsrc = wave < 2 ? p.b2c : p.b2f;
    int base[NTW];
#pragma unroll
    for (int i = 0; i < NTW; ++i) {
      int q = 16 * (i0 + i) + r16;
      q = q < P2 ? q : P2 - 1;
      base[i] = (q / R2W) * R1W + (q % R2W);
    }
    floatx4 acc[NTW][JN2];
#pragma unroll
    for (int i = 0; i < NTW; ++i)
#pragma unroll
      for (int j = 0; j < JN2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    menc2_stage<NTW, JN2, 18, 3, 576>(
        acc, R, base, wsrc, 0, lane,
        [](int st) { const int tap = st >> 1, ky = tap / 3; return ky * R1W + (tap - ky * 3); },
        [&](int st) { return (cb + 32 * (st & 1) + kofs) >> 3; });
    float bias4[JN2][4];
#pragma unroll
    for (int j = 0; j < JN2; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) bias4[j][rr] = bsrc[16 * j + 4 * (lane >> 4) + rr];
    __syncthreads();  // every wave has read S1
#pragma unroll
    for (int i = 0; i < NTW; ++i) {
      const int q = 16 * (i0 + i) + r16;
      if (q >= P2) continue;
      const int r = q / R2W, c = q - r * R2W;
      const bool in = (unsigned)(ty0 - 1 + r) < (unsigned)p.H && (unsigned)(tx0 - 1 + c) < (unsigned)p.W;
#pragma unroll
      for (int j = 0; j < JN2; ++j) {
        const int col = cb + 16 * j + 4 * (lane >> 4);
        half4 h;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) h[rr] = (f16)(in ? fmaxf(acc[i][j][rr] + bias4[j][rr], 0.f) : 0.f);
        *reinterpret_cast<half4*>(R + sw(q, col >> 3) + (col & 7) * 2) = h;
      }
    }
  }
  __syncthreads();
  stamp(4);

  // ---------------- stage 3: out = relu(conv([cor2 | flo2])) over 8 x 16, K = 9 x 128 ----------------
  // wave w: row tiles 4 (w & 1) .. + 3 of the 8 x output channels 64 (w >> 1) .. + 63
  {
    constexpr int NTW = 4, JN3 = 4;
    const int i0 = (wave & 1) * NTW;
    const int nb = (wave >> 1) * 64;
    int base[NTW];
#pragma unroll
    for (int i = 0; i < NTW; ++i) {
      const int q = 16 * (i0 + i) + r16;
      base[i] = (q / TW) * R2W + (q % TW);
    }
    floatx4 acc[NTW][JN3];
#pragma unroll
    for (int i = 0; i < NTW; ++i)
#pragma unroll
      for (int j = 0; j < JN3; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    menc2_stage<NTW, JN3, 36, MENC2_D3, 1152>(
        acc, R, base, p.w3, nb, lane,
        [](int st) { const int tap = st >> 2, ky = tap / 3; return ky * R2W + (tap - ky * 3); },
        [&](int st) { return (32 * (st & 3) + kofs) >> 3; });
    stamp(5);
    __syncthreads();  // every wave has read S2
#pragma unroll
    for (int j = 0; j < JN3; ++j) {
      const int col0 = nb + 16 * j + 4 * (lane >> 4);
      float bj[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) bj[rr] = col0 + rr < 126 ? p.b3[col0 + rr] : 0.f;
#pragma unroll
      for (int i = 0; i < NTW; ++i) {
        const int q = 16 * (i0 + i) + r16;
        const float fx = fl[((q / TW) + 5) * FW + (q % TW) + 5];
        half4 h;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int col = col0 + rr;
          h[rr] = (f16)(col < 126 ? fmaxf(acc[i][j][rr] + bj[rr], 0.f) : (col == 126 ? fx : 0.f));
        }
        *reinterpret_cast<half4*>(R + sw(q, col0 >> 3) + (col0 & 7) * 2) = h;
      }
    }
    __syncthreads();
    for (int i = tid; i < TH * TW * 16; i += NT) {
      const int q = i >> 4, ch = i & 15;
      const int y = ty0 + q / TW, x = tx0 + q % TW;
      if (y < p.H && x < p.W)
        *reinterpret_cast<half8*>(p.out + (img_base + (long)y * p.W + x) * p.os + ch * 8) =
            *reinterpret_cast<const half8*>(R + sw(q, ch));
    }
  }
  stamp(6);
  (void)NW;
}

unsigned long long* g_stamps = nullptr;
int g_menc_variant = -1;  // -1: SA_RAFT_MENC (default 1), 1: v1, 2: v2

}  // namespace

extern "C" void sa_raft_motion_encoder_variant(int v) { g_menc_variant = v; }

// diagnostics: record s_memrealtime (100 MHz) stage marks of every workgroup into `buf` ([blocks][8][64] u64) on later launches
extern "C" void sa_raft_motion_encoder_stamps(void* buf) { g_stamps = (unsigned long long*)buf; }

extern "C" int sa_raft_motion_encoder(const float* pyr, const float* flow, int B, int H, int W, int W2, int levels,
                                      int radius, const void* w1, const float* b1, const void* w2c, const float* b2c,
                                      const void* w2f, const float* b2f, const void* w3, const float* b3, void* out,
                                      int os, hipStream_t stream) {
  return sa_raft_motion_encoder_proj(pyr, flow, B, H, W, W2, levels, radius, w1, b1, w2c, b2c, w2f, b2f, w3, b3, out,
                                     os, nullptr, nullptr, nullptr, stream);
}

extern "C" int sa_raft_motion_encoder_proj(const float* pyr, const float* flow, int B, int H, int W, int W2,
                                           int levels, int radius, const void* w1, const float* b1, const void* w2c,
                                           const float* b2c, const void* w2f, const float* b2f, const void* w3,
                                           const float* b3, void* out, int os, const float* proj,
                                           const float* proj_bias, float* flow_out, hipStream_t stream) {
  if (levels != 4 || radius != 4 || os < 128 || os % 8 || B < 1 || H < 1 || W < 1) return -2;
  if (proj && (!flow_out || flow_out == flow)) return -2;
  if (((uintptr_t)out | (uintptr_t)w1 | (uintptr_t)w2c | (uintptr_t)w2f | (uintptr_t)w3) & 15) return -2;
  long off[4] = {0, 0, 0, 0};
  long acc = 0;
  int Wl = W2;
  for (int l = 0; l < levels; ++l) {
    off[l] = acc;
    acc += (long)B * H * W * Wl;
    Wl >>= 1;
  }
  const long blocks = (long)B * ((H + TH - 1) / TH) * ((W + TW - 1) / TW);
  if (blocks > 0x7fffffffL) return -2;
  MotionEncArgs a;
  a.pyr = pyr;
  a.lvl_off1 = off[1];
  a.lvl_off2 = off[2];
  a.lvl_off3 = off[3];
  a.flow = flow;
  a.B = B;
  a.H = H;
  a.W = W;
  a.W2 = W2;
  a.levels = levels;
  a.radius = radius;
  a.w1 = (const f16*)w1;
  a.b1 = b1;
  a.w2c = (const f16*)w2c;
  a.b2c = b2c;
  a.w2f = (const f16*)w2f;
  a.b2f = b2f;
  a.w3 = (const f16*)w3;
  a.b3 = b3;
  a.out = (f16*)out;
  a.os = os;
  a.stamps = g_stamps;
  a.proj = proj;
  a.proj_bias = proj_bias;
  a.flow_out = flow_out;
  int variant = g_menc_variant;
  if (variant < 0) {
    const char* e = std::getenv("SA_RAFT_MENC");
    variant = e ? std::atoi(e) : 1;  // v2 measured slower (b8 40.71 -> 41.95 ms, b1 8.30 -> 8.68)
  }
  const bool vec = W2 % 32 == 0 && ((uintptr_t)pyr & 15) == 0;
  if (variant == 2) {
    if (vec)
      hipLaunchKernelGGL((raft_motion_encoder_v2_kernel<true>), dim3((unsigned)blocks), dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((raft_motion_encoder_v2_kernel<false>), dim3((unsigned)blocks), dim3(256), 0, stream, a);
    return (int)hipGetLastError();
  }
  if (variant == 3) {  // v1 with the conflict-free LDS layout (perm16 rows, swc pixel swizzle, bswz weight rings)
    if (vec)
      hipLaunchKernelGGL((raft_motion_encoder_kernel<4, true, true>), dim3((unsigned)blocks), dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((raft_motion_encoder_kernel<4, false, true>), dim3((unsigned)blocks), dim3(256), 0, stream, a);
    return (int)hipGetLastError();
  }
  // 4 waves (an 8-wave variant measured no faster at batch 1 and 1 % slower at batch 8)
  if (vec)
    hipLaunchKernelGGL((raft_motion_encoder_kernel<4, true>), dim3((unsigned)blocks), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL((raft_motion_encoder_kernel<4, false>), dim3((unsigned)blocks), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}