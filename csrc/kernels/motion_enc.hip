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
// resident, shared by all workgroups) are loaded as B fragments straight into registers six k-steps ahead.
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
constexpr int D = 6;                           // B-fragment prefetch depth (k-steps)

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
};

// byte offset of (pixel, 16-B chunk) in a 256-B-per-pixel LDS image
__device__ __forceinline__ int sw(int pix, int chunk) { return pix * 256 + ((chunk ^ (pix & 15)) << 4); }

// NW waves per workgroup (4: one per SIMD, 2 x 16 output channels per wave in stages 2 / 3; 8: two per SIMD,
// one 16-channel column tile per wave)
template <int NW>
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
  const int ntap = 2 * p.radius + 1, nc = p.levels * ntap;

  // ---------------- stage 0: flow patch (image rows ty0-5 .., cols tx0-5 ..), zero outside ----------------
  for (int i = tid; i < FH * FW; i += NT) {
    const int y = ty0 - 5 + i / FW, x = tx0 - 5 + i % FW;
    fl[i] = ((unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W) ? p.flow[img_base + (long)y * p.W + x] : 0.f;
  }
  __syncthreads();

  // ---------------- stage 1a: the [240 x 96] operand ----------------
  // correlation taps: one (pixel, level) per work item (bilinear, align_corners, zero padding; the same
  // arithmetic as sa_corr1d_lookup / sa_raft_motion_head).  U items per thread per pass with all their
  // ntap + 1 <= 10 row values loaded before any is used, so a pass costs one global latency, not 10 U.
  constexpr int MAXT = 10, U = NW == 4 ? 4 : 2;  // items per thread per pass (960 items of 4 levels)
  const int nitems = P1 * p.levels;
  for (int base = 0; base < nitems; base += U * NT) {
    float v[U][MAXT];
    float wa[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int it = base + u * NT + tid;
      wa[u] = 0.f;
#pragma unroll
      for (int k = 0; k < MAXT; ++k) v[u][k] = 0.f;
      if (it < nitems) {
        const int q = it / P1, pix = it - q * P1;
        const int r = pix / R1W, c = pix - r * R1W;
        const int y = ty0 - 2 + r, x = tx0 - 2 + c;
        if ((unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W) {
          const float fx = fl[(r + 3) * FW + (c + 3)];
          const long off = q == 0 ? 0 : (q == 1 ? p.lvl_off1 : (q == 2 ? p.lvl_off2 : p.lvl_off3));
          const int Wl = p.W2 >> q;
          const float* row = p.pyr + off + (img_base + (long)y * p.W + x) * Wl;
          const float xl = ((float)x + fx) / (float)(1 << q) - (float)p.radius;
          const float x0f = floorf(xl);
          wa[u] = xl - x0f;
          const int x0 = (int)x0f;
#pragma unroll
          for (int k = 0; k < MAXT; ++k) {
            const int xi = x0 + k;
            if (k <= ntap && xi >= 0 && xi < Wl) v[u][k] = row[xi];
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int it = base + u * NT + tid;
      if (it < nitems) {
        const int q = it / P1, pix = it - q * P1;
        f16* ar = a1 + pix * AS + q * ntap;
        const float a = wa[u];
#pragma unroll
        for (int k = 0; k < MAXT - 1; ++k)
          if (k < ntap) ar[k] = (f16)((1.f - a) * v[u][k] + a * v[u][k + 1]);
      }
    }
  }
  // flow taps (k = nc + ky*7 + kx) and the zero tail up to KP
  for (int it = tid; it < P1 * (KP - nc); it += NT) {
    const int pix = it / (KP - nc), k = nc + (it - pix * (KP - nc));
    const int r = pix / R1W, c = pix - r * R1W;
    float v = 0.f;
    if (k < nc + 49) {
      const int t = k - nc, ky = t / 7, kx = t - ky * 7;
      v = fl[(r + ky) * FW + (c + kx)];
    }
    a1[pix * AS + k] = (f16)v;
  }
  __syncthreads();

  // ---------------- stage 1b: S1 = relu([lookup | flow taps] x blockdiag(convc1, convf1)) ----------------
  // wave w: column tiles w * JN .. w * JN + JN - 1 of all 15 row tiles
  {
    constexpr int NT1 = P1 / 16;  // 15
    half8 bfr[JN][3];
    float bias[JN];
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int n = 16 * (wave * JN + j) + r16;
      bias[j] = p.b1[n];
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
        const half8 a = *reinterpret_cast<const half8*>(a1 + (16 * i + r16) * AS + ks * 32 + kofs);
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bfr[j][ks], acc[i][j], 0, 0, 0);
      }
#pragma unroll
    for (int i = 0; i < NT1; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int pix = 16 * i + (lane >> 4) * 4 + rr;
        const int r = pix / R1W, c = pix - r * R1W;
        const bool in = (unsigned)(ty0 - 2 + r) < (unsigned)p.H && (unsigned)(tx0 - 2 + c) < (unsigned)p.W;
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int col = 16 * (wave * JN + j) + r16;
          const float v = in ? fmaxf(acc[i][j][rr] + bias[j], 0.f) : 0.f;
          *reinterpret_cast<f16*>(s1 + sw(pix, col >> 3) + (col & 7) * 2) = (f16)v;
        }
      }
  }
  __syncthreads();

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
#pragma unroll
    for (int i = 0; i < NT2; ++i) {
      int q = 16 * i + r16;
      q = q < P2 ? q : P2 - 1;
      base[i] = (q / R2W) * R1W + (q % R2W);
    }
    const f16* wrow[JN];
#pragma unroll
    for (int j = 0; j < JN; ++j) wrow[j] = wsrc + (size_t)(nb + 16 * j + r16) * 576 + kofs;
    floatx4 acc[NT2][JN];
#pragma unroll
    for (int i = 0; i < NT2; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // B fragments D k-steps ahead in a register shift queue (a partially unrolled loop keeps every index
    // compile-time)
    half8 bq[D][JN];
#pragma unroll
    for (int st = 0; st < D; ++st)
#pragma unroll
      for (int j = 0; j < JN; ++j) bq[st][j] = *reinterpret_cast<const half8*>(wrow[j] + st * 32);
#pragma unroll 2
    for (int st = 0; st < NS2; ++st) {
      half8 b[JN];
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        b[j] = bq[0][j];
#pragma unroll
        for (int d = 0; d + 1 < D; ++d) bq[d][j] = bq[d + 1][j];
        if (st + D < NS2) bq[D - 1][j] = *reinterpret_cast<const half8*>(wrow[j] + (st + D) * 32);
      }
      const int tap = st >> 1, ky = tap / 3, kx = tap - ky * 3;
      const int toff = ky * R1W + kx;
      const int chunk = (cb + 32 * (st & 1) + kofs) >> 3;
#pragma unroll
      for (int i = 0; i < NT2; ++i) {
        const half8 a = *reinterpret_cast<const half8*>(s1 + sw(base[i] + toff, chunk));
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b[j], acc[i][j], 0, 0, 0);
      }
    }
    float bias[JN];
#pragma unroll
    for (int j = 0; j < JN; ++j) bias[j] = bsrc[nb + 16 * j + r16];
#pragma unroll
    for (int i = 0; i < NT2; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int q = 16 * i + (lane >> 4) * 4 + rr;
        if (q >= P2) continue;
        const int r = q / R2W, c = q - r * R2W;
        const bool in = (unsigned)(ty0 - 1 + r) < (unsigned)p.H && (unsigned)(tx0 - 1 + c) < (unsigned)p.W;
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int col = cb + nb + 16 * j + r16;
          const float v = in ? fmaxf(acc[i][j][rr] + bias[j], 0.f) : 0.f;
          *reinterpret_cast<f16*>(s2 + sw(q, col >> 3) + (col & 7) * 2) = (f16)v;
        }
      }
  }
  __syncthreads();

  // ---------------- stage 3: out = relu(conv([cor2 | flo2])) over the 8 x 16 tile, K = 9 x 128 ----------------
  {
    constexpr int NT3 = TH * TW / 16;  // 8 row tiles
    constexpr int NS3 = 36;            // 9 taps x 4 k32 quarters of 128 channels
    const int nb = wave * JN * 16;     // this wave's first output channel
    int base[NT3];
#pragma unroll
    for (int i = 0; i < NT3; ++i) {
      const int q = 16 * i + r16;
      base[i] = (q / TW) * R2W + (q % TW);
    }
    const f16* wrow[JN];
#pragma unroll
    for (int j = 0; j < JN; ++j) wrow[j] = p.w3 + (size_t)(nb + 16 * j + r16) * 1152 + kofs;
    floatx4 acc[NT3][JN];
#pragma unroll
    for (int i = 0; i < NT3; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // B fragments D k-steps ahead in a register shift queue (a partially unrolled loop keeps every index
    // compile-time)
    half8 bq[D][JN];
#pragma unroll
    for (int st = 0; st < D; ++st)
#pragma unroll
      for (int j = 0; j < JN; ++j) bq[st][j] = *reinterpret_cast<const half8*>(wrow[j] + st * 32);
#pragma unroll 2
    for (int st = 0; st < NS3; ++st) {
      half8 b[JN];
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        b[j] = bq[0][j];
#pragma unroll
        for (int d = 0; d + 1 < D; ++d) bq[d][j] = bq[d + 1][j];
        if (st + D < NS3) bq[D - 1][j] = *reinterpret_cast<const half8*>(wrow[j] + (st + D) * 32);
      }
      const int tap = st >> 2, ky = tap / 3, kx = tap - ky * 3;
      const int toff = ky * R2W + kx;
      const int chunk = (32 * (st & 3) + kofs) >> 3;
#pragma unroll
      for (int i = 0; i < NT3; ++i) {
        const half8 a = *reinterpret_cast<const half8*>(s2 + sw(base[i] + toff, chunk));
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b[j], acc[i][j], 0, 0, 0);
      }
    }
    // bias + relu (channels < 126), [fx, 0] tail, staged in the (finished) S1 area
    char* so = s1;
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int col = nb + 16 * j + r16;
      const float bj = col < 126 ? p.b3[col] : 0.f;
#pragma unroll
      for (int i = 0; i < NT3; ++i)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int q = 16 * i + (lane >> 4) * 4 + rr;
          const float fx = fl[((q / TW) + 5) * FW + (q % TW) + 5];
          const float v = col < 126 ? fmaxf(acc[i][j][rr] + bj, 0.f) : (col == 126 ? fx : 0.f);
          *reinterpret_cast<f16*>(so + sw(q, col >> 3) + (col & 7) * 2) = (f16)v;
        }
    }
    __syncthreads();
    for (int i = tid; i < TH * TW * 16; i += NT) {
      const int q = i >> 4, ch = i & 15;
      const int y = ty0 + q / TW, x = tx0 + q % TW;
      if (y < p.H && x < p.W)
        *reinterpret_cast<half8*>(p.out + (img_base + (long)y * p.W + x) * p.os + ch * 8) =
            *reinterpret_cast<const half8*>(so + sw(q, ch));
    }
  }
}

}  // namespace

extern "C" int sa_raft_motion_encoder(const float* pyr, const float* flow, int B, int H, int W, int W2, int levels,
                                      int radius, const void* w1, const float* b1, const void* w2c, const float* b2c,
                                      const void* w2f, const float* b2f, const void* w3, const float* b3, void* out,
                                      int os, hipStream_t stream) {
  if (levels < 1 || levels > 4 || radius < 0 || radius > 4 || levels * (2 * radius + 1) > 36 || os < 128 || os % 8 ||
      B < 1 || H < 1 || W < 1)
    return -2;
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
  // SA_MENC_WAVES=4|8 (default 4: 8 waves measured no faster at batch 1 and 1 % slower at batch 8), read per
  // launch (a frame graph captures it once)
  const char* e = std::getenv("SA_MENC_WAVES");
  const int nw = e && e[0] == '8' ? 8 : 4;
  if (nw == 4) hipLaunchKernelGGL(raft_motion_encoder_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, stream, a);
  else hipLaunchKernelGGL(raft_motion_encoder_kernel<8>, dim3((unsigned)blocks), dim3(512), 0, stream, a);
  return (int)hipGetLastError();
}
