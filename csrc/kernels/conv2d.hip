// Implicit-GEMM 2-D convolution on CDNA4 matrix cores (gfx950).
//
// GEMM view: M = N*Ho*Wo output pixels (rows), N = Cout, K = KH*KW*Cin (ordered kh, kw, ci).
// A (im2col) is gathered on the fly from NHWC fp16 activations — up to four channel-concatenated
// sources, so torch.cat([h, x...]) in ConvGRU / motion encoder never materialises.  B is the
// pre-packed fp16 weight [Cout_pad][Kpad].  Tiles: BMxBNx32 staged through LDS with register
// double buffering, v_mfma_f32_16x16x32_f16 with fp32 accumulation, 256-thread workgroups
// (4 wave64), XOR-swizzled 64-B LDS rows so the ds_read_b128 fragment reads are conflict-free
// for the 4x16-lane read groups of gfx950.
//
// Epilogues are fused: bias/scale/activation, residual+activation, ConvGRU gate math
// (z/r sigmoid, r*h, q tanh + state update), RAFT coordinate update, and per-channel
// instance-norm statistics.  This replaces the TensorRT-fused convolutions that the reference
// hides inside its engines (RAFTStereo/src/TRTRAFTStereo.cpp:137; upstream network layers per
// SURVEY.md §2.2 M1/M2).
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "sa/kernels.h"

namespace {

typedef _Float16 f16;
typedef f16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

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

__device__ __forceinline__ float sigmoidf_(float v) { return 1.f / (1.f + __expf(-v)); }
__device__ __forceinline__ float tanhf_(float v) { return act_apply(v, SA_ACT_TANH, 0.f); }

__device__ __forceinline__ void load8(const f16* p, float* v) {
  half8 h = *reinterpret_cast<const half8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)h[j];
}
__device__ __forceinline__ void store8(f16* p, const float* v) {
  half8 h;
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = (f16)v[j];
  *reinterpret_cast<half8*>(p) = h;
}

// Main-loop staging modes
enum : int {
  kRegK32 = 0,  // register-staged, BK = 32 (K not a multiple of 64)
  kRegK64 = 2,  // register-staged, BK = 64: 8 x 16-B loads in flight per thread, one barrier per 64-deep step
  kFastK64 = 3,  // kRegK64 when every source's channel count is a multiple of 64: the (tap, source,
                 // channel) position of a k-step is wave-uniform, so the im2col gather is one
                 // address add + one validity-bit test per row (per-row tap masks precomputed)
  kGlds3 = 4,    // kFastK64's uniform-k gather issued as global->LDS DMA into a 3-deep LDS ring:
                 // 8 waves, one block per CU, counted vmcnt keeps the next stage in flight across
                 // the (raw) barrier, XCD-aware tile order
  kWide = 5,     // wide tiles (256x256 / 512x128) for the big RAFT GRU / flow-head GEMMs: the same
                 // uniform-k DMA gather in BK = 32 stages through a 4-deep LDS ring (3 stages in
                 // flight), v_mfma_f32_32x32x16_f16 on a 128x64 wave tile (8 waves), one raw barrier
                 // per stage, fragment reads software-pipelined at k16 granularity; epilogue in two
                 // row bands (the fp32 C tile is staged through LDS one band at a time)
  kGldsDeep = 6,  // kGlds3 with the LDS ring as deep as 160 KB allows (up to 8 stages, NSTAGE - 1 in
                  // flight): for the small-M / deep-K convs of the coarse GRU levels and the motion
                  // encoder, whose k-steps wait on DMA latency rather than on the MFMAs
  kPing = 7,  // 8-wave ping-pong: the kWide uniform-k DMA gather (BK = 32, channel-major K order) into a 4- or
              // 6-deep LDS ring, waves 0-3 (one per SIMD) and 4-7 offset by one barrier so that on every SIMD
              // one wave runs a 16x16x32 MFMA cluster while the other reads its next fragments and issues DMA
              // (cdna_hip_programming.md §5 "256^2 8-phase template", T3-T5)
  kHalo = 9,    // 3x3 / stride 1 convs with halo reuse: the output tile is a TH x TW patch of one image (8 x 32),
                // the K loop runs channel-chunk-major (64 channels, then the 9 taps), and each chunk's input patch
                // (TH+2) x (TW+2) x 64 is DMA'd into LDS ONCE and read by all 9 taps at shifted offsets -- the im2col
                // gather fetches it 9 times.  Per 64-deep k-step the L2 -> LDS traffic drops from 48 KB (256x128
                // im2col tile) to ~21 KB (weights + 1/9 of the patch), below the per-CU LDS-DMA gather rate that
                // bounds the im2col tiles (MI355X_MICROARCH.md 'Indexed rows: gather into LDS': 66-73 GB/s per CU)
  kHalo16 = 10,  // kHalo with 16 x 16 output patches (narrow images: the 1/8 and 1/16 GRU levels)
  kHaloP = 11,   // kHalo with the input patch stored PLANAR in LDS: [8 planes of 8 channels][pixels][16 B], planes
                 // 256-B aligned.  The 16 lanes of an A fragment read 16 consecutive pixels of one plane, which hit
                 // 16 distinct 16-B bank slots at ANY start pixel, so a tap's shifted read needs no XOR swizzle: its
                 // address is the lane's tap-0 address plus a wave-uniform offset.  kHalo's swizzled image costs
                 // ~6 VALU per fragment address (3.7 VALU per MFMA on the b8 GRU conv, PMC) and 2-way conflicts
                 // on odd tap shifts (SQ_LDS_BANK_CONFLICT above the LDS instruction count)
  kHaloP16 = 12,  // kHaloP with 16 x 16 output patches
  kHaloW = 13,    // wide halo tile for the batch-8 GRU / flow-head convs: a 16 x 32 output patch (512 pixels) x 128
                  // channels, 8 waves of 128 x 64 (v_mfma_f32_16x16x32_f16, 8 x 4 fragments: 0.375 LDS reads per
                  // MFMA instead of 0.5), K in 32-channel chunks (step = chunk, tap; K = 32 per step), the input
                  // patch 18 x 34 x 32 stored planar (4 planes of 8 channels, as kHaloP) in two 40 KB buffers and a
                  // 6-deep ring of 8 KB weight stages (64-B rows, XOR-swizzled on the DMA source).  The weights --
                  // most of the L2 -> LDS traffic of a 3x3 tile -- are shared by twice the pixels of kHaloP's
                  // 256-pixel tile: 12.3 KB of DMA per 256x128x64 of MFMA work instead of 20.8
  kHaloW12 = 14,  // kHaloW with 12 x 32 output patches (384 pixels, 8 waves of 96 x 64): 120-row feature maps tile
                  // exactly (10 patch rows), no idle MFMA rows in the bottom patch
  kHaloQ = 15,    // kHaloW's tile and LDS images with a PING-PONG schedule (cdna_hip_programming.md §5 "256² 8-phase
                  // template", T3-T5): waves 0-3 (one per SIMD) and 4-7 run one barrier apart, each step is two
                  // clusters of FM/2 x FN MFMAs, and every barrier interval one group issues its MFMA cluster while
                  // the other reads its next cluster's fragments and issues DMA.  kHaloW runs both waves of a SIMD in
                  // phase, so per step the pipe idles through the barrier, the DMA issue and the LDS drain of both
                  // (ablation: the MFMA-free kernel took 75 % of the full kernel's time)
  kHaloQ12 = 16,  // kHaloQ with 12 x 32 output patches
  kRegAll = 17,   // register-staged gather (any source widths), but the global loads of the WHOLE K range (<= 8 64-deep
                  // steps) are issued up front into registers; the 2-buffer LDS stage then only pays a store + barrier
                  // per step, not a load latency.  For the tiny-K / tiny-grid convs of the latency presets (HITNet's
                  // 32-channel tile updates, K = 320), whose 2-stage pipeline waited on one load per k-step
};
__host__ __device__ constexpr bool is_glds(int mode) { return mode == kGlds3 || mode == kGldsDeep; }
__host__ __device__ constexpr bool is_halop(int mode) { return mode == kHaloP || mode == kHaloP16; }
__host__ __device__ constexpr bool is_haloq(int mode) { return mode == kHaloQ || mode == kHaloQ12; }
// kHaloW geometry (32-channel chunks, 16 x 32 / 12 x 32 patches, 6-deep 64-B-row weight ring): kHaloW and kHaloQ
__host__ __device__ constexpr bool is_halow(int mode) {
  return mode == kHaloW || mode == kHaloW12 || is_haloq(mode);
}
__host__ __device__ constexpr bool is_halo(int mode) {
  return mode == kHalo || mode == kHalo16 || is_halop(mode) || is_halow(mode);
}

template <int BM, int BN, int WM, int WN, int MODE = kRegK32>
struct ConvCfg {
  static constexpr bool WIDE = MODE == kWide;
  static constexpr bool PING = MODE == kPing;
  static constexpr bool HALOW = is_halow(MODE);
  static constexpr bool BANDED = WIDE || PING || HALOW;  // C tile staged through LDS in row bands
  static constexpr int BK = (MODE == kRegK32 || WIDE || PING || HALOW) ? 32 : 64;
  static constexpr int KCH = BK / 8;  // 16-byte chunks per row per stage
  static constexpr int TM = BM / WM, TN = BN / WN;
  // 16x16 fragment repeats (kWide keeps its own 32x32 accumulators: a 1x1 placeholder here)
  static constexpr int FM = WIDE ? 1 : TM / 16, FN = WIDE ? 1 : TN / 16;
  static constexpr int A_CH = BM * KCH, B_CH = BN * KCH;  // 16-byte chunks per stage
  static constexpr int NW = WM * WN, NT = 64 * NW;  // waves / threads per workgroup
  static constexpr int A_PT = (A_CH + NT - 1) / NT, B_PT = (B_CH + NT - 1) / NT;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  // kGlds3: three-deep LDS ring; kGldsDeep: as deep as 160 KB allows (<= 8); kWide: four-deep; everything
  // else double-buffered
  static constexpr int DEEP_NS = 163840 / (A_BYTES + B_BYTES) < 8 ? 163840 / (A_BYTES + B_BYTES) : 8;
  // kPing: as deep as 144 KB allows, at most 6 (256x256: 4 stages, 256x128: 6; a 5-deep 256x256 ring measured
  // the same)
  static constexpr int PING_NS = 147456 / (A_BYTES + B_BYTES) < 6 ? 147456 / (A_BYTES + B_BYTES) : 6;
  static constexpr bool HALO = is_halo(MODE);
  static constexpr int NSTAGE = is_haloq(MODE) ? 9 : HALOW ? 6 : MODE == kGlds3 || HALO ? 3 : MODE == kGldsDeep ? DEEP_NS : PING ? PING_NS : (WIDE ? 4 : 2);
  // kHalo: output patch TH x TW, input patch (TH+2) x (TW+2) pixels of 128 B (one 64-channel chunk) in 1-KB DMA
  // pieces of 8 pixels, HALO_NA pieces per wave; two patch buffers + a 3-deep ring of weight stages
  static constexpr int TW = (MODE == kHalo16 || MODE == kHaloP16) ? 16 : 32;
  static constexpr int HALO_PIX = (BM / TW + 2) * (TW + 2);
  // kHaloP: plane length in pixels (a multiple of 16: planes start on 256-B boundaries); 8 planes of HALO_RPP 16-B
  // slots fill HALO_RPP / 8 DMA instructions of 64 lanes
  static constexpr bool HALOP = is_halop(MODE);
  static constexpr int HALO_RPP = (HALO_PIX + 15) / 16 * 16;
  // kHaloW: 4 planes of 8 channels (a 32-channel chunk)
  static constexpr int HALO_PLANES = HALOW ? 4 : 8;
  static constexpr int HALO_CH = HALOW ? 32 : 64;  // channels per K chunk (a split launch cuts K at chunk boundaries)
  static constexpr int HALO_NA = !HALO ? 1
                                 : (HALOP || HALOW) ? (HALO_RPP * HALO_PLANES / 64 + NW - 1) / NW
                                                    : ((HALO_PIX + 7) / 8 + NW - 1) / NW;
  static constexpr int A_PATCH = HALO_NA * NW * 1024;
  static constexpr int STAGE_BYTES = HALO ? 2 * A_PATCH + NSTAGE * B_BYTES : NSTAGE * (A_BYTES + B_BYTES);
  // fp32 C tile, unpadded rows; columns XOR-swizzled in 16-float blocks (cswz) so the MFMA
  // write-out (4 row groups x 16 lanes) hits 64 distinct banks; aliases the stage buffers.
  // kWide stages it in bands of CROWS rows (128 KB of fp32 per band)
  static constexpr int CST = BN;
  // kHaloW: bands of whole wave rows (TM), 2 per band (128 KB at 16 x 32)
  static constexpr int CROWS = HALOW ? 2 * TM : BANDED ? (32768 / BN < BM ? 32768 / BN : BM) : BM;
  static constexpr int C_BYTES = CROWS * CST * 4;
  static constexpr int SMEM = STAGE_BYTES > C_BYTES ? STAGE_BYTES : C_BYTES;
  static_assert(WM * WN == 4 || (WM * WN == 8 && (is_glds(MODE) || WIDE || PING || HALO)), "4 waves (8 for kGlds3; 4 or 8 for kWide) per workgroup");
  static_assert(!HALO || (BM % TW == 0 && TM % 16 == 0 && TW % 16 == 0 && BK == (HALOW ? 32 : 64)), "halo tiles: 16-pixel fragments inside one output row");
  static_assert(!HALOW || (WM == 4 && WN == 2 && TM % TW == 0), "kHaloW: 4 x 2 waves, whole patch rows per wave");
  static_assert(!PING || (WM == 2 && WN == 4 && BM == 256), "kPing: 2 x 4 waves, one 128-row half of the tile per wave group");
  static_assert(!is_glds(MODE) || NSTAGE >= 3, "DMA rings keep at least one stage in flight across the barrier");
  static_assert(TM % 16 == 0 && TN % 16 == 0, "wave tile must be 16-aligned");
  static_assert(!WIDE || (TM == 128 && (TN == 64 || TN == 128)), "kWide: 128x64 or 128x128 wave tiles");
};

// swizzled byte offset of (row, 16B-chunk) inside a [rows][32 halfs] stage buffer
__device__ __forceinline__ int swz(int row, int c) { return row * 64 + ((c ^ (((row >> 3) & 1) * 3)) << 4); }
// C-tile column swizzle: 16-float blocks XOR ((row >> 2) & 3) (keeps 8-float chunks contiguous);
// identity when the tile is narrower than 64 columns
template <int BN>
__device__ __forceinline__ int cswz_t(int row, int col) {
  if constexpr (BN >= 64) return col ^ (((row >> 2) & 3) << 4);
  else return col;
}
#define cswz(row, col) cswz_t<BN>(row, col)
// [rows][64 halfs] stage buffer (128-B rows): chunk XOR (row>>1)&7 — the 16 rows x one chunk of a
// ds_read_b128 lane group land in 16 distinct 16-B bank slots
__device__ __forceinline__ int swz64(int row, int c) { return row * 128 + ((c ^ ((row >> 1) & 7)) << 4); }

// 16 zero bytes in global memory: the source of every padded / out-of-range im2col chunk in the
// DMA path (a masked-off lane would leave stale LDS behind)
__device__ __attribute__((aligned(16))) const unsigned char g_zero16[64] = {0};

typedef __attribute__((address_space(3))) void lds_void_t;

// compile-time loop: f(std::integral_constant<int, I>{}) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Ablation switches of the halo main loops (tools/exp_build.sh -DSA_EXP_HALO_...; timing experiments only, results
// are wrong): no LDS DMA, no fragment reads, no barriers, no MFMAs
#ifdef SA_EXP_HALO_NODMA
#define SA_HALO_GLDS(g, l, n, o, x) asm volatile("" ::"v"(g))
#else
#define SA_HALO_GLDS __builtin_amdgcn_global_load_lds
#endif
#ifdef SA_EXP_HALO_NOREAD
#define SA_HALO_LD(p) (__extension__({ half8 v_; asm volatile("" : "=v"(v_)); v_; }))
#else
#define SA_HALO_LD(p) (*reinterpret_cast<const half8*>(p))
#endif
#ifdef SA_EXP_HALO_NOBAR
#define SA_HALO_BAR() do { } while (0)
#else
#define SA_HALO_BAR() __builtin_amdgcn_s_barrier()
#endif
#ifdef SA_EXP_HALO_NOMFMA
#define SA_HALO_MFMA(a, b, c, x, y, z) (__extension__({ asm volatile("" :: "v"(a), "v"(b)); (c); }))
#else
#define SA_HALO_MFMA __builtin_amdgcn_mfma_f32_16x16x32_f16
#endif

#define SA_STR2(x) #x
#define SA_STR(x) SA_STR2(x)
// s_waitcnt vmcnt(N) with a compile-time N (the asm string needs a literal)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 32, "vmcnt literal");
#define SA_VMCNT_CASE(k) \
  if constexpr (N == k) asm volatile("s_waitcnt vmcnt(" SA_STR(k) ")" ::: "memory");
  SA_VMCNT_CASE(0) SA_VMCNT_CASE(1) SA_VMCNT_CASE(2) SA_VMCNT_CASE(3) SA_VMCNT_CASE(4) SA_VMCNT_CASE(5)
  SA_VMCNT_CASE(6) SA_VMCNT_CASE(7) SA_VMCNT_CASE(8) SA_VMCNT_CASE(9) SA_VMCNT_CASE(10) SA_VMCNT_CASE(11)
  SA_VMCNT_CASE(12) SA_VMCNT_CASE(13) SA_VMCNT_CASE(14) SA_VMCNT_CASE(15) SA_VMCNT_CASE(16) SA_VMCNT_CASE(17)
  SA_VMCNT_CASE(18) SA_VMCNT_CASE(19) SA_VMCNT_CASE(20) SA_VMCNT_CASE(21) SA_VMCNT_CASE(22) SA_VMCNT_CASE(23)
  SA_VMCNT_CASE(24) SA_VMCNT_CASE(25) SA_VMCNT_CASE(26) SA_VMCNT_CASE(27) SA_VMCNT_CASE(28) SA_VMCNT_CASE(29)
  SA_VMCNT_CASE(30) SA_VMCNT_CASE(31) SA_VMCNT_CASE(32)
#undef SA_VMCNT_CASE
}

// s_waitcnt vmcnt(s * PER) for a wave-uniform s in [0, K]: "at most s stages of PER DMA instructions each are
// still in flight"
template <int PER, int K>
__device__ __forceinline__ void wait_stages(int s) {
  if constexpr (K <= 0) {
    wait_vmcnt<0>();
  } else {
    if (s >= K) wait_vmcnt<K * PER>();
    else wait_stages<PER, K - 1>(s);
  }
}

// One (tile, k-range) work item of the implicit GEMM: the output tile (bx, by) over k-steps [kt0, kt0 + nk).
// S > 1: this item is contributor z of the S items of tile `ctr`; it writes its partial sums to its slab and
// the last contributor to arrive (counter ctr) sums the S contributors' slabs in contributor order and runs
// the epilogue.  Grid mode (skG == 0): contributor c's slab is slab_base + c.  Stream-K (skG = G blocks over
// skI k-steps): contributor c is block b = slab_base + c, and since only a block's first and last segments
// can be partial tiles its slab is 2b (the segment starts the block's range) or 2b + 1, so 2G slabs cover
// any tile count.  Called once per block (grid tiling / split-K) or once per segment of a stream-K block.
//
// EXT (split-K over workgroups without a cross-workgroup handshake, tactics 37 / 38): EXT = 1 runs the K range and
// stores the fp32 partial tile into slice z of the row-major [S][M][LD] workspace p.ws (LD = Cout rounded up to 64),
// no epilogue; EXT = 2 replaces the main loop by the sum of the p.splitk slices of its own (smaller) tile in fixed
// order and runs the normal epilogue.  The two are separate launches on one stream, so the kernel boundary orders
// the partials: no agent-scope release / acquire fences (~3.5 us each per workgroup, the cost that made the
// last-arriver split slower than no split on the small coarse-level GRU grids).
template <int BM, int BN, int WM, int WN, int MODE, int EXT = 0>
__device__ __forceinline__ void conv_tile(const SaConvArgs& p, char* smem, const int bx, const int by, const int kt0,
                                          const int nk, const int S, const int z, const int slab_base,
                                          const int ctr, const int skG, const long skI) {
  using C = ConvCfg<BM, BN, WM, WN, MODE>;
  static_assert(EXT == 0 || (!C::BANDED && !C::HALO), "workgroup split-K: plain tiles only");

  // opaque per call: in the stream-K segment loop nothing lane-dependent is hoisted out of the loop (it would
  // stay live across the main loop)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar LDS bases)
  const int wm = wave / WN, wn = wave % WN;

  constexpr int NT = C::NT;
  const int HWo = p.Ho * p.Wo;
  // 3-D mode (KD > 0): rows enumerate (n, do, oh, ow); 2-D is KD = Di = Do = 1
  const int KD = p.KD > 0 ? p.KD : 1, Di = p.Di > 0 ? p.Di : 1, Do = p.Do > 0 ? p.Do : 1;
  const int sd = p.sd > 0 ? p.sd : 1;
  const int M = p.N * Do * HWo;
  // kHalo: bx enumerates (image, patch row, patch column); m0 is the image's first pixel (statistics bookkeeping)
  const int halo_tx = C::HALO ? (p.Wo + C::TW - 1) / C::TW : 1, halo_ty = C::HALO ? (p.Ho + BM / C::TW - 1) / (BM / C::TW) : 1;
  const int halo_img = C::HALO ? bx / (halo_tx * halo_ty) : 0;
  const int halo_oy0 = C::HALO ? ((bx - halo_img * halo_tx * halo_ty) / halo_tx) * (BM / C::TW) : 0;
  const int halo_ox0 = C::HALO ? ((bx - halo_img * halo_tx * halo_ty) % halo_tx) * C::TW : 0;
  const int m0 = C::HALO ? halo_img * HWo : bx * BM;
  const int n0 = by * BN;
  const int khw = p.KH * p.KW;
  const int taps = KD * khw;

  floatx4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // kWide: 4 x (2 or 4) blocks of 32x32 per wave (C/D: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5))
  constexpr int WFM = C::WIDE ? 4 : 1, WFN = C::WIDE ? C::TN / 32 : 1;
  floatx16 acc32[WFM][WFN];
  if constexpr (C::WIDE) {
#pragma unroll
    for (int i = 0; i < WFM; ++i)
#pragma unroll
      for (int j = 0; j < WFN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc32[i][j][r] = 0.f;
  }
  if constexpr (EXT == 2) {
    // ---------------- split-K reduction: sum the S partial slices (fixed order) into the accumulators ----------------
    // slice layout [S][LD][Mp] (column-major: a lane's 4 accumulator rows are one 16-B load); all S x FM x FN loads
    // are issued before the sums
    const int LD = (p.Cout + 63) & ~63, Mp = (M + 3) & ~3;
    const int Sx = p.splitk;
    floatx4 part[8][C::FM][C::FN];
#pragma unroll
    for (int sl = 0; sl < 8; ++sl)
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) {
          const int m = m0 + wm * C::TM + i * 16 + (lane >> 4) * 4;
          const int n = n0 + wn * C::TN + j * 16 + (lane & 15);
          part[sl][i][j] = (sl < Sx && m < M && n < LD)
                               ? *reinterpret_cast<const floatx4*>(p.ws + ((size_t)sl * LD + n) * Mp + m)
                               : floatx4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        floatx4 v = part[0][i][j];
#pragma unroll
        for (int sl = 1; sl < 8; ++sl) v += part[sl][i][j];
        acc[i][j] = v;
      }
  } else if constexpr (MODE == kFastK64) {
    // ---------------- uniform-k im2col, register staged, BK = 64 ----------------
    constexpr int RPT = C::A_PT;  // A rows per thread: (tid >> 3) + 32 i
    const int cth = tid & 7;
    const int KH = p.KH, KW = p.KW;
    long pixb[RPT];
    unsigned long long vmask[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int row = (tid >> 3) + 32 * i;
      const int m = m0 + row;
      const bool ok = m < M;
      const int mm = ok ? m : 0;
      const int img = mm / HWo;
      const int r = mm - img * HWo;
      const int oh = r / p.Wo, ow = r - oh * p.Wo;
      const int n = img / Do, od = img - n * Do;
      const int ih0 = oh * p.sh - p.ph, iw0 = ow * p.sw - p.pw, id0 = od * sd - p.pd;
      pixb[i] = (((long)n * Di + id0) * p.H + ih0) * p.W + iw0;
      unsigned long long mk = 0ull;
      int t = 0;
      for (int kd = 0; kd < KD; ++kd)
        for (int kh = 0; kh < KH; ++kh)
          for (int kw = 0; kw < KW; ++kw, ++t) {
            const int dd = id0 + kd, ih = ih0 + kh * p.dh, iw = iw0 + kw * p.dw;
            if (ok && dd >= 0 && dd < Di && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W) mk |= 1ull << t;
          }
      vmask[i] = mk;
    }
    // wave-uniform k position: tap (kd, kh, kw), pixel offset of the tap, channel within the tap
    int kc = kt0 * 64;
    int tap = kc / p.Cin, ci0 = kc - tap * p.Cin;
    int kd_ = tap / (KH * KW), kr = tap - kd_ * KH * KW;
    int kh_ = kr / KW, kw_ = kr - kh_ * KW;
    long toff = ((long)kd_ * p.H + (long)kh_ * p.dh) * p.W + (long)kw_ * p.dw;
    const int sb1 = p.src[0].channels;
    const int sb2 = sb1 + (p.nsrc > 1 ? p.src[1].channels : 0);
    const int sb3 = sb2 + (p.nsrc > 2 ? p.src[2].channels : 0);
    const f16* wrow[C::B_PT];
#pragma unroll
    for (int j = 0; j < C::B_PT; ++j) {
      const int row = (tid >> 3) + 32 * j;
      wrow[j] = reinterpret_cast<const f16*>(p.weight) + (size_t)(n0 + (row < BN ? row : 0)) * p.Kpad + kc + cth * 8;
    }
    const half8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
    half8 ra[RPT], rb[C::B_PT];
    auto load_tile = [&]() {
      const int s = (ci0 >= sb1) + (ci0 >= sb2) + (ci0 >= sb3);
      const int cbase = s == 0 ? 0 : (s == 1 ? sb1 : (s == 2 ? sb2 : sb3));
      const f16* sp = reinterpret_cast<const f16*>(p.src[s].ptr) + (ci0 - cbase) + cth * 8;
      const long sst = p.src[s].stride;
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const bool v = (vmask[i] >> tap) & 1ull;
        const f16* a = sp + (pixb[i] + toff) * sst;
        ra[i] = v ? *reinterpret_cast<const half8*>(a) : zero8;
      }
#pragma unroll
      for (int j = 0; j < C::B_PT; ++j) {
        if ((tid >> 3) + 32 * j < BN) rb[j] = *reinterpret_cast<const half8*>(wrow[j]);
        wrow[j] += 64;
      }
      // advance the uniform k position by 64 channels
      ci0 += 64;
      if (ci0 >= p.Cin) {
        ci0 = 0;
        ++tap;
        ++kw_;
        toff += p.dw;
        if (kw_ == KW) {
          kw_ = 0;
          toff += (long)p.dh * p.W - (long)KW * p.dw;
          ++kh_;
          if (kh_ == KH) {
            kh_ = 0;
            toff += (long)p.H * p.W - (long)KH * p.dh * p.W;
          }
        }
      }
    };
    auto store_tile = [&](int buf) {
      char* sa = smem + buf * (C::A_BYTES + C::B_BYTES);
      char* sb = sa + C::A_BYTES;
#pragma unroll
      for (int i = 0; i < RPT; ++i) *reinterpret_cast<half8*>(sa + swz64((tid >> 3) + 32 * i, cth)) = ra[i];
#pragma unroll
      for (int j = 0; j < C::B_PT; ++j)
        if ((tid >> 3) + 32 * j < BN) *reinterpret_cast<half8*>(sb + swz64((tid >> 3) + 32 * j, cth)) = rb[j];
    };
    const int frow = lane & 15;
    if (nk > 0) {
      load_tile();
      store_tile(0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) load_tile();
      const char* sa = smem + cur * (C::A_BYTES + C::B_BYTES);
      const char* sb = sa + C::A_BYTES;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        half8 af[C::FM], bf[C::FN];
        const int lc = (lane >> 4) + 4 * kk;
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
          af[i] = *reinterpret_cast<const half8*>(sa + swz64(wm * C::TM + i * 16 + frow, lc));
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          bf[j] = *reinterpret_cast<const half8*>(sb + swz64(wn * C::TN + j * 16 + frow, lc));
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
      if (kt + 1 < nk) store_tile(cur ^ 1);
      __syncthreads();
    }
  } else if constexpr (is_haloq(MODE)) {
    // ---------------- kHaloQ: kHaloW's LDS images, ping-pong schedule ----------------
    // Group g = wave >> 2 (waves 0-3 / 4-7: one wave of each group per SIMD).  Barrier interval n: group 0 is in the
    // LOAD segment of step n / 2 (n even) or runs that step's MFMAs (n odd); group 1 the same one interval later (its
    // extra barrier before the loop, and group 0's after it, keep the barrier counts equal), so on every SIMD one
    // wave's FM x FN MFMA cluster (512 cycles at 16 x 32) runs beside the partner's LOAD segment.  Per step:
    //   LOAD: DMA issue (patch(c + 1) at tap 1, then W(s + L)), all FM + FN fragment reads of the step, vmcnt wait
    //         for W(s + 1); s_barrier
    //   MFMA: lgkmcnt(0) (own reads), setprio 1, FM x FN MFMAs, setprio 0; s_barrier
    // The loop runs per 32-channel chunk with its 9 taps unrolled and a 9-slot weight ring (slot = tap), so every
    // LDS offset is an immediate and every vmcnt count a constant: past the K range the DMA issues continue as
    // dummies (an in-range source into a slot / patch buffer no later step reads), keeping the counts static.
    // (A first version with runtime step arithmetic ran ~150 SALU/VALU per wave and step: its MFMA-free ablation
    // took 290 us of the 329 us zr8 conv; two 16-MFMA clusters per step were 15-20 % slower than one of 32.)
    // RAW: W(s + 1) is waited for by EVERY wave in its LOAD(s), before the barrier that precedes group 0's LOAD(s + 1)
    // (for group 0 one barrier early).  Patch(c + 1) is issued 8 steps before its first read and waited for from
    // tap L on.  WAR: W(s + L) refills the slot of W(s + L - 9), read >= 3 steps back and consumed by an MFMA
    // segment of every wave since; patch(c + 1) (tap 1 of chunk c) refills chunk c - 1's buffer, last read in step
    // 9c - 1, likewise consumed since.
    constexpr int TW = C::TW, PW = TW + 2, RP = C::HALO_PIX;
    constexpr int NAH = C::HALO_NA, NS = C::NSTAGE, L = 6;
    static_assert(NS == 9 && L <= NS - 3, "kHaloQ: one weight slot per tap, the refilled slot read >= 3 steps back");
    constexpr int NB = BN * 4 / NT;
    static_assert(NB * NT == BN * 4 && NB >= 1, "whole-wave weight DMA pieces");
    constexpr int APB = C::A_PATCH, BST = BN * 64;
    constexpr int RPP = C::HALO_RPP, APL = RPP * 16;
    static_assert(2 * APB + NS * BST <= C::SMEM, "kHaloQ buffers fit");
    static_assert(NAH * C::NW * 64 >= 4 * RPP && RPP % 16 == 0, "kHaloQ: the DMA instructions cover all 4 planes");
    char* const abuf0 = smem;
    char* const bbuf0 = smem + 2 * APB;
    const int Cin = p.Cin;
    const int grp = wave >> 2;
    const int cb = kt0 / 9, ce = (kt0 + nk) / 9;
    const int nch = Cin >> 5;  // chunks of the whole K (dummy DMA sources stay below it)
    // patch DMA: piece (wave, i) fills LDS slots (wave * NAH + i) * 64 + lane = plane * RPP + pixel; apix[i] is the
    // source pixel (-1: padding / outside the patch -> zeros), the plane is recomputed at issue time
    int apix[NAH];
#pragma unroll
    for (int i = 0; i < NAH; ++i) {
      const int slot = (wave * NAH + i) * 64 + lane;
      const int pl = slot / RPP, q = slot - pl * RPP;
      const int qy = q / PW, qx = q - qy * PW;
      const int iy = halo_oy0 - 1 + qy, ix = halo_ox0 - 1 + qx;
      const bool ok = pl < 4 && q < RP && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
      apix[i] = ok ? (halo_img * p.H + iy) * p.W + ix : -1;
    }
    const int sb1 = p.src[0].channels;
    const int sb2 = sb1 + (p.nsrc > 1 ? p.src[1].channels : 0);
    const int sb3 = sb2 + (p.nsrc > 2 ? p.src[2].channels : 0);
    const f16* sp0 = reinterpret_cast<const f16*>(p.src[0].ptr);
    const f16* sp1 = reinterpret_cast<const f16*>(p.src[p.nsrc > 1 ? 1 : 0].ptr);
    const f16* sp2 = reinterpret_cast<const f16*>(p.src[p.nsrc > 2 ? 2 : 0].ptr);
    const f16* sp3 = reinterpret_cast<const f16*>(p.src[p.nsrc > 3 ? 3 : 0].ptr);
    const int ss0 = p.src[0].stride, ss1 = p.src[p.nsrc > 1 ? 1 : 0].stride;
    const int ss2 = p.src[p.nsrc > 2 ? 2 : 0].stride, ss3 = p.src[p.nsrc > 3 ? 3 : 0].stride;
    const f16* wrow[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int row = (wave * NB + j) * 16 + (lane >> 2);
      const int g = (0 - (row >> 2)) & 3;
      wrow[j] = reinterpret_cast<const f16*>(p.weight) + (size_t)(n0 + row) * p.Kpad + (((lane & 3) ^ g) << 3);
    }
    const char* const zero_src = reinterpret_cast<const char*>(g_zero16);
    // patch of chunk c (clamped into the K range: a dummy past it) into buffer buf
    auto issue_a = [&](int c, int buf) {
      const int ci = (c < nch ? c : nch - 1) << 5;
      const f16* sp;
      int sst;
      if (ci < sb1) { sp = sp0 + ci; sst = ss0; }
      else if (ci < sb2) { sp = sp1 + (ci - sb1); sst = ss1; }
      else if (ci < sb3) { sp = sp2 + (ci - sb2); sst = ss2; }
      else { sp = sp3 + (ci - sb3); sst = ss3; }
      char* dst = abuf0 + buf * APB;
#pragma unroll
      for (int i = 0; i < NAH; ++i) {
        const int pl = ((wave * NAH + i) * 64 + lane) / RPP;
        const f16* src = sp + (size_t)(apix[i] < 0 ? 0 : apix[i]) * sst + (pl << 3);
        const void* g = apix[i] >= 0 ? (const void*)src : (const void*)zero_src;
        SA_HALO_GLDS(g, (lds_void_t*)(dst + (wave * NAH + i) * 1024), 16, 0, 0);
      }
    };
    // weights of (chunk c, tap t) into slot t (c clamped into the K range: a dummy past it)
    auto issue_b = [&](int c, int t) {
      const int koff = t * Cin + ((c < nch ? c : nch - 1) << 5);
      char* dst = bbuf0 + t * BST;
#pragma unroll
      for (int j = 0; j < NB; ++j)
        SA_HALO_GLDS((const void*)(wrow[j] + koff), (lds_void_t*)(dst + (wave * NB + j) * 1024), 16, 0, 0);
    };
    const int frow = lane & 15;
    const int abase = (lane >> 4) * APL + ((wm * (C::TM / TW)) * PW + frow) * 16;
    const int bbase = (wn * C::TN + frow) * 64 + (((lane >> 4) ^ ((0 - (frow >> 2)) & 3)) << 4);
    char* const bptr = bbuf0 + bbase;
    // prologue: patch(cb) and W(s0 .. s0 + L - 1), all landed before the first barrier
    issue_a(cb, cb & 1);
#pragma unroll
    for (int k = 0; k < L; ++k) issue_b(cb + k / 9, k % 9);
    wait_vmcnt<0>();
    SA_HALO_BAR();
    if (grp == 1) SA_HALO_BAR();
    asm volatile("" ::: "memory");
    half8 a[C::FM], b[C::FN];
    for (int c = cb; c < ce; ++c) {
      char* const aptr = abuf0 + (c & 1) * APB + abase;
      static_for<0, 9>([&](auto T) {
        constexpr int t = decltype(T)::value;
        constexpr int ty = t / 3, tx = t % 3;
        // ---- step (c, t): LOAD -- DMA issue, every fragment of the step, wait for W(s + 1) ----
        if constexpr (t == 1) issue_a(c + 1, (c + 1) & 1);
        issue_b(c + (t + L) / 9, (t + L) % 9);
#pragma unroll
        for (int j = 0; j < C::FN; ++j) b[j] = SA_HALO_LD(bptr + t * BST + j * 1024);
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
          a[i] = SA_HALO_LD(aptr + (((i * 16) / TW + ty) * PW + (i * 16) % TW + tx) * 16);
        // pieces issued after W(s + 1): W(s + 2 .. s + L) and, at taps 1 .. L - 1, this chunk's patch
        if constexpr (t >= 1 && t < L) wait_vmcnt<(L - 1) * NB + NAH>();
        else wait_vmcnt<(L - 1) * NB>();
        SA_HALO_BAR();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        // ---- step (c, t): MFMA ----
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j) acc[i][j] = SA_HALO_MFMA(a[i], b[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        SA_HALO_BAR();
      });
    }
    if (grp == 0) SA_HALO_BAR();
    wait_vmcnt<0>();  // the trailing dummy DMAs land before the epilogue reuses LDS
    __syncthreads();
  } else if constexpr (C::HALOW) {
    // ---------------- kHaloW: 3x3 halo patch (32-channel chunks) + 6-deep weight ring, 128 x 64 wave tiles ------
    // Step s = (chunk c = s / 9 of 32 channels, tap t = s % 9), K = 32 per step (one v_mfma_f32_16x16x32_f16 per
    // fragment pair).  LDS: patch buffers [2][A_PATCH] (planar: plane pl = 8 channels at pl * APL, pixel q of the
    // (TH+2) x (TW+2) patch at q * 16 B), then the weight ring [NS][BN rows][64 B] whose 16-B slot kb of row n holds
    // channels 8 (kb ^ g(n)), g(n) = -(n >> 2) & 3 (applied to the DMA SOURCE address, the image stays lane-linear),
    // so every ds_read_b128 lane group of a B fragment hits 16 distinct bank slots.
    // Schedule of step s (one raw barrier per step):
    //   B_s: lgkmcnt(0) (this wave's reads of step s into Fc are done), vmcnt(<= pieces issued after W(s+1)),
    //        s_barrier -- W(s+1) and the patch of s+1's chunk have landed for every wave, and every wave finished
    //        reading step s - 1's weight slot and, at a chunk boundary, the previous chunk's patch buffer
    //   issue: patch(c + 2) into buffer c & 1 when t == 8; W(s + NS - 1) into slot (s - 1) % NS
    //   MFMAs of step s (Fc) with the fragment reads of step s + 1 (Fn) interleaved, one read per MFMA
    constexpr int TW = C::TW, TH = BM / TW, PW = TW + 2, RP = C::HALO_PIX;
    constexpr int NAH = C::HALO_NA, NS = C::NSTAGE;
    constexpr int NB = BN * 4 / NT;  // 1-KB weight pieces per wave per step (16 rows of 64 B each)
    static_assert(NB * NT == BN * 4 && NB >= 1, "whole-wave weight DMA pieces");
    constexpr int APB = C::A_PATCH, BST = BN * 64;
    constexpr int RPP = C::HALO_RPP, APL = RPP * 16;
    static_assert(2 * APB + NS * BST <= C::SMEM, "kHaloW buffers fit");
    static_assert(NAH * C::NW * 64 >= 4 * RPP && RPP % 16 == 0, "kHaloW: the DMA instructions cover all 4 planes");
    static_assert(C::FM * C::FN >= C::FM + C::FN, "one fragment read per MFMA slot");
    char* const abuf0 = smem;
    char* const bbuf0 = smem + 2 * APB;
    const int Cin = p.Cin;
    const int cb = kt0 / 9, ce = (kt0 + nk) / 9;
    const int s0 = kt0, s1 = kt0 + nk;
    // patch DMA: instruction (wave, i) fills LDS slots (wave * NAH + i) * 64 + lane = plane * RPP + pixel; apix[i]
    // is the source pixel (-1: padding / outside the patch, loads zeros), the plane is recomputed at issue time
    int apix[NAH];
#pragma unroll
    for (int i = 0; i < NAH; ++i) {
      const int slot = (wave * NAH + i) * 64 + lane;
      const int pl = slot / RPP, q = slot - pl * RPP;
      const int qy = q / PW, qx = q - qy * PW;
      const int iy = halo_oy0 - 1 + qy, ix = halo_ox0 - 1 + qx;
      const bool ok = pl < 4 && q < RP && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
      apix[i] = ok ? (halo_img * p.H + iy) * p.W + ix : -1;
    }
    const int sb1 = p.src[0].channels;
    const int sb2 = sb1 + (p.nsrc > 1 ? p.src[1].channels : 0);
    const int sb3 = sb2 + (p.nsrc > 2 ? p.src[2].channels : 0);
    const f16* sp0 = reinterpret_cast<const f16*>(p.src[0].ptr);
    const f16* sp1 = reinterpret_cast<const f16*>(p.src[p.nsrc > 1 ? 1 : 0].ptr);
    const f16* sp2 = reinterpret_cast<const f16*>(p.src[p.nsrc > 2 ? 2 : 0].ptr);
    const f16* sp3 = reinterpret_cast<const f16*>(p.src[p.nsrc > 3 ? 3 : 0].ptr);
    const int ss0 = p.src[0].stride, ss1 = p.src[p.nsrc > 1 ? 1 : 0].stride;
    const int ss2 = p.src[p.nsrc > 2 ? 2 : 0].stride, ss3 = p.src[p.nsrc > 3 ? 3 : 0].stride;
    // weight DMA: piece j of this wave = rows (wave * NB + j) * 16 + (lane >> 2), slot lane & 3 <- channels
    // 8 ((lane & 3) ^ g(row))
    const f16* wrow[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int row = (wave * NB + j) * 16 + (lane >> 2);
      const int g = (0 - (row >> 2)) & 3;
      wrow[j] = reinterpret_cast<const f16*>(p.weight) + (size_t)(n0 + row) * p.Kpad + (((lane & 3) ^ g) << 3);
    }
    const void* zero_src = g_zero16;
    auto issue_a = [&](int c, int buf) {
      const int ci = c << 5;
      const f16* sp;
      int sst;
      if (ci < sb1) { sp = sp0 + ci; sst = ss0; }
      else if (ci < sb2) { sp = sp1 + (ci - sb1); sst = ss1; }
      else if (ci < sb3) { sp = sp2 + (ci - sb2); sst = ss2; }
      else { sp = sp3 + (ci - sb3); sst = ss3; }
      char* dst = abuf0 + buf * APB;
#pragma unroll
      for (int i = 0; i < NAH; ++i) {
        const int pl = ((wave * NAH + i) * 64 + lane) / RPP;
        const void* g = apix[i] >= 0 ? (const void*)(sp + (size_t)apix[i] * sst + (pl << 3)) : zero_src;
        __builtin_amdgcn_global_load_lds(g, (lds_void_t*)(dst + (wave * NAH + i) * 1024), 16, 0, 0);
      }
    };
    auto issue_b = [&](int st) {
      const int c = st / 9, t = st - c * 9;
      const int koff = t * Cin + (c << 5);
      char* dst = bbuf0 + (st % NS) * BST;
#pragma unroll
      for (int j = 0; j < NB; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(wrow[j] + koff), (lds_void_t*)(dst + (wave * NB + j) * 1024), 16,
                                         0, 0);
    };
    const int frow = lane & 15;
    // fragment i of this wave: output pixels (wm * TM + i * 16 + frow) -> patch row wm * TM / TW + (i * 16) / TW,
    // column (i * 16) % TW + frow; the lane reads plane lane >> 4.  Everything but the lane base is an immediate.
    const int abase = (lane >> 4) * APL + ((wm * (C::TM / TW)) * PW + frow) * 16;
    const int bbase = (wn * C::TN + frow) * 64 + (((lane >> 4) ^ ((0 - (frow >> 2)) & 3)) << 4);
    auto addr_a = [&](int st, int i) {
      const int c = st / 9, t = st - c * 9;
      const int ty = t / 3, tx = t - ty * 3;
      return abuf0 + (c & 1) * APB + abase + (((i * 16) / TW + ty) * PW + (i * 16) % TW + tx) * 16;
    };
    auto addr_b = [&](int st, int j) { return bbuf0 + (st % NS) * BST + bbase + j * 16 * 64; };
    // MFMAs of one step, fragment-row-major, with the next step's fragment reads interleaved: the B fragments of
    // the next step go to the other B set (bn), and A fragment i of the next step REPLACES a[i] right after its
    // last MFMA (i, FN - 1) -- one A set instead of two keeps the 128 accumulators + fragments within 256 VGPRs
    // The reads are unconditional: after the last step they re-read in-bounds LDS nobody uses (a runtime condition
    // per read makes hipcc branch around every ds_read inside the MFMA stream)
    // sched_group_barrier pins the interleave: M R M R M R M R | R | (M M M M R) x (FM - 1) -- every read issued
    // right behind the MFMA that frees its register, so it has the rest of the step to land
    auto mfma_step = [&](half8* a, const half8* b, int stn, half8* bn) {
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
#pragma unroll
        for (int j = 0; j < C::FN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
          if (i == 0) bn[j] = *reinterpret_cast<const half8*>(addr_b(stn, j));
        }
        a[i] = *reinterpret_cast<const half8*>(addr_a(stn, i));
      }
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
      for (int i = 1; i < C::FM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, C::FN, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    };
    // issue times (x4 so the order inside an iteration is total): a steady-state patch at 4 st, W(k) at
    // 4 (k - NS + 1) + 2 (the prologue's weights before its patch at 4 (s0 - 1) + 3)
    int patch_time = -(1 << 30);
    issue_a(cb, cb & 1);
#pragma unroll
    for (int k = 0; k < NS - 1; ++k)
      if (s0 + k < s1) issue_b(s0 + k);
    if (ce - cb > 1) {
      issue_a(cb + 1, (cb + 1) & 1);
      patch_time = 4 * (s0 - 1) + 3;
    }
    // pieces issued after W(st) at the barrier of step st - 1 (or the prologue for st = s0)
    auto allowed_after = [&](int st) {
      const int w_issued_end = (st - 1) + NS - 1 < s1 ? (st - 1) + NS - 1 : s1;  // W(s0 .. w_issued_end - 1) issued
      int nw = w_issued_end - (st + 1);
      if (nw < 0) nw = 0;
      const int wtime = 4 * (st - NS + 1) + 2;
      return nw * NB + (patch_time > wtime ? NAH : 0);
    };
    auto wait_le = [&](int n) {
      if (n >= 3 * NB + NAH) wait_vmcnt<3 * NB + NAH>();
      else if (n >= 2 * NB + NAH) wait_vmcnt<2 * NB + NAH>();
      else if (n >= NB + NAH) wait_vmcnt<NB + NAH>();
      else if (n >= NAH) wait_vmcnt<NAH>();
      else if (n >= 4 * NB) wait_vmcnt<4 * NB>();
      else if (n >= 3 * NB) wait_vmcnt<3 * NB>();
      else if (n >= 2 * NB) wait_vmcnt<2 * NB>();
      else if (n >= NB) wait_vmcnt<NB>();
      else wait_vmcnt<0>();
    };
    static_assert(NS - 2 <= 4, "wait_le covers up to 4 weight stages after the one waited for");
    // prologue wait: W(s0) and patch(cb) (issued first) landed; after W(s0): W(s0+1 .. s0+NS-2), patch(cb+1)
    {
      int nw = (s0 + NS - 1 < s1 ? s0 + NS - 1 : s1) - (s0 + 1);
      if (nw < 0) nw = 0;
      wait_le(nw * NB + (ce - cb > 1 ? NAH : 0));
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    half8 a[C::FM], b0[C::FN], b1[C::FN];
#pragma unroll
    for (int j = 0; j < C::FN; ++j) b0[j] = *reinterpret_cast<const half8*>(addr_b(s0, j));
#pragma unroll
    for (int i = 0; i < C::FM; ++i) a[i] = *reinterpret_cast<const half8*>(addr_a(s0, i));
    auto step = [&](int st, const half8* bm, half8* br) {
      const bool more = st + 1 < s1;
      if (more) {
        const int c = st / 9, t = st - c * 9;
        // WAR on the patch buffer refilled below: its last reads (step st's A fragments, issued during step st - 1)
        // must have returned on this wave before the barrier.  The weight slot refilled below was read two steps
        // back, by fragments step st - 1's MFMAs already consumed.
        if (t == 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        wait_le(allowed_after(st + 1));
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (t == 8 && c + 2 < ce) {
          issue_a(c + 2, c & 1);
          patch_time = 4 * st;
        }
        if (st + NS - 1 < s1) issue_b(st + NS - 1);
      }
      mfma_step(a, bm, st + 1, br);
    };
    for (int st = s0; st < s1; st += 2) {
      step(st, b0, b1);
      if (st + 1 < s1) step(st + 1, b1, b0);
    }
    __syncthreads();  // all fragment reads done before the epilogue reuses LDS
  } else if constexpr (C::HALO) {
    // ---------------- 3x3 halo patch + weight ring via global->LDS DMA, channel-chunk-major K ----------------
    // Step s = (chunk c = s / 9, tap t = s % 9) over the whole K (never split).  LDS: patch buffers [2][A_PATCH]
    // (pixel q = row-major in the (TH+2) x (TW+2) patch, 128 B per pixel, chunk XOR ((q >> 1) & 7) on the SOURCE
    // side and on the fragment reads: the 16 pixels of a fragment's lane group hit 16 distinct bank slots), then
    // the weight ring [3][BN][128 B] (rows swizzled the same way as kGlds3).
    // Issue order inside a step: the next chunk's patch (first tap of a chunk only), then the weights of step
    // s + 2, so waiting for the weights of step s with vmcnt(#pieces issued in step s - 1) also covers the patch
    // of step s's chunk (issued before them).  One raw barrier per step: afterwards every wave's DMA for step s
    // has landed and every wave has finished reading step s - 1's weight stage and, at a chunk's first tap, the
    // previous chunk's patch buffer, which the issues of this step then refill.
    constexpr int TW = C::TW, TH = BM / TW, PW = TW + 2, RP = C::HALO_PIX;
    constexpr int NAH = C::HALO_NA;
    constexpr int NB = BN * 8 / NT;
    static_assert(NB * NT == BN * 8 && NB >= 1, "whole-wave weight DMA pieces");
    constexpr int APB = C::A_PATCH, BST = BN * 128;
    static_assert(2 * APB + 3 * BST <= C::SMEM, "halo buffers fit");
    char* const abuf0 = smem;
    char* const bbuf0 = smem + 2 * APB;
    const int Cin = p.Cin;
    // k-steps [kt0, kt0 + nk) of the 9 * Cin / 64 (chunk-major, then tap): whole chunks (a split launch cuts K at
    // chunk boundaries, conv_igemm_kernel), so chunk cb's patch is the first one DMA'd
    const int cb = kt0 / 9, ce = (kt0 + nk) / 9;
    const int s0 = kt0, s1 = kt0 + nk;
    int apix[NAH], alch[NAH];
    bool aok[NAH];
    constexpr int RPP = C::HALO_RPP, APL = RPP * 16;  // kHaloP: plane length (pixels) and plane stride (bytes)
#pragma unroll
    for (int i = 0; i < NAH; ++i) {
      if constexpr (C::HALOP) {
        // DMA instruction (wave, i) fills the 64 LDS slots from 64 (wave * NAH + i): slot = plane * RPP + pixel;
        // each lane loads its pixel's 8 channels of that plane
        const int slot = (wave * NAH + i) * 64 + lane;
        const int pl = slot / RPP, q = slot - pl * RPP;
        const int qy = q / PW, qx = q - qy * PW;
        const int iy = halo_oy0 - 1 + qy, ix = halo_ox0 - 1 + qx;
        aok[i] = pl < 8 && q < RP && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        apix[i] = aok[i] ? (halo_img * p.H + iy) * p.W + ix : 0;
        alch[i] = pl << 3;
      } else {
        const int q = (wave * NAH + i) * 8 + (lane >> 3);
        const int qy = q / PW, qx = q - qy * PW;
        const int iy = halo_oy0 - 1 + qy, ix = halo_ox0 - 1 + qx;
        aok[i] = q < RP && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        apix[i] = aok[i] ? (halo_img * p.H + iy) * p.W + ix : 0;
        alch[i] = ((lane & 7) ^ ((q >> 1) & 7)) << 3;
      }
    }
    static_assert(!C::HALOP || NAH * C::NW * 64 >= 8 * RPP, "kHaloP: the DMA instructions cover all 8 planes");
    static_assert(!C::HALOP || (RPP % 16 == 0 && 4 * APL < 65536), "kHaloP: 256-B planes, immediate plane offsets");
    const int sb1 = p.src[0].channels;
    const int sb2 = sb1 + (p.nsrc > 1 ? p.src[1].channels : 0);
    const int sb3 = sb2 + (p.nsrc > 2 ? p.src[2].channels : 0);
    const f16* sp0 = reinterpret_cast<const f16*>(p.src[0].ptr);
    const f16* sp1 = reinterpret_cast<const f16*>(p.src[p.nsrc > 1 ? 1 : 0].ptr);
    const f16* sp2 = reinterpret_cast<const f16*>(p.src[p.nsrc > 2 ? 2 : 0].ptr);
    const f16* sp3 = reinterpret_cast<const f16*>(p.src[p.nsrc > 3 ? 3 : 0].ptr);
    const int ss0 = p.src[0].stride, ss1 = p.src[p.nsrc > 1 ? 1 : 0].stride;
    const int ss2 = p.src[p.nsrc > 2 ? 2 : 0].stride, ss3 = p.src[p.nsrc > 3 ? 3 : 0].stride;
    const f16* wrow[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int row = (wave * NB + j) * 8 + (lane >> 3);
      const int lch = (lane & 7) ^ ((row >> 1) & 7);
      wrow[j] = reinterpret_cast<const f16*>(p.weight) + (size_t)(n0 + row) * p.Kpad + lch * 8;
    }
    const void* zero_src = g_zero16;

    auto issue_a = [&](int c, int buf) {
      const int ci = c << 6;
      const f16* sp;
      int sst;
      if (ci < sb1) { sp = sp0 + ci; sst = ss0; }
      else if (ci < sb2) { sp = sp1 + (ci - sb1); sst = ss1; }
      else if (ci < sb3) { sp = sp2 + (ci - sb2); sst = ss2; }
      else { sp = sp3 + (ci - sb3); sst = ss3; }
      char* dst = abuf0 + buf * APB;
#pragma unroll
      for (int i = 0; i < NAH; ++i) {
        const void* g = aok[i] ? (const void*)(sp + (size_t)apix[i] * sst + alch[i]) : zero_src;
        SA_HALO_GLDS(g, (lds_void_t*)(dst + (wave * NAH + i) * 1024), 16, 0, 0);
      }
    };
    auto issue_b = [&](int st, int buf) {
      const int c = st / 9, t = st - c * 9;
      const int koff = t * Cin + (c << 6);
      char* dst = bbuf0 + buf * BST;
#pragma unroll
      for (int j = 0; j < NB; ++j)
        SA_HALO_GLDS((const void*)(wrow[j] + koff), (lds_void_t*)(dst + (wave * NB + j) * 1024), 16,
                                         0, 0);
    };

    const int frow = lane & 15;
    // A fragment rows of this wave: output pixel (py, px) of fragment i, lane row frow
    int aq0[C::FM];
#pragma unroll
    for (int i = 0; i < C::FM; ++i) {
      const int r = wm * C::TM + i * 16 + frow;
      aq0[i] = (r / TW) * PW + (r % TW);
    }
    // lane-constant parts of the fragment addresses.  B (swizzled rows): the row and chunk of (j, kk) never change,
    // only the ring slot does.  kHaloP A: the tap-0 pixel of fragment i in plane (lane >> 4); a tap, a k-half and
    // the chunk's patch buffer only add wave-uniform byte offsets.
    int boff[C::FN][2], aoff[C::FM];
#pragma unroll
    for (int j = 0; j < C::FN; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int row = wn * C::TN + j * 16 + frow;
        const int lc = (lane >> 4) + 4 * kk;
        boff[j][kk] = row * 128 + ((lc ^ ((row >> 1) & 7)) << 4);
      }
#pragma unroll
    for (int i = 0; i < C::FM; ++i) aoff[i] = (lane >> 4) * APL + aq0[i] * 16;
    // fragment reads of k-half kk of step st (patch buffer of its chunk, tap offset, weight slot st % 3)
    auto frag_addr_a = [&](int st, int i, int kk) {
      const int c = st / 9, t = st - c * 9;
      if constexpr (C::HALOP) {
        const int u = (c & 1) * APB + kk * 4 * APL + ((t / 3) * PW + (t - (t / 3) * 3)) * 16;  // wave-uniform
        return abuf0 + aoff[i] + u;
      } else {
        const int q = aq0[i] + (t / 3) * PW + (t - (t / 3) * 3);
        const int lc = (lane >> 4) + 4 * kk;
        return abuf0 + (c & 1) * APB + q * 128 + ((lc ^ ((q >> 1) & 7)) << 4);
      }
    };
    auto frag_addr_b = [&](int st, int j, int kk) { return bbuf0 + (st % 3) * BST + boff[j][kk]; };
    auto read_half = [&](int st, int kk, half8* af, half8* bf) {
#pragma unroll
      for (int i = 0; i < C::FM; ++i) af[i] = SA_HALO_LD(frag_addr_a(st, i, kk));
#pragma unroll
      for (int j = 0; j < C::FN; ++j) bf[j] = SA_HALO_LD(frag_addr_b(st, j, kk));
    };
    auto mfma_half = [&](const half8* af, const half8* bf) {
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          acc[i][j] = SA_HALO_MFMA(af[i], bf[j], acc[i][j], 0, 0, 0);
    };
    // the MFMAs of one k-half with the fragment reads of another interleaved one read per MFMA (as kGlds3)
    auto mfma_read = [&](const half8* am, const half8* bm, int st, int kk, half8* ar, half8* br) {
#pragma unroll
      for (int tt = 0; tt < C::FM * C::FN; ++tt) {
        const int i = tt / C::FN, j = tt - (tt / C::FN) * C::FN;
        acc[i][j] = SA_HALO_MFMA(am[i], bm[j], acc[i][j], 0, 0, 0);
        if (tt < C::FM) ar[tt] = SA_HALO_LD(frag_addr_a(st, tt, kk));
        else if (tt < C::FM + C::FN) br[tt - C::FM] = SA_HALO_LD(frag_addr_b(st, tt - C::FM, kk));
      }
      static_assert(C::FM + C::FN <= C::FM * C::FN, "one read per MFMA slot");
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
      for (int tt = 0; tt < C::FM + C::FN; ++tt) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, C::FM * C::FN - C::FM - C::FN - 1, 0);
    };
    // Schedule (kGlds3's, with a 3-slot weight ring and two patch buffers).  Iteration st:
    //   [A] MFMAs of half 0 of step st + fragment reads of its half 1
    //   lgkmcnt(0); vmcnt(<= pieces issued in iteration st - 1); raw s_barrier -- step st + 1's weights (and, at
    //       a chunk boundary, its patch) have landed for every wave, and every wave is done reading step st
    //   [B] MFMAs of half 1 of step st + fragment reads of half 0 of step st + 1
    //   refill: the patch of chunk c + 2 into chunk c's buffer when st is chunk c's last step, then the weights
    //       of step st + 3 into slot st % 3 (patch first, so waiting for a step's weights covers its patch)
    // Prologue: patch 0, weights 0, 1, 2, patch 1.
    issue_a(cb, cb & 1);
    issue_b(s0, s0 % 3);
    if (nk > 1) issue_b(s0 + 1, (s0 + 1) % 3);
    if (nk > 2) issue_b(s0 + 2, (s0 + 2) % 3);
    if (ce - cb > 1) issue_a(cb + 1, (cb + 1) & 1);
    // pieces issued after the weights of step 0 / step 1 (the first two waits)
    const int after0 = (nk > 1 ? NB : 0) + (nk > 2 ? NB : 0) + (ce - cb > 1 ? NAH : 0);
    if (after0 >= 2 * NB + NAH) wait_vmcnt<2 * NB + NAH>();
    else if (after0 >= NB + NAH) wait_vmcnt<NB + NAH>();
    else if (after0 >= 2 * NB) wait_vmcnt<2 * NB>();
    else if (after0 >= NB) wait_vmcnt<NB>();
    else wait_vmcnt<0>();
    SA_HALO_BAR();
    asm volatile("" ::: "memory");
    half8 a0[C::FM], b0[C::FN], a1[C::FM], b1[C::FN];
    read_half(s0, 0, a0, b0);
    int prev = (nk > 2 ? NB : 0) + (ce - cb > 1 ? NAH : 0);  // issued after step 1's weights
    for (int st = s0; st < s1; ++st) {
      mfma_read(a0, b0, st, 1, a1, b1);
      if (st + 1 < s1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (prev >= NB + NAH) wait_vmcnt<NB + NAH>();
        else if (prev >= NB) wait_vmcnt<NB>();
        else if (prev >= NAH) wait_vmcnt<NAH>();
        else wait_vmcnt<0>();
        SA_HALO_BAR();
        asm volatile("" ::: "memory");
        mfma_read(a1, b1, st + 1, 0, a0, b0);
        const int c = st / 9, t = st - c * 9;
        int issued = 0;
        if (t == 8 && c + 2 < ce) {
          issue_a(c + 2, c & 1);
          issued += NAH;
        }
        if (st + 3 < s1) {
          issue_b(st + 3, st % 3);
          issued += NB;
        }
        prev = issued;
      } else {
        mfma_half(a1, b1);
      }
    }
    __syncthreads();  // all fragment reads done before the epilogue reuses LDS
  } else if constexpr (is_glds(MODE)) {
    // ---------------- uniform-k im2col via global->LDS DMA, 3-deep LDS ring, BK = 64 -------------
    // Stage image per operand: [rows][64 halfs] (128-B rows), lane-linear per wave instruction
    // (slot q*16 = row*128 + pch*16) with the XOR swizzle on the SOURCE chunk (lch = pch ^
    // ((row>>1)&7)), read back through the same involution (cdna_hip_programming.md §5.4 rule 21).
    // Pipeline: stages kt and kt+1 are in flight when iteration kt waits with vmcnt(NA+NB) (= one
    // stage of DMA left outstanding), crosses a raw s_barrier (so every wave's DMA of stage kt has
    // landed and every wave finished reading stage kt-1), then issues stage kt+2 into the buffer
    // stage kt-1 used and runs the MFMAs of stage kt.
    constexpr int NA = BM * 8 / NT, NB = BN * 8 / NT;  // DMA instructions per thread per stage
    static_assert(NA * NT == BM * 8 && NB * NT == BN * 8 && NA + NB <= 8, "whole-wave DMA pieces");
    constexpr int STG = (BM + BN) * 128;
    const int KH = p.KH, KW = p.KW;
    int pixb[NA];  // input pixel index of the row's (kd, kh, kw) = 0 tap (32-bit: tensors < 2^31 elements)
    unsigned long long vmask[NA];
    int lcho[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int row = (wave * NA + i) * 8 + (lane >> 3);
      lcho[i] = (((lane & 7) ^ ((row >> 1) & 7)) << 3);
      const int m = m0 + row;
      const bool ok = m < M;
      const int mm = ok ? m : 0;
      const int img = mm / HWo;
      const int r = mm - img * HWo;
      const int oh = r / p.Wo, ow = r - oh * p.Wo;
      const int n = img / Do, od = img - n * Do;
      const int ih0 = oh * p.sh - p.ph, iw0 = ow * p.sw - p.pw, id0 = od * sd - p.pd;
      pixb[i] = ((n * Di + id0) * p.H + ih0) * p.W + iw0;
      unsigned long long mk = 0ull;
      int t = 0;
      for (int kd = 0; kd < KD; ++kd)
        for (int kh = 0; kh < KH; ++kh)
          for (int kw = 0; kw < KW; ++kw, ++t) {
            const int dd = id0 + kd, ih = ih0 + kh * p.dh, iw = iw0 + kw * p.dw;
            if (ok && dd >= 0 && dd < Di && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W) mk |= 1ull << t;
          }
      vmask[i] = mk;
    }
    int kc = kt0 * 64;
    int tap = kc / p.Cin, ci0 = kc - tap * p.Cin;
    int kd_ = tap / (KH * KW), kr = tap - kd_ * KH * KW;
    int kh_ = kr / KW, kw_ = kr - kh_ * KW;
    int toff = (kd_ * p.H + kh_ * p.dh) * p.W + kw_ * p.dw;
    const int sb1 = p.src[0].channels;
    const int sb2 = sb1 + (p.nsrc > 1 ? p.src[1].channels : 0);
    const int sb3 = sb2 + (p.nsrc > 2 ? p.src[2].channels : 0);
    // source pointers / strides held in registers: indexing the kernarg array per stage would put an
    // s_load + lgkmcnt(0) (which also waits for the stage's ds_reads) in front of every DMA issue
    const f16* sp0 = reinterpret_cast<const f16*>(p.src[0].ptr);
    const f16* sp1 = reinterpret_cast<const f16*>(p.src[p.nsrc > 1 ? 1 : 0].ptr);
    const f16* sp2 = reinterpret_cast<const f16*>(p.src[p.nsrc > 2 ? 2 : 0].ptr);
    const f16* sp3 = reinterpret_cast<const f16*>(p.src[p.nsrc > 3 ? 3 : 0].ptr);
    const int ss0 = p.src[0].stride, ss1 = p.src[p.nsrc > 1 ? 1 : 0].stride;
    const int ss2 = p.src[p.nsrc > 2 ? 2 : 0].stride, ss3 = p.src[p.nsrc > 3 ? 3 : 0].stride;
    const f16* wrow[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int row = (wave * NB + j) * 8 + (lane >> 3);
      const int lch = (lane & 7) ^ ((row >> 1) & 7);
      wrow[j] = reinterpret_cast<const f16*>(p.weight) + (size_t)(n0 + row) * p.Kpad + kc + lch * 8;
    }
    const void* zero_src = g_zero16;
    auto issue = [&](int buf) {
      char* sa = smem + buf * STG;
      char* sb = sa + BM * 128;
      const f16* sp;
      int sst;
      if (ci0 < sb1) { sp = sp0 + ci0; sst = ss0; }
      else if (ci0 < sb2) { sp = sp1 + (ci0 - sb1); sst = ss1; }
      else if (ci0 < sb3) { sp = sp2 + (ci0 - sb2); sst = ss2; }
      else { sp = sp3 + (ci0 - sb3); sst = ss3; }
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const bool v = (vmask[i] >> tap) & 1ull;
        const f16* ga = sp + ((pixb[i] + toff) * sst + lcho[i]);
        const void* g = v ? (const void*)ga : zero_src;
        __builtin_amdgcn_global_load_lds(g, (lds_void_t*)(sa + (wave * NA + i) * 1024), 16, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        __builtin_amdgcn_global_load_lds((const void*)wrow[j], (lds_void_t*)(sb + (wave * NB + j) * 1024), 16, 0, 0);
        wrow[j] += 64;
      }
      ci0 += 64;
      if (ci0 >= p.Cin) {
        ci0 = 0;
        ++tap;
        ++kw_;
        toff += p.dw;
        if (kw_ == KW) {
          kw_ = 0;
          toff += p.dh * p.W - KW * p.dw;
          ++kh_;
          if (kh_ == KH) {
            kh_ = 0;
            toff += p.H * p.W - KH * p.dh * p.W;
          }
        }
      }
    };
    const int frow = lane & 15;
    // fragment reads of one 32-deep half (kk) of the stage in buffer `buf`
    auto read_half = [&](int buf, int kk, half8* af, half8* bf) {
      const char* sa = smem + buf * STG;
      const char* sb = sa + BM * 128;
      const int lc = (lane >> 4) + 4 * kk;
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        const int row = wm * C::TM + i * 16 + frow;
        af[i] = *reinterpret_cast<const half8*>(sa + row * 128 + ((lc ^ ((row >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const int row = wn * C::TN + j * 16 + frow;
        bf[j] = *reinterpret_cast<const half8*>(sb + row * 128 + ((lc ^ ((row >> 1) & 7)) << 4));
      }
    };
    auto mfma_half = [&](const half8* af, const half8* bf) {
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    };
    // the MFMAs of one half (operands am/bm, already in registers) with the fragment reads of
    // another half interleaved one read per MFMA: the first MFMA waits only for its own (old)
    // operands and the reads land under the MFMA stream
    auto mfma_read = [&](const half8* am, const half8* bm, int buf, int kk, half8* ar, half8* br) {
      const char* sa = smem + buf * STG;
      const char* sb = sa + BM * 128;
      const int lc = (lane >> 4) + 4 * kk;
#pragma unroll
      for (int t = 0; t < C::FM * C::FN; ++t) {
        const int i = t / C::FN, j = t - (t / C::FN) * C::FN;
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(am[i], bm[j], acc[i][j], 0, 0, 0);
        if (t < C::FM) {
          const int row = wm * C::TM + t * 16 + frow;
          ar[t] = *reinterpret_cast<const half8*>(sa + row * 128 + ((lc ^ ((row >> 1) & 7)) << 4));
        } else if (t < C::FM + C::FN) {
          const int row = wn * C::TN + (t - C::FM) * 16 + frow;
          br[t - C::FM] = *reinterpret_cast<const half8*>(sb + row * 128 + ((lc ^ ((row >> 1) & 7)) << 4));
        }
      }
      static_assert(C::FM + C::FN <= C::FM * C::FN, "one read per MFMA slot");
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
      for (int t = 0; t < C::FM + C::FN; ++t) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, C::FM * C::FN - C::FM - C::FN - 1, 0);
    };
    // Two phases per 64-deep stage, one barrier: (A) the kk=0 MFMAs of stage kt with the kk=1
    // fragment reads of stage kt interleaved; (B) retire those reads, wait for stage kt+1's DMA
    // (stage kt+2 stays in flight), barrier, the kk=1 MFMAs of stage kt with the kk=0 reads of
    // stage kt+1 interleaved, then refill stage kt's now-free buffer with stage kt+3.  Each
    // stage's DMA has two k-steps to land; LDS reads always run under MFMAs.
    // Generalised to an NS-deep ring (kGldsDeep): the prologue issues NS stages, iteration kt waits for
    // stage kt + 1 with min(nk - kt - 2, NS - 2) later stages still in flight and refills stage kt's buffer
    // with stage kt + NS.
    constexpr int NS = C::NSTAGE;
    static_assert((NS - 1) * (NA + NB) <= 32, "vmcnt literal range");
    half8 a0[C::FM], b0[C::FN], a1[C::FM], b1[C::FN];
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (nk > s) issue(s);
    wait_stages<NA + NB, NS - 1>(nk < NS ? nk - 1 : NS - 1);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (nk > 0) read_half(0, 0, a0, b0);
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      mfma_read(a0, b0, cur, 1, a1, b1);
      const int nxt = cur == NS - 1 ? 0 : cur + 1;
      if (kt + 1 < nk) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        wait_stages<NA + NB, NS - 2>(nk - kt - 2 < NS - 2 ? nk - kt - 2 : NS - 2);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        mfma_read(a1, b1, nxt, 0, a0, b0);
        if (kt + NS < nk) issue(cur);
      } else {
        mfma_half(a1, b1);
      }
      cur = nxt;
    }
    __syncthreads();  // all fragment reads done before the epilogue reuses LDS
  } else if constexpr (MODE == kWide || C::PING) {
    // ---------------- wide tile: uniform-k DMA gather, BK = 32, 4-deep LDS ring, 32x32x16 MFMA ----------
    // (kPing shares the gather and the stage image, and runs its own ping-pong schedule below)
    // Stage image per operand: [rows][32 halfs] (64-B rows), lane-linear per wave instruction (16 rows x 4
    // chunks per 1 KB DMA piece) with the chunk XOR ((row >> 2) & 3) applied on the SOURCE side and on
    // the fragment reads (same involution; cdna_hip_programming.md §5.4 rule 21): the 16 lanes of each
    // ds_read_b128 group then hit 16 distinct 16-B bank slots.
    // Schedule of stage t (buffer t % 4; stages t+1..t+3 in flight at its start):
    //   [A] MFMAs of k16 half 0 (fragments X) + fragment reads of half 1 (-> Y)
    //   lgkmcnt(0); vmcnt(<= 2 stages); raw s_barrier   -- stage t+1 has landed for every wave and every
    //                                                     wave is done reading buffer t % 4
    //   DMA of stage t+4 into buffer t % 4
    //   [B] MFMAs of half 1 (Y) + fragment reads of stage t+1 half 0 (-> X)
    // so every stage has three stages of MFMA work to land and LDS reads always run under MFMAs.
    constexpr int NA = BM * 4 / NT, NB = BN * 4 / NT;  // 1-KB DMA pieces per thread per stage
    static_assert(NA * NT == BM * 4 && NB * NT == BN * 4 && NA >= 1 && NB >= 1, "whole-wave DMA pieces");
    constexpr int NAB = NA + NB;
    constexpr int STG = (BM + BN) * 64;
    static_assert(C::NSTAGE * STG <= C::SMEM && (C::PING || C::NSTAGE == 4), "ring fits");
    const int KH = p.KH, KW = p.KW;
    int pixb[NA];
    unsigned long long vmask[NA];
    int lcho[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int row = (wave * NA + i) * 16 + (lane >> 2);
      lcho[i] = (((lane & 3) ^ ((row >> 2) & 3)) << 3);
      const int m = m0 + row;
      const bool ok = m < M;
      const int mm = ok ? m : 0;
      const int img = mm / HWo;
      const int r = mm - img * HWo;
      const int oh = r / p.Wo, ow = r - oh * p.Wo;
      const int n = img / Do, od = img - n * Do;
      const int ih0 = oh * p.sh - p.ph, iw0 = ow * p.sw - p.pw, id0 = od * sd - p.pd;
      pixb[i] = ((n * Di + id0) * p.H + ih0) * p.W + iw0;
      unsigned long long mk = 0ull;
      int t = 0;
      for (int kd = 0; kd < KD; ++kd)
        for (int kh = 0; kh < KH; ++kh)
          for (int kw = 0; kw < KW; ++kw, ++t) {
            const int dd = id0 + kd, ih = ih0 + kh * p.dh, iw = iw0 + kw * p.dw;
            if (ok && dd >= 0 && dd < Di && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W) mk |= 1ull << t;
          }
      vmask[i] = mk;
    }
    // K loop in channel-chunk-major order: for each 32-channel chunk, all KD*KH*KW taps.  Consecutive
    // stages then re-read the same input pixels shifted by one tap (L1 / L2 reuse distance of one stage);
    // tap-major order streams a whole tile's A panel between two uses and thrashes the XCD's L2 once 32
    // CUs each hold a different 256-row panel.  (kWide is never split: kt0 = 0.)
    const int taps_all = KD * KH * KW;
    // (kWide is never split; a kPing split-K slice starts at stage kt0 = chunk * taps_all + tap)
    int ci0 = (kt0 / taps_all) * 32, tap = kt0 - (kt0 / taps_all) * taps_all;
    int kh_ = (tap % (KH * KW)) / KW, kw_ = tap % KW;
    int toff = ((tap / (KH * KW)) * p.H + kh_ * p.dh) * p.W + kw_ * p.dw;
    const int sb1 = p.src[0].channels;
    const int sb2 = sb1 + (p.nsrc > 1 ? p.src[1].channels : 0);
    const int sb3 = sb2 + (p.nsrc > 2 ? p.src[2].channels : 0);
    const f16* sp0 = reinterpret_cast<const f16*>(p.src[0].ptr);
    const f16* sp1 = reinterpret_cast<const f16*>(p.src[p.nsrc > 1 ? 1 : 0].ptr);
    const f16* sp2 = reinterpret_cast<const f16*>(p.src[p.nsrc > 2 ? 2 : 0].ptr);
    const f16* sp3 = reinterpret_cast<const f16*>(p.src[p.nsrc > 3 ? 3 : 0].ptr);
    const int ss0 = p.src[0].stride, ss1 = p.src[p.nsrc > 1 ? 1 : 0].stride;
    const int ss2 = p.src[p.nsrc > 2 ? 2 : 0].stride, ss3 = p.src[p.nsrc > 3 ? 3 : 0].stride;
    // weight rows past the packed Cout (a multiple of 128, ConvLayer::upload) re-read the last packed row:
    // those output columns are never stored (nvalid), and a finite row keeps them finite
    const int cout_pad = (p.Cout + 127) & ~127;
    const f16* wrow[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int row = (wave * NB + j) * 16 + (lane >> 2);
      const int lch = (lane & 3) ^ ((row >> 2) & 3);
      const int wr = n0 + row < cout_pad ? n0 + row : cout_pad - 1;
      wrow[j] = reinterpret_cast<const f16*>(p.weight) + (size_t)wr * p.Kpad + lch * 8;
    }
    const void* zero_src = g_zero16;
    auto issue = [&](int buf) {
      char* sa = smem + buf * STG;
      char* sb = sa + BM * 64;
      const f16* sp;
      int sst;
      if (ci0 < sb1) { sp = sp0 + ci0; sst = ss0; }
      else if (ci0 < sb2) { sp = sp1 + (ci0 - sb1); sst = ss1; }
      else if (ci0 < sb3) { sp = sp2 + (ci0 - sb2); sst = ss2; }
      else { sp = sp3 + (ci0 - sb3); sst = ss3; }
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const bool v = (vmask[i] >> tap) & 1ull;
        const f16* ga = sp + ((pixb[i] + toff) * sst + lcho[i]);
        __builtin_amdgcn_global_load_lds(v ? (const void*)ga : zero_src, (lds_void_t*)(sa + (wave * NA + i) * 1024), 16, 0, 0);
      }
      const int koff = tap * p.Cin + ci0;  // packed K order is (tap, channel)
#pragma unroll
      for (int j = 0; j < NB; ++j)
        // (explicit void* source: a conditional or typed source makes the host pass drop the kernel stub)
        __builtin_amdgcn_global_load_lds((const void*)(wrow[j] + koff), (lds_void_t*)(sb + (wave * NB + j) * 1024), 16, 0, 0);
      // next tap; after the last tap the next 32-channel chunk
      ++tap;
      ++kw_;
      toff += p.dw;
      if (kw_ == KW) {
        kw_ = 0;
        toff += p.dh * p.W - KW * p.dw;
        ++kh_;
        if (kh_ == KH) {
          kh_ = 0;
          toff += p.H * p.W - KH * p.dh * p.W;
        }
      }
      if (tap == taps_all) {
        tap = 0;
        toff = 0;
        ci0 += 32;
      }
    };
    if constexpr (C::PING) {
      // ---- ping-pong schedule.  Wave group g = wave >> 2 (waves 0-3 and 4-7: one wave of each group per
      // SIMD) owns the tile rows [128 g, 128 g + 128).  Between consecutive raw barriers ("slots") one group
      // runs the MFMA cluster of a whole stage (8 x FN 16x16x32 MFMAs) while the other reads its fragments of
      // a stage from LDS and issues its share of a later stage's DMA; group 1 starts one barrier late, so
      //   slot 2s:   G0 MFMA(s)               G1 read(s) + DMA(s + NS - 1)
      //   slot 2s+1: G0 read(s+1) + DMA(s+NS) G1 MFMA(s)
      // RAW: every wave retires its DMA of stage s+1 (counted vmcnt, NS-2 later stages left in flight) before
      // the barrier that opens slot 2s+1, the first slot reading s+1.  WAR: the buffer refilled in slot 2s
      // (2s+1) was last read in slot 2s-2 (2s) and those reads were retired (lgkmcnt(0)) before the barrier.
      // Each wave issues the stages strictly in order (issue() walks the k position).
      constexpr int NS = C::NSTAGE;
      static_assert(NS >= 3 && (NS - 2) * NAB <= 32, "ring depth / vmcnt literal range");
      const int g = wave >> 2;
      const int frow = lane & 15, lc = lane >> 4;
      half8 fa[C::FM], fb[C::FN];
      // 16x16x32 operands: lane (frow, lc) holds row frow, k = 8 lc .. 8 lc + 7 (64-B rows, chunk XOR (row>>2)&3)
      auto read_stage = [&](int buf) {
#ifdef SA_EXP_NOLDSREAD
        if (buf < 0)  // never: the reads are skipped, the registers stay live (timing experiments only)
#endif
        {
        const char* sa = smem + buf * STG;
        const char* sb = sa + BM * 64;
#pragma unroll
        for (int i = 0; i < C::FM; ++i) {
          const int row = wm * C::TM + i * 16 + frow;
          fa[i] = *reinterpret_cast<const half8*>(sa + row * 64 + ((lc ^ ((row >> 2) & 3)) << 4));
        }
#pragma unroll
        for (int j = 0; j < C::FN; ++j) {
          const int row = wn * C::TN + j * 16 + frow;
          fb[j] = *reinterpret_cast<const half8*>(sb + row * 64 + ((lc ^ ((row >> 2) & 3)) << 4));
        }
        }
      };
      auto mfma_stage = [&]() {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j) {
#ifdef SA_EXP_NOMFMA
            asm volatile("" ::"v"(fa[i]), "v"(fb[j]));
#else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
#endif
          }
        __builtin_amdgcn_s_setprio(0);
      };
      // raw barrier pinned in the instruction stream (no MFMA / ds_read moves across it)
      auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
#ifndef SA_EXP_NOBAR
        __builtin_amdgcn_s_barrier();
#endif
        __builtin_amdgcn_sched_barrier(0);
      };
      auto lgkm0 = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      };
      // stage s+1 landed (own DMA), later stages up to min(s + NS - 1, nk - 1) may stay in flight
      auto wait_next = [&](int s) {
        const int last = s + NS - 1 < nk - 1 ? s + NS - 1 : nk - 1;
        wait_stages<NAB, NS - 2>(last - (s + 1));
      };
      // prologue: stages 0 .. NS-2 in flight, stage 0 landed
#pragma unroll
      for (int t = 0; t < NS - 1; ++t)
        if (t < nk) issue(t);
      if (nk > 0) wait_stages<NAB, NS - 2>((nk - 1 < NS - 2 ? nk - 1 : NS - 2));
      bar();
      if (g == 0) {
        int rbuf = 0;       // buffer of the next stage to read (s + 1 after the first read)
        int ibuf = NS - 1;  // buffer of the next stage to issue
        if (nk > 0) read_stage(0);
        if (NS - 1 < nk) issue(ibuf);
        ibuf = 0;
        rbuf = 1;
        lgkm0();
        bar();
        for (int s = 0; s < nk; ++s) {
          mfma_stage();
          if (s + 1 < nk) wait_next(s);
          bar();
          if (s + 1 < nk) {
            read_stage(rbuf);
#ifndef SA_EXP_NODMA
            if (s + NS < nk) issue(ibuf);
#endif
            rbuf = rbuf == NS - 1 ? 0 : rbuf + 1;
            ibuf = ibuf == NS - 1 ? 0 : ibuf + 1;
          }
          lgkm0();
          bar();
        }
      } else {
        int rbuf = 0, ibuf = NS - 1;
        bar();
        for (int s = 0; s < nk; ++s) {
          read_stage(rbuf);
#ifndef SA_EXP_NODMA
          if (s + NS - 1 < nk) issue(ibuf);
#endif
          rbuf = rbuf == NS - 1 ? 0 : rbuf + 1;
          ibuf = ibuf == NS - 1 ? 0 : ibuf + 1;
          lgkm0();
          if (s + 1 < nk) wait_next(s);
          bar();
          mfma_stage();
          bar();
        }
      }
      __syncthreads();  // all fragment reads done before the epilogue reuses LDS
    } else {
    // 32x32x16 fragments of k16 half h of the stage in `buf`: lane = (r, hl) holds row r, k = 16h + 8hl..+7
    const int fr = lane & 31, fh = lane >> 5;
    auto frag = [&](const char* base, int row, int h) {
      return *reinterpret_cast<const half8*>(base + row * 64 + (((2 * h + fh) ^ ((row >> 2) & 3)) << 4));
    };
    auto read = [&](int buf, int h, half8* a, half8* b) {
      const char* sa = smem + buf * STG;
      const char* sb = sa + BM * 64;
#pragma unroll
      for (int i = 0; i < WFM; ++i) a[i] = frag(sa, wm * 128 + i * 32 + fr, h);
#pragma unroll
      for (int j = 0; j < WFN; ++j) b[j] = frag(sb, wn * C::TN + j * 32 + fr, h);
    };
    // 8 MFMAs on (a, b) with the 6 fragment reads of (buf, h) interleaved, one per MFMA slot.
    // SA_EXP_* (tools/exp_build.sh, timing experiments only -- results are garbage): NOMFMA drops the
    // MFMAs (operands kept live), NOLDSREAD the fragment reads, NODMA the in-loop DMA, NOBAR the barrier
    auto mfma_read = [&](const half8* a, const half8* b, int buf, int h, half8* ar, half8* br) {
      const char* sa = smem + buf * STG;
      const char* sb = sa + BM * 64;
#pragma unroll
      for (int t = 0; t < WFM * WFN; ++t) {
        const int i = t / WFN, j = t % WFN;
#ifdef SA_EXP_NOMFMA
        asm volatile("" ::"v"(a[i]), "v"(b[j]));
#else
        acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc32[i][j], 0, 0, 0);
#endif
#ifndef SA_EXP_NOLDSREAD
        if (t < WFM) ar[t] = frag(sa, wm * 128 + t * 32 + fr, h);
        else if (t < WFM + WFN) br[t - WFM] = frag(sb, wn * C::TN + (t - WFM) * 32 + fr, h);
#endif
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
      for (int t = 0; t < WFM + WFN; ++t) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, WFM * WFN - WFM - WFN - 1, 0);
    };
    auto mfma_only = [&](const half8* a, const half8* b) {
#pragma unroll
      for (int t = 0; t < WFM * WFN; ++t) {
        const int i = t / WFN, j = t % WFN;
        acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc32[i][j], 0, 0, 0);
      }
    };
    half8 xa[WFM], xb[WFN], ya[WFM], yb[WFN];
    // prologue: stages 0..3 in flight, wait for stage 0
    if (nk > 0) issue(0);
    if (nk > 1) issue(1);
    if (nk > 2) issue(2);
    if (nk > 3) issue(3);
    if (nk > 3) wait_vmcnt<3 * NAB>();
    else if (nk > 2) wait_vmcnt<2 * NAB>();
    else if (nk > 1) wait_vmcnt<NAB>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (nk > 0) read(0, 0, xa, xb);
    // the last stage is peeled so the loop body has one control path for the accumulators (a branch
    // around the MFMAs makes the compiler copy all 128 of them at the merge)
    for (int kt = 0; kt < nk - 1; ++kt) {
      const int cur = kt & 3;
      mfma_read(xa, xb, cur, 1, ya, yb);  // [A]
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // stage kt+1 must have landed; stages issued beyond it may stay in flight
      const int ahead = (nk - 1 < kt + 3 ? nk - 1 : kt + 3) - (kt + 1);
      if (ahead >= 2) wait_vmcnt<2 * NAB>();
      else if (ahead == 1) wait_vmcnt<NAB>();
      else wait_vmcnt<0>();
#ifndef SA_EXP_NOBAR
      __builtin_amdgcn_s_barrier();
#endif
      asm volatile("" ::: "memory");
#ifndef SA_EXP_NODMA
      if (kt + 4 < nk) issue(cur);
#endif
      mfma_read(ya, yb, (kt + 1) & 3, 0, xa, xb);  // [B]
    }
    if (nk > 0) {
      mfma_read(xa, xb, (nk - 1) & 3, 1, ya, yb);
      mfma_only(ya, yb);
    }
    __syncthreads();  // all fragment reads done before the epilogue reuses LDS
    }  // kWide schedule
  } else {
  // ---------------- per-thread A-row precompute ----------------
  const int cth = tid % C::KCH;  // chunk index this thread loads (constant over k)
  int a_ih0[C::A_PT], a_iw0[C::A_PT], a_nb[C::A_PT], a_d0[C::A_PT];
  bool a_ok[C::A_PT];
#pragma unroll
  for (int i = 0; i < C::A_PT; ++i) {
    int q = tid + NT * i;
    int row = q / C::KCH;
    int m = m0 + row;
    bool ok = (q < C::A_CH) && (m < M);
    int mm = ok ? m : 0;
    int img = mm / HWo;
    int r = mm - img * HWo;
    int oh = r / p.Wo, ow = r - oh * p.Wo;
    int n = img / Do, od = img - n * Do;
    a_ih0[i] = oh * p.sh - p.ph;
    a_iw0[i] = ow * p.sw - p.pw;
    a_d0[i] = od * sd - p.pd;
    a_nb[i] = n * Di + a_d0[i];
    a_ok[i] = ok;
  }
  // k-position tracking for this thread's chunk
  int k_tap, k_ci;
  {
    int kc = kt0 * C::BK + cth * 8;
    k_tap = kc / p.Cin;
    k_ci = kc - k_tap * p.Cin;
  }
  // source channel boundaries
  int sb1 = p.src[0].channels;
  int sb2 = sb1 + (p.nsrc > 1 ? p.src[1].channels : 0);
  int sb3 = sb2 + (p.nsrc > 2 ? p.src[2].channels : 0);

  const f16* wptr = reinterpret_cast<const f16*>(p.weight);

  half8 ra[C::A_PT], rb[C::B_PT];
  const half8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};

  auto load_tile = [&](int kt) {
    // A: im2col gather
    int kd = k_tap / khw, t2 = k_tap - kd * khw;
    int kh = t2 / p.KW, kw = t2 - kh * p.KW;
    bool kok = k_tap < taps;
    int s = (k_ci >= sb1) + (k_ci >= sb2) + (k_ci >= sb3);
    int cbase = s == 0 ? 0 : (s == 1 ? sb1 : (s == 2 ? sb2 : sb3));
    const f16* sptr = reinterpret_cast<const f16*>(p.src[s].ptr) + (k_ci - cbase);
    int sstride = p.src[s].stride;
#pragma unroll
    for (int i = 0; i < C::A_PT; ++i) {
      int ih = a_ih0[i] + kh * p.dh;
      int iw = a_iw0[i] + kw * p.dw;
      int dd = a_d0[i] + kd;
      bool ok = a_ok[i] && kok && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W && dd >= 0 && dd < Di;
      if (ok) {
        size_t pix = ((size_t)(a_nb[i] + kd) * p.H + ih) * p.W + iw;
        ra[i] = *reinterpret_cast<const half8*>(sptr + pix * sstride);
      } else {
        ra[i] = zero8;
      }
    }
    // B: packed weights, always in bounds (Cout padded to a multiple of 128)
#pragma unroll
    for (int i = 0; i < C::B_PT; ++i) {
      int q = tid + NT * i;
      if (q < C::B_CH) {
        int row = q / C::KCH;
        rb[i] = *reinterpret_cast<const half8*>(wptr + (size_t)(n0 + row) * p.Kpad +
                                                 (kt0 + kt) * C::BK + (q % C::KCH) * 8);
      }
    }
    // advance k position by BK for the next tile
    k_ci += C::BK;
    while (k_ci >= p.Cin) {
      k_ci -= p.Cin;
      ++k_tap;
    }
  };

  auto store_tile = [&](int buf) {
    char* sa = smem + buf * (C::A_BYTES + C::B_BYTES);
    char* sb = sa + C::A_BYTES;
#pragma unroll
    for (int i = 0; i < C::A_PT; ++i) {
      int q = tid + NT * i;
      if (q < C::A_CH) {
        if constexpr (C::BK == 64) *reinterpret_cast<half8*>(sa + swz64(q >> 3, q & 7)) = ra[i];
        else *reinterpret_cast<half8*>(sa + swz(q >> 2, q & 3)) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < C::B_PT; ++i) {
      int q = tid + NT * i;
      if (q < C::B_CH) {
        if constexpr (C::BK == 64) *reinterpret_cast<half8*>(sb + swz64(q >> 3, q & 7)) = rb[i];
        else *reinterpret_cast<half8*>(sb + swz(q >> 2, q & 3)) = rb[i];
      }
    }
  };


  // fragment read offsets (row = lane&15, chunk = lane>>4, swizzled)
  const int frow = lane & 15;
  const int foff = frow * 64 + (((lane >> 4) ^ (((frow >> 3) & 1) * 3)) << 4);

  if constexpr (MODE == kRegAll) {
    // the loads of every k-step issued up front (registers), then per step: store to LDS buffer kt & 1, barrier,
    // MFMAs.  Buffer kt & 1 was last read by the MFMAs of step kt - 2, which every wave finished before the barrier
    // of step kt - 1.
    static_assert(C::BK == 64, "kRegAll: 64-deep steps");
    constexpr int NS = 8;
    half8 xa[NS][C::A_PT], xb[NS][C::B_PT];
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      if (st < nk) {
        load_tile(st);
#pragma unroll
        for (int i = 0; i < C::A_PT; ++i) xa[st][i] = ra[i];
#pragma unroll
        for (int i = 0; i < C::B_PT; ++i) xb[st][i] = rb[i];
      }
    }
#pragma unroll
    for (int kt = 0; kt < NS; ++kt) {
      if (kt >= nk) break;
#pragma unroll
      for (int i = 0; i < C::A_PT; ++i) ra[i] = xa[kt][i];
#pragma unroll
      for (int i = 0; i < C::B_PT; ++i) rb[i] = xb[kt][i];
      store_tile(kt & 1);
      __syncthreads();
      const char* sa = smem + (kt & 1) * (C::A_BYTES + C::B_BYTES);
      const char* sb = sa + C::A_BYTES;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        half8 af[C::FM], bf[C::FN];
        const int lc = (lane >> 4) + 4 * kk;
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
          af[i] = *reinterpret_cast<const half8*>(sa + swz64(wm * C::TM + i * 16 + frow, lc));
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          bf[j] = *reinterpret_cast<const half8*>(sb + swz64(wn * C::TN + j * 16 + frow, lc));
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();  // the epilogue's C tile aliases the stage buffers
  } else {
  load_tile(0);
  store_tile(0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile(kt + 1);
    const char* sa = smem + cur * (C::A_BYTES + C::B_BYTES);
    const char* sb = sa + C::A_BYTES;
    if constexpr (C::BK == 64) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        half8 af[C::FM], bf[C::FN];
        const int lc = (lane >> 4) + 4 * kk;
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
          af[i] = *reinterpret_cast<const half8*>(sa + swz64(wm * C::TM + i * 16 + frow, lc));
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          bf[j] = *reinterpret_cast<const half8*>(sb + swz64(wn * C::TN + j * 16 + frow, lc));
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
    } else {
      half8 af[C::FM], bf[C::FN];
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
        af[i] = *reinterpret_cast<const half8*>(sa + (wm * C::TM + i * 16) * 64 + foff);
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
        bf[j] = *reinterpret_cast<const half8*>(sb + (wn * C::TN + j * 16) * 64 + foff);
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }
  }  // two-stage pipeline

  }  // register-staged path

  if constexpr (EXT == 1) {
    // workgroup split-K: this K slice's partial tile -> workspace slice z, column-major [LD][Mp] (Mp = M rounded up to
    // 4): one 16-B store per accumulator (rows < Mp, columns < LD)
    const int LD = (p.Cout + 63) & ~63, Mp = (M + 3) & ~3;
    float* dst = p.ws + (size_t)z * LD * Mp;
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const int m = m0 + wm * C::TM + i * 16 + (lane >> 4) * 4;
        const int n = n0 + wn * C::TN + j * 16 + (lane & 15);
        // non-temporal: the partials bypass this XCD's L2 (the reduce launch reads them from other XCDs, and the
        // end-of-kernel write-back of ~10 MB of dirty L2 lines is not on the chain)
        if (m < M && n < LD) __builtin_nontemporal_store(acc[i][j], reinterpret_cast<floatx4*>(dst + (size_t)n * Mp + m));
      }
    return;
  }

  // ---------------- split-K: partial slabs + last-arriver reduction ----------------
  // Protocol of cdna_hip_programming.md "Projection GEMM at M = 256" item 2 (agent-scope release
  // by every slice, acquire by the last arriver), valid for any placement of slices over XCDs.
  if (!C::WIDE && S > 1) {  // (kWide is always launched unsplit)
    const int tile = ctr;
    constexpr int SLAB = BM * BN;
    auto slab_of = [&](int c) -> size_t {
      if (skG == 0) return (size_t)slab_base + c;
      const int b = slab_base + c;
      const int first_tile = (int)((long)b * skI / skG / (p.Kpad / C::BK));
      return 2 * (size_t)b + (first_tile == ctr ? 0 : 1);
    };
    float* slab = p.ws + slab_of(z) * SLAB;
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) slab[((i * C::FN + j) * 4 + r) * NT + tid] = acc[i][j][r];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == S - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      *flag = last;
    }
    __syncthreads();
    const int last = *flag;
    __syncthreads();
    if (!last) return;
    // fixed summation order over all slices (own slab included) => bitwise deterministic
    // regardless of which slice arrives last
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int sl = 0; sl < S; ++sl) {
      const float* os = p.ws + slab_of(sl) * SLAB;
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += os[((i * C::FN + j) * 4 + r) * NT + tid];
    }
  }

  // ---------------- epilogue: stage C through LDS, one TM-row band of waves at a time ----------
  float* ct = reinterpret_cast<float*>(smem);

  constexpr int CPR = BN / 8;  // 8-channel chunks per row
  constexpr int RPI = NT / CPR;  // rows per pass
  const int cc = tid % CPR;
  const int co = n0 + cc * 8;
  // kHaloW carries 128 accumulators per lane into the epilogue: it is never launched with statistics (launch_halo),
  // so the 32 statistics registers are compiled out there
  const bool do_stats = !C::HALOW && p.stats != nullptr;
  // Instance-norm statistics: per-thread partial sums for the (at most) two images a BM-row tile
  // can straddle, reduced across the block in LDS, then ONE double atomic per (block, image,
  // channel).  Per-thread atomics to the same N*C addresses serialise at the memory side
  // (MI355X_MICROARCH.md, global float atomics: one-row contention is ~14x slower) and cost
  // 20 ms per full-resolution RAFT fnet conv.  Tiles spanning > 2 images (HWo < BM, tiny test
  // shapes only) fall back to per-thread atomics.
  const int img_lo = m0 / HWo;
  const int m_last = (m0 + BM < M ? m0 + BM : M) - 1;
  const bool block_reduce = (m_last / HWo) - img_lo <= 1;
  float ssum[8], ssq[8], ssum1[8], ssq1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ssum[j] = ssq[j] = ssum1[j] = ssq1[j] = 0.f;
  int cur_img = -1;
  const int nvalid = p.Cout - co;  // channels valid in this chunk (may be <=0 or <8)

  // this block's copy of the statistics (stats_slots copies of [N][Cout][2])
  sa_stat_t* const stats_blk =
      p.stats_slots > 1 ? p.stats + (size_t)((blockIdx.y * gridDim.x + blockIdx.x) % p.stats_slots) * p.N * p.Cout * 2
                        : p.stats;
  auto flush_stats = [&](int img) {
    if (img < 0) return;
    for (int j = 0; j < 8 && j < nvalid; ++j) {
      unsigned long long* sp = reinterpret_cast<unsigned long long*>(stats_blk) + ((size_t)img * p.Cout + co + j) * 2;
      atomicAdd(sp, (unsigned long long)__double2ll_rn((double)ssum[j] * SA_STAT_SCALE));
      atomicAdd(sp + 1, (unsigned long long)__double2ll_rn((double)ssq[j] * SA_STAT_SCALE));
      ssum[j] = ssq[j] = 0.f;
    }
  };

  float bias8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bias8[j] = (p.bias && j < nvalid) ? p.bias[co + j] : 0.f;

  if constexpr (!C::BANDED) {
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int row = wm * C::TM + i * 16 + (lane >> 4) * 4 + r;
          int col = wn * C::TN + j * 16 + (lane & 15);
          ct[row * C::CST + cswz(row, col)] = acc[i][j][r];
        }
    __syncthreads();
  }

  // rows [r0, r1) of the tile, their C values staged in LDS at row - cbase
  auto epi_rows = [&](const int r0, const int r1, const int cbase) {
    for (int row = r0 + tid / CPR; row < r1; row += RPI) {
      int m;
      if constexpr (C::HALO) {  // patch pixel -> image pixel; patches may overhang the right / bottom edge
        const int oy = halo_oy0 + row / C::TW, ox = halo_ox0 + row % C::TW;
        if (oy >= p.Ho || ox >= p.Wo) continue;
        m = m0 + oy * p.Wo + ox;
      } else {
        m = m0 + row;
        if (m >= M) break;
      }
      float v[8];
      const int crow = row - cbase;
      const float* cp = ct + crow * C::CST + cswz(crow, cc * 8);
      floatx4 c0 = *reinterpret_cast<const floatx4*>(cp);
      floatx4 c1 = *reinterpret_cast<const floatx4*>(cp + 4);
      v[0] = c0[0]; v[1] = c0[1]; v[2] = c0[2]; v[3] = c0[3];
      v[4] = c1[0]; v[5] = c1[1]; v[6] = c1[2]; v[7] = c1[3];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] * p.scale + bias8[j];
      const bool full = nvalid >= 8;

      if (p.epi == SA_EPI_STORE || p.epi == SA_EPI_STORE_F32) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = act_apply(v[j], p.act, p.alpha);
        if (p.res) {
          const f16* rp = reinterpret_cast<const f16*>(p.res) + (size_t)m * p.res_stride + co;
          float r8[8];
          if (full) load8(rp, r8);
          else for (int j = 0; j < 8; ++j) r8[j] = j < nvalid ? (float)rp[j] : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = act_apply(v[j] + r8[j], p.act2, p.alpha);
        }
        if (p.gate) {  // channel attention, broadcast over depth
          const int img = m / HWo;
          const size_t gpix = (size_t)(img / Do) * HWo + (m - img * HWo);
          const f16* gp = reinterpret_cast<const f16*>(p.gate) + gpix * p.gate_stride + co;
          float g8[8];
          if (full) load8(gp, g8);
          else for (int j = 0; j < 8; ++j) g8[j] = j < nvalid ? (float)gp[j] : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= g8[j];
        }
        if (p.up) {
          // transposed conv: channel co + j belongs to parity class (co + j) / cout_real
          const int img = m / HWo;
          const int r = m - img * HWo;
          const int oh = r / p.Wo, ow = r - oh * p.Wo;
          const int n = img / Do, od = img - n * Do;
          const int Ho2 = 2 * p.Ho, Wo2 = 2 * p.Wo, Do2 = p.up == 3 ? 2 * Do : 1;
          for (int j = 0; j < 8 && j < nvalid; ++j) {
            const int cj = co + j;
            const int pi = cj / p.cout_real, c = cj - pi * p.cout_real;
            const int pb = pi & 1, pa = (pi >> 1) & 1, pc = p.up == 3 ? (pi >> 2) : 0;
            const int dz = p.up == 3 ? 2 * od + pc : 0;
            const size_t opix = (((size_t)n * Do2 + dz) * Ho2 + 2 * oh + pa) * Wo2 + 2 * ow + pb;
            if (p.epi == SA_EPI_STORE) reinterpret_cast<f16*>(p.out)[opix * p.out_stride + c] = (f16)v[j];
            else reinterpret_cast<float*>(p.out)[opix * p.out_stride + c] = v[j];
          }
        } else if (p.epi == SA_EPI_STORE) {
          f16* op = reinterpret_cast<f16*>(p.out) + (size_t)m * p.out_stride + co;
          if (full) store8(op, v);
          else for (int j = 0; j < nvalid; ++j) op[j] = (f16)v[j];
        } else {
          float* op = reinterpret_cast<float*>(p.out) + (size_t)m * p.out_stride + co;
          for (int j = 0; j < 8 && j < nvalid; ++j) op[j] = v[j];
        }
        if (do_stats) {
          const int img = m / HWo;
          if (block_reduce) {
            if (img == img_lo) {
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                ssum[j] += v[j];
                ssq[j] += v[j] * v[j];
              }
            } else {
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                ssum1[j] += v[j];
                ssq1[j] += v[j] * v[j];
              }
            }
          } else {
            if (img != cur_img) {
              flush_stats(cur_img);
              cur_img = img;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              ssum[j] += v[j];
              ssq[j] += v[j] * v[j];
            }
          }
        }
      } else if (p.epi == SA_EPI_GRU_ZR || p.epi == SA_EPI_GRU_ZRQ) {
        const int Hd = p.epi == SA_EPI_GRU_ZR ? p.Cout >> 1 : p.Cout / 3;
        float c8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (p.ctx) load8(reinterpret_cast<const f16*>(p.ctx) + (size_t)m * p.ctx_stride + co, c8);
        if (co < Hd) {
          float z[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) z[j] = sigmoidf_(v[j] + c8[j]);
          store8(reinterpret_cast<f16*>(p.aux) + (size_t)m * p.aux_stride + co, z);
        } else if (co < 2 * Hd) {
          const int ch = co - Hd;
          float h8[8], rh[8];
          load8(reinterpret_cast<const f16*>(p.hbuf) + (size_t)m * p.h_stride + ch, h8);
#pragma unroll
          for (int j = 0; j < 8; ++j) rh[j] = sigmoidf_(v[j] + c8[j]) * h8[j];
          store8(reinterpret_cast<f16*>(p.rh) + (size_t)m * p.rh_stride + ch, rh);
        } else {
          // SA_EPI_GRU_ZRQ: the x-input half of convq's pre-activation (+ its bias and context) for the q conv
          float q8[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) q8[j] = v[j] + c8[j];
          store8(reinterpret_cast<f16*>(p.out) + (size_t)m * p.out_stride + (co - 2 * Hd), q8);
        }
      } else if (p.epi == SA_EPI_GRU_Q) {
        float c8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, z8[8], h8[8];
        if (p.ctx) load8(reinterpret_cast<const f16*>(p.ctx) + (size_t)m * p.ctx_stride + co, c8);
        if (p.res) {  // the x half of the pre-activation, computed by the SA_EPI_GRU_ZRQ conv
          float x8[8];
          load8(reinterpret_cast<const f16*>(p.res) + (size_t)m * p.res_stride + co, x8);
#pragma unroll
          for (int j = 0; j < 8; ++j) c8[j] += x8[j];
        }
        load8(reinterpret_cast<const f16*>(p.aux) + (size_t)m * p.aux_stride + co, z8);
        f16* hp = reinterpret_cast<f16*>(p.hbuf) + (size_t)m * p.h_stride + co;
        load8(hp, h8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float q = tanhf_(v[j] + c8[j]);
          h8[j] = (1.f - z8[j]) * h8[j] + z8[j] * q;
        }
        store8(hp, h8);
      } else if (p.epi == SA_EPI_TAPPROJ) {
        // the next conv's tap projections of y = fp16(act(v)) (what a stored y would hold): per tap, this lane's 8
        // channels by fp16 dot products, then the sum over the CPR lanes of the row (one 128-channel n-tile)
        typedef _Float16 half2v __attribute__((ext_vector_type(2)));
        half8 h;
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = (f16)act_apply(v[j], p.act, p.alpha);
        const f16* wt = reinterpret_cast<const f16*>(p.tapw) + co;
        float mine = 0.f, mine2 = 0.f;  // lane cc keeps the totals of taps cc and cc + CPR
#pragma unroll
        for (int t = 0; t < 18; ++t) {
          if (t >= p.taps) break;
          const half8 w8 = *reinterpret_cast<const half8*>(wt + (size_t)t * p.Cout);
          float sacc = 0.f;
#pragma unroll
          for (int j = 0; j < 8; j += 2)
            sacc = __builtin_amdgcn_fdot2(half2v{h[j], h[j + 1]}, half2v{w8[j], w8[j + 1]}, sacc, false);
#pragma unroll
          for (int o = 1; o < CPR; o <<= 1) sacc += __shfl_xor(sacc, o);
          if (cc == t) mine = sacc;
          if (cc + CPR == t) mine2 = sacc;
        }
        float* pp = reinterpret_cast<float*>(p.out) + (size_t)m * p.out_stride + (n0 / BN) * p.taps;
        if (cc < p.taps) pp[cc] = mine;
        if (cc + CPR < p.taps) pp[cc + CPR] = mine2;
      } else if (p.epi == SA_EPI_FLOW_ACC) {
        if (co == 0) {  // flow state += delta (RAFT: x only, stride 1; CREStereo: x and y)
          float* fp = reinterpret_cast<float*>(p.out) + (size_t)m * p.out_stride;
          const int nc = p.Cout < p.out_stride ? p.Cout : p.out_stride;
          for (int j = 0; j < nc && j < 8; ++j) fp[j] += v[j];
        }
      }
    }
  };
  // SA_EPI_TAPPROJ on the banded (LDS-staged) tiles: the next conv's tap projections on the matrix cores.  Phase 1
  // turns the band's fp32 C rows into y = fp16(act(scale c + bias)) IN PLACE (the first 256 B of each 512-B row, 16-B
  // slot cc ^ (row & 15); a row's 16 chunk threads sit in one wave, whose LDS reads issue before its writes); phase 2
  // is the GEMM P[row][tap] = y[row][0:128] . tapw[tap][n0:n0+128] as v_mfma_f32_16x16x32_f16 (4 k-steps per 16-row
  // fragment, taps padded to 16 columns).  Replaces round 4's fdot2 + 4-level shuffle reduction per tap and row
  // (profiles/round4_notes.md: dearer than the store it saved).
  auto tapproj_band = [&](const int b0) {
   if constexpr (C::BANDED && BN == 128) {
    static_assert(C::CST == 128 && C::CROWS % 16 == 0, "tap projection: 128-channel n-tiles, 16-row fragments");
    char* const cb8 = reinterpret_cast<char*>(ct);
    for (int crow = tid / CPR; crow < C::CROWS; crow += RPI) {
      const float* cp = ct + crow * C::CST + cswz(crow, cc * 8);
      const floatx4 c0 = *reinterpret_cast<const floatx4*>(cp);
      const floatx4 c1 = *reinterpret_cast<const floatx4*>(cp + 4);
      asm volatile("" ::: "memory");  // every lane's reads of this row issue before any lane's write into it
      half8 h;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        h[j] = (f16)act_apply(c0[j] * p.scale + bias8[j], p.act, p.alpha);
        h[j + 4] = (f16)act_apply(c1[j] * p.scale + bias8[j + 4], p.act, p.alpha);
      }
      *reinterpret_cast<half8*>(cb8 + crow * (C::CST * 4) + ((cc ^ (crow & 15)) << 4)) = h;
    }
    __syncthreads();
    const int r16 = lane & 15, g = lane >> 4;
    const f16* wt = reinterpret_cast<const f16*>(p.tapw);
    // taps <= 18: one or two 16-column tiles (RAFT 9 x 1, CREStereo 9 x 2)
    for (int t0 = 0; t0 < p.taps; t0 += 16) {
      const int tap = t0 + r16;
      half8 bw[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        half8 z;
#pragma unroll
        for (int j = 0; j < 8; ++j) z[j] = (f16)0.f;
        bw[ks] = tap < p.taps ? *reinterpret_cast<const half8*>(wt + (size_t)tap * p.Cout + n0 + ks * 32 + g * 8) : z;
      }
      for (int f = wave; f < C::CROWS / 16; f += C::NW) {
        const int crow = f * 16 + r16;
        floatx4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const half8 a =
              *reinterpret_cast<const half8*>(cb8 + crow * (C::CST * 4) + (((ks * 4 + g) ^ (crow & 15)) << 4));
          d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bw[ks], d, 0, 0, 0);
        }
        if (tap < p.taps) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = b0 + f * 16 + 4 * g + r;
            int m;
            if constexpr (C::HALO) {
              const int oy = halo_oy0 + row / C::TW, ox = halo_ox0 + row % C::TW;
              if (oy >= p.Ho || ox >= p.Wo) continue;
              m = m0 + oy * p.Wo + ox;
            } else {
              m = m0 + row;
              if (m >= M) continue;
            }
            reinterpret_cast<float*>(p.out)[(size_t)m * p.out_stride + (n0 / BN) * p.taps + tap] = d[r];
          }
        }
      }
    }
   }
  };
  if constexpr (C::BANDED) {
    // row bands: the waves owning a band's rows stage their accumulators, everyone stores
#pragma unroll
    for (int band = 0; band < BM / C::CROWS; ++band) {
      const int b0 = band * C::CROWS;
      if (wm * C::TM >= b0 && wm * C::TM < b0 + C::CROWS) {
        if constexpr (C::WIDE) {
#pragma unroll
          for (int i = 0; i < WFM; ++i)
#pragma unroll
            for (int j = 0; j < WFN; ++j)
#pragma unroll
              for (int r = 0; r < 16; ++r) {
                const int row = wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) - b0;
                const int col = wn * C::TN + j * 32 + (lane & 31);
                ct[row * C::CST + cswz(row, col)] = acc32[i][j][r];
              }
        } else {
#pragma unroll
          for (int i = 0; i < C::FM; ++i)
#pragma unroll
            for (int j = 0; j < C::FN; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int row = wm * C::TM + i * 16 + (lane >> 4) * 4 + r - b0;
                const int col = wn * C::TN + j * 16 + (lane & 15);
                ct[row * C::CST + cswz(row, col)] = acc[i][j][r];
              }
        }
      }
      __syncthreads();
      if (BN == 128 && p.epi == SA_EPI_TAPPROJ) tapproj_band(b0);
      else if (nvalid > 0) epi_rows(b0, b0 + C::CROWS, b0);
      __syncthreads();  // band consumed before the next one overwrites the staging LDS
    }
  } else {
    if (nvalid > 0) epi_rows(0, BM, 0);
  }
  if (do_stats) {
    if (!block_reduce) {
      flush_stats(cur_img);
      return;
    }
    // wave reduction over the lanes sharing a channel chunk (lane bits >= log2(CPR)), then the
    // 4 waves' partials meet in LDS red[q][wave][BN] (q = sum0, sq0, sum1, sq1; reuses C tile)
#pragma unroll
    for (int off = CPR; off < 64; off <<= 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ssum[j] += __shfl_xor(ssum[j], off);
        ssq[j] += __shfl_xor(ssq[j], off);
        ssum1[j] += __shfl_xor(ssum1[j], off);
        ssq1[j] += __shfl_xor(ssq1[j], off);
      }
    }
    constexpr int RG = C::NW;
    static_assert(4 * RG * BN * 4 <= C::SMEM, "stats reduction must fit in the staging LDS");
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();  // everyone finished reading the C tile
    if (lane < CPR) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = cc * 8 + j;
        red[(0 * RG + wave) * BN + col] = ssum[j];
        red[(1 * RG + wave) * BN + col] = ssq[j];
        red[(2 * RG + wave) * BN + col] = ssum1[j];
        red[(3 * RG + wave) * BN + col] = ssq1[j];
      }
    }
    __syncthreads();
    const bool two = (m_last / HWo) != img_lo;
    for (int t = tid; t < 4 * BN; t += NT) {
      const int q = t / BN, col = t - q * BN;
      const int c = n0 + col;
      if (c >= p.Cout || (q >= 2 && !two)) continue;
      float acc = 0.f;
      for (int r = 0; r < RG; ++r) acc += red[(q * RG + r) * BN + col];
      const int img = img_lo + (q >> 1);
      atomicAdd(reinterpret_cast<unsigned long long*>(stats_blk) + ((size_t)img * p.Cout + c) * 2 + (q & 1),
                (unsigned long long)__double2ll_rn((double)acc * SA_STAT_SCALE));
    }
  }
}

// Grid tiling (+ split-K over gridDim.z), or stream-K for the DMA-ring family (p.splitk == -1, grid (G, 1, 1)):
// the T x nk_all k-steps of all tiles are cut into G equal contiguous ranges, block b walks its range as
// (tile, k-range) segments (a segment ends at a tile or range boundary), and tiles whose k-steps span several
// blocks are finished by the last contributor (conv_tile's split-K path, 2G partial slabs).
// Every block does the same amount of MFMA work whatever T is, so grids of 150 or 600 tiles no longer leave
// CUs idle in the last wave (Osama et al., "Stream-K", PPoPP'23).
template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(64 * WM * WN) void conv_igemm_streamk_kernel(const SaConvArgs p) {
  static_assert(MODE == kGlds3, "stream-K is built for the DMA-ring family");
  using C = ConvCfg<BM, BN, WM, WN, MODE>;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  const int nk_all = p.Kpad / C::BK;
  const int M = p.N * (p.Do > 0 ? p.Do : 1) * p.Ho * p.Wo;
  const int gy = (p.Cout + BN - 1) / BN;
  const long T = (long)((M + BM - 1) / BM) * gy;
  const long I = T * nk_all;
  const int G = gridDim.x;
  // XCD-major logical block id: consecutive ranges (which share tiles and A panels) on one XCD's L2
  const int b = (G & 7) ? (int)blockIdx.x : (int)((blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3));
  long it = (long)b * I / G;
  const long end = (long)(b + 1) * I / G;
  // the argument block is re-read through an opaque pointer per segment: otherwise every kernarg load of the
  // tile body is hoisted out of this loop and the live SGPRs spill
  // (p is the kernel's only explicit argument: it sits at offset 0 of the kernarg segment.  Taking &p instead
  // would give the address of a private copy.)
  typedef const __attribute__((address_space(4))) SaConvArgs* kernarg_ptr;  // constant (kernarg) address space
  kernarg_ptr pp = (kernarg_ptr)__builtin_amdgcn_kernarg_segment_ptr();
  while (it < end) {
    const int t = (int)(it / nk_all);
    const int kb = (int)(it - (long)t * nk_all);
    const int ke = (int)((long)nk_all < kb + (end - it) ? nk_all : kb + (end - it));
    // contributors of tile t: the blocks whose ranges meet [t * nk_all, (t + 1) * nk_all)
    const int bf = (int)((((long)t * nk_all + 1) * G + I - 1) / I) - 1;
    const int bl = (int)((((long)(t + 1) * nk_all) * G + I - 1) / I) - 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" : "+s"(pp));
    conv_tile<BM, BN, WM, WN, MODE>(*(const SaConvArgs*)pp, smem, t / gy, t % gy, kb, ke - kb, bl - bf + 1, b - bf, bf, t, G, I);
    it += ke - kb;
    __syncthreads();  // the next segment's DMA reuses the LDS this segment's epilogue read
  }
}

template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(64 * WM * WN) void conv_igemm_kernel(const SaConvArgs p) {
  using C = ConvCfg<BM, BN, WM, WN, MODE>;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  const int nk_all = p.Kpad / C::BK;
  // grid tiling; kGlds3 / kWide walk the (m, n) tiles in an XCD-aware order: consecutive dispatch ids
  // round-robin over the 8 XCDs, so give each XCD a contiguous run of m-major tiles (neighbour tiles share
  // input rows through the 3x3 halo, the n tiles of one m share the whole A panel)
  int bx = blockIdx.x, by = blockIdx.y;
  if constexpr (C::PING) {
    // 1-D grid: the first `full` dispatch ids are whole tiles (XCD-aware order), the remaining ones split each
    // of the last T - full tiles into S = p.splitk K slices, so a tile count that is not a multiple of the CU
    // count does not leave most CUs idle in the last round (launch_ping)
    const int M = p.N * (p.Do > 0 ? p.Do : 1) * p.Ho * p.Wo;
    const int gy = (p.Cout + BN - 1) / BN;
    const int T = ((M + BM - 1) / BM) * gy;
    const int S = p.splitk > 1 ? p.splitk : 1;
    const int nb = gridDim.x;
    const int full = S > 1 ? (S * T - nb) / (S - 1) : T;
    const int bid = blockIdx.x;
    if (bid < full) {
      const int q = full >> 3, r = full & 7, xcd = bid & 7;
      const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
      bx = lin / gy;
      by = lin - bx * gy;
      conv_tile<BM, BN, WM, WN, MODE>(p, smem, bx, by, 0, nk_all, 1, 0, 0, 0, 0, 0);
    } else {
      const int b2 = bid - full, t = b2 / S, z = b2 - t * S;
      bx = (full + t) / gy;
      by = full + t - bx * gy;
      const int kt0 = (int)((long)z * nk_all / S);
      const int nk = (int)((long)(z + 1) * nk_all / S) - kt0;
      conv_tile<BM, BN, WM, WN, MODE>(p, smem, bx, by, kt0, nk, S, z, t * S, t, 0, 0);
    }
    return;
  }
  if constexpr (is_halo(MODE)) {
    if (p.splitk > 1) {
      // tail split (launch_halo): a 1-D grid whose first `full` dispatch ids are whole tiles (XCD-aware order) and
      // whose remaining ones cut each of the last T - full tiles into S K-ranges of whole 64-channel chunks, so a
      // tile count just above a multiple of the CU count does not leave most CUs idle in the last round
      constexpr int TH = BM / C::TW;
      const int gy = (p.Cout + BN - 1) / BN;
      const int T = p.N * ((p.Ho + TH - 1) / TH) * ((p.Wo + C::TW - 1) / C::TW) * gy;
      const int S = p.splitk, nchunk = p.Cin / C::HALO_CH;
      const int nb = gridDim.x;
      const int full = (S * T - nb) / (S - 1);
      const int bid = blockIdx.x;
      if (bid < full) {
        const int q = full >> 3, r = full & 7, xcd = bid & 7;
        const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
        conv_tile<BM, BN, WM, WN, MODE>(p, smem, lin / gy, lin % gy, 0, nk_all, 1, 0, 0, 0, 0, 0);
      } else {
        const int b2 = bid - full, t = b2 / S, z = b2 - t * S;
        const int c0 = z * nchunk / S, c1 = (z + 1) * nchunk / S;
        conv_tile<BM, BN, WM, WN, MODE>(p, smem, (full + t) / gy, (full + t) % gy, 9 * c0, 9 * (c1 - c0), S, z, t * S,
                                        t, 0, 0);
      }
      return;
    }
  }
  if constexpr (is_glds(MODE) || MODE == kWide || is_halo(MODE)) {
    const int nwg = gridDim.x * gridDim.y;
    const int bid = blockIdx.y * gridDim.x + blockIdx.x;
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
    const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    bx = lin / gridDim.y;
    by = lin - bx * gridDim.y;
  }
  // split-K slice of the K loop handled by this block
  const int S = gridDim.z, z = blockIdx.z;
  const int kt0 = (int)((long)z * nk_all / S);
  const int nk = (int)((long)(z + 1) * nk_all / S) - kt0;
  const int tile = by * gridDim.x + bx;
  conv_tile<BM, BN, WM, WN, MODE>(p, smem, bx, by, kt0, nk, S, z, tile * S, tile, 0, 0);
}

template <int BM, int BN, int WM, int WN, int MODE>
void launch_kernel(dim3 grid, const SaConvArgs* a, hipStream_t stream) {
  hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, MODE>), grid, dim3(64 * WM * WN), 0, stream, *a);
}

thread_local long g_split_floats = 0, g_split_tiles = 0;
inline void note_split(int S, long tiles, long tile_floats) {
  g_split_floats = S > 1 ? (long)S * tiles * tile_floats : 0;
  g_split_tiles = S > 1 ? tiles : 0;
}

// CUs of the current device (stream-K grids are sized to one or two waves of blocks over them)
int device_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int BM, int BN, int WM, int WN>
int launch_cfg(const SaConvArgs* a, hipStream_t stream) {
  // register-staged family (the DMA-ring tiles live in launch_glds3 / launch_halo / launch_wide / launch_ping).
  // BK = 64 doubles the staging LDS: only for tiles whose C tile needs that LDS anyway (BN >= 64)
  const bool k64 = BN >= 64 && a->Kpad % 64 == 0;
  // uniform-k fast gather: every source a multiple of 64 channels, K unpadded, <= 64 taps
  const int taps = (a->KD > 0 ? a->KD : 1) * a->KH * a->KW;
  bool fast = k64 && taps <= 64 && (long)taps * a->Cin == a->Kpad;
  for (int i = 0; i < a->nsrc; ++i) fast = fast && a->src[i].channels % 64 == 0;
  const int M = a->N * (a->Do > 0 ? a->Do : 1) * a->Ho * a->Wo;
  const int gx = (M + BM - 1) / BM, gy = (a->Cout + BN - 1) / BN;
  const long tiles = (long)gx * gy;
  const int nk = a->Kpad / (k64 ? 64 : 32);
  if (a->splitk < 0) return -4;  // stream-K exists for the DMA-ring (kGlds3) family only
  int S = a->splitk;
  if (S == 0) {
    // auto: split the K loop when the tile grid cannot fill 256 CUs (small-M levels of the
    // RAFT GRU pyramid at batch 1); keep >= 4 k-steps of 32 per slice
    S = 1;
    if (a->ws && a->counters && !a->stats && tiles < 320) {
      S = (int)((640 + tiles - 1) / tiles);
      if (S > 8) S = 8;
      if (S > nk / (k64 ? 2 : 4)) S = nk / (k64 ? 2 : 4);
      while (S > 1 && ((long)S * tiles * BM * BN > a->ws_floats || tiles > a->n_counters)) --S;
      if (S < 1) S = 1;
    }
  }
  if (S > 1 && (a->stats || !a->ws || !a->counters || (long)S * tiles * BM * BN > a->ws_floats ||
                tiles > a->n_counters || S > nk))
    return -4;
  dim3 grid(gx, gy, S);
  note_split(S, tiles, BM * BN);
  if (fast) launch_kernel<BM, BN, WM, WN, kFastK64>(grid, a, stream);
  else if (k64) launch_kernel<BM, BN, WM, WN, kRegK64>(grid, a, stream);
  else launch_kernel<BM, BN, WM, WN, kRegK32>(grid, a, stream);
  return (int)hipGetLastError();
}

// kRegAll launcher (tactic 39): any gather, the whole K (<= NSTAGE 64-deep steps) loaded up front, never split.
// Returns 1 when the shape does not qualify.
template <int BM, int BN, int WM, int WN>
int launch_regall(const SaConvArgs* a, hipStream_t stream) {
  if (a->Kpad % 64 != 0 || a->Kpad / 64 > 8 || a->splitk < 0 || a->splitk > 1) return 1;
  const long M = (long)a->N * (a->Do > 0 ? a->Do : 1) * a->Ho * a->Wo;
  const long gx = (M + BM - 1) / BM, gy = (a->Cout + BN - 1) / BN;
  if (gx >= (1L << 31) || gy > 65535) return 1;
  note_split(1, 0, 0);
  launch_kernel<BM, BN, WM, WN, kRegAll>(dim3((unsigned)gx, (unsigned)gy, 1), a, stream);
  return (int)hipGetLastError();
}

// kGlds3 launcher (8 waves, 1 block per CU): only for the uniform-k fast gather (every source a
// multiple of 64 channels, K unpadded, <= 64 taps).  Returns 1 when the shape does not qualify.
bool glds3_eligible(const SaConvArgs* a);

template <int BM, int BN, int WM, int WN, int MODE = kGlds3>
int launch_glds3(const SaConvArgs* a, hipStream_t stream, bool forced) {
  if (!glds3_eligible(a)) return 1;
  const int M = a->N * (a->Do > 0 ? a->Do : 1) * a->Ho * a->Wo;
  const int gx = (M + BM - 1) / BM, gy = (a->Cout + BN - 1) / BN;
  const long tiles = (long)gx * gy;
  const int nk = a->Kpad / 64;
  if constexpr (MODE != kGlds3) {
    if (a->splitk == -1) return forced ? -4 : 1;  // stream-K: 3-deep ring only
  } else if (a->splitk == -1) {
    // stream-K: G resident blocks (LDS / waves per CU), 2G partial slabs, T tile counters
    using C = ConvCfg<BM, BN, WM, WN, kGlds3>;
    int per_cu = 163840 / C::SMEM;
    if (per_cu > 8 / C::NW) per_cu = 8 / C::NW;  // <= 2 waves per SIMD
    if (per_cu < 1) per_cu = 1;
    long G = (long)device_cus() * per_cu;
    if (G > tiles * nk) G = tiles * nk;
    const long slabs = 2 * G;
    if (a->stats || !a->ws || !a->counters || slabs * BM * BN > a->ws_floats || tiles > a->n_counters ||
        tiles * nk * (long)G >= (1L << 62))
      return forced ? -4 : 1;
    g_split_floats = slabs * BM * BN;
    g_split_tiles = tiles;
    hipLaunchKernelGGL((conv_igemm_streamk_kernel<BM, BN, WM, WN, kGlds3>), dim3((unsigned)G), dim3(C::NT), 0, stream,
                       *a);
    return (int)hipGetLastError();
  }
  int S = a->splitk;
  if (S == 0) {
    // auto: one block per CU, so aim for >= ~2 blocks per CU over the 256 CUs
    S = 1;
    if (a->ws && a->counters && !a->stats && tiles < 384) {
      S = (int)((512 + tiles - 1) / tiles);
      if (S > 8) S = 8;
      if (S > nk / 3) S = nk / 3;
      while (S > 1 && ((long)S * tiles * BM * BN > a->ws_floats || tiles > a->n_counters)) --S;
      if (S < 1) S = 1;
    }
  }
  if (S > 1 && (a->stats || !a->ws || !a->counters || (long)S * tiles * BM * BN > a->ws_floats ||
                tiles > a->n_counters || S > nk))
    return forced ? -4 : 1;
  note_split(S, tiles, BM * BN);
  launch_kernel<BM, BN, WM, WN, MODE>(dim3(gx, gy, S), a, stream);
  return (int)hipGetLastError();
}

// Workgroup split-K (tactics 37 / 38): the small-M, deep-K convs of the coarse GRU levels at batch 1 (M = 1200 /
// 4800 pixels, K = 2304 / 3456) give 38-228 tiles of a 256-CU chip, each walking 36-54 k-steps at the DMA gather
// rate of ONE CU.  Here S workgroups share a tile's K range and store fp32 partials (conv_tile EXT = 1), and a second
// launch sums them per 32 x 64 tile and runs the conv's epilogue (EXT = 2; GRU gates, statistics, residual, ...).
template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(64 * WM * WN) void conv_splitx_kernel(const SaConvArgs p) {
  using C = ConvCfg<BM, BN, WM, WN, MODE>;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  const int nk_all = p.Kpad / C::BK;
  const int S = gridDim.z, z = blockIdx.z;
  const int kt0 = (int)((long)z * nk_all / S);
  const int nk = (int)((long)(z + 1) * nk_all / S) - kt0;
  conv_tile<BM, BN, WM, WN, MODE, 1>(p, smem, blockIdx.x, blockIdx.y, kt0, nk, S, z, 0, 0, 0, 0);
}

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void conv_splitx_reduce_kernel(const SaConvArgs p) {
  using C = ConvCfg<BM, BN, WM, WN, kFastK64>;
  static_assert(4 * C::NW * BN * 4 <= C::C_BYTES, "the epilogue's statistics reduction fits the C tile");
  __shared__ __attribute__((aligned(16))) char smem[C::C_BYTES];
  conv_tile<BM, BN, WM, WN, kFastK64, 2>(p, smem, blockIdx.x, blockIdx.y, 0, 0, 1, 0, 0, 0, 0, 0);
}

// Returns 1 when the shape does not qualify (not the uniform-k gather, a grid that needs no split, workspace short).
template <int BM, int BN, int WM, int WN, int MODE>
int launch_splitx(const SaConvArgs* a, hipStream_t stream) {
  if (!glds3_eligible(a) || a->splitk < 0 || a->epi == SA_EPI_TAPPROJ) return 1;
  const long M = (long)a->N * (a->Do > 0 ? a->Do : 1) * a->Ho * a->Wo;
  const int LD = (a->Cout + 63) & ~63;
  const long gx = (M + BM - 1) / BM, gy = (a->Cout + BN - 1) / BN;
  const long tiles = gx * gy;
  const int nk = a->Kpad / 64;
  const int cus = device_cus();
  // at most one workgroup per CU (one round), >= 3 k-steps per slice, <= 8 slices (the reduction unrolls 8)
  int S = (int)(cus / tiles);
  if (S > 8) S = 8;
  if (S > nk / 3) S = nk / 3;
  const long Mp = (M + 3) & ~3L;
  if (S < 2 || M >= (1L << 31) || (long)S * Mp * LD >= (1L << 31)) return 1;
  if (!a->ws || (long)S * Mp * LD > a->ws_floats || ((uintptr_t)a->ws & 15)) return 1;
  using CP = ConvCfg<BM, BN, WM, WN, MODE>;
  hipLaunchKernelGGL((conv_splitx_kernel<BM, BN, WM, WN, MODE>), dim3((unsigned)gx, (unsigned)gy, S), dim3(CP::NT), 0,
                     stream, *a);
  SaConvArgs b = *a;
  b.splitk = S;
  using CR = ConvCfg<32, 64, 2, 2, kFastK64>;
  hipLaunchKernelGGL((conv_splitx_reduce_kernel<32, 64, 2, 2>), dim3((unsigned)((M + 31) / 32), (unsigned)(LD / 64)),
                     dim3(CR::NT), 0, stream, b);
  g_split_floats = (long)S * Mp * LD;
  g_split_tiles = 0;
  return (int)hipGetLastError();
}

// kHalo launcher (8 waves, 1 block per CU, never split): 3x3 / stride 1 / pad 1 / dilation 1 2-D convs whose
// sources are multiples of 64 channels, K unpadded.  Returns 1 when the shape does not qualify.
template <int MODE>
int launch_halo(const SaConvArgs* a, hipStream_t stream) {
  constexpr int BM = (MODE == kHaloW || MODE == kHaloQ) ? 512 : (MODE == kHaloW12 || MODE == kHaloQ12) ? 384 : 256;
  constexpr int BN = 128;
  bool ok = a->KD <= 0 && a->KH == 3 && a->KW == 3 && a->sh == 1 && a->sw == 1 && a->ph == 1 && a->pw == 1 &&
            a->dh == 1 && a->dw == 1 && a->up == 0 && a->Cin % 64 == 0 && a->Kpad == 9 * a->Cin &&
            a->Ho == a->H && a->Wo == a->W && a->splitk >= 0 && a->splitk <= 1;
  for (int i = 0; i < a->nsrc; ++i) ok = ok && a->src[i].channels % 64 == 0;
  if (is_halow(MODE) && a->stats) ok = false;  // epilogue compiled without instance-norm statistics
  if (!ok) return 1;
  using C = ConvCfg<BM, BN, 4, 2, MODE>;
  const int th = BM / C::TW;
  const long tiles = (long)a->N * ((a->Ho + th - 1) / th) * ((a->Wo + C::TW - 1) / C::TW);
  const int gy = (a->Cout + BN - 1) / BN;
  if (tiles * gy >= (1L << 31) || (long)a->N * a->H * a->W >= (1L << 31)) return 1;
  // splitk 0 (auto): the tiles of the last, partial round are split into S K-ranges of whole 64-channel chunks over
  // the idle CUs (conv_igemm_kernel's tail split); splitk 1: whole tiles only
  const long T = tiles * gy;
  const int cus = device_cus();
  const long rem = T % cus;
  const int nchunk = a->Cin / C::HALO_CH;
  int S = 1;
  if (a->splitk == 0 && a->ws && a->counters && !a->stats && rem > 0 && 2 * rem <= cus) {
    S = (int)(cus / rem);
    if (S > 4) S = 4;
    if (S > nchunk) S = nchunk;
    while (S > 1 && ((long)S * rem * BM * BN > a->ws_floats || rem > a->n_counters)) --S;
  }
  if (S > 1) {
    SaConvArgs b = *a;
    b.splitk = S;
    note_split(S, rem, BM * BN);
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 4, 2, MODE>), dim3((unsigned)(T - rem + S * rem)), dim3(C::NT), 0,
                       stream, b);
    return (int)hipGetLastError();
  }
  SaConvArgs b = *a;
  b.splitk = 1;
  note_split(1, 0, 0);
  launch_kernel<BM, BN, 4, 2, MODE>(dim3((unsigned)tiles, gy, 1), &b, stream);
  return (int)hipGetLastError();
}

// kWide launcher (8 waves, 1 block per CU, never split): uniform-k gather.
// Returns 1 when the shape does not qualify.
template <int BM, int BN, int WM, int WN>
int launch_wide(const SaConvArgs* a, hipStream_t stream) {
  if (!glds3_eligible(a) || a->splitk > 1) return 1;
  const int M = a->N * (a->Do > 0 ? a->Do : 1) * a->Ho * a->Wo;
  const int gx = (M + BM - 1) / BM, gy = (a->Cout + BN - 1) / BN;
  note_split(1, 0, 0);
  hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, kWide>), dim3(gx, gy, 1), dim3(64 * WM * WN), 0,
                     stream, *a);
  return (int)hipGetLastError();
}

// kPing launcher (8 waves, 1 block per CU, never split): uniform-k gather.  Returns 1 when the shape does not
// qualify.
int device_cus();

template <int BM, int BN>
int launch_ping(const SaConvArgs* a, hipStream_t stream) {
  if (!glds3_eligible(a) || a->splitk > 1 || a->splitk < 0) return 1;
  const int M = a->N * (a->Do > 0 ? a->Do : 1) * a->Ho * a->Wo;
  const int gx = (M + BM - 1) / BM, gy = (a->Cout + BN - 1) / BN;
  const long T = (long)gx * gy;
  // splitk 0 (auto): split the tiles of the last, partial round over the CUs (all tiles when T < CUs);
  // splitk 1: whole tiles only
  using C = ConvCfg<BM, BN, 2, 4, kPing>;
  const int nk = a->Kpad / C::BK;
  const int cus = device_cus();
  const long rem = T % cus;
  int S = 1;
  if (a->splitk == 0 && a->ws && a->counters && !a->stats && rem > 0 && 2 * rem <= cus) {
    S = (int)(cus / rem);
    if (S > 4) S = 4;
    while (S > 1 && ((long)S * rem * BM * BN > a->ws_floats || rem > a->n_counters || nk / S < 2 * C::NSTAGE)) --S;
  }
  SaConvArgs b = *a;
  b.splitk = S;
  const long nb = S > 1 ? T - rem + S * rem : T;
  note_split(S, S > 1 ? rem : 0, BM * BN);
  hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 2, 4, kPing>), dim3((unsigned)nb), dim3(512), 0, stream, b);
  return (int)hipGetLastError();
}

// the uniform-k DMA kernels need every source a multiple of 64 channels, K unpadded, <= 64 taps
bool glds3_eligible(const SaConvArgs* a) {
  const int taps = (a->KD > 0 ? a->KD : 1) * a->KH * a->KW;
  bool ok = a->Kpad % 64 == 0 && taps <= 64 && (long)taps * a->Cin == a->Kpad;
  for (int i = 0; i < a->nsrc; ++i) ok = ok && a->src[i].channels % 64 == 0;
  return ok;
}

int pick_cfg(const SaConvArgs* a) {
  if (a->tile_cfg >= 0) return a->tile_cfg;
  if (a->epi == SA_EPI_TAPPROJ) return 4;  // 128-wide n-tiles
  const int M = a->N * (a->Do > 0 ? a->Do : 1) * a->Ho * a->Wo;
  if (a->Cout > 64 && glds3_eligible(a) && (a->splitk <= 1 || a->ws)) {
    // measured on MI355X (tools/conv_bench.py): 256x128 / 8 waves wins once its grid covers the
    // chip >= 2x (RAFT batch-8 GRU, flow head, motion encoder); 128x64 / 4 waves (2 blocks per CU)
    // wins for deep K (GRU convs at any batch) and for grids the register path would split
    const long tiles256 = (long)((M + 255) / 256) * ((a->Cout + 127) / 128);
    const long tiles128 = (long)((M + 127) / 128) * ((a->Cout + 63) / 64);
    if (tiles256 >= 512) return 4;
    if (a->Kpad >= 2304 || (tiles128 < 320 && a->ws && a->counters && !a->stats)) return 5;
  }
  if (a->Cout <= 16) return 2;
  if (a->Cout <= 64) return 1;
  // prefer the 128x128 tile only when it still fills the chip
  const long tiles128 = (long)((M + 127) / 128) * ((a->Cout + 127) / 128);
  return tiles128 >= 512 ? 0 : 1;
}

}  // namespace

extern "C" void sa_conv2d_last_split(long* ws_floats, long* tiles) {
  *ws_floats = g_split_floats;
  *tiles = g_split_tiles;
}

// LDS bytes per workgroup of a tile config (the BK = 64 form of the register-staged tiles); -1 for the
// special-purpose kernels (stem / direct / point) whose footprint the tuner does not compare
extern "C" int sa_conv2d_tile_lds(int cfg) {
  switch (cfg) {
    case 0: return ConvCfg<128, 128, 2, 2, kFastK64>::SMEM;
    case 1: return ConvCfg<128, 64, 2, 2, kFastK64>::SMEM;
    case 2: return ConvCfg<256, 16, 4, 1, kFastK64>::SMEM;
    case 3: return ConvCfg<64, 64, 2, 2, kFastK64>::SMEM;
    case 4: return ConvCfg<256, 128, 4, 2, kGlds3>::SMEM;
    case 5: return ConvCfg<128, 64, 2, 2, kGlds3>::SMEM;
    case 7: return ConvCfg<128, 128, 2, 4, kGlds3>::SMEM;
    case 8: return ConvCfg<256, 64, 4, 2, kGlds3>::SMEM;
    case 10: return ConvCfg<256, 256, 2, 4, kWide>::SMEM;
    case 11: return ConvCfg<512, 128, 4, 2, kWide>::SMEM;
    case 14: return ConvCfg<128, 64, 2, 2, kGldsDeep>::SMEM;
    case 15: return ConvCfg<128, 128, 2, 4, kGldsDeep>::SMEM;
    case 16: return ConvCfg<64, 64, 2, 2, kGldsDeep>::SMEM;
    case 17: return ConvCfg<256, 64, 4, 2, kGldsDeep>::SMEM;
    case 18: return ConvCfg<256, 256, 2, 4, kPing>::SMEM;
    case 19: return ConvCfg<256, 128, 2, 4, kPing>::SMEM;
    case 26: return ConvCfg<256, 128, 4, 2, kHalo>::SMEM;
    case 27: return ConvCfg<256, 128, 4, 2, kHalo16>::SMEM;
    case 28: return ConvCfg<256, 128, 4, 2, kHaloP>::SMEM;
    case 29: return ConvCfg<256, 128, 4, 2, kHaloP16>::SMEM;
    case 30: return ConvCfg<512, 128, 4, 2, kHaloW>::SMEM;
    case 31: return ConvCfg<384, 128, 4, 2, kHaloW12>::SMEM;
    case 32: return ConvCfg<512, 128, 4, 2, kHaloQ>::SMEM;
    case 33: return ConvCfg<384, 128, 4, 2, kHaloQ12>::SMEM;
    case 37: return ConvCfg<128, 128, 2, 4, kGldsDeep>::SMEM;
    case 39: return ConvCfg<64, 64, 2, 2, kRegAll>::SMEM;
    case 38: return ConvCfg<64, 64, 2, 2, kGldsDeep>::SMEM;
    default: return -1;
  }
}

// ---------------------------------------------------------------------------------------------------------------
// One ConvGRU level in ONE launch (the coarse levels' launch / join bind at batch 1).  Phase A
// runs the z/r(/q-x) conv with its gate epilogue (SA_EPI_GRU_ZR or _ZRQ: z, r*h, and with ZRQ the x half of q's
// pre-activation), a grid-wide barrier, then phase B the q conv with its state-update epilogue (SA_EPI_GRU_Q, h
// updated in place; q's 3x3 taps read r*h of neighbouring tiles, hence the barrier).  Each phase's (tile, K-slice)
// items are dealt round-robin to the G workgroups and run by conv_tile exactly as conv_igemm_kernel's split-K
// grid runs them (last-arriving slice sums the slabs in fixed order and runs the epilogue).
//
// Grid barrier: a generation counter in `bar` ([0] arrivals, [1] generation, [2] timeout flag).  Every workgroup
// reads the generation BEFORE it arrives, so the last arriver's bump is always seen as a change; agent-scope
// release fence before arriving and acquire fence after leaving (the split-K protocol of conv_tile, valid across
// XCDs).  The arrivals counter returns to 0, so graph replays need no reset.  G <= 128 workgroups of <= 80 KB LDS:
// they are co-resident on 256 CUs even beside another queue's kernels (those never wait on this one, so their CUs
// free up); the spin still gives up after ~2^24 polls and raises bar[2] instead of hanging the GPU.
namespace {
__device__ __forceinline__ void gru_grid_sync(unsigned* bar, unsigned nwg) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned gen = __hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == nwg - 1) {
      __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_store(bar + 1, gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 24)) {
          __hip_atomic_store(bar + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

template <int BM, int BN, int WM, int WN, int MODE>
__device__ __forceinline__ void gru_level_phase(const SaConvArgs& p, char* smem, int S) {
  using C = ConvCfg<BM, BN, WM, WN, MODE>;
  const int M = p.N * p.Ho * p.Wo;
  const int gy = (p.Cout + BN - 1) / BN;
  const int T = ((M + BM - 1) / BM) * gy;
  const int nk_all = p.Kpad / C::BK;
  for (int it = blockIdx.x; it < T * S; it += gridDim.x) {
    const int tile = it / S, z = it - tile * S;
    const int kt0 = (int)((long)z * nk_all / S);
    const int nk = (int)((long)(z + 1) * nk_all / S) - kt0;
    conv_tile<BM, BN, WM, WN, MODE>(p, smem, tile / gy, tile % gy, kt0, nk, S, z, tile * S, tile, 0, 0);
    __syncthreads();  // the next item's prologue reuses the LDS this item's epilogue read
  }
}

template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(64 * WM * WN) void gru_level_kernel(const SaConvArgs za, const SaConvArgs qa,
                                                                  unsigned* bar, int Sa, int Sb) {
  using C = ConvCfg<BM, BN, WM, WN, MODE>;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  gru_level_phase<BM, BN, WM, WN, MODE>(za, smem, Sa);
  gru_grid_sync(bar, gridDim.x);
  gru_level_phase<BM, BN, WM, WN, MODE>(qa, smem, Sb);
}

// split of one phase: about `grid` items, K slices of at least 16 k-steps, slabs / counters within the workspace
int gru_level_split(const SaConvArgs* a, int grid, int BM, int BN, int BK) {
  const int M = a->N * a->Ho * a->Wo;
  const long T = (long)((M + BM - 1) / BM) * ((a->Cout + BN - 1) / BN);
  const int nk = a->Kpad / BK;
  int S = (int)((grid + T - 1) / T);
  if (S > 8) S = 8;
  while (S > 1 && (nk / S < 16 || (long)S * T * BM * BN > a->ws_floats || T > a->n_counters)) --S;
  return S < 1 ? 1 : S;
}
}  // namespace

template <int MODE>
int launch_gru_level(const SaConvArgs* za, const SaConvArgs* qa, unsigned* bar, int grid, hipStream_t stream) {
  constexpr int BM = 64, BN = 64;
  using C = ConvCfg<BM, BN, 2, 2, MODE>;
  for (const SaConvArgs* a : {za, qa}) {
    if (a->Kpad % 32 != 0 || a->nsrc < 1 || a->nsrc > 4 || !glds3_eligible(a) || a->stats || a->up || a->gate ||
        a->KD > 0 || !a->ws || !a->counters)
      return -2;
  }
  if (!(za->epi == SA_EPI_GRU_ZR || za->epi == SA_EPI_GRU_ZRQ) || qa->epi != SA_EPI_GRU_Q) return -2;
  const int Sa = gru_level_split(za, grid, BM, BN, C::BK), Sb = gru_level_split(qa, grid, BM, BN, C::BK);
  // workspace high-water mark of the two phases (sa_conv2d_last_split: the engine right-sizes its workspaces)
  auto tiles = [&](const SaConvArgs* a) { return (long)((a->N * a->Ho * a->Wo + BM - 1) / BM) * ((a->Cout + BN - 1) / BN); };
  const long fa = Sa > 1 ? Sa * tiles(za) : 0, fb = Sb > 1 ? Sb * tiles(qa) : 0;
  g_split_floats = (fa > fb ? fa : fb) * BM * BN;
  g_split_tiles = (Sa > 1 || Sb > 1) ? (tiles(za) > tiles(qa) ? tiles(za) : tiles(qa)) : 0;
  hipLaunchKernelGGL((gru_level_kernel<BM, BN, 2, 2, MODE>), dim3((unsigned)grid), dim3(C::NT), 0, stream, *za, *qa,
                     bar, Sa, Sb);
  return (int)hipGetLastError();
}

// tiles: 64x64 over 4 waves, register-staged (kFastK64, 32 KB of LDS: co-resides with the other queue's kernels) by
// default, or the 8-deep DMA ring (kGldsDeep, 128 KB) with SA_GRU_LEVEL_CFG=6
extern "C" int sa_gru_level(const SaConvArgs* za, const SaConvArgs* qa, unsigned* bar, int grid, hipStream_t stream) {
  if (!za || !qa || !bar || grid < 1 || grid > 128) return -2;
  static const int cfg = [] {
    const char* e = std::getenv("SA_GRU_LEVEL_CFG");
    return e ? std::atoi(e) : 3;
  }();
  return cfg == 6 ? launch_gru_level<kGldsDeep>(za, qa, bar, grid, stream)
                  : launch_gru_level<kFastK64>(za, qa, bar, grid, stream);
}

extern "C" int sa_conv2d(const SaConvArgs* a, hipStream_t stream) {
  if (a->Kpad % 32 != 0 || a->Cin % 8 != 0 || a->nsrc < 1 || a->nsrc > 4) return -2;
  // the folded input norm exists in the direct 64-channel kernel only
  if (a->in_stats && a->tile_cfg >= 0 && a->tile_cfg != 23) return -5;
  const int cfg = a->in_stats ? 23 : pick_cfg(a);
  if (a->epi == SA_EPI_TAPPROJ) {
    // partial sums per 128-channel n-tile: the tile configs with BN = 128 only
    const bool bn128 = cfg == 0 || cfg == 4 || cfg == 7 || cfg == 11 || cfg == 15 || cfg == 19 || (cfg >= 26 && cfg <= 33);
    if (!bn128) return -5;
    // exactly two 128-channel n-tile partials per pixel at stride 2 * taps: sa_tapproj_stencil sums q[0] + q[taps]
    // (Cout 128 read unwritten partials, Cout 384 dropped the third)
    if (!a->tapw || a->taps < 1 || a->taps > 18 || a->stats || a->up || a->gate || a->Cout != 256 ||
        a->out_stride != 2 * a->taps)
      return -2;
  }
  switch (cfg) {
    case 0: return launch_cfg<128, 128, 2, 2>(a, stream);
    case 1: return launch_cfg<128, 64, 2, 2>(a, stream);
    case 2: return launch_cfg<256, 16, 4, 1>(a, stream);
    case 3: return launch_cfg<64, 64, 2, 2>(a, stream);
    case 23: {
      // direct conv (conv_direct.hip): one 64-channel source, 64 outputs, 3x3 / stride 1 / pad 1, store epilogue
      // with optional IN statistics or residual
      const bool ok = a->nsrc == 1 && a->src[0].channels == 64 && a->Cin == 64 && a->Cout == 64 && a->KH == 3 &&
                      a->KW == 3 && a->sh == 1 && a->sw == 1 && a->ph == 1 && a->pw == 1 && a->dh == 1 &&
                      a->dw == 1 && a->KD <= 0 && a->up == 0 && !a->gate && a->epi == SA_EPI_STORE &&
                      a->scale == 1.f && a->Kpad >= 576 && a->out_stride % 8 == 0 && a->src[0].stride % 8 == 0 &&
                      a->Ho == a->H && a->Wo == a->W;
      if (!ok) return -5;
      note_split(1, 0, 0);
      return sa_conv3x3_c64_direct2(a->src[0].ptr, a->src[0].stride, a->weight, a->Kpad, a->bias, a->out,
                                    a->out_stride, a->N, a->H, a->W, a->act, a->alpha, a->stats, a->stats_slots,
                                    a->res, a->res_stride, a->act2, a->in_stats, a->in_slots, a->in_eps, 0, stream);
    }
    case 24: {
      // direct 3x3 -> 96 (conv_direct96.hip): one 96-channel source at stride 1 or a 64-channel one at stride 2,
      // pad 1, store epilogue with optional IN statistics or residual
      const bool shape = (a->Cin == 96 && a->sh == 1 && a->Ho == a->H && a->Wo == a->W) ||
                         (a->Cin == 64 && a->sh == 2 && a->Ho == (a->H - 1) / 2 + 1 && a->Wo == (a->W - 1) / 2 + 1);
      const bool ok = shape && a->nsrc == 1 && a->src[0].channels == a->Cin && a->Cout == 96 && a->KH == 3 &&
                      a->KW == 3 && a->sw == a->sh && a->ph == 1 && a->pw == 1 && a->dh == 1 && a->dw == 1 &&
                      a->KD <= 0 && a->up == 0 && !a->gate && a->epi == SA_EPI_STORE && a->scale == 1.f &&
                      a->Kpad >= 9 * a->Cin && a->out_stride % 4 == 0 && a->src[0].stride % 8 == 0;
      if (!ok) return -5;
      note_split(1, 0, 0);
      return sa_conv3x3_c96_direct(a->src[0].ptr, a->src[0].stride, a->Cin, a->sh, a->weight, a->Kpad, a->bias, a->out,
                                   a->out_stride, a->N, a->H, a->W, a->act, a->alpha, a->stats, a->stats_slots,
                                   a->res, a->res_stride, a->act2, stream);
    }
    case 34: {
      // direct 3x3x3 conv for small channel counts (conv3d_small.hip): one 8 / 16 / 32-channel source, <= 32 outputs,
      // stride 1, pad 1, store epilogue with optional gate
      const int sd = a->sd > 0 ? a->sd : 1;
      const bool ok = a->KD == 3 && a->KH == 3 && a->KW == 3 && sd == a->sh && a->sh == a->sw &&
                      (sd == 1 || (sd == 2 && a->Cin <= 16 && a->up == 0)) && a->pd == 1 &&
                      a->ph == 1 && a->pw == 1 && a->dh == 1 && a->dw == 1 && a->nsrc == 1 &&
                      a->src[0].channels == a->Cin && (a->Cin == 8 || a->Cin == 16 || a->Cin == 32) &&
                      a->Cout <= 32 && (a->up == 0 || (a->up == 3 && !a->gate)) && !a->res && !a->stats &&
                      (a->epi == SA_EPI_STORE || a->epi == SA_EPI_STORE_F32) && a->Do == (a->Di - 1) / sd + 1 &&
                      a->Ho == (a->H - 1) / sd + 1 && a->Wo == (a->W - 1) / sd + 1;
      if (!ok) return -5;
      note_split(1, 0, 0);
      return sa_conv3d_small(a->src[0].ptr, a->src[0].stride, a->Cin, a->weight, a->Kpad, a->bias, a->out,
                             a->out_stride, a->N, a->Di, a->H, a->W, a->Cout, a->act, a->alpha, a->scale, a->gate,
                             a->gate_stride, a->epi == SA_EPI_STORE_F32, a->up == 3 ? a->cout_real : 0, sd, stream);
    }
    case 36: {
      // direct 3x3 / stride 1 conv for small channel counts (conv2d_small.hip): one or two sources, Cin 8-64, Cout <= 64,
      // dilation 1 / 2 / 4, fp16 store epilogue with optional residual or fp32 store
      const bool ok = (a->nsrc == 1 || a->nsrc == 2) && a->Cout <= 64 && a->KH == 3 && a->KW == 3 && a->KD <= 0 &&
                      a->sh == a->sw && (a->sh == 1 || (a->sh == 2 && a->dh == 1 && a->up == 0 && a->Cin <= 32)) &&
                      a->dh == a->dw && (a->dh == 1 || a->dh == 2 || a->dh == 4) &&
                      a->ph == a->dh && a->pw == a->dw && (a->up == 0 || (a->up == 2 && !a->res)) && !a->gate &&
                      !a->stats && (a->epi == SA_EPI_STORE || (a->epi == SA_EPI_STORE_F32 && !a->res)) &&
                      a->Ho == (a->H - 1) / a->sh + 1 && a->Wo == (a->W - 1) / a->sw + 1 &&
                      a->src[0].channels + (a->nsrc == 2 ? a->src[1].channels : 0) == a->Cin &&
                      (a->Cin == 8 || a->Cin == 16 || a->Cin == 32 || a->Cin == 48 || a->Cin == 64 || a->Cin == 96);
      if (!ok) return -5;
      note_split(1, 0, 0);
      return sa_conv2d_small(a->src[0].ptr, a->src[0].stride, a->src[0].channels, a->nsrc == 2 ? a->src[1].ptr : nullptr,
                             a->nsrc == 2 ? a->src[1].stride : 0, a->Cin, a->weight, a->Kpad, a->bias, a->out,
                             a->out_stride, a->N, a->H, a->W, a->Cout, a->act, a->alpha, a->scale, a->res,
                             a->res_stride, a->act2, a->dh, a->epi == SA_EPI_STORE_F32,
                             a->up == 2 ? a->cout_real : 0, a->sh, stream);
    }
    case 35: {
      // pointwise 1x1 stride-1 conv for narrow GEMMs (conv_pw.hip): one or two sources of <= 256 channels, <= 256
      // outputs, store epilogue with optional residual, or the transposed k = 2 / s = 2 parity scatter
      const bool ok = (a->nsrc == 1 || a->nsrc == 2) &&
                      a->src[0].channels + (a->nsrc == 2 ? a->src[1].channels : 0) == a->Cin && a->Cin <= 256 &&
                      a->Cout <= 256 && a->KH == 1 && a->KW == 1 && a->KD <= 0 && a->sh == 1 && a->sw == 1 &&
                      a->ph == 0 && a->pw == 0 && a->dh == 1 && a->dw == 1 && (a->up == 0 || (a->up == 2 && !a->res)) &&
                      !a->gate && !a->stats && a->epi == SA_EPI_STORE && a->Ho == a->H && a->Wo == a->W;
      if (!ok) return -5;
      note_split(1, 0, 0);
      return sa_conv_pw(a->src[0].ptr, a->src[0].stride, a->src[0].channels, a->nsrc == 2 ? a->src[1].ptr : nullptr,
                        a->nsrc == 2 ? a->src[1].stride : 0, a->Cin, a->weight, a->Kpad, a->bias, a->out,
                        a->out_stride, a->N, a->H, a->W, a->Cout, a->act, a->alpha, a->scale, a->res, a->res_stride,
                        a->act2, a->up == 2 ? a->cout_real : 0, stream);
    }
    case 25: {
      // strided 1x1 conv (conv_point.hip): 64 -> 96 / 96 -> 128, weights in registers, no LDS
      const bool ok = a->nsrc == 1 && a->src[0].channels == a->Cin && a->KH == 1 && a->KW == 1 && a->ph == 0 &&
                      a->pw == 0 && a->sh == a->sw && a->sh >= 1 && a->dh == 1 && a->dw == 1 && a->KD <= 0 &&
                      a->up == 0 && !a->gate && !a->res && a->epi == SA_EPI_STORE && a->scale == 1.f &&
                      a->Ho == (a->H - 1) / a->sh + 1 && a->Wo == (a->W - 1) / a->sw + 1 &&
                      a->out_stride % 8 == 0 && a->src[0].stride % 8 == 0;
      if (!ok) return -5;
      note_split(1, 0, 0);
      return sa_conv1x1_point(a->src[0].ptr, a->src[0].stride, a->Cin, a->weight, a->Kpad, a->bias, a->out,
                              a->out_stride, a->Cout, a->N, a->H, a->W, a->sh, a->act, a->alpha, a->stats,
                              a->stats_slots, stream);
    }
    case 22: {
      // 7x7 stem conv (conv_stem.hip): one <= 4-real-channel source, 64 outputs, pad 3, stride 1 / 2
      const int cr = a->cin_real > 0 ? a->cin_real : a->Cin;
      const bool ok = a->nsrc == 1 && a->src[0].channels == a->Cin && cr <= 4 && a->KH == 7 && a->KW == 7 &&
                      a->sh == a->sw && (a->sh == 1 || a->sh == 2) && a->ph == 3 && a->pw == 3 && a->dh == 1 &&
                      a->dw == 1 && a->KD <= 0 && a->up == 0 && !a->gate && !a->res && a->epi == SA_EPI_STORE &&
                      a->scale == 1.f && a->Cout == 64 && a->Kpad >= 49 * a->Cin && a->out_stride % 8 == 0 &&
                      a->src[0].stride % 4 == 0 &&
                      (a->act == SA_ACT_NONE || a->act == SA_ACT_RELU || a->act == SA_ACT_LEAKY);
      if (!ok) return -5;
      note_split(1, 0, 0);
      return sa_conv7x7_stem(a->src[0].ptr, a->src[0].stride, cr, a->weight, a->Kpad, a->Cin, a->bias, a->out,
                             a->out_stride, a->N, a->H, a->W, a->sh, a->act, a->alpha, a->stats, a->stats_slots,
                             stream);
    }
    case 4: case 5: case 7: case 8: {
      const int r = cfg == 4 ? launch_glds3<256, 128, 4, 2>(a, stream, true)
                  : cfg == 5 ? launch_glds3<128, 64, 2, 2>(a, stream, true)
                  : cfg == 7 ? launch_glds3<128, 128, 2, 4>(a, stream, true)
                             : launch_glds3<256, 64, 4, 2>(a, stream, true);
      return r == 1 ? -5 : r;
    }
    case 14: case 15: case 16: case 17: {
      // deep DMA rings (kGldsDeep): 128x64 / 4 waves (6 stages), 128x128 / 8 waves (5), 64x64 / 4 waves (8),
      // 256x64 / 8 waves (4); one block per CU
      const int r = cfg == 14 ? launch_glds3<128, 64, 2, 2, kGldsDeep>(a, stream, true)
                  : cfg == 15 ? launch_glds3<128, 128, 2, 4, kGldsDeep>(a, stream, true)
                  : cfg == 16 ? launch_glds3<64, 64, 2, 2, kGldsDeep>(a, stream, true)
                              : launch_glds3<256, 64, 4, 2, kGldsDeep>(a, stream, true);
      return r == 1 ? -5 : r;
    }
    case 39: {
      // 64x64 register-staged tile with the whole K (<= 512) in flight at once
      const int r = launch_regall<64, 64, 2, 2>(a, stream);
      return r == 1 ? -5 : r;
    }
    case 37: case 38: {
      // workgroup split-K + reduce / epilogue launch: 128x128 (37) / 64x64 (38) deep DMA ring partial tiles (a slice
      // is only a few k-steps: the whole of it in flight)
      const int r = cfg == 37 ? launch_splitx<128, 128, 2, 4, kGldsDeep>(a, stream)
                              : launch_splitx<64, 64, 2, 2, kGldsDeep>(a, stream);
      return r == 1 ? -5 : r;
    }
    case 10: case 11: {
      // 8 waves of 128x64 (2 per SIMD): 256x256 (10) / 512x128 (11)
      const int r = cfg == 10 ? launch_wide<256, 256, 2, 4>(a, stream) : launch_wide<512, 128, 4, 2>(a, stream);
      return r == 1 ? -5 : r;
    }
    case 26: case 27: case 28: case 29: case 30: case 31: case 32: case 33: {
      // halo-reuse 3x3 tiles: 8 x 32 (26) / 16 x 16 (27) output patches x 128 channels; 28 / 29 the same with the
      // planar patch image (kHaloP); 30 / 31 the wide 16 x 32 / 12 x 32 patches in 32-channel chunks (kHaloW)
      const int r = cfg == 26 ? launch_halo<kHalo>(a, stream)
                  : cfg == 27 ? launch_halo<kHalo16>(a, stream)
                  : cfg == 28 ? launch_halo<kHaloP>(a, stream)
                  : cfg == 29 ? launch_halo<kHaloP16>(a, stream)
                  : cfg == 30 ? launch_halo<kHaloW>(a, stream)
                  : cfg == 31 ? launch_halo<kHaloW12>(a, stream)
                  : cfg == 32 ? launch_halo<kHaloQ>(a, stream)
                              : launch_halo<kHaloQ12>(a, stream);
      return r == 1 ? -5 : r;
    }
    case 18: case 19: {
      // 8-wave ping-pong (kPing): 256x256 (4-deep ring) / 256x128 (6-deep ring), DMA issued in the read slot
      const int r = cfg == 18 ? launch_ping<256, 256>(a, stream) : launch_ping<256, 128>(a, stream);
      return r == 1 ? -5 : r;
    }
    default: return -3;
  }
}

namespace {
// Flow-head tail in one launch: the per-pixel 3x3-tap projections of a C -> 1 conv over a (TH+2) x (TW+2) halo
// region (MFMA, fp32 planes in LDS; halo pixels outside the image project zero activations, which is exactly the
// following conv's zero padding), then the 9-tap stencil + bias accumulated into the fp32 flow.  One launch and
// no HBM round trip of the 9 tap planes on every GRU iteration's critical path; the halo recompute (2.1x at
// 2 x 32 tiles, 1.5x at 4 x 64) only re-reads activations.
template <int TH, int TW, int OC>
__global__ __launch_bounds__(256) void flow_head_tail_kernel(const f16* __restrict__ y, int ys, int C,
                                                             const f16* __restrict__ w16, const float* __restrict__ bias,
                                                             float* __restrict__ flow, int N, int H, int W) {
  // OC output channels (RAFT: the x flow; CREStereo: x and y): 9 * OC projection taps, tap j = (ky*3+kx)*OC + o,
  // in NB 16-column MFMA tiles; flow is [N][H][W][OC] fp32
  constexpr int RH = TH + 2, RW = TW + 2, R = RH * RW, NF = (R + 15) / 16, PS = 9 * OC, NB = (PS + 15) / 16;
  __shared__ float P[NF * 16 * PS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int frow = lane & 15, kq = lane >> 4;
  const int tiles_x = (W + TW - 1) / TW, tiles_y = (H + TH - 1) / TH;
  const int t = blockIdx.x, n = t / (tiles_x * tiles_y), rr = t - n * tiles_x * tiles_y;
  const int ty = rr / tiles_x, tx = rr - ty * tiles_x;
  const int y0 = ty * TH - 1, x0 = tx * TW - 1;
  const int ks = C >> 5;
  const half8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
  half8 b[NB][8];  // B = 16 tap rows of the projection per tile, column frow, k = kq*8 .. of each 32-deep step
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k)
      b[j][k] = k < ks ? *reinterpret_cast<const half8*>(w16 + (size_t)(16 * j + frow) * C + k * 32 + kq * 8) : zero8;
  for (int f = wave; f < NF; f += 4) {
    const int q = f * 16 + frow;  // halo pixel of this lane's A row
    const int hy = q / RW, hx = q - hy * RW;
    const int gy = y0 + hy, gx = x0 + hx;
    const bool ok = q < R && gy >= 0 && gy < H && gx >= 0 && gx < W;
    const f16* src = y + ((size_t)((size_t)n * H + (ok ? gy : 0)) * W + (ok ? gx : 0)) * ys + kq * 8;
    half8 a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = (ok && k < ks) ? *reinterpret_cast<const half8*>(src + k * 32) : zero8;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[k], b[j][k], acc, 0, 0, 0);
      // acc[r]: halo pixel f*16 + kq*4 + r, tap 16 j + frow
      const int tap = 16 * j + frow;
      if (tap < PS)
#pragma unroll
        for (int r = 0; r < 4; ++r) P[(f * 16 + kq * 4 + r) * PS + tap] = acc[r];
    }
  }
  __syncthreads();
  for (int o = threadIdx.x; o < TH * TW * OC; o += 256) {
    const int c = o % OC, px = o / OC;
    const int oy = px / TW, ox = px - oy * TW;
    const int gy = ty * TH + oy, gx = tx * TW + ox;
    if (gy >= H || gx >= W) continue;
    float s = bias ? bias[c] : 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) s += P[((oy + ky) * RW + ox + kx) * PS + (ky * 3 + kx) * OC + c];
    flow[(((size_t)n * H + gy) * W + gx) * OC + c] += s;
  }
}
__global__ __launch_bounds__(256) void tapproj_stencil_kernel(const float* __restrict__ P, int taps, int oc,
                                                              const float* __restrict__ bias, float* __restrict__ flow,
                                                              int N, int H, int W) {
  const long total = (long)N * H * W * oc;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int o = (int)(i % oc);
    const long px = i / oc;
    const int x = (int)(px % W);
    const long r = px / W;
    const int y = (int)(r % H);
    const long n = r / H;
    float s = bias ? bias[o] : 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int yy = y + ky - 1, xx = x + kx - 1;
        if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
        const float* q = P + ((n * H + yy) * W + xx) * 2 * taps + (ky * 3 + kx) * oc + o;
        s += q[0] + q[taps];
      }
    flow[px * oc + o] += s;
  }
}
}  // namespace

extern "C" int sa_tapproj_stencil(const float* P, int taps, int oc, const float* bias, float* flow, int N, int H,
                                  int W, hipStream_t stream) {
  if (!P || !flow || (oc != 1 && oc != 2) || taps != 9 * oc || N < 1 || H < 1 || W < 1) return -2;
  const long total = (long)N * H * W * oc;
  long g = (total + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(tapproj_stencil_kernel, dim3((unsigned)g), dim3(256), 0, stream, P, taps, oc, bias, flow, N, H, W);
  return (int)hipGetLastError();
}

extern "C" int sa_flow_head_tail_oc(const void* y, int ys, int C, const void* w16, int oc, const float* bias,
                                    float* flow, int N, int H, int W, hipStream_t stream) {
  if (C % 32 || C > 256 || C < 32 || ys < C || ys % 8 || N < 1 || H < 1 || W < 1 || (oc != 1 && oc != 2)) return -2;
  const long M = (long)N * H * W;
  // small frames (batch 1 at 1/4 resolution): 2 x 32 tiles, enough blocks to cover the CUs; else 4 x 64 (less halo)
  const bool small = M <= 40000;
  const long tiles = small ? (long)N * ((H + 1) / 2) * ((W + 31) / 32) : (long)N * ((H + 3) / 4) * ((W + 63) / 64);
  const f16* yy = (const f16*)y;
  const f16* ww = (const f16*)w16;
  if (oc == 1 && small)
    hipLaunchKernelGGL((flow_head_tail_kernel<2, 32, 1>), dim3((unsigned)tiles), dim3(256), 0, stream, yy, ys, C, ww,
                       bias, flow, N, H, W);
  else if (oc == 1)
    hipLaunchKernelGGL((flow_head_tail_kernel<4, 64, 1>), dim3((unsigned)tiles), dim3(256), 0, stream, yy, ys, C, ww,
                       bias, flow, N, H, W);
  else if (small)
    hipLaunchKernelGGL((flow_head_tail_kernel<2, 32, 2>), dim3((unsigned)tiles), dim3(256), 0, stream, yy, ys, C, ww,
                       bias, flow, N, H, W);
  else
    hipLaunchKernelGGL((flow_head_tail_kernel<4, 64, 2>), dim3((unsigned)tiles), dim3(256), 0, stream, yy, ys, C, ww,
                       bias, flow, N, H, W);
  return (int)hipGetLastError();
}

extern "C" int sa_flow_head_tail(const void* y, int ys, int C, const void* w16, const float* bias, float* flow, int N,
                                 int H, int W, hipStream_t stream) {
  return sa_flow_head_tail_oc(y, ys, C, w16, 1, bias, flow, N, H, W, stream);
}
