// Launch-argument structs and host launchers for every hand-written CDNA4 kernel.
// The structs are plain C so that the Python ctypes layer (stereoalgorithms_amd/_native.py)
// can mirror them field-for-field for numerics tests against PyTorch.
//
// Layout conventions (all kernels):
//   * activations are NHWC, fp16, with an explicit per-pixel stride in ELEMENTS so that a
//     tensor can be a channel slice of a wider buffer (concat-free producers/consumers);
//   * channel counts/offsets/strides used by vectorised paths are multiples of 8 (16 B);
//   * weights for convolutions are pre-packed fp16 [Cout_pad][Kpad], K ordered (kh, kw, ci).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Instance-norm statistics are accumulated as 64-bit fixed point (value * 2^24) with integer
// atomics: integer addition is associative, so the sums -- and every replay of a captured frame --
// are bitwise deterministic regardless of the order blocks arrive in.
typedef long long sa_stat_t;
#define SA_STAT_SCALE 16777216.0

enum SaAct { SA_ACT_NONE = 0, SA_ACT_RELU = 1, SA_ACT_LEAKY = 2, SA_ACT_TANH = 3, SA_ACT_SIGMOID = 4, SA_ACT_RELU6 = 5 };

enum SaEpi {
  SA_EPI_STORE = 0,     // y = act(acc*scale + bias) [; y = act2(y + res)] -> fp16
  SA_EPI_GRU_ZR = 1,    // z = sig(acc+b+cz) -> aux ; r = sig(acc+b+cr) -> rh = r*h
  SA_EPI_GRU_Q = 2,     // q = tanh(acc+b+cq) ; h = (1-z)h + zq  (in place on h)
  SA_EPI_FLOW_ACC = 3,  // fp32 out[m*out_stride + c] += acc*scale + bias for c < min(Cout, out_stride)
  SA_EPI_STORE_F32 = 4,  // y = act(acc*scale + bias) -> fp32
  // 5: retired (projection epilogue; the flow-head conv2 is sa_flow_head_tail now)
  SA_EPI_GRU_ZRQ = 6,    // Cout = 3 Hd stacked [convz | convr | convq restricted to the x inputs]: z -> aux,
                         // r*h -> rh as SA_EPI_GRU_ZR, and the x half of q's pre-activation (acc + bias + cq)
                         // -> out (fp16); the following SA_EPI_GRU_Q conv over r*h alone adds it back (res)
  SA_EPI_TAPPROJ = 7     // flow-head conv1 with the next 3x3 -> oc conv's tap projections fused: y = fp16(act(acc +
                         // bias)) is never stored; out (fp32) [m][n-tile][taps] gets, per 128-channel n-tile, the
                         // partial sums over its channels of y * tapw[t] (tapw fp16 [taps][Cout], taps = 9 oc <= 18);
                         // sa_tapproj_stencil adds both partials' 3x3 neighbourhoods into the flow.  128-wide n-tiles
                         // only (other tile configs return -5)
};

typedef struct {
  const void* ptr;  // fp16 data, already offset to this source's first channel
  int32_t channels; // multiple of 8
  int32_t stride;   // elements between consecutive pixels
} SaConvSrc;

typedef struct {
  SaConvSrc src[4];
  int32_t nsrc;
  int32_t N, H, W, Cin;  // Cin = sum(src[i].channels)
  int32_t KH, KW, sh, sw, ph, pw, dh, dw;
  int32_t Ho, Wo;
  const void* weight;  // fp16 [Cout_pad][Kpad]
  const float* bias;   // [Cout] or NULL
  int32_t Cout, Kpad;
  void* out;
  int32_t out_stride;
  int32_t epi, act, act2;
  float alpha;  // leaky slope
  float scale;  // multiplies acc before bias
  const void* res;  // residual fp16 (SA_EPI_STORE); SA_EPI_GRU_Q: pre-activation addend (the ZRQ conv's out)
  int32_t res_stride;
  const void* ctx;  // GRU context biases fp16: ZR reads [cz | cr], Q reads cq (NULL = none)
  int32_t ctx_stride;
  void* aux;  // GRU z buffer fp16
  int32_t aux_stride;
  void* hbuf;  // GRU hidden state fp16
  int32_t h_stride;
  void* rh;  // GRU r*h output fp16 (ZR)
  int32_t rh_stride;
  sa_stat_t* stats;  // optional per-(n, cout) fixed-point {sum, sumsq} of the stored value
  int32_t tile_cfg;  // -1 = auto
  // split-K: 0 = auto (needs ws/counters), 1 = off, >1 = forced slice count.  Slices write fp32
  // partial slabs to `ws`; the last-arriving block of a tile (agent-scope counter) sums them and
  // runs the fused epilogue.  `counters` must be zero-initialised once (arrivers reset them).
  int32_t splitk;
  float* ws;
  int32_t* counters;
  int64_t ws_floats;
  int32_t n_counters;
  // 3-D convolution (0 = 2-D): volumes are [N][D][H][W][C]; output slice do reads input slices
  // do*sd - pd + kd (kd < KD), K ordered (kd, kh, kw, ci)
  int32_t KD, Di, Do, sd, pd;
  // transposed-conv output mode: the packed weights hold 4 (2-D) / 8 (3-D) parity classes of
  // cout_real channels; the epilogue scatters them to the 2x upsampled output (up = 2 or 3)
  int32_t up, cout_real;
  // optional channel gate (Fast-ACVNet channelAtt): y *= gate[n][oh][ow][co] after the activation,
  // broadcast over depth
  const void* gate;
  int32_t gate_stride;
  // instance-norm statistics spread over `stats_slots` copies of [N][Cout][2] (block b adds into
  // copy b % slots): atomics of the thousands of blocks of one image no longer pile onto one row of
  // addresses.  sa_stats_reduce() folds the copies into copy 0 before the statistics are read.
  int32_t stats_slots;
  // real input channels when the single source is zero-padded beyond them (0 = all channels real); lets
  // the 7x7 stem kernel (tile_cfg 22) stage only the real channels
  int32_t cin_real;
  // SA_EPI_TAPPROJ: the projection weights fp16 [taps][Cout] and their count
  const void* tapw;
  int32_t taps;
  // input instance norm folded into the conv (tile_cfg 23 only; other tactics return -5): src[0] is a conv's RAW
  // output and in_stats its slotted statistics ([in_slots][N][Cin][2]); the conv reads relu(IN(src[0])) (eps in_eps)
  const sa_stat_t* in_stats;
  int32_t in_slots;
  float in_eps;
} SaConvArgs;

int sa_conv2d(const SaConvArgs* a, hipStream_t stream);
// direct 3x3 / stride 1 or 2 conv for small channel counts (tile_cfg 36; stride 2: dilation 1, no scatter): Cin in {8, 16, 32, 48, 64, 96} from one source or
// two channel-concatenated ones (x0: c0 channels, x1: Cin - c0), Cout <= 64, dilation = padding in {1, 2, 4};
// y = act(acc * scale + bias) [; y = act2(y + res)] -> fp16, or fp32 with out_f32 (no residual); cout_real > 0: the
// 4 parity classes of a k4 / s2 transposed conv scattered to the 2x output (no residual)
int sa_conv2d_small(const void* x0, int xs0, int c0, const void* x1, int xs1, int Cin, const void* w, int Kpad,
                    const float* bias, void* out, int os, int N, int H, int W, int Cout, int act, float alpha,
                    float scale, const void* res, int rs, int act2, int dil, int out_f32, int cout_real, int stride,
                    hipStream_t stream);
// pointwise 1x1 / stride 1 conv for narrow GEMMs (tile_cfg 35): Cin <= 256 (multiple of 8) from x (c0 channels) and
// x1 (the rest), Cout <= 256, NHWC fp16 over N x H x W pixels; y = act(acc * scale + bias) [; y = act2(y + res)] ->
// fp16; cout_real > 0: Cout = 4 parity classes scattered to the 2x output (transposed k = 2, s = 2), no residual
int sa_conv_pw(const void* x, int xs, int c0, const void* x1, int xs1, int Cin, const void* w, int Kpad,
               const float* bias, void* out, int os, int N, int H, int W, int Cout, int act, float alpha, float scale,
               const void* res, int rs, int act2, int cout_real, hipStream_t stream);
// direct 3x3x3 / pad 1 conv over NDHWC fp16 volumes with Cin in {8, 16, 32}, Cout <= 32 (tile_cfg 34), stride 1 (or 2
// for Cin <= 16):
// y = act(acc * scale + bias) [* gate[n][h][w][c]] -> fp16 (fp32 with out_f32); cout_real > 0: the 8 parity classes
// of a k4 / s2 transposed conv3d scattered to the 2x output volume (no gate)
int sa_conv3d_small(const void* x, int xs, int Cin, const void* w, int Kpad, const float* bias, void* out, int os,
                    int N, int D, int H, int W, int Cout, int act, float alpha, float scale, const void* gate, int gs,
                    int out_f32, int cout_real, int stride, hipStream_t stream);
// One ConvGRU level in one launch: the z/r conv `za` (SA_EPI_GRU_ZR or SA_EPI_GRU_ZRQ), a grid-wide barrier, the q
// conv `qa` (SA_EPI_GRU_Q), on `grid` <= 128 co-resident workgroups (64x64 deep-ring tiles, split-K slices over the
// workspace both args carry).  `bar`: 4 zero-initialised uints owned by this level (arrivals, generation, timeout
// flag), reusable across launches and graph replays.  Sources must be multiples of 64 channels (3x3 or 1x1, no
// statistics).  Returns -2 on ineligible args.
int sa_gru_level(const SaConvArgs* za, const SaConvArgs* qa, unsigned* bar, int grid, hipStream_t stream);
// flow [N][H][W][oc] fp32 += bias[o] + sum over the 3x3 neighbourhood (zero padding) of the two n-tile partials of
// tap (ky*3+kx)*oc + o in P [N][H][W][2][taps] (an SA_EPI_TAPPROJ conv's output)
int sa_tapproj_stencil(const float* P, int taps, int oc, const float* bias, float* flow, int N, int H, int W,
                       hipStream_t stream);
// 7x7 / pad 3 / stride 1 or 2 stem conv, <= 4 real input channels (pixel stride xs, 8-B aligned) -> 64
// channels, weights packed [>=64][kpad] with K ordered (kh, kw, ci < cpad); act none / relu / leaky; optional
// slotted IN statistics.  Also reachable through sa_conv2d with tile_cfg = 22.
int sa_conv7x7_stem(const void* x, int xs, int creal, const void* w, int kpad, int cpad, const float* bias, void* out,
                    int os, int N, int H, int W, int stride, int act, float alpha, sa_stat_t* stats, int slots,
                    hipStream_t stream);
// Direct 3x3 / stride 1 / pad 1 conv, 64 -> 64 channels (8-wave persistent workgroups over 2x64-pixel tiles,
// channel-split weights stationary in registers, DMA ring, register epilogue with buffer stores): bias / act,
// optional slotted IN statistics or residual y = act2(act(acc + bias) + res) (not both); tile_cfg = 23.
// in_stats (no residual): x is a conv's raw output with those slotted statistics and the conv reads relu(IN(x)).
// -5 when the output span exceeds 32-bit buffer offsets.
int sa_conv3x3_c64_direct2(const void* x, int xs, const void* w, int kpad, const float* bias, void* out, int os,
                           int N, int H, int W, int act, float alpha, sa_stat_t* stats, int slots, const void* res,
                           int rs, int act2, const sa_stat_t* in_stats, int in_slots, float in_eps, int max_blocks,
                           hipStream_t stream);
// Direct 3x3 / pad 1 conv to 96 channels: 96 -> 96 at stride 1 or 64 -> 96 at stride 2 (12-wave persistent
// tiles, weights stationary in registers, DMA ring); act none / relu / leaky, optional slotted IN statistics or
// residual (not both); tile_cfg = 24.  -5 for other shapes or an output span past 32-bit buffer offsets.
int sa_conv3x3_c96_direct(const void* x, int xs, int cin, int stride, const void* w, int kpad, const float* bias,
                          void* out, int os, int N, int H, int W, int act, float alpha, sa_stat_t* stats, int slots,
                          const void* res, int rs, int act2, hipStream_t stream);
// Strided 1x1 conv, 64 -> 96 or 96 -> 128 channels (the encoders' residual downsample), weights in registers,
// B fragments loaded straight from global memory; act none / relu / leaky, optional slotted IN statistics
// (needs Ho * Wo % 16 == 0); tile_cfg = 25.  -5 for other shapes.
int sa_conv1x1_point(const void* x, int xs, int cin, const void* w, int kpad, const float* bias, void* out, int os,
                     int cout, int N, int H, int W, int stride, int act, float alpha, sa_stat_t* stats, int slots,
                     hipStream_t stream);
// split-K footprint of the calling thread's last successful sa_conv2d launch: slab floats and tile
// counters it used (0, 0 when it did not split)
void sa_conv2d_last_split(long* ws_floats, long* tiles);
// LDS bytes per workgroup of tile config cfg (-1: not a tile config the tuner compares by footprint)
int sa_conv2d_tile_lds(int cfg);
// Flow-head conv2 (3x3 C -> 1, the RAFT flow head) in one launch: MFMA tap projections of a halo-tiled region
// (planes in LDS) + the 9-tap stencil, accumulated into the flow:
// flow[n][y][x] += bias[0] + sum_{ky,kx} sum_c y[n][y+ky-1][x+kx-1][c] * w16[ky*3+kx][c] (zero padding);
// w16 fp16 [16][C] (taps >= 9 zero), C % 32 == 0, C <= 256, flow fp32 [N][H][W].
int sa_flow_head_tail(const void* y, int ys, int C, const void* w16, const float* bias, float* flow, int N, int H,
                      int W, hipStream_t stream);
// the same for a 3x3 C -> oc (1 or 2) conv: flow [N][H][W][oc] fp32 += bias[o] + taps, w16 fp16 [16 or 32][C] with
// row (ky*3+kx)*oc + o (rows >= 9 oc zero)
int sa_flow_head_tail_oc(const void* y, int ys, int C, const void* w16, int oc, const float* bias, float* flow, int N,
                         int H, int W, hipStream_t stream);

// ---- normalisation / elementwise ------------------------------------------------------------
// Instance-norm apply (biased var, eps): y = act(norm(x)); if res: y = act2(res_act(resnorm(res)) + y)
typedef struct {
  const void* x; int32_t x_stride;
  const sa_stat_t* stats;      // [N][C][2] fixed-point sums of x (stat_slots copies of it, summed here)
  const void* res; int32_t res_stride;
  const sa_stat_t* res_stats;  // NULL -> residual used raw
  void* out; int32_t out_stride;
  int32_t N, HW, C;
  int32_t act, act2;
  float eps, alpha;
  int32_t stat_slots;          // copies of [N][C][2] the conv epilogues accumulated into (0 / 1: one, reduced)
  int32_t res_act;             // activation of the normalised residual (res_stats only)
} SaNormArgs;
int sa_instnorm_apply(const SaNormArgs* a, hipStream_t stream);
// stats[0][i] = sum_r stats[r][i], stats[r>0][i] = 0 for i < count (idempotent)
int sa_stats_reduce(sa_stat_t* stats, int slots, long count, hipStream_t stream);
// res[0] = max |a - b| (NaN / inf -> +inf), res[1] = max |b| over n fp16 (f32 = 0) or fp32 elements, as float
// bits merged with atomicMax: the caller zeroes res first.
int sa_absdiff_max(const void* a, const void* b, long n, int f32, unsigned* res, hipStream_t stream);
// buf[idx] = wall_clock64() once everything queued before on `stream` has finished
int sa_stamp(unsigned long long* buf, int idx, hipStream_t stream);
// zero `bytes` with a kernel (16-B vector stores when p / bytes are 16-B multiples, else 4-B stores; p and bytes
// must be 4-B multiples); graph-capturable, and unlike a hipMemsetAsync node it is an ordinary kernel node
int sa_zero(void* p, size_t bytes, hipStream_t stream);

// F.avg_pool2d(x, 3, stride=2, padding=1) (count_include_pad) on NHWC fp16
int sa_avgpool3s2(const void* x, int x_stride, void* out, int out_stride, int N, int H, int W,
                  int C, hipStream_t stream);
// F.avg_pool2d(x, k, stride=k) (k = 2, 4, ...)
int sa_avgpool_k(const void* x, int x_stride, void* out, int out_stride, int N, int H, int W,
                 int C, int k, hipStream_t stream);
// F.interpolate(x, (Ho, Wo), mode='bilinear', align_corners) on NHWC fp16, optional scale
int sa_interp_bilinear(const void* x, int x_stride, void* out, int out_stride, int N, int H,
                       int W, int C, int Ho, int Wo, int align_corners, float mul,
                       hipStream_t stream);
// sa_avgpool3s2 (p*) and sa_interp_bilinear (i*) in one launch (disjoint block ranges; bitwise the same results)
int sa_pool_interp(const void* px, int pxs, void* pout, int pos, int pN, int pH, int pW, int pC, const void* ix,
                   int ixs, void* iout, int ios, int iN, int iH, int iW, int iC, int iHo, int iWo, int align_corners,
                   float mul, hipStream_t stream);

// ---- RAFT-Stereo correlation ----------------------------------------------------------------
// corr[b,h,w1,w2] = <f1[b,h,w1,:], f2[b,h,w2,:]>/sqrt(C), plus avg-pool pyramid along w2.
// pyr points to levels laid out back to back: level l is [B*H][W1][W2_l] fp32.
int sa_corr1d_pyramid(const void* f1, const void* f2, int stride, int B, int H, int W1, int W2,
                      int C, int levels, float* pyr, hipStream_t stream);
// Lookup: for each pixel, levels x (2r+1) bilinear taps along w2 at coords/2^l + dx.
// flow = fp32 x-flow [B*H*W1]; coords_x = w1 + flow.  Writes fp16 corr features (out, C_out
// channels, zero padded), and optionally flow features [flow_x, 0, ...] into flow_out slots.
int sa_corr1d_lookup(const float* pyr, const float* flow, int B, int H, int W1, int W2,
                     int levels, int radius, void* out, int out_stride, int out_channels,
                     void* flow_out, int flow_stride, int flow_channels, void* flow_out2,
                     int flow_stride2, hipStream_t stream);

// Fused RAFT motion-encoder head: lookup (as sa_corr1d_lookup) -> cor1 = relu(convc1) and
// flo1 = relu(convf1 7x7 on [flow_x, 0]) as fp16 NHWC (64 channels each), plus [flow_x, 0] into
// fcopy.  wc: fp32 [levels*(2r+1)][64], wf: fp32 [49][64] (x-channel taps), biases [64].
int sa_raft_motion_head(const float* pyr, const float* flow, int B, int H, int W1, int W2, int levels,
                        int radius, const float* wc, const float* bc, const float* wf, const float* bf,
                        void* cor, int cstride, void* flo, int fstride, void* fcopy, int fcstride,
                        hipStream_t stream);
// The whole RAFT motion encoder in one kernel (motion_enc.hip): lookup -> relu(convc1) / relu(convf1) ->
// relu(convc2) / relu(convf2) -> relu(conv) + [fx, 0] tail, every intermediate kept in LDS per 8x16 output tile.
// w1: fp16 [128][96] block-diagonal [convc1 (rows 0-63, k < L(2r+1)) | convf1 x-taps (rows 64-127, 49 k from
// L(2r+1))], b1 [128]; w2c / w2f: convc2 / convf2 packed fp16 [>=64][576]; w3: conv packed [>=128][1152] (K order
// (kh, kw, ci), ci over [cor2 | flo2]); b3 [126].  levels = radius = 4.  out: fp16 [B][H][W][os >= 128].
int sa_raft_motion_encoder(const float* pyr, const float* flow, int B, int H, int W, int W2, int levels, int radius,
                           const void* w1, const float* b1, const void* w2c, const float* b2c, const void* w2f,
                           const float* b2f, const void* w3, const float* b3, void* out, int os, hipStream_t stream);
// the same with the previous flow head's tap projections (SA_EPI_TAPPROJ output P [B][H][W][2][9], bias: the tail
// conv's) applied while the flow is read: flow_out (!= flow) receives flow + stencil(P) -- sa_tapproj_stencil fused
int sa_raft_motion_encoder_proj(const float* pyr, const float* flow, int B, int H, int W, int W2, int levels,
                                int radius, const void* w1, const float* b1, const void* w2c, const float* b2c,
                                const void* w2f, const float* b2f, const void* w3, const float* b3, void* out, int os,
                                const float* proj, const float* proj_bias, float* flow_out, hipStream_t stream);
// diagnostics: s_memrealtime (100 MHz) stage marks of every workgroup of later sa_raft_motion_encoder launches into `buf`
// ([blocks][8 marks][64] u64; NULL turns it off)
void sa_raft_motion_encoder_stamps(void* buf);
// kernel variant of later sa_raft_motion_encoder launches: 1 = one 159-KB workgroup per CU (LDS weight rings),
// 2 = two 63-KB workgroups per CU (register weight pipeline), -1 = SA_RAFT_MENC (default 1)
void sa_raft_motion_encoder_variant(int v);

// ---- upsampling -----------------------------------------------------------------------------
// RAFT convex upsampling: mask [B*H*W][9*f*f] fp16 (softmax over the 9), flow fp32 [B*H*W]
// (x component).  Writes full-res fp32 output = sign * (f * flow) combination.
int sa_convex_upsample(const void* mask, int mask_stride, const float* flow, int B, int H, int W,
                       int factor, float sign, float* out, hipStream_t stream);
// multi-channel variant: flow fp32 [B][H][W][fc]; out fp32 [B][H*f][W*f][oc] gets the first oc
// channels of sign * convex(f * flow)
int sa_convex_upsample_c(const void* mask, int mask_stride, const float* flow, int fc, int B, int H, int W,
                         int factor, float sign, float* out, int oc, hipStream_t stream);

// ---- pre / post processing ------------------------------------------------------------------
enum SaNormMode {
  SA_PRE_RAW = 0,        // RGB 0..255 (RAFT/CREStereo reference inputs)
  SA_PRE_UNIT = 1,       // RGB / 255 (HITNet)
  SA_PRE_IMAGENET = 2,   // (RGB/255 - mean)/std (Fast-ACVNet+)
  SA_PRE_SIGNED = 3      // 2*(RGB/255) - 1 (RAFT / CREStereo in-network normalisation)
};
// u8 BGR [B][H][W][3] -> fp16 NHWC, channels [c_off, c_off+3) of a stride-`out_stride` pixel,
// remaining channels up to `zero_to` zero-filled.
int sa_preprocess(const uint8_t* bgr, int B, int H, int W, int mode, void* out, int out_stride,
                  int c_off, int zero_to, hipStream_t stream);
// Bilinear remap (cv::remap INTER_LINEAR, BORDER_CONSTANT 0) of u8 BGR with float maps
// [H][W][2]; B images share `maps` index b % nmaps.
int sa_remap_bgr(const uint8_t* src, int B, int Hs, int Ws, const float* maps, int nmaps,
                 int H, int W, uint8_t* dst, hipStream_t stream);
// disparity -> XYZRGB point cloud (cv::reprojectImageTo3D with the full 4x4 Q) + signed copy
// of the disparity.  disp_in has `disp_stride` floats per pixel (channel 0 used).
int sa_reproject(const float* disp_in, int disp_stride, float sign, const uint8_t* left_bgr,
                 int B, int H, int W, const float* Q16, float* disp_out, float* cloud,
                 hipStream_t stream);
// re-point disp_out / cloud of a captured sa_reproject node of an instantiated graph (other arguments unchanged)
int sa_reproject_update_node(hipGraphExec_t exec, hipGraphNode_t node, const float* disp_in, int disp_stride, float sign,
                             const uint8_t* left_bgr, int B, int H, int W, const float* Q16, float* disp_out,
                             float* cloud);

// both frame images from mapped host memory (a, b: device addresses of registered / pinned host arrays) into device
// buffers; bytes % 16 == 0, 16-B aligned.  _update_node re-points a captured node's sources.
int sa_copy_frames(const void* a, const void* b, void* da, void* db, long bytes, hipStream_t stream);
int sa_copy_frames_update_node(hipGraphExec_t exec, hipGraphNode_t node, const void* a, const void* b, void* da,
                               void* db, long bytes);

// ---- CREStereo / Fast-ACVNet+ / HITNet ops (stereo_ops.hip) ---------------------------------
typedef struct {
  const void* f1; int32_t f1_stride;      // left features fp16 NHWC, C channels (4 groups)
  const void* f2; int32_t f2_stride;      // right features
  const float* flow;                      // fp32 [N][H][W][2]
  const void* offset; int32_t offset_stride;  // fp16 [N][H][W][18] learned (x, y) offsets or NULL
  int32_t N, H, W, C;
  int32_t small_patch;  // 0: 1x9 window, 1: 3x3
  int32_t iter_mode;    // 1: warp-then-window (replicate pad); 0: offset sampling (zero pad)
  void* out; int32_t out_stride; int32_t out_channels;  // fp16, 36 used, rest zero-filled
} SaAgclArgs;
int sa_agcl_corr(const SaAgclArgs* a, hipStream_t stream);
// iter-mode AGCL + the motion encoder's convc1 (1x1, 36 -> cout = 256, + bias, relu) in one launch (a->out unused):
// w16 [256][64] fp16 (columns >= 36 zero), bias fp32 [256], out fp16 NHWC with pixel stride out_stride
int sa_agcl_conv1x1(const SaAgclArgs* a, const void* w16, const float* bias, int cout, void* out, int out_stride,
                    hipStream_t stream);
// CREStereo motion-encoder head in one launch (iter mode): AGCL -> convc1 (as sa_agcl_conv1x1) and, when wf16 is set,
// convf1 (7x7, 2 -> 128, pad 3, + fbias, relu) on the fp16 flow into flo, plus the fp16 flow copy into fcopy[0:2]
typedef struct {
  const void* w16; const float* bias; void* cor; int32_t cor_stride;      // convc1: [256][64] fp16, k >= 36 zero
  const void* wf16; const float* fbias; void* flo; int32_t flo_stride;    // convf1: [128][128] fp16, k = c*49+ky*7+kx
  void* fcopy; int32_t fcopy_stride;                                      // fp16 (x, y) of the flow per pixel
} SaCreHeadArgs;
int sa_cre_motion_head(const SaAgclArgs* a, const SaCreHeadArgs* h, hipStream_t stream);
// the same head from a correlation already in a->out (a->out_stride, 36 channels; offset mode: sa_agcl_corr first);
// convf1 / fcopy required
int sa_cre_motion_head_pre(const SaAgclArgs* a, const SaCreHeadArgs* h, hipStream_t stream);

// ws: fp32 workspace of sa_linear_attention_ws_floats(N, S, heads, dim) floats (per-chunk partial KV / Ksum)
long sa_linear_attention_ws_floats(int N, int S, int heads, int dim);
int sa_linear_attention(const void* q, int qs, const void* k, int ks, const void* v, int vs, void* out, int os,
                        int N, int L, int S, int heads, int dim, float eps, float* ws, hipStream_t stream);
int sa_layernorm(const void* x, int xs, const float* gamma, const float* beta, const void* res, int rs, void* out,
                 int os, long rows, int C, float eps, hipStream_t stream);

// out[p][c] = act(x[p][c]*scale + add[p][c] + bcast[p % period][c]) over P pixels x C channels
typedef struct {
  const void* x; int32_t x_stride;
  const void* add; int32_t add_stride;   // optional fp16 addend
  const float* bcast; int64_t bcast_period;  // optional fp32 [period][C] addend
  void* out; int32_t out_stride;
  int64_t P; int32_t C;
  int32_t act; float scale;
} SaEwArgs;
int sa_ew(const SaEwArgs* a, hipStream_t stream);

// fp32 flow [P][fc] -> fp16 (fx, fy, 0...) into out1 (c1 channels, stride s1) and/or (fx, fy) into out2
int sa_flow_features(const float* flow, int fc, long P, void* out1, int s1, int c1, void* out2, int s2,
                     hipStream_t stream);
// fp32 NHWC bilinear resize (align_corners=True) x mul
int sa_interp_flow(const float* x, float* out, int N, int H, int W, int C, int Ho, int Wo, float mul,
                   hipStream_t stream);

// ---- Fast-ACVNet+ volume ops (volume_ops.hip) -------------------------------------------------
// depthwise 3x3 conv, pad 1, stride 1/2 (MobileNetV2), fp32 folded weights [C][9] + bias [C]
int sa_dwconv3x3(const void* x, int xs, const float* w, const float* b, void* out, int os, int N, int H, int W,
                 int C, int stride, int act, hipStream_t stream);
// normalised correlation volume [N][D][H][W][os] (channel 0; 1..7 zero)
int sa_norm_corr_volume(const void* l, int ls, const void* r, int rs, int N, int H, int W, int C, int D, void* out,
                        int os, hipStream_t stream);
// softmax over D + top-K planes (indices re-sorted ascending) -> prob / disparity [N][H][W][K] fp32
int sa_topk_disparity(const void* att, int as, int att_f32, int N, int D, int H, int W, int K, float* prob,
                      float* disp, hipStream_t stream);
// attention-weighted concatenation volume [N][K][H][W][2*Cl] at the sampled disparities
int sa_concat_volume(const void* l, int ls, const void* r, int rs, const float* prob, const float* disp, int N, int H,
                     int W, int Cl, int K, void* out, int os, hipStream_t stream);
// top-`top` softmax regression over K cost planes -> disparity [N][H][W] fp32
int sa_topk_regress(const void* cost, int cs, int cost_f32, const float* disp, int N, int K, int H, int W, int top,
                    float* out, hipStream_t stream);
// superpixel context upsampling: softmax(9 spx logits) x 3x3 neighbourhood of the 1/f prediction
int sa_spx_upsample(const void* spx, int ss, const float* pred, int N, int h, int w, int f, float scale, float* out,
                    hipStream_t stream);

// ---- HITNet tile hypotheses (hitnet_ops.hip) --------------------------------------------------
// L1 tile matching cost over d in [0, D) + argmin -> cmin (fp16, channel 0 of a stride-cs pixel; 1..7
// zero) and d_init (fp32) per tile; tl [B][th][tw][16], tr [B][th][wr][16] (stride-(4,1) tile features)
int sa_hitnet_tile_init(const void* tl, int tls, const void* tr, int trs, int B, int th, int tw, int wr, int D,
                        void* cmin, int cs, float* dinit, hipStream_t stream);
// hyp [P][16] fp32 = [d_init, 0, 0, desc[0..12]]
int sa_hitnet_hyp_init(const float* dinit, const void* desc, int ds, long P, float* hyp, hipStream_t stream);
// local warped L1 cost of T x T tiles (T = 4, 2, 1: 3*T*T costs) + fp16 hypothesis copy (16 ch): candidate k
// of tile q -> out[q][k*ccand ...] (row stride ostride); hyp [ncand][B*th*tw][16], th = H/T
int sa_hitnet_warp_cost(const void* el, int els, const void* er, int ers, int B, int H, int W, int C, int T,
                        const float* hyp, int ncand, void* out, int ostride, int ccand, hipStream_t stream);
// refine (cand + delta, delta block of candidate k at channel k*dcand of a stride-dstr row) and, with
// confidences (channel 16 of each block), keep the most confident of ncand candidates -> out [P][16]
int sa_hitnet_select(const float* cand, int ncand, long P, const float* delta, int dstr, int dcand, int has_conf,
                     float* out, hipStream_t stream);
// slanted-plane 2x upsampling of tile hypotheses to the next finer level [B][th][tw][16] -> [B][2th][2tw][16]
int sa_hitnet_upsample(const float* h, int B, int th, int tw, float* out, hipStream_t stream);
// split T x T tiles (T = 4, 2) into T/2 x T/2 tiles of the same level -> [B][2th][2tw][16]
int sa_hitnet_split(const float* h, int B, int th, int tw, int T, float* out, hipStream_t stream);
// disparity [B][T th][T tw] from tiles of size T (plane evaluated per pixel, clamped at 0)
int sa_hitnet_expand(const float* h, int B, int th, int tw, int T, float* disp, hipStream_t stream);

#ifdef __cplusplus
}
#endif
