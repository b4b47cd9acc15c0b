// RAFT-Stereo (sceneflow and realtime presets) as a native op graph.
//
// Reference pins: I/O contract of RAFTStereo/src/TRTRAFTStereo.cpp:13-20
// (inputs left/right [1,3,480,640] RGB 0..255, output flow_up [1,1,H,W] = negative disparity,
// optional low-res flow "diff"), export flags at README_en.md:88-101.  The network itself follows
// upstream RAFT-Stereo (core/raft_stereo.py, extractor.py, update.py, corr.py) with weight names
// identical to the upstream state_dict, so converted checkpoints load unchanged.
//
// Per frame (B stereo pairs):
//   preprocess (2x/255-1, fp16 NHWC)            1 launch
//   feature / context encoders                  ~40-60 launches (instance-norm stats fused in conv)
//   corr pyramid (MFMA, pooled levels fused)    1 launch
//   iters x [lookup, motion encoder x5, ConvGRU(zr+q fused gates) per level, flow head (+coords
//            update fused)]; mask head + convex upsample on the last iteration only
//   reprojection (base class)
// The entire frame is one hipGraph.
#include <cmath>
#include <cstdlib>

#include "blocks.h"

namespace sa {
namespace {

struct RaftCfg {
  int n_downsample = 2;
  int n_gru = 3;
  bool slow_fast = false;
  bool shared = false;
  int iters = 32;
  int hidden = 128;
  int levels = 4;
  int radius = 4;
  Norm context_norm = Norm::Batch;
};

RaftCfg preset(const std::string& name) {
  RaftCfg c;
  if (name == "raftstereo-sceneflow" || name == "raftstereo") {
    // upstream defaults (train_stereo.py / demo.py): n_downsample 2, 3 GRUs, 32 valid iters
  } else if (name == "raftstereo-realtime") {
    // README_en.md:95-101: --shared_backbone --n_downsample 3 --n_gru_layers 2 --slow_fast_gru
    // --valid_iters 7 --mixed_precision
    c.n_downsample = 3;
    c.n_gru = 2;
    c.slow_fast = true;
    c.shared = true;
    c.iters = 7;
  } else {
    throw Error("unknown RAFT-Stereo preset " + name);
  }
  return c;
}

int conv_out(int x, int k, int s, int p) { return (x + 2 * p - k) / s + 1; }

class RaftStereo : public StereoEngine {
 public:
  explicit RaftStereo(const EngineConfig& cfg) : StereoEngine(cfg), rc_(preset(cfg.model)) {
    if (cfg.iters > 0) rc_.iters = cfg.iters;
  }
  const char* name() const override { return "RAFTStereo"; }
  const float* aux_output(int* n) const override {
    *n = B() * lh_[0] * lw_[0];
    return flow_();
  }

 protected:
  void build(WeightSource& src) override;
  void forward(hipStream_t s) override;

 private:
  void gru(hipStream_t s, int lvl, const std::vector<Tensor>& x) const;

  RaftCfg rc_;
  StatsPool sp_;
  Tensor img_;  // [2B][H][W][8] preprocessed
  Tensor imgc_;  // [B][H][W][8] the context trunk's own copy of the left images (SA_RAFT_EARLY_FORK)
  // same-process A/B: b1 8.299 -> 8.218 ms, b8 40.74 -> 40.69 ms; SA_RAFT_EARLY_FORK=0 forks after the preprocessing
  bool early_fork_ = !(std::getenv("SA_RAFT_EARLY_FORK") && std::getenv("SA_RAFT_EARLY_FORK")[0] == '0');
  Trunk fnet_, cnet_;
  ConvLayer fconv2_;          // fnet.conv2 (1x1 128->256) (non-shared)
  ResBlock shared_rb_;        // conv2.0 (shared backbone)
  ConvLayer shared_conv_;     // conv2.1
  std::vector<ResBlock> layer4_, layer5_;
  // context heads [level][net/ctx]
  ResBlock head_rb_[3][2];
  ConvLayer head_conv_[3][2];
  ConvLayer zqr_[3];
  Tensor fmap_;              // [2B][h0][w0][256]
  Tensor net_[3], ctxh_[3], czrq_[3];
  // update block
  ConvLayer convc1_, convc2_, convf1_, convf2_, mconv_;
  ConvLayer gzr_[3], gq_[3];
  // ConvGRU with q's x-input half hoisted into the z/r conv (SA_EPI_GRU_ZRQ): gzrq_ = [convz | convr | convq with
  // its h-input taps zeroed] over [h, x] (Cout 3 hd), gqh_ = convq's h-input taps over r*h alone (K = 9 hd instead
  // of 9 (hd + x)), qx_ = the hoisted x half of q's pre-activation.  Same sums, regrouped: the q conv on the
  // recurrent chain gets 3x shorter, the z/r conv gets a third more columns (more workgroups at batch 1).  The
  // hoisted columns still run the h-input taps (zero weights), +11 % MACs: a latency win at batch <= 2 (b1 network
  // SF 9.05 -> 8.42 ms, RT 2.25 -> 2.10 ms, profiles/timeline_r03.md), a throughput loss at batch 8, so it is on
  // for batch <= 2.  SA_RAFT_GRU_SPLIT=0/1 forces it.
  ConvLayer gzrq_[3], gqh_[3];
  Tensor qx_[3];
  int gru_split_mode_ = std::getenv("SA_RAFT_GRU_SPLIT") ? std::atoi(std::getenv("SA_RAFT_GRU_SPLIT")) : -1;
  bool gru_split_ = false;
  // Pipeline mode 2 layout: motion encoder on the main stream and the finest interp on side2 (default), or round 3's
  // layout with the motion encoder on a third stream (SA_RAFT_M2_MAIN=0).  Measured and dropped in round 4: the
  // finest ZRQ conv split by input source into three convs so that only the motion third stays on the chain -- each
  // batch-1 conv carries ~11 us of fixed cost (prologue, epilogue, launch) and the parts were ~3x less efficient per
  // K step, so the frame got slower, serial schedule included (profiles/round4_notes.md).
  bool m2_main_ = !(std::getenv("SA_RAFT_M2_MAIN") && std::getenv("SA_RAFT_M2_MAIN")[0] == '0');
  ConvLayer fh1_, fh1mask_, mask2_;
  Tensor corr_feat_, flow_feat_, cor1_, flo1_, corflo_, motion_;
  Tensor z_[3], rh_[3];
  Tensor pool_[2], interp_[2];  // pool_[i] = pool2x(net[i]) at level i+1; interp_[i] = interp(net[i+1]) at level i
  Tensor fh_, mask_;
  // flow head conv2 (256 -> 1, 3x3; only the x component of the flow is used): bias, and its taps as fp16 [16][256]
  // (taps 9..15 zero) for sa_flow_head_tail, which projects conv1's output onto the 9 taps over a halo tile and
  // adds the stencil into the flow in one launch (round 2 A/Bs of the alternatives -- conv2 as an N = 1 implicit
  // GEMM, fused into conv1's epilogue, or tap projection + stencil as two launches -- all lost:
  // profiles/flow_head_tail_r02.txt)
  float* fh2_b_ = nullptr;
  void* fh2_w16_ = nullptr;
  // SA_RAFT_FH_PROJ: flow-head conv1 stores conv2's tap projections (SA_EPI_TAPPROJ) instead of its 256-channel
  // output, and a stencil adds them into the flow (all but the last iteration, whose conv1 also feeds the mask
  // head).  Round 4 had it on for the realtime preset only (its per-tap lane reductions cost more than the store
  // they saved on the SF chain: b1 8.26 -> 8.85, b8 43.8 -> 45.4); round 6 computes the projections with MFMAs on
  // the LDS-staged C tile of the banded tiles and is on by default (SA_RAFT_FH_PROJ=0 turns it off)
  int fh_proj_env_ = std::getenv("SA_RAFT_FH_PROJ") ? std::atoi(std::getenv("SA_RAFT_FH_PROJ")) : -1;
  float* fhP_ = nullptr;  // [B][h0][w0][2 n-tiles][9] fp32
  // SA_RAFT_FUSED_LEVEL (bit i = GRU level i): the level's z/r(+q-x) conv, a grid barrier and its q conv in ONE
  // launch (sa_gru_level) at batch <= 2 with the GRU split; lvl_bar_ holds each level's barrier words.  Measured at
  // batch 1 (same-process A/B, profiles/round6_notes.md): coarsest level fused 8.49 -> 9.27 ms (128 workgroups of
  // 128-KB deep-ring tiles), 8.55 -> 10.18 / 8.65 -> 10.38 ms (64 / 128 workgroups of 32-KB register-staged tiles),
  // both coarse levels 11.54 ms: off by default (0)
  int fused_level_mask_ = std::getenv("SA_RAFT_FUSED_LEVEL") ? std::atoi(std::getenv("SA_RAFT_FUSED_LEVEL")) : 0;
  unsigned* lvl_bar_ = nullptr;
  // fused lookup + convc1 + convf1 (sa_raft_motion_head): fp32 [k][64] weights and biases
  float *mh_wc_ = nullptr, *mh_bc_ = nullptr, *mh_wf_ = nullptr, *mh_bf_ = nullptr;
  void* me_w1_ = nullptr;  // fused motion encoder stage-1 weights (fp16 [128][96]) and bias [128]
  float* me_b1_ = nullptr;
  bool fuse_motion_ = true;  // the fused head kernels exist for levels * (2 radius + 1) <= 36 correlation planes
  // the whole motion encoder (head + convc2/convf2 + conv) as one kernel (sa_raft_motion_encoder): bitwise the
  // same output as the head kernel + three convs (same fp16 operands, same k order), 4 launches -> 1 per
  // iteration.  Measured in-process (tools/ab_engine.py): b1 9.94 vs 10.57 ms, b8 53.61 vs 55.75 ms/step.
  // SA_RAFT_FUSE_MENC=0/1 forces the unfused / fused path (default: by tile count, forward()).
  int fuse_menc_mode_ = std::getenv("SA_RAFT_FUSE_MENC") ? std::atoi(std::getenv("SA_RAFT_FUSE_MENC")) : -1;
  bool fuse_menc_ = true;
  // SA_RAFT_PARALLEL=0: run the motion encoder and the coarse GRU levels on one stream
  bool par_ = !(std::getenv("SA_RAFT_PARALLEL") && std::getenv("SA_RAFT_PARALLEL")[0] == '0');
  // Cross-iteration pipeline on a third stream (the 1/16 and 1/8 GRU levels of iteration t+1 under the finest
  // level + flow head of t).  Round 2 first measured it neutral at batch 8 (56.19 vs 56.17 ms/step) and turned it
  // off there, to keep the data-parallel step's copy / RCCL / torch streams within the 4 hardware queues per
  // process; once the encoders and flow head got faster the same A/B in bench.py gives mode 2 at batch 8 172.0 ->
  // 176.2 FPS, and with the RCCL all-gather forced at world size 1 (SA_DP_GATHER_WORLD1=1) 174.2 -> 177.2 FPS
  // (profiles/pipeline_b8_r02.txt), so mode 2 is now the default at every batch.
  // SA_RAFT_PIPELINE=0/1/2 forces a mode (1: G32 one iteration ahead; 2: G32 and G16 ahead, see forward()).
  int cnet_first_mode_ = std::getenv("SA_RAFT_CNET_FIRST") ? std::atoi(std::getenv("SA_RAFT_CNET_FIRST")) : -1;
  int pipeline_mode_ = std::getenv("SA_RAFT_PIPELINE") ? std::atoi(std::getenv("SA_RAFT_PIPELINE")) : -1;
  float* pyr_ = nullptr;
  // flow state, ping-pong: flowbuf_[flow_cur_] holds the current flow; with the stencil fused into the motion
  // encoder (SA_RAFT_FH_FUSE) a head leaves its tap projections pending and the next motion encoder writes
  // flow + stencil into the other buffer (its neighbours still read the old one).  forward() resets the state, so
  // every capture / eager pass walks the same buffers.
  float* flowbuf_[2] = {nullptr, nullptr};
  int flow_cur_ = 0;
  bool flow_pending_ = false;
  float* flow_() const { return flowbuf_[flow_cur_]; }
  // SA_RAFT_FH_FUSE=1: the tap stencil applied inside the next motion encoder's flow-patch load instead of as its
  // own launch after the flow-head conv (one launch and one flow round trip less per iteration).  Measured slower at
  // batch 8 (bench-shaped A/B 39.92 -> 40.13 ms scattered loads, 40.79 -> 41.83 ms LDS-staged): the motion encoder's
  // one-workgroup-per-CU prologue is on the chain and the separate stencil overlaps the coarse levels.  Off by default.
  bool fh_fuse_ = std::getenv("SA_RAFT_FH_FUSE") && std::getenv("SA_RAFT_FH_FUSE")[0] == '1';
  int lh_[3], lw_[3];
};

void RaftStereo::build(WeightSource& src) {
  DeviceArena& a = arena_;
  const int Bn = B();
  const int hd = rc_.hidden;
  img_ = make_tensor(a, 2 * Bn, H(), W(), 8);
  if (early_fork_) imgc_ = make_tensor(a, Bn, H(), W(), 8);

  // ---------------- encoders ----------------
  // conv1 stride 1 + (n_downsample > 2); layer strides 1, 1 + (n_downsample > 1), 1 + (n_downsample > 0)
  const int c1s = 1 + (rc_.n_downsample > 2);
  const int strides[3] = {1, 1 + (rc_.n_downsample > 1), 1 + (rc_.n_downsample > 0)};
  cnet_.build(a, src, sp_, "cnet", rc_.context_norm, rc_.shared ? 2 * Bn : Bn, H(), W(), c1s, strides);
  lh_[0] = cnet_.out().h;
  lw_[0] = cnet_.out().w;
  if (!rc_.shared) {
    fnet_.build(a, src, sp_, "fnet", Norm::Instance, 2 * Bn, H(), W(), c1s, strides);
    src.conv("fnet.conv2", 256, 128, 1, 1);
    ConvSpec s1;
    fconv2_.build(a, *src.ws, {"fnet.conv2"}, {{128, 128}}, s1);
  } else {
    shared_rb_.build(a, src, sp_, "conv2.0", 128, 128, 1, Norm::Instance, 2 * Bn, lh_[0], lw_[0]);
    src.conv("conv2.1", 256, 128, 3, 3);
    ConvSpec s3;
    shared_conv_.build(a, *src.ws, {"conv2.1"}, {{128, 128}}, s3);
  }
  fmap_ = make_tensor(a, 2 * Bn, lh_[0], lw_[0], 256);

  // context levels 2,3 (layer4/5 always exist in MultiBasicEncoder)
  layer4_.resize(2);
  layer5_.resize(2);
  {
    int h = lh_[0], w = lw_[0];
    for (int b = 0; b < 2; ++b) {
      layer4_[b].build(a, src, sp_, "cnet.layer4." + std::to_string(b), 128, 128, b == 0 ? 2 : 1,
                       rc_.context_norm, Bn, h, w);
      h = layer4_[b].out.h;
      w = layer4_[b].out.w;
    }
    lh_[1] = h;
    lw_[1] = w;
    for (int b = 0; b < 2; ++b) {
      layer5_[b].build(a, src, sp_, "cnet.layer5." + std::to_string(b), 128, 128, b == 0 ? 2 : 1,
                       rc_.context_norm, Bn, h, w);
      h = layer5_[b].out.h;
      w = layer5_[b].out.w;
    }
    lh_[2] = h;
    lw_[2] = w;
  }
  const char* lvl_names[3] = {"outputs08", "outputs16", "outputs32"};
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 2; ++j) {
      std::string p = std::string("cnet.") + lvl_names[i] + "." + std::to_string(j);
      ConvSpec s3;
      if (i < 2) {
        head_rb_[i][j].build(a, src, sp_, p + ".0", 128, 128, 1, rc_.context_norm, Bn, lh_[i], lw_[i]);
        src.conv(p + ".1", hd, 128, 3, 3);
        head_conv_[i][j].build(a, *src.ws, {p + ".1"}, {{128, 128}}, s3);
      } else {
        src.conv(p, hd, 128, 3, 3);
        head_conv_[i][j].build(a, *src.ws, {p}, {{128, 128}}, s3);
      }
    }
  }
  for (int i = 0; i < rc_.n_gru; ++i) {
    net_[i] = make_tensor(a, Bn, lh_[i], lw_[i], hd);
    ctxh_[i] = make_tensor(a, Bn, lh_[i], lw_[i], hd);
    czrq_[i] = make_tensor(a, Bn, lh_[i], lw_[i], 3 * hd);
    std::string p = "context_zqr_convs." + std::to_string(i);
    src.conv(p, 3 * hd, hd, 3, 3);
    ConvSpec s3;
    zqr_[i].build(a, *src.ws, {p}, {{hd, hd}}, s3);
  }

  // ---------------- correlation ----------------
  {
    long tot = 0;
    int wl = lw_[0];
    for (int l = 0; l < rc_.levels; ++l) {
      tot += (long)Bn * lh_[0] * lw_[0] * wl;
      wl >>= 1;
    }
    pyr_ = (float*)a.alloc(tot * 4);
  }
  flowbuf_[0] = (float*)a.alloc((size_t)Bn * lh_[0] * lw_[0] * 4);
  flowbuf_[1] = (float*)a.alloc((size_t)Bn * lh_[0] * lw_[0] * 4);
  lvl_bar_ = (unsigned*)a.alloc(3 * 4 * sizeof(unsigned));
  HIP_CHECK(hipMemset(lvl_bar_, 0, 3 * 4 * sizeof(unsigned)));

  // ---------------- update block ----------------
  const int cor_planes = rc_.levels * (2 * rc_.radius + 1);
  const int corp = round_up(cor_planes, 8);
  const std::string u = "update_block.";
  src.conv(u + "encoder.convc1", 64, cor_planes, 1, 1);
  src.conv(u + "encoder.convc2", 64, 64, 3, 3);
  src.conv(u + "encoder.convf1", 64, 2, 7, 7);
  src.conv(u + "encoder.convf2", 64, 64, 3, 3);
  src.conv(u + "encoder.conv", 128 - 2, 128, 3, 3);
  const WeightStore& ws = *src.ws;
  ConvSpec s3, s1, s7;
  s1.kh = s1.kw = 1;
  convc1_.build(a, ws, {u + "encoder.convc1"}, {{cor_planes, corp}}, s1);
  convc2_.build(a, ws, {u + "encoder.convc2"}, {{64, 64}}, s3);
  convf1_.build(a, ws, {u + "encoder.convf1"}, {{2, 8}}, s7);
  convf2_.build(a, ws, {u + "encoder.convf2"}, {{64, 64}}, s3);
  if (cor_planes <= 36) {
    const HostTensor& wc = ws.get(u + "encoder.convc1.weight");  // [64][cor_planes][1][1]
    const HostTensor& wf = ws.get(u + "encoder.convf1.weight");  // [64][2][7][7]
    std::vector<float> hc((size_t)cor_planes * 64), hf(49 * 64);
    for (int o = 0; o < 64; ++o) {
      for (int k = 0; k < cor_planes; ++k) hc[(size_t)k * 64 + o] = wc.data[(size_t)o * cor_planes + k];
      for (int t = 0; t < 49; ++t) hf[(size_t)t * 64 + o] = wf.data[(size_t)o * 98 + t];  // x channel
    }
    auto up = [&](const std::vector<float>& v) {
      float* d = (float*)a.alloc(v.size() * 4);
      HIP_CHECK(hipMemcpy(d, v.data(), v.size() * 4, hipMemcpyHostToDevice));
      return d;
    };
    mh_wc_ = up(hc);
    mh_wf_ = up(hf);
    mh_bc_ = up(ws.get(u + "encoder.convc1.bias").data);
    mh_bf_ = up(ws.get(u + "encoder.convf1.bias").data);
    // the fused encoder's stage-1 operand: block-diagonal fp16 [128][96] (convc1 | convf1 x-taps), bias [128]
    std::vector<_Float16> w1((size_t)128 * 96, (_Float16)0.f);
    for (int o = 0; o < 64; ++o) {
      for (int k = 0; k < cor_planes; ++k) w1[(size_t)o * 96 + k] = (_Float16)hc[(size_t)k * 64 + o];
      for (int t = 0; t < 49; ++t) w1[(size_t)(64 + o) * 96 + cor_planes + t] = (_Float16)hf[(size_t)t * 64 + o];
    }
    me_w1_ = a.alloc(w1.size() * 2);
    HIP_CHECK(hipMemcpy(me_w1_, w1.data(), w1.size() * 2, hipMemcpyHostToDevice));
    std::vector<float> b1(128);
    for (int o = 0; o < 64; ++o) {
      b1[o] = ws.get(u + "encoder.convc1.bias").data[o];
      b1[64 + o] = ws.get(u + "encoder.convf1.bias").data[o];
    }
    me_b1_ = up(b1);
    if (rc_.levels != 4 || rc_.radius != 4) fuse_menc_ = false;  // the fused kernel's K layout
  } else {
    fuse_motion_ = false;
  }
  mconv_.build(a, ws, {u + "encoder.conv"}, {{128, 128}}, s3);

  gru_split_ = gru_split_mode_ >= 0 ? gru_split_mode_ != 0 : Bn <= 2;
  const char* gnames[3] = {"gru08", "gru16", "gru32"};
  for (int i = 0; i < rc_.n_gru; ++i) {
    int xin;
    if (i == 0) xin = 128 + (rc_.n_gru > 1 ? hd : 0);
    else if (i == 1) xin = hd + (rc_.n_gru == 3 ? hd : 0);
    else xin = hd;
    std::string p = u + gnames[i];
    src.conv(p + ".convz", hd, hd + xin, 3, 3);
    src.conv(p + ".convr", hd, hd + xin, 3, 3);
    src.conv(p + ".convq", hd, hd + xin, 3, 3);
    std::vector<ChanSeg> segs = {{hd, hd}};
    for (int k = 0; k < xin / 128; ++k) segs.push_back({128, 128});
    gzr_[i].build(a, ws, {p + ".convz", p + ".convr"}, segs, s3);
    gq_[i].build(a, ws, {p + ".convq"}, segs, s3);
    z_[i] = make_tensor(a, Bn, lh_[i], lw_[i], hd);
    rh_[i] = make_tensor(a, Bn, lh_[i], lw_[i], hd);
    if (gru_split_) {
      // convq [hd][hd + xin][3][3] -> x half (h taps zeroed, bias kept) and h half [hd][hd][3][3] (no bias)
      const HostTensor& wq = ws.get(p + ".convq.weight");
      const int ci = hd + xin;
      HostTensor qxw = wq, qhw;
      qhw.shape = {hd, hd, 3, 3};
      qhw.data.resize((size_t)hd * hd * 9);
      for (int o = 0; o < hd; ++o)
        for (int c = 0; c < hd; ++c)
          for (int t = 0; t < 9; ++t) {
            qhw.data[((size_t)o * hd + c) * 9 + t] = wq.data[((size_t)o * ci + c) * 9 + t];
            qxw.data[((size_t)o * ci + c) * 9 + t] = 0.f;
          }
      src.ws->put(p + ".convq@x.weight", std::move(qxw));
      src.ws->put(p + ".convq@x.bias", ws.get(p + ".convq.bias"));
      src.ws->put(p + ".convq@h.weight", std::move(qhw));
      gzrq_[i].build(a, ws, {p + ".convz", p + ".convr", p + ".convq@x"}, segs, s3);
      gqh_[i].build(a, ws, {p + ".convq@h"}, {{hd, hd}}, s3);
      qx_[i] = make_tensor(a, Bn, lh_[i], lw_[i], hd);
    }
  }
  const int f = 1 << rc_.n_downsample;
  src.conv(u + "flow_head.conv1", 256, hd, 3, 3);
  src.conv(u + "flow_head.conv2", 2, 256, 3, 3);
  src.conv(u + "mask.0", 256, hd, 3, 3);
  src.conv(u + "mask.2", f * f * 9, 256, 1, 1);
  fh1_.build(a, ws, {u + "flow_head.conv1"}, {{hd, hd}}, s3);
  fh1mask_.build(a, ws, {u + "flow_head.conv1", u + "mask.0"}, {{hd, hd}}, s3);
  {
    // only the x component of delta_flow is used (upstream zeroes delta_flow[:,1]): conv2's x-output taps
    const HostTensor& w2 = ws.get(u + "flow_head.conv2.weight");  // [2][256][3][3]
    const HostTensor& b2 = ws.get(u + "flow_head.conv2.bias");
    std::vector<_Float16> w16(16 * 256, (_Float16)0.f);
    for (int c = 0; c < 256; ++c)
      for (int t = 0; t < 9; ++t) w16[t * 256 + c] = (_Float16)w2.data[c * 9 + t];
    fh2_w16_ = a.alloc(w16.size() * 2);
    HIP_CHECK(hipMemcpy(fh2_w16_, w16.data(), w16.size() * 2, hipMemcpyHostToDevice));
    fh2_b_ = (float*)a.alloc(4);
    HIP_CHECK(hipMemcpy(fh2_b_, b2.data.data(), 4, hipMemcpyHostToDevice));
  }
  mask2_.build(a, ws, {u + "mask.2"}, {{256, 256}}, s1, {}, 0.25f);

  const int h0 = lh_[0], w0 = lw_[0];
  corr_feat_ = make_tensor(a, Bn, h0, w0, corp);
  flow_feat_ = make_tensor(a, Bn, h0, w0, 8);
  cor1_ = make_tensor(a, Bn, h0, w0, 64);
  flo1_ = make_tensor(a, Bn, h0, w0, 64);
  corflo_ = make_tensor(a, Bn, h0, w0, 128);
  motion_ = make_tensor(a, Bn, h0, w0, 128);
  fh_ = make_tensor(a, Bn, h0, w0, 512);
  fhP_ = (float*)a.alloc((size_t)Bn * h0 * w0 * 18 * 4);
  mask_ = make_tensor(a, Bn, h0, w0, round_up(f * f * 9, 8));
  for (int i = 0; i + 1 < rc_.n_gru; ++i) {
    pool_[i] = make_tensor(a, Bn, lh_[i + 1], lw_[i + 1], hd);
    interp_[i] = make_tensor(a, Bn, lh_[i], lw_[i], hd);
  }
  sp_.finalize(a);
}

void RaftStereo::gru(hipStream_t s, int i, const std::vector<Tensor>& x) const {
  // the coarse levels of the default schedule (mode-2 pipeline) run beside the finest level's chain (side2): at
  // batch <= 2 their small-grid convs are tuned for co-residency.  Decided by the preset and batch alone -- not by
  // the schedule knobs -- so the eager tuning pass and the capture agree and every schedule runs the same tactics
  // (tests/test_raft_modes_gpu.py: bitwise-equal schedules).  Same-process A/B: b1 8.438 -> 7.991 ms; at b8 (large
  // grids) it cost 1.6 %, so not there.
  // Round 5: the finest level's GRU convs too (they share the chip with the coarse levels' chain, which is the
  // longer path of the b1 iteration cycle): same-process A/B b1 8.208 -> 8.078 ms.  SA_RAFT_SIDE_MASK: bit i marks
  // level i, bit 3 the flow head (default 15; 6 = round 4's coarse levels only; 4 / 0: b1 8.51 / 8.62 ms).
  const int side_mask = std::getenv("SA_RAFT_SIDE_MASK") ? std::atoi(std::getenv("SA_RAFT_SIDE_MASK")) : 15;
  ScopedSideBranch sb(((side_mask >> i) & 1) && B() <= 2 && rc_.n_gru == 3 && !rc_.slow_fast);
  // SA_RAFT_WG_SPLIT (bit i = level i, default 0): the workgroup split-K tactics (37 / 38) become candidates for the
  // level's GRU convs.  All levels on: b1 SF 8.22 -> 8.59 ms, realtime 1.87 -> 1.95 (profiles/round6_notes.md)
  const int wgs_mask = std::getenv("SA_RAFT_WG_SPLIT") ? std::atoi(std::getenv("SA_RAFT_WG_SPLIT")) : 0;
  ScopedWgSplit wgs((wgs_mask >> i) & 1);
  std::vector<Tensor> srcs = {net_[i]};
  srcs.insert(srcs.end(), x.begin(), x.end());
  if (gru_split_) {
    SaConvArgs za = gzrq_[i].args(srcs, qx_[i]);
    za.epi = SA_EPI_GRU_ZRQ;
    za.ctx = czrq_[i].ptr;  // [cz | cr | cq]
    za.ctx_stride = czrq_[i].stride;
    za.aux = z_[i].ptr;
    za.aux_stride = z_[i].stride;
    za.hbuf = net_[i].ptr;
    za.h_stride = net_[i].stride;
    za.rh = rh_[i].ptr;
    za.rh_stride = rh_[i].stride;
    SaConvArgs qa = gqh_[i].args({rh_[i]}, net_[i]);
    qa.epi = SA_EPI_GRU_Q;
    qa.ctx = nullptr;  // cq and convq's bias are in qx
    qa.res = qx_[i].ptr;
    qa.res_stride = qx_[i].stride;
    qa.aux = z_[i].ptr;
    qa.aux_stride = z_[i].stride;
    qa.hbuf = net_[i].ptr;
    qa.h_stride = net_[i].stride;
    if (((fused_level_mask_ >> i) & 1) && B() <= 2 && za.ws && qa.ws) {
      // one launch: z/r/q-x conv, grid barrier, q conv (sa_gru_level); untuned fixed tiles, so nothing is planned
      static const int grid = std::getenv("SA_GRU_LEVEL_GRID") ? std::atoi(std::getenv("SA_GRU_LEVEL_GRID")) : 64;
      const int rc = sa_gru_level(&za, &qa, lvl_bar_ + 4 * i, grid, s);
      if (rc == 0) {
        SA_LAUNCH_CHECK(s);
        if (const SplitKWorkspace* sk = current_splitk()) {
          long fl = 0, tiles = 0;
          sa_conv2d_last_split(&fl, &tiles);
          sk->max_floats = std::max<int64_t>(sk->max_floats, fl);
          sk->max_counters = std::max<int32_t>(sk->max_counters, (int32_t)tiles);
        }
        return;
      }
      SA_LOGW("fused GRU level %d not eligible (rc %d): two launches", i, rc);
    }
    gzrq_[i].launch(s, za);
    gqh_[i].launch(s, qa);
    return;
  }
  SaConvArgs za = gzr_[i].args(srcs, z_[i]);
  za.epi = SA_EPI_GRU_ZR;
  za.ctx = czrq_[i].ptr;
  za.ctx_stride = czrq_[i].stride;
  za.aux = z_[i].ptr;
  za.aux_stride = z_[i].stride;
  za.hbuf = net_[i].ptr;
  za.h_stride = net_[i].stride;
  za.rh = rh_[i].ptr;
  za.rh_stride = rh_[i].stride;
  gzr_[i].launch(s, za);
  srcs[0] = rh_[i];
  SaConvArgs qa = gq_[i].args(srcs, net_[i]);
  qa.epi = SA_EPI_GRU_Q;
  qa.ctx = czrq_[i].slice_c(2 * rc_.hidden, rc_.hidden).ptr;
  qa.ctx_stride = czrq_[i].stride;
  qa.aux = z_[i].ptr;
  qa.aux_stride = z_[i].stride;
  qa.hbuf = net_[i].ptr;
  qa.h_stride = net_[i].stride;
  gq_[i].launch(s, qa);
}

static void check(int rc, const char* what) { SA_REQUIRE(rc == 0, "%s failed (rc=%d)", what, rc); }

void RaftStereo::forward(hipStream_t s) {
  const int Bn = B();
  const int hd = rc_.hidden;
  const bool par0 = par_ && !tuning_pass_;
  // SA_RAFT_EARLY_FORK=1: the two encoder branches fork before the preprocessing (each preprocesses what it reads),
  // so neither waits on a node of the other's queue
  const bool early = early_fork_ && par0 && !rc_.shared;
  hipStream_t fs_early = early ? fork(s) : nullptr;
  hipStream_t sf = early ? fs_early : s;
  sp_.zero(sf);
  // preprocess: left images -> img[0:B], right -> img[B:2B], 2*(x/255)-1, RGB, 8-ch padded
  check(sa_preprocess(in_left_, Bn, H(), W(), SA_PRE_SIGNED, img_.ptr, 8, 0, 8, sf), "preprocess");
  check(sa_preprocess(in_right_, Bn, H(), W(), SA_PRE_SIGNED, img_.slice_n(Bn, Bn).ptr, 8, 0, 8, sf), "preprocess");
  if (early) check(sa_preprocess(in_left_, Bn, H(), W(), SA_PRE_SIGNED, imgc_.ptr, 8, 0, 8, s), "preprocess");

  // encoders.  The feature branch (fnet -> fmap -> correlation pyramid) and the context branch
  // (cnet -> levels -> heads) are independent after the shared trunk: parallel graph branches.
  const int h0 = lh_[0], w0 = lw_[0];
  const bool par = par_ && !tuning_pass_;
  auto feature_branch = [&](hipStream_t fs) {
    ScopedSplitK sk2(par ? &splitk_side_ : current_splitk());
    if (rc_.shared) {
      shared_rb_.run(fs, sp_, cnet_.out());
      shared_conv_.run(fs, {shared_rb_.out}, fmap_);
    } else {
      fnet_.run(fs, sp_, img_);
      fconv2_.run(fs, {fnet_.out()}, fmap_);
    }
    check(sa_corr1d_pyramid(fmap_.ptr, fmap_.slice_n(Bn, Bn).ptr, 256, Bn, h0, w0, w0, 256, rc_.levels, pyr_, fs),
          "corr pyramid");
  };
  if (rc_.shared) cnet_.run(s, sp_, img_);  // shared trunk on both images
  // SA_RAFT_CNET_FIRST=1: capture the context trunk's first node before the feature branch's (the graph executor keeps
  // a node's first child on the parent's queue), so the two trunks' queue assignment swaps.  Default: on for the
  // realtime preset only (same-process A/B b1: realtime 1.884 -> 1.864 ms, sceneflow 8.50 -> 8.63 ms)
  const bool cnet_first = cnet_first_mode_ >= 0 ? cnet_first_mode_ != 0 : rc_.slow_fast;
  if (cnet_first && par && !rc_.shared && !early) {
    hipStream_t fs = fork(s);
    cnet_.run(s, sp_, img_.slice_n(0, Bn));
    feature_branch(fs);
  } else if (early) {
    // the two trunks' launches interleaved layer by layer in capture order: the graph's host-side enqueue follows
    // it, and a branch captured whole after the other one started ~0.8 ms late (timeline_r5_sf)
    // (with SA_RAFT_CNET_FIRST=1 the context trunk's layer goes first in each pair; it reads imgc_, preprocessed on
    // its own queue, never img_, which the feature queue writes)
    const int n = std::max(fnet_.steps(), cnet_.steps());
    for (int k = 0; k < n; ++k) {
      if (cnet_first && k < cnet_.steps()) cnet_.run_step(s, sp_, imgc_, k);
      if (k < fnet_.steps()) {
        ScopedSplitK sk2(&splitk_side_);
        fnet_.run_step(fs_early, sp_, img_, k);
      }
      if (!cnet_first && k < cnet_.steps()) cnet_.run_step(s, sp_, imgc_, k);
    }
    ScopedSplitK sk2(&splitk_side_);
    fconv2_.run(fs_early, {fnet_.out()}, fmap_);
    check(sa_corr1d_pyramid(fmap_.ptr, fmap_.slice_n(Bn, Bn).ptr, 256, Bn, h0, w0, w0, 256, rc_.levels, pyr_,
                            fs_early),
          "corr pyramid");
  } else {
    feature_branch(par ? fork(s) : s);
    if (!rc_.shared) cnet_.run(s, sp_, img_.slice_n(0, Bn));
  }
  Tensor x = cnet_.out().slice_n(0, Bn);
  Tensor lvl_in[3];
  lvl_in[0] = x;
  auto heads = [&](hipStream_t st, int i) {  // hidden state, context and its z/r/q biases of level i
    Tensor hin[2] = {lvl_in[i], lvl_in[i]};
    if (i < 2) {
      head_rb_[i][0].run(st, sp_, lvl_in[i]);
      head_rb_[i][1].run(st, sp_, lvl_in[i]);
      hin[0] = head_rb_[i][0].out;
      hin[1] = head_rb_[i][1].out;
    }
    head_conv_[i][0].run(st, {hin[0]}, net_[i], SA_ACT_TANH);
    head_conv_[i][1].run(st, {hin[1]}, ctxh_[i], SA_ACT_RELU);
    zqr_[i].run(st, {ctxh_[i]}, czrq_[i]);
  };
  // The context heads of the finer levels only need their level's input: at batch 1 their ~15 small convs
  // (38-150 workgroups each) are latency-bound, so they run on side2 beside the coarser trunk layers
  // (level 0 after the trunk, level 1 after layer4; main: layer4, layer5, level-2 heads).  Events 5-7.
  const bool par_heads = par && rc_.n_gru >= 2;
  if (par_heads) rec(s, 5);
  if (par_heads) {
    ScopedSplitK k2(&splitk_side2_);
    wait(side2_, 5);
    heads(side2_, 0);
  }
  if (rc_.n_gru >= 2) {
    layer4_[0].run(s, sp_, x);
    layer4_[1].run(s, sp_, layer4_[0].out);
    lvl_in[1] = layer4_[1].out;
  }
  if (par_heads) {
    rec(s, 6);
    ScopedSplitK k2(&splitk_side2_);
    wait(side2_, 6);
    heads(side2_, 1);
    rec(side2_, 7);
  }
  if (rc_.n_gru >= 3) {
    layer5_[0].run(s, sp_, lvl_in[1]);
    layer5_[1].run(s, sp_, layer5_[0].out);
    lvl_in[2] = layer5_[1].out;
  }
  for (int i = par_heads ? 2 : 0; i < rc_.n_gru; ++i) heads(s, i);
  if (par_heads) wait(s, 7);
  if (par) join(s);
  flow_cur_ = 0;
  flow_pending_ = false;
  device_zero(flow_(), (size_t)Bn * h0 * w0 * 4, s);
  stage(s, "encoders+corr");

  auto pool = [&](hipStream_t st, int i) {  // pool_[i] = pool2x(net[i])
    check(sa_avgpool3s2(net_[i].ptr, net_[i].stride, pool_[i].ptr, pool_[i].stride, Bn, lh_[i],
                        lw_[i], hd, st),
          "pool2x");
  };
  auto interp = [&](hipStream_t st, int i) {  // interp_[i] = interp(net[i+1], net[i])
    check(sa_interp_bilinear(net_[i + 1].ptr, net_[i + 1].stride, interp_[i].ptr, interp_[i].stride,
                             Bn, lh_[i + 1], lw_[i + 1], hd, lh_[i], lw_[i], 1, 1.f, st),
          "interp");
  };
  auto gru32 = [&](hipStream_t st) {
    pool(st, 1);
    gru(st, 2, {pool_[1]});
  };
  auto gru16 = [&](hipStream_t st) {
    if (rc_.n_gru == 3) {
      // pool2x(net[0]) and interp(net[2]) as one launch (disjoint block ranges)
      check(sa_pool_interp(net_[0].ptr, net_[0].stride, pool_[0].ptr, pool_[0].stride, Bn, lh_[0], lw_[0], hd,
                           net_[2].ptr, net_[2].stride, interp_[1].ptr, interp_[1].stride, Bn, lh_[2], lw_[2], hd,
                           lh_[1], lw_[1], 1, 1.f, st),
            "pool2x + interp");
      gru(st, 1, {pool_[0], interp_[1]});
    } else {
      pool(st, 0);
      gru(st, 1, {pool_[0]});
    }
  };
  // motion encoder: lookup -> convc1/convf1 -> convc2/convf2 -> conv (+ [flow, 0] tail)
  // fused by default at every size: round 3 measured the realtime preset's 1/8 grid at batch 1 (40 tiles) a little
  // faster unfused (2.39 vs 2.41 ms); with round 4's motion-encoder kernel the fused path wins there too (1.961 ->
  // 1.838 ms network, tools/ab_engine.py, profiles/round4_notes.md)
  const bool menc = fuse_motion_ && fuse_menc_ && (fuse_menc_mode_ >= 0 ? fuse_menc_mode_ != 0 : true);
  auto motion = [&](hipStream_t ms) {
    const bool pend = flow_pending_;
    flow_pending_ = false;
    if (pend && !menc) {  // unfused motion encoder: the pending stencil as its own launch first
      check(sa_tapproj_stencil(fhP_, 9, 1, fh2_b_, flow_(), Bn, h0, w0, ms), "flow-head tap stencil");
    }
    if (menc) {
      const SaConvArgs c2 = convc2_.args({cor1_}, corflo_.slice_c(0, 64));
      const SaConvArgs f2 = convf2_.args({flo1_}, corflo_.slice_c(64, 64));
      const SaConvArgs m3 = mconv_.args({corflo_}, motion_.slice_c(0, 126));
      SA_REQUIRE(c2.Kpad == 576 && f2.Kpad == 576 && m3.Kpad == 1152 && motion_.stride >= 128,
                 "fused motion encoder layout (Kpad %d/%d/%d)", c2.Kpad, f2.Kpad, m3.Kpad);
      float* fin = flow_();
      float* fout = nullptr;
      if (pend) {  // flow(t) = flow(t-1) + the previous head's stencil, written to the other buffer by this kernel
        flow_cur_ ^= 1;
        fout = flow_();
      }
      check(sa_raft_motion_encoder_proj(pyr_, fin, Bn, h0, w0, w0, rc_.levels, rc_.radius, me_w1_, me_b1_, c2.weight,
                                        c2.bias, f2.weight, f2.bias, m3.weight, m3.bias, motion_.ptr, motion_.stride,
                                        pend ? fhP_ : nullptr, pend ? fh2_b_ : nullptr, fout, ms),
            "motion encoder");
      return;
    }
    if (fuse_motion_) {
      check(sa_raft_motion_head(pyr_, flow_(), Bn, h0, w0, w0, rc_.levels, rc_.radius, mh_wc_, mh_bc_, mh_wf_,
                                mh_bf_, cor1_.ptr, cor1_.stride, flo1_.ptr, flo1_.stride,
                                motion_.slice_c(126, 2).ptr, motion_.stride, ms),
            "motion head");
    } else {
      check(sa_corr1d_lookup(pyr_, flow_(), Bn, h0, w0, w0, rc_.levels, rc_.radius, corr_feat_.ptr,
                             corr_feat_.stride, corr_feat_.c, flow_feat_.ptr, flow_feat_.stride, 8,
                             motion_.slice_c(126, 2).ptr, motion_.stride, ms),
            "corr lookup");
      convc1_.run(ms, {corr_feat_}, cor1_, SA_ACT_RELU);
      convf1_.run(ms, {flow_feat_}, flo1_, SA_ACT_RELU);
    }
    convc2_.run(ms, {cor1_}, corflo_.slice_c(0, 64), SA_ACT_RELU);
    convf2_.run(ms, {flo1_}, corflo_.slice_c(64, 64), SA_ACT_RELU);
    mconv_.run(ms, {corflo_}, motion_.slice_c(0, 126), SA_ACT_RELU);
  };
  // flow head: conv1 (+ the mask head's conv on the last iteration), then conv2's taps + stencil into the flow
  // (x only) in one launch; mask head 1x1 on the last iteration
  auto head = [&](hipStream_t st, bool last) {
    // SA_RAFT_SIDE_MASK bit 3: the flow head's conv1 tuned for co-residency as well (b1 7.960 -> 7.924 ms)
    const int side_mask = std::getenv("SA_RAFT_SIDE_MASK") ? std::atoi(std::getenv("SA_RAFT_SIDE_MASK")) : 15;
    ScopedSideBranch sb(((side_mask >> 3) & 1) && Bn <= 2 && rc_.n_gru == 3 && !rc_.slow_fast);
    // default: the realtime preset (flow head beside the chain) and batch > 2 (round 6: the projection runs on the
    // matrix cores; b8 timeline 941 -> 893 us per iteration, bench-shaped A/B 41.65 -> 41.37 ms); sceneflow at batch 1
    // measured 8.419 (off) vs 8.473 ms (on), so off there (profiles/round6_notes.md)
    const bool fh_proj = fh_proj_env_ >= 0 ? fh_proj_env_ != 0 : ((rc_.n_gru == 2 && rc_.slow_fast) || Bn > 2);
    if (!last && fh_proj) {
      // conv1's output never reaches memory: its epilogue leaves conv2's x-output tap projections per 128-channel
      // n-tile ([2][9] floats per pixel instead of 256 fp16), the stencil sums their 3x3 neighbourhoods into the flow
      const Tensor pt{fhP_, Bn, h0, w0, 18, 18, DT::F32};
      SaConvArgs pa = fh1_.args({net_[0]}, pt);
      pa.epi = SA_EPI_TAPPROJ;
      pa.act = SA_ACT_RELU;
      pa.tapw = fh2_w16_;
      pa.taps = 9;
      fh1_.launch(st, pa);
      // fused: the next motion encoder applies the stencil while it loads the flow (no launch here)
      if (fh_fuse_) flow_pending_ = true;
      else check(sa_tapproj_stencil(fhP_, 9, 1, fh2_b_, flow_(), Bn, h0, w0, st), "flow-head tap stencil");
      return;
    }
    if (last) fh1mask_.run(st, {net_[0]}, fh_, SA_ACT_RELU);
    else fh1_.run(st, {net_[0]}, fh_.slice_c(0, 256), SA_ACT_RELU);
    check(sa_flow_head_tail(fh_.ptr, fh_.stride, 256, fh2_w16_, fh2_b_, flow_(), Bn, h0, w0, st), "flow-head tail");
    if (last) mask2_.run(st, {fh_.slice_c(256, 256)}, mask_);
  };
  // finest GRU + flow head
  auto fine_and_head = [&](bool last, bool head_only = false) {
    if (head_only) {
      // (the finest GRU was enqueued by the caller)
    } else if (rc_.n_gru > 1) {
      interp(s, 0);
      gru(s, 0, {motion_, interp_[0]});
    } else {
      gru(s, 0, {motion_});
    }
    head(s, last);
  };

  const int f = 1 << rc_.n_downsample;
  // 0 = off, 1 = G32 ahead, 2 = G32 + G16 ahead (the default at every batch, profiles/pipeline_b8_r02.txt)
  const int pmode = pipeline_mode_ >= 0 ? pipeline_mode_ : 2;
  SA_REQUIRE(pmode >= 0 && pmode <= 2, "SA_RAFT_PIPELINE=%d (0..2)", pmode);
  const bool pipe = par && pmode > 0 && rc_.n_gru == 3 && !rc_.slow_fast;
  // realtime preset (2 levels, slow-fast): the recurrence G08(t) -> pool -> G16 -> G16 -> interp -> G08(t + 1) stays
  // on the main stream, the flow head and next motion encoder run beside it (side stream), so per iteration only
  // max(G16 chain, flow head + motion encoder) follows G08.  b1 network 2.10 -> 1.92 ms (GRU split on); on unless
  // SA_RAFT_PIPELINE=0.
  const bool rt_pipe = par && pmode > 0 && rc_.n_gru == 2 && rc_.slow_fast;
  // finest GRU (interp + z/r + q) and flow head as two halves, for the deeper pipeline
  auto fine = [&]() {
    interp(s, 0);
    gru(s, 0, {motion_, interp_[0]});
  };
  if (rt_pipe) {
    // the slow-fast update runs the 1/16 GRU twice on the same pooled 1/8 state (net0 is unchanged between the
    // two calls), so the pooling is done once per iteration
    auto g16x2 = [&]() {
      pool(s, 0);
      gru(s, 1, {pool_[0]});
      gru(s, 1, {pool_[0]});
    };
    rec(s, 4);
    {
      ScopedSplitK k1(&splitk_side_);
      wait(side_, 4);
      motion(side_);
      rec(side_, 3);
    }
    g16x2();
    for (int it = 0; it < rc_.iters; ++it) {
      const bool last = it == rc_.iters - 1;
      interp(s, 0);
      wait(s, 3);
      gru(s, 0, {motion_, interp_[0]});
      rec(s, 4);
      if (!last) g16x2();
      {
        ScopedSplitK k1(&splitk_side_);
        wait(side_, 4);
        head(side_, last);
        if (!last) motion(side_);
        rec(side_, last ? 1 : 3);
      }
    }
    wait(s, 1);
  } else if (pipe && pmode == 2 && m2_main_) {
    // Mode 2, chain on one stream.  The batch-1 critical chain is q(t-1) -> FH(t-1) -> M(t) -> G08 z/r(t) -> q(t);
    // the coarse levels and the finest interp run beside it.  Per iteration t:
    //   side2: G32(t); G16(t) once q(t-1) is done; interp(t)           (event 0)
    //   main : M(t); G08(t) once side2's interp(t) is done; FH(t)      (event 4 after the q conv)
    // With M on the main stream the chain carries no cross-stream edge of its own (round 3's layout put M on a third
    // stream: two event edges per iteration, ~12 us each on the timeline, and the interp on the chain); side2 ends
    // before M does, so the one join (event 0) is normally already signalled when main reaches it.
    rec(s, 4);
    wait(side2_, 4);  // the first G32 reads the encoders' hidden states / context
    for (int it = 0; it < rc_.iters; ++it) {
      const bool last = it == rc_.iters - 1;
      {
        ScopedSplitK k2(&splitk_side2_);
        gru32(side2_);
        wait(side2_, 4);
        gru16(side2_);
        interp(side2_, 0);
        rec(side2_, 0);
      }
      motion(s);
      wait(s, 0);
      gru(s, 0, {motion_, interp_[0]});
      rec(s, 4);
      head(s, last);
    }
  } else if (pipe && pmode == 2) {
    // Deeper cross-iteration pipeline (sceneflow, every batch).  Per iteration t:
    //   side2: G32(t); then G16(t) once the finest q conv of t-1 is done (needs net0(t-1); the finest
    //          interp of t-1, the last reader of net1(t-1), ran before it)
    //   side : M(t) after FH(t-1) (needs flow(t-1); overwrites motion read by G08(t-1))
    //   main : G08(t) after G16(t) and M(t); FH(t)
    // so G16(t + 1) overlaps FH(t) + M(t + 1) instead of following them.  G32 and G16 share the side2
    // split-K workspace (same stream).  Events: 0 = G16 done, 1 = FH done, 3 = M done, 4 = G08 q done.
    rec(s, 1);
    rec(s, 4);
    rec(s, 0);
    wait(side2_, 0);  // the first G32 reads the encoders' hidden states / context
    for (int it = 0; it < rc_.iters; ++it) {
      {
        ScopedSplitK k2(&splitk_side2_);
        gru32(side2_);
        wait(side2_, 4);
        gru16(side2_);
        rec(side2_, 0);
      }
      {
        ScopedSplitK k1(&splitk_side_);
        wait(side_, 1);
        motion(side_);
        rec(side_, 3);
      }
      wait(s, 0);
      wait(s, 3);
      fine();
      rec(s, 4);
      fine_and_head(it == rc_.iters - 1, true);
      rec(s, 1);
    }
  } else if (pipe) {
    // Cross-iteration pipeline on three streams (sceneflow: 3 levels, no slow-fast).  Per iteration t:
    //   side2: G32(t)  after G16(t-1)   (needs net1(t-1), net2(t-1); overwrites net2 read by G16(t-1))
    //   side : M(t)    after FH(t-1)    (needs flow(t-1); overwrites motion read by G08(t-1))
    //   main : G16(t) after G32(t); G08(t) + FH(t) after M(t)
    // so G32(t) overlaps G08(t-1) + FH(t-1), and M(t) overlaps G16(t).  Events (latest record binds):
    //   0 = G16 done, 1 = FH done, 2 = G32 done, 3 = M done.
    rec(s, 0);
    rec(s, 1);
    for (int it = 0; it < rc_.iters; ++it) {
      {
        ScopedSplitK k2(&splitk_side2_);
        wait(side2_, 0);
        gru32(side2_);
        rec(side2_, 2);
      }
      {
        ScopedSplitK k1(&splitk_side_);
        wait(side_, 1);
        motion(side_);
        rec(side_, 3);
      }
      wait(s, 2);
      gru16(s);
      rec(s, 0);
      wait(s, 3);
      fine_and_head(it == rc_.iters - 1);
      rec(s, 1);
    }
  } else {
    for (int it = 0; it < rc_.iters; ++it) {
      // The motion encoder depends only on the correlation pyramid and the flow, the coarse GRU
      // levels only on the hidden states: two parallel branches that join before the finest GRU.
      hipStream_t ms = par ? fork(s) : s;
      {
        ScopedSplitK sk2(par ? &splitk_side_ : current_splitk());
        motion(ms);
      }
      if (rc_.n_gru == 3 && rc_.slow_fast) gru32(s);
      if (rc_.n_gru >= 2 && rc_.slow_fast) {
        if (rc_.n_gru == 3) gru32(s);
        gru16(s);
      }
      if (rc_.n_gru == 3) gru32(s);
      if (rc_.n_gru >= 2) gru16(s);
      if (par) join(s);
      fine_and_head(it == rc_.iters - 1);
    }
  }
  stage(s, "gru_iterations");
  // convex upsampling; disparity = -flow_up
  SA_REQUIRE(!flow_pending_, "flow-head stencil left pending after the last iteration");
  check(sa_convex_upsample(mask_.ptr, mask_.stride, flow_(), Bn, h0, w0, f, -1.f, disp_, s),
        "convex upsample");
  (void)hd;
}

}  // namespace

std::unique_ptr<StereoEngine> make_raft_stereo(const EngineConfig& cfg) {
  return std::unique_ptr<StereoEngine>(new RaftStereo(cfg));
}

}  // namespace sa
