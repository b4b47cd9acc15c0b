// HITNet (presets hitnet-d400, hitnet-xl) as a native op graph.
//
// Reference pins: one 6-channel input = [L RGB; R RGB] / 255
// (HitNet/src/HitNet_preprocess.cu:19-51, HitNet.cpp:78), output H*W positive disparity
// (HitNet.cpp:15-17); export middlebury_d400 (HitNet/test/main.cpp:9).  Network and parameter names:
// stereoalgorithms_amd/models/hitnet.py (the oracle).
//
// Layout: both images run the U-Net as one 2B batch (NHWC fp16, every conv an MFMA implicit GEMM with
// fused bias + LeakyReLU(0.2); the 2x2 transposed convs are 1x1 convs whose epilogue scatters the 4
// parity classes).  Tile hypotheses are fp32; each update network sees [local cost | fp16 hypothesis
// copy] of all its candidates side by side as one multi-candidate source written by the warp kernel
// (joint update, per-candidate deltas + confidences, argmax selection); the level-0 winner is then split
// into 2x2 and 1x1 tiles and refined twice more on the full-resolution features.
#include "blocks.h"

namespace sa {
namespace {

constexpr int kLevels = 5, kHypLevels = 4;
constexpr float kSlope = 0.2f;

// Presets (stereoalgorithms_amd/models/hitnet.py PRESETS; the oracle's docstring lists which numbers the
// published description fixes and which are our choices)
struct HitCfg {
  int maxdisp;
  int ch[kLevels];
  int width;                 // level update networks
  std::vector<int> dils;     // residual-block dilations of the level update networks
  int rwidth[2];             // final refinement (2x2 tiles, 1x1 tiles)
  std::vector<int> rdils[2];
};

HitCfg preset(const std::string& name) {
  if (name == "hitnet-d400" || name == "hitnet") return HitCfg{400, {16, 16, 24, 24, 32}, 32, {1, 2, 4}, {32, 16}, {{1, 2}, {1, 1}}};
  if (name == "hitnet-xl") return HitCfg{320, {32, 32, 48, 48, 64}, 64, {1, 2, 4, 8, 1}, {48, 24}, {{1, 2}, {1, 1}}};
  throw Error("unknown HITNet preset " + name);
}

static void check(int rc, const char* what) { SA_REQUIRE(rc == 0, "%s failed (rc=%d)", what, rc); }

ConvSpec spec(int k, int s = 1, int pad = -1, int dil = 1) {
  ConvSpec sp;
  sp.kh = sp.kw = k;
  sp.sh = sp.sw = s;
  sp.ph = sp.pw = pad;
  sp.dh = sp.dw = dil;
  return sp;
}

// Joint update of ncand hypotheses of tile size t (oracle: hitnet.UpdateNet): x = [cost_k (3t^2), h_k (16)]
// per candidate k (each block padded to 8 channels) -> 1x1 conv -> residual blocks -> 3x3 conv -> per
// candidate 16 deltas (+ a confidence when conf).
struct UpdateNet {
  int t = 4, ncand = 1, nout = 17, cin = 64, cin_pad = 64;
  ConvLayer inp, out;
  std::vector<ConvLayer> c1, c2;
  std::vector<int> dils;
  Tensor x, a, b, c, delta;
  void build(DeviceArena& ar, WeightSource& src, const std::string& p, int t_, int ncand_, int width,
             const std::vector<int>& dils_, bool conf, int N, int th, int tw) {
    t = t_;
    ncand = ncand_;
    nout = conf ? 17 : 16;
    cin = 3 * t * t + 16;
    cin_pad = round_up(cin, 8);
    dils = dils_;
    src.conv(p + ".inp", width, ncand * cin, 1, 1);
    std::vector<ChanSeg> segs(ncand, ChanSeg{cin, cin_pad});
    inp.build(ar, *src.ws, {p + ".inp"}, segs, spec(1, 1, 0));
    c1.resize(dils.size());
    c2.resize(dils.size());
    for (size_t i = 0; i < dils.size(); ++i) {
      const std::string n = p + ".res." + std::to_string(i) + ".conv";
      src.conv(n + "1", width, width, 3, 3);
      src.conv(n + "2", width, width, 3, 3);
      c1[i].build(ar, *src.ws, {n + "1"}, {{width, width}}, spec(3, 1, -1, dils[i]));
      c2[i].build(ar, *src.ws, {n + "2"}, {{width, width}}, spec(3, 1, -1, dils[i]));
    }
    src.conv(p + ".out", ncand * nout, width, 3, 3);
    out.build(ar, *src.ws, {p + ".out"}, {{width, width}}, spec(3));
    x = make_tensor(ar, N, th, tw, ncand * cin_pad);
    a = make_tensor(ar, N, th, tw, width);
    b = make_tensor(ar, N, th, tw, width);
    c = make_tensor(ar, N, th, tw, width);
    delta = make_tensor(ar, N, th, tw, ncand * nout, DT::F32, round_up(ncand * nout, 8));
  }
  void run(hipStream_t s) const {
    inp.run(s, {x}, a, SA_ACT_LEAKY, nullptr, SA_ACT_NONE, nullptr, kSlope);
    const Tensor* cur = &a;
    const Tensor* nxt = &c;
    for (size_t i = 0; i < dils.size(); ++i) {
      c1[i].run(s, {*cur}, b, SA_ACT_LEAKY, nullptr, SA_ACT_NONE, nullptr, kSlope);
      c2[i].run(s, {b}, *nxt, SA_ACT_NONE, cur, SA_ACT_LEAKY, nullptr, kSlope);
      std::swap(cur, nxt);
    }
    out.run(s, {*cur}, delta);
  }
};

class HitNet : public StereoEngine {
 public:
  explicit HitNet(const EngineConfig& cfg) : StereoEngine(cfg), hc_(preset(cfg.model)) {}
  const char* name() const override { return "HitNet"; }

 protected:
  void build(WeightSource& src) override;
  void forward(hipStream_t s) override;

 private:
  HitCfg hc_;
  // two-chain schedule (forward): SA_HIT_PARALLEL=0 keeps everything on one stream
  bool par_ = !(std::getenv("SA_HIT_PARALLEL") && std::getenv("SA_HIT_PARALLEL")[0] == '0');
  void init_level(hipStream_t s, int l);
  void prop_level(hipStream_t s, int l);
  Tensor img_;
  std::vector<ConvLayer> down_[kLevels];
  std::vector<Tensor> dt_[kLevels];  // per-conv outputs of the down path (last = d_l)
  ConvLayer up_deconv_[4], up_merge_[4], up_conv_[4];
  Tensor up_t_[4], up_m_[4], e_[kLevels];  // e_[4] aliases the last down output
  struct Lvl {
    ConvLayer tile_l, tile_r, desc;
    Tensor tl, tr, cmin, dsc;
    float* dinit = nullptr;
    float* cand = nullptr;  // [ncand][B][th][tw][16]
    float* hyp = nullptr;   // selected [B][th][tw][16]
    int th = 0, tw = 0, wr = 0, ncand = 1;
    UpdateNet prop;
  } lv_[kHypLevels];
  struct Refine {  // final refinement at tile size t (2, then 1) on the level-0 features
    int t = 2, th = 0, tw = 0;
    float* cand = nullptr;  // split of the previous stage's hypotheses [B][th][tw][16]
    float* hyp = nullptr;
    UpdateNet net;
  } rf_[2];
};

void HitNet::build(WeightSource& src) {
  DeviceArena& a = arena_;
  const int B = this->B(), N2 = 2 * B;
  const int* kCh = hc_.ch;
  SA_REQUIRE(H() % 32 == 0 && W() % 32 == 0, "HITNet needs H, W multiples of 32");
  img_ = make_tensor(a, N2, H(), W(), 8);
  // ---- U-Net down path
  int h = H(), w = W();
  for (int l = 0; l < kLevels; ++l) {
    const std::string p = "feature.down." + std::to_string(l) + ".";
    const int nconv = l == 0 ? 2 : 3;
    down_[l].resize(nconv);
    for (int i = 0; i < nconv; ++i) {
      const bool strided = l > 0 && i == 0;
      const int cin = i == 0 ? (l == 0 ? 3 : kCh[l - 1]) : kCh[l];
      const int k = strided ? 2 : 3;
      src.conv(p + std::to_string(i), kCh[l], cin, k, k);
      const std::vector<ChanSeg> segs = {{cin, round_up(cin, 8)}};
      down_[l][i].build(a, *src.ws, {p + std::to_string(i)}, segs, strided ? spec(2, 2, 0) : spec(3));
      if (strided) {
        h /= 2;
        w /= 2;
      }
      dt_[l].push_back(make_tensor(a, N2, h, w, kCh[l]));
    }
  }
  e_[4] = dt_[4].back();
  // ---- U-Net up path
  for (int l = 3; l >= 0; --l) {
    const std::string p = "feature.up." + std::to_string(l) + ".";
    const int c = kCh[l], cin = kCh[l + 1];
    const float bound = 1.f / std::sqrt((float)(c * 4));
    src.param(p + "deconv.weight", {cin, c, 2, 2}, -bound, bound);
    src.param(p + "deconv.bias", {c}, -bound, bound);
    up_deconv_[l].build_deconv(a, *src.ws, p + "deconv", false, {{cin, cin}});
    src.conv(p + "merge", c, 2 * c, 1, 1);
    up_merge_[l].build(a, *src.ws, {p + "merge"}, {{c, c}, {c, c}}, spec(1, 1, 0));
    src.conv(p + "conv", c, c, 3, 3);
    up_conv_[l].build(a, *src.ws, {p + "conv"}, {{c, c}}, spec(3));
    const Tensor& d = dt_[l].back();
    up_t_[l] = make_tensor(a, N2, d.h, d.w, c);
    up_m_[l] = make_tensor(a, N2, d.h, d.w, c);
    e_[l] = make_tensor(a, N2, d.h, d.w, c);
  }
  // ---- tile hypotheses + propagation per level
  for (int l = 0; l < kHypLevels; ++l) {
    Lvl& L = lv_[l];
    const std::string p = "init." + std::to_string(l) + ".";
    const int c = kCh[l], Hl = e_[l].h, Wl = e_[l].w;
    L.th = Hl / 4;
    L.tw = Wl / 4;
    L.wr = Wl - 3;
    L.ncand = l == kHypLevels - 1 ? 1 : 2;
    src.conv(p + "tile", 16, c, 4, 4);
    L.tile_l.build(a, *src.ws, {p + "tile"}, {{c, c}}, spec(4, 4, 0));
    ConvSpec sr = spec(4, 1, 0);
    sr.sh = 4;
    L.tile_r.build(a, *src.ws, {p + "tile"}, {{c, c}}, sr);
    src.conv(p + "desc", 13, 17, 1, 1);
    L.desc.build(a, *src.ws, {p + "desc"}, {{1, 8}, {16, 16}}, spec(1, 1, 0));
    L.tl = make_tensor(a, B, L.th, L.tw, 16);
    L.tr = make_tensor(a, B, L.th, L.wr, 16);
    L.cmin = make_tensor(a, B, L.th, L.tw, 8);
    L.dsc = make_tensor(a, B, L.th, L.tw, 13, DT::F16, 16);
    const size_t P = (size_t)B * L.th * L.tw;
    L.dinit = (float*)a.alloc(P * 4);
    L.cand = (float*)a.alloc(P * L.ncand * 16 * 4);
    L.hyp = (float*)a.alloc(P * 16 * 4);
    L.prop.build(a, src, "prop." + std::to_string(l), 4, L.ncand, hc_.width, hc_.dils, true, B, L.th, L.tw);
  }
  // ---- final refinement: 2x2 tiles (half resolution) then per pixel, on e_0
  for (int j = 0; j < 2; ++j) {
    Refine& R = rf_[j];
    R.t = j == 0 ? 2 : 1;
    R.th = H() / R.t;
    R.tw = W() / R.t;
    const size_t P = (size_t)B * R.th * R.tw;
    R.cand = (float*)a.alloc(P * 16 * 4);
    R.hyp = (float*)a.alloc(P * 16 * 4);
    R.net.build(a, src, "refine." + std::to_string(j), R.t, 1, hc_.rwidth[j], hc_.rdils[j], false, B, R.th, R.tw);
  }
}

// Tile hypotheses of level l from its features alone: tile features, initial matching cost / disparity, descriptor,
// the level's own candidate (last slot of cand)
void HitNet::init_level(hipStream_t s, int l) {
  const int B = this->B();
  Lvl& L = lv_[l];
  const Tensor el = e_[l].slice_n(0, B), er = e_[l].slice_n(B, B);
  const long P = (long)B * L.th * L.tw;
  L.tile_l.run(s, {el}, L.tl);
  L.tile_r.run(s, {er}, L.tr);
  tap(s, ("tl" + std::to_string(l)).c_str(), L.tl);
  tap(s, ("tr" + std::to_string(l)).c_str(), L.tr);
  check(sa_hitnet_tile_init(L.tl.ptr, L.tl.stride, L.tr.ptr, L.tr.stride, B, L.th, L.tw, L.wr, hc_.maxdisp >> l,
                            L.cmin.ptr, L.cmin.stride, L.dinit, s),
        "tile init");
  L.desc.run(s, {L.cmin, L.tl}, L.dsc, SA_ACT_LEAKY, nullptr, SA_ACT_NONE, nullptr, kSlope);
  // own init goes to the last candidate slot; slot 0 = upsampled coarser hypothesis
  float* init_slot = L.cand + (size_t)(L.ncand - 1) * P * 16;
  check(sa_hitnet_hyp_init(L.dinit, L.dsc.ptr, L.dsc.stride, P, init_slot, s), "hyp init");
}

// Propagation of level l: the coarser level's winner upsampled into slot 0, warped costs, update net, selection
void HitNet::prop_level(hipStream_t s, int l) {
  const int B = this->B();
  Lvl& L = lv_[l];
  const Tensor el = e_[l].slice_n(0, B), er = e_[l].slice_n(B, B);
  const long P = (long)B * L.th * L.tw;
  if (L.ncand > 1) {
    const Lvl& C = lv_[l + 1];
    check(sa_hitnet_upsample(C.hyp, B, C.th, C.tw, L.cand, s), "hyp upsample");
  }
  const UpdateNet& U = L.prop;
  check(sa_hitnet_warp_cost(el.ptr, el.stride, er.ptr, er.stride, B, e_[l].h, e_[l].w, hc_.ch[l], 4, L.cand, L.ncand,
                            U.x.ptr, U.x.stride, U.cin_pad, s),
        "warp cost");
  U.run(s);
  check(sa_hitnet_select(L.cand, L.ncand, P, (const float*)U.delta.ptr, U.delta.stride, U.nout, 1, L.hyp, s),
        "select");
  tap_f32(s, ("cand" + std::to_string(l)).c_str(), L.cand, L.ncand * B, L.th, L.tw, 16);
  tap(s, ("cost" + std::to_string(l)).c_str(), U.x);
  tap(s, ("delta" + std::to_string(l)).c_str(), U.delta);
  tap_f32(s, ("hyp" + std::to_string(l)).c_str(), L.hyp, B, L.th, L.tw, 16);
}

// Two chains once the coarsest decoder level exists (b1: every conv of the coarse levels is a 5-75 workgroup,
// latency-bound launch, so a single stream leaves the chip mostly idle):
//   main: decoder levels 2, 1, 0 and, after each, that level's tile init (events 2, 1, 0)
//   side: init + propagation of the coarsest level, then propagation of each finer level once its init is done,
//         the two refinement stages and the final expansion; joined into main at the end
void HitNet::forward(hipStream_t s) {
  const int B = this->B();
  const bool par = par_ && !tuning_pass_;
  check(sa_preprocess(in_left_, B, H(), W(), SA_PRE_UNIT, img_.ptr, 8, 0, 8, s), "preprocess");
  check(sa_preprocess(in_right_, B, H(), W(), SA_PRE_UNIT, img_.slice_n(B, B).ptr, 8, 0, 8, s), "preprocess");
  const Tensor* x = &img_;
  for (int l = 0; l < kLevels; ++l)
    for (size_t i = 0; i < down_[l].size(); ++i) {
      down_[l][i].run(s, {*x}, dt_[l][i], SA_ACT_LEAKY, nullptr, SA_ACT_NONE, nullptr, kSlope);
      x = &dt_[l][i];
    }
  auto up = [&](int l) {
    up_deconv_[l].run(s, {e_[l + 1]}, up_t_[l], SA_ACT_LEAKY, nullptr, SA_ACT_NONE, nullptr, kSlope);
    up_merge_[l].run(s, {up_t_[l], dt_[l].back()}, up_m_[l], SA_ACT_LEAKY, nullptr, SA_ACT_NONE, nullptr, kSlope);
    up_conv_[l].run(s, {up_m_[l]}, e_[l], SA_ACT_LEAKY, nullptr, SA_ACT_NONE, nullptr, kSlope);
    tap(s, ("e" + std::to_string(l)).c_str(), e_[l]);
  };
  tap(s, "e4", e_[4]);
  constexpr int top = kHypLevels - 1;
  for (int l = kLevels - 2; l >= top; --l) up(l);
  hipStream_t hs = s;  // the hypothesis chain
  if (par) {
    hs = fork(s);
    for (int l = top - 1; l >= 0; --l) {
      up(l);
      init_level(s, l);
      rec(s, l);
    }
  }
  {
    ScopedSplitK sk(par ? &splitk_side_ : current_splitk());
    for (int l = top; l >= 0; --l) {
      if (!par && l < top) up(l);
      if (!par || l == top) init_level(hs, l);
      if (par && l < top) wait(hs, l);
      prop_level(hs, l);
    }
    // final refinement on the level-0 (full-resolution) features
    const Tensor e0l = e_[0].slice_n(0, B), e0r = e_[0].slice_n(B, B);
    const float* prev = lv_[0].hyp;
    int pth = lv_[0].th, ptw = lv_[0].tw, pt = 4;
    for (int j = 0; j < 2; ++j) {
      const Refine& R = rf_[j];
      const long P = (long)B * R.th * R.tw;
      check(sa_hitnet_split(prev, B, pth, ptw, pt, R.cand, hs), "hyp split");
      const UpdateNet& U = R.net;
      check(sa_hitnet_warp_cost(e0l.ptr, e0l.stride, e0r.ptr, e0r.stride, B, H(), W(), hc_.ch[0], R.t, R.cand, 1,
                                U.x.ptr, U.x.stride, U.cin_pad, hs),
            "warp cost");
      U.run(hs);
      check(sa_hitnet_select(R.cand, 1, P, (const float*)U.delta.ptr, U.delta.stride, U.nout, 0, R.hyp, hs), "refine");
      tap_f32(hs, ("rcand" + std::to_string(j)).c_str(), R.cand, B, R.th, R.tw, 16);
      tap(hs, ("rcost" + std::to_string(j)).c_str(), U.x);
      tap(hs, ("rdelta" + std::to_string(j)).c_str(), U.delta);
      tap_f32(hs, ("rhyp" + std::to_string(j)).c_str(), R.hyp, B, R.th, R.tw, 16);
      prev = R.hyp;
      pth = R.th;
      ptw = R.tw;
      pt = R.t;
    }
    check(sa_hitnet_expand(prev, B, pth, ptw, 1, disp_, hs), "expand");
  }
  if (par) join(s);
}

}  // namespace

std::unique_ptr<StereoEngine> make_hitnet(const EngineConfig& cfg) {
  return std::unique_ptr<StereoEngine>(new HitNet(cfg));
}

}  // namespace sa
