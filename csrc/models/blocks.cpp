#include "blocks.h"

namespace sa {

Norm parse_norm(const std::string& s) {
  if (s == "batch") return Norm::Batch;
  if (s == "instance") return Norm::Instance;
  if (s == "none" || s.empty()) return Norm::None;
  throw Error("unsupported norm " + s);
}

void instnorm(hipStream_t s, const Tensor& x, const sa_stat_t* stats, const Tensor& out, int act,
              const Tensor* res, const sa_stat_t* res_stats, int act2, int res_act) {
  // the apply kernel folds the conv epilogues' kStatSlots statistic copies itself (per block, into LDS)
  SaNormArgs a{};
  a.stat_slots = kStatSlots;
  a.x = x.ptr;
  a.x_stride = x.stride;
  a.stats = stats;
  a.res = res ? res->ptr : nullptr;
  a.res_stride = res ? res->stride : 0;
  a.res_stats = res_stats;
  a.out = out.ptr;
  a.out_stride = out.stride;
  a.N = x.n;
  a.HW = x.h * x.w;
  a.C = x.c;
  a.act = act;
  a.act2 = act2;
  a.res_act = res_act;
  a.eps = 1e-5f;
  a.alpha = 0.01f;
  const int rc = sa_instnorm_apply(&a, s);
  SA_REQUIRE(rc == 0, "instnorm failed");
  SA_LAUNCH_CHECK(s);
}

// The instance-norm blocks of the 64-channel full-resolution layer materialised relu(IN(conv1)) before conv2 (and
// relu(IN(stem)) before layer1).  With SA_FOLD_IN the direct conv (conv_direct.hip, NIN) reads
// the raw tensor and normalises its own DMA'd pieces in LDS one tile ahead, and the residual apply normalises the raw
// block input itself: 3 of the 5 full-resolution apply passes of a RAFT / CREStereo feature trunk are gone.  Round
// 2's version (a serial in-LDS phase between two extra barriers of the round-2 kernel) measured neutral
// (profiles/fused_input_norm_r02.txt).
bool fold_in_enabled() {  // read per engine build: an in-process A/B knob (tools/ab_engine.py)
  const char* e = std::getenv("SA_FOLD_IN");
  return !(e && e[0] == '0');
}

void ResBlock::build(DeviceArena& a, WeightSource& src, StatsPool& sp, const std::string& p,
                     int in_planes, int planes, int stride, Norm nrm, int N, int H, int W, ActPlan* plan,
                     const Tensor* x) {
  norm = nrm;
  has_down = !(stride == 1 && in_planes == planes);
  src.conv(p + ".conv1", planes, in_planes, 3, 3);
  src.conv(p + ".conv2", planes, planes, 3, 3);
  if (has_down) src.conv(p + ".downsample.0", planes, in_planes, 1, 1);
  const bool bn = norm == Norm::Batch;
  if (bn) {
    src.bn(p + ".norm1", planes);
    src.bn(p + ".norm2", planes);
    if (has_down) src.bn(p + ".norm3", planes);
  }
  const WeightStore& ws = *src.ws;
  ConvSpec s3;
  s3.sh = s3.sw = stride;
  c1.build(a, ws, {p + ".conv1"}, {{in_planes, in_planes}}, s3, bn ? std::vector<std::string>{p + ".norm1"} : std::vector<std::string>{});
  ConvSpec s1;
  c2.build(a, ws, {p + ".conv2"}, {{planes, planes}}, s1, bn ? std::vector<std::string>{p + ".norm2"} : std::vector<std::string>{});
  if (has_down) {
    ConvSpec sd;
    sd.sh = sd.sw = stride;
    sd.ph = sd.pw = 0;
    down.build(a, ws, {p + ".downsample.0"}, {{in_planes, in_planes}}, sd,
               bn ? std::vector<std::string>{p + ".norm3"} : std::vector<std::string>{});
  }
  const int Ho = c1.out_h(H), Wo = c1.out_w(W);
  // the direct kernel's shape (sa_conv2d tile_cfg 23): 64 -> 64, 3x3, stride 1, 32-bit buffer offsets
  fold = norm == Norm::Instance && !has_down && planes == 64 && fold_in_enabled() &&
         (size_t)N * Ho * Wo * 64 * 2 < 0xFFFFFF00ull;
  SA_REQUIRE(!x_raw || fold, "ResBlock: a raw (un-normalised) input needs the folded instance norm");
  if (norm == Norm::Instance) {
    st1 = sp.take(N, planes);
    st2 = sp.take(N, planes);
    if (has_down) std_ = sp.take(N, planes);
  }
  if (plan) {
    // lifetimes in run() order (see below); x is the block input (tracked only if the plan owns it)
    if (norm == Norm::Instance && fold) {
      plan->use(x), plan->def(&y1, N, Ho, Wo, planes), plan->next();                   // c1(x) -> y1
      plan->use(&y1), plan->def(&y2, N, Ho, Wo, planes), plan->next();                 // c2(relu(IN(y1))) -> y2
      plan->use(&y2), plan->use(x), plan->def(&out, N, Ho, Wo, planes), plan->next();
    } else if (norm == Norm::Instance) {
      plan->use(x), plan->def(&y1, N, Ho, Wo, planes), plan->next();                   // c1(x) -> y1
      plan->use(&y1), plan->def(&a1, N, Ho, Wo, planes), plan->next();                 // IN -> a1
      plan->use(&a1), plan->def(&y2, N, Ho, Wo, planes), plan->next();                 // c2(a1) -> y2
      if (has_down) plan->use(x), plan->def(&yd, N, Ho, Wo, planes), plan->next();     // down(x) -> yd
      plan->use(&y2), plan->use(has_down ? &yd : x), plan->def(&out, N, Ho, Wo, planes), plan->next();
    } else {
      plan->use(x), plan->def(&a1, N, Ho, Wo, planes), plan->next();                   // c1(x) -> a1
      if (has_down) plan->use(x), plan->def(&yd, N, Ho, Wo, planes), plan->next();     // down(x) -> yd
      plan->use(&a1), plan->use(has_down ? &yd : x), plan->def(&out, N, Ho, Wo, planes), plan->next();
    }
    return;
  }
  if (norm == Norm::Instance) {
    y1 = make_tensor(a, N, Ho, Wo, planes);
    y2 = make_tensor(a, N, Ho, Wo, planes);
  }
  if (!fold) a1 = make_tensor(a, N, Ho, Wo, planes);
  if (has_down) yd = make_tensor(a, N, Ho, Wo, planes);
  out = make_tensor(a, N, Ho, Wo, planes);
}


void ResBlock::run(hipStream_t s, const StatsPool& sp, const Tensor& x, const sa_stat_t* x_stats) const {
  SA_REQUIRE(x_raw == (x_stats != nullptr), "ResBlock: raw input without its statistics (or the reverse)");
  if (norm == Norm::Instance && fold) {
    c1.run(s, {x}, y1, SA_ACT_NONE, nullptr, SA_ACT_NONE, sp.resolve(st1), 0.01f, x_stats);
    c2.run(s, {y1}, y2, SA_ACT_NONE, nullptr, SA_ACT_NONE, sp.resolve(st2), 0.01f, sp.resolve(st1));
    instnorm(s, y2, sp.resolve(st2), out, SA_ACT_RELU, &x, x_stats, SA_ACT_RELU, x_stats ? SA_ACT_RELU : SA_ACT_NONE);
  } else if (norm == Norm::Instance) {
    c1.run(s, {x}, y1, SA_ACT_NONE, nullptr, SA_ACT_NONE, sp.resolve(st1));
    instnorm(s, y1, sp.resolve(st1), a1, SA_ACT_RELU);
    c2.run(s, {a1}, y2, SA_ACT_NONE, nullptr, SA_ACT_NONE, sp.resolve(st2));
    if (has_down) {
      down.run(s, {x}, yd, SA_ACT_NONE, nullptr, SA_ACT_NONE, sp.resolve(std_));
      instnorm(s, y2, sp.resolve(st2), out, SA_ACT_RELU, &yd, sp.resolve(std_), SA_ACT_RELU);
    } else {
      instnorm(s, y2, sp.resolve(st2), out, SA_ACT_RELU, &x, nullptr, SA_ACT_RELU);
    }
  } else {
    c1.run(s, {x}, a1, SA_ACT_RELU);
    if (has_down) {
      down.run(s, {x}, yd, SA_ACT_NONE);
      c2.run(s, {a1}, out, SA_ACT_RELU, &yd, SA_ACT_RELU);
    } else {
      c2.run(s, {a1}, out, SA_ACT_RELU, &x, SA_ACT_RELU);
    }
  }
}

void Trunk::build(DeviceArena& a, WeightSource& src, StatsPool& sp, const std::string& p, Norm nrm, int N, int H,
                  int W, int s1, const int strides[3]) {
  norm = nrm;
  src.conv(p + ".conv1", 64, 3, 7, 7);
  if (norm == Norm::Batch) src.bn(p + ".norm1", 64);
  ConvSpec sp7;
  sp7.sh = sp7.sw = s1;
  conv1.build(a, *src.ws, {p + ".conv1"}, {{3, 8}}, sp7,
              norm == Norm::Batch ? std::vector<std::string>{p + ".norm1"} : std::vector<std::string>{});
  int h = conv1.out_h(H), w = conv1.out_w(W);
  // the trunk's activations go through a liveness plan: at most ~3 full-resolution tensors are alive
  // at once (batch 8 RAFT-Stereo sceneflow: several GB less than one buffer per tensor)
  ActPlan plan;
  // stem fold: layer1.0 is a 64 -> 64 stride-1 block whose conv1 and residual normalise c1y themselves
  stem_fold = norm == Norm::Instance && fold_in_enabled() && strides[0] == 1 &&
              (size_t)N * h * w * 64 * 2 < 0xFFFFFF00ull;
  if (norm == Norm::Instance && stem_fold) {
    c1st = sp.take(N, 64);
    plan.def(&c1y, N, h, w, 64), plan.next();                      // conv1(img) -> c1y (raw)
  } else if (norm == Norm::Instance) {
    c1st = sp.take(N, 64);
    plan.def(&c1y, N, h, w, 64), plan.next();                      // conv1(img) -> c1y
    plan.use(&c1y), plan.def(&c1a, N, h, w, 64), plan.next();      // IN -> c1a
  } else {
    plan.def(&c1a, N, h, w, 64), plan.next();                      // conv1(img) -> c1a
  }
  const int dims[3] = {64, 96, 128};
  int inp = 64;
  layers.resize(6);  // sized up front: the plan holds pointers into the blocks
  const Tensor* x = stem_fold ? &c1y : &c1a;
  for (int l = 0; l < 3; ++l)
    for (int b = 0; b < 2; ++b) {
      ResBlock& rb = layers[l * 2 + b];
      rb.x_raw = stem_fold && l == 0 && b == 0;
      rb.build(a, src, sp, p + ".layer" + std::to_string(l + 1) + "." + std::to_string(b), inp, dims[l],
               b == 0 ? strides[l] : 1, norm, N, h, w, &plan, x);
      x = &rb.out;
      h = rb.out.h;
      w = rb.out.w;
      inp = dims[l];
    }
  plan.keep(&layers.back().out);
  plan.commit(a);
}

void Trunk::run_step(hipStream_t s, const StatsPool& sp, const Tensor& img, int k) const {
  if (k == 0) {
    if (norm == Norm::Instance) {
      conv1.run(s, {img}, c1y, SA_ACT_NONE, nullptr, SA_ACT_NONE, sp.resolve(c1st));
      if (!stem_fold) instnorm(s, c1y, sp.resolve(c1st), c1a, SA_ACT_RELU);
    } else {
      conv1.run(s, {img}, c1a, SA_ACT_RELU);
    }
    return;
  }
  if (k == 1 && stem_fold) {
    layers[0].run(s, sp, c1y, sp.resolve(c1st));
    return;
  }
  layers[k - 1].run(s, sp, k == 1 ? c1a : layers[k - 2].out);
}

void Trunk::run(hipStream_t s, const StatsPool& sp, const Tensor& img) const {
  for (int k = 0; k < steps(); ++k) run_step(s, sp, img, k);
}

}  // namespace sa
