// StereoEngine base: io buffers, rectification + reprojection around the model forward,
// graph capture, host-side timed path.
#include "sa/engine.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cerrno>
#include <sys/stat.h>

namespace sa {

// ------------------------------------------------------------------ deterministic init
static uint64_t fnv1a(const std::string& s, uint64_t seed) {
  uint64_t h = 1469598103934665603ull ^ (seed * 0x9E3779B97F4A7C15ull);
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

struct SplitMix {
  uint64_t x;
  uint64_t next() {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  float uniform(float lo, float hi) { return lo + (hi - lo) * (float)((next() >> 40) * (1.0 / 16777216.0)); }
};

void WeightSource::param(const std::string& name, std::vector<int64_t> shape, float lo, float hi) {
  if (ws->has(name)) {
    const auto& t = ws->get(name);
    SA_REQUIRE(t.shape == shape, "weight %s has unexpected shape", name.c_str());
    return;
  }
  SA_REQUIRE(random, "missing weight %s", name.c_str());
  HostTensor t;
  t.shape = shape;
  t.data.resize(t.numel());
  SplitMix rng{fnv1a(name, seed)};
  for (auto& v : t.data) v = lo == hi ? lo : rng.uniform(lo, hi);
  ws->put(name, std::move(t));
}

void WeightSource::conv(const std::string& name, int cout, int cin, int kh, int kw, bool bias) {
  float bound = 1.f / std::sqrt((float)(cin * kh * kw));
  param(name + ".weight", {cout, cin, kh, kw}, -bound, bound);
  if (bias) param(name + ".bias", {cout}, -bound, bound);
}

void WeightSource::bn(const std::string& name, int c) {
  param(name + ".weight", {c}, 1.f, 1.f);
  param(name + ".bias", {c}, 0.f, 0.f);
  param(name + ".running_mean", {c}, 0.f, 0.f);
  param(name + ".running_var", {c}, 1.f, 1.f);
}

void WeightSource::linear(const std::string& name, int out, int in, bool bias) {
  float bound = 1.f / std::sqrt((float)in);
  param(name + ".weight", {out, in}, -bound, bound);
  if (bias) param(name + ".bias", {out}, -bound, bound);
}

void WeightSource::ln(const std::string& name, int c) {
  param(name + ".weight", {c}, 1.f, 1.f);
  param(name + ".bias", {c}, 0.f, 0.f);
}

// ------------------------------------------------------------------ engine
StereoEngine::StereoEngine(const EngineConfig& cfg) : cfg_(cfg) {
  for (int i = 0; i < 16; ++i) Q_[i] = 0.f;
}

StereoEngine::~StereoEngine() {
  if (stream_) (void)hipStreamSynchronize(stream_);
  for (int r = 0; r < 4; ++r) unregister_host(r);
  for (GraphExec& g : graph_) g.reset();
  copy_pool_.reset();
  for (auto& e : ev_copy_)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : host_ev_)
    if (e) (void)hipEventDestroy(e);
  if (pin_in_) (void)hipHostFree(pin_in_);
  if (pin_out_) (void)hipHostFree(pin_out_);
  if (ev_in_) (void)hipEventDestroy(ev_in_);
  if (ev_out_) (void)hipEventDestroy(ev_out_);
  if (ev_fork_) (void)hipEventDestroy(ev_fork_);
  if (ev_join_) (void)hipEventDestroy(ev_join_);
  if (side_) {
    // An exported copy stream stays alive: torch's pinned-host allocator records an event on every stream a
    // pinned block was copied on when that block is FREED, which may be long after the engine is gone (a
    // destroyed stream there is a use-after-free at interpreter exit).  One stream per such engine is leaked.
    if (side_exported_) (void)hipStreamSynchronize(side_);
    else (void)hipStreamDestroy(side_);
  }
  if (side2_) (void)hipStreamDestroy(side2_);
  for (hipEvent_t e : ev_dep_)
    if (e) (void)hipEventDestroy(e);

  if (stream_) {
    if (main_exported_) (void)hipStreamSynchronize(stream_);
    else (void)hipStreamDestroy(stream_);
  }
  arena_.release();
}

std::unique_ptr<StereoEngine> StereoEngine::create(const EngineConfig& cfg_in) {
  EngineConfig cfg = cfg_in;
  HIP_CHECK(hipSetDevice(cfg.device));
  std::unique_ptr<WeightStore> store;
  if (!cfg.weights.empty()) {
    store = WeightStore::load_safetensors(cfg.weights);
    if (cfg.model.empty()) cfg.model = store->meta("model");
  } else {
    store = std::make_unique<WeightStore>();
  }
  SA_REQUIRE(!cfg.model.empty(), "no model preset given and none in weights metadata");
  std::unique_ptr<StereoEngine> e;
  const std::string& m = cfg.model;
  if (m.rfind("raftstereo", 0) == 0) e = make_raft_stereo(cfg);
  else if (m.rfind("crestereo", 0) == 0) e = make_crestereo(cfg);
  else if (m.rfind("hitnet", 0) == 0) e = make_hitnet(cfg);
  else if (m.rfind("fastacvnet", 0) == 0) e = make_fast_acvnet(cfg);
  else throw Error("unknown model preset: " + m);
  e->store_ = std::move(store);
  e->init();
  return e;
}

void StereoEngine::init() {
  HIP_CHECK(hipSetDevice(cfg_.device));
  if (const char* e = std::getenv("SA_NO_GRAPH"))
    if (e[0] == '1') cfg_.use_graph = false;  // debugging: eager launches (with SA_DEBUG_SYNC=1)
  // Non-blocking engine stream: every dependency on caller work is explicit (launch_frame records an event
  // on the caller's stream and the engine stream waits on it, and the reverse after the frame), so the frame
  // never implicitly serialises with the legacy null stream.  Round 1 used a blocking stream to dodge replay
  // corruption it could not explain; its cause was the hipMemsetAsync nodes in the frame graph (replays with
  // packet capture on a non-blocking stream diverged, profiles/graph_replay_memset_r02.md).  Frames now zero
  // memory with kernel nodes only (device_zero).  SA_ENGINE_STREAM_BLOCKING=1 restores the blocking stream.
  static const bool blocking = [] {
    const char* e = std::getenv("SA_ENGINE_STREAM_BLOCKING");
    return e && e[0] == '1';
  }();
  HIP_CHECK(hipStreamCreateWithFlags(&stream_, blocking ? hipStreamDefault : hipStreamNonBlocking));
  HIP_CHECK(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
  HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  HIP_CHECK(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
  HIP_CHECK(hipStreamCreateWithFlags(&side2_, hipStreamNonBlocking));
  for (hipEvent_t& e : ev_dep_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (const char* st = std::getenv("SA_STAGE_TIMES")) stage_on_ = st[0] == '1';
  if (stage_on_) stage_ts_ = (unsigned long long*)arena_.alloc(kMaxStages * sizeof(unsigned long long));
  const size_t img = (size_t)B() * H() * W() * 3;
  in_left_ = (uint8_t*)arena_.alloc(img);
  in_right_ = (uint8_t*)arena_.alloc(img);
  raw_left_ = (uint8_t*)arena_.alloc(img);
  raw_right_ = (uint8_t*)arena_.alloc(img);
  disp_ = (float*)arena_.alloc((size_t)B() * H() * W() * 4);
  cloud_ = (float*)arena_.alloc((size_t)B() * H() * W() * 6 * 4);
  HIP_CHECK(hipHostMalloc((void**)&pin_in_, 2 * img, hipHostMallocDefault));
  HIP_CHECK(hipHostMalloc((void**)&pin_out_, (size_t)B() * H() * W() * 7 * 4 + 2 * img, hipHostMallocDefault));
  HIP_CHECK(hipHostGetDevicePointer((void**)&pin_out_dev_, pin_out_, 0));
  HIP_CHECK(hipHostGetDevicePointer((void**)&pin_in_dev_, pin_in_, 0));
  for (auto& e : ev_copy_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (const char* ht = std::getenv("SA_HOST_TIMES"))
    if (ht[0] == '1')
      for (auto& e : host_ev_) HIP_CHECK(hipEventCreate(&e));
  copy_pool_ = std::make_unique<HostCopyPool>(3);
  // generous split-K / stream-K workspaces for the tuning pass (128 MiB of fp32 slabs, 8192 tile counters);
  // right-sized to the tuned plan's high-water mark afterwards
  splitk_.alloc(arena_, 32l << 20, 8192);
  splitk_side_.alloc(arena_, 32l << 20, 8192);
  splitk_side2_.alloc(arena_, 32l << 20, 8192);
  WeightSource src{store_.get(), cfg_.weights.empty(), cfg_.seed};
  TraceRange tr("engine build");
  build(src);
  store_.reset();  // host copies no longer needed
  HIP_CHECK(hipDeviceSynchronize());
  if (conv_tuning_enabled()) {
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, cfg_.device));
    conv_plan_set_arch(prop.gcnArchName);
    // tuned-plan cache next to the model, the analogue of the reference's "<stem>_batch=1.engine"
    // (RAFTStereo/src/TRTRAFTStereo.cpp:25-46): a second Initialize of the same model / shape / device
    // arch skips tactic timing entirely
    plan_path_ = default_plan_path();
    if (!plan_path_.empty()) {
      plan_loaded_ = conv_plan_load(plan_path_);
      if (plan_loaded_ >= 0) SA_LOGI("tactic plan %s: %d entries loaded", plan_path_.c_str(), plan_loaded_);
      else if (plan_loaded_ == -2)
        SA_LOGW("tactic plan %s was written by another library build: ignored (re-tuning)", plan_path_.c_str());
    }
    const long tuned0 = conv_tune_count();
    std::vector<std::string> keys;
    {
      // eager tuning pass: every conv shape of the frame is timed over the launcher's tactics (on
      // whatever the buffers hold) and the plan is fixed before the frame graph is captured
      ScopedSplitK sk(&splitk_);
      ScopedConvTuning tune(true);
      ScopedPlanCollect collect(&keys);
      TraceRange ttr("conv tactic selection");
      tuning_pass_ = true;
      forward(stream_);
      tuning_pass_ = false;
      HIP_CHECK(hipStreamSynchronize(stream_));
    }
    tuned_shapes_ = conv_tune_count() - tuned0;
    plan_keys_ = keys;
    // Save whenever this engine's own plan file lacks a shape it consulted, not only when it tuned one: an engine
    // whose shapes were all tuned by an earlier engine in the same process (crestereo-iter10 after iter2 / iter5)
    // still gets its "<stem>_batch=1.engine"-style file, so a fresh process running it alone does not re-tune.
    if (!plan_path_.empty() && (tuned_shapes_ > 0 || conv_plan_missing(plan_path_, keys) > 0)) {
      plan_saved_ = conv_plan_save(plan_path_, keys);
      if (plan_saved_ == 0) SA_LOGI("tactic plan saved to %s", plan_path_.c_str());
      else SA_LOGE("could not write tactic plan %s: %s", plan_path_.c_str(), std::strerror(plan_saved_));
    }
    // right-size the split-K workspaces to what the tuned plan actually launches (every stream's
    // workspace serves a subset of the same convs, so the pass's high-water mark bounds each)
    const int64_t fl = splitk_.max_floats;
    const int32_t nc = splitk_.max_counters;
    HIP_CHECK(hipDeviceSynchronize());
    splitk_.alloc(arena_, fl, nc);
    splitk_side_.alloc(arena_, fl, nc);
    splitk_side2_.alloc(arena_, fl, nc);
  }
  SA_LOGI("%s: built, %.1f MiB device memory", name(), arena_.bytes() / 1048576.0);
}

long StereoEngine::nonzero_splitk_counters() {
  HIP_CHECK(hipStreamSynchronize(stream_));
  long bad = 0;
  for (const SplitKWorkspace* w : {&splitk_, &splitk_side_, &splitk_side2_}) {
    if (!w->counters || w->n_counters <= 0) continue;
    std::vector<int32_t> h((size_t)w->n_counters);
    HIP_CHECK(hipMemcpy(h.data(), w->counters, h.size() * 4, hipMemcpyDeviceToHost));
    for (int32_t v : h) bad += v != 0;
  }
  return bad;
}

std::string StereoEngine::default_plan_path() const {
  // SA_PLAN_CACHE=<file> (process-wide plan file, appended), SA_PLAN_CACHE=0 / SA_PLAN_DIR="" disable
  if (const char* e = std::getenv("SA_PLAN_CACHE")) {
    (void)e;
    return std::string();
  }
  std::string dir, stem;
  if (!cfg_.weights.empty()) {
    const size_t slash = cfg_.weights.find_last_of('/');
    dir = slash == std::string::npos ? "." : cfg_.weights.substr(0, slash);
    stem = cfg_.weights.substr(slash == std::string::npos ? 0 : slash + 1);
    const size_t dot = stem.rfind('.');
    if (dot != std::string::npos) stem = stem.substr(0, dot);
  } else {
    stem = cfg_.model + "_seed" + std::to_string(cfg_.seed);
  }
  if (const char* d = std::getenv("SA_PLAN_DIR")) {
    if (!d[0]) return std::string();
    dir = d;
  } else if (dir.empty()) {
    const char* xdg = std::getenv("XDG_CACHE_HOME");
    const char* home = std::getenv("HOME");
    if (xdg && xdg[0]) dir = std::string(xdg) + "/stereoalgorithms_amd";
    else if (home && home[0]) dir = std::string(home) + "/.cache/stereoalgorithms_amd";
    else return std::string();
  }
  for (size_t i = 1; i <= dir.size(); ++i)  // mkdir -p
    if (i == dir.size() || dir[i] == '/') {
      const std::string part = dir.substr(0, i);
      if (::mkdir(part.c_str(), 0755) != 0 && errno != EEXIST) return std::string();
    }
  char tail[160];
  std::snprintf(tail, sizeof(tail), "_b%d_%dx%d_it%d_%s.plan", B(), H(), W(), cfg_.iters, conv_plan_arch().c_str());
  return dir + "/" + stem + tail;
}

hipStream_t StereoEngine::fork(hipStream_t s) {
  HIP_CHECK(hipEventRecord(ev_fork_, s));
  HIP_CHECK(hipStreamWaitEvent(side_, ev_fork_, 0));
  return side_;
}

void StereoEngine::join(hipStream_t s) {
  HIP_CHECK(hipEventRecord(ev_join_, side_));
  HIP_CHECK(hipStreamWaitEvent(s, ev_join_, 0));
}

void StereoEngine::rec(hipStream_t s, int i) { HIP_CHECK(hipEventRecord(ev_dep_[i], s)); }
void StereoEngine::wait(hipStream_t s, int i) { HIP_CHECK(hipStreamWaitEvent(s, ev_dep_[i], 0)); }

void StereoEngine::set_Q(const float* q16) {
  std::memcpy(Q_, q16, sizeof(Q_));
  have_Q_ = true;
  for (GraphExec& g : graph_) g.reset();  // Q is baked into the reprojection launch
  for (int i = 0; i < 8; ++i) repro_node_[i] = in_node_[i] = nullptr;
}

void StereoEngine::set_rectify_maps(const float* ml, const float* mr) {
  const size_t n = (size_t)H() * W() * 2;
  if (!rect_maps_) rect_maps_ = (float*)arena_.alloc(2 * n * 4);
  HIP_CHECK(hipMemcpy(rect_maps_, ml, n * 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(rect_maps_ + n, mr, n * 4, hipMemcpyHostToDevice));
}

void StereoEngine::tap(hipStream_t s, const char* name, const Tensor& t) const {
  if (cfg_.use_graph) return;
  const char* dir = std::getenv("SA_TAP_DIR");
  if (!dir || !dir[0]) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_CHECK(hipStreamIsCapturing(s, &cs));
  if (cs != hipStreamCaptureStatusNone) return;
  HIP_CHECK(hipStreamSynchronize(s));
  std::vector<char> host(t.nbytes());
  HIP_CHECK(hipMemcpy(host.data(), t.ptr, host.size(), hipMemcpyDeviceToHost));
  const std::string path = std::string(dir) + "/" + name + ".sat";
  FILE* f = std::fopen(path.c_str(), "wb");
  SA_REQUIRE(f != nullptr, "cannot write tap %s", path.c_str());
  const int32_t hdr[7] = {t.n, t.d, t.h, t.w, t.c, t.stride, (int32_t)t.dt};
  std::fwrite(hdr, sizeof(hdr), 1, f);
  std::fwrite(host.data(), 1, host.size(), f);
  std::fclose(f);
}

void StereoEngine::tap_f32(hipStream_t s, const char* name, const float* p, int n, int h, int w, int c) const {
  Tensor t;
  t.ptr = const_cast<float*>(p);
  t.n = n;
  t.h = h;
  t.w = w;
  t.c = t.stride = c;
  t.dt = DT::F32;
  tap(s, name, t);
}

void StereoEngine::stage(hipStream_t s, const char* name) {
  if (!stage_on_ || tuning_pass_ || nstage_ >= kMaxStages) return;
  stage_name_[nstage_] = name;
  const int rc = sa_stamp(stage_ts_, nstage_, s);
  SA_REQUIRE(rc == 0, "stage stamp failed");
  ++nstage_;
}

std::vector<std::pair<std::string, float>> StereoEngine::stage_times() const {
  std::vector<std::pair<std::string, float>> out;
  if (!stage_on_ || nstage_ < 2) return out;
  HIP_CHECK(hipStreamSynchronize(stream_));
  unsigned long long ts[kMaxStages];
  HIP_CHECK(hipMemcpy(ts, stage_ts_, nstage_ * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  int khz = 0;
  HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, cfg_.device));
  for (int i = 1; i < nstage_; ++i)
    out.emplace_back(stage_name_[i], khz > 0 ? (float)((double)(ts[i] - ts[i - 1]) / khz) : -1.f);
  return out;
}

void StereoEngine::frame(hipStream_t s, bool rectify, bool host_out, bool host_in) {
  ScopedSplitK sk(&splitk_);
  nstage_ = 0;
  stage(s, "start");
  const int gi = (rectify ? 1 : 0) + (host_out ? 2 : 0) + (host_in ? 4 : 0);
  auto captured_node = [&](hipGraphNode_t* node) {  // the node just captured on s (when capturing)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    HIP_CHECK(hipStreamGetCaptureInfo_v2(s, &cs, nullptr, nullptr, &deps, &nd));
    if (cs == hipStreamCaptureStatusActive && nd == 1) {
      *node = deps[0];
      return true;
    }
    return false;
  };
  if (host_in) {
    const size_t img = (size_t)B() * H() * W() * 3;
    const int rc = sa_copy_frames(in_src_[0], in_src_[1], rectify ? raw_left_ : in_left_, rectify ? raw_right_ : in_right_,
                                  (long)img, s);
    SA_REQUIRE(rc == 0, "input copy failed (%d)", rc);
    if (captured_node(&in_node_[gi])) {
      in_ptrs_[gi][0] = in_src_[0];
      in_ptrs_[gi][1] = in_src_[1];
    }
    stage(s, "input");  // the PCIe read of the frame: its own stage, not the network's
  }
  if (rectify) {
    SA_REQUIRE(rect_maps_ != nullptr, "rectification requested but no maps set");
    // left images use map 0, right images map 1 (maps laid out [2][H][W][2])
    int rc = sa_remap_bgr(raw_left_, B(), H(), W(), rect_maps_, 1, H(), W(), in_left_, s);
    SA_REQUIRE(rc == 0, "remap failed");
    rc = sa_remap_bgr(raw_right_, B(), H(), W(), rect_maps_ + (size_t)H() * W() * 2, 1, H(), W(), in_right_, s);
    SA_REQUIRE(rc == 0, "remap failed");
  }
  if (rectify) stage(s, "rectify");
  forward(s);
  stage(s, "network");
  if (have_Q_) {
    // host_out: disparity and cloud go straight into host memory (the engine's pinned outputs or registered caller
    // buffers, zero-copy run_host), no D2H copy; the captured node is re-pointed when a frame targets other buffers
    int rc;
    if (host_out) {
      rc = sa_reproject(disp_, 1, 1.f, in_left_, B(), H(), W(), Q_, out_target_[0], out_target_[1], s);
      if (rc == 0 && captured_node(&repro_node_[gi])) {
        repro_ptrs_[gi][0] = out_target_[0];
        repro_ptrs_[gi][1] = out_target_[1];
      }
    } else {
      rc = sa_reproject(disp_, 1, 1.f, in_left_, B(), H(), W(), Q_, nullptr, cloud_, s);
    }
    SA_REQUIRE(rc == 0, "reproject failed");
    stage(s, "reproject");
  }
  SA_LAUNCH_CHECK(s);
}

void StereoEngine::launch_frame(hipStream_t s, bool rectify, bool host_out, bool host_in) {
  const int gi = (rectify ? 1 : 0) + (host_out ? 2 : 0) + (host_in ? 4 : 0);
  GraphExec& g = graph_[gi];
  // The frame always executes on the engine's own stream (where its graphs were captured); a
  // caller stream is ordered against it with events on both sides, so graph execs are never
  // replayed on a foreign (e.g. the legacy null) stream.
  const bool foreign = s != stream_;
  if (foreign) {
    HIP_CHECK(hipEventRecord(ev_in_, s));
    HIP_CHECK(hipStreamWaitEvent(stream_, ev_in_, 0));
  }
  TraceRange tr("frame");
  if (cfg_.use_graph) {
    if (!g.ready()) g.capture(stream_, [&] { frame(stream_, rectify, host_out, host_in); });
    if (host_in && (in_ptrs_[gi][0] != in_src_[0] || in_ptrs_[gi][1] != in_src_[1])) {
      SA_REQUIRE(in_node_[gi] != nullptr, "host-input graph without its input-copy node");
      const size_t img = (size_t)B() * H() * W() * 3;
      const int rc = sa_copy_frames_update_node(g.exec(), in_node_[gi], in_src_[0], in_src_[1],
                                                rectify ? raw_left_ : in_left_, rectify ? raw_right_ : in_right_, (long)img);
      SA_REQUIRE(rc == 0, "re-pointing the input-copy node failed (%d)", rc);
      in_ptrs_[gi][0] = in_src_[0];
      in_ptrs_[gi][1] = in_src_[1];
    }
    if (host_out && (repro_ptrs_[gi][0] != out_target_[0] || repro_ptrs_[gi][1] != out_target_[1])) {
      SA_REQUIRE(repro_node_[gi] != nullptr, "host-output graph without its reprojection node");
      const int rc = sa_reproject_update_node(g.exec(), repro_node_[gi], disp_, 1, 1.f, in_left_, B(), H(), W(), Q_,
                                              out_target_[0], out_target_[1]);
      SA_REQUIRE(rc == 0, "re-pointing the reprojection node failed (%d)", rc);
      repro_ptrs_[gi][0] = out_target_[0];
      repro_ptrs_[gi][1] = out_target_[1];
    }
    g.launch(stream_);
  } else {
    frame(stream_, rectify, host_out, host_in);
  }
  static const bool sync_frame = [] {
    const char* v = std::getenv("SA_SYNC_FRAME");
    return v && v[0] == '1';
  }();
  if (sync_frame) HIP_CHECK(hipStreamSynchronize(stream_));  // diagnostic: host-ordered hand-off
  if (foreign) {
    HIP_CHECK(hipEventRecord(ev_out_, stream_));
    HIP_CHECK(hipStreamWaitEvent(s, ev_out_, 0));
  }
  launches_per_frame_++;
}

void StereoEngine::run_device(const uint8_t* left, const uint8_t* right, float* disp, float* cloud,
                              bool rectify, hipStream_t s, uint8_t* rect_left, uint8_t* rect_right) {
  HIP_CHECK(hipSetDevice(cfg_.device));
  const size_t img = (size_t)B() * H() * W() * 3;
  // Straight through the frame graph: the graph's input-copy node reads the caller's device
  // images and its reprojection node writes disparity + cloud into the caller's tensors -- the same two nodes
  // run_host re-points at host memory (launch_frame updates them when the pointers change), so no D2D copy runs
  // around the graph.  SA_DEVICE_DIRECT=0, no Q (no reprojection node), unaligned inputs or requested rectified
  // outputs keep the copy path.
  static const bool direct_on = [] {
    const char* e = std::getenv("SA_DEVICE_DIRECT");
    return !(e && e[0] == '0');
  }();
  const bool direct = direct_on && cfg_.use_graph && have_Q_ && img % 16 == 0 && (disp || cloud) &&
                      (((uintptr_t)left | (uintptr_t)right) & 15) == 0 && !(rectify && (rect_left || rect_right));
  if (direct) {
    in_src_[0] = left;
    in_src_[1] = right;
    out_target_[0] = disp;
    out_target_[1] = have_Q_ ? cloud : nullptr;
    launch_frame(s, rectify, true, true);
    return;
  }
  uint8_t* dl = rectify ? raw_left_ : in_left_;
  uint8_t* dr = rectify ? raw_right_ : in_right_;
  HIP_CHECK(hipMemcpyAsync(dl, left, img, hipMemcpyDeviceToDevice, s));
  HIP_CHECK(hipMemcpyAsync(dr, right, img, hipMemcpyDeviceToDevice, s));
  launch_frame(s, rectify);
  const size_t n = (size_t)B() * H() * W();
  if (disp) HIP_CHECK(hipMemcpyAsync(disp, disp_, n * 4, hipMemcpyDeviceToDevice, s));
  if (cloud && have_Q_) HIP_CHECK(hipMemcpyAsync(cloud, cloud_, n * 24, hipMemcpyDeviceToDevice, s));
  if (rectify && rect_left) HIP_CHECK(hipMemcpyAsync(rect_left, in_left_, img, hipMemcpyDeviceToDevice, s));
  if (rectify && rect_right) HIP_CHECK(hipMemcpyAsync(rect_right, in_right_, img, hipMemcpyDeviceToDevice, s));
}

void StereoEngine::host_buffers(uint8_t** left, uint8_t** right, float** disp, float** cloud) const {
  const size_t img = (size_t)B() * H() * W() * 3;
  const size_t n = (size_t)B() * H() * W();
  *left = pin_in_;
  *right = pin_in_ + img;
  *disp = pin_out_;
  *cloud = pin_out_ + n;
}

void StereoEngine::unregister_host(int role) {
  HostReg& r = host_reg_[role];
  if (r.dev) (void)hipHostUnregister(r.host);
  r = HostReg{};
}

float* StereoEngine::resolve_host_out(int role, void* p, size_t bytes) {
  const size_t n = (size_t)B() * H() * W();
  if (role == 0 && p == pin_out_) return pin_out_dev_;
  if (role == 1 && p == pin_out_ + n) return pin_out_dev_ + n;
  return static_cast<float*>(resolve_host_reg(role, p, bytes));
}

// Device address of a caller host buffer for role `role`: mapped (hipHostRegister) once the same (pointer, size)
// comes back for a second frame, nullptr before that, after a failed registration, or with SA_HOST_REGISTER=0.
void* StereoEngine::resolve_host_reg(int role, void* p, size_t bytes) {
  static const bool on = [] {
    const char* e = std::getenv("SA_HOST_REGISTER");
    return !(e && e[0] == '0');
  }();
  if (!on) return nullptr;
  HostReg& r = host_reg_[role];
  if (r.host != p || r.bytes != bytes) {  // a new buffer: the copy path this frame, mapped if it comes back
    unregister_host(role);
    r.host = p;
    r.bytes = bytes;
    return nullptr;
  }
  if (r.dev || r.failed) return r.dev;
  void* dev = nullptr;
  if (hipHostRegister(p, bytes, hipHostRegisterMapped) != hipSuccess) {
    (void)hipGetLastError();
    r.failed = true;  // e.g. overlapping an already registered range: keep copying
    SA_LOGW("run_host: caller buffer %p (%zu B) could not be mapped; copies stay", p, bytes);
    return nullptr;
  }
  if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess || !dev) {
    (void)hipGetLastError();
    (void)hipHostUnregister(p);
    r.failed = true;
    return nullptr;
  }
  r.dev = dev;
  return dev;
}

void StereoEngine::run_host(uint8_t* left, uint8_t* right, float* disp, float* cloud, bool rectify) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  HIP_CHECK(hipSetDevice(cfg_.device));
  hipStream_t s = stream_;
  const size_t img = (size_t)B() * H() * W() * 3;
  const size_t n = (size_t)B() * H() * W();
  // Buffers handed out by host_buffers() are the pinned staging itself: a caller that fills / reads them in place
  // skips the pageable <-> pinned copies (the D2H lands in the caller's array directly).
  // Zero-copy inputs (SA_HOST_IN=0: DMA copies from the pinned staging instead): the frame graph's first node reads
  // the images over PCIe from the engine's pinned staging (host_buffers()) or from the caller's arrays once mapped
  // (a caller passing the same input arrays again, like a camera's frame buffers); otherwise the caller's arrays
  // are staged into the pinned buffers first.
  static const bool host_in_on = [] {
    const char* e = std::getenv("SA_HOST_IN");
    return !(e && e[0] == '0');
  }();
  const bool host_in = host_in_on && cfg_.use_graph && img % 16 == 0;
  const uint8_t* src[2] = {nullptr, nullptr};
  std::vector<HostCopyPool::Task> in;
  for (int i = 0; i < 2; ++i) {
    uint8_t* user = i ? right : left;
    uint8_t* pin = pin_in_ + i * img;
    if (user == pin) {
      src[i] = pin_in_dev_ + i * img;
      continue;
    }
    const uint8_t* dev =
        host_in && ((uintptr_t)user & 15) == 0 ? static_cast<const uint8_t*>(resolve_host_reg(2 + i, user, img)) : nullptr;
    if (dev) {
      src[i] = dev;
    } else {
      in.push_back({pin, user, img, nullptr});
      src[i] = pin_in_dev_ + i * img;
    }
  }
  copy_pool_->run(in);
  const auto t1 = clk::now();
  if (host_ev_[0]) HIP_CHECK(hipEventRecord(host_ev_[0], s));
  if (host_in) {
    in_src_[0] = src[0];
    in_src_[1] = src[1];
  } else {
    uint8_t* dl = rectify ? raw_left_ : in_left_;
    uint8_t* dr = rectify ? raw_right_ : in_right_;
    HIP_CHECK(hipMemcpyAsync(dl, pin_in_, img, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(dr, pin_in_ + img, img, hipMemcpyHostToDevice, s));
  }
  if (host_ev_[1]) HIP_CHECK(hipEventRecord(host_ev_[1], s));
  // zero-copy outputs: the frame graph's reprojection writes disparity and cloud straight into host memory over
  // PCIe and no D2H copy follows -- into the engine's pinned buffers (host_buffers()) or into the caller's own
  // buffers once mapped (resolve_host_out: a buffer the caller passes again, as the reference's demo reuses its
  // point cloud, RAFTStereo/test/main.cpp:20)
  float* dd = disp ? resolve_host_out(0, disp, n * 4) : nullptr;
  float* dc = cloud ? resolve_host_out(1, cloud, n * 24) : nullptr;
  const bool zero_copy = have_Q_ && (disp || cloud) && (!disp || dd) && (!cloud || dc);
  if (zero_copy) {
    out_target_[0] = dd;
    out_target_[1] = dc;
  }
  launch_frame(s, rectify, zero_copy, host_in);
  if (host_ev_[2]) HIP_CHECK(hipEventRecord(host_ev_[2], s));
  float* pd = pin_out_;
  float* pc = pin_out_ + n;
  uint8_t* pr = reinterpret_cast<uint8_t*>(pin_out_ + 7 * n);
  // outputs: each D2H piece gets an event; the pool copies a piece into the caller's array once it landed,
  // overlapping the rest of the transfer (nothing to copy when the caller's array is the pinned buffer)
  std::vector<HostCopyPool::Task> out;
  int ev = 0;
  auto d2h = [&](void* dst, void* pinned, const void* dev, size_t bytes) {
    HIP_CHECK(hipMemcpyAsync(pinned, dev, bytes, hipMemcpyDeviceToHost, s));
    if (dst == pinned) return;
    HIP_CHECK(hipEventRecord(ev_copy_[ev], s));
    out.push_back({dst, pinned, bytes, ev_copy_[ev]});
    ++ev;
  };
  if (disp && !zero_copy) d2h(disp, pd, disp_, n * 4);
  if (cloud && have_Q_ && !zero_copy) {
    constexpr int kChunks = kCopyEvents - 3;
    const size_t total = n * 24, step = (total / kChunks + 4095) & ~(size_t)4095;
    for (size_t o = 0; o < total; o += step) {
      const size_t b = std::min(step, total - o);
      d2h(reinterpret_cast<char*>(cloud) + o, reinterpret_cast<char*>(pc) + o, reinterpret_cast<const char*>(cloud_) + o,
          b);
    }
  }
  if (rectify) {  // reference semantics: inputs are overwritten with their rectified versions
    d2h(left, pr, in_left_, img);
    d2h(right, pr + img, in_right_, img);
  }
  SA_REQUIRE(ev <= kCopyEvents, "run_host: %d copy events", ev);
  if (host_ev_[3]) HIP_CHECK(hipEventRecord(host_ev_[3], s));
  const auto t2 = clk::now();
  copy_pool_->run(out);
  // SA_HOST_SPIN=1: poll the stream instead of the blocking wait (no wake-up latency; burns the calling core)
  static const bool spin = [] {
    const char* e = std::getenv("SA_HOST_SPIN");
    return e && e[0] == '1';
  }();
  if (spin) {
    hipError_t q;
    while ((q = hipStreamQuery(s)) == hipErrorNotReady) {
    }
    HIP_CHECK(q);
  } else {
    HIP_CHECK(hipStreamSynchronize(s));
  }
  const auto t3 = clk::now();
  auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<float, std::milli>(b - a).count(); };
  host_times_[0] = ms(t0, t3);  // whole timed region
  host_times_[1] = ms(t0, t1);  // caller -> pinned input copies
  host_times_[2] = ms(t1, t2);  // enqueue (H2D, graph launch, D2H)
  host_times_[3] = ms(t2, t3);  // wait for the device + pinned -> caller output copies
  if (host_ev_[0]) {  // SA_HOST_TIMES=1: device-side split of the same frame
    HIP_CHECK(hipEventElapsedTime(&host_times_[4], host_ev_[0], host_ev_[1]));  // H2D
    // zero-copy inputs: the frame graph's first node reads the images over PCIe, so nothing lies between the first
    // two events -- the H2D is inside 'graph' (reporting ~0 ms here misread against round-4 records)
    if (host_in) host_times_[4] = -1.f;
    HIP_CHECK(hipEventElapsedTime(&host_times_[5], host_ev_[1], host_ev_[2]));  // frame graph
    HIP_CHECK(hipEventElapsedTime(&host_times_[6], host_ev_[2], host_ev_[3]));  // D2H
  }
}

}  // namespace sa
