// Engine runtime: device arena (static memory plan), NHWC tensor views, host weight store
// (safetensors), packed convolution layers, hipGraph capture.
//
// The reference's runtime is TensorRT (engine build / deserialize / enqueue:
// common/ONNX2TRT.cpp:43-128, RAFTStereo/src/TRTRAFTStereo.cpp:48-113).  Here the model graph is
// our own C++ code: every activation is carved from one arena at init (shapes are static), all
// launches go to one stream and the whole frame is captured into a hipGraph once.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "sa/common.h"
#include "sa/kernels.h"

namespace sa {

// ------------------------------------------------------------------ device arena
class DeviceArena {
 public:
  DeviceArena() = default;
  ~DeviceArena();
  DeviceArena(const DeviceArena&) = delete;
  DeviceArena& operator=(const DeviceArena&) = delete;
  // Allocations are individually hipMalloc'd (so ASan-like tooling sees bounds) and freed
  // together; sizes are rounded to 256 B.
  void* alloc(size_t bytes);
  void free(void* p);  // one allocation of this arena
  size_t bytes() const { return total_; }
  void release();

 private:
  std::vector<void*> ptrs_;
  std::vector<size_t> sizes_;
  size_t total_ = 0;
};


// ------------------------------------------------------------------ tensors
enum class DT { F16 = 0, F32 = 1, U8 = 2 };
inline size_t dt_size(DT d) { return d == DT::F16 ? 2 : (d == DT::F32 ? 4 : 1); }

// NHWC view.  `stride` = elements between consecutive pixels (>= c); ptr points at channel 0 of
// this view (so a channel slice is a pointer offset).
struct Tensor {
  void* ptr = nullptr;
  int n = 0, h = 0, w = 0, c = 0, stride = 0;
  DT dt = DT::F16;
  int d = 1;  // depth of a 3-D volume [n][d][h][w][c] (cost volumes)
  long pixels() const { return (long)n * d * h * w; }
  size_t nbytes() const { return (size_t)pixels() * stride * dt_size(dt); }
  Tensor slice_c(int off, int cnt) const {
    Tensor t = *this;
    t.ptr = (char*)ptr + (size_t)off * dt_size(dt);
    t.c = cnt;
    return t;
  }
  Tensor slice_n(int off, int cnt) const {
    Tensor t = *this;
    t.ptr = (char*)ptr + (size_t)off * d * h * w * stride * dt_size(dt);
    t.n = cnt;
    return t;
  }
  template <typename T>
  T* as() const { return reinterpret_cast<T*>(ptr); }
};

Tensor make_tensor(DeviceArena& a, int n, int h, int w, int c, DT dt = DT::F16, int stride = -1);
Tensor make_volume(DeviceArena& a, int n, int d, int h, int w, int c, DT dt = DT::F16, int stride = -1);

// ------------------------------------------------------------------ activation memory planner
// Liveness-based placement of the activations of a straight-line run (a chain of encoder blocks):
// each tensor is declared with the step that defines it and the last step that reads it; commit()
// packs all of them into ONE allocation (greedy best-fit by size over address intervals of tensors
// whose lifetimes overlap) and patches their pointers.  Tensors must not need zero-initialised
// padding (they share bytes with dead tensors) and must only be touched inside their interval.
class ActPlan {
 public:
  static constexpr int kForever = 1 << 30;
  void def(Tensor* t, int n, int h, int w, int c, DT dt = DT::F16);  // defined at the current step
  void use(const Tensor* t);    // read at the current step (extends the lifetime)
  void keep(const Tensor* t);   // live past the run (outputs)
  void next() { ++step_; }
  int step() const { return step_; }
  size_t commit(DeviceArena& a);  // returns the bytes of the shared allocation
  size_t naive_bytes() const;     // what one allocation per tensor would take
 private:
  struct Item {
    Tensor* t;
    size_t bytes;
    int first, last;
    size_t off = 0;
  };
  Item* find(const Tensor* t);
  std::vector<Item> items_;
  int step_ = 0;
};

// ------------------------------------------------------------------ host weights
struct HostTensor {
  std::vector<int64_t> shape;
  std::vector<float> data;  // converted to fp32 on load
  int64_t numel() const {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    return n;
  }
};

class WeightStore {
 public:
  // safetensors file (F32 / F16 / BF16 tensors).  `__metadata__` entries are kept as strings.
  static std::unique_ptr<WeightStore> load_safetensors(const std::string& path);
  bool has(const std::string& name) const { return t_.count(name) > 0; }
  const HostTensor& get(const std::string& name) const;
  std::string meta(const std::string& key, const std::string& dflt = "") const;
  void put(const std::string& name, HostTensor t) { t_[name] = std::move(t); }
  void set_meta(const std::string& k, const std::string& v) { meta_[k] = v; }
  const std::map<std::string, HostTensor>& all() const { return t_; }

 private:
  std::map<std::string, HostTensor> t_;
  std::map<std::string, std::string> meta_;
};

// ------------------------------------------------------------------ split-K workspace
// fp32 partial slabs + arrival counters shared by every conv of one engine (its kernels run in
// stream order, so one workspace suffices).  Installed thread-locally while a frame is
// recorded; ConvLayer launches pick it up and let sa_conv2d choose the split.
struct SplitKWorkspace {
  float* ws = nullptr;
  int32_t* counters = nullptr;
  int64_t ws_floats = 0;
  int32_t n_counters = 0;
  // high-water mark of what launches under this workspace actually used (ConvLayer::launch)
  mutable int64_t max_floats = 0;
  mutable int32_t max_counters = 0;
  void alloc(DeviceArena& a, int64_t floats, int32_t counters);  // (re)allocates
};
// Zero device memory inside a frame.  Always a kernel node (sa_zero): hipMemsetAsync nodes in a graph replayed
// with packet capture on a non-blocking stream were seen executing out of order with the kernels around them
// (tools/diag/replay_stress.py, tools/graph_repro/overlap_repro.hip).  SA_ZERO_MEMSET=1 restores the memset
// node for that A/B.
void device_zero(void* p, size_t bytes, hipStream_t s);
const SplitKWorkspace* current_splitk();
struct ScopedSplitK {
  const SplitKWorkspace* prev;
  explicit ScopedSplitK(const SplitKWorkspace* w);
  ~ScopedSplitK();
};

// Convs enqueued while a ScopedSideBranch(true) is alive belong to a branch that runs beside the frame's critical
// chain in the frame graph (set identically in the eager tuning pass and in the capture).  Their plan key carries
// the mark, and the tuner picks among the tactics within SA_TUNE_LDS_TOL (default 0.08) of the fastest the one with
// the smallest LDS footprint, so the branch's workgroups co-reside with the chain's instead of taking whole CUs.
struct ScopedSideBranch {
  bool prev;
  explicit ScopedSideBranch(bool on);
  ~ScopedSideBranch();
};
bool side_branch();

// Convs enqueued while a ScopedWgSplit(true) is alive may be tuned to the workgroup split-K tactics (37 / 38: fp32
// partial tiles of S K-slices + a reduce / epilogue launch).  Faster alone on small-M / deep-K grids (coarse GRU
// shapes 10-25 %), but they fill the chip for two launches: on schedules whose branches share the GPU (RAFT's
// pipelined levels) the frame got slower (RAFT-SF b1 8.22 -> 8.59 ms, realtime 1.87 -> 1.95), on CREStereo's
// serial chain faster (iter10 5.72 -> 5.64).  Opt-in per model; the plan key carries the mark.
struct ScopedWgSplit {
  bool prev;
  explicit ScopedWgSplit(bool on);
  ~ScopedWgSplit();
};
bool wg_split_allowed();

// ------------------------------------------------------------------ conv tactic selection
// The MI355X analogue of TensorRT's tactic selection at engine build (common/ONNX2TRT.cpp:111):
// during the engine's eager tuning pass every distinct conv shape is timed over the tile / split-K
// candidates of sa_conv2d (outputs redirected to scratch, so in-place epilogues are not disturbed)
// and the fastest is recorded in a process-wide plan keyed by shape; graph capture and later
// engines reuse it.  SA_TUNE=0 disables (launcher heuristics only); SA_PLAN_CACHE=<file> persists
// plans across processes (one "key tile_cfg splitk us" line per shape).
struct ScopedConvTuning {
  bool prev;
  explicit ScopedConvTuning(bool on);
  ~ScopedConvTuning();
};
bool conv_tuning_enabled();
// Look up (and, inside a ScopedConvTuning(true) scope outside stream capture, tune) the plan for
// `a`; sets a.tile_cfg / a.splitk when a plan exists.
void conv_apply_plan(SaConvArgs& a, hipStream_t s);
size_t conv_plan_entries();
long conv_tune_count();     // shapes tuned (timed) in this process
long conv_tune_rejects();   // tactic candidates rejected by the tuner's output verification
void conv_plan_clear();     // drop the in-process plan (tests: prove a plan file is used)
void conv_plan_set_arch(const std::string& gcn_arch_name);  // plan keys carry the device's arch
const std::string& conv_plan_arch();
// merge a plan file; returns entries added, -1 if absent, -2 if it was written by another library build
int conv_plan_load(const std::string& file);
// append one entry to the SA_PLAN_CACHE file (header written when the file is new, foreign or was deleted)
void conv_plan_cache_append(const std::string& key, int cfg, int splitk, float us);
// write the plan entries of `keys` (atomic rename); 0 or the errno of the failing step
int conv_plan_save(const std::string& file, const std::vector<std::string>& keys);
const std::string& conv_plan_build_id();  // hash of the loaded kernel library (plan files carry it)
// how many of `keys` have an in-process plan but no entry in `file` (all of them if the file is absent / stale)
int conv_plan_missing(const std::string& file, const std::vector<std::string>& keys);
void conv_plan_put(const std::string& key, int cfg, int splitk, float us);  // tests: seed the in-process plan
// DP ranks that merged rank 0's broadcast table: later plan-file loads keep every entry already in the process
void conv_plan_pin(bool on);
// 16-hex FNV-1a digest of the (key, cfg, splitk) the process plan holds for `keys` plus the library build id: equal
// digests = identical kernels launched for those shapes
std::string conv_plan_digest(const std::vector<std::string>& keys);
// collects every plan key consulted by conv_apply_plan in this thread (the engine's own shapes)
struct ScopedPlanCollect {
  std::vector<std::string>* prev;
  explicit ScopedPlanCollect(std::vector<std::string>* keys);
  ~ScopedPlanCollect();
};

// ------------------------------------------------------------------ conv layers
// Copies of every instance-norm statistics buffer the conv epilogues spread their atomics over
// (SaConvArgs.stats_slots); StatsPool reserves this many, instnorm() folds them (sa_stats_reduce).
constexpr int kStatSlots = 16;

// Describes how the conv's (padded) input channels map to the checkpoint's input channels:
// a list of {real, padded} segments concatenated along channels.
struct ChanSeg {
  int real, padded;
};

struct ConvSpec {
  int kh = 3, kw = 3, sh = 1, sw = 1, ph = -1, pw = -1, dh = 1, dw = 1;
  int kd = 0, sd = 1, pd = -1;  // kd > 0: 3-D convolution
};

class ConvLayer {
 public:
  ConvLayer() = default;
  // weight: [Cout][Cin][KH][KW] from `ws`, bias optional; optional BatchNorm fold with prefix
  // `bn` (weight, bias, running_mean, running_var); `scale` multiplies weights and bias.
  // Several checkpoint convs may be stacked along Cout (`wnames`).
  void build(DeviceArena& arena, const WeightStore& ws, const std::vector<std::string>& wnames,
             const std::vector<ChanSeg>& in_segs, ConvSpec spec,
             const std::vector<std::string>& bn_names = {}, float scale = 1.f, float bn_eps = 1e-5f);
  // 3-D conv (weight [Cout][Cin][KD][KH][KW], optional BatchNorm3d fold)
  void build3d(DeviceArena& arena, const WeightStore& ws, const std::string& wname, const std::vector<ChanSeg>& in_segs,
               ConvSpec spec, const std::string& bn_name = "", float bn_eps = 1e-5f);
  // ConvTranspose2d/3d(k=4, s=2, p=1) (weight [Cin][Cout][4][4](4), optional bias / BN fold) as a
  // 3x3(x3) conv producing 4 (8) parity classes scattered by the epilogue (SaConvArgs.up);
  // ConvTranspose2d(k=2, s=2) weights ([Cin][Cout][2][2]) become a 1x1 conv with the same scatter.
  void build_deconv(DeviceArena& arena, const WeightStore& ws, const std::string& wname, bool is3d,
                    const std::vector<ChanSeg>& in_segs, const std::string& bn_name = "", float bn_eps = 1e-5f);
  // Build from explicit host arrays (used by the native random-init path and tests).
  void build_raw(DeviceArena& arena, const std::vector<float>& w, const std::vector<float>& b,
                 int cout, int cin, const std::vector<ChanSeg>& in_segs, ConvSpec spec);

  int cout() const { return cout_; }
  int cin_padded() const { return cin_pad_; }
  int out_h(int h) const {
    return up_ ? 2 * h : (h + 2 * spec_.ph - spec_.dh * (spec_.kh - 1) - 1) / spec_.sh + 1;
  }
  int out_w(int w) const {
    return up_ ? 2 * w : (w + 2 * spec_.pw - spec_.dw * (spec_.kw - 1) - 1) / spec_.sw + 1;
  }
  int out_d(int d) const {
    if (spec_.kd <= 0) return 1;
    return up_ == 3 ? 2 * d : (d + 2 * spec_.pd - (spec_.kd - 1) - 1) / spec_.sd + 1;
  }

  // Fill launch args for inputs (channel-concatenated sources) -> output view.
  SaConvArgs args(const std::vector<Tensor>& srcs, const Tensor& out) const;
  void run(hipStream_t s, const std::vector<Tensor>& srcs, const Tensor& out, int act = SA_ACT_NONE,
           const Tensor* res = nullptr, int act2 = SA_ACT_NONE, sa_stat_t* stats = nullptr,
           float alpha = 0.01f, const sa_stat_t* in_stats = nullptr) const;  // in_stats: SaConvArgs.in_stats
  void launch(hipStream_t s, SaConvArgs& a) const;

 private:
  void upload(DeviceArena& arena, const std::vector<float>& w, const std::vector<float>& b, int cout,
              int cin, const std::vector<ChanSeg>& segs, int kd = 1);
  ConvSpec spec_;
  int cout_ = 0, cin_pad_ = 0, cin_real_ = 0, kpad_ = 0;
  int up_ = 0, cout_real_ = 0;  // transposed-conv parity scatter (2: 2-D, 3: 3-D)
  void* wdev_ = nullptr;
  float* bdev_ = nullptr;
};

// ------------------------------------------------------------------ graph capture
class GraphExec {
 public:
  ~GraphExec() { reset(); }
  template <typename F>
  void capture(hipStream_t s, F&& fn) {
    reset();
    HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    try {
      fn();
    } catch (...) {
      hipGraph_t g;
      (void)hipStreamEndCapture(s, &g);
      if (g) (void)hipGraphDestroy(g);
      throw;
    }
    HIP_CHECK(hipStreamEndCapture(s, &graph_));
    HIP_CHECK(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0));
  }
  void launch(hipStream_t s) const { HIP_CHECK(hipGraphLaunch(exec_, s)); }
  bool ready() const { return exec_ != nullptr; }
  hipGraphExec_t exec() const { return exec_; }
  void reset();

 private:
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
};

}  // namespace sa
