// StereoEngine: one model instance on one GPU, one HIP stream, static memory plan, whole-frame
// hipGraph.  Replaces the reference's per-model TensorRT wrappers (RAFTStereo/src/TRTRAFTStereo.cpp,
// HitNet/src/HitNet.cpp, CREStereo/src/TRTCREStereo.cpp, FastACVNet_plus/src/TRTFastACVNet_plus.cpp)
// with a single base class; per-model subclasses only describe the network.
//
// Per frame:  [remap (optional rectification)] -> model forward (incl. its fused preprocess)
//             -> reprojection (disparity -> XYZRGB with Q)  — all inside one captured graph.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "sa/hostcopy.h"
#include "sa/runtime.h"

namespace sa {

struct EngineConfig {
  std::string model;       // preset name (e.g. "raftstereo-realtime"); empty = from weights metadata
  std::string weights;     // .safetensors path; empty = deterministic random init (seed)
  int height = 480, width = 640, batch = 1;
  int iters = -1;          // override iteration count (RAFT / CREStereo); -1 = preset default
  int device = 0;
  bool use_graph = true;
  uint64_t seed = 0;
};

// Deterministic random-init helpers: in "random" mode missing weights are synthesised with the
// PyTorch default conv init (U(-1/sqrt(fan_in), +1/sqrt(fan_in))) and identity BatchNorm.
struct WeightSource {
  WeightStore* ws = nullptr;
  bool random = false;
  uint64_t seed = 0;
  void conv(const std::string& name, int cout, int cin, int kh, int kw, bool bias = true);
  void bn(const std::string& name, int c);
  void linear(const std::string& name, int out, int in, bool bias = true);
  void ln(const std::string& name, int c);
  void param(const std::string& name, std::vector<int64_t> shape, float lo, float hi);
};

struct StageTimes {
  float total_ms = 0;  // device time of the captured frame
};

class StereoEngine {
 public:
  virtual ~StereoEngine();
  static std::unique_ptr<StereoEngine> create(const EngineConfig& cfg);

  const EngineConfig& config() const { return cfg_; }
  virtual const char* name() const = 0;
  // Output the network produces before sign correction (RAFT flow is negative disparity).
  int H() const { return cfg_.height; }
  int W() const { return cfg_.width; }
  int B() const { return cfg_.batch; }

  // Q (4x4, row-major) for reprojection; rectification maps [2][H][W][2] (left, right).
  void set_Q(const float* q16);
  void set_rectify_maps(const float* maps_left, const float* maps_right);
  bool has_rectify() const { return rect_maps_ != nullptr; }

  // Device-side frame: u8 BGR [B][H][W][3] device pointers in, fp32 disparity [B][H][W] and
  // optional XYZRGB cloud [B][H][W][6] out (device pointers).  Runs on `stream` (the caller's) —
  // the engine's graph is launched there.  rectified_* (optional) receive the remapped inputs.
  void run_device(const uint8_t* left, const uint8_t* right, float* disp, float* cloud,
                  bool rectify, hipStream_t stream, uint8_t* rect_left = nullptr,
                  uint8_t* rect_right = nullptr);
  // Host-side frame = the reference's timed region (RAFTStereo/src/TRTRAFTStereo.cpp:119-146):
  // pinned staging, H2D, graph, D2H of disparity and point cloud, synchronise.
  void run_host(uint8_t* left, uint8_t* right, float* disp, float* cloud, bool rectify);
  // The pinned host staging run_host uses: inputs u8 BGR [B][H][W][3] x 2, disparity fp32 [B][H][W], cloud fp32
  // [B][H][W][6].  Passing these very pointers to run_host skips the pageable <-> pinned copies (a camera writes
  // frames straight into pinned memory, the D2H lands where the caller reads).  Valid for the engine's lifetime;
  // overwritten by the next run_host.
  void host_buffers(uint8_t** left, uint8_t** right, float** disp, float** cloud) const;
  // ms of the last run_host: [0] whole timed region, [1] input copies, [2] enqueue, [3] device wait + output
  // copies; with SA_HOST_TIMES=1 at engine creation also the device-side [4] H2D, [5] frame graph, [6] D2H
  const float* host_times() const { return host_times_; }
  bool host_times_device() const { return host_ev_[0] != nullptr; }  // SA_HOST_TIMES=1 split measured

  hipStream_t stream() const { return stream_; }
  // The engine stream handed to a caller that makes it its current stream (bench.py's data-parallel step): like
  // an exported copy stream it outlives the engine, since the caller's allocator may still hold blocks keyed to it.
  hipStream_t export_stream() const {
    main_exported_ = true;
    return stream_;
  }
  // The engine's side stream.  It only carries work while a frame is being captured (graph replays run every
  // branch from the instantiated graph), so between frames it is free for the caller's input copies: the
  // data-parallel step issues its H2D prefetch there instead of on a stream of its own, keeping a rank within
  // GPU_MAX_HW_QUEUES = 4 (engine, copy/side, caller, RCCL).  Once handed out, the stream outlives the engine
  // (see ~StereoEngine).
  hipStream_t copy_stream() const {
    side_exported_ = true;
    return side_;
  }
  size_t device_bytes() const { return arena_.bytes(); }
  // tuned-plan file used by this engine ("" = none) and how many conv shapes it had to time
  const std::string& plan_path() const { return plan_path_; }
  long tuned_shapes() const { return tuned_shapes_; }
  // the conv shapes this engine consulted during its tuning pass (what its frame graph launches)
  const std::vector<std::string>& plan_keys() const { return plan_keys_; }
  // plan file at build: entries loaded (-1 absent, -2 other library build, -3 not consulted); save result
  // (0 ok, errno of the failing step, -1 not attempted because nothing was tuned)
  int plan_loaded() const { return plan_loaded_; }
  int plan_saved() const { return plan_saved_; }
  // diagnostic: split-K tile counters that are not zero (every split conv's last arriver resets its
  // tiles' counters, so a non-zero one after a completed frame means two launches raced on them)
  long nonzero_splitk_counters();
  // low-resolution flow / auxiliary output (RAFT "diff" = coords1 - coords0), may be null
  virtual const float* aux_output(int* n) const {
    *n = 0;
    return nullptr;
  }
  long frames_run() const { return launches_per_frame_; }
  // Per-stage device times of the last frame in ms (SA_STAGE_TIMES=1 at engine creation): events
  // recorded at stage boundaries of the frame (event nodes of the captured graph).  Each entry is
  // (stage that ENDS at the mark, ms since the previous mark).  Empty when disabled.
  std::vector<std::pair<std::string, float>> stage_times() const;

 protected:
  explicit StereoEngine(const EngineConfig& cfg);
  void init();  // allocs io buffers, calls build(), warms up, captures
  // subclass hooks
  virtual void build(WeightSource& src) = 0;
  // consume in_left_/in_right_ (device u8 BGR, already rectified if requested), write disp_
  // (positive disparity, fp32 [B][H][W]).
  virtual void forward(hipStream_t s) = 0;

  // Activation taps (debugging / numerics bisection): with SA_TAP_DIR set and eager launches
  // (SA_NO_GRAPH=1) each tapped tensor is written to $SA_TAP_DIR/<name>.sat after the stream drains
  // (int32 header n,d,h,w,c,stride,dtype then the raw strided elements).  No-op otherwise.
  void tap(hipStream_t s, const char* name, const Tensor& t) const;
  void tap_f32(hipStream_t s, const char* name, const float* p, int n, int h, int w, int c) const;

  // Independent branches of a frame run on a second stream: fork() makes the side stream wait for
  // everything queued on `s` so far and returns it, join() makes `s` wait for the side stream.  Under
  // capture the two become parallel hipGraph branches.  Convs enqueued on the side stream must run
  // under ScopedSplitK(&splitk_side_) (split-K slabs / tile counters are per stream).
  hipStream_t fork(hipStream_t s);
  void join(hipStream_t s);
  // General dependency edges for deeper pipelines: record named event i on a stream / make a stream
  // wait for its latest record (reused across iterations: a wait binds to the record enqueued last).
  void rec(hipStream_t s, int i);
  void wait(hipStream_t s, int i);

  // stage boundary on the frame's main stream (no-op unless stage timing is on)
  void stage(hipStream_t s, const char* name);

  // the captured body; host_out: the reprojection writes the disparity and the cloud straight into pin_out_
  // host_in: the frame's first node copies the inputs from mapped host memory (in_src_) into the device buffers
  void frame(hipStream_t s, bool rectify, bool host_out = false, bool host_in = false);
  void launch_frame(hipStream_t s, bool rectify, bool host_out = false, bool host_in = false);

  EngineConfig cfg_;
  DeviceArena arena_;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
  std::unique_ptr<WeightStore> store_;
  uint8_t* in_left_ = nullptr;   // model input (rectified or raw copy)
  uint8_t* in_right_ = nullptr;
  uint8_t* raw_left_ = nullptr;  // pre-rectification staging
  uint8_t* raw_right_ = nullptr;
  float* disp_ = nullptr;
  float* cloud_ = nullptr;
  float* rect_maps_ = nullptr;  // [2][H][W][2]
  float Q_[16];
  bool have_Q_ = false;
  GraphExec graph_[8];  // [rectify + 2 * host_out + 4 * host_in]: host_out graphs reproject straight into host memory
  float* pin_out_dev_ = nullptr;  // device address of pin_out_ (kernels write the zero-copy outputs through it)
  // host-output frames: the reprojection node of each host-output graph (captured writing to the targets of the
  // frame that captured it) and the {disparity, cloud} device pointers it currently writes; a frame with other
  // targets re-points the node (sa_reproject_update_node) before the launch
  hipGraphNode_t repro_node_[8] = {};
  float* repro_ptrs_[8][2] = {};
  float* out_target_[2] = {};  // targets of the frame being launched (read by frame() at capture)
  // host-input frames: the input-copy node of each host_in graph and the {left, right} sources it reads
  hipGraphNode_t in_node_[8] = {};
  const uint8_t* in_ptrs_[8][2] = {};
  const uint8_t* in_src_[2] = {};  // device addresses of the mapped inputs of the frame being launched
  uint8_t* pin_in_dev_ = nullptr;
  // caller output buffers of run_host mapped for the GPU (hipHostRegister) once a buffer comes back for a second
  // frame: role 0 disparity, 1 cloud.  A different pointer for a role unregisters the previous one; all go with
  // the engine.  SA_HOST_REGISTER=0 disables (caller buffers are then filled from the pinned staging).
  struct HostReg {
    void* host = nullptr;
    size_t bytes = 0;
    void* dev = nullptr;
    bool failed = false;
  };
  HostReg host_reg_[4];  // roles 0 disparity, 1 cloud, 2 left input, 3 right input
  float* resolve_host_out(int role, void* p, size_t bytes);
  void* resolve_host_reg(int role, void* p, size_t bytes);
  void unregister_host(int role);
  std::string default_plan_path() const;
  std::string plan_path_;
  long tuned_shapes_ = 0;
  std::vector<std::string> plan_keys_;
  int plan_loaded_ = -3, plan_saved_ = -1;
  SplitKWorkspace splitk_;
  hipStream_t side_ = nullptr;
  mutable bool side_exported_ = false;  // copy_stream() was handed to a caller
  mutable bool main_exported_ = false;  // export_stream() was handed to a caller
  hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
  SplitKWorkspace splitk_side_;
  hipStream_t side2_ = nullptr;  // third stream for pipelined schedules
  SplitKWorkspace splitk_side2_;
  static constexpr int kEvents = 8;
  hipEvent_t ev_dep_[kEvents] = {};
  bool tuning_pass_ = false;
  static constexpr int kMaxStages = 16;
  bool stage_on_ = false;
  int nstage_ = 0;
  unsigned long long* stage_ts_ = nullptr;  // device wall-clock stamps [kMaxStages]
  const char* stage_name_[kMaxStages] = {};  // set during the eager conv-tuning forward (branches serialised)
  uint8_t* pin_in_ = nullptr;
  float* pin_out_ = nullptr;
  // run_host: chunked D2H (one event per chunk) copied out by a small thread pool as the chunks land
  static constexpr int kCopyEvents = 8;
  hipEvent_t ev_copy_[kCopyEvents] = {};
  hipEvent_t host_ev_[4] = {};  // SA_HOST_TIMES=1: timing events around H2D / graph / D2H
  float host_times_[8] = {};
  std::unique_ptr<HostCopyPool> copy_pool_;
  long launches_per_frame_ = 0;
};

// model factories (models/*.cpp)
std::unique_ptr<StereoEngine> make_raft_stereo(const EngineConfig& cfg);
std::unique_ptr<StereoEngine> make_crestereo(const EngineConfig& cfg);
std::unique_ptr<StereoEngine> make_hitnet(const EngineConfig& cfg);
std::unique_ptr<StereoEngine> make_fast_acvnet(const EngineConfig& cfg);

}  // namespace sa
