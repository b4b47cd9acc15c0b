// Reusable network blocks built on ConvLayer: residual blocks with batch (folded) / instance /
// no normalisation, and the instance-norm statistics pool.
#pragma once
#include <cstdlib>
#include <string>
#include <vector>

#include "sa/engine.h"

namespace sa {

enum class Norm { None, Batch, Instance };
Norm parse_norm(const std::string& s);

// Per-forward instance-norm statistics (fixed-point {sum, sumsq} per (n, c)), zeroed by one memset.
class StatsPool {
 public:
  sa_stat_t* take(int n, int c) {
    size_t need = (size_t)kStatSlots * n * c * 2;
    reserve_.push_back(need);
    offs_.push_back(total_);
    total_ += need;
    return reinterpret_cast<sa_stat_t*>((size_t)offs_.size());  // placeholder resolved in finalize
  }
  void finalize(DeviceArena& a) {
    base_ = (sa_stat_t*)a.alloc(std::max<size_t>(total_, 1) * sizeof(sa_stat_t));
  }
  sa_stat_t* resolve(sa_stat_t* handle) const {
    if (!handle) return nullptr;
    size_t idx = (size_t)handle - 1;
    return base_ + offs_[idx];
  }
  void zero(hipStream_t s) const { device_zero(base_, std::max<size_t>(total_, 1) * sizeof(sa_stat_t), s); }

 private:
  std::vector<size_t> reserve_, offs_;
  size_t total_ = 0;
  sa_stat_t* base_ = nullptr;
};

// ResidualBlock of RAFT-Stereo / CREStereo extractors (upstream core/extractor.py):
//   y = relu(norm1(conv1(x))); y = relu(norm2(conv2(y))); x' = downsample(x) if needed;
//   out = relu(x' + y)
struct ResBlock {
  ConvLayer c1, c2, down;
  bool has_down = false;
  Norm norm = Norm::None;
  // instance norm folded into the direct 64-channel convs (fold_in_enabled(), 64 -> 64 stride 1 blocks): conv2 reads
  // conv1's raw output y1 (no a1 pass); with x_raw (set before build) the block input x is itself a raw conv output
  // whose statistics run() receives -- conv1 and the residual apply normalise it on the fly
  bool fold = false, x_raw = false;
  Tensor y1, a1, y2, yd, out;
  sa_stat_t *st1 = nullptr, *st2 = nullptr, *std_ = nullptr;  // StatsPool handles
  // plan != nullptr: the block's activations are declared in `plan` (lifetimes in run() order, x =
  // the block input) instead of being allocated; the caller commits the plan
  void build(DeviceArena& a, WeightSource& src, StatsPool& sp, const std::string& prefix, int in_planes,
             int planes, int stride, Norm norm, int N, int H, int W, ActPlan* plan = nullptr,
             const Tensor* x = nullptr);
  void run(hipStream_t s, const StatsPool& sp, const Tensor& x, const sa_stat_t* x_stats = nullptr) const;
};

// SA_FOLD_IN (default on): fold the instance-norm applies that feed a direct 64-channel conv into that conv
bool fold_in_enabled();

// BasicEncoder / MultiBasicEncoder trunk shared by RAFT-Stereo and CREStereo (upstream
// core/extractor.py): conv1 7x7 (stride s1) + norm + ReLU, then layer1..3 of two residual
// blocks each (dims 64/96/128, first block of each layer strided).
struct Trunk {
  ConvLayer conv1;
  Norm norm = Norm::None;
  Tensor c1y, c1a;
  sa_stat_t* c1st = nullptr;
  bool stem_fold = false;  // relu(IN(conv1)) never materialised: layer1.0 reads c1y raw (ResBlock::x_raw)
  std::vector<ResBlock> layers;
  void build(DeviceArena& a, WeightSource& src, StatsPool& sp, const std::string& prefix, Norm norm, int N, int H,
             int W, int conv1_stride, const int strides[3]);
  void run(hipStream_t s, const StatsPool& sp, const Tensor& img) const;
  // the trunk in steps (0: conv1 [+ norm], k >= 1: residual layer k - 1), for interleaving two trunks' launches
  int steps() const { return 1 + (int)layers.size(); }
  void run_step(hipStream_t s, const StatsPool& sp, const Tensor& img, int k) const;
  const Tensor& out() const { return layers.back().out; }
};

// norm apply helper
void instnorm(hipStream_t s, const Tensor& x, const sa_stat_t* stats, const Tensor& out, int act,
              const Tensor* res = nullptr, const sa_stat_t* res_stats = nullptr, int act2 = SA_ACT_NONE,
              int res_act = SA_ACT_NONE);

}  // namespace sa
