// Device arena, safetensors reader, conv weight packing, graph helper.
#include "sa/runtime.h"

#include <cmath>
#include <cstring>
#include <fstream>

#include "sa/json.h"

namespace sa {

// ------------------------------------------------------------------ arena
DeviceArena::~DeviceArena() { release(); }

void* DeviceArena::alloc(size_t bytes) {
  if (fault_inject("alloc")) throw Error("fault injection: alloc");
  bytes = (bytes + 255) & ~(size_t)255;
  if (bytes == 0) bytes = 256;
  void* p = nullptr;
  HIP_CHECK(hipMalloc(&p, bytes));
  HIP_CHECK(hipMemset(p, 0, bytes));
  ptrs_.push_back(p);
  total_ += bytes;
  return p;
}

void DeviceArena::release() {
  for (void* p : ptrs_) (void)hipFree(p);
  ptrs_.clear();
  total_ = 0;
}

Tensor make_tensor(DeviceArena& a, int n, int h, int w, int c, DT dt, int stride) {
  Tensor t;
  t.n = n;
  t.h = h;
  t.w = w;
  t.c = c;
  t.stride = stride < 0 ? c : stride;
  t.dt = dt;
  t.ptr = a.alloc(t.nbytes());
  return t;
}

// ------------------------------------------------------------------ safetensors
static float half_to_float(uint16_t h) {
  uint32_t sign = (h >> 15) & 1, exp = (h >> 10) & 0x1f, mant = h & 0x3ff;
  float v;
  if (exp == 0) v = std::ldexp((float)mant, -24);
  else if (exp == 31) v = mant ? NAN : INFINITY;
  else v = std::ldexp((float)(mant | 0x400), (int)exp - 25);
  return sign ? -v : v;
}

std::unique_ptr<WeightStore> WeightStore::load_safetensors(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  SA_REQUIRE(f.good(), "cannot open weights file %s", path.c_str());
  uint64_t hlen = 0;
  f.read(reinterpret_cast<char*>(&hlen), 8);
  SA_REQUIRE(f.good() && hlen > 0 && hlen < (1ull << 30), "bad safetensors header in %s", path.c_str());
  std::string header(hlen, '\0');
  f.read(&header[0], (std::streamsize)hlen);
  f.seekg(0, std::ios::end);
  const uint64_t fsize = (uint64_t)f.tellg();
  const uint64_t base = 8 + hlen;
  json::Value root = json::parse(header);
  SA_REQUIRE(root.is_object(), "safetensors header is not an object");
  auto ws = std::make_unique<WeightStore>();
  for (const auto& kv : root.obj) {
    if (kv.first == "__metadata__") {
      for (const auto& m : kv.second.obj) ws->meta_[m.first] = m.second.str;
      continue;
    }
    const json::Value& d = kv.second;
    const std::string dtype = d.at("dtype").str;
    HostTensor t;
    for (const auto& s : d.at("shape").arr) t.shape.push_back((int64_t)s.num);
    const auto& offs = d.at("data_offsets").arr;
    uint64_t b0 = (uint64_t)offs.at(0).num, b1 = (uint64_t)offs.at(1).num;
    SA_REQUIRE(base + b1 <= fsize && b0 <= b1, "tensor %s out of file bounds", kv.first.c_str());
    std::vector<char> raw(b1 - b0);
    f.seekg((std::streamoff)(base + b0));
    f.read(raw.data(), (std::streamsize)raw.size());
    int64_t n = t.numel();
    t.data.resize(n);
    if (dtype == "F32") {
      SA_REQUIRE((int64_t)raw.size() == n * 4, "size mismatch %s", kv.first.c_str());
      std::memcpy(t.data.data(), raw.data(), raw.size());
    } else if (dtype == "F16") {
      SA_REQUIRE((int64_t)raw.size() == n * 2, "size mismatch %s", kv.first.c_str());
      const uint16_t* p = reinterpret_cast<const uint16_t*>(raw.data());
      for (int64_t i = 0; i < n; ++i) t.data[i] = half_to_float(p[i]);
    } else if (dtype == "BF16") {
      SA_REQUIRE((int64_t)raw.size() == n * 2, "size mismatch %s", kv.first.c_str());
      const uint16_t* p = reinterpret_cast<const uint16_t*>(raw.data());
      for (int64_t i = 0; i < n; ++i) {
        uint32_t u = (uint32_t)p[i] << 16;
        std::memcpy(&t.data[i], &u, 4);
      }
    } else if (dtype == "I64" || dtype == "I32") {
      // integer buffers (e.g. BatchNorm num_batches_tracked) are not needed for inference
      continue;
    } else {
      throw Error("unsupported safetensors dtype " + dtype);
    }
    ws->t_[kv.first] = std::move(t);
  }
  return ws;
}

const HostTensor& WeightStore::get(const std::string& name) const {
  auto it = t_.find(name);
  if (it == t_.end()) throw Error("missing weight: " + name);
  return it->second;
}

std::string WeightStore::meta(const std::string& key, const std::string& dflt) const {
  auto it = meta_.find(key);
  return it == meta_.end() ? dflt : it->second;
}

// ------------------------------------------------------------------ conv packing
static uint16_t float_to_half(float f) {
  _Float16 h = (_Float16)f;
  uint16_t u;
  std::memcpy(&u, &h, 2);
  return u;
}

void ConvLayer::upload(DeviceArena& arena, const std::vector<float>& w, const std::vector<float>& b,
                       int cout, int cin, const std::vector<ChanSeg>& segs) {
  int real_sum = 0, pad_sum = 0;
  for (auto s : segs) {
    real_sum += s.real;
    pad_sum += s.padded;
    SA_REQUIRE(s.padded % 8 == 0 && s.padded >= s.real, "bad channel segment");
  }
  SA_REQUIRE(real_sum == cin, "conv input segments (%d) != checkpoint Cin (%d)", real_sum, cin);
  cout_ = cout;
  cin_pad_ = pad_sum;
  const int KH = spec_.kh, KW = spec_.kw;
  const int K = KH * KW * cin_pad_;
  kpad_ = round_up(K, 64);  // 64-aligned K enables the DMA-staged BK=64 conv path
  const int cout_pad = round_up(cout, 128);
  std::vector<uint16_t> packed((size_t)cout_pad * kpad_, 0);
  // padded channel -> real channel index (or -1)
  std::vector<int> cmap(cin_pad_, -1);
  {
    int pc = 0, rc = 0;
    for (auto s : segs) {
      for (int i = 0; i < s.padded; ++i) cmap[pc + i] = i < s.real ? rc + i : -1;
      pc += s.padded;
      rc += s.real;
    }
  }
  for (int o = 0; o < cout; ++o)
    for (int y = 0; y < KH; ++y)
      for (int x = 0; x < KW; ++x)
        for (int c = 0; c < cin_pad_; ++c) {
          int rc = cmap[c];
          float v = rc < 0 ? 0.f : w[(((size_t)o * cin + rc) * KH + y) * KW + x];
          packed[(size_t)o * kpad_ + (y * KW + x) * cin_pad_ + c] = float_to_half(v);
        }
  wdev_ = arena.alloc(packed.size() * 2);
  HIP_CHECK(hipMemcpy(wdev_, packed.data(), packed.size() * 2, hipMemcpyHostToDevice));
  std::vector<float> bias(round_up(cout, 8), 0.f);
  for (int o = 0; o < cout && o < (int)b.size(); ++o) bias[o] = b[o];
  bdev_ = (float*)arena.alloc(bias.size() * 4);
  HIP_CHECK(hipMemcpy(bdev_, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
}

void ConvLayer::build(DeviceArena& arena, const WeightStore& ws,
                      const std::vector<std::string>& wnames, const std::vector<ChanSeg>& in_segs,
                      ConvSpec spec, const std::vector<std::string>& bn_names, float scale,
                      float bn_eps) {
  std::vector<float> W, Bv;
  int cout = 0, cin = -1, kh = -1, kw = -1;
  for (size_t i = 0; i < wnames.size(); ++i) {
    const HostTensor& wt = ws.get(wnames[i] + ".weight");
    SA_REQUIRE(wt.shape.size() == 4, "%s: expected 4-D conv weight", wnames[i].c_str());
    int co = (int)wt.shape[0], ci = (int)wt.shape[1];
    if (cin < 0) {
      cin = ci;
      kh = (int)wt.shape[2];
      kw = (int)wt.shape[3];
    }
    SA_REQUIRE(ci == cin && kh == wt.shape[2] && kw == wt.shape[3], "stacked conv shape mismatch");
    std::vector<float> w = wt.data;
    std::vector<float> b(co, 0.f);
    if (ws.has(wnames[i] + ".bias")) b = ws.get(wnames[i] + ".bias").data;
    if (i < bn_names.size() && !bn_names[i].empty()) {
      const auto& g = ws.get(bn_names[i] + ".weight").data;
      const auto& be = ws.get(bn_names[i] + ".bias").data;
      const auto& mu = ws.get(bn_names[i] + ".running_mean").data;
      const auto& var = ws.get(bn_names[i] + ".running_var").data;
      const int per = ci * kh * kw;
      for (int o = 0; o < co; ++o) {
        float s = g[o] / std::sqrt(var[o] + bn_eps);
        for (int j = 0; j < per; ++j) w[(size_t)o * per + j] *= s;
        b[o] = (b[o] - mu[o]) * s + be[o];
      }
    }
    if (scale != 1.f) {
      for (auto& v : w) v *= scale;
      for (auto& v : b) v *= scale;
    }
    W.insert(W.end(), w.begin(), w.end());
    Bv.insert(Bv.end(), b.begin(), b.end());
    cout += co;
  }
  spec.kh = kh;
  spec.kw = kw;
  if (spec.ph < 0) spec.ph = (kh / 2) * spec.dh;
  if (spec.pw < 0) spec.pw = (kw / 2) * spec.dw;
  spec_ = spec;
  upload(arena, W, Bv, cout, cin, in_segs);
}

void ConvLayer::build_raw(DeviceArena& arena, const std::vector<float>& w, const std::vector<float>& b,
                          int cout, int cin, const std::vector<ChanSeg>& in_segs, ConvSpec spec) {
  if (spec.ph < 0) spec.ph = (spec.kh / 2) * spec.dh;
  if (spec.pw < 0) spec.pw = (spec.kw / 2) * spec.dw;
  spec_ = spec;
  upload(arena, w, b, cout, cin, in_segs);
}

SaConvArgs ConvLayer::args(const std::vector<Tensor>& srcs, const Tensor& out) const {
  SaConvArgs a;
  std::memset(&a, 0, sizeof(a));
  SA_REQUIRE(!srcs.empty() && srcs.size() <= 4, "conv needs 1..4 sources");
  int cin = 0;
  for (size_t i = 0; i < srcs.size(); ++i) {
    const Tensor& s = srcs[i];
    SA_REQUIRE(s.dt == DT::F16 && s.c % 8 == 0 && s.stride % 8 == 0, "conv source must be fp16, 8-aligned");
    SA_REQUIRE(s.n == srcs[0].n && s.h == srcs[0].h && s.w == srcs[0].w, "conv sources differ in shape");
    a.src[i].ptr = s.ptr;
    a.src[i].channels = s.c;
    a.src[i].stride = s.stride;
    cin += s.c;
  }
  SA_REQUIRE(cin == cin_pad_, "conv input channels %d != packed %d", cin, cin_pad_);
  a.nsrc = (int)srcs.size();
  a.N = srcs[0].n;
  a.H = srcs[0].h;
  a.W = srcs[0].w;
  a.Cin = cin;
  a.KH = spec_.kh;
  a.KW = spec_.kw;
  a.sh = spec_.sh;
  a.sw = spec_.sw;
  a.ph = spec_.ph;
  a.pw = spec_.pw;
  a.dh = spec_.dh;
  a.dw = spec_.dw;
  a.Ho = out_h(a.H);
  a.Wo = out_w(a.W);
  SA_REQUIRE(out.n == a.N && out.h == a.Ho && out.w == a.Wo, "conv output shape mismatch (%dx%dx%d vs %dx%dx%d)",
             out.n, out.h, out.w, a.N, a.Ho, a.Wo);
  a.weight = wdev_;
  a.bias = bdev_;
  a.Cout = cout_;
  a.Kpad = kpad_;
  a.out = out.ptr;
  a.out_stride = out.stride;
  a.epi = out.dt == DT::F32 ? SA_EPI_STORE_F32 : SA_EPI_STORE;
  a.scale = 1.f;
  a.alpha = 0.01f;
  a.tile_cfg = -1;
  if (const SplitKWorkspace* sk = current_splitk()) {
    a.splitk = 0;  // auto
    a.ws = sk->ws;
    a.counters = sk->counters;
    a.ws_floats = sk->ws_floats;
    a.n_counters = sk->n_counters;
  } else {
    a.splitk = 1;
  }
  return a;
}

void ConvLayer::launch(hipStream_t s, SaConvArgs& a) const {
  if (fault_inject("launch")) throw Error("fault injection: launch");
  int rc = sa_conv2d(&a, s);
  SA_REQUIRE(rc == 0, "sa_conv2d failed rc=%d", rc);
  SA_LAUNCH_CHECK(s);
}

void ConvLayer::run(hipStream_t s, const std::vector<Tensor>& srcs, const Tensor& out, int act,
                    const Tensor* res, int act2, sa_stat_t* stats, float alpha) const {
  SaConvArgs a = args(srcs, out);
  SA_REQUIRE(out.c >= cout_ || stats == nullptr, "conv output view too narrow");
  a.act = act;
  a.alpha = alpha;
  if (res) {
    a.res = res->ptr;
    a.res_stride = res->stride;
    a.act2 = act2;
  }
  a.stats = stats;
  launch(s, a);
}

static thread_local const SplitKWorkspace* g_splitk = nullptr;
const SplitKWorkspace* current_splitk() { return g_splitk; }
ScopedSplitK::ScopedSplitK(const SplitKWorkspace* w) : prev(g_splitk) { g_splitk = w; }
ScopedSplitK::~ScopedSplitK() { g_splitk = prev; }

void SplitKWorkspace::alloc(DeviceArena& a, int64_t floats, int32_t ncnt) {
  ws = (float*)a.alloc((size_t)floats * 4);
  counters = (int32_t*)a.alloc((size_t)ncnt * 4);
  HIP_CHECK(hipMemset(counters, 0, (size_t)ncnt * 4));
  ws_floats = floats;
  n_counters = ncnt;
}

void GraphExec::reset() {
  if (exec_) (void)hipGraphExecDestroy(exec_);
  if (graph_) (void)hipGraphDestroy(graph_);
  exec_ = nullptr;
  graph_ = nullptr;
}

}  // namespace sa
