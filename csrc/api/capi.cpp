// Flat C API over the engine for the Python package (ctypes) and other FFI users.
// Every entry point catches C++ exceptions and returns a negative status; the last error
// message is retrievable with sa_last_error().
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "sa/algorithm.h"
#include "sa/capi.h"
#include "sa/engine.h"

namespace {
thread_local std::string g_err;
template <typename F>
int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    SA_LOGE("%s", e.what());
    return -1;
  } catch (...) {
    g_err = "unknown error";
    return -1;
  }
}
}  // namespace

extern "C" {

const char* sa_version(void) { return SA_VERSION_STRING; }

// sizeof of the launch-argument structs the Python ctypes layer mirrors (checked when the library is loaded, so a
// field added on one side only fails at import instead of shifting every later field)
long sa_struct_size(const char* name) {
  const std::string n = name ? name : "";
  if (n == "SaConvArgs") return (long)sizeof(SaConvArgs);
  if (n == "SaNormArgs") return (long)sizeof(SaNormArgs);
  if (n == "SaAgclArgs") return (long)sizeof(SaAgclArgs);
  if (n == "SaEwArgs") return (long)sizeof(SaEwArgs);
  if (n == "SaConvSrc") return (long)sizeof(SaConvSrc);
  return -1;
}
const char* sa_last_error(void) { return g_err.c_str(); }

void* sa_engine_create(const char* model, const char* weights, int height, int width, int batch,
                       int iters, int device, int use_graph, unsigned long long seed) {
  sa::StereoEngine* out = nullptr;
  int rc = guarded([&] {
    sa::EngineConfig cfg;
    cfg.model = model ? model : "";
    cfg.weights = weights ? weights : "";
    cfg.height = height;
    cfg.width = width;
    cfg.batch = batch;
    cfg.iters = iters;
    cfg.device = device;
    cfg.use_graph = use_graph != 0;
    cfg.seed = seed;
    out = sa::StereoEngine::create(cfg).release();
  });
  return rc == 0 ? out : nullptr;
}

void sa_engine_destroy(void* e) { delete static_cast<sa::StereoEngine*>(e); }

int sa_engine_set_q(void* e, const float* q16) {
  return guarded([&] { static_cast<sa::StereoEngine*>(e)->set_Q(q16); });
}

int sa_engine_set_rectify_maps(void* e, const float* ml, const float* mr) {
  return guarded([&] { static_cast<sa::StereoEngine*>(e)->set_rectify_maps(ml, mr); });
}

int sa_engine_run_device(void* e, const void* left, const void* right, float* disp, float* cloud,
                         int rectify, void* stream, void* rect_left, void* rect_right) {
  return guarded([&] {
    static_cast<sa::StereoEngine*>(e)->run_device((const uint8_t*)left, (const uint8_t*)right, disp,
                                                  cloud, rectify != 0, (hipStream_t)stream,
                                                  (uint8_t*)rect_left, (uint8_t*)rect_right);
  });
}

int sa_engine_run_host(void* e, void* left, void* right, float* disp, float* cloud, int rectify) {
  return guarded([&] {
    static_cast<sa::StereoEngine*>(e)->run_host((uint8_t*)left, (uint8_t*)right, disp, cloud,
                                                rectify != 0);
  });
}

void sa_engine_host_buffers(void* e, void** left, void** right, float** disp, float** cloud) {
  static_cast<sa::StereoEngine*>(e)->host_buffers((uint8_t**)left, (uint8_t**)right, disp, cloud);
}
int sa_engine_host_times(void* e, float* out, int max) {
  // the device-side split (h2d / graph / d2h) exists only for engines created with SA_HOST_TIMES=1; without it
  // only the 4 host-clock entries are returned, so unmeasured device times are never reported as 0
  auto* eng = static_cast<sa::StereoEngine*>(e);
  const float* t = eng->host_times();
  const int avail = eng->host_times_device() ? 7 : 4;
  int n = 0;
  for (; n < max && n < avail; ++n) out[n] = t[n];
  return n;
}
void* sa_engine_copy_stream(void* e) { return static_cast<sa::StereoEngine*>(e)->copy_stream(); }
long long sa_engine_device_bytes(void* e) {
  return (long long)static_cast<sa::StereoEngine*>(e)->device_bytes();
}

const float* sa_engine_aux_output(void* e, int* n) {
  return static_cast<sa::StereoEngine*>(e)->aux_output(n);
}

const char* sa_engine_plan_path(void* e) { return static_cast<sa::StereoEngine*>(e)->plan_path().c_str(); }
long sa_engine_tuned_shapes(void* e) { return static_cast<sa::StereoEngine*>(e)->tuned_shapes(); }
// plan file at build: *loaded = entries loaded (-1 absent, -2 written by another library build, -3 not consulted),
// *saved = 0 ok / errno of the failed write / -1 not attempted (nothing tuned)
void sa_engine_plan_status(void* e, int* loaded, int* saved) {
  *loaded = static_cast<sa::StereoEngine*>(e)->plan_loaded();
  *saved = static_cast<sa::StereoEngine*>(e)->plan_saved();
}
const char* sa_plan_build_id() { return sa::conv_plan_build_id().c_str(); }
// digest of the tactics this engine's graph launches (from the process plan, not a file: VERDICT r5 / ADVICE r5)
const char* sa_engine_tactics_digest(void* e) {
  static thread_local std::string d;
  d = sa::conv_plan_digest(static_cast<sa::StereoEngine*>(e)->plan_keys());
  return d.c_str();
}
// write this engine's plan entries to `file` (a DP job's rank 0 broadcasts those bytes); 0 or errno
int sa_engine_plan_export(void* e, const char* file) {
  return sa::conv_plan_save(file, static_cast<sa::StereoEngine*>(e)->plan_keys());
}
void sa_conv_plan_pin(int on) { sa::conv_plan_pin(on != 0); }
long sa_engine_nonzero_splitk_counters(void* e) { return static_cast<sa::StereoEngine*>(e)->nonzero_splitk_counters(); }
long sa_conv_tune_count(void) { return sa::conv_tune_count(); }
long sa_conv_tune_rejects(void) { return sa::conv_tune_rejects(); }
void sa_conv_plan_clear(void) { sa::conv_plan_clear(); }
// plan-file round trip without a GPU (tests pin the on-disk format the native writer produces): put seeds the
// in-process plan, save writes the entries of the newline-separated `keys`, load merges a file (-1 absent, -2 stale)
void sa_conv_plan_put(const char* key, int cfg, int splitk, float us) { sa::conv_plan_put(key, cfg, splitk, us); }
int sa_conv_plan_save(const char* file, const char* keys) {
  std::vector<std::string> k;
  std::string cur;
  for (const char* p = keys; ; ++p) {
    if (*p == '\n' || *p == 0) {
      if (!cur.empty()) k.push_back(cur);
      cur.clear();
      if (*p == 0) break;
    } else {
      cur += *p;
    }
  }
  return sa::conv_plan_save(file, k);
}
int sa_conv_plan_load(const char* file) { return sa::conv_plan_load(file); }
void sa_conv_plan_cache_append(const char* key, int cfg, int splitk, float us) {
  sa::conv_plan_cache_append(key, cfg, splitk, us);
}
long sa_conv_plan_entries(void) { return (long)sa::conv_plan_entries(); }

void* sa_engine_stream(void* e) { return (void*)static_cast<sa::StereoEngine*>(e)->export_stream(); }

int sa_engine_stage_times(void* e, float* ms, const char** names, int max) {
  static thread_local std::vector<std::string> keep;
  int n = -1;
  const int rc = guarded([&] {
    auto st = static_cast<sa::StereoEngine*>(e)->stage_times();
    keep.clear();
    for (auto& p : st) keep.push_back(p.first);
    n = 0;
    for (size_t i = 0; i < st.size() && (int)i < max; ++i, ++n) {
      ms[i] = st[i].second;
      names[i] = keep[i].c_str();
    }
  });
  return rc == 0 ? n : -1;
}

void* sa_algorithm_create(const char* model, int gpu_id, const char* calibration_path, const char* default_preset) {
  auto* a = new sa::StereoAlgorithm();
  if (a->Initialize(model ? model : "", gpu_id, calibration_path ? calibration_path : "",
                    default_preset ? default_preset : "") != 0) {
    g_err = a->last_error();
    delete a;
    return nullptr;
  }
  return a;
}

int sa_algorithm_frame_size(void* alg, int* rows, int* cols) {
  auto* a = static_cast<sa::StereoAlgorithm*>(alg);
  if (!a || !a->initialized()) {
    g_err = "not initialized";
    return -1;
  }
  *rows = a->height();
  *cols = a->width();
  return 0;
}

int sa_algorithm_run(void* alg, unsigned char* left, unsigned char* right, int rows, int cols, float* disparity,
                     float* cloud, int rectify) {
  auto* a = static_cast<sa::StereoAlgorithm*>(alg);
  if (!a) {
    g_err = "null algorithm handle";
    return -1;
  }
  int rc = -1;
  const int g = guarded([&] {
    sa::Mat l(rows, cols, sa::SA_8UC3, left), r(rows, cols, sa::SA_8UC3, right), d;
    std::vector<float> scratch;
    float* pc = cloud;
    if (!pc) {  // the facade always reprojects; a caller that does not want the cloud gets it discarded
      scratch.resize((size_t)rows * cols * 6);
      pc = scratch.data();
    }
    rc = a->Run(l, r, pc, d, rectify != 0);
    if (rc != 0) {
      g_err = a->last_error();
      return;
    }
    for (int y = 0; y < rows; ++y) std::memcpy(disparity + (size_t)y * cols, d.ptr<float>(y), (size_t)cols * 4);
  });
  return g != 0 ? g : rc;
}

float sa_algorithm_last_ms(void* alg) {
  if (!alg) {
    g_err = "null algorithm handle";
    return -1.f;
  }
  return static_cast<sa::StereoAlgorithm*>(alg)->last_ms();
}

void sa_algorithm_destroy(void* alg) { delete static_cast<sa::StereoAlgorithm*>(alg); }

}  // extern "C"
