// Common runtime utilities for the MI355X stereo engine: status codes, HIP error checks,
// leveled logger.  Replaces the reference's assert-based CUDA_CHECK
// (RAFTStereo/include/TRTRAFTStereo.h:17-26) and the vendored TensorRT Logger
// (common/logging.h:201-435) with checks that are active in release builds.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <string>

namespace sa {

enum Status : int { kOk = 0, kError = -1 };

enum class LogLevel : int { kFatal = 0, kError = 1, kWarning = 2, kInfo = 3, kVerbose = 4 };

// Level comes from SA_LOG_LEVEL (0..4, default 2 = warning), same default severity as the
// reference logger (common/logging.h:204).
LogLevel log_level();
void log_msg(LogLevel lvl, const char* file, int line, const char* fmt, ...)
    __attribute__((format(printf, 4, 5)));

// Set by SA_DEBUG_SYNC=1: synchronize + check after every kernel launch (race/fault triage).
bool debug_sync_enabled();
// Fault injection for the error paths (SA_FAULT_INJECT=alloc|launch).
bool fault_inject(const char* what);

// roctx range (rocprofv3 --marker-trace shows it): engine build, tuning pass, frames
struct TraceRange {
  explicit TraceRange(const char* name);
  ~TraceRange();
};

}  // namespace sa

#define SA_LOG(lvl, ...)                                                        \
  do {                                                                          \
    if ((int)(lvl) <= (int)::sa::log_level()) ::sa::log_msg(lvl, __FILE__, __LINE__, __VA_ARGS__); \
  } while (0)
#define SA_LOGE(...) SA_LOG(::sa::LogLevel::kError, __VA_ARGS__)
#define SA_LOGW(...) SA_LOG(::sa::LogLevel::kWarning, __VA_ARGS__)
#define SA_LOGI(...) SA_LOG(::sa::LogLevel::kInfo, __VA_ARGS__)
#define SA_LOGV(...) SA_LOG(::sa::LogLevel::kVerbose, __VA_ARGS__)

// Always-on HIP check: logs file:line and throws (caught at the C ABI boundary, which turns
// it into a -1 status instead of the reference's silent assert).
#define HIP_CHECK(expr)                                                                   \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) {                                                               \
      ::sa::log_msg(::sa::LogLevel::kError, __FILE__, __LINE__, "HIP error %s: %s", #expr, \
                    hipGetErrorString(_e));                                               \
      throw ::sa::HipError(_e, #expr);                                                    \
    }                                                                                     \
  } while (0)

// Post-launch check (cheap: hipGetLastError) + optional full sync in debug mode.
#define SA_LAUNCH_CHECK(stream)                                          \
  do {                                                                   \
    HIP_CHECK(hipGetLastError());                                        \
    if (::sa::debug_sync_enabled()) HIP_CHECK(hipStreamSynchronize(stream)); \
  } while (0)

#define SA_REQUIRE(cond, ...)                                   \
  do {                                                          \
    if (!(cond)) {                                              \
      ::sa::log_msg(::sa::LogLevel::kError, __FILE__, __LINE__, __VA_ARGS__); \
      throw ::sa::Error(#cond);                                 \
    }                                                           \
  } while (0)

namespace sa {
struct Error : public std::exception {
  std::string msg;
  explicit Error(std::string m) : msg(std::move(m)) {}
  const char* what() const noexcept override { return msg.c_str(); }
};
struct HipError : public Error {
  hipError_t code;
  HipError(hipError_t c, const char* expr) : Error(std::string("hip: ") + expr), code(c) {}
};

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
inline int64_t ceil_div64(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int round_up(int a, int b) { return ceil_div(a, b) * b; }
}  // namespace sa
