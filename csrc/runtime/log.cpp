// Leveled logger with the reference's [F]/[E]/[W]/[I]/[V] prefixes and timestamp
// (common/logging.h:71-80, 374-385), configured by environment instead of code.
#include "sa/common.h"

#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>

#include <rocprofiler-sdk-roctx/roctx.h>

namespace sa {

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  return std::atoi(v);
}

LogLevel log_level() {
  static const int lvl = env_int("SA_LOG_LEVEL", 2);
  return (LogLevel)lvl;
}

bool debug_sync_enabled() {
  static const bool on = env_int("SA_DEBUG_SYNC", 0) != 0;
  return on;
}

bool fault_inject(const char* what) {
  const char* v = std::getenv("SA_FAULT_INJECT");
  return v && std::strcmp(v, what) == 0;
}

TraceRange::TraceRange(const char* name) { roctxRangePushA(name); }
TraceRange::~TraceRange() { roctxRangePop(); }

void log_msg(LogLevel lvl, const char* file, int line, const char* fmt, ...) {
  static std::mutex mu;
  static const char* tags[] = {"[F]", "[E]", "[W]", "[I]", "[V]"};
  char buf[2048];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  auto now = std::chrono::system_clock::now();
  std::time_t t = std::chrono::system_clock::to_time_t(now);
  std::tm tm{};
  localtime_r(&t, &tm);
  char ts[32];
  std::strftime(ts, sizeof(ts), "%m/%d/%Y-%H:%M:%S", &tm);
  const char* base = std::strrchr(file, '/');
  base = base ? base + 1 : file;
  std::lock_guard<std::mutex> g(mu);
  std::fprintf(stderr, "[%s] %s %s:%d %s\n", ts, tags[(int)lvl < 5 ? (int)lvl : 4], base, line, buf);
}

}  // namespace sa
