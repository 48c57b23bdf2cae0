// Tracing: roctx ranges around compute phases (visible in
// `rocprofv3 --marker-trace`), replacing the reference's Stopwatch-only
// instrumentation (Worker.cs:753-807) with timeline-level markers.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

#include <string>

namespace cek {

inline bool trace_enabled() {
  static const bool on = [] {
    const char* e = getenv("CEK_TRACE");
    return e && *e && *e != '0';
  }();
  return on;
}

struct TraceRange {
  bool on;
  explicit TraceRange(const std::string& name) : on(trace_enabled()) {
    if (on) roctxRangePushA(name.c_str());
  }
  ~TraceRange() {
    if (on) roctxRangePop();
  }
};

}  // namespace cek
