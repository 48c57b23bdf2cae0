// Common definitions for the cekirdekler_amd native runtime (_cek).
//
// The runtime replaces the reference's out-of-tree OpenCL backend "KutuphaneCL"
// (its C ABI is the 135 DllImport sites, e.g. Cekirdekler/Cores.cs:39-49,
// Worker.cs:36-65, ClBuffer.cs:32-260) with a HIP-native core for MI355X
// (gfx950): hiprtc JIT, HIP streams/events, pinned host memory, RCCL.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace cek {

// Events that only time device work (compute spans, copy spans): no
// system-scope fence when they complete.  A default event's fence writes the
// L2 back and invalidates it between two back-to-back computes (≈10 µs of
// idle GPU per compute in enqueue mode); data reaches the host through the
// runtime's own copies and stream synchronisation, never through these.
constexpr unsigned kTimingEventFlags = hipEventDisableSystemFence;

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

[[noreturn]] void throw_hip(hipError_t e, const char* expr, const char* file, int line);

#define CEK_HIP(expr)                                         \
  do {                                                        \
    hipError_t _e = (expr);                                   \
    if (_e != hipSuccess) ::cek::throw_hip(_e, #expr, __FILE__, __LINE__); \
  } while (0)

// Device type codes (reference: ClPlatform.cs:47-65 CODE_CPU/GPU/ACC,
// AcceleratorType in ClNumberCruncher.cs:32-49).
enum DevType : int { kCPU = 1, kGPU = 2, kACC = 4 };

inline double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// Element-type codes shared with Python (ClArray dtype); sizes in bytes.
enum ElemType : int {
  kU8 = 0, kI8 = 1, kI16 = 2, kI32 = 3, kU32 = 4, kI64 = 5, kF32 = 6, kF64 = 7,
  kBF16 = 8, kF16 = 9, kU16 = 10, kU64 = 11
};

}  // namespace cek
