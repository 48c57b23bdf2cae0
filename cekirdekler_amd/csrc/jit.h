// Kernel-source JIT: hiprtc for gfx950, host compiler + dlopen for the CPU
// device.  Replaces the reference's per-device clBuildProgram path
// (ClProgram.cs:59-69, createProgram/getProgramErr/readProgramErrString) and
// the kernel-name regex of ClNumberCruncher.cs:218-228.
//
// Source contract (HIP C++ kernel strings):
//   extern "C" optional; every `__global__ void NAME(array params...)` is a
//   kernel.  The runtime appends two hidden parameters to each kernel,
//   `long long __cek_off, long long __cek_gsize`, so a range-partitioned
//   launch sees absolute OpenCL-style ids (the reference relies on
//   clEnqueueNDRangeKernel's global offset, Worker.cs:1033-1038).
//   Prelude helpers: get_global_id(0), get_local_id(0), get_group_id(0)
//   (device-local, OpenCL semantics), get_global_offset(0), get_global_size(0),
//   get_local_size(0), get_num_groups(0), cek_global_group_id().
//   An OpenCL-C dialect (`__kernel void`, `__global`, `__local`,
//   `barrier(CLK_LOCAL_MEM_FENCE)`) is accepted and rewritten to HIP.
#pragma once
#include "common.h"
#include "device.h"

#include <map>
#include <unordered_map>
#include <mutex>
#include <set>

namespace cek {

struct KernelSig {
  std::string name;
  int arity = 0;  // number of user (array) parameters
};

// Kernel names in source order (duplicates removed).
std::vector<KernelSig> parse_kernels(const std::string& src);
// True when the source is written in the OpenCL-C dialect.
bool is_opencl_dialect(const std::string& src);
// Source after dialect translation + hidden-argument rewrite + GPU prelude.
std::string gpu_rewrite(const std::string& src);
// Source after dialect translation + CPU prelude + per-kernel runner stubs.
std::string cpu_rewrite(const std::string& src);

// Per-item CPU runner signature generated for each kernel:
//   runs items [first, first+count) of a launch with local size L,
//   hidden offset `off` and global size `gsize`; `args` are array pointers.
using CpuRunner = void (*)(void** args, long long off, long long gsize, long long first,
                           long long count, int L);

// A compiled program for one device.
class Program {
 public:
  // src may be empty when only prebuilt code objects are used.
  static std::shared_ptr<Program> build(const DeviceInfo& dev, const std::string& src,
                                        const std::vector<std::string>& options,
                                        const std::vector<std::string>& prebuilt);
  ~Program();

  bool ok() const { return ok_; }
  const std::string& log() const { return log_; }
  const std::vector<KernelSig>& kernels() const { return kernels_; }
  // user-parameter count of a kernel (-1: unknown name or unparsed), by a
  // hash lookup (compute() checks it on every call)
  int arity(const std::string& name) const;
  bool has(const std::string& name) const;
  hipFunction_t gpu_fn(const std::string& name) const;
  CpuRunner cpu_fn(const std::string& name) const;
  int device_type() const { return type_; }
  double build_ms() const { return build_ms_; }
  // Device-side enqueue (cek_enqueue in the source): kernels take the queue
  // and level as extra hidden arguments, and a kernel that enqueues has a
  // generated "__cek_dispatch_<name>" that runs one level of child launches.
  bool dynamic() const { return dynamic_; }
  bool has_dispatcher(const std::string& kernel) const { return dispatchers_.count(kernel) > 0; }

 private:
  bool dynamic_ = false;
  std::set<std::string> dispatchers_;
  int type_ = kGPU;
  bool ok_ = false;
  std::string log_;
  double build_ms_ = 0;
  std::vector<KernelSig> kernels_;
  std::vector<hipModule_t> modules_;
  std::map<std::string, hipFunction_t> gpu_fns_;
  mutable std::mutex arity_mu_;
  mutable std::unordered_map<std::string, int> arity_;  // built from kernels_ on first use
  void* dl_ = nullptr;
  std::map<std::string, CpuRunner> cpu_fns_;
};

// Device-side enqueue: levels (parent = level 0) and records per level of
// the per-device queue; layout shared with the generated prelude.
constexpr int kDynLevels = 4;
constexpr int kDynCap = 16384;
constexpr size_t kDynHeaderBytes = 64;  // int count[8]; int errors; pad
constexpr size_t kDynQueueBytes = kDynHeaderBytes + size_t(kDynLevels) * kDynCap * 24;
bool uses_device_enqueue(const std::string& src);

// Compile to a gfx950 code object (cached in memory and on disk).  Returns
// false and fills log on error.
bool compile_gpu(const std::string& rewritten_src, const std::vector<std::string>& options,
                 const std::string& arch, std::string& code, std::string& log);
// Compile to a host shared object (cached on disk); returns path.
bool compile_cpu(const std::string& rewritten_src, const std::vector<std::string>& options,
                 std::string& so_path, std::string& log);

std::string cache_dir();
std::string hash_hex(const std::string& s);

}  // namespace cek
