// Device discovery: the MI355X-native replacement for the reference's
// platform/device wrappers (ClPlatform.cs:28-116, ClDevice.cs:26-161) and
// their native calls (platformList, createDevice, createDeviceAsPartition,
// deviceGDDR, deviceComputeUnits, deviceMemSize).
//
// There is one "ROCm HIP" platform (every visible GPU) and one "Host CPU"
// platform (a single CPU device driven by a native thread pool; the
// reference's CPU fission to N-1 cores, ClDevice.cs:85-95, becomes the pool
// size).
#pragma once
#include "common.h"

namespace cek {

struct DeviceInfo {
  int type = kCPU;        // DevType
  int ordinal = -1;       // HIP ordinal, -1 for the CPU device
  std::string name;
  std::string arch;       // gcnArchName (gfx950...)
  std::string vendor;
  std::string platform;
  int compute_units = 0;
  uint64_t mem_bytes = 0;
  bool dedicated_memory = false;  // reference "GDDR" flag (!HOST_UNIFIED_MEMORY)
  bool streaming = false;         // prefer zero-copy (reference "stream" flag)
  int cpu_threads = 0;            // CPU device pool size
  int pci_bus = -1;
  int pci_device = -1;
  int clock_khz = 0;
  uint64_t lds_per_block = 0;
  // CU partition of a logical GPU device (cu_parts > 1): every stream of its
  // worker is created with a CU mask holding only partition cu_part's CUs
  // (partition_cus), so logical devices of one GPU run side by side on
  // disjoint CUs instead of sharing all of them
  int cu_part = -1;
  int cu_parts = 0;
  std::string describe() const;
};

// CUs of partition p of `parts` equal partitions of a GPU with `ncu` CUs
// (ncu divisible by parts; MI355X: 256 CUs in 8 XCDs of 32).  CU c belongs to
// partition (c mod parts + c div (ncu / parts)) mod parts.  Whether the CU
// mask numbers the CUs XCD by XCD (XCD = c div 32) or round robin over the
// XCDs (XCD = c mod 8), each partition gets the same number of CUs on every
// XCD: ncu / parts / 8 (tests/test_cu_partition.py checks both numberings).
std::vector<int> partition_cus(int ncu, int parts, int p);

// Number of HIP GPUs (0 when no runtime / no device; never throws).
int gpu_count();
// All devices: GPUs first (HIP ordinal order) then the CPU device.
std::vector<DeviceInfo> enumerate_devices();
DeviceInfo gpu_info(int ordinal);
DeviceInfo cpu_info(int threads = -1);

// Peer access matrix between GPUs (xGMI); enables access where possible.
std::vector<std::vector<int>> enable_peer_access();
// The same among the given GPU ordinals only: m[i][j] = 1 when ordinals[i]
// can access ordinals[j]'s memory (access enabled in both directions where
// hipDeviceCanAccessPeer allows; the diagonal is 1).
std::vector<std::vector<int>> enable_peer_access_among(const std::vector<int>& ordinals);
// Device-to-device path of a device set from the peer matrix of its distinct
// GPUs: "none" (at most one distinct GPU: copies stay inside one GPU),
// "xgmi" (every pair peers: copies go over the xGMI links), "staged" (some
// pair cannot peer: the runtime bounces those copies through host memory).
std::string peer_path(const std::vector<std::vector<int>>& m);

// Host-clock time (now_ms() scale) at which a completed timing event was
// reached on GPU `ordinal`: each GPU's event clock is anchored once per
// process to the host clock (an event recorded, synchronised, and the host
// clock read right after; error ≈ the sync latency, tens of µs).  Puts
// spans of different GPUs on one time line (overlap of copies with kernels
// on other devices).
double event_host_ms(int ordinal, hipEvent_t ev);

}  // namespace cek
