#include "device.h"

#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <thread>

namespace cek {

[[noreturn]] void throw_hip(hipError_t e, const char* expr, const char* file, int line) {
  std::ostringstream os;
  os << "HIP error " << static_cast<int>(e) << " (" << hipGetErrorString(e) << ") in " << expr
     << " at " << file << ":" << line;
  throw Error(os.str());
}

std::string DeviceInfo::describe() const {
  std::ostringstream os;
  os << (type == kGPU ? "GPU" : type == kCPU ? "CPU" : "ACC") << " " << name;
  if (!arch.empty()) os << " [" << arch << "]";
  os << " CUs=" << compute_units << " mem=" << (mem_bytes >> 20) << "MiB";
  if (type == kCPU) os << " threads=" << cpu_threads;
  os << (dedicated_memory ? " dedicated" : " shared") << (streaming ? " stream" : "");
  if (cu_parts > 1) os << " cu-part=" << cu_part << "/" << cu_parts;
  return os.str();
}

std::vector<int> partition_cus(int ncu, int parts, int p) {
  if (parts < 1 || ncu < parts || ncu % parts != 0) throw Error("partition_cus: CUs must split into whole partitions");
  if (p < 0 || p >= parts) throw Error("partition_cus: partition index out of range");
  const int block = ncu / parts;
  std::vector<int> out;
  for (int c = 0; c < ncu; ++c)
    if ((c % parts + c / block) % parts == p) out.push_back(c);
  return out;
}

int gpu_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

DeviceInfo gpu_info(int ordinal) {
  hipDeviceProp_t p;
  CEK_HIP(hipGetDeviceProperties(&p, ordinal));
  DeviceInfo d;
  d.type = kGPU;
  d.ordinal = ordinal;
  d.name = p.name;
  d.arch = p.gcnArchName;
  d.vendor = "Advanced Micro Devices, Inc.";
  d.platform = "AMD ROCm HIP";
  d.compute_units = p.multiProcessorCount;
  d.mem_bytes = p.totalGlobalMem;
  d.dedicated_memory = !p.integrated;
  d.streaming = p.integrated;
  d.pci_bus = p.pciBusID;
  d.pci_device = p.pciDeviceID;
  d.clock_khz = p.clockRate;
  d.lds_per_block = p.sharedMemPerBlock;
  return d;
}

static std::string cpu_model_name() {
  std::ifstream f("/proc/cpuinfo");
  std::string line;
  while (std::getline(f, line)) {
    if (line.rfind("model name", 0) == 0) {
      auto pos = line.find(':');
      if (pos != std::string::npos) {
        auto s = line.substr(pos + 1);
        while (!s.empty() && s.front() == ' ') s.erase(s.begin());
        return s;
      }
    }
  }
  return "Host CPU";
}

static uint64_t host_mem_bytes() {
  std::ifstream f("/proc/meminfo");
  std::string key;
  uint64_t kb = 0;
  std::string unit;
  while (f >> key >> kb >> unit) {
    if (key == "MemTotal:") return kb * 1024ull;
  }
  return 0;
}

DeviceInfo cpu_info(int threads) {
  DeviceInfo d;
  d.type = kCPU;
  d.ordinal = -1;
  d.name = cpu_model_name();
  d.vendor = "Host";
  d.platform = "Host CPU";
  int hw = static_cast<int>(std::thread::hardware_concurrency());
  if (hw <= 0) hw = 1;
  d.compute_units = hw;
  // Reference fission keeps one core for the host (ClDevice.cs:85-95).
  d.cpu_threads = threads > 0 ? threads : (hw > 1 ? hw - 1 : 1);
  d.mem_bytes = host_mem_bytes();
  d.dedicated_memory = false;
  d.streaming = true;
  return d;
}

std::vector<DeviceInfo> enumerate_devices() {
  std::vector<DeviceInfo> out;
  int n = gpu_count();
  for (int i = 0; i < n; ++i) out.push_back(gpu_info(i));
  out.push_back(cpu_info());
  return out;
}

std::vector<std::vector<int>> enable_peer_access_among(const std::vector<int>& ordinals) {
  const int n = static_cast<int>(ordinals.size());
  std::vector<std::vector<int>> m(n, std::vector<int>(n, 0));
  int cur = -1;
  const bool restore = hipGetDevice(&cur) == hipSuccess;
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < n; ++j) {
      if (ordinals[i] == ordinals[j]) {
        m[i][j] = 1;
        continue;
      }
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, ordinals[i], ordinals[j]) == hipSuccess && can) {
        CEK_HIP(hipSetDevice(ordinals[i]));
        hipError_t e = hipDeviceEnablePeerAccess(ordinals[j], 0);
        if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) m[i][j] = 1;
      }
      (void)hipGetLastError();
    }
  }
  if (restore && cur >= 0) (void)hipSetDevice(cur);
  return m;
}

std::vector<std::vector<int>> enable_peer_access() {
  std::vector<int> all(gpu_count());
  for (size_t i = 0; i < all.size(); ++i) all[i] = static_cast<int>(i);
  return enable_peer_access_among(all);
}

std::string peer_path(const std::vector<std::vector<int>>& m) {
  if (m.size() < 2) return "none";
  for (size_t i = 0; i < m.size(); ++i)
    for (size_t j = 0; j < m.size(); ++j)
      if (!m[i][j] || !m[j][i]) return "staged";
  return "xgmi";
}

namespace {
struct Epoch {
  hipEvent_t ev = nullptr;
  double host_ms = 0;
};
std::mutex g_epoch_mu;
std::map<int, Epoch> g_epochs;
}  // namespace

double event_host_ms(int ordinal, hipEvent_t ev) {
  Epoch e;
  {
    std::lock_guard<std::mutex> g(g_epoch_mu);
    auto it = g_epochs.find(ordinal);
    if (it == g_epochs.end()) {
      int cur = -1;
      (void)hipGetDevice(&cur);
      CEK_HIP(hipSetDevice(ordinal));
      hipStream_t s;
      CEK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      CEK_HIP(hipEventCreate(&e.ev));
      CEK_HIP(hipEventRecord(e.ev, s));
      CEK_HIP(hipEventSynchronize(e.ev));
      e.host_ms = now_ms();
      (void)hipStreamDestroy(s);
      if (cur >= 0) (void)hipSetDevice(cur);
      g_epochs[ordinal] = e;
    } else {
      e = it->second;
    }
  }
  float ms = 0.f;
  CEK_HIP(hipEventElapsedTime(&ms, e.ev, ev));
  return e.host_ms + ms;
}

}  // namespace cek
