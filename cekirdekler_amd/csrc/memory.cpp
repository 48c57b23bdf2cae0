#include "memory.h"

#include <cstdlib>
#include <unordered_map>

#include "device.h"

namespace cek {

namespace {
struct HostEntry {
  bool pinned;      // hipHostMalloc
  void* raw;        // pointer to free (posix_memalign)
};
std::mutex g_mu;
std::unordered_map<const void*, HostEntry> g_allocs;
std::unordered_map<const void*, int> g_registered;  // refcount
}  // namespace

void* host_alloc(uint64_t bytes, uint64_t align, bool* pinned) {
  if (bytes == 0) bytes = 1;
  if (align < 64) align = 64;
  void* p = nullptr;
  bool pin = false;
  if (gpu_count() > 0) {
    // hipHostMalloc returns page-aligned memory; over-align if asked for more.
    if (align <= 4096 &&
        hipHostMalloc(&p, bytes, hipHostMallocPortable | hipHostMallocMapped) == hipSuccess) {
      pin = true;
    } else {
      (void)hipGetLastError();
      p = nullptr;
    }
  }
  if (!p) {
    if (posix_memalign(&p, align, bytes) != 0) throw Error("host_alloc: out of memory");
  }
  std::lock_guard<std::mutex> g(g_mu);
  g_allocs[p] = {pin, p};
  if (pinned) *pinned = pin;
  return p;
}

void host_free(void* p) {
  if (!p) return;
  HostEntry e{false, p};
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_allocs.find(p);
    if (it == g_allocs.end()) return;
    e = it->second;
    g_allocs.erase(it);
  }
  if (e.pinned)
    (void)hipHostFree(p);
  else
    free(e.raw);
}

bool host_is_pinned(const void* p) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_allocs.find(p);
  if (it != g_allocs.end()) return it->second.pinned;
  return g_registered.count(p) > 0;
}

bool host_register(void* p, uint64_t bytes) {
  if (gpu_count() == 0) return false;
  std::lock_guard<std::mutex> g(g_mu);
  auto a = g_allocs.find(p);
  if (a != g_allocs.end() && a->second.pinned) return true;
  auto it = g_registered.find(p);
  if (it != g_registered.end()) {
    ++it->second;
    return true;
  }
  if (hipHostRegister(p, bytes, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  g_registered[p] = 1;
  return true;
}

void host_unregister(void* p) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_registered.find(p);
  if (it == g_registered.end()) return;
  if (--it->second == 0) {
    (void)hipHostUnregister(p);
    g_registered.erase(it);
  }
}

void* host_device_ptr(void* p) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
    (void)hipGetLastError();
    return p;  // unified addressing: the host VA is device-visible
  }
  return d;
}

void copy_memory(void* dst, const void* src, uint64_t bytes) { std::memcpy(dst, src, bytes); }

}  // namespace cek
