// Launch-rate probe: how many kernel launches per
// second HIP accepts from T host threads, each on its own stream of ONE
// device, with no synchronisation until the end.  It separates the runtime's
// own per-device serialisation from the cost of the runtime's worker
// hand-off: Cores' fan-out over D logical devices of one GPU cannot enqueue
// faster than this.
#include "probe.h"

#include <atomic>
#include <thread>

namespace cek {

// mode 0: kernelParams (an array of pointers to each argument, which the
// runtime packs by the kernel's metadata); mode 1: the arguments pre-packed
// into one buffer (HIP_LAUNCH_PARAM_BUFFER_POINTER)
LaunchRate launch_rate_probe(int ordinal, const std::string& code_object, const std::string& kernel, int threads,
                             int launches, int mode) {
  if (threads < 1 || threads > 64 || launches < 1) throw Error("launch_rate_probe: 1..64 threads, >= 1 launch");
  CEK_HIP(hipSetDevice(ordinal));
  hipModule_t mod = nullptr;
  CEK_HIP(hipModuleLoad(&mod, code_object.c_str()));
  hipFunction_t fn = nullptr;
  CEK_HIP(hipModuleGetFunction(&fn, mod, kernel.c_str()));
  void* buf = nullptr;
  CEK_HIP(hipMalloc(&buf, 4096));
  std::vector<hipStream_t> streams(threads, nullptr);
  for (auto& s : streams) CEK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // warm-up: one launch per stream
  void* src = buf;
  void* dst = static_cast<char*>(buf) + 2048;
  long long off = 0, gsize = 1;
  void* args[] = {&src, &dst, &off, &gsize};
  for (auto s : streams) CEK_HIP(hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, s, args, nullptr));
  CEK_HIP(hipDeviceSynchronize());
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::vector<double> ms(threads, 0.0);
  std::vector<std::string> err(threads);
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      try {
        CEK_HIP(hipSetDevice(ordinal));
        void* a[] = {&src, &dst, &off, &gsize};
        struct {
          void* s;
          void* d;
          long long o, g;
        } packed{src, dst, off, gsize};
        size_t psize = sizeof(packed);
        void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &packed, HIP_LAUNCH_PARAM_BUFFER_SIZE, &psize,
                         HIP_LAUNCH_PARAM_END};
        ++ready;
        while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
        const double t0 = now_ms();
        for (int k = 0; k < launches; ++k) {
          if (mode == 1)
            CEK_HIP(hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, streams[t], nullptr, extra));
          else
            CEK_HIP(hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, streams[t], a, nullptr));
        }
        ms[t] = now_ms() - t0;
      } catch (const std::exception& e) {
        err[t] = e.what();
      }
    });
  while (ready.load() < threads) std::this_thread::yield();
  const double t0 = now_ms();
  go.store(true, std::memory_order_release);
  for (auto& x : th) x.join();
  const double host_ms = now_ms() - t0;
  CEK_HIP(hipDeviceSynchronize());
  const double drain_ms = now_ms() - t0;
  for (auto s : streams) (void)hipStreamDestroy(s);
  (void)hipFree(buf);
  (void)hipModuleUnload(mod);
  for (auto& e : err)
    if (!e.empty()) throw Error("launch_rate_probe: " + e);
  LaunchRate r;
  r.threads = threads;
  r.launches = launches;
  r.host_ms = host_ms;
  r.drain_ms = drain_ms;
  r.per_thread_ms = ms;
  r.launches_per_s = threads * static_cast<double>(launches) / (host_ms * 1e-3);
  return r;
}

}  // namespace cek
