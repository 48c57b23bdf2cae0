#include "worker.h"

#include <map>
#include <unistd.h>
#include <set>

#include <algorithm>

#include "memory.h"

// hip/hip_ext.h declares this AMD launch (kernel start/stop events stamped by
// the dispatch) next to a template that needs the device-compiler headers;
// the host build takes the C declaration alone
extern "C" hipError_t hipExtModuleLaunchKernel(hipFunction_t f, uint32_t globalWorkSizeX, uint32_t globalWorkSizeY,
                                               uint32_t globalWorkSizeZ, uint32_t localWorkSizeX,
                                               uint32_t localWorkSizeY, uint32_t localWorkSizeZ,
                                               size_t sharedMemBytes, hipStream_t hStream, void** kernelParams,
                                               void** extra, hipEvent_t startEvent, hipEvent_t stopEvent,
                                               uint32_t flags);

namespace cek {

// ----------------------------------------------------------------- CpuPool --

// Pool threads alive in the process: spinning only pays while every spinner
// has a core (two CPU devices of one host would otherwise spin 2·(N-1)
// threads on N cores and starve each other).
// Off by default (CEK_POOL_SPIN_US): measured on an 8-vCPU VM, spinning pool
// threads made a tiny CPU-device compute 1.5-3x slower (20 -> 33-60 µs; two
// CPU devices 42-51 -> 130-141 µs), and under a cgroup CPU quota (the GPU
// boxes give a process a 16-CPU share of a much larger machine) every
// spinning thread burns the share the computing threads need.
static std::atomic<int> g_pool_threads{0};
static double env_pool_spin_us() {
  const char* e = std::getenv("CEK_POOL_SPIN_US");
  return e ? std::max(0.0, std::atof(e)) : 0.0;
}
static const double g_pool_spin_us = env_pool_spin_us();
static bool pool_may_spin() {
  static const int cores = std::max(1u, std::thread::hardware_concurrency());
  return g_pool_spin_us > 0 && g_pool_threads.load(std::memory_order_relaxed) < cores;
}

CpuPool::CpuPool(int threads) : pid_(static_cast<long>(getpid())) {
  for (int i = 1; i < threads; ++i) threads_.emplace_back([this] { loop(); });
  g_pool_threads += static_cast<int>(threads_.size());
}

CpuPool::~CpuPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
  g_pool_threads -= static_cast<int>(threads_.size());
}

static inline void pool_relax() { __builtin_ia32_pause(); }


void CpuPool::loop() {
  uint64_t seen = 0;
  for (;;) {
    if (pool_may_spin()) {  // a new generation usually follows within µs
      const double until = now_ms() + g_pool_spin_us * 1e-3;
      int k = 0;
      while (gen_.load(std::memory_order_acquire) == seen) {
        pool_relax();
        if ((++k & 63) == 0 && now_ms() > until) break;
      }
    }
    const std::function<void(long long)>* fn;
    long long n;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || gen_.load(std::memory_order_relaxed) != seen; });
      if (stop_) return;
      seen = gen_.load(std::memory_order_relaxed);
      fn = fn_;
      n = n_;
      if (!fn) continue;
      active_.fetch_add(1, std::memory_order_acq_rel);
    }
    for (long long i = next_++; i < n; i = next_++) (*fn)(i);
    {
      std::lock_guard<std::mutex> g(mu_);
      active_.fetch_sub(1, std::memory_order_acq_rel);
    }
    done_cv_.notify_all();
  }
}

std::shared_ptr<CpuPool> CpuPool::shared(int threads, int slot) {
  static const bool on = [] {
    const char* e = std::getenv("CEK_SHARED_CPU_POOL");
    return !(e && std::string(e) == "0");
  }();
  threads = std::max(1, threads);
  if (!on) return std::make_shared<CpuPool>(threads);
  static std::mutex mu;
  static std::map<std::pair<int, int>, std::weak_ptr<CpuPool>> pools;
  std::lock_guard<std::mutex> g(mu);
  auto& w = pools[{threads, slot}];
  auto p = w.lock();
  // a pool inherited through fork() has no threads in this process
  if (p && p->pid_ != static_cast<long>(getpid())) p.reset();
  if (!p) {
    p = std::make_shared<CpuPool>(threads);
    w = p;
  }
  return p;
}

void CpuPool::parallel_for(long long n, const std::function<void(long long)>& fn) {
  if (n <= 0) return;
  if (threads_.empty() || n == 1) {
    for (long long i = 0; i < n; ++i) fn(i);
    return;
  }
  std::lock_guard<std::mutex> turn(call_mu_);
  {
    std::lock_guard<std::mutex> g(mu_);
    fn_ = &fn;
    n_ = n;
    next_ = 0;
    gen_.fetch_add(1, std::memory_order_release);
  }
  // wake only as many pool threads as there are items beyond the caller's
  // first (a small range need not wake the whole pool)
  if (n - 1 >= static_cast<long long>(threads_.size())) {
    cv_.notify_all();
  } else {
    for (long long k = 0; k < n - 1; ++k) cv_.notify_one();
  }
  for (long long i = next_++; i < n; i = next_++) fn(i);
  // every item is claimed; wait (spinning first) for the threads still running one
  if (pool_may_spin()) {
    const double until = now_ms() + g_pool_spin_us * 1e-3;
    int k = 0;
    while (active_.load(std::memory_order_acquire) != 0) {
      pool_relax();
      if ((++k & 63) == 0 && now_ms() > until) break;
    }
  }
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return active_.load(std::memory_order_acquire) == 0 && next_ >= n; });
  fn_ = nullptr;
}

// ------------------------------------------------------------------ Worker --

Worker::Worker(const DeviceInfo& dev, std::shared_ptr<Program> prog, int queue_concurrency,
               bool no_pipelining, int cpu_slot)
    : dev_(dev), prog_(std::move(prog)), qconc_(queue_concurrency < 1 ? 1 : (queue_concurrency > 16 ? 16 : queue_concurrency)),
      no_pipelining_(no_pipelining) {
  cq_.assign(16, nullptr);
  marker_issued_per_slot_.assign(32, 0);
  rings_.resize(32);
  if (const char* e = std::getenv("CEK_MARKERS")) write_value_markers_ = std::string(e) == "writevalue";
  if (gpu()) {
    set_device();
    apply_sync_mode(dev_.ordinal);
    bool pinned = false;
    marker_words_ = static_cast<uint64_t*>(host_alloc(32 * sizeof(uint64_t), 4096, &pinned));
    std::memset(marker_words_, 0, 32 * sizeof(uint64_t));
    // one lookup here instead of a runtime call (under HIP's lock) per marker
    marker_dev_ = static_cast<uint64_t*>(host_device_ptr(marker_words_));
  } else {
    pool_ = CpuPool::shared(dev_.cpu_threads > 0 ? dev_.cpu_threads : 1, cpu_slot);
  }
  th_ = std::thread([this] { thread_loop(); });
}

Worker::~Worker() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
  if (gpu()) {
    try {
      set_device();
      sync_all();
    } catch (...) {
    }
    release_all();
    for (auto& dq : dyn_queues_) (void)hipFree(dq.second);
    for (auto& g : graphs_) (void)hipGraphExecDestroy(g.second);
    for (auto e : events_) (void)hipEventDestroy(e);
    for (auto e : join_ev_)
      if (e) (void)hipEventDestroy(e);
    if (sys_ev_) (void)hipEventDestroy(sys_ev_);
    if (sleep_ev_) (void)hipEventDestroy(sleep_ev_);
    if (main_) (void)hipStreamDestroy(main_);
    for (auto s : cq_)
      if (s) (void)hipStreamDestroy(s);
    for (auto& h : pq_)
      for (auto s : h)
        if (s) (void)hipStreamDestroy(s);
    host_free(marker_words_);
    for (auto& k : kstamps_) {
      (void)hipEventDestroy(k.start);
      (void)hipEventDestroy(k.stop);
    }
    for (auto e : kstamp_spare_) (void)hipEventDestroy(e);
    for (auto& r : rings_) {
      for (auto& e : r.pending) (void)hipEventDestroy(e.first);
      for (auto e : r.spare) (void)hipEventDestroy(e);
      for (auto e : r.spare_fenced) (void)hipEventDestroy(e);
    }
  }
}

// CEK_HIP_SYNC=blocking|yield|spin: how a host thread waits in stream and
// event synchronisation on this device (hipSetDeviceFlags).  The default
// leaves HIP's own choice.  A waiting thread that spins takes a CPU from a
// co-executing CPU device's share; "blocking" sleeps until the GPU signals.
void apply_sync_mode(int ordinal) {
  static const unsigned flags = [] {
    const char* e = std::getenv("CEK_HIP_SYNC");
    const std::string m = e ? e : "";
    if (m == "blocking") return static_cast<unsigned>(hipDeviceScheduleBlockingSync);
    if (m == "yield") return static_cast<unsigned>(hipDeviceScheduleYield);
    if (m == "spin") return static_cast<unsigned>(hipDeviceScheduleSpin);
    return 0u;
  }();
  if (!flags) return;
  static std::mutex mu;
  static std::set<int> done;
  std::lock_guard<std::mutex> g(mu);
  if (!done.insert(ordinal).second) return;
  if (hipSetDeviceFlags(flags) != hipSuccess) (void)hipGetLastError();  // too late for this device: keep HIP's mode
}

void Worker::set_device() const {
  if (gpu()) CEK_HIP(hipSetDevice(dev_.ordinal));
}

void* Worker::buffer(const ArraySpec& a) {
  void* p = buffer_impl(a);
  std::lock_guard<std::mutex> g(buf_mu_);
  if (cap_log_) cap_log_->emplace_back(a.uid, p);
  return p;
}

void Worker::set_capture_log(std::vector<std::pair<uint64_t, void*>>* log) {
  std::lock_guard<std::mutex> g(buf_mu_);
  cap_log_ = log;
}

// A copy captured into a graph replays against the host pages it was
// captured with; from pageable memory the runtime would stage it through a
// bounce buffer at capture time, so the replay would not read (or write) the
// array's current contents.  Only pinned / registered host memory may be
// captured.
void Worker::check_capturable(const ArraySpec& a) {
  {
    std::lock_guard<std::mutex> g(buf_mu_);
    if (!cap_log_) return;
  }
  if (!host_is_pinned(a.host))
    throw Error("graph capture: array " + std::to_string(a.uid) + " (" + std::to_string(a.bytes) +
                " bytes) is pageable host memory; a captured copy needs pinned or registered memory "
                "(use a FastArr-backed ClArray, or set ClArray.auto_pin_min_bytes below its size)");
}

bool Worker::buffer_is(uint64_t uid, const void* ptr) {
  std::lock_guard<std::mutex> g(buf_mu_);
  auto it = bufs_.find(uid);
  if (it != bufs_.end()) return it->second.first == ptr;
  auto z = zc_ptr_.find(uid);
  return z != zc_ptr_.end() && z->second == ptr;
}

void* Worker::buffer_impl(const ArraySpec& a) {
  if (!gpu()) return a.host;
  if (a.zc) {
    // The array owns its registration (ClArray registers once, unregisters
    // on dispose); registering here per launch would leak refcounts and leave
    // a stale mapping behind once the host memory is freed.
    if (!host_is_pinned(a.host))
      throw Error("zero-copy array is neither pinned nor registered with HIP");
    std::lock_guard<std::mutex> g(buf_mu_);
    zc_[a.uid] = true;
    return zc_ptr_[a.uid] = host_device_ptr(a.host);
  }
  std::lock_guard<std::mutex> g(buf_mu_);
  auto it = bufs_.find(a.uid);
  const bool checks = debug_checks.load(std::memory_order_relaxed);
  void* keep = nullptr;  // old replica whose contents move into a guarded one
  uint64_t keep_bytes = 0;
  if (it != bufs_.end()) {
    void* d = it->second.first;
    const uint64_t cap = it->second.second;  // usable bytes (a guard, if any, lies past them)
    if (cap >= a.bytes) {
      if (!checks) return d;
      auto gi = guarded_.find(a.uid);
      if (gi != guarded_.end() && gi->second == a.bytes) return d;
      // Debug checks need the guard right at the current extent: re-stamp it
      // there when the allocation has room (a guarded buffer reused at a
      // smaller size has), else move the contents into a guarded allocation.
      const uint64_t room = gi != guarded_.end() ? gi->second + kGuardBytes : cap;
      if (room >= a.bytes + kGuardBytes) {
        set_device();
        CEK_HIP(hipMemset(static_cast<char*>(d) + a.bytes, kGuardByte, kGuardBytes));
        guarded_[a.uid] = a.bytes;
        return d;
      }
      keep = d;
      keep_bytes = std::min<uint64_t>(cap, a.bytes);
    } else {
      (void)hipFree(d);
    }
    bytes_allocated_ -= cap;
    bufs_.erase(it);
  }
  void* d = nullptr;
  set_device();
  const size_t guard = checks ? kGuardBytes : 0;
  hipError_t e = hipMalloc(&d, (a.bytes ? a.bytes : 1) + guard);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    throw Error("hipMalloc of " + std::to_string(a.bytes) + " bytes failed on " + dev_.name);
  }
  if (keep) {
    CEK_HIP(hipMemcpy(d, keep, keep_bytes, hipMemcpyDeviceToDevice));
    (void)hipFree(keep);
  }
  if (guard) {
    CEK_HIP(hipMemset(static_cast<char*>(d) + a.bytes, kGuardByte, guard));
    guarded_[a.uid] = a.bytes;
  } else {
    guarded_.erase(a.uid);
  }
  bufs_[a.uid] = {d, a.bytes};
  bytes_allocated_ += a.bytes;
  return d;
}

void Worker::release(uint64_t uid) {
  std::lock_guard<std::mutex> g(buf_mu_);
  auto it = bufs_.find(uid);
  if (it != bufs_.end()) {
    set_device();
    (void)hipFree(it->second.first);
    bytes_allocated_ -= it->second.second;
    bufs_.erase(it);
  }
  guarded_.erase(uid);
  zc_.erase(uid);
  zc_ptr_.erase(uid);
}

void Worker::release_all() {
  std::lock_guard<std::mutex> g(buf_mu_);
  if (gpu()) {
    (void)hipSetDevice(dev_.ordinal);
    for (auto& kv : bufs_) (void)hipFree(kv.second.first);
  }
  bufs_.clear();
  guarded_.clear();
  zc_.clear();
  zc_ptr_.clear();
  bytes_allocated_ = 0;
}

hipStream_t Worker::new_stream(bool copy_cus) {
  set_device();
  hipStream_t s = nullptr;
  if (dev_.cu_parts > 1) {
    // a CU-partitioned logical device: every stream (copy-kernel ones too)
    // sees its partition's CUs only
    const int ncu = std::max(1, dev_.compute_units);
    std::vector<uint32_t> mask((ncu + 31) / 32, 0);
    for (int cu : partition_cus(ncu, dev_.cu_parts, dev_.cu_part)) mask[cu / 32] |= 1u << (cu % 32);
    CEK_HIP(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data()));
    return s;
  }
  if (cu_reserve_ <= 0) {
    CEK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
  }
  const int ncu = std::max(1, dev_.compute_units);
  const int every = std::max(1, ncu / cu_reserve_);
  std::vector<uint32_t> mask((ncu + 31) / 32, 0);
  for (int cu = 0; cu < ncu; ++cu) {
    const bool reserved = (cu % every) == every - 1 && cu / every < cu_reserve_;
    if (reserved == copy_cus) mask[cu / 32] |= 1u << (cu % 32);
  }
  CEK_HIP(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data()));
  return s;
}

void Worker::destroy_streams() {
  if (!gpu()) return;
  sync_all();
  set_device();
  for (auto& dq : dyn_queues_) (void)hipFree(dq.second);
  dyn_queues_.clear();
  if (main_) (void)hipStreamDestroy(main_);
  main_ = nullptr;
  for (auto& s : cq_) {
    if (s) (void)hipStreamDestroy(s);
    s = nullptr;
  }
  for (auto& h : pq_)
    for (auto& s : h) {
      if (s) (void)hipStreamDestroy(s);
      s = nullptr;
    }
}

void Worker::set_cu_reserve(int n) {
  if (!gpu()) return;
  n = std::max(0, std::min(n, std::max(0, dev_.compute_units / 2)));
  if (n == cu_reserve_) return;
  destroy_streams();
  cu_reserve_ = n;
}

hipStream_t Worker::main_stream() {
  if (!gpu()) return nullptr;
  if (!main_) main_ = new_stream(false);
  return main_;
}

hipStream_t Worker::compute_stream(int i) {
  if (!gpu()) return nullptr;
  // one queue: the main stream itself.  A separate stream would cost a
  // hardware queue more for no concurrency — and a CU-masked stream (a
  // partitioned device) owns a hardware queue of its own, so 8 partitions
  // x 2 streams oversubscribe the GPU's queue slots
  if (qconc_ == 1) return main_stream();
  i %= 16;
  if (!cq_[i]) cq_[i] = new_stream(false);
  return cq_[i];
}

hipStream_t Worker::pipe_stream(int half, int role) {
  if (!gpu()) return nullptr;
  hipStream_t& s = pq_[half & 1][role % 3];
  if (!s) s = new_stream(role % 3 == 2);
  return s;
}

int Worker::next_compute_queue() { return rr_.fetch_add(1) % qconc_; }

hipEvent_t Worker::event(int slot) {
  while (static_cast<int>(events_.size()) <= slot) {
    set_device();
    hipEvent_t e;
    CEK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    events_.push_back(e);
  }
  return events_[slot];
}

void Worker::join_streams(hipStream_t target) {
  if (!gpu()) return;
  set_device();
  if (join_ev_.empty()) join_ev_.assign(32, nullptr);
  auto join = [&](hipStream_t s) {
    if (!s || s == target) return;
    hipEvent_t& e = join_ev_[stream_slot(s)];
    if (!e) CEK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CEK_HIP(hipEventRecord(e, s));
    CEK_HIP(hipStreamWaitEvent(target, e, 0));
  };
  join(main_);
  for (auto s : cq_) join(s);
  for (auto& h : pq_)
    for (auto s : h) join(s);
}

void Worker::wait_stream(hipStream_t s, bool sleep) {
  if (!gpu()) return;
  if (!sleep) {
    CEK_HIP(hipStreamSynchronize(s));
    return;
  }
  if (!sleep_ev_) {
    set_device();
    CEK_HIP(hipEventCreateWithFlags(&sleep_ev_, hipEventBlockingSync | hipEventDisableTiming));
  }
  CEK_HIP(hipEventRecord(sleep_ev_, s));
  CEK_HIP(hipEventSynchronize(sleep_ev_));
}

void Worker::system_release(hipStream_t s) {
  if (!gpu()) return;
  if (!sys_ev_) {
    set_device();
    CEK_HIP(hipEventCreateWithFlags(&sys_ev_, hipEventDisableTiming));  // system fence kept
  }
  CEK_HIP(hipEventRecord(sys_ev_, s));
}

void Worker::sync_all() {
  if (!gpu()) return;
  set_device();
  if (main_) CEK_HIP(hipStreamSynchronize(main_));
  for (auto s : cq_)
    if (s) CEK_HIP(hipStreamSynchronize(s));
  for (auto& h : pq_)
    for (auto s : h)
      if (s) CEK_HIP(hipStreamSynchronize(s));
}

void Worker::gate_all_streams(const uint32_t* word, uint32_t value) {
  if (!gpu()) return;
  set_device();
  void* dptr = host_device_ptr(const_cast<uint32_t*>(word));
  auto gate = [&](hipStream_t s) {
    CEK_HIP(hipStreamWaitValue32(s, dptr, value, hipStreamWaitValueGte, 0xffffffffu));
  };
  gate(main_stream());
  for (int i = 0; i < qconc_; ++i) gate(compute_stream(i));
  for (int h = 0; h < 2; ++h)
    for (int r = 0; r < 3; ++r) gate(pipe_stream(h, r));
}

void Worker::launch_graph(hipStream_t s, const std::string& key,
                          const std::function<void(hipStream_t)>& fn) {
  auto it = graphs_.find(key);
  if (it == graphs_.end()) {
    hipGraph_t g = nullptr;
    CEK_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    try {
      fn(s);
    } catch (...) {
      (void)hipStreamEndCapture(s, &g);
      if (g) (void)hipGraphDestroy(g);
      throw;
    }
    CEK_HIP(hipStreamEndCapture(s, &g));
    hipGraphExec_t ex = nullptr;
    hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    CEK_HIP(e);
    if (graphs_.size() >= 64) {  // bounded cache: drop everything, recapture on demand
      for (auto& kv : graphs_) (void)hipGraphExecDestroy(kv.second);
      graphs_.clear();
    }
    it = graphs_.emplace(key, ex).first;
  }
  CEK_HIP(hipGraphLaunch(it->second, s));
}

int Worker::stream_slot(hipStream_t s) {
  if (s == main_) return 0;
  for (int i = 0; i < 16; ++i)
    if (cq_[i] == s) return 1 + i;
  for (int h = 0; h < 2; ++h)
    for (int r = 0; r < 3; ++r)
      if (pq_[h][r] == s) return 17 + h * 3 + r;
  return 31;
}

void Worker::h2d(hipStream_t s, const ArraySpec& a, uint64_t elem_begin, uint64_t elem_count) {
  if (!gpu() || a.zc || elem_count == 0) return;
  check_capturable(a);
  uint64_t off = elem_begin * a.elem_size, n = elem_count * a.elem_size;
  if (off >= a.bytes) return;
  if (off + n > a.bytes) n = a.bytes - off;
  char* d = static_cast<char*>(buffer(a));
  CEK_HIP(hipMemcpyAsync(d + off, static_cast<const char*>(a.host) + off, n, hipMemcpyHostToDevice, s));
}

void Worker::d2h(hipStream_t s, const ArraySpec& a, uint64_t elem_begin, uint64_t elem_count) {
  if (!gpu() || a.zc || elem_count == 0) return;
  check_capturable(a);
  uint64_t off = elem_begin * a.elem_size, n = elem_count * a.elem_size;
  if (off >= a.bytes) return;
  if (off + n > a.bytes) n = a.bytes - off;
  char* d = static_cast<char*>(buffer(a));
  if (kernel_d2h.load(std::memory_order_relaxed) && d2h_by_kernel(s, a.host, off, d + off, n)) return;
  CEK_HIP(hipMemcpyAsync(static_cast<char*>(a.host) + off, d + off, n, hipMemcpyDeviceToHost, s));
}

// 16 bytes per lane per iteration; a grid of at most 64 work-groups: PCIe
// (≈ 55 GB/s) is the limit, so the copy leaves the rest of the chip to the
// kernels it overlaps
static const char* kCopySrc = R"CEK(
typedef unsigned int cek_u32x4 __attribute__((ext_vector_type(4)));
__global__ void cek_copy16_to_host(const cek_u32x4* src, cek_u32x4* dst, long long n16) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (; i < n16; i += stride) dst[i] = src[i];
}
)CEK";

bool Worker::d2h_by_kernel(hipStream_t s, void* host_base, uint64_t off, const void* src_dev, uint64_t n) {
  char* dst_host = static_cast<char*>(host_base) + off;
  if (n < kKernelD2HMinBytes || (reinterpret_cast<uintptr_t>(dst_host) | reinterpret_cast<uintptr_t>(src_dev) | n) & 15)
    return false;
  if (!host_is_pinned(host_base)) return false;  // pinned / registered: looked up by the array's base
  set_device();
  char* base_dev = static_cast<char*>(host_device_ptr(host_base));
  if (!base_dev) return false;
  void* dst = base_dev + off;
  {
    std::lock_guard<std::mutex> g(copy_mu_);
    if (!copy_fn_) {
      copy_prog_ = Program::build(dev_, kCopySrc, {}, {});
      if (!copy_prog_->ok()) throw Error("kernel-D2H copy kernel failed to build: " + copy_prog_->log());
      copy_fn_ = copy_prog_->gpu_fn("cek_copy16_to_host");
    }
  }
  long long n16 = static_cast<long long>(n / 16), hidden_off = 0, gs = n16;
  const void* src = src_dev;
  void* params[] = {&src, &dst, &n16, &hidden_off, &gs};
  const long long per_group = 256ll * 16;  // 16 iterations of 256 lanes per work-group at least
  const unsigned groups = static_cast<unsigned>(std::max(1ll, std::min(64ll, (n16 + per_group - 1) / per_group)));
  CEK_HIP(hipModuleLaunchKernel(copy_fn_, groups, 1, 1, 256, 1, 1, 0, s, params, nullptr));
  kernel_d2h_bytes_ += n;
  return true;
}

void Worker::launch(hipStream_t s, const std::string& kernel, const std::vector<ArraySpec>& arrs,
                    long long offset, long long count, int local, long long gsize) {
  if (count <= 0) return;
  if (local <= 0) throw Error("local range must be positive");
  if (count % local != 0)
    throw Error("range " + std::to_string(count) + " is not a multiple of local range " +
                std::to_string(local));
  if (gpu()) {
    hipFunction_t f = prog_->gpu_fn(kernel);
    std::vector<void*> ptrs(arrs.size());
    for (size_t i = 0; i < arrs.size(); ++i) ptrs[i] = buffer(arrs[i]);
    long long off = offset, gs = gsize;
    const bool dyn = prog_->dynamic();
    void* q = dyn ? dyn_queue(s) : nullptr;
    int level = 0;
    std::vector<void*> params(arrs.size() + (dyn ? 4 : 2));
    for (size_t i = 0; i < arrs.size(); ++i) params[i] = &ptrs[i];
    params[arrs.size()] = &off;
    params[arrs.size() + 1] = &gs;
    if (dyn) {
      params[arrs.size() + 2] = &q;
      params[arrs.size() + 3] = &level;
      // fresh level counts for this parent (errors accumulate)
      CEK_HIP(hipMemsetAsync(q, 0, 8 * sizeof(int), s));
    }
    unsigned grid = static_cast<unsigned>(count / local);
    if (kernel_times_on.load(std::memory_order_relaxed)) {
      hipEvent_t a = kstamp_event(), b = kstamp_event();
      CEK_HIP(hipExtModuleLaunchKernel(f, grid * static_cast<unsigned>(local), 1, 1, static_cast<unsigned>(local),
                                       1, 1, dyn_lds_, s, params.data(), nullptr, a, b, 0));
      std::lock_guard<std::mutex> g(kstamp_mu_);
      if (kstamps_.size() >= kMaxKernelStamps) {  // recording left on: keep the newest
        kstamp_spare_.push_back(kstamps_.front().start);
        kstamp_spare_.push_back(kstamps_.front().stop);
        kstamps_.pop_front();
      }
      kstamps_.push_back({kernel, a, b});
    } else {
      CEK_HIP(hipModuleLaunchKernel(f, grid, 1, 1, static_cast<unsigned>(local), 1, 1, dyn_lds_, s,
                                    params.data(), nullptr));
    }
    if (dyn && prog_->has_dispatcher(kernel)) {
      // one launch per child level, same stream: level L's records were
      // written by level L-1's kernel, which the stream has completed
      hipFunction_t d = prog_->gpu_fn("__cek_dispatch_" + kernel);
      const unsigned dgrid = static_cast<unsigned>(std::max(1, dev_.compute_units) * 4);
      for (int L = 1; L <= std::min(device_enqueue_levels, kDynLevels - 1); ++L) {
        level = L;
        CEK_HIP(hipModuleLaunchKernel(d, dgrid, 1, 1, 256, 1, 1, 0, s, params.data(), nullptr));
      }
    }
    if (debug_checks.load(std::memory_order_relaxed)) check_guards(s, kernel, arrs);
  } else {
    CpuRunner fn = prog_->cpu_fn(kernel);
    std::vector<void*> ptrs(arrs.size());
    for (size_t i = 0; i < arrs.size(); ++i) ptrs[i] = arrs[i].host;
    long long groups = count / local;
    // chunk groups so every pool thread gets several (amortise dispatch)
    long long nthreads = pool_->size();
    long long tasks_max = std::max<long long>(1, std::min(groups, (nthreads + 1) * 8));
    // ...but no task shorter than kCpuMinTaskNs by this kernel's measured
    // cost per work item: a small range (the CPU's share of a GPU+CPU wave
    // frame is ~1,400 vertices) runs on the calling thread alone instead of
    // paying every pool thread's wake-up
    double& est = cpu_item_ns_[kernel];
    if (est > 0) {
      const double by_work = est * static_cast<double>(count) / kCpuMinTaskNs;
      tasks_max = std::max<long long>(1, std::min<long long>(tasks_max, static_cast<long long>(by_work)));
    }
    const long long per = (groups + tasks_max - 1) / tasks_max;
    const long long tasks = (groups + per - 1) / per;
    void** argv = ptrs.data();
    const double t0 = now_ms();
    pool_->parallel_for(tasks, [&](long long t) {
      long long g0 = t * per, g1 = std::min(groups, g0 + per);
      fn(argv, offset, gsize, offset + g0 * local, (g1 - g0) * local, local);
    });
    // per-item cost on one thread: wall time × the threads that ran
    const double used = static_cast<double>(std::min<long long>(tasks, nthreads + 1));
    const double ns = (now_ms() - t0) * 1e6 * used / static_cast<double>(std::max<long long>(1, count));
    est = est > 0 ? 0.7 * est + 0.3 * ns : ns;
  }
}

hipEvent_t Worker::kstamp_event() {
  {
    std::lock_guard<std::mutex> g(kstamp_mu_);
    if (!kstamp_spare_.empty()) {
      hipEvent_t e = kstamp_spare_.back();
      kstamp_spare_.pop_back();
      return e;
    }
  }
  set_device();
  hipEvent_t e = nullptr;
  CEK_HIP(hipEventCreate(&e));  // timing enabled
  return e;
}

std::vector<std::pair<std::string, double>> Worker::kernel_times() {
  std::deque<KernelStamp> st;
  {
    std::lock_guard<std::mutex> g(kstamp_mu_);
    st.swap(kstamps_);
  }
  std::vector<std::pair<std::string, double>> out;
  out.reserve(st.size());
  for (auto& k : st) {
    CEK_HIP(hipEventSynchronize(k.stop));
    float ms = 0.f;
    CEK_HIP(hipEventElapsedTime(&ms, k.start, k.stop));
    out.emplace_back(k.kernel, ms);
  }
  std::lock_guard<std::mutex> g(kstamp_mu_);
  for (auto& k : st) {
    kstamp_spare_.push_back(k.start);
    kstamp_spare_.push_back(k.stop);
  }
  return out;
}

void Worker::check_guards(hipStream_t s, const std::string& kernel, const std::vector<ArraySpec>& arrs) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return;  // graph replay
  hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    throw Error("kernel '" + kernel + "' failed on " + dev_.name + ": " + hipGetErrorString(e));
  }
  std::vector<unsigned char> tail(kGuardBytes);
  for (size_t i = 0; i < arrs.size(); ++i) {
    void* d = nullptr;
    uint64_t at = 0;
    {
      std::lock_guard<std::mutex> g(buf_mu_);
      auto gi = guarded_.find(arrs[i].uid);
      auto bi = bufs_.find(arrs[i].uid);
      if (gi == guarded_.end() || bi == bufs_.end()) continue;
      d = bi->second.first;
      at = gi->second;
    }
    CEK_HIP(hipMemcpy(tail.data(), static_cast<char*>(d) + at, kGuardBytes, hipMemcpyDeviceToHost));
    size_t bad = 0, first = kGuardBytes;
    for (size_t b = 0; b < kGuardBytes; ++b)
      if (tail[b] != kGuardByte) {
        ++bad;
        if (first == kGuardBytes) first = b;
      }
    if (bad) {
      CEK_HIP(hipMemset(static_cast<char*>(d) + at, kGuardByte, kGuardBytes));
      throw Error("kernel '" + kernel + "' wrote past the end of array #" + std::to_string(i) + " (" +
                  std::to_string(at) + " bytes) on " + dev_.name + ": " + std::to_string(bad) +
                  " guard bytes changed, first at +" + std::to_string(first));
    }
  }
}

void* Worker::dyn_queue(hipStream_t s) {
  void*& q = dyn_queues_[s];
  if (!q) {
    set_device();
    CEK_HIP(hipMalloc(&q, kDynQueueBytes));
    CEK_HIP(hipMemset(q, 0, kDynHeaderBytes));
  }
  return q;
}

int Worker::device_enqueue_errors() {
  if (!gpu() || dyn_queues_.empty()) return 0;
  set_device();
  sync_all();
  int total = 0;
  for (auto& dq : dyn_queues_) {
    int e = 0;
    CEK_HIP(hipMemcpy(&e, static_cast<char*>(dq.second) + 8 * sizeof(int), sizeof(int), hipMemcpyDeviceToHost));
    total += e;
  }
  return total;
}

hipStream_t Worker::slot_stream(int slot) const {
  if (slot == 0) return main_;
  if (slot >= 1 && slot <= 16) return cq_[slot - 1];
  if (slot >= 17 && slot < 23) return pq_[(slot - 17) / 3][(slot - 17) % 3];
  return nullptr;
}

void Worker::defer_marker(hipStream_t s, bool release) {
  if (!gpu()) {  // a CPU device's compute is done when it returns
    add_marker(s, release);
    return;
  }
  const int slot = stream_slot(s);
  if (slot >= 31 || !slot_stream(slot)) {  // not a slot flush_markers() can find again
    add_marker(s, release);
    return;
  }
  last_slot_ = slot;  // markers_issued_ counts the marker when it is recorded
  last_value_ = marker_issued_per_slot_[slot] + 1;
  deferred_slots_ |= 1u << slot;
  if (release) deferred_release_ |= 1u << slot;
}

void Worker::flush_markers() {
  for (int slot = 0; deferred_slots_ != 0 && slot < 31; ++slot)
    if (deferred_slots_ & (1u << slot)) add_marker(slot_stream(slot), false);
}

void Worker::add_marker(hipStream_t s, bool release) {
  ++markers_issued_;
  if (!gpu()) {
    last_slot_ = -1;
    last_value_ = static_cast<uint64_t>(markers_issued_);
    return;
  }
  int slot = stream_slot(s);
  if (slot < 31 && (deferred_slots_ & (1u << slot))) {
    // this marker also completes the computes deferred on the same stream
    release = release || (deferred_release_ & (1u << slot));
    deferred_slots_ &= ~(1u << slot);
    deferred_release_ &= ~(1u << slot);
  }
  uint64_t v = ++marker_issued_per_slot_[slot];
  last_slot_ = slot;
  last_value_ = v;
  if (write_value_markers_) {
    CEK_HIP(hipStreamWriteValue64(s, marker_dev_ + slot, v, 0));
    return;
  }
  std::lock_guard<std::mutex> g(marker_mu_);
  MarkerRing& r = rings_[slot];
  auto& spare = release ? r.spare_fenced : r.spare;
  hipEvent_t e = nullptr;
  if (!spare.empty()) {
    e = spare.front();
    spare.pop_front();
  } else {
    set_device();
    // no timing; no system-scope release unless host memory was written: a
    // completion signal only
    CEK_HIP(hipEventCreateWithFlags(&e, release ? hipEventDisableTiming
                                                : (hipEventDisableTiming | hipEventDisableSystemFence)));
  }
  CEK_HIP(hipEventRecord(e, s));
  r.pending.emplace_back(e, release);
}

uint64_t Worker::marker_word(int slot) {
  if (!gpu() || slot < 0) return static_cast<uint64_t>(markers_issued_);
  if (write_value_markers_) return __atomic_load_n(&marker_words_[slot], __ATOMIC_ACQUIRE);
  std::lock_guard<std::mutex> g(marker_mu_);
  MarkerRing& r = rings_[slot];
  while (!r.pending.empty()) {
    const auto front = r.pending.front();
    const hipError_t q = hipEventQuery(front.first);
    if (q == hipErrorNotReady) break;
    if (q != hipSuccess) {
      (void)hipGetLastError();
      throw Error("marker event query failed on " + dev_.name);
    }
    (front.second ? r.spare_fenced : r.spare).push_back(front.first);
    r.pending.pop_front();
    ++r.done;
  }
  return r.done;
}

long long Worker::markers_reached() {
  if (!gpu()) return markers_issued_;
  long long r = 0;
  for (int i = 0; i < 32; ++i) r += static_cast<long long>(marker_word(i));
  return r;
}

static double env_spin_us() {
  const char* e = std::getenv("CEK_SPIN_US");
  return e ? std::max(0.0, std::atof(e)) : 50.0;
}
double Worker::spin_us = env_spin_us();

static inline void cpu_relax() { __builtin_ia32_pause(); }

void Worker::post(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(std::move(fn));
    posted_.fetch_add(1, std::memory_order_release);
  }
  if (sleeping_.load(std::memory_order_acquire)) cv_.notify_one();
}

void Worker::wait() {
  const uint64_t target = posted_.load(std::memory_order_acquire);
  // spin only on a GPU worker: a CPU device's job runs on the CPU pool,
  // which needs every core the caller would spin on
  if (finished_.load(std::memory_order_acquire) < target && spin_us > 0 && gpu()) {
    const double until = now_ms() + spin_us * 1e-3;
    int n = 0;
    while (finished_.load(std::memory_order_acquire) < target) {
      cpu_relax();
      if ((++n & 63) == 0 && now_ms() > until) break;
    }
  }
  std::unique_lock<std::mutex> lk(mu_);
  if (finished_.load(std::memory_order_acquire) < target) {
    waiter_blocked_.store(true, std::memory_order_release);
    idle_cv_.wait(lk, [&] { return q_.empty() && !busy_; });
    waiter_blocked_.store(false, std::memory_order_release);
  }
  if (err_) {
    auto e = err_;
    err_ = nullptr;
    std::rethrow_exception(e);
  }
}

void Worker::thread_loop() {
  bool device_set = false;
  for (;;) {
    std::function<void()> job;
    // spin for new work first (a hot loop of computes posts every few µs);
    // GPU workers only (a CPU worker's spin competes with its own pool)
    if (spin_us > 0 && !stop_ && gpu()) {
      const uint64_t seen = finished_.load(std::memory_order_acquire);
      const double until = now_ms() + spin_us * 1e-3;
      int n = 0;
      while (posted_.load(std::memory_order_acquire) == seen) {
        cpu_relax();
        if ((++n & 63) == 0 && now_ms() > until) break;
      }
    }
    {
      std::unique_lock<std::mutex> lk(mu_);
      if (q_.empty() && !stop_) {
        sleeping_.store(true, std::memory_order_release);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        sleeping_.store(false, std::memory_order_release);
      }
      if (stop_ && q_.empty()) return;
      job = std::move(q_.front());
      q_.pop_front();
      busy_ = true;
    }
    try {
      if (!device_set && gpu()) {
        set_device();
        device_set = true;
      }
      job();
    } catch (...) {
      std::lock_guard<std::mutex> g(mu_);
      if (!err_) err_ = std::current_exception();
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      busy_ = false;
      finished_.fetch_add(1, std::memory_order_release);
    }
    if (waiter_blocked_.load(std::memory_order_acquire)) idle_cv_.notify_all();
  }
}

}  // namespace cek
