// Per-device worker: the MI355X-native counterpart of the reference's
// ClObject.Worker (Worker.cs:33-1738).  A worker owns one device, a lazily
// created pool of HIP streams (main, up to 16 round-robin compute streams,
// and read/compute/write streams for the two event-pipeline halves — the
// reference's 20-21 OpenCL queues, Worker.cs:75-259), the compiled program,
// one full-length device replica per host array (Worker.cs:576-720), marker
// words for fine-grained queue control, and a persistent host thread that
// executes fan-out jobs (replacing Parallel.For, Cores.cs:747-834).
//
// The CPU device executes the same kernel source compiled for the host on a
// thread pool; it works directly on host memory (no copies).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <exception>
#include <map>
#include <thread>
#include <unordered_map>

#include "common.h"
#include "device.h"
#include "jit.h"

namespace cek {

// One kernel-parameter array of a compute() call (ClArray flags,
// ClArray.cs:1742-1888; token semantics Worker.cs:827-834, :1349-1356).
struct ArraySpec {
  uint64_t uid = 0;       // identity of the host array (buffer-cache key)
  void* host = nullptr;   // host pointer
  uint64_t bytes = 0;     // total bytes of the host array
  int elem_size = 4;
  bool read = true;       // H2D the whole array to every device
  bool partial = false;   // H2D only this device's slice (wins over read)
  bool write = true;      // D2H this device's slice
  bool write_all = false; // device (index mod D) D2H the whole array
  bool ro = false, wo = false;  // access hints
  bool zc = false;        // zero-copy: kernel reads/writes host memory
  // keep-resident gather: after the kernels, every device's written slice
  // is copied into every other device's replica (event-ordered device→device
  // copies over xGMI in one process, an RCCL all-gather across ranks), so an
  // iterative kernel reads everybody's results without a host round trip
  bool gather = false;
  int epw = 1;            // elements per work item
  int epg = 0;            // >0: elements per work-GROUP instead (per-group outputs)
  // explicit blob slices (event pipeline with ComputeCall::blob_bounds):
  // blob k moves elements [blob_begin[k], blob_begin[k] + blob_count[k])
  // instead of the slice proportional to its work items — e.g. blob k of a
  // square-shell GEMM needs row panel k of A and of B
  std::vector<uint64_t> blob_begin, blob_count;
  // Element slice [begin, begin+count) owned by work items [ref, ref+range).
  void slice(long long ref, long long range, long long local, uint64_t& begin, uint64_t& count) const {
    if (epg > 0) {
      begin = static_cast<uint64_t>(ref / local) * epg;
      count = static_cast<uint64_t>(range / local) * epg;
    } else {
      begin = static_cast<uint64_t>(ref) * epw;
      count = static_cast<uint64_t>(range) * epw;
    }
  }
};

class CpuPool {
 public:
  explicit CpuPool(int threads);
  ~CpuPool();
  // Run fn(i) for i in [0, n) across the pool; blocks until done.  Callers
  // on different threads take turns (a pool may be shared, see shared()).
  void parallel_for(long long n, const std::function<void(long long)>& fn);
  int size() const { return static_cast<int>(threads_.size()) + 1; }
  // The process-wide pool of `threads` threads for the `slot`-th CPU device
  // of a device set: every cruncher's first CPU device of a given size runs
  // on the same threads, as an OpenCL CPU runtime shares one thread pool
  // among its contexts.  Separate crunchers on one host then see the same
  // CPU device (on a shared host a pool's speed depends on where its
  // threads landed: 3.0-4.4 ms for the same stream in four crunchers of one
  // process, profiles/r6/README.md) and do not oversubscribe the host when
  // used in turn; two CPU devices of ONE set (slots 0 and 1) still run side
  // by side.  CEK_SHARED_CPU_POOL=0: a pool per device.
  static std::shared_ptr<CpuPool> shared(int threads, int slot);

 private:
  void loop();
  long pid_ = 0;  // the process that started the threads (a forked child has none of them)
  std::mutex call_mu_;  // one parallel_for at a time
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(long long)>* fn_ = nullptr;
  long long n_ = 0;
  std::atomic<long long> next_{0};
  std::atomic<int> active_{0};
  // generation of the current parallel_for: pool threads may spin on it for
  // CEK_POOL_SPIN_US (default 0) before sleeping on cv_ (a frame loop calls
  // parallel_for every few tens of µs; a futex wake per thread per call
  // was the CPU device's fixed cost)
  std::atomic<uint64_t> gen_{0};
  bool stop_ = false;
};

// How host threads wait for GPU `ordinal` (env CEK_HIP_SYNC, worker.cpp).
void apply_sync_mode(int ordinal);

class Worker {
 public:
  // cpu_slot: this CPU device's index among the CPU devices of its set
  // (CpuPool::shared); ignored for a GPU
  Worker(const DeviceInfo& dev, std::shared_ptr<Program> prog, int queue_concurrency,
         bool no_pipelining, int cpu_slot = 0);
  ~Worker();

  const DeviceInfo& dev() const { return dev_; }
  bool gpu() const { return dev_.type == kGPU; }
  uintptr_t cpu_pool_id() const { return reinterpret_cast<uintptr_t>(pool_.get()); }
  Program& program() { return *prog_; }

  // --- buffers ---------------------------------------------------------
  void* buffer(const ArraySpec& a);  // device-visible pointer for a
  // graph capture: while a log is set, every (uid, pointer) handed out is
  // appended to it; buffer_is() tells whether uid still has that pointer
  void set_capture_log(std::vector<std::pair<uint64_t, void*>>* log);
  bool buffer_is(uint64_t uid, const void* ptr);
  void release(uint64_t uid);
  void release_all();
  uint64_t bytes_allocated() const { return bytes_allocated_; }

  // --- streams ---------------------------------------------------------
  hipStream_t main_stream();
  hipStream_t compute_stream(int i);        // i in [0, queue_concurrency)
  hipStream_t pipe_stream(int half, int role);  // role 0=read 1=compute 2=write
  // Reserve `n` CUs (spread evenly over the XCDs) for copy kernels: the
  // pipeline's write streams run on those CUs only and every other stream
  // on the rest (hipExtStreamCreateWithCUMask).  A download by copy kernel
  // (kernel_d2h) then never waits for a GEMM work-group to leave a CU, so
  // it runs beside the SDMA uploads (PCIe full duplex).  0: no masks.
  // Drains and re-creates the worker's streams.
  void set_cu_reserve(int n);
  int cu_reserve() const { return cu_reserve_; }
  int next_compute_queue();                 // round robin (Worker.cs:435-458)
  int queue_concurrency() const { return qconc_; }
  hipEvent_t event(int slot);               // pooled, timing disabled
  // wait until stream s is idle: hipStreamSynchronize, or (sleep) a
  // blocking-sync event the host thread sleeps on
  void wait_stream(hipStream_t s, bool sleep);
  // `target` waits for everything queued so far on every other stream of
  // this worker (compute queues and pipeline streams): a copy issued next on
  // `target` neither overtakes a kernel still reading its destination nor
  // reads a source a kernel is still writing
  void join_streams(hipStream_t target);
  // A marker with a SYSTEM-scope release on s (a default-flag event): stores
  // that kernels made straight into host memory (zero-copy arrays) are
  // visible to the host once s is synchronised, independent of the
  // fence-free timing events around them
  void system_release(hipStream_t s);
  void sync_all();                          // finish every created stream
  void set_device() const;

  // --- ops (enqueue on GPU; synchronous on the CPU device) --------------
  void h2d(hipStream_t s, const ArraySpec& a, uint64_t elem_begin, uint64_t elem_count);
  void d2h(hipStream_t s, const ArraySpec& a, uint64_t elem_begin, uint64_t elem_count);
  void launch(hipStream_t s, const std::string& kernel, const std::vector<ArraySpec>& arrs,
              long long offset, long long count, int local, long long gsize);
  void set_dynamic_lds(unsigned bytes) { dyn_lds_ = bytes; }
  // Device-side enqueue: child levels run after each parent launch (1..3)
  // and errors counted on the device (queue level full / too deep).
  int device_enqueue_levels = kDynLevels - 1;
  // Debug checks: buffers allocated while on get a guard tail
  // of kGuardBytes filled with kGuardByte; every launch is then synchronised
  // (a fault names its kernel) and the guards of its arrays are verified, so
  // a kernel writing past the end of an array is reported by name.
  static constexpr size_t kGuardBytes = 4096;
  static constexpr unsigned char kGuardByte = 0xCE;
  // atomic: Cores::set_debug_checks flips it while job threads read it
  std::atomic<bool> debug_checks{false};
  // D2H of pinned / registered host memory by a copy kernel on the stream
  // (device writes straight into the host pages) instead of
  // hipMemcpyAsync, for copies of at least kKernelD2HMinBytes with 16-byte
  // aligned ends: keeps downloads off the SDMA rings the uploads use, so a
  // download gated on a kernel never blocks an upload queued behind it
  std::atomic<bool> kernel_d2h{false};
  // Kernel profiling timestamps (the counterpart of OpenCL's
  // CL_PROFILING_COMMAND_START / END): while on, every launch goes through
  // hipExtModuleLaunchKernel with a start and a stop event that the runtime
  // stamps from the dispatch itself — the kernel's own execution time,
  // without the gap between back-to-back launches that stream events or a
  // host clock include.  kernel_times() drains them: (kernel, ms) in launch order.
  std::atomic<bool> kernel_times_on{false};
  std::vector<std::pair<std::string, double>> kernel_times();
  static constexpr uint64_t kKernelD2HMinBytes = 1ull << 20;
  uint64_t kernel_d2h_bytes() const { return kernel_d2h_bytes_; }
  int device_enqueue_errors();

  // --- markers (fine-grained queue control, ClCommandQueue.cs:103-112) ---
  // release: the marker also makes earlier writes to HOST memory visible
  // (a system-scope release; set when the compute downloaded results)
  void add_marker(hipStream_t s, bool release = false);
  // A compute that takes its completion from the NEXT marker of its stream:
  // last_marker() becomes (slot, the value that marker will carry) and no
  // HIP call is made; flush_markers() records that marker on every stream
  // with such computes (a device pool coalesces the markers of consecutive
  // tasks: one hipEventRecord per batch instead of per task)
  void defer_marker(hipStream_t s, bool release = false);
  void flush_markers();
  bool has_deferred_markers() const { return deferred_slots_ != 0; }
  long long markers_reached();
  // (slot, value) of the newest marker; a marker is reached once
  // marker_word(slot) >= value.  CPU device: slot -1 (always reached).
  std::pair<int, uint64_t> last_marker() const { return {last_slot_, last_value_}; }
  uint64_t marker_word(int slot);
  long long markers_issued() const { return markers_issued_; }

  // --- user-event gating (ClUserEvent.cs:102-117) -------------------------
  // Every stream of this worker (created on demand) waits until *word >= value.
  void gate_all_streams(const uint32_t* word, uint32_t value);

  // --- graph replay of a repeat loop (hipGraph instead of N launches) ------
  // Launches `fn`'s stream work on `s`; the first call with `key` captures
  // it into a hipGraph, later calls replay the instantiated graph.
  void launch_graph(hipStream_t s, const std::string& key, const std::function<void(hipStream_t)>& fn);
  size_t graphs_cached() const { return graphs_.size(); }

  // --- job thread --------------------------------------------------------
  // Hand-off to a GPU worker's thread.  Both sides spin (with pause) for up
  // to spin_us before blocking on a condition variable: back-to-back computes
  // (a loop of enqueue-mode calls, ~10-20 µs apart) then cost an atomic
  // store and a cache-line transfer per device instead of a futex wake-up
  // (tens of µs on a busy host).  CEK_SPIN_US sets it (0: block at once).
  void post(std::function<void()> fn);
  void wait();  // rethrows the first job exception
  static double spin_us;

  // --- timing (Worker.cs:753-807) ---------------------------------------
  std::map<int, double> bench_ms;

 private:
  void thread_loop();
  int stream_slot(hipStream_t s);

  DeviceInfo dev_;
  std::shared_ptr<Program> prog_;
  int qconc_;
  bool no_pipelining_;
  unsigned dyn_lds_ = 0;
  // device-side enqueue queues (kDynQueueBytes each), one per stream so
  // blobs in flight on concurrent streams never share level counts
  std::unordered_map<hipStream_t, void*> dyn_queues_;
  void* dyn_queue(hipStream_t s);
  std::unordered_map<uint64_t, std::pair<void*, uint64_t>> bufs_;
  std::unordered_map<uint64_t, bool> zc_;
  std::unordered_map<uint64_t, uint64_t> guarded_;  // uid -> guard offset (bytes)
  std::unordered_map<uint64_t, void*> zc_ptr_;      // zero-copy uid -> device view of its host memory
  std::vector<std::pair<uint64_t, void*>>* cap_log_ = nullptr;
  std::shared_ptr<Program> copy_prog_;  // the kernel-D2H copy kernel, built on first use
  hipFunction_t copy_fn_ = nullptr;
  std::mutex copy_mu_;
  std::atomic<uint64_t> kernel_d2h_bytes_{0};
  bool d2h_by_kernel(hipStream_t s, void* host_base, uint64_t off, const void* src_dev, uint64_t n);
  void* buffer_impl(const ArraySpec& a);
  void check_capturable(const ArraySpec& a);  // throws for pageable memory while capturing
  void check_guards(hipStream_t s, const std::string& kernel, const std::vector<ArraySpec>& arrs);
  uint64_t bytes_allocated_ = 0;
  std::mutex buf_mu_;

  int cu_reserve_ = 0;
  hipStream_t new_stream(bool copy_cus);
  void destroy_streams();
  hipStream_t main_ = nullptr;
  std::vector<hipStream_t> cq_;
  hipStream_t pq_[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};
  std::vector<hipEvent_t> events_;
  std::vector<hipEvent_t> join_ev_;  // one per stream slot (join_streams)
  hipEvent_t sleep_ev_ = nullptr;
  hipEvent_t sys_ev_ = nullptr;      // system_release
  std::atomic<int> rr_{0};

  // markers: one 64-bit word per stream slot in pinned host memory
  uint64_t* marker_words_ = nullptr;
  uint64_t* marker_dev_ = nullptr;  // device address of marker_words_ (looked up once)
  std::vector<uint64_t> marker_issued_per_slot_;
  // Event markers (the default): per stream slot, the recorded events not
  // yet seen complete (in issue order: a stream completes them in order),
  // spare events, and how many have completed.  A marker is a barrier packet
  // with a completion signal; hipStreamWriteValue64 runs as a blit kernel
  // (__amd_rocclr_streamOpsWrite) — a kernel dispatch per marker, ~10× the
  // host cost under 8 submitting threads (profiles/r5/README.md).
  struct MarkerRing {
    std::deque<std::pair<hipEvent_t, bool>> pending;  // (event, system-scope release)
    std::deque<hipEvent_t> spare, spare_fenced;
    uint64_t done = 0;
  };
  std::vector<MarkerRing> rings_;
  struct KernelStamp {
    std::string kernel;
    hipEvent_t start, stop;
  };
  // CPU device: measured ns per work item per kernel (one thread), and the
  // shortest task worth handing to a pool thread
  std::unordered_map<std::string, double> cpu_item_ns_;
  static constexpr double kCpuMinTaskNs = 20000.0;
  std::deque<KernelStamp> kstamps_;  // ring: the oldest are dropped past kMaxKernelStamps
  static constexpr size_t kMaxKernelStamps = 1 << 16;
  std::vector<hipEvent_t> kstamp_spare_;
  std::mutex kstamp_mu_;
  hipEvent_t kstamp_event();
  std::mutex marker_mu_;
  bool write_value_markers_ = false;  // CEK_MARKERS=writevalue: the old path
  uint32_t deferred_slots_ = 0;          // bit per stream slot with deferred markers
  uint32_t deferred_release_ = 0;        // ... whose marker must also release host writes
  hipStream_t slot_stream(int slot) const;
  long long markers_issued_ = 0;
  int last_slot_ = -1;
  uint64_t last_value_ = 0;

  std::shared_ptr<CpuPool> pool_;
  std::unordered_map<std::string, hipGraphExec_t> graphs_;

  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  std::deque<std::function<void()>> q_;
  bool busy_ = false, stop_ = false;
  std::atomic<uint64_t> posted_{0}, finished_{0};  // jobs handed over / completed
  std::atomic<bool> sleeping_{false}, waiter_blocked_{false};
  std::exception_ptr err_;
};

}  // namespace cek
