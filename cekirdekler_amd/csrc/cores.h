// Multi-device scheduler — the MI355X-native counterpart of the reference's
// `Cores` (Cores.cs:37-1982): one worker per device, per-compute-id range
// tables driven by the iterative load balancer, and three execution shapes
// per device:
//   * 3-phase (H2D → kernels → D2H) on one in-order stream
//     (Cores.cs:745-835, Worker.cs:821-840/:1033-1114/:1343-1361),
//   * event-driven pipeline: the device's range cut into `blobs` chunks that
//     stream through two half-pipelines, each {read, compute, write} HIP
//     streams joined by hipEvents (Cores.cs:1197-1367, Worker.cs:1411-1567),
//   * driver pipeline: chunk k on round-robin stream k mod Q (Q = queue
//     concurrency, by default the GPU_MAX_HW_QUEUES hardware queues)
//     (Cores.cs:1368-1958).
// plus enqueue mode / async enqueue / no-compute / fine-grained markers /
// repeat + sync kernel (ClNumberCruncher.cs:66-187, Cores.cs:72-126,
// :449, :796-809).  Fan-out runs on persistent worker threads with the GIL
// released, one Python→C++ crossing per compute().
//
// Distributed mode (one process per GPU): the balancer runs on the global
// device list; each rank executes its own device's range and the per-device
// times are exchanged through an Exchanger, so every rank derives the
// identical next split.  Optional RCCL data plane: broadcast `read` arrays
// from rank 0 and all-gather written slices into every replica.
#pragma once
#include <condition_variable>
#include <map>
#include <mutex>

#include "balancer.h"
#include "dist.h"
#include "worker.h"

namespace cek {

struct ComputeCall {
  std::vector<std::string> kernels;
  int repeats = 1;
  std::string repeat_kernel;
  std::vector<ArraySpec> arrays;
  long long global_range = 0;
  long long local_range = 256;
  long long global_offset = 0;
  int compute_id = 1;
  bool pipeline = false;
  bool pipeline_event = true;  // PIPELINE_EVENT=true, PIPELINE_DRIVER=false
  int blobs = 4;
  // Split granularity in work items (0 = local range): every device range is
  // a multiple of it, e.g. to keep the K-split work-groups of one GEMM tile
  // on the same device.  Must be a multiple of local_range.
  long long granularity = 0;
  // Explicit, possibly uneven pipeline blobs (event pipeline, one device
  // holding the whole range): blob k = work items [blob_bounds[k],
  // blob_bounds[k+1]) of the range; blobs alternate between the two
  // half-pipelines.  Arrays may carry per-blob slices (ArraySpec::blob_begin).
  std::vector<long long> blob_bounds;
};

struct CoresConfig {
  int queue_concurrency = 16;
  bool no_pipelining = false;
  bool smooth = true;
  std::vector<std::string> options;
  std::vector<std::string> prebuilt;  // "path|name1,name2"
};

struct ComputeRecord {  // structured per-call record (observability)
  int compute_id = 0;
  double wall_ms = 0;
  std::vector<long long> ranges, references;
  std::vector<double> device_ms;
  uint64_t h2d_bytes = 0, d2h_bytes = 0;
  uint64_t p2p_bytes = 0;     // device→device bytes (read fan-out + keep-resident gather)
  uint64_t gather_bytes = 0;  // of which the keep-resident gather
  uint64_t staged_bytes = 0;  // of p2p_bytes: between GPUs without peer access (host-bounced)
  // where this call's device→device bytes went: "none" (no such copy),
  // "local" (logical devices of one GPU), "xgmi" (peer copies between GPUs),
  // "staged" (some pair without peer access), "pcie" (the read fan-out fell
  // back to one PCIe upload per device because a pair cannot peer)
  std::string p2p_path = "none";
  bool pipelined = false;
};

// Host-triggered event gating device streams (reference ClUserEvent, a
// "development cancelled" feature there, Worker.cs:487-560): gated streams
// execute hipStreamWaitValue32 on a pinned host word; trigger() stores the
// awaited value.  Words come from a never-freed pinned slab, so a stream can
// never poll released memory.
class UserEvent {
 public:
  UserEvent();
  ~UserEvent();
  uint32_t arm();       // value the next gates wait for
  void trigger();
  bool armed() const { return armed_; }
  const uint32_t* word() const { return word_; }

 private:
  uint32_t* word_ = nullptr;
  uint32_t gen_ = 0;
  bool armed_ = false;
};

// Host rendezvous of the local devices inside one compute() (reference
// phase separation: every device finishes reading and computing before any
// device writes back, Cores.cs:751-831).
class PhaseBarrier {
 public:
  explicit PhaseBarrier(int n) : n_(n) {}
  void arrive_and_wait() {
    std::unique_lock<std::mutex> lk(mu_);
    const int gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen_ != gen || broken_; });
    }
  }
  void arrive_and_drop() {  // a failing device must not block the others
    std::lock_guard<std::mutex> lk(mu_);
    --n_;
    if (count_ >= n_ && count_ > 0) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    }
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, count_ = 0, gen_ = 0;
  bool broken_ = false;
};

// A compute() in which one or more local devices raised.
struct DeviceFailure : std::exception {
  std::vector<int> devices;
  std::string msg;
  void add(int w, const std::string& m) {
    devices.push_back(w);
    msg += (msg.empty() ? "" : "; ") + ("device " + std::to_string(w) + ": " + m);
  }
  const char* what() const noexcept override { return msg.c_str(); }
};

class Cores {
 public:
  Cores(const std::vector<DeviceInfo>& devices, const std::string& source, const CoresConfig& cfg);
  ~Cores();

  int error_code() const { return error_code_; }
  const std::string& error_message() const { return error_; }
  std::vector<KernelSig> kernels() const;
  int num_devices() const { return static_cast<int>(workers_.size()); }
  int num_global_devices() const { return global_devices_; }
  const DeviceInfo& device(int i) const { return workers_.at(i)->dev(); }
  double build_ms() const { return build_ms_; }

  void compute(const ComputeCall& call);

  // ---- modes ----
  bool enqueue_mode() const { return enqueue_mode_; }
  void set_enqueue_mode(bool on);
  bool async_enqueue = false;
  bool no_compute = false;
  bool fine_grained = false;
  // with fine_grained: this compute's marker is deferred (Worker::defer_marker)
  // until flush_markers(); the device pool sets it per task
  bool defer_marker = false;
  void flush_markers(int dev) { workers_.at(dev)->flush_markers(); }
  bool smooth = true;
  bool serial = false;  // run devices one after another (isolated timings)
  // Repeat loops with at least this many launches per device are captured
  // into a hipGraph and replayed (0 disables graphs).
  int graph_min_launches = 8;
  // Gate every stream of local device `device` (-1: all) on `ev`: work
  // enqueued afterwards starts only once ev.trigger() (ClUserEvent.cs:102-117).
  void gate(class UserEvent& ev, int device);
  void set_time_scale(int device, double scale);  // injected heterogeneity (tests/bench)
  // injected fixed cost per compute on a device (ms of host time spent before
  // its work, counted in its measured time): tests of the overhead-aware split
  void set_time_offset(int device, double ms);
  // Opt-in overhead-aware balancing (balancer.h predict_split): fits
  // t = a + b·range per device and may leave a device out; single-process
  // jobs only (the law stays the default and the distributed rule).
  bool balancer_predictor = false;
  const FitState* fit_state(int id) const {
    auto it = state_.find(id);
    return it == state_.end() ? nullptr : &it->second.fit;
  }
  // ---- failure handling ----
  // A disabled device gets no range; the balancer runs over the others.
  void set_device_enabled(int device, bool on);
  bool device_enabled(int device) const { return enabled_.at(device); }
  // Make the next `count` computes on local device `device` fail (tests).
  void inject_failure(int device, int count);
  // When a device fails during compute(): disable it and re-run the call on
  // the remaining devices (single-process jobs only).
  bool auto_failover = false;
  // ---- schedule recording (pipeline dependency checks) ----
  // Every transfer / kernel / event edge the pipelines issue is appended as
  // (device, op, logical stream, first work item, work items, event).
  // Logical streams: 0 main, 1+k compute queue k, 17+3h+r pipeline half h
  // role r (0 read, 1 compute, 2 write).
  struct SchedOp {
    int device;
    std::string op;  // h2d | kernel | d2h | rec | wait
    int stream;
    long long begin, count;
    int event;
  };
  bool record_schedule = false;
  std::vector<SchedOp> schedule() {
    std::lock_guard<std::mutex> g(sched_mu_);
    return sched_;
  }
  void clear_schedule() {
    std::lock_guard<std::mutex> g(sched_mu_);
    sched_.clear();
  }
  int failovers() const { return failovers_; }
  void set_dynamic_lds(unsigned bytes);
  // device-side enqueue (cek_enqueue): child levels per parent launch, and
  // the errors counted on the devices so far (syncs)
  void set_device_enqueue_levels(int levels);
  // debug checks: guard tails on new buffers, synchronous checked launches
  void set_debug_checks(bool on);
  bool debug_checks() const { return debug_checks_; }
  // downloads of pinned / registered host memory by a copy kernel instead
  // of hipMemcpyAsync (Worker::kernel_d2h; env CEK_KERNEL_D2H)
  void set_kernel_d2h(bool on) {
    for (auto& w : workers_) w->kernel_d2h = on;
  }
  bool kernel_d2h() const { return !workers_.empty() && workers_[0]->kernel_d2h.load(); }
  // kernel profiling timestamps (Worker::kernel_times_on)
  void set_kernel_times(bool on) {
    for (auto& w : workers_) w->kernel_times_on = on;
  }
  bool kernel_times_on() const { return !workers_.empty() && workers_[0]->kernel_times_on.load(); }
  std::vector<std::pair<std::string, double>> kernel_times(int dev) { return workers_.at(dev)->kernel_times(); }
  // CUs reserved per GPU for copy kernels (Worker::set_cu_reserve); drains
  // and re-creates the streams
  void set_copy_cus(int n) {
    std::lock_guard<std::recursive_mutex> g(call_mu_);
    if (capturing_) throw Error("copy CUs cannot change during a graph capture");
    for (auto& w : workers_) w->set_cu_reserve(n);
  }
  int copy_cus() const { return workers_.empty() ? 0 : workers_[0]->cu_reserve(); }
  // identity of device w's host thread pool (0 for a GPU): equal across
  // crunchers that share one (CpuPool::shared)
  uintptr_t cpu_pool_id(int w) const {
    return (w < 0 || w >= static_cast<int>(workers_.size())) ? 0 : workers_[w]->cpu_pool_id();
  }
  uint64_t kernel_d2h_bytes() const {
    uint64_t b = 0;
    for (auto& w : workers_) b += w->kernel_d2h_bytes();
    return b;
  }
  int device_enqueue_errors();
  // ---- device timeline ----
  // With record_timeline on, the kernels of every compute are bracketed by
  // timing hipEvents on the stream they run on (host clock on the CPU
  // device).  timeline() waits for the recorded work and returns
  // (device, compute id, begin ms, end ms) per span, relative to the first
  // span of that device, then clears the list.
  struct TimelineSpan {
    int device, compute_id;
    double begin_ms, end_ms;
    double abs_begin_ms, abs_end_ms;  // host clock (event_host_ms): comparable across devices
  };
  bool record_timeline = false;
  std::vector<TimelineSpan> timeline();

  // ---- state ----
  bool has_state(int id) const { return state_.count(id) > 0; }
  std::vector<long long> ranges(int id) const;
  std::vector<long long> references(int id) const;
  std::vector<double> benchmarks(int id) const;
  std::vector<std::vector<double>> history(int id) const;
  void set_state(int id, const std::vector<long long>& ranges,
                 const std::vector<std::vector<double>>& history, const std::vector<double>& bench);
  std::vector<int> compute_ids() const;
  int last_compute_id() const { return last_id_; }
  ComputeRecord last_record() const { return last_record_; }

  long long markers_reached();
  long long markers_issued();
  std::pair<int, uint64_t> last_marker(int dev) const { return workers_.at(dev)->last_marker(); }
  uint64_t marker_word(int dev, int slot) { return workers_.at(dev)->marker_word(slot); }
  void finish();  // synchronise every stream of every device
  void release_array(uint64_t uid);
  uint64_t device_bytes(int i) const { return workers_.at(i)->bytes_allocated(); }
  // Raw device pointer of a cached replica (allocates if needed).
  uint64_t device_pointer(int i, const ArraySpec& a);
  void upload(int i, const ArraySpec& a);    // whole array H2D (sync)
  void download(int i, const ArraySpec& a);  // whole array D2H (sync)
  // Keep-resident all-gather inside one process: every device's slice of
  // `a` (by the ranges of compute id `id`) is copied into every other
  // device's replica, GPU↔GPU as peer copies over xGMI (no host bounce).
  // Event-ordered (no host sync in enqueue mode); later computes and
  // downloads wait for the copies on the device.
  void share_slices(int id, const ArraySpec& a, long long local_range);
  // ---- peer topology ----
  // Distinct GPU ordinals of this Cores' devices and hipDeviceCanAccessPeer
  // among them; access is enabled at construction when they span >= 2 GPUs.
  const std::vector<int>& peer_ordinals() const { return peer_ordinals_; }
  const std::vector<std::vector<int>>& peer_matrix() const { return peer_matrix_; }
  const std::string& p2p_path() const { return p2p_path_; }
  bool can_peer(int w1, int w2) const;  // local workers: same GPU, or peer access on
  void copy_between(int src_dev, const ArraySpec& src, int dst_dev, const ArraySpec& dst,
                    uint64_t bytes);  // device→device (peer/xGMI) copy, sync

  // ---- compute graphs (hipGraph capture of a sequence of computes) ----
  // capture_begin() puts every GPU's main stream into (relaxed) stream
  // capture; the computes that follow are recorded, not run: enqueue-mode
  // semantics (split frozen, no host syncs), main stream only, no markers,
  // device spans, peer-read staging or nested repeat graphs.  capture_end()
  // instantiates one graph per GPU and returns its id; graph_launch(id, n)
  // replays it n times back to back on each GPU's main stream — one
  // hipGraphLaunch per GPU per replay instead of one host call per kernel
  // and copy.  Host transfers inside the graph read / write the host
  // arrays at replay time (pinned or registered memory only).  Buffers must
  // exist before capture: run the computes once first.
  void capture_begin();
  int capture_end();
  void graph_launch(int id, int times, bool sync);
  // Host-resident GEMM C = A·Bᵀ streamed in square shells of P row panels
  // (csrc/shell_gemm.cpp): uploads, kernels and downloads of consecutive
  // shells overlap; C comes back shell by shell.  Synchronous.
  void gemm_host_shells(int local_dev, const std::string& kernel, const ArraySpec& A, const ArraySpec& B,
                        const ArraySpec& C, int M, int N, int K, int panels, int group_m, int BM, int BN, int L);
  void graph_destroy(int id);
  bool capturing() const { return capturing_; }

  // ---- distributed ----
  void set_distributed(std::shared_ptr<Exchanger> ex, std::shared_ptr<Comm> comm,
                       int global_devices, int global_base);
  bool dist_gather_writes = false;
  bool dist_broadcast_reads = false;
  // identical host copies on every rank: each uploads 1/N, RCCL all-gathers
  bool dist_split_reads = false;
  int global_base() const { return global_base_; }

  // ---- xGMI fan-out of full `read` arrays ----
  // The reference uploads every `read` array to every device
  // (Worker.cs:833-860): D PCIe copies contending for the host.  With two or
  // more local GPUs computing, an array of at least peer_read_min_bytes that
  // the kernels do not write is instead uploaded 1/D per GPU (each over its
  // own PCIe link) and every GPU pulls the other D-1 chunks straight from its
  // peers' replicas with hipMemcpyPeerAsync: an all-gather over the
  // point-to-point xGMI mesh, one link per peer pair, ordered by events (no
  // host sync).  PCIe carries the array once instead of D times.
  bool peer_reads = true;
  // event pipeline: issue each blob's D2H on its compute stream
  bool pipeline_writes_on_compute_stream = false;
  // event pipeline: every blob's D2H on one write stream (blob order)
  bool pipeline_writes_one_stream = false;
  // event pipeline: issue every blob's uploads on the main stream, after the
  // full reads (one in-order chain; the copies share the SDMA engine
  // anyway).  With separate read streams, the first call after any
  // device-wide sync left the uploads idle ~5 ms after the full reads and
  // some processes stayed at 14 ms per streamed GEMM call instead of 8
  // (profiles/hostres_streaming.md, tools/hostres_stall_probe.py)
  bool pipeline_reads_on_main_stream = true;
  bool pipeline_reads_two_streams = false;
  // driver pipeline (Cores.cs:1368-1858): blob k's upload and kernels stay on
  // queue k mod Q, its download goes to one download stream gated by the
  // blob's kernel event, so no blob's D2H waits in a compute queue ahead of a
  // later blob's upload.  Off: the reference's
  // read→compute→write on the one queue.
  bool driver_downloads_own_stream = true;
  // driver pipeline: blob uploads on the main stream (one in-order chain of
  // copies, as the event pipeline's), each blob's queue waiting for its own
  bool driver_reads_on_main_stream = true;
  // a mixed CPU + GPU call runs the participant with the largest share on
  // the calling thread (off, the default: the CPU device).  Measured on the
  // wave frame: the GPU inline left the CPU a 1 % share and 0.044 ms per
  // frame, the CPU inline an 11 % share and 0.033 ms (GPU alone 0.030)
  bool inline_largest_share = false;
  // CPU + GPU sets: GPU workers sleep-wait in calls whose previous GPU time
  // for the compute id exceeded sleep_wait_min_ms (CEK_ADAPTIVE_SLEEP=0: off)
  bool adaptive_sleep_waits = true;
  double sleep_wait_min_ms = 0.25;
  // GPU workers wait for their streams by sleeping on a blocking-sync event
  // (off by default; CEK_SLEEP_WAITS=1)
  bool sleep_waits = false;  // explicit blobs: partial arrays alternate over two upload streams (slower: 12.7 vs 7.1 ms for the shells, the extra stream shares a hardware queue)
  uint64_t peer_read_min_bytes = 1u << 20;

 private:
  PhaseBarrier* phase_ = nullptr;  // set while a hazardous compute runs
  bool collective(const ComputeCall& c) const;
  void run_device(int w, const ComputeCall& c, long long ref, long long range, bool pipelined,
                  double* out_ms, uint64_t* h2d, uint64_t* d2h);
  void run_device_body(int w, const ComputeCall& c, long long ref, long long range, bool pipelined,
                  double* out_ms, uint64_t* h2d, uint64_t* d2h);
  void run_3phase(Worker& wk, int gidx, const ComputeCall& c, long long ref, long long range,
                  uint64_t* h2d, uint64_t* d2h);
  void run_event_pipeline(Worker& wk, int gidx, const ComputeCall& c, long long ref,
                          long long range, uint64_t* h2d, uint64_t* d2h);
  void run_driver_pipeline(Worker& wk, int gidx, const ComputeCall& c, long long ref,
                           long long range, uint64_t* h2d, uint64_t* d2h);
  void launch_kernels(Worker& wk, hipStream_t s, const ComputeCall& c, long long ref,
                      long long range);
  void launch_kernels_body(Worker& wk, hipStream_t s, const ComputeCall& c, long long ref,
                           long long range);
  struct PendingSpan {
    int device, compute_id;
    hipEvent_t begin, end;      // GPU: timing events (device epoch: first span's begin)
    double host_begin, host_end;  // CPU device: host clock
  };
  std::mutex tl_mu_;
  std::vector<PendingSpan> pending_spans_;
  void full_reads(Worker& wk, hipStream_t s, const ComputeCall& c, uint64_t* h2d);
  // per-call peer fan-out: which arrays were staged, and per local worker the
  // event its streams wait on before using them
  struct PeerEvents {
    hipEvent_t up = nullptr;      // this GPU's chunk uploaded
    hipEvent_t pulled = nullptr;  // every other chunk pulled into this GPU
  };
  std::vector<PeerEvents> peer_ev_;
  std::vector<hipEvent_t> peer_ready_;  // every participant pulled: kernels may modify the staged arrays
  std::vector<char> staged_arr_;  // by array index, for the current call
  std::vector<char> staged_dev_;  // by local worker, for the current call
  uint64_t stage_peer_reads(const ComputeCall& c, const std::vector<long long>& ranges,
                            std::vector<uint64_t>& h2d);
  int worker_index(const Worker& wk) const;
  // peer topology
  std::vector<int> peer_ordinals_;
  std::vector<std::vector<int>> peer_matrix_;
  std::string p2p_path_ = "none";
  std::vector<int> ord_index_;  // local worker -> index into peer_ordinals_ (-1: CPU device)
  void init_peer_topology();
  // per-call device→device accounting
  struct D2DCount {
    uint64_t bytes = 0, xgmi = 0, local = 0, staged = 0;
    bool pcie_fallback = false;
  } d2d_;
  void count_d2d(int ws, int wd, uint64_t bytes);
  uint64_t d2d_copy(int ws, int wd, char* dst, const char* src, uint64_t bytes, hipStream_t s, int stream_worker);
  // keep-resident gather (ArraySpec::gather): kernels-done event per worker,
  // copies-done event per GPU worker; later work waits on every copies-done
  // event while gather_pending_
  std::vector<hipEvent_t> kdone_, pushed_;
  bool gather_pending_ = false;
  bool all_gpu_ = true;  // every local device is a GPU (device-time spans feed the balancer)
  bool call_gathers_ = false;  // the running call gathers in-process
  hipEvent_t gather_event(std::vector<hipEvent_t>& v, int w);
  void wait_gather(Worker& wk, hipStream_t s);
  uint64_t issue_gather(const ComputeCall& c, const struct BalancerState& st, const std::vector<int>& arrays,
                        const std::vector<std::vector<std::pair<long long, long long>>>* owned = nullptr);

  std::vector<std::unique_ptr<Worker>> workers_;
  std::map<int, BalancerState> state_;
  std::vector<double> time_scale_;
  std::vector<double> time_offset_;
  std::vector<bool> enabled_;
  // one compute()/state access at a time per Cores (Python releases the GIL
  // during compute, so two threads may call into the same cruncher)
  mutable std::recursive_mutex call_mu_;
  std::mutex sched_mu_;
  std::vector<SchedOp> sched_;
  void log_op(int gidx, const char* op, int stream, long long begin, long long count, int event = -1) {
    if (!record_schedule) return;
    std::lock_guard<std::mutex> g(sched_mu_);
    sched_.push_back({gidx, op, stream, begin, count, event});
  }
  std::vector<int> inject_;
  int failovers_ = 0;
  bool debug_checks_ = false;
  void compute_once(const ComputeCall& call, struct DeviceFailure* failed);
  void balance(struct BalancerState& st, bool first, long long G, long long step);
  std::string error_;
  int error_code_ = 0;
  double build_ms_ = 0;
  bool enqueue_mode_ = false;
  bool capturing_ = false;
  bool sleep_this_call_ = false;  // compute_once: GPU waits of this call sleep
  std::vector<void*> shell_dims_;         // gemm_host_shells: per-kernel dims, per worker
  std::vector<size_t> shell_dims_cap_;
  std::vector<std::vector<int>> shell_dims_host_;  // what shell_dims_ holds (re-uploaded only on change)
  std::vector<void*> shell_dims_pin_;               // pinned staging for that upload
  void restore_capture_state();  // the modes capture_begin saved
  struct CaptureSaved {
    bool device_spans, peer_reads, async_enqueue, fine_grained, enqueue_mode, record_timeline;
    int graph_min_launches;
    bool kernel_times;
  } cap_saved_{};
  std::map<int, std::vector<hipGraphExec_t>> graphs_;  // id -> one exec per local worker (null: CPU)
  // buffers each worker handed out while capturing: (uid, pointer) — a graph
  // replays those pointers, so graph_launch refuses to run once any of them
  // was released or reallocated
  std::vector<std::vector<std::pair<uint64_t, void*>>> cap_logs_;
  std::map<int, std::vector<std::vector<std::pair<uint64_t, void*>>>> graph_bufs_;
  int next_graph_id_ = 1;
  double enqueue_t0_ = 0;
  int last_id_ = 0;
  // ---- device-time spans for the balancer ----
  // Each GPU device's work in a compute is bracketed by a pair of timing
  // hipEvents on the stream it starts and ends on; the balancer gets the
  // device time between them (hipEventElapsedTime) instead of host wall
  // clock.  Sync mode reuses pair 0; enqueue mode takes a fresh pair per
  // compute and, when the mode is left, credits each device with the union
  // of its spans (so devices of one process re-balance by their own device
  // time, not the shared wall clock).
  struct DevSpans {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
    int used = 0;
    hipEvent_t gap_a = nullptr, gap_b = nullptr;  // phase-barrier idle gap
    bool gap = false;
    hipStream_t batch = nullptr;  // enqueue mode: stream of the open batch span
  };
  std::vector<DevSpans> spans_;
 public:
  bool device_spans = true;  // CEK_DEVICE_SPANS=0: host wall clock instead
  // async enqueue computes' downloads after the next compute's uploads
  // (CEK_DEFER_DOWNLOADS=0: in each compute's own order)
  bool deferred_downloads = true;
  bool single_device_spans = false;  // spans with one device in the job too (CEK_SINGLE_DEVICE_SPANS=1)
  // a system-scope release marker after kernels that may store into
  // zero-copy host memory (per compute in sync mode, once per batch when
  // enqueue mode is left); CEK_ZC_RELEASE=0 turns it off
  bool zc_release = true;
 private:
  bool spans_on() const;
  bool one_span_per_batch() const;
  void close_batch_spans();
  void span_begin(Worker& wk, hipStream_t s);
  void span_end(Worker& wk, hipStream_t s);
  double span_ms(int w);              // sync mode: the last span (stream drained)
  double enqueue_spans_ms(int w);     // enqueue mode: union of the spans so far
  // Async enqueue mode: a compute's downloads are issued after the NEXT
  // compute's uploads (or when the batch ends).  A stream's copies go to an
  // SDMA queue that other streams share and that runs in submission order:
  // a download, which waits for its kernel, would hold back every later
  // compute's upload behind it, and the computes would run one after the
  // other instead of side by side (rocprofv3 trace, profiles/r5/README.md).
  struct PendingD2H {
    hipStream_t s;
    ArraySpec a;
    uint64_t begin, count;
  };
  struct PendingSpanEnd {
    hipStream_t s;
    int index;
  };
  std::vector<std::vector<PendingD2H>> pending_d2h_;          // per local device
  std::vector<std::vector<PendingSpanEnd>> pending_span_end_;  // per local device
  std::vector<std::vector<hipEvent_t>> order_events_;          // per local device (flush ordering)
  bool defer_downloads(const Worker& wk) const;
  bool must_flush_before(const Worker& wk, hipStream_t s, const ComputeCall& c) const;
  void flush_downloads(Worker& wk, hipStream_t next = nullptr, const ComputeCall* c = nullptr);
  ComputeRecord last_record_;
  CoresConfig cfg_;

  std::shared_ptr<Exchanger> ex_;
  std::shared_ptr<Comm> comm_;
  int global_devices_ = 0;
  int global_base_ = 0;
};

}  // namespace cek
