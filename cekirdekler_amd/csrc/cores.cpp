#include "cores.h"

#include <cstring>

#include <algorithm>
#include <map>
#include <numeric>
#include <sstream>
#include <thread>

#include "memory.h"
#include "trace.h"
#include "xgmi.h"

namespace cek {

Cores::Cores(const std::vector<DeviceInfo>& devices, const std::string& source,
             const CoresConfig& cfg)
    : cfg_(cfg) {
  smooth = cfg.smooth;
  double t0 = now_ms();
  // One code object per architecture, one module per device.
  std::ostringstream errs;
  int cpu_slot = 0;
  for (size_t i = 0; i < devices.size(); ++i) {
    const auto& d = devices[i];
    std::shared_ptr<Program> prog;
    try {
      prog = Program::build(d, source, cfg.options, d.type == kGPU ? cfg.prebuilt : std::vector<std::string>{});
    } catch (const std::exception& e) {
      errs << "device " << i << " (" << d.name << "): " << e.what() << "\n";
      error_code_ = 1;
      continue;
    }
    if (!prog->ok()) {
      errs << "device " << i << " (" << d.name << ") build failed:\n" << prog->log() << "\n";
      error_code_ = 1;
      continue;
    }
    workers_.emplace_back(new Worker(d, prog, cfg.queue_concurrency, cfg.no_pipelining,
                                     d.type == kGPU ? 0 : cpu_slot++));
  }
  error_ = errs.str();
  if (workers_.empty() && error_code_ == 0) {
    error_code_ = 1;
    error_ = "no device selected";
  }
  global_devices_ = static_cast<int>(workers_.size());
  spans_.resize(workers_.size());
  pending_d2h_.resize(workers_.size());
  pending_span_end_.resize(workers_.size());
  order_events_.resize(workers_.size());
  if (const char* e = std::getenv("CEK_DEVICE_SPANS")) device_spans = std::string(e) != "0";
  if (const char* e = std::getenv("CEK_SINGLE_DEVICE_SPANS")) single_device_spans = std::string(e) == "1";
  if (const char* e = std::getenv("CEK_DEFER_DOWNLOADS")) deferred_downloads = std::string(e) != "0";
  if (const char* e = std::getenv("CEK_INLINE_LARGEST")) inline_largest_share = std::string(e) != "0";
  if (const char* e = std::getenv("CEK_ADAPTIVE_SLEEP")) adaptive_sleep_waits = std::string(e) != "0";
  if (const char* e = std::getenv("CEK_KERNEL_D2H")) set_kernel_d2h(std::string(e) != "0");
  if (const char* e = std::getenv("CEK_ZC_RELEASE")) zc_release = std::string(e) != "0";
  // CEK_SLEEP_WAITS=1: GPU workers wait for their streams by sleeping on a
  // blocking-sync event instead of HIP's default wait, leaving the core to a
  // co-executing CPU device.  Off by default: measured on the wave example
  // it adds ~5 µs of wake-up per GPU frame (0.038 -> 0.043 ms) and gains
  // nothing on host-resident co-execution (profiles/round4_session6.md)
  if (const char* e = std::getenv("CEK_SLEEP_WAITS")) sleep_waits = std::string(e) != "0";
  time_scale_.assign(workers_.size(), 1.0);
  time_offset_.assign(workers_.size(), 0.0);
  enabled_.assign(workers_.size(), true);
  inject_.assign(workers_.size(), 0);
  init_peer_topology();
  all_gpu_ = std::all_of(workers_.begin(), workers_.end(), [](const std::unique_ptr<Worker>& w) { return w->gpu(); });
  build_ms_ = now_ms() - t0;
}

// Distinct GPUs of this device set: enable peer access among them (xGMI) so
// the read fan-out, the keep-resident gather and copy_between move bytes
// GPU↔GPU directly.  A pair that cannot peer is recorded: the read fan-out
// then falls back to one PCIe upload per device, and gather copies between
// that pair are counted as staged.
void Cores::init_peer_topology() {
  ord_index_.assign(workers_.size(), -1);
  peer_ordinals_.clear();
  for (size_t w = 0; w < workers_.size(); ++w) {
    if (!workers_[w]->gpu()) continue;
    const int o = workers_[w]->dev().ordinal;
    auto it = std::find(peer_ordinals_.begin(), peer_ordinals_.end(), o);
    ord_index_[w] = static_cast<int>(it - peer_ordinals_.begin());
    if (it == peer_ordinals_.end()) peer_ordinals_.push_back(o);
  }
  if (peer_ordinals_.size() >= 2) {
    peer_matrix_ = enable_peer_access_among(peer_ordinals_);
  } else {
    peer_matrix_.assign(peer_ordinals_.size(), std::vector<int>(peer_ordinals_.size(), 1));
  }
  p2p_path_ = peer_path(peer_matrix_);
}

bool Cores::can_peer(int w1, int w2) const {
  const int a = ord_index_.at(w1), b = ord_index_.at(w2);
  if (a < 0 || b < 0) return false;
  return a == b || (peer_matrix_[a][b] && peer_matrix_[b][a]);
}

void Cores::count_d2d(int ws, int wd, uint64_t bytes) {
  d2d_.bytes += bytes;
  if (ord_index_[ws] == ord_index_[wd])
    d2d_.local += bytes;
  else if (can_peer(ws, wd))
    d2d_.xgmi += bytes;
  else
    d2d_.staged += bytes;
}

// One device→device copy on stream s of local worker sw (either end): a D2D
// copy inside one GPU, a peer copy between GPUs (over xGMI when peer access
// is on; the runtime stages it through host memory otherwise), by SDMA or a
// copy kernel on sw's GPU, whichever the calibrated engine table says is
// faster for this pair and size (xgmi.h; SDMA for an uncalibrated pair).
uint64_t Cores::d2d_copy(int ws, int wd, char* dst, const char* src, uint64_t bytes, hipStream_t s, int sw) {
  if (!bytes || dst == src) return 0;
  const int os = workers_[ws]->dev().ordinal, od = workers_[wd]->dev().ordinal;
  const bool peer_ok = os == od || can_peer(ws, wd);
  if (peer_ok)
    peer_copy(dst, od, src, os, bytes, s, workers_[sw]->dev().ordinal);
  else
    CEK_HIP(hipMemcpyPeerAsync(dst, od, src, os, bytes, s));  // staged by the runtime
  count_d2d(ws, wd, bytes);
  return bytes;
}

hipEvent_t Cores::gather_event(std::vector<hipEvent_t>& v, int w) {
  if (v.size() < workers_.size()) v.resize(workers_.size(), nullptr);
  if (!v[w]) {
    workers_[w]->set_device();
    CEK_HIP(hipEventCreateWithFlags(&v[w], hipEventDisableTiming));
  }
  return v[w];
}

// Work about to run on stream s of wk must see the last gather's copies, and
// must not overwrite a slice the copies are still reading.
void Cores::wait_gather(Worker& wk, hipStream_t s) {
  if (!gather_pending_) return;
  for (size_t g = 0; g < pushed_.size(); ++g) {
    if (!pushed_[g]) continue;
    if (wk.gpu())
      CEK_HIP(hipStreamWaitEvent(s, pushed_[g], 0));
    else
      CEK_HIP(hipEventSynchronize(pushed_[g]));
  }
}

// Keep-resident gather of the call's `arrays` (indices into c.arrays): each
// device's slice (by this call's split) lands in every other device's replica.
// Issued from the calling thread once every device has enqueued its kernels:
// GPU g's main stream waits for the kernels of every GPU (no replica is
// overwritten while a kernel of this call still reads it), pulls the CPU
// device's slices from host memory, pushes its own slice to every other
// replica (peer copies over xGMI), and records pushed_[g].  No host sync in
// enqueue mode; otherwise the copies are complete when compute() returns.
uint64_t Cores::issue_gather(const ComputeCall& c, const BalancerState& st, const std::vector<int>& arrays,
                             const std::vector<std::vector<std::pair<long long, long long>>>* owned) {
  const int n = num_devices();
  std::vector<int> on;  // enabled local devices: they hold replicas
  for (int w = 0; w < n; ++w)
    if (enabled_[w]) on.push_back(w);
  if (on.size() < 2 || arrays.empty()) return 0;
  // the work-item ranges each device holds fresh results for: its own slice
  // of this call's split, or (after a failover) its slice plus the slices it
  // recomputed for failed devices
  std::vector<std::vector<std::pair<long long, long long>>> own(n);
  for (int w : on) {
    if (owned)
      own[w] = (*owned)[w];
    else
      own[w].push_back({st.references[global_base_ + w], st.ranges[global_base_ + w]});
  }
  uint64_t moved = 0;
  struct Piece {
    std::vector<char*> ptr;
    std::vector<std::vector<std::pair<uint64_t, uint64_t>>> seg;  // per worker: (byte offset, bytes)
  };
  std::vector<Piece> pcs(arrays.size());
  for (size_t i = 0; i < arrays.size(); ++i) {
    const ArraySpec& a = c.arrays[arrays[i]];
    Piece& p = pcs[i];
    p.ptr.assign(n, nullptr);
    p.seg.assign(n, {});
    for (int w : on) {
      for (auto& r : own[w]) {
        uint64_t b, k;
        a.slice(r.first, r.second, c.local_range, b, k);
        const uint64_t off = std::min<uint64_t>(b * a.elem_size, a.bytes);
        const uint64_t len = std::min<uint64_t>(k * a.elem_size, a.bytes - off);
        if (len) p.seg[w].push_back({off, len});
      }
      workers_[w]->set_device();
      p.ptr[w] = static_cast<char*>(workers_[w]->buffer(a));
    }
  }
  std::vector<int> gpus;
  for (int w : on)
    if (workers_[w]->gpu()) gpus.push_back(w);
  for (int g : gpus) {
    Worker& wg = *workers_[g];
    wg.set_device();
    hipStream_t m = wg.main_stream();
    for (int d : gpus)
      if (kdone_.size() > static_cast<size_t>(d) && kdone_[d]) CEK_HIP(hipStreamWaitEvent(m, kdone_[d], 0));
    for (size_t i = 0; i < arrays.size(); ++i) {
      const ArraySpec& a = c.arrays[arrays[i]];
      Piece& p = pcs[i];
      for (int s : on) {  // the CPU device's slices: host → this replica
        if (workers_[s]->gpu()) continue;
        for (auto& sg : p.seg[s]) {
          CEK_HIP(hipMemcpyAsync(p.ptr[g] + sg.first, static_cast<const char*>(a.host) + sg.first, sg.second,
                                 hipMemcpyHostToDevice, m));
          moved += sg.second;
        }
      }
      for (auto& sg : p.seg[g]) {
        for (int d : on) {  // this GPU's slices → every other replica
          if (d == g || p.ptr[d] == p.ptr[g]) continue;
          if (workers_[d]->gpu()) {
            moved += d2d_copy(g, d, p.ptr[d] + sg.first, p.ptr[g] + sg.first, sg.second, m, g);
            log_op(global_base_ + d, "gather", 0, static_cast<long long>(sg.first), static_cast<long long>(sg.second),
                   global_base_ + g);
          } else {
            CEK_HIP(hipMemcpyAsync(p.ptr[d] + sg.first, p.ptr[g] + sg.first, sg.second, hipMemcpyDeviceToHost, m));
            moved += sg.second;
          }
        }
      }
    }
    CEK_HIP(hipEventRecord(gather_event(pushed_, g), m));
  }
  gather_pending_ = true;
  if (!enqueue_mode_) {
    for (int g : gpus) {
      workers_[g]->set_device();
      CEK_HIP(hipStreamSynchronize(workers_[g]->main_stream()));
    }
    gather_pending_ = false;
  }
  return moved;
}

Cores::~Cores() {
  try {
    finish();
  } catch (...) {
  }
  if (capturing_) {
    for (auto& w : workers_) {
      w->set_device();
      hipGraph_t g = nullptr;
      if (hipStreamEndCapture(w->main_stream(), &g) == hipSuccess && g) (void)hipGraphDestroy(g);
      (void)hipGetLastError();
    }
    capturing_ = false;
  }
  for (auto& kv : graphs_)
    for (size_t i = 0; i < kv.second.size() && i < workers_.size(); ++i)
      if (kv.second[i]) {
        workers_[i]->set_device();
        (void)hipGraphExecDestroy(kv.second[i]);
      }
  graphs_.clear();
  for (size_t w = 0; w < spans_.size() && w < workers_.size(); ++w) {
    workers_[w]->set_device();
    for (auto& p : spans_[w].pool) {
      (void)hipEventDestroy(p.first);
      (void)hipEventDestroy(p.second);
    }
    if (spans_[w].gap_a) (void)hipEventDestroy(spans_[w].gap_a);
    if (spans_[w].gap_b) (void)hipEventDestroy(spans_[w].gap_b);
    if (w < order_events_.size())
      for (hipEvent_t e : order_events_[w]) (void)hipEventDestroy(e);
  }
  for (size_t w = 0; w < shell_dims_.size() && w < workers_.size(); ++w)
    if (shell_dims_[w]) {
      workers_[w]->set_device();
      (void)hipFree(shell_dims_[w]);
    }
  for (void* p : shell_dims_pin_) host_free(p);
  for (size_t w = 0; w < peer_ev_.size() && w < workers_.size(); ++w) {
    if (!peer_ev_[w].up) continue;
    workers_[w]->set_device();
    (void)hipEventDestroy(peer_ev_[w].up);
    (void)hipEventDestroy(peer_ev_[w].pulled);
  }
  for (auto* v : {&peer_ready_, &kdone_, &pushed_})
    for (size_t w = 0; w < v->size() && w < workers_.size(); ++w)
      if ((*v)[w]) {
        workers_[w]->set_device();
        (void)hipEventDestroy((*v)[w]);
      }
  workers_.clear();
}

std::vector<KernelSig> Cores::kernels() const {
  if (workers_.empty()) return {};
  return workers_[0]->program().kernels();
}

void Cores::set_time_scale(int device, double scale) {
  if (device < 0 || device >= static_cast<int>(time_scale_.size())) throw Error("bad device index");
  time_scale_[device] = scale;
}

void Cores::set_time_offset(int device, double ms) {
  if (device < 0 || device >= static_cast<int>(time_offset_.size())) throw Error("bad device index");
  time_offset_[device] = ms;
}

void Cores::set_device_enabled(int device, bool on) {
  if (device < 0 || device >= static_cast<int>(enabled_.size())) throw Error("bad device index");
  if (!on && ex_) throw Error("devices cannot be disabled in a distributed job");
  const bool rejoin = on && !enabled_[device];
  enabled_[device] = on;
  // A re-enabled device has no range and no timing: restart every compute id
  // from the equal split so that it rejoins with a real share instead of
  // whatever a stale bench value would give it.
  if (rejoin)
    for (auto& kv : state_) {
      std::fill(kv.second.ranges.begin(), kv.second.ranges.end(), 0LL);
      std::fill(kv.second.bench.begin(), kv.second.bench.end(), 0.0);
      for (auto& h : kv.second.history) std::fill(h.begin(), h.end(), 0.0);
    }
}

void Cores::inject_failure(int device, int count) {
  if (device < 0 || device >= static_cast<int>(inject_.size())) throw Error("bad device index");
  inject_[device] = count;
}

// Runs the reference law over the enabled devices only (all of them unless
// some were disabled); disabled devices keep a zero range.
void Cores::balance(BalancerState& st, bool first, long long G, long long step) {
  const int D = global_devices_;
  std::vector<int> on;
  for (int i = 0; i < D; ++i)
    if (i < global_base_ || i >= global_base_ + num_devices() || enabled_[i - global_base_]) on.push_back(i);
  if (on.empty()) throw Error("every device is disabled");
  if (static_cast<int>(on.size()) == D) {
    if (first)
      initial_split(D, smooth, st.history, G, st.ranges, step);
    else if (!(balancer_predictor && !ex_ && predict_split(st.fit, st.bench, st.last_wall_ms, G, st.ranges, step, st.calls >= 2)))
      load_balance(st.bench, smooth, st.history, G, st.ranges, step);
    return;
  }
  const size_t n = on.size();
  std::vector<long long> r(n);
  std::vector<double> b(n);
  std::vector<std::vector<double>> h(st.history.size(), std::vector<double>(n));
  for (size_t j = 0; j < n; ++j) {
    r[j] = st.ranges.empty() ? 0 : st.ranges[on[j]];
    b[j] = st.bench.empty() ? 0.0 : st.bench[on[j]];
    for (size_t d = 0; d < st.history.size(); ++d) h[d][j] = st.history[d][on[j]];
  }
  const bool sub_first = first || std::all_of(r.begin(), r.end(), [](long long x) { return x == 0; });
  if (sub_first)
    initial_split(static_cast<int>(n), smooth, h, G, r, step);
  else
    load_balance(b, smooth, h, G, r, step);
  st.ranges.assign(D, 0);
  for (size_t j = 0; j < n; ++j) {
    st.ranges[on[j]] = r[j];
    for (size_t d = 0; d < st.history.size(); ++d) st.history[d][on[j]] = h[d][j];
  }
}

void Cores::set_device_enqueue_levels(int levels) {
  if (levels < 0 || levels > kDynLevels - 1)
    throw Error("device enqueue levels must be in [0, " + std::to_string(kDynLevels - 1) + "]");
  for (auto& w : workers_) w->device_enqueue_levels = levels;
}

void Cores::set_debug_checks(bool on) {
  debug_checks_ = on;
  for (auto& w : workers_) w->debug_checks = on;
}

int Cores::device_enqueue_errors() {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  int e = 0;
  for (auto& w : workers_) e += w->device_enqueue_errors();
  return e;
}

void Cores::set_dynamic_lds(unsigned bytes) {
  for (auto& w : workers_) w->set_dynamic_lds(bytes);
}

void Cores::set_distributed(std::shared_ptr<Exchanger> ex, std::shared_ptr<Comm> comm,
                            int global_devices, int global_base) {
  ex_ = std::move(ex);
  comm_ = std::move(comm);
  global_devices_ = global_devices;
  global_base_ = global_base;
  state_.clear();
}

void Cores::set_enqueue_mode(bool on) {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  if (capturing_) throw Error("enqueue mode cannot change during a graph capture");
  if (on && !enqueue_mode_) {
    enqueue_t0_ = now_ms();
  } else if (!on && enqueue_mode_) {
    close_batch_spans();
    if (zc_release)  // one system-scope release per device for the whole batch (zero-copy stores)
      for (auto& w : workers_)
        if (w->gpu()) {
          w->join_streams(w->main_stream());
          w->system_release(w->main_stream());
        }
    finish();
    double el = now_ms() - enqueue_t0_;
    auto it = state_.find(last_id_);
    std::vector<double> ms(num_devices());
    for (int w = 0; w < num_devices(); ++w) {
      // GPU: union of this device's timed spans; CPU device: wall clock
      double dev = workers_[w]->gpu() ? enqueue_spans_ms(w) : -1.0;
      if (!all_gpu_) dev = -1.0;  // mixed CPU+GPU: one clock for everybody
      ms[w] = (dev > 0 ? dev : el) * time_scale_[w];
    }
    // every rank leaves enqueue mode together: exchange so all ranks keep the
    // identical benchmark vector (and hence derive the identical next split)
    std::vector<double> all = ex_ ? ex_->allgather(ms) : ms;
    if (it != state_.end()) {
      if (ex_ && all.size() == it->second.bench.size()) {
        it->second.bench = all;
      } else {
        for (int w = 0; w < num_devices(); ++w) {
          size_t g = static_cast<size_t>(global_base_ + w);
          if (g < it->second.bench.size()) it->second.bench[g] = ms[w];
        }
      }
    }
  }
  enqueue_mode_ = on;
}

std::vector<long long> Cores::ranges(int id) const {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  auto it = state_.find(id);
  return it == state_.end() ? std::vector<long long>{} : it->second.ranges;
}
std::vector<long long> Cores::references(int id) const {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  auto it = state_.find(id);
  return it == state_.end() ? std::vector<long long>{} : it->second.references;
}
std::vector<double> Cores::benchmarks(int id) const {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  auto it = state_.find(id);
  return it == state_.end() ? std::vector<double>{} : it->second.bench;
}
std::vector<std::vector<double>> Cores::history(int id) const {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  auto it = state_.find(id);
  return it == state_.end() ? std::vector<std::vector<double>>{} : it->second.history;
}
std::vector<int> Cores::compute_ids() const {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  std::vector<int> out;
  for (auto& kv : state_) out.push_back(kv.first);
  return out;
}

void Cores::set_state(int id, const std::vector<long long>& ranges,
                      const std::vector<std::vector<double>>& history, const std::vector<double>& bench) {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  auto& st = state_[id];
  st.ranges = ranges;
  st.history = history;
  st.bench = bench;
  st.global_range = std::accumulate(ranges.begin(), ranges.end(), 0LL);
  st.references.assign(ranges.size(), 0);
  long long acc = st.global_offset;
  for (size_t i = 0; i < ranges.size(); ++i) {
    st.references[i] = acc;
    acc += ranges[i];
  }
}

long long Cores::markers_reached() {
  long long r = 0;
  for (auto& w : workers_) r += w->markers_reached();
  return r;
}

long long Cores::markers_issued() {
  long long r = 0;
  for (auto& w : workers_) r += w->markers_issued();
  return r;
}

void Cores::capture_begin() {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  if (capturing_) throw Error("capture_begin: already capturing");
  for (auto& w : workers_)
    if (!w->gpu()) throw Error("compute graphs need GPU devices only (the CPU device runs computes at once)");
  if (debug_checks_) throw Error("compute graphs cannot be captured with debug checks on (they synchronise)");
  for (auto& w : workers_) {
    w->wait();
    flush_downloads(*w);
    w->sync_all();
  }
  cap_saved_ = {device_spans, peer_reads, async_enqueue, fine_grained, enqueue_mode_, record_timeline,
                graph_min_launches, kernel_times_on()};
  set_kernel_times(false);  // stamped launches are not captured (their events would never be recorded)
  device_spans = false;
  record_timeline = false;
  peer_reads = false;
  async_enqueue = false;
  fine_grained = false;
  graph_min_launches = 0;
  enqueue_mode_ = true;  // split frozen, no syncs (state is restored by capture_end)
  cap_logs_.assign(workers_.size(), {});
  for (size_t i = 0; i < workers_.size(); ++i) {
    Worker& w = *workers_[i];
    w.set_device();
    hipError_t e = hipStreamBeginCapture(w.main_stream(), hipStreamCaptureModeRelaxed);
    if (e != hipSuccess) {
      // undo: end the captures already begun and restore the modes
      (void)hipGetLastError();
      for (size_t j = 0; j < i; ++j) {
        workers_[j]->set_device();
        hipGraph_t g = nullptr;
        if (hipStreamEndCapture(workers_[j]->main_stream(), &g) == hipSuccess && g) (void)hipGraphDestroy(g);
        workers_[j]->set_capture_log(nullptr);
      }
      restore_capture_state();
      throw Error(std::string("hipStreamBeginCapture failed on ") + w.dev().name + ": " + hipGetErrorString(e));
    }
    w.set_capture_log(&cap_logs_[i]);
  }
  capturing_ = true;
}

void Cores::restore_capture_state() {
  device_spans = cap_saved_.device_spans;
  peer_reads = cap_saved_.peer_reads;
  async_enqueue = cap_saved_.async_enqueue;
  fine_grained = cap_saved_.fine_grained;
  graph_min_launches = cap_saved_.graph_min_launches;
  enqueue_mode_ = cap_saved_.enqueue_mode;
  record_timeline = cap_saved_.record_timeline;
  set_kernel_times(cap_saved_.kernel_times);
}

int Cores::capture_end() {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  if (!capturing_) throw Error("capture_end: not capturing");
  for (auto& w : workers_) {
    w->wait();
    w->set_capture_log(nullptr);
  }
  std::vector<hipGraphExec_t> execs(workers_.size(), nullptr);
  std::string err;
  for (size_t i = 0; i < workers_.size(); ++i) {
    Worker& w = *workers_[i];
    w.set_device();
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(w.main_stream(), &g);
    if (e != hipSuccess || !g) {
      (void)hipGetLastError();
      err = std::string("stream capture failed on ") + w.dev().name + ": " + hipGetErrorString(e);
      continue;
    }
    e = hipGraphInstantiate(&execs[i], g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      err = std::string("graph instantiation failed on ") + w.dev().name + ": " + hipGetErrorString(e);
    }
  }
  capturing_ = false;
  restore_capture_state();
  for (auto& sp : spans_) sp.used = 0;
  if (!err.empty()) {
    for (size_t i = 0; i < execs.size(); ++i)
      if (execs[i]) {
        workers_[i]->set_device();
        (void)hipGraphExecDestroy(execs[i]);
      }
    throw Error(err);
  }
  const int id = next_graph_id_++;
  graphs_[id] = std::move(execs);
  graph_bufs_[id] = std::move(cap_logs_);
  cap_logs_.clear();
  return id;
}

void Cores::graph_launch(int id, int times, bool sync) {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  auto it = graphs_.find(id);
  if (it == graphs_.end()) throw Error("graph_launch: unknown graph id");
  const auto& bufs = graph_bufs_[id];
  for (size_t i = 0; i < bufs.size() && i < workers_.size(); ++i)
    for (const auto& ub : bufs[i])
      if (!workers_[i]->buffer_is(ub.first, ub.second))
        throw Error("graph " + std::to_string(id) + " is stale: array " + std::to_string(ub.first) +
                    " was released or reallocated on " + workers_[i]->dev().name +
                    " since the capture (capture it again)");
  for (size_t i = 0; i < workers_.size(); ++i) {
    if (!it->second[i]) continue;
    Worker& w = *workers_[i];
    w.set_device();
    for (int r = 0; r < times; ++r) CEK_HIP(hipGraphLaunch(it->second[i], w.main_stream()));
  }
  if (sync)
    for (size_t i = 0; i < workers_.size(); ++i) {
      workers_[i]->set_device();
      CEK_HIP(hipStreamSynchronize(workers_[i]->main_stream()));
    }
}

void Cores::graph_destroy(int id) {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  auto it = graphs_.find(id);
  if (it == graphs_.end()) return;
  for (size_t i = 0; i < it->second.size(); ++i)
    if (it->second[i]) {
      workers_[i]->set_device();
      (void)hipGraphExecDestroy(it->second[i]);
    }
  graphs_.erase(it);
  graph_bufs_.erase(id);
}

void Cores::finish() {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  if (capturing_) throw Error("finish() during a graph capture (end the capture first)");
  for (auto& w : workers_) {
    w->wait();
    flush_downloads(*w);
    w->sync_all();
  }
  gather_pending_ = false;  // every gather copy (on the main streams) is done
}

// A deferred download of the array being released still targets its host
// buffer: issue it and let it land before the device buffer goes away (the
// host buffer is alive for the duration of the caller's __del__).
void Cores::release_array(uint64_t uid) {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  for (size_t w = 0; w < workers_.size(); ++w) {
    Worker& wk = *workers_[w];
    if (w < pending_d2h_.size()) {
      std::vector<hipStream_t> streams;
      for (const auto& p : pending_d2h_[w])
        if (p.a.uid == uid && std::find(streams.begin(), streams.end(), p.s) == streams.end()) streams.push_back(p.s);
      if (!streams.empty()) {
        flush_downloads(wk);
        if (wk.gpu())
          for (hipStream_t s : streams) CEK_HIP(hipStreamSynchronize(s));
      }
    }
    wk.release(uid);
  }
}

uint64_t Cores::device_pointer(int i, const ArraySpec& a) {
  Worker& w = *workers_.at(i);
  w.set_device();
  return reinterpret_cast<uint64_t>(w.buffer(a));
}

void Cores::upload(int i, const ArraySpec& a) {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  Worker& w = *workers_.at(i);
  w.set_device();
  flush_downloads(w);
  hipStream_t s = w.main_stream();
  wait_gather(w, s);
  w.h2d(s, a, 0, a.bytes / a.elem_size);
  if (w.gpu()) CEK_HIP(hipStreamSynchronize(s));
}

void Cores::download(int i, const ArraySpec& a) {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  Worker& w = *workers_.at(i);
  w.set_device();
  flush_downloads(w);
  hipStream_t s = w.main_stream();
  wait_gather(w, s);
  w.d2h(s, a, 0, a.bytes / a.elem_size);
  if (w.gpu()) CEK_HIP(hipStreamSynchronize(s));
}

void Cores::copy_between(int src_dev, const ArraySpec& src, int dst_dev, const ArraySpec& dst,
                         uint64_t bytes) {
  Worker& ws = *workers_.at(src_dev);
  Worker& wd = *workers_.at(dst_dev);
  if (bytes > src.bytes || bytes > dst.bytes) throw Error("copy_between: size exceeds array");
  if (!ws.gpu() && !wd.gpu()) {
    std::memcpy(dst.host, src.host, bytes);
    return;
  }
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  if (ws.gpu() && wd.gpu()) {
    // On the source's main stream, after everything queued on either
    // device (every stream: with async enqueue a compute may sit on a
    // compute queue, still writing the source or reading the destination).
    // Later work on ANY stream of either device waits for the copy through
    // the gather-pending events (no host sync in enqueue mode).
    ws.set_device();
    void* sp = ws.buffer(src);
    wd.set_device();
    void* dp = wd.buffer(dst);
    wd.join_streams(wd.main_stream());
    hipEvent_t before = gather_event(kdone_, dst_dev);
    CEK_HIP(hipEventRecord(before, wd.main_stream()));
    ws.set_device();
    hipStream_t s = ws.main_stream();
    wait_gather(ws, s);
    ws.join_streams(s);
    CEK_HIP(hipStreamWaitEvent(s, before, 0));
    d2d_ = D2DCount();
    d2d_copy(src_dev, dst_dev, static_cast<char*>(dp), static_cast<const char*>(sp), bytes, s, src_dev);
    hipEvent_t after = gather_event(pushed_, src_dev);
    CEK_HIP(hipEventRecord(after, s));
    wd.set_device();
    CEK_HIP(hipStreamWaitEvent(wd.main_stream(), after, 0));
    gather_pending_ = true;  // compute streams of both devices wait on `after` too
    if (!enqueue_mode_) {
      ws.set_device();
      CEK_HIP(hipStreamSynchronize(s));
      gather_pending_ = false;
    }
    return;
  }
  if (ws.gpu()) {  // GPU → CPU device (host memory)
    ws.set_device();
    hipStream_t s = ws.main_stream();
    CEK_HIP(hipMemcpyAsync(dst.host, ws.buffer(src), bytes, hipMemcpyDeviceToHost, s));
    CEK_HIP(hipStreamSynchronize(s));
  } else {  // CPU → GPU
    wd.set_device();
    hipStream_t s = wd.main_stream();
    CEK_HIP(hipMemcpyAsync(wd.buffer(dst), src.host, bytes, hipMemcpyHostToDevice, s));
    CEK_HIP(hipStreamSynchronize(s));
  }
}

void Cores::share_slices(int id, const ArraySpec& a, long long local_range) {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  auto it = state_.find(id);
  if (it == state_.end()) throw Error("share_slices: unknown compute id");
  if (capturing_) throw Error("share_slices during a graph capture");
  // the copies follow whatever is queued on every GPU's main stream
  for (int w = 0; w < num_devices(); ++w) {
    if (!workers_[w]->gpu() || !enabled_[w]) continue;
    workers_[w]->set_device();
    wait_gather(*workers_[w], workers_[w]->main_stream());
    CEK_HIP(hipEventRecord(gather_event(kdone_, w), workers_[w]->main_stream()));
  }
  ComputeCall c;
  c.arrays = {a};
  c.local_range = local_range;
  d2d_ = D2DCount();
  issue_gather(c, it->second, {0});
}

// ------------------------------------------------------------- compute --

// time the calling worker spent in the phase barrier of the current compute
static thread_local double t_phase_wait = 0;
static thread_local bool t_phase_arrived = false;

// ---------------------------------------------------------------- UserEvent --

namespace {
std::mutex g_ue_mu;
uint32_t* g_ue_slab = nullptr;
int g_ue_next = 0;
constexpr int kUserEventSlots = 4096;
}  // namespace

UserEvent::UserEvent() {
  std::lock_guard<std::mutex> g(g_ue_mu);
  if (!g_ue_slab) {
    bool pinned = false;
    g_ue_slab = static_cast<uint32_t*>(host_alloc(kUserEventSlots * sizeof(uint32_t), 4096, &pinned));
    std::memset(g_ue_slab, 0, kUserEventSlots * sizeof(uint32_t));
  }
  if (g_ue_next >= kUserEventSlots) throw Error("too many user events in this process");
  word_ = &g_ue_slab[g_ue_next++];
}

UserEvent::~UserEvent() {
  if (armed_) trigger();  // never leave a stream blocked on a dead event
}

uint32_t UserEvent::arm() {
  armed_ = true;
  return gen_ + 1;
}

void UserEvent::trigger() {
  __atomic_store_n(word_, gen_ + 1, __ATOMIC_RELEASE);
  ++gen_;
  armed_ = false;
}

void Cores::gate(UserEvent& ev, int device) {
  const uint32_t v = ev.arm();
  for (int w = 0; w < num_devices(); ++w)
    if (device < 0 || device == w) workers_[w]->gate_all_streams(ev.word(), v);
}

void Cores::launch_kernels(Worker& wk, hipStream_t s, const ComputeCall& c, long long ref,
                           long long range) {
  if (!record_timeline || no_compute) {
    launch_kernels_body(wk, s, c, ref, range);
    return;
  }
  int dev = 0;
  while (dev < num_devices() && workers_[dev].get() != &wk) ++dev;
  PendingSpan sp{dev, c.compute_id, nullptr, nullptr, 0, 0};
  if (wk.gpu()) {
    CEK_HIP(hipEventCreateWithFlags(&sp.begin, kTimingEventFlags));
    CEK_HIP(hipEventCreateWithFlags(&sp.end, kTimingEventFlags));
    CEK_HIP(hipEventRecord(sp.begin, s));
    launch_kernels_body(wk, s, c, ref, range);
    CEK_HIP(hipEventRecord(sp.end, s));
  } else {
    sp.host_begin = now_ms();
    launch_kernels_body(wk, s, c, ref, range);
    sp.host_end = now_ms();
  }
  std::lock_guard<std::mutex> g(tl_mu_);
  pending_spans_.push_back(sp);
}

std::vector<Cores::TimelineSpan> Cores::timeline() {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  std::vector<PendingSpan> spans;
  {
    std::lock_guard<std::mutex> g(tl_mu_);
    spans.swap(pending_spans_);
  }
  std::vector<TimelineSpan> out;
  std::map<int, PendingSpan> epoch;  // first span per device
  for (auto& sp : spans) epoch.emplace(sp.device, sp);
  for (auto& sp : spans) {
    const PendingSpan& e0 = epoch.at(sp.device);
    TimelineSpan t{sp.device, sp.compute_id, 0, 0, 0, 0};
    if (sp.begin) {
      CEK_HIP(hipEventSynchronize(sp.end));
      float b = 0, e = 0;
      CEK_HIP(hipEventElapsedTime(&b, e0.begin, sp.begin));
      CEK_HIP(hipEventElapsedTime(&e, e0.begin, sp.end));
      t.begin_ms = b;
      t.end_ms = e;
      const int ord = workers_[sp.device]->dev().ordinal;
      t.abs_begin_ms = event_host_ms(ord, sp.begin);
      t.abs_end_ms = event_host_ms(ord, sp.end);
    } else {
      t.begin_ms = sp.host_begin - e0.host_begin;
      t.end_ms = sp.host_end - e0.host_begin;
      t.abs_begin_ms = sp.host_begin;
      t.abs_end_ms = sp.host_end;
    }
    out.push_back(t);
  }
  for (auto& sp : spans)
    if (sp.begin) {
      (void)hipEventDestroy(sp.begin);
      (void)hipEventDestroy(sp.end);
    }
  return out;
}

void Cores::launch_kernels_body(Worker& wk, hipStream_t s, const ComputeCall& c, long long ref,
                                long long range) {
  if (no_compute) return;
  const int reps = std::max(1, c.repeats);
  auto body = [&](hipStream_t st) {
    for (int r = 0; r < reps; ++r) {
      for (auto& k : c.kernels)
        wk.launch(st, k, c.arrays, ref, range, static_cast<int>(c.local_range), c.global_range);
      if (!c.repeat_kernel.empty())
        wk.launch(st, c.repeat_kernel, c.arrays, 0, c.local_range, static_cast<int>(c.local_range),
                  c.local_range);
    }
  };
  const int launches = reps * (static_cast<int>(c.kernels.size()) + (c.repeat_kernel.empty() ? 0 : 1));
  if (!wk.gpu() || graph_min_launches <= 0 || launches < graph_min_launches || range <= 0) {
    body(s);
    return;
  }
  // A launch-bound repeat loop is captured once into a hipGraph and replayed;
  // the key holds everything the captured launches bake in (kernels, ranges,
  // device buffer addresses).
  std::string key = std::to_string(reps) + "|" + c.repeat_kernel + "|" + std::to_string(ref) + "|" +
                    std::to_string(range) + "|" + std::to_string(c.local_range) + "|" +
                    std::to_string(c.global_range);
  for (auto& k : c.kernels) key += "|" + k;
  for (auto& a : c.arrays) key += "|" + std::to_string(reinterpret_cast<uintptr_t>(wk.buffer(a)));
  wk.launch_graph(s, key, body);
}

// Enqueue mode with one device in the whole job: nothing to balance, so no
// span events between the back-to-back computes (the host clock times the
// enqueued batch when the mode is left).
// Device-time span events only where they are read: every local device a
// GPU (with a CPU device in the set all devices share the host clock, see
// run_device_body) and more than one device in the whole job.  With one
// device there is no split to balance, so its compute time is the host's
// stopwatch (the reference's clock, Worker.cs:779-807) and no span events go
// into its streams (two event records and an elapsed-time query per
// synchronous compute).  CEK_SINGLE_DEVICE_SPANS=1 keeps them there.
bool Cores::spans_on() const {
  return device_spans && all_gpu_ && (global_devices_ > 1 || single_device_spans);
}

// An enqueued batch gets one span per device (opened by its first compute,
// closed when the mode is left) when no two local devices share a GPU: one
// local device (a rank of a distributed job) or distinct GPUs in one
// process.  Logical devices of one GPU keep a span per compute — their
// batches overlap on shared hardware, and only per-compute spans separate
// their busy time.
bool Cores::one_span_per_batch() const {
  if (!enqueue_mode_ || async_enqueue) return false;
  std::vector<int> ords;
  for (int w = 0; w < num_devices(); ++w) {
    if (!workers_[w]->gpu()) continue;
    const int o = workers_[w]->dev().ordinal;
    if (std::find(ords.begin(), ords.end(), o) != ords.end()) return false;
    ords.push_back(o);
  }
  return true;
}

void Cores::span_begin(Worker& wk, hipStream_t s) {
  if (!wk.gpu() || !spans_on()) return;
  const int w = worker_index(wk);
  DevSpans& d = spans_[w];
  if (one_span_per_batch()) {
    // no event marker sits between two back-to-back computes of the batch
    if (d.used > 0) return;
    if (d.pool.empty()) {
      hipEvent_t a, b;
      CEK_HIP(hipEventCreateWithFlags(&a, kTimingEventFlags));
      CEK_HIP(hipEventCreateWithFlags(&b, kTimingEventFlags));
      d.pool.emplace_back(a, b);
    }
    d.used = 1;
    d.batch = s;
    d.gap = false;
    CEK_HIP(hipEventRecord(d.pool[0].first, s));
    return;
  }
  // enqueue mode keeps up to kMaxSpans pairs; past that the last pair's end
  // is re-recorded, so its span stretches over the remaining computes
  constexpr int kMaxSpans = 1024;
  if (enqueue_mode_ && d.used >= kMaxSpans) return;
  const int i = enqueue_mode_ ? d.used++ : 0;
  while (static_cast<int>(d.pool.size()) <= i) {
    hipEvent_t a, b;
    CEK_HIP(hipEventCreateWithFlags(&a, kTimingEventFlags));
    CEK_HIP(hipEventCreateWithFlags(&b, kTimingEventFlags));
    d.pool.emplace_back(a, b);
  }
  d.gap = false;
  CEK_HIP(hipEventRecord(d.pool[i].first, s));
}

void Cores::span_end(Worker& wk, hipStream_t s) {
  if (!wk.gpu() || !spans_on()) return;
  DevSpans& d = spans_[worker_index(wk)];
  if (one_span_per_batch()) return;  // closed at the mode's end
  const int i = enqueue_mode_ ? d.used - 1 : 0;
  if (i < 0) return;
  CEK_HIP(hipEventRecord(d.pool[i].second, s));
}

double Cores::span_ms(int w) {
  DevSpans& d = spans_[w];
  if (!spans_on() || d.pool.empty()) return -1.0;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, d.pool[0].first, d.pool[0].second) != hipSuccess) {
    (void)hipGetLastError();
    return -1.0;
  }
  double out = ms;
  if (d.gap) {
    float g = 0.f;
    if (hipEventElapsedTime(&g, d.gap_a, d.gap_b) == hipSuccess)
      out -= g;
    else
      (void)hipGetLastError();
  }
  return out;
}

void Cores::close_batch_spans() {
  for (int w = 0; w < num_devices(); ++w) {
    DevSpans& d = spans_[w];
    if (!d.batch || d.used <= 0) continue;
    workers_[w]->set_device();
    CEK_HIP(hipEventRecord(d.pool[0].second, d.batch));
    d.batch = nullptr;
  }
}

double Cores::enqueue_spans_ms(int w) {
  DevSpans& d = spans_[w];
  const int n = d.used;
  d.used = 0;
  if (n <= 0) return -1.0;
  workers_[w]->set_device();
  std::vector<std::pair<double, double>> iv;
  for (int i = 0; i < n; ++i) {
    float b = 0.f, e = 0.f;
    if (hipEventElapsedTime(&b, d.pool[0].first, d.pool[i].first) != hipSuccess ||
        hipEventElapsedTime(&e, d.pool[0].first, d.pool[i].second) != hipSuccess) {
      (void)hipGetLastError();
      return -1.0;
    }
    iv.emplace_back(b, e);
  }
  std::sort(iv.begin(), iv.end());
  double total = 0, cb = iv[0].first, ce = iv[0].second;
  for (size_t i = 1; i < iv.size(); ++i) {
    if (iv[i].first > ce) {
      total += ce - cb;
      cb = iv[i].first;
      ce = iv[i].second;
    } else {
      ce = std::max(ce, iv[i].second);
    }
  }
  return total + (ce - cb);
}

int Cores::worker_index(const Worker& wk) const {
  for (int i = 0; i < num_devices(); ++i)
    if (workers_[i].get() == &wk) return i;
  return -1;
}

uint64_t Cores::stage_peer_reads(const ComputeCall& c, const std::vector<long long>& ranges,
                                 std::vector<uint64_t>& h2d) {
  const int nloc = num_devices();
  staged_arr_.assign(c.arrays.size(), 0);
  staged_dev_.assign(nloc, 0);
  if (!peer_reads || (comm_ && (dist_broadcast_reads || dist_split_reads))) return 0;
  std::vector<int> part;  // local GPUs computing in this call
  for (int w = 0; w < nloc; ++w)
    if (workers_[w]->gpu() && enabled_[w] && ranges[global_base_ + w] > 0) part.push_back(w);
  const int P = static_cast<int>(part.size());
  if (P < 2) return 0;
  // every pair of distinct GPUs must peer; otherwise each device uploads the
  // whole array over its own PCIe link (reference behaviour), explicitly
  for (int x = 0; x < P; ++x)
    for (int y = 0; y < P; ++y)
      if (!can_peer(part[x], part[y])) {
        d2d_.pcie_fallback = true;
        return 0;
      }
  bool any = false;
  for (size_t i = 0; i < c.arrays.size(); ++i) {
    const auto& a = c.arrays[i];
    if (!a.zc && a.read && !a.partial && !a.write && !a.wo && !a.write_all && a.bytes >= peer_read_min_bytes) {
      staged_arr_[i] = 1;
      any = true;
    }
  }
  if (!any) return 0;
  if (static_cast<int>(peer_ev_.size()) < nloc) peer_ev_.resize(nloc);
  for (int w : part) {
    Worker& wk = *workers_[w];
    wk.set_device();
    if (!peer_ev_[w].up) {
      CEK_HIP(hipEventCreateWithFlags(&peer_ev_[w].up, hipEventDisableTiming));
      CEK_HIP(hipEventCreateWithFlags(&peer_ev_[w].pulled, hipEventDisableTiming));
    }
    staged_dev_[w] = 1;
  }
  uint64_t p2p = 0;
  for (size_t i = 0; i < c.arrays.size(); ++i) {
    if (!staged_arr_[i]) continue;
    const auto& a = c.arrays[i];
    // chunk k of P: 4 KiB-aligned byte ranges (multiples of every element size)
    uint64_t chunk = (a.bytes + P - 1) / P;
    chunk = (chunk + 4095) / 4096 * 4096;
    std::vector<uint64_t> off(P), len(P);
    std::vector<char*> ptr(P);
    for (int k = 0; k < P; ++k) {
      off[k] = std::min<uint64_t>(k * chunk, a.bytes);
      len[k] = std::min<uint64_t>(chunk, a.bytes - off[k]);
      workers_[part[k]]->set_device();
      ptr[k] = static_cast<char*>(workers_[part[k]]->buffer(a));
    }
    // 1) every GPU uploads its chunk over its own PCIe link, after the peers
    //    finished pulling from its replica in the previous call (enqueue mode
    //    runs ahead without host syncs)
    for (int k = 0; k < P; ++k) {
      Worker& wk = *workers_[part[k]];
      wk.set_device();
      hipStream_t m = wk.main_stream();
      for (int j = 0; j < P; ++j)
        if (j != k) CEK_HIP(hipStreamWaitEvent(m, peer_ev_[part[j]].pulled, 0));
      if (len[k]) {
        CEK_HIP(hipMemcpyAsync(ptr[k] + off[k], static_cast<const char*>(a.host) + off[k], len[k],
                               hipMemcpyHostToDevice, m));
        h2d[part[k]] += len[k];
      }
      CEK_HIP(hipEventRecord(peer_ev_[part[k]].up, m));
    }
    // 2) every GPU pulls the other chunks from their owners over xGMI
    for (int k = 0; k < P; ++k) {
      Worker& wd = *workers_[part[k]];
      wd.set_device();
      hipStream_t m = wd.main_stream();
      for (int j = 0; j < P; ++j) {
        if (j == k || !len[j]) continue;
        Worker& ws = *workers_[part[j]];
        CEK_HIP(hipStreamWaitEvent(m, peer_ev_[part[j]].up, 0));
        p2p += d2d_copy(part[j], part[k], ptr[k] + off[j], ptr[j] + off[j], len[j], m, part[k]);
        (void)ws;
        log_op(global_base_ + part[k], "p2p", 0, static_cast<long long>(off[j]), static_cast<long long>(len[j]),
               global_base_ + part[j]);
      }
      CEK_HIP(hipEventRecord(peer_ev_[part[k]].pulled, m));
    }
  }
  // 3) a GPU's kernels may modify a staged array in place (read without
  //    write-back does not mean const): they start only once every peer has
  //    pulled this GPU's chunk out of its replica
  if (peer_ready_.size() < static_cast<size_t>(nloc)) peer_ready_.resize(nloc, nullptr);
  for (int k = 0; k < P; ++k) {
    Worker& wk = *workers_[part[k]];
    wk.set_device();
    hipStream_t m = wk.main_stream();
    for (int j = 0; j < P; ++j)
      if (j != k) CEK_HIP(hipStreamWaitEvent(m, peer_ev_[part[j]].pulled, 0));
    if (!peer_ready_[part[k]]) CEK_HIP(hipEventCreateWithFlags(&peer_ready_[part[k]], hipEventDisableTiming));
    CEK_HIP(hipEventRecord(peer_ready_[part[k]], m));
  }
  return p2p;
}

void Cores::full_reads(Worker& wk, hipStream_t s, const ComputeCall& c, uint64_t* h2d) {
  const bool dist = comm_ && dist_broadcast_reads;
  const int w = worker_index(wk);
  if (w >= 0 && w < static_cast<int>(staged_dev_.size()) && staged_dev_[w] && s != wk.main_stream())
    CEK_HIP(hipStreamWaitEvent(s, peer_ready_[w], 0));  // staged on the main stream
  for (size_t i = 0; i < c.arrays.size(); ++i) {
    const auto& a = c.arrays[i];
    if (a.zc || a.partial || !a.read) continue;
    if (w >= 0 && w < static_cast<int>(staged_dev_.size()) && staged_dev_[w] && i < staged_arr_.size() &&
        staged_arr_[i])
      continue;  // already staged by the xGMI fan-out
    if (comm_ && dist_split_reads) {
      // Split upload + all-gather (every rank's host copy holds the same
      // data): rank g copies chunk g of the array over its own PCIe link,
      // then one RCCL ring all-gather over xGMI completes every replica.
      // Each link carries 1/N of the array instead of all of it.
      const int W = global_devices_;
      uint64_t chunk = (a.bytes + W - 1) / W;
      chunk = (chunk + a.elem_size - 1) / a.elem_size * a.elem_size;
      std::vector<uint64_t> offs(W), sizes(W);
      for (int g = 0; g < W; ++g) {
        offs[g] = std::min<uint64_t>(g * chunk, a.bytes);
        sizes[g] = std::min<uint64_t>(chunk, a.bytes - offs[g]);
      }
      wk.h2d(s, a, offs[global_base_] / a.elem_size, sizes[global_base_] / a.elem_size);
      *h2d += sizes[global_base_];
      comm_->allgatherv(wk.buffer(a), offs, sizes, s);
    } else if (dist) {
      if (global_base_ == 0) {
        wk.h2d(s, a, 0, a.bytes / a.elem_size);
        *h2d += a.bytes;
      }
      comm_->broadcast(wk.buffer(a), a.bytes, 0, s);
    } else {
      wk.h2d(s, a, 0, a.bytes / a.elem_size);
      *h2d += a.bytes;
    }
  }
}

// The call issues RCCL collectives (broadcast / split-read all-gather /
// written-slice all-gather) that every rank must join, whatever its range.
bool Cores::collective(const ComputeCall& c) const {
  if (!comm_) return false;
  if (dist_gather_writes || dist_broadcast_reads || dist_split_reads) return true;
  return std::any_of(c.arrays.begin(), c.arrays.end(), [](const ArraySpec& a) { return a.gather && !a.zc; });
}

// Kernels that may store into zero-copy (host) memory: close the device's
// work with a system-scope release (the span events carry none).
static bool writes_host_memory(const ComputeCall& c) {
  return std::any_of(c.arrays.begin(), c.arrays.end(), [](const ArraySpec& a) { return a.zc && !a.ro; });
}

// A marker after this compute must release host-memory writes (system
// scope): kernels stored into zero-copy memory, or results were downloaded
// (a blit-kernel D2H into hipHostMalloc pages is a kernel store to host
// memory).  Device-resident computes get a fence-less marker.
static bool marker_needs_release(const ComputeCall& c) {
  return std::any_of(c.arrays.begin(), c.arrays.end(),
                     [](const ArraySpec& a) { return (a.zc && !a.ro) || (!a.zc && (a.write || a.write_all)); });
}

bool Cores::defer_downloads(const Worker& wk) const {
  // not with markers (a task's marker must follow its own download, and a
  // deferred one would wait for the next task), collectives, phase barriers
  // or a graph capture
  return deferred_downloads && wk.gpu() && enqueue_mode_ && async_enqueue && !fine_grained && !capturing_ &&
         !phase_ && !comm_;
}

// A deferred download may not be overtaken by the next compute's uploads
// when they share an in-order stream (the download would follow the upload)
// or touch the same array (a stale host copy going up over the result, or
// the next upload reading host memory the download has not filled yet).
bool Cores::must_flush_before(const Worker& wk, hipStream_t s, const ComputeCall& c) const {
  const int w = worker_index(wk);
  if (w < 0 || w >= static_cast<int>(pending_d2h_.size())) return false;
  for (const auto& p : pending_d2h_[w]) {
    if (p.s == s) return true;
    for (const auto& a : c.arrays)
      if (!a.zc && a.uid == p.a.uid) return true;
  }
  return false;
}

// Issue the pending downloads.  With `next` (the stream the next compute
// runs on) and that compute `c`, `next` also waits for every pending
// download on another stream whose array the compute touches.
void Cores::flush_downloads(Worker& wk, hipStream_t next, const ComputeCall* c) {
  const int w = worker_index(wk);
  if (w < 0 || w >= static_cast<int>(pending_d2h_.size())) return;
  auto& pd = pending_d2h_[w];
  auto& ps = pending_span_end_[w];
  if (pd.empty() && ps.empty()) return;
  wk.set_device();
  std::vector<hipStream_t> order;  // streams `next` must wait for
  for (const auto& p : pd) {
    wk.d2h(p.s, p.a, p.begin, p.count);
    if (c && p.s != next && std::find(order.begin(), order.end(), p.s) == order.end())
      for (const auto& a : c->arrays)
        if (!a.zc && a.uid == p.a.uid) {
          order.push_back(p.s);
          break;
        }
  }
  if (!order.empty() && wk.gpu()) {
    auto& ev = order_events_[w];
    while (ev.size() < order.size()) {
      hipEvent_t e;
      CEK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ev.push_back(e);
    }
    for (size_t i = 0; i < order.size(); ++i) {
      CEK_HIP(hipEventRecord(ev[i], order[i]));
      CEK_HIP(hipStreamWaitEvent(next, ev[i], 0));
    }
  }
  pd.clear();
  DevSpans& d = spans_[w];
  for (const auto& p : ps)
    if (p.index >= 0 && p.index < static_cast<int>(d.pool.size())) CEK_HIP(hipEventRecord(d.pool[p.index].second, p.s));
  ps.clear();
}

void Cores::run_3phase(Worker& wk, int gidx, const ComputeCall& c, long long ref, long long range,
                       uint64_t* h2d, uint64_t* d2h) {
  hipStream_t s = nullptr;
  if (wk.gpu())
    s = (enqueue_mode_ && async_enqueue) ? wk.compute_stream(wk.next_compute_queue()) : wk.main_stream();
  const bool defer = defer_downloads(wk);
  if (!defer || must_flush_before(wk, s, c))
    flush_downloads(wk, s, &c);  // this compute runs after every earlier download
  if (wk.gpu() && s != wk.main_stream()) wait_gather(wk, s);
  span_begin(wk, s);
  // across ranks: written slices all-gathered by RCCL (every written array
  // with dist_gather_writes, else the arrays flagged gather)
  const bool gather = comm_ && (dist_gather_writes || std::any_of(c.arrays.begin(), c.arrays.end(),
                                                                  [](const ArraySpec& a) { return a.gather; }));
  auto gathered = [&](const ArraySpec& a) {
    return comm_ && !a.zc && !a.write_all && (a.gather || (dist_gather_writes && (a.write || a.wo)));
  };
  // phase 1: host → device (partial slice wins over full read; an array
  // with explicit blob slices, run without its pipeline, goes up whole)
  for (auto& a : c.arrays) {
    if (a.zc) continue;
    if (a.partial) {
      uint64_t b, n;
      if (!a.blob_begin.empty()) {
        b = 0;
        n = a.bytes / a.elem_size;
      } else {
        a.slice(ref, range, c.local_range, b, n);
      }
      wk.h2d(s, a, b, n);
      *h2d += n * a.elem_size;
    }
  }
  full_reads(wk, s, c, h2d);
  // the earlier computes' downloads go into the copy queues after this
  // compute's uploads
  if (defer) flush_downloads(wk);
  // phase 2: kernels
  launch_kernels(wk, s, c, ref, range);
  if (call_gathers_ && wk.gpu()) {  // in-process gather: this device's kernels are enqueued
    const int w = worker_index(wk);
    CEK_HIP(hipEventRecord(gather_event(kdone_, w), s));
  }
  // optional device-side all-gather of written slices (distributed keep-resident)
  if (gather) {
    auto& st = state_[c.compute_id];
    for (auto& a : c.arrays) {
      if (!gathered(a)) continue;
      std::vector<uint64_t> offs(global_devices_), sizes(global_devices_);
      for (int g = 0; g < global_devices_; ++g) {
        uint64_t b, n;
        a.slice(st.references[g], st.ranges[g], c.local_range, b, n);
        offs[g] = b * a.elem_size;
        sizes[g] = n * a.elem_size;
        if (offs[g] + sizes[g] > a.bytes) sizes[g] = offs[g] < a.bytes ? a.bytes - offs[g] : 0;
      }
      comm_->allgatherv(wk.buffer(a), offs, sizes, s);
    }
  }
  // Phase separation when an array is both read whole and written back:
  // no device may write its slice into host memory another device is still
  // reading (reference: all reads and computes finish before any write).
  if (phase_) {
    DevSpans* ds = wk.gpu() ? &spans_[worker_index(wk)] : nullptr;
    if (ds) {
      if (!ds->gap_a) {
        CEK_HIP(hipEventCreateWithFlags(&ds->gap_a, kTimingEventFlags));
        CEK_HIP(hipEventCreateWithFlags(&ds->gap_b, kTimingEventFlags));
      }
      CEK_HIP(hipEventRecord(ds->gap_a, s));
    }
    if (wk.gpu()) wk.wait_stream(s, sleep_waits || sleep_this_call_);
    t_phase_arrived = true;
    const double w0 = now_ms();
    phase_->arrive_and_wait();
    t_phase_wait = now_ms() - w0;  // not this device's work: kept out of its time
    if (ds) {
      CEK_HIP(hipEventRecord(ds->gap_b, s));
      ds->gap = true;
    }
  }
  // phase 3: device → host (deferred in async enqueue mode, see PendingD2H)
  const int wi = defer ? worker_index(wk) : -1;
  auto download = [&](const ArraySpec& a, uint64_t b, uint64_t n) {
    if (wi >= 0)
      pending_d2h_[wi].push_back({s, a, b, n});
    else
      wk.d2h(s, a, b, n);
  };
  bool deferred_any = false;
  for (size_t i = 0; i < c.arrays.size(); ++i) {
    const auto& a = c.arrays[i];
    if (a.zc || !a.write) continue;
    deferred_any = wi >= 0;
    if (a.write_all) {
      if (static_cast<int>(i % global_devices_) == gidx) {
        download(a, 0, a.bytes / a.elem_size);
        *d2h += a.bytes;
      }
    } else if (gathered(a)) {  // the replica holds every rank's slice
      download(a, 0, a.bytes / a.elem_size);
      *d2h += a.bytes;
    } else {
      uint64_t b, n;
      a.slice(ref, range, c.local_range, b, n);
      download(a, b, n);
      *d2h += n * a.elem_size;
    }
  }
  if (deferred_any && wk.gpu() && spans_on()) {
    // the span closes after the deferred download too
    const DevSpans& d = spans_[wi];
    pending_span_end_[wi].push_back({s, d.used - 1});
  } else {
    span_end(wk, s);
  }
  if (zc_release && !enqueue_mode_ && writes_host_memory(c)) wk.system_release(s);
  if (fine_grained) {
    if (defer_marker)
      wk.defer_marker(s, marker_needs_release(c));
    else
      wk.add_marker(s, marker_needs_release(c));
  }
  if (!enqueue_mode_ && wk.gpu()) wk.wait_stream(s, sleep_waits || sleep_this_call_);
}

void Cores::run_event_pipeline(Worker& wk, int gidx, const ComputeCall& c, long long ref,
                               long long range, uint64_t* h2d, uint64_t* d2h) {
  const long long B = std::max(1, c.blobs);
  const long long chunk = range / B;
  const int halves = (B % 2 == 0) ? 2 : 1;
  const long long per_half = B / halves;
  hipStream_t m = wk.main_stream();
  span_begin(wk, m);
  full_reads(wk, m, c, h2d);
  log_op(gidx, "h2d", 0, -1, -1);  // full reads
  int slot = 0;
  hipEvent_t ev_full = nullptr;
  if (wk.gpu()) {
    ev_full = wk.event(slot);
    CEK_HIP(hipEventRecord(ev_full, m));
    for (int h = 0; h < halves; ++h) CEK_HIP(hipStreamWaitEvent(wk.pipe_stream(h, 1), ev_full, 0));
  }
  log_op(gidx, "rec", 0, 0, 0, slot);
  for (int h = 0; h < halves; ++h) log_op(gidx, "wait", 17 + 3 * h + 1, 0, 0, slot);
  ++slot;
  // Interleave the two half-pipelines' chunks so both read streams start
  // early; explicit blobs (c.blob_bounds) alternate between the halves.
  const bool explicit_blobs = !c.blob_bounds.empty();
  const long long nblob = explicit_blobs ? static_cast<long long>(c.blob_bounds.size()) - 1 : per_half * halves;
  const int used_halves = explicit_blobs ? (nblob >= 2 ? 2 : 1) : halves;
  // Optional (pipeline_reads_two_streams, off): the partial arrays of an
  // explicit blob alternate between the main stream and a second upload
  // stream, and each blob's kernels wait for both.  Alone, one stream of
  // 8 MiB copies pays ~11 µs per copy that two streams hide (5.04 vs
  // 4.72 ms for 256 MiB); inside the shell pipeline the extra stream shares
  // a hardware queue with kernel and download streams and the call slows
  // from 7.1 to 12.7 ms (profiles/round4_session4.md), so it stays off.
  const bool two_reads = explicit_blobs && pipeline_reads_on_main_stream && pipeline_reads_two_streams;
  hipStream_t rs2 = nullptr;
  const int rs2id = 17;  // pipe_stream(0, 0), as logged for the schedule checker
  if (two_reads) {
    if (wk.gpu()) {
      rs2 = wk.pipe_stream(0, 0);
      CEK_HIP(hipStreamWaitEvent(rs2, ev_full, 0));
    }
    log_op(gidx, "wait", rs2id, 0, 0, 0);
  }
  for (long long q = 0; q < nblob; ++q) {
    {
      const long long k = explicit_blobs ? q : q / halves;
      const int h = explicit_blobs ? static_cast<int>(q % 2) : static_cast<int>(q % halves);
      // reads_on_main_stream: every blob's upload follows the full reads on
      // the main stream (one in-order chain of copies).  Explicit blobs always
      // upload there: blob q's kernels may read panels uploaded by earlier
      // blobs of the OTHER half (shell s reads panels 0..s), which only one
      // in-order upload chain orders before them
      const bool reads_main = pipeline_reads_on_main_stream || explicit_blobs;
      hipStream_t rs = reads_main ? m : wk.pipe_stream(h, 0), ks = wk.pipe_stream(h, 1);
      // writes_on_compute_stream: a blob's D2H follows its kernel on the same
      // stream (in-stream order) instead of a write stream gated by an event
      hipStream_t ws = pipeline_writes_on_compute_stream ? ks : wk.pipe_stream(pipeline_writes_one_stream ? 0 : h, 2);
      const long long off = explicit_blobs ? ref + c.blob_bounds[q] : ref + h * (range / halves) + k * chunk;
      const long long len = explicit_blobs ? c.blob_bounds[q + 1] - c.blob_bounds[q] : chunk;
      const int ksid = 17 + 3 * h + 1;
      const int wsid = pipeline_writes_on_compute_stream ? ksid : (pipeline_writes_one_stream ? 19 : ksid + 1);
      const int rsid = reads_main ? 0 : ksid - 1;  // as logged for the schedule checker
      auto blob_slice = [&](const ArraySpec& a, uint64_t& b, uint64_t& n) {
        if (explicit_blobs && a.blob_begin.size() == c.blob_bounds.size() - 1) {
          b = a.blob_begin[q];
          n = a.blob_count[q];
        } else {
          a.slice(off, len, c.local_range, b, n);
        }
      };
      int pi = 0;
      for (auto& a : c.arrays) {
        if (a.zc || !a.partial) continue;
        uint64_t b, n;
        blob_slice(a, b, n);
        const bool on2 = two_reads && (pi++ % 2 == 1);
        wk.h2d(on2 ? rs2 : rs, a, b, n);
        *h2d += n * a.elem_size;
      }
      log_op(gidx, "h2d", rsid, off, len);
      if (wk.gpu()) {
        hipEvent_t er = wk.event(slot);
        CEK_HIP(hipEventRecord(er, rs));
        CEK_HIP(hipStreamWaitEvent(ks, er, 0));
      }
      log_op(gidx, "rec", rsid, off, len, slot);
      log_op(gidx, "wait", ksid, off, len, slot);
      ++slot;
      if (two_reads) {
        // every blob's kernels wait for the second stream too, also a blob
        // that uploads nothing there (its kernels may need an earlier blob's
        // panel, and consecutive blobs' kernels run on different streams)
        log_op(gidx, "h2d", rs2id, off, len);
        if (wk.gpu()) {
          hipEvent_t er2 = wk.event(slot);
          CEK_HIP(hipEventRecord(er2, rs2));
          CEK_HIP(hipStreamWaitEvent(ks, er2, 0));
        }
        log_op(gidx, "rec", rs2id, off, len, slot);
        log_op(gidx, "wait", ksid, off, len, slot);
        ++slot;
      }
      launch_kernels(wk, ks, c, off, len);
      log_op(gidx, "kernel", ksid, off, len);
      if (wk.gpu() && ws != ks) {
        hipEvent_t ek = wk.event(slot);
        CEK_HIP(hipEventRecord(ek, ks));
        CEK_HIP(hipStreamWaitEvent(ws, ek, 0));
      }
      log_op(gidx, "rec", ksid, off, len, slot);
      log_op(gidx, "wait", wsid, off, len, slot);
      ++slot;
      for (auto& a : c.arrays) {
        if (a.zc || !a.write || a.write_all) continue;
        uint64_t b, n;
        blob_slice(a, b, n);
        wk.d2h(ws, a, b, n);
        *d2h += n * a.elem_size;
      }
      log_op(gidx, "d2h", wsid, off, len);
    }
  }
  // write-all owners download after every chunk's kernels
  bool any_all = false;
  for (auto& a : c.arrays) any_all |= (a.write && a.write_all && !a.zc);
  for (int h = 0; h < used_halves; ++h) {
    if (wk.gpu()) {
      hipEvent_t e = wk.event(slot);
      CEK_HIP(hipEventRecord(e, wk.pipe_stream(h, 1)));
      CEK_HIP(hipStreamWaitEvent(m, e, 0));
      hipEvent_t e2 = wk.event(slot + 1);
      CEK_HIP(hipEventRecord(e2, wk.pipe_stream(h, 2)));
      CEK_HIP(hipStreamWaitEvent(m, e2, 0));
    }
    log_op(gidx, "rec", 17 + 3 * h + 1, 0, 0, slot);
    log_op(gidx, "wait", 0, 0, 0, slot);
    log_op(gidx, "rec", 17 + 3 * h + 2, 0, 0, slot + 1);
    log_op(gidx, "wait", 0, 0, 0, slot + 1);
    slot += 2;
  }
  if (any_all) {
    for (size_t i = 0; i < c.arrays.size(); ++i) {
      const auto& a = c.arrays[i];
      if (a.write && a.write_all && !a.zc && static_cast<int>(i % global_devices_) == gidx) {
        wk.d2h(m, a, 0, a.bytes / a.elem_size);
        *d2h += a.bytes;
      }
    }
  }
  span_end(wk, m);
  if (zc_release && !enqueue_mode_ && writes_host_memory(c)) wk.system_release(m);
  if (fine_grained) {
    if (defer_marker)
      wk.defer_marker(m, marker_needs_release(c));
    else
      wk.add_marker(m, marker_needs_release(c));
  }
  if (wk.gpu()) wk.wait_stream(m, sleep_waits || sleep_this_call_);
}

void Cores::run_driver_pipeline(Worker& wk, int gidx, const ComputeCall& c, long long ref,
                                long long range, uint64_t* h2d, uint64_t* d2h) {
  const long long B = std::max(1, c.blobs);
  const long long chunk = range / B;
  hipStream_t m = wk.main_stream();
  span_begin(wk, m);
  full_reads(wk, m, c, h2d);
  log_op(gidx, "h2d", 0, -1, -1);  // full reads
  int slot = 0;
  hipEvent_t ev_full = nullptr;
  if (wk.gpu()) {
    ev_full = wk.event(slot);
    CEK_HIP(hipEventRecord(ev_full, m));
  }
  log_op(gidx, "rec", 0, 0, 0, slot);
  const int full_slot = slot++;
  const int nq = wk.queue_concurrency();
  std::vector<char> used(16, 0);
  // the download stream (the event pipeline's first write stream, id 19 in
  // the schedule log)
  const bool own_dl = driver_downloads_own_stream;
  hipStream_t ds = own_dl && wk.gpu() ? wk.pipe_stream(0, 2) : nullptr;
  const int dsid = 19;
  bool ds_used = false;
  for (long long k = 0; k < B; ++k) {
    int qi = static_cast<int>(k % nq);
    hipStream_t s = wk.compute_stream(qi);
    if (!used[qi]) {
      if (wk.gpu()) CEK_HIP(hipStreamWaitEvent(s, ev_full, 0));
      log_op(gidx, "wait", 1 + qi, 0, 0, full_slot);
    }
    used[qi] = 1;
    long long off = ref + k * chunk;
    // reads_main: the blob's upload goes into the main stream's one in-order
    // chain of copies and its queue waits for it, so no upload waits behind
    // an earlier blob's kernel in a compute queue
    const bool reads_main = driver_reads_on_main_stream && wk.gpu();
    hipStream_t rs = reads_main ? m : s;
    bool reads = false;
    for (auto& a : c.arrays) {
      if (a.zc || !a.partial) continue;
      uint64_t b, n;
      a.slice(off, chunk, c.local_range, b, n);
      wk.h2d(rs, a, b, n);
      *h2d += n * a.elem_size;
      reads = true;
    }
    log_op(gidx, "h2d", reads_main ? 0 : 1 + qi, off, chunk);
    if (reads_main && reads) {
      hipEvent_t er = wk.event(slot);
      CEK_HIP(hipEventRecord(er, m));
      CEK_HIP(hipStreamWaitEvent(s, er, 0));
      log_op(gidx, "rec", 0, off, chunk, slot);
      log_op(gidx, "wait", 1 + qi, off, chunk, slot);
      ++slot;
    }
    launch_kernels(wk, s, c, off, chunk);
    log_op(gidx, "kernel", 1 + qi, off, chunk);
    bool writes = false;
    for (auto& a : c.arrays) writes |= !a.zc && a.write && !a.write_all;
    hipStream_t w = s;
    const bool to_ds = own_dl && writes && wk.gpu();
    if (to_ds) {
      hipEvent_t ek = wk.event(slot);
      CEK_HIP(hipEventRecord(ek, s));
      CEK_HIP(hipStreamWaitEvent(ds, ek, 0));
      w = ds;
      log_op(gidx, "rec", 1 + qi, off, chunk, slot);
      log_op(gidx, "wait", dsid, off, chunk, slot);
      ++slot;
      ds_used = true;
    }
    for (auto& a : c.arrays) {
      if (a.zc || !a.write || a.write_all) continue;
      uint64_t b, n;
      a.slice(off, chunk, c.local_range, b, n);
      wk.d2h(w, a, b, n);
      *d2h += n * a.elem_size;
    }
    log_op(gidx, "d2h", to_ds ? dsid : 1 + qi, off, chunk);
  }
  if (ds_used) {  // the call ends after the last download
    if (wk.gpu()) {
      hipEvent_t e = wk.event(slot);
      CEK_HIP(hipEventRecord(e, ds));
      CEK_HIP(hipStreamWaitEvent(m, e, 0));
    }
    log_op(gidx, "rec", dsid, 0, 0, slot);
    log_op(gidx, "wait", 0, 0, 0, slot);
    ++slot;
  }
  for (int q = 0; q < 16; ++q) {
    if (!used[q]) continue;
    if (wk.gpu()) {
      hipEvent_t e = wk.event(slot);
      CEK_HIP(hipEventRecord(e, wk.compute_stream(q)));
      CEK_HIP(hipStreamWaitEvent(m, e, 0));
    }
    log_op(gidx, "rec", 1 + q, 0, 0, slot);
    log_op(gidx, "wait", 0, 0, 0, slot);
    ++slot;
  }
  for (size_t i = 0; i < c.arrays.size(); ++i) {
    const auto& a = c.arrays[i];
    if (a.write && a.write_all && !a.zc && static_cast<int>(i % global_devices_) == gidx) {
      wk.d2h(m, a, 0, a.bytes / a.elem_size);
      *d2h += a.bytes;
    }
  }
  span_end(wk, m);
  if (zc_release && !enqueue_mode_ && writes_host_memory(c)) wk.system_release(m);
  if (fine_grained) {
    if (defer_marker)
      wk.defer_marker(m, marker_needs_release(c));
    else
      wk.add_marker(m, marker_needs_release(c));
  }
  if (wk.gpu()) wk.wait_stream(m, sleep_waits || sleep_this_call_);
}

void Cores::run_device(int w, const ComputeCall& c, long long ref, long long range, bool pipelined,
                       double* out_ms, uint64_t* h2d, uint64_t* d2h) {
  t_phase_arrived = false;
  try {
    run_device_body(w, c, ref, range, pipelined, out_ms, h2d, d2h);
  } catch (...) {
    // a failing device must not leave the others waiting in the phase barrier
    if (phase_ && !t_phase_arrived && range > 0) phase_->arrive_and_drop();
    throw;
  }
}

void Cores::run_device_body(int w, const ComputeCall& c, long long ref, long long range, bool pipelined,
                       double* out_ms, uint64_t* h2d, uint64_t* d2h) {
  Worker& wk = *workers_[w];
  const int gidx = global_base_ + w;
  TraceRange tr(trace_enabled() ? "cek.device" + std::to_string(gidx) + ".id" + std::to_string(c.compute_id)
                                : std::string());
  t_phase_wait = 0;
  if (range > 0 && inject_[w] > 0) {
    --inject_[w];
    throw Error("injected failure on device " + std::to_string(w));
  }
  double t0 = now_ms();
  if (!wk.gpu()) wait_gather(wk, nullptr);  // host memory: the copies into it are done
  const double offset = range > 0 ? time_offset_[w] : 0.0;
  if (offset > 0) {  // injected fixed cost per compute (tests): real host time
    const double until = now_ms() + offset;
    while (now_ms() < until) std::this_thread::yield();
  }
  if (range > 0) {
    wk.set_device();
    if (pipelined) flush_downloads(wk);  // the pipelines' copies follow every earlier download
    if (!pipelined)
      run_3phase(wk, gidx, c, ref, range, h2d, d2h);
    else if (c.pipeline_event)
      run_event_pipeline(wk, gidx, c, ref, range, h2d, d2h);
    else
      run_driver_pipeline(wk, gidx, c, ref, range, h2d, d2h);
  } else if (collective(c)) {
    // still take part in the collectives (a rank the split rounded down to
    // an empty range must join every RCCL call the others make).  On the
    // inline path the calling thread's device is the caller's, not this
    // worker's: its streams, events and communicator need the worker's
    wk.set_device();
    run_3phase(wk, gidx, c, ref, 0, h2d, d2h);
  }
  double el = now_ms() - t0 - t_phase_wait;
  // Device-time spans only when every local device is a GPU: a CPU device
  // has only the host clock, and a GPU's span leaves out its launch, sync
  // and staging overhead, so the two would not be comparable (the reference
  // times every device with one host stopwatch, Worker.cs:779-807).
  if (range > 0 && wk.gpu() && !enqueue_mode_ && all_gpu_) {
    const double dev = span_ms(w);  // the stream was drained: device time of this compute
    if (dev > 0) el = dev + offset;
  }
  *out_ms = el * time_scale_[w];
}

void Cores::compute(const ComputeCall& c) {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  DeviceFailure f;
  compute_once(c, (auto_failover && !ex_) ? &f : nullptr);
  if (f.devices.empty()) return;
  // Failover: the surviving devices' slices are complete; each failed
  // device's slice is recomputed on a surviving device (from the same host
  // inputs), and the failed device is dropped from later splits.
  for (int w : f.devices) enabled_[w] = false;
  int survivor = -1;
  for (int w = 0; w < num_devices() && survivor < 0; ++w)
    if (enabled_[w]) survivor = w;
  if (survivor < 0) throw Error(std::string("every device failed: ") + f.what());
  auto& st = state_[c.compute_id];
  // keep-resident arrays: the recomputed slices must reach every surviving
  // replica too (the regular gather was skipped for this call)
  std::vector<int> gather_idx;
  for (size_t i = 0; i < c.arrays.size(); ++i)
    if (c.arrays[i].gather && !c.arrays[i].zc) gather_idx.push_back(static_cast<int>(i));
  const bool regather = !gather_idx.empty() && !comm_ && num_devices() > 1;
  call_gathers_ = regather;  // the survivor records its kernels-done event
  for (int w : f.devices) {
    const int g = global_base_ + w;
    double ms = 0;
    uint64_t h = 0, d = 0;
    try {
      run_device(survivor, c, st.references[g], st.ranges[g], false, &ms, &h, &d);
    } catch (...) {
      call_gathers_ = false;
      throw;
    }
  }
  call_gathers_ = false;
  if (regather) {
    std::vector<std::vector<std::pair<long long, long long>>> owned(num_devices());
    for (int w = 0; w < num_devices(); ++w)
      if (enabled_[w]) owned[w].push_back({st.references[global_base_ + w], st.ranges[global_base_ + w]});
    for (int w : f.devices) owned[survivor].push_back({st.references[global_base_ + w], st.ranges[global_base_ + w]});
    d2d_ = D2DCount();
    last_record_.gather_bytes = issue_gather(c, st, gather_idx, &owned);
  }
  ++failovers_;
}

void Cores::compute_once(const ComputeCall& c, DeviceFailure* failed) {
  if (error_code_ != 0) throw Error("cannot compute, initialisation failed: " + error_);
  const long long G = c.global_range, L = c.local_range;
  if (G <= 0) throw Error("global range must be positive");
  if (L <= 0 || L > 1024) throw Error("local range must be in [1, 1024]");
  if (G % L != 0) throw Error("global range must be a multiple of local range");
  for (auto& k : c.kernels)
    if (!workers_[0]->program().has(k)) throw Error("unknown kernel: " + k);
  if (!c.repeat_kernel.empty() && !workers_[0]->program().has(c.repeat_kernel))
    throw Error("unknown repeat kernel: " + c.repeat_kernel);
  // Every kernel of a compute receives the same array list (Worker.cs:990-1021
  // binds them positionally); a count mismatch would shift the hidden offset
  // argument onto a pointer and make the kernel address wild memory.
  {
    const int nargs = static_cast<int>(c.arrays.size());
    auto check = [&](const std::string& k) {
      const int ar = workers_[0]->program().arity(k);
      if (ar >= 0 && ar != nargs)
        throw Error("kernel " + k + " takes " + std::to_string(ar) + " array parameter(s) but compute passes " +
                    std::to_string(nargs));
    };
    for (auto& k : c.kernels) check(k);
    if (!c.repeat_kernel.empty()) check(c.repeat_kernel);
  }
  const int D = global_devices_;
  const int nloc = num_devices();
  // equal blobs split every device's range, so ranges move in steps of
  // blobs × unit; explicit blob bounds describe the whole range of the one
  // holding device and put no constraint on the step (their count need not
  // divide the range: 16 square shells plus split ones)
  const long long B = c.blob_bounds.empty() ? std::max(1, c.blobs) : 1;
  const bool pipe_req = c.pipeline && !cfg_.no_pipelining;
  const long long U = c.granularity > 0 ? c.granularity : L;  // balancer unit
  if (U % L != 0) throw Error("granularity must be a multiple of the local range");
  if (G % U != 0) throw Error("global range must be a multiple of the granularity");
  TraceRange tr(trace_enabled() ? "cek.compute.id" + std::to_string(c.compute_id) : std::string());
  double wall0 = now_ms();

  auto it = state_.find(c.compute_id);
  bool fresh = it == state_.end() || it->second.global_range != G ||
               (it->second.local_range != 0 && it->second.local_range != L) ||
               static_cast<int>(it->second.ranges.size()) != D;
  BalancerState& st = state_[c.compute_id];
  if (fresh) {
    st = BalancerState();
    st.history.assign(kHistoryDepth, std::vector<double>(D, 0.0));
    st.bench.assign(D, 0.0);
    st.global_range = G;
    st.local_range = L;
  }
  st.global_offset = c.global_offset;
  st.local_range = L;  // (restored states carry no local range)
  if (st.history.size() != static_cast<size_t>(kHistoryDepth))
    st.history.assign(kHistoryDepth, std::vector<double>(D, 0.0));
  if (st.bench.size() != static_cast<size_t>(D)) st.bench.assign(D, 0.0);
  const bool first = fresh || std::all_of(st.ranges.begin(), st.ranges.end(), [](long long r) { return r == 0; });
  if (!(enqueue_mode_ && !first)) {
    int active = 0;
    for (int i = 0; i < D; ++i)
      if (i < global_base_ || i >= global_base_ + nloc || enabled_[i - global_base_]) ++active;
    if (first) {
      // Cores.cs:569-596
      std::vector<long long> eq(active, G / std::max(active, 1));
      if (active) eq[0] += G - (G / active) * active;
      bool b1 = std::all_of(eq.begin(), eq.end(), [&](long long r) { return r >= B * U; });
      long long step = (b1 && pipe_req && G >= B * U) ? B * U : U;
      balance(st, true, G, step);
    } else {
      bool b1 = true;
      for (int i = 0; i < D; ++i)
        if (st.ranges[i] != 0 && st.ranges[i] < B * U) b1 = false;
      long long step = (b1 && pipe_req && G >= B * U) ? B * U : U;
      balance(st, false, G, step);
    }
  }
  st.references.assign(D, 0);
  long long acc = c.global_offset;
  for (int i = 0; i < D; ++i) {
    st.references[i] = acc;
    acc += st.ranges[i];
  }
  // Host-memory hazard: an array read whole by every device and written back
  // by slices.  With several local devices the phases must be separated.
  bool hazard = false;
  if (nloc > 1)
    for (auto& a : c.arrays)
      if (!a.zc && a.read && !a.partial && a.write) hazard = true;
  // Pipelining eligibility (Cores.cs:624-652), decided per call for all devices.
  // keep-resident gather arrays (in process; across ranks RCCL does it)
  std::vector<int> gather_idx;
  for (size_t i = 0; i < c.arrays.size(); ++i)
    if (c.arrays[i].gather && !c.arrays[i].zc) gather_idx.push_back(static_cast<int>(i));
  if (!gather_idx.empty() && capturing_) throw Error("keep-resident gather arrays cannot be captured into a graph");
  if (!gather_idx.empty() && ex_ && !comm_ && global_devices_ > nloc)
    throw Error("gather across ranks needs an RCCL communicator (DistributedCruncher(comm=True))");
  call_gathers_ = !gather_idx.empty() && !comm_ && nloc > 1;
  bool pipelined = pipe_req && c.repeats <= 1 && !enqueue_mode_ && !hazard && gather_idx.empty();
  if (!c.blob_bounds.empty()) {
    // explicit blobs describe the whole range on one device
    const auto& bb = c.blob_bounds;
    bool ok = bb.size() >= 2 && bb.front() == 0 && bb.back() == G && c.pipeline_event;
    for (size_t k = 1; ok && k < bb.size(); ++k) ok = bb[k] > bb[k - 1] && bb[k] % L == 0;
    if (!ok) throw Error("blob_bounds must rise from 0 to the global range in whole work-groups (event pipeline)");
    for (const auto& a : c.arrays)
      if (!a.blob_begin.empty() && (a.blob_begin.size() != bb.size() - 1 || a.blob_count.size() != bb.size() - 1))
        throw Error("an array's blob slices must have one entry per blob");
    int holders = 0;
    for (int i = 0; i < D; ++i) holders += st.ranges[i] > 0;
    if (holders != 1) pipelined = false;  // split over devices: the plain path
  } else {
    for (int i = 0; i < D && pipelined; ++i)
      if (st.ranges[i] != 0 && (st.ranges[i] % (B * U) != 0 || st.ranges[i] < B * U)) pipelined = false;
  }
  if (collective(c)) pipelined = false;

  // A GPU that shares the call with a CPU device sleeps on its stream when
  // its last time for this compute id was long: a spinning wait would take
  // a core (an SMT sibling) from the CPU device's threads for milliseconds.
  // Short GPU waits (a 0.03 ms wave frame) keep spinning, where a wake-up
  // would cost more than the core.
  sleep_this_call_ = false;
  if (!all_gpu_ && adaptive_sleep_waits)
    for (int w = 0; w < nloc; ++w)
      if (workers_[w]->gpu() && st.bench[global_base_ + w] > sleep_wait_min_ms) sleep_this_call_ = true;
  std::vector<double> ms(nloc, 0.0);
  std::vector<uint64_t> h2d(nloc, 0), d2h(nloc, 0);
  // xGMI fan-out of full reads, enqueued before the per-device work (its
  // time lands on the devices' streams, inside their measured span only
  // through the event waits in full_reads)
  d2d_ = D2DCount();
  if (gather_pending_)  // the last gather's copies finish before this call touches any replica
    for (int w = 0; w < nloc; ++w)
      if (workers_[w]->gpu()) {
        workers_[w]->set_device();
        wait_gather(*workers_[w], workers_[w]->main_stream());
      }
  stage_peer_reads(c, st.ranges, h2d);
  DeviceFailure failure;
  int participants = 0;
  std::vector<char> part(nloc, 0);
  for (int w = 0; w < nloc; ++w)
    if (st.ranges[global_base_ + w] > 0 || collective(c)) {
      part[w] = 1;
      ++participants;
    }
  PhaseBarrier phase(participants);
  if (hazard && !enqueue_mode_ && participants > 1) phase_ = &phase;
  struct ResetPhase {
    PhaseBarrier*& p;
    ~ResetPhase() { p = nullptr; }
  } reset_phase{phase_};
  // A device with an empty range does no device work; with at most one
  // participant there is nothing to overlap, so no worker-thread hand-off
  // (a device the overhead-aware balancer left out costs nothing per call).
  if (nloc == 1 || (serial && !phase_) || participants <= 1) {
    for (int w = 0; w < nloc; ++w) {
      int g = global_base_ + w;
      try {
        run_device(w, c, st.references[g], st.ranges[g], pipelined, &ms[w], &h2d[w], &d2h[w]);
      } catch (const std::exception& e) {
        failure.add(w, e.what());
      }
    }
  } else {
    // One participant runs on the calling thread: a hand-off fewer per call
    // (the wave frame's GPU+CPU split pays one wake-up instead of two).  A
    // CPU device is preferred there — its work is the calling thread plus
    // the CPU pool either way, and the GPU workers are posted first so
    // their launches go out while the CPU computes.
    // Option (inline_largest_share): the participant holding the largest
    // share runs here instead (measured slower on the wave frame, off).
    int inline_w = -1;
    if (inline_largest_share && !all_gpu_) {
      for (int w = 0; w < nloc; ++w)
        if (part[w] && (inline_w < 0 || st.ranges[global_base_ + w] > st.ranges[global_base_ + inline_w] ||
                        (st.ranges[global_base_ + w] == st.ranges[global_base_ + inline_w] && !workers_[w]->gpu())))
          inline_w = w;
    } else {
      for (int w = 0; w < nloc; ++w)
        if (part[w] && (inline_w < 0 || !workers_[w]->gpu())) inline_w = w;
    }
    for (int w = 0; w < nloc; ++w) {
      if (!part[w] || w == inline_w) continue;
      int g = global_base_ + w;
      long long ref = st.references[g], rng = st.ranges[g];
      workers_[w]->post([=, &c, &ms, &h2d, &d2h] {
        run_device(w, c, ref, rng, pipelined, &ms[w], &h2d[w], &d2h[w]);
      });
    }
    // the calling thread's current device is the caller's (torch allocates
    // on it): restored after a GPU participant ran here
    struct RestoreDevice {
      int dev = -1;
      explicit RestoreDevice(bool gpu) {
        if (gpu && hipGetDevice(&dev) != hipSuccess) dev = -1;
      }
      ~RestoreDevice() {
        if (dev >= 0) (void)hipSetDevice(dev);
      }
    } restore(inline_w >= 0 && workers_[inline_w]->gpu());
    for (int w = 0; w < nloc; ++w) {
      if (part[w] && w != inline_w) continue;
      try {
        run_device(w, c, st.references[global_base_ + w], part[w] ? st.ranges[global_base_ + w] : 0,
                   pipelined, &ms[w], &h2d[w], &d2h[w]);
      } catch (const std::exception& e) {
        failure.add(w, e.what());
      }
    }
    for (int w = 0; w < nloc; ++w) {
      if (!part[w] || w == inline_w) continue;
      try {
        workers_[w]->wait();
      } catch (const std::exception& e) {
        failure.add(w, e.what());
      }
    }
  }
  if (!failure.devices.empty()) {
    call_gathers_ = false;
    if (!failed) throw Error(failure.what());
    *failed = failure;
  }
  uint64_t gathered = 0;
  if (call_gathers_) {
    call_gathers_ = false;
    gathered = issue_gather(c, st, gather_idx);
  }
  last_id_ = c.compute_id;
  if (!enqueue_mode_) {
    std::vector<double> all = ms;
    if (ex_) all = ex_->allgather(ms);
    if (static_cast<int>(all.size()) == D) st.bench = all;
  }
  ++st.calls;
  last_record_.compute_id = c.compute_id;
  last_record_.wall_ms = now_ms() - wall0;
  st.last_wall_ms = last_record_.wall_ms;
  last_record_.ranges = st.ranges;
  last_record_.references = st.references;
  last_record_.device_ms = st.bench;
  last_record_.h2d_bytes = std::accumulate(h2d.begin(), h2d.end(), 0ull);
  last_record_.d2h_bytes = std::accumulate(d2h.begin(), d2h.end(), 0ull);
  last_record_.p2p_bytes = d2d_.bytes;
  last_record_.gather_bytes = gathered;
  last_record_.staged_bytes = d2d_.staged;
  last_record_.p2p_path = d2d_.pcie_fallback ? "pcie"
                          : d2d_.staged       ? "staged"
                          : d2d_.xgmi         ? "xgmi"
                          : d2d_.local        ? "local"
                                              : "none";
  last_record_.pipelined = pipelined;
}

}  // namespace cek
