// Native device pool (see pool.h).  Reference: ClDevicePool producer /
// DevicePoolThread consumer loops, ClPipeline.cs:4132-4312 and :4841-5047.
#include "pool.h"

#include <chrono>

namespace cek {

// a consumer's own counter: one writer, readers only sum
static void add_ms(std::atomic<double>& a, double v) {
  a.store(a.load(std::memory_order_relaxed) + v, std::memory_order_relaxed);
}
static void add_one(std::atomic<long long>& a) { a.store(a.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed); }

std::vector<double> DevicePool::host_profile() {
  std::vector<double> r(4, 0.0);
  for (int i = 0; i < num_devices(); ++i) {
    r[0] += prof_[i].issue_ms.load();
    r[1] += prof_[i].retire_ms.load();
    r[2] += static_cast<double>(prof_[i].tasks.load());
    r[3] += static_cast<double>(prof_[i].polls.load());
  }
  return r;
}

DevicePool::DevicePool(std::vector<std::shared_ptr<Cores>> devices, int max_in_flight, int policy)
    : devs_(std::move(devices)), max_in_flight_(std::max(1, std::min(16, max_in_flight))), policy_(policy) {
  if (devs_.empty()) throw Error("device pool needs at least one device");
  if (policy != 0 && policy != 1) throw Error("device pool policy must be 0 (compute at will) or 1 (round robin)");
  for (auto& d : devs_) {
    if (!d) throw Error("device pool: null cruncher");
    if (d->num_devices() != 1) throw Error("device pool: every entry must be a single-device cruncher");
  }
  counts_.assign(devs_.size(), 0);
  busy_ms_.assign(devs_.size(), 0.0);
  inflight_.assign(devs_.size(), 0);
  speed_.assign(devs_.size(), Speed());
  prof_.reset(new Prof[devs_.size()]);
  for (int i = 0; i < num_devices(); ++i) threads_.emplace_back([this, i] { consumer(i); });
}

DevicePool::~DevicePool() {
  try {
    close();
  } catch (...) {
  }
}

void DevicePool::close() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_ && threads_.empty()) return;
    closed_ = true;
  }
  work_cv_.notify_all();
  for (auto& t : threads_) {
    if (!t.joinable()) continue;
    if (t.get_id() == std::this_thread::get_id())
      t.detach();  // the last reference dropped on a consumer thread: it exits on return
    else
      t.join();
  }
  threads_.clear();
}

void DevicePool::enqueue(std::vector<PoolTask> tasks, long long pool_total, bool append) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) throw Error("device pool is closed");
    // append: the tasks continue the last enqueued pool (a pool handed over
    // in chunks, so the consumers start on the first chunk while the caller
    // prepares the next); pool_total pre-sizes a new pool's task count for
    // the queue-depth policy
    if (!append || pools_.empty()) {
      pools_.push_back(PoolProgress());
      if (pool_total > 0) pools_.back().preset = pool_total;
      sync_carry_ = false;
    }
    bool sync_next = sync_carry_;
    const int pid = static_cast<int>(pools_.size()) - 1;
    for (auto& task : tasks) {
      Item it;
      it.task = std::move(task);
      it.pool = pid;
      const PoolTask& t = it.task;
      // GLOBAL_SYNC_LAST of the previous task = a barrier before this one
      if (sync_next) it.task.type |= kTaskSyncFirst;
      sync_next = (t.type & kTaskSyncLast) != 0;
      if (t.type & kTaskBroadcast) {
        for (int d = 0; d < num_devices(); ++d) {
          Item c = it;
          c.target = d;
          // the first copy is the barrier; the others follow it at once
          if (d > 0) c.task.type &= ~static_cast<uint32_t>(kTaskSyncFirst);
          queue_.push_back(std::move(c));
          ++outstanding_;
          ++pools_[pid].total;
        }
      } else {
        if (policy_ == 1) {
          // strict rotation; a select/serial group keeps its first task's
          // device.  Barrier tasks (SyncFirst, also inherited from the
          // previous task's SyncLast) are targeted too: the barrier itself is
          // enforced at take time, and a group whose BEGIN or END carries one
          // must still open / close its rotation slot
          if (rr_group_ >= 0) {
            it.target = rr_group_;
          } else {
            it.target = static_cast<int>(rr_next_++ % num_devices());
            if (t.type & (kTaskSelectBegin | kTaskSerialBegin)) rr_group_ = it.target;
          }
          if (t.type & (kTaskSelectEnd | kTaskSerialEnd)) rr_group_ = -1;
        }
        queue_.push_back(std::move(it));
        ++outstanding_;
        ++pools_[pid].total;
      }
    }
    sync_carry_ = sync_next;
  }
  work_cv_.notify_all();
}

int DevicePool::least_loaded_locked() const {
  int best = 0;
  for (int d = 1; d < num_devices(); ++d)
    if (inflight_[d] < inflight_[best]) best = d;
  return best;
}

int DevicePool::limit_locked() {
  if (queue_.empty()) return max_in_flight_;
  const PoolProgress& p = pools_[queue_.front().pool];
  const long long n = std::max(p.total, p.preset), sub = p.taken, rem = n - sub;
  long long q;
  if (rem < 3)
    q = 1;
  else if (sub < n / 10)
    q = n / 10;
  else if (sub < n / 5)
    q = n / 20;
  else if (sub < n / 3)
    q = n / 33;
  else if (sub < n / 2)
    q = n / 50;
  else
    q = 2;
  q /= num_devices();
  // Floor of 2 (when the pool allows 2): with one task in flight a device
  // idles for the host's enqueue + marker-retirement turnaround (10-20 µs)
  // between tasks; two in flight hide it and the tail stays balanced.
  static const int min_inflight = [] {
    const char* e = std::getenv("CEK_POOL_MIN_INFLIGHT");
    return e ? std::max(1, std::atoi(e)) : 2;
  }();
  const long long floor_q = std::min(min_inflight, max_in_flight_);
  const int lim = static_cast<int>(std::max<long long>(floor_q, std::min<long long>(q, max_in_flight_)));
  if (limit_history_.empty() || limit_history_.back() != lim) limit_history_.push_back(lim);
  return lim;
}

bool DevicePool::take_locked(int dev, Item& out) {
  for (size_t j = 0; j < queue_.size(); ++j) {
    Item& u = queue_[j];
    if (u.task.type & kTaskSyncFirst) {
      // a barrier: every earlier task has retired and nothing precedes it;
      // no later task passes it, whichever device it is targeted at
      if (u.target >= 0 && u.target != dev) return false;
      if (j != 0 || running_ > 0) return false;
    }
    if (u.target >= 0 && u.target != dev) continue;  // another device's broadcast copy / rotation slot
    if (u.target < 0 && owner_ >= 0 && owner_ != dev) return false;  // group pinned elsewhere
    if (u.target < 0 && owner_ < 0 && (u.task.type & (kTaskSelectBegin | kTaskSerialBegin))) {
      // a new select/serial group: pin it to the least-loaded device
      owner_ = least_loaded_locked();
      if (owner_ != dev) {
        work_cv_.notify_all();
        return false;
      }
    }
    out = std::move(u);
    queue_.erase(queue_.begin() + static_cast<long>(j));
    const uint32_t ty = out.task.type;
    if (ty & (kTaskSelectBegin | kTaskSerialBegin)) owner_ = dev;
    out.serial = (ty & (kTaskSerialBegin | kTaskSerialEnd)) != 0 || (owner_ == dev && serial_owner_);
    if (ty & kTaskSerialBegin) serial_owner_ = true;
    if (ty & (kTaskSelectEnd | kTaskSerialEnd)) {
      if (owner_ == dev) owner_ = -1;
      serial_owner_ = false;
    }
    ++running_;
    ++inflight_[dev];
    ++pools_[out.pool].taken;
    return true;
  }
  return false;
}

// Retires one task.  Only a notify task (a callback) or a failure makes a
// record the caller reads; the wake-ups go only to whoever can proceed now:
// finish() when the pool drains, idle consumers when a barrier or a pinned
// group may have been waiting for this retirement.
void DevicePool::complete_locked(int dev, long long id, bool notify, double ms, const std::string& err,
                                 Wake& w) {
  if (id >= 0) {
    if (static_cast<size_t>(id) >= results_.size())  // geometric growth: ids rise by one per task
      results_.resize(std::max<size_t>(static_cast<size_t>(id) + 1, 2 * results_.size() + 1024));
    results_[static_cast<size_t>(id)] = {dev, static_cast<float>(ms)};
  }
  if (!err.empty()) errors_.push_back({id, dev, ms, err});
  if (notify) {
    done_.push_back({id, dev, ms, err});
    w.comp = true;
  }
  ++counts_[dev];
  busy_ms_[dev] += ms;
  --outstanding_;
  --running_;
  --inflight_[dev];
  w.done = w.done || outstanding_ == 0;
  w.work = w.work || running_ == 0 || owner_ >= 0 ||
           (!queue_.empty() && (queue_.front().task.type & kTaskSyncFirst));
}

void DevicePool::wake(const Wake& w) {
  if (w.comp) comp_cv_.notify_all();
  if (w.done) done_cv_.notify_all();
  if (w.work) work_cv_.notify_all();
}

void DevicePool::complete(int dev, long long id, bool notify, double ms, const std::string& err) {
  Wake w;
  {
    std::lock_guard<std::mutex> g(mu_);
    complete_locked(dev, id, notify, ms, err, w);
  }
  wake(w);
}

std::vector<PoolCompletion> DevicePool::take_errors() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<PoolCompletion> out;
  out.swap(errors_);
  return out;
}

void DevicePool::results(long long first, long long n, std::vector<int>& dev, std::vector<double>& ms) {
  std::lock_guard<std::mutex> g(mu_);
  dev.assign(static_cast<size_t>(std::max(0LL, n)), -1);
  ms.assign(dev.size(), 0.0);
  for (long long i = 0; i < n; ++i) {
    const long long id = first + i;
    if (id < 0 || static_cast<size_t>(id) >= results_.size()) continue;
    dev[static_cast<size_t>(i)] = results_[static_cast<size_t>(id)].device;
    ms[static_cast<size_t>(i)] = results_[static_cast<size_t>(id)].ms;
  }
}

int DevicePool::retire(int dev, std::vector<Inflight>& inflight) {
  Cores& cr = *devs_[dev];
  // one marker query per stream slot per poll (a slot's markers retire in
  // order), not one per task in flight: every query takes the HIP runtime's
  // lock that the other consumers' launches need
  int slots[16];
  uint64_t words[16];
  int nslots = 0;
  auto word = [&](int slot) {
    for (int j = 0; j < nslots; ++j)
      if (slots[j] == slot) return words[j];
    const uint64_t w = cr.marker_word(0, slot);
    if (nslots < 16) {
      slots[nslots] = slot;
      words[nslots++] = w;
    }
    return w;
  };
  // the reached tasks move to the end, then retire under ONE lock (a batch
  // of tasks sharing a marker retires together)
  size_t keep = 0;
  for (size_t i = 0; i < inflight.size(); ++i)
    if (word(inflight[i].slot) < inflight[i].value) std::swap(inflight[keep++], inflight[i]);
  const int n = static_cast<int>(inflight.size() - keep);
  if (n > 0) {
    Wake w;
    {
      std::lock_guard<std::mutex> g(mu_);
      const double t = now_ms();
      for (size_t i = keep; i < inflight.size(); ++i)
        complete_locked(dev, inflight[i].id, inflight[i].notify, t - inflight[i].t0, "", w);
      Speed& sp = speed_[dev];  // marker-reach speed (ClPipeline.cs:4788-4817)
      if (sp.last_ms >= 0) sp.hist[sp.n++ % 15] = n / (t - sp.last_ms + 0.001);
      sp.last_ms = t;
    }
    inflight.resize(keep);
    wake(w);
  }
  return n;
}

int pool_marker_batch() {
  static const int k = [] {
    const char* e = std::getenv("CEK_POOL_MARKER_BATCH");
    const int v = e ? std::atoi(e) : 8;
    return std::max(1, std::min(64, v));
  }();
  return k;
}

void DevicePool::consumer(int dev) {
  Cores& cr = *devs_[dev];
  const bool async = max_in_flight_ > 1;
  if (async) cr.fine_grained = true;  // a marker word after every compute
  std::vector<Inflight> inflight;
  ComputeCall call;                            // scratch: the task being issued
  const ComputeCall* call_tmpl = nullptr;      // the template `call` was copied from
  std::shared_ptr<const ComputeCall> call_keep;  // keeps that template alive
  double last_progress = now_ms();
  bool issued = false;  // the previous iteration issued a task
  const int batch = pool_marker_batch();
  int deferred = 0;     // tasks in flight whose marker is not recorded yet
  auto flush = [&] {
    if (deferred > 0) {
      cr.flush_markers(0);
      deferred = 0;
    }
  };
  int last_lim = max_in_flight_;
  int issues_since_poll = 0;
  static const int poll_every = [] {  // CEK_POOL_POLL_EVERY: issues between polls while flowing
    const char* e = std::getenv("CEK_POOL_POLL_EVERY");
    return std::max(1, std::min(64, e ? std::atoi(e) : kPollBatch));
  }();
  for (;;) {
    // while tasks keep flowing, poll the markers only once a few are in
    // flight, and then every kPollBatch issues or when the queue-depth limit
    // is about to stop the issuing: each poll is a HIP call that costs about
    // as much as a launch, and a batch of tasks sharing a marker cannot
    // retire before its marker is recorded anyway
    const int nin = static_cast<int>(inflight.size());
    if (nin > 0 && (!issued || (nin >= kPollBatch && (issues_since_poll >= poll_every || nin + 1 >= last_lim)))) {
      issues_since_poll = 0;
      const double r0 = now_ms();
      const int done = retire(dev, inflight);
      const double r1 = now_ms();
      add_ms(prof_[dev].retire_ms, r1 - r0);
      add_one(prof_[dev].polls);
      if (done > 0) last_progress = r1;
    }
    issued = false;
    Item it;
    bool got = false, idle = false, stop = false, more = false;
    int lim = 1;
    {
      std::unique_lock<std::mutex> lk(mu_);
      lim = limit_locked();
      last_lim = lim;
      if (static_cast<int>(inflight.size()) < lim) got = take_locked(dev, it);
      more = !queue_.empty();
      if (!got && inflight.empty()) {
        if (closed_ && queue_.empty())
          stop = true;
        else
          idle = true;
      }
    }
    if (stop) break;
    if (idle) {
      // nothing in flight here: leave enqueue mode (syncs this device's
      // streams) and sleep until new work, a retirement elsewhere (a barrier
      // or a pinned group may be waiting on it) or close()
      try {
        if (cr.enqueue_mode()) cr.set_enqueue_mode(false);
      } catch (...) {
      }
      std::unique_lock<std::mutex> lk(mu_);
      work_cv_.wait_for(lk, std::chrono::milliseconds(5));
      continue;
    }
    if (!got) {  // only in-flight tasks: poll their markers
      flush();  // (a deferred marker would never be reached otherwise)
      // yield-spin while tasks keep retiring: a sleep, however short it is
      // asked to be, costs ~60 µs on Linux — longer than most tasks on a
      // partition, and a late retirement leaves the device idle (median
      // 40-60 µs gaps between a queue's kernels in a rocprofv3 trace of the
      // 256-task pool, profiles/r5/README.md).  Only after 2 ms without a
      // retirement does the consumer fall back to short sleeps.
      if (now_ms() - last_progress < 2.0)
        std::this_thread::yield();
      else
        std::this_thread::sleep_for(std::chrono::microseconds(10));
      continue;
    }
    last_progress = now_ms();
    const double t0 = last_progress;
    PoolTask& t = it.task;
    const bool notify = (t.type & kTaskNotify) != 0;
    if (!t.tmpl || t.tmpl->kernels.empty()) {  // a pure barrier / message task
      complete(dev, t.id, notify, 0.0, "");
      continue;
    }
    try {
      // the consumer's call: the template's fields copied only when the
      // template changes, the task's arrays moved in
      if (t.tmpl.get() != call_tmpl) {
        call = *t.tmpl;
        call_tmpl = t.tmpl.get();
        call_keep = t.tmpl;
      }
      call.arrays = std::move(t.arrays);
      cr.no_compute = (t.type & kTaskNoCompute) != 0;
      if (async) {
        if (!cr.enqueue_mode()) cr.set_enqueue_mode(true);
        cr.async_enqueue = !it.serial;  // serial groups stay on one in-order stream
        // coalesce this task's marker with the next tasks' while more work
        // follows at once (the batch's last task records it).  A batch
        // retires only when its last task is done, so it is at most half the
        // queue-depth limit: the next batch is issued while one runs (with a
        // shallow limit in the pool's tail, every task keeps its own marker
        // and retires as soon as it is done)
        const int eff_batch = std::min(batch, lim / 2);
        const bool defer = eff_batch > 1 && !notify && !it.serial && more && deferred + 1 < eff_batch;
        cr.defer_marker = defer;
        const double i0 = now_ms();
        try {
          cr.compute(call);
        } catch (...) {
          cr.defer_marker = false;
          throw;
        }
        cr.defer_marker = false;
        if (defer)
          ++deferred;
        else
          flush();  // this task's marker covers its stream; record the others'
        add_ms(prof_[dev].issue_ms, now_ms() - i0);
        add_one(prof_[dev].tasks);
        auto m = cr.last_marker(0);
        inflight.push_back({t.id, notify, m.first, m.second, t0});
        issued = true;
        ++issues_since_poll;
      } else {
        cr.compute(call);
        complete(dev, t.id, notify, now_ms() - t0, "");
      }
    } catch (const std::exception& e) {
      complete(dev, t.id, notify, now_ms() - t0, e.what());
    }
  }
  try {
    if (cr.enqueue_mode()) cr.set_enqueue_mode(false);
  } catch (...) {
  }
}

void DevicePool::finish() {
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return outstanding_ == 0; });
}

std::vector<PoolCompletion> DevicePool::completions(double timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  if (done_.empty() && timeout_ms > 0)
    comp_cv_.wait_for(lk, std::chrono::microseconds(static_cast<long long>(timeout_ms * 1e3)),
                      [&] { return !done_.empty(); });
  std::vector<PoolCompletion> out(std::make_move_iterator(done_.begin()), std::make_move_iterator(done_.end()));
  done_.clear();
  return out;
}

long long DevicePool::outstanding() {
  std::lock_guard<std::mutex> g(mu_);
  return outstanding_;
}

std::vector<long long> DevicePool::device_task_counts() {
  std::lock_guard<std::mutex> g(mu_);
  return counts_;
}

std::vector<double> DevicePool::device_busy_ms() {
  std::lock_guard<std::mutex> g(mu_);
  return busy_ms_;
}

int DevicePool::queue_limit() {
  std::lock_guard<std::mutex> g(mu_);
  return limit_locked();
}

std::vector<int> DevicePool::queue_limit_history() {
  std::lock_guard<std::mutex> g(mu_);
  return limit_history_;
}

std::vector<double> DevicePool::marker_speeds() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<double> out;
  for (auto& sp : speed_) {
    double s = 0;
    for (double h : sp.hist) s += h;
    out.push_back(s / 15.0 + 0.001);
  }
  return out;
}

std::vector<int> DevicePool::device_in_flight() {
  std::lock_guard<std::mutex> g(mu_);
  return inflight_;
}

}  // namespace cek
