// Native task pool × device pool: the MI355X-native counterpart of the
// reference's ClDevicePool / DevicePoolThread (ClPipeline.cs:3891-5077).
//
// The reference runs one producer thread plus one C# consumer thread per
// device; consumers pop frozen compute() calls (ClTask, :3331-3520) from a
// shared FIFO and run them on the device's own cruncher ("compute at will",
// :4841-5047).  Here every consumer is a C++ thread that owns one
// single-device `Cores`; it takes the next task under one mutex, issues it in
// enqueue mode on the device's round-robin HIP streams, and retires it when
// the device reaches the task's completion marker (a fence-less hipEvent,
// shared by a batch of consecutive tasks) — no host callback, no GIL, no
// Python per task.  Up to `max_in_flight` tasks per device are outstanding.
//
// Task type flags (ClTaskType, ClPipeline.cs:3247-3321):
//   SELECT_BEGIN/END, SERIAL_BEGIN/END  pin the group to the device that took
//                                       its first task (serial groups also run
//                                       in issue order on one stream)
//   SYNC_FIRST                          barrier: taken only when no task is
//                                       running anywhere
//   SYNC_LAST                           barrier after the task (becomes
//                                       SYNC_FIRST of the next one)
//   BROADCAST                           duplicated onto every device
//   NO_COMPUTE                          transfers only
// Completions (task id, device, ms, error) are queued for the caller, which
// runs user callbacks off the device threads.
//
// Scheduling policy (reference producer, ClPipeline.cs:4100-4236, :4788-4817):
//   * a select/serial group goes to the least-loaded device — fewest tasks
//     taken and not yet retired (the reference's remaining tasks + markers
//     remaining), first index on ties;
//   * per-device queue depth follows the pool's progress: with N tasks in
//     the pool of which `taken` have been handed out, the limit is N/10
//     until 10 % are out, N/20 until 20 %, N/33 until 33 %, N/50 until half,
//     then 2 (1 once fewer than 3 remain), divided by the device count and
//     clamped to [min(2, max_in_flight), max_in_flight] — deep queues while
//     the pool is full, shallow ones in the tail so the last tasks spread
//     over every device (the floor of 2 is ours: one task in flight leaves
//     the device idle for the host turnaround between tasks);
//   * each device keeps a smoothed marker-reach speed (markers retired per
//     ms, 15-sample moving average).
// Device policy (ClDevicePoolType, ClPipeline.cs:3792-3806): COMPUTE_AT_WILL
// (0) — an idle device takes the next task; ROUND_ROBIN (1, a stub in the
// reference, "better for identical devices") — task k of the stream goes to
// device k mod D in strict rotation (a select/serial group as a whole takes
// one rotation slot; barriers stay untargeted so every device stops at them).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>

#include "cores.h"

namespace cek {

enum PoolTaskFlags : uint32_t {
  kTaskSelectBegin = 1,
  kTaskSelectEnd = 2,
  kTaskSyncFirst = 4,
  kTaskSyncLast = 8,
  kTaskBroadcast = 16,
  kTaskNoCompute = 32,
  kTaskSerialBegin = 64,
  kTaskSerialEnd = 128,
};

// Not a ClTaskType bit: the caller wants a completion record for the task
// (it has a callback).  Other tasks retire natively without a record; their
// device and time are kept in the pool's result table (results()).
constexpr uint32_t kTaskNotify = 1u << 30;
// a consumer issuing back to back polls its markers once this many tasks are
// in flight (and whenever it cannot issue)
constexpr int kPollBatch = 3;
// Consecutive tasks of a consumer share one completion marker (one
// hipEventRecord per stream per batch, recorded after the batch's last
// task): at most this many per batch; a batch also ends when the consumer
// runs out of tasks to take, at a callback or serial-group task, and before
// it would wait for a retirement (CEK_POOL_MARKER_BATCH, 1 = a marker per task)
int pool_marker_batch();

struct PoolTask {
  // the compute without its arrays, shared by every task of one shape (a
  // batch of 4096 tasks holds one template, not 4096 copies of it)
  std::shared_ptr<const ComputeCall> tmpl;
  std::vector<ArraySpec> arrays;  // this task's frozen arrays
  uint32_t type = 0;
  long long id = 0;  // caller's handle, reported back on completion
  ComputeCall call() const {
    ComputeCall c = tmpl ? *tmpl : ComputeCall();
    c.arrays = arrays;
    return c;
  }
  void set_call(const ComputeCall& c) {
    auto t = std::make_shared<ComputeCall>(c);
    arrays = std::move(t->arrays);
    t->arrays.clear();
    tmpl = std::move(t);
  }
};

struct PoolCompletion {
  long long id = 0;
  int device = -1;
  double ms = 0;  // issue → retirement (host clock)
  std::string error;
};

class DevicePool {
 public:
  // One consumer thread per entry of `devices` (the same physical device may
  // appear several times, ClPipeline.cs:4337, as separate Cores).
  DevicePool(std::vector<std::shared_ptr<Cores>> devices, int max_in_flight, int policy = 0);
  int policy() const { return policy_; }
  ~DevicePool();

  // Appends one task pool (FIFO order kept); broadcast tasks are duplicated
  // per device, SYNC_LAST turns into SYNC_FIRST of the next task.
  void enqueue(std::vector<PoolTask> tasks, long long pool_total = -1, bool append = false);
  // Blocks until every enqueued task has retired.
  void finish();
  // Completions of kTaskNotify tasks since the last call; waits up to
  // timeout_ms for one (0: poll).
  std::vector<PoolCompletion> completions(double timeout_ms);
  // Failed tasks since the last call (every task, notified or not).
  std::vector<PoolCompletion> take_errors();
  // Device and issue→retirement ms of tasks [first, first + n) (device -1:
  // not retired yet, or never enqueued).
  void results(long long first, long long n, std::vector<int>& dev, std::vector<double>& ms);
  long long outstanding();
  std::vector<long long> device_task_counts();
  std::vector<double> device_busy_ms();
  // current per-device queue-depth limit (policy above) and its history
  int queue_limit();
  std::vector<int> queue_limit_history();
  std::vector<double> marker_speeds();  // smoothed markers per ms, per device
  std::vector<int> device_in_flight();
  // consumer host time by part, summed over devices (ms): issuing computes,
  // polling markers, everything else (queue lock, bookkeeping, idle waits)
  std::vector<double> host_profile();
  int num_devices() const { return static_cast<int>(devs_.size()); }
  int max_in_flight() const { return max_in_flight_; }
  void close();  // drain, stop and join the consumer threads

 private:
  struct Item {
    PoolTask task;
    int target = -1;  // broadcast copy: only this device may take it
    bool serial = false;
    int pool = 0;     // enqueue() call it came from
  };
  struct PoolProgress {
    long long total = 0, taken = 0;
    long long preset = 0;  // the whole pool's size when it arrives in chunks
  };
  bool sync_carry_ = false;  // a SYNC_LAST at the end of the last chunk
  int limit_locked();
  int least_loaded_locked() const;
  struct Inflight {
    long long id;
    bool notify;
    int slot;
    uint64_t value;
    double t0;
  };
  bool take_locked(int dev, Item& out);
  void consumer(int dev);
  void complete(int dev, long long id, bool notify, double ms, const std::string& err);
  struct Wake {
    bool comp = false, done = false, work = false;
  };
  void complete_locked(int dev, long long id, bool notify, double ms, const std::string& err, Wake& w);
  void wake(const Wake& w);
  int retire(int dev, std::vector<Inflight>& inflight);

  std::vector<std::shared_ptr<Cores>> devs_;
  int max_in_flight_;
  int policy_ = 0;
  long long rr_next_ = 0;  // round robin: next device in the rotation
  int rr_group_ = -1;      // round robin: device of the open select/serial group
  std::mutex mu_;
  std::condition_variable work_cv_, done_cv_, comp_cv_;
  std::deque<Item> queue_;
  std::deque<PoolCompletion> done_;     // notify tasks
  std::vector<PoolCompletion> errors_;  // failed tasks
  struct Result {
    int device = -1;
    float ms = 0;
  };
  std::vector<Result> results_;  // by task id
  long long outstanding_ = 0;
  int running_ = 0;  // taken and not yet retired
  int owner_ = -1;   // device holding a select/serial group
  bool serial_owner_ = false;  // that group is a serial-mode group
  bool closed_ = false;
  std::vector<long long> counts_;
  std::vector<double> busy_ms_;
  std::vector<int> inflight_;              // taken, not retired, per device
  std::vector<PoolProgress> pools_;
  std::vector<int> limit_history_;
  struct Speed {
    double last_ms = -1;
    double hist[15] = {0};
    long long n = 0;
  };
  std::vector<Speed> speed_;
  std::vector<std::thread> threads_;
  // host-time profile, one cache line per consumer (written by that consumer
  // only: shared counters bounced one line between 8 consumer threads)
  struct alignas(64) Prof {
    std::atomic<double> issue_ms{0}, retire_ms{0};
    std::atomic<long long> tasks{0}, polls{0};
  };
  std::unique_ptr<Prof[]> prof_;
};

}  // namespace cek
