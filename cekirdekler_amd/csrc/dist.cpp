#include "dist.h"

#include <fcntl.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <thread>

namespace cek {

namespace {
constexpr uint32_t kMagic = 0xCE4D1ADu;
struct ShmHeader {
  std::atomic<uint32_t> magic;
  int32_t world;
  int32_t maxv;
  int32_t pad;
};
constexpr size_t kLine = 64;
size_t shm_size(int world, int maxv) {
  return kLine + static_cast<size_t>(world) * kLine + 2ull * world * maxv * sizeof(double);
}
}  // namespace

ShmExchanger::ShmExchanger(const std::string& name, int rank, int world, int max_values,
                           double timeout_s)
    : name_(name[0] == '/' ? name : "/" + name), rank_(rank), world_(world), maxv_(max_values),
      timeout_s_(timeout_s) {
  size_ = shm_size(world, max_values);
  int fd = -1;
  double t0 = now_ms();
  if (rank == 0) {
    shm_unlink(name_.c_str());
    fd = shm_open(name_.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0) throw Error("shm_open(create) failed for " + name_);
    if (ftruncate(fd, static_cast<off_t>(size_)) != 0) {
      close(fd);
      throw Error("ftruncate failed for " + name_);
    }
  } else {
    for (;;) {
      fd = shm_open(name_.c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && static_cast<size_t>(st.st_size) >= size_) break;
        close(fd);
        fd = -1;
      }
      if (now_ms() - t0 > timeout_s_ * 1000) throw Error("timeout attaching to " + name_);
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
  }
  base_ = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base_ == MAP_FAILED) throw Error("mmap failed for " + name_);
  auto* h = static_cast<ShmHeader*>(base_);
  if (rank == 0) {
    std::memset(static_cast<char*>(base_) + kLine, 0, size_ - kLine);
    h->world = world;
    h->maxv = max_values;
    h->magic.store(kMagic, std::memory_order_release);
  } else {
    while (h->magic.load(std::memory_order_acquire) != kMagic) {
      if (now_ms() - t0 > timeout_s_ * 1000) throw Error("timeout waiting for " + name_);
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (h->world != world || h->maxv < max_values) throw Error("shm segment shape mismatch");
  }
}

ShmExchanger::~ShmExchanger() {
  if (base_ && base_ != MAP_FAILED) munmap(base_, size_);
}

void ShmExchanger::unlink() { shm_unlink(name_.c_str()); }

std::vector<double> ShmExchanger::allgather(const std::vector<double>& local) {
  const int n = static_cast<int>(local.size());
  if (n > maxv_) throw Error("ShmExchanger: too many values");
  char* b = static_cast<char*>(base_);
  auto epoch_word = [&](int r) {
    return reinterpret_cast<std::atomic<uint64_t>*>(b + kLine + static_cast<size_t>(r) * kLine);
  };
  double* vals = reinterpret_cast<double*>(b + kLine + static_cast<size_t>(world_) * kLine);
  uint64_t e = ++epoch_;
  int buf = static_cast<int>(e & 1);
  double* mine = vals + (static_cast<size_t>(buf) * world_ + rank_) * maxv_;
  for (int i = 0; i < n; ++i) mine[i] = local[i];
  epoch_word(rank_)->store(e, std::memory_order_release);
  double t0 = now_ms();
  long spins = 0;
  for (int r = 0; r < world_; ++r) {
    while (epoch_word(r)->load(std::memory_order_acquire) < e) {
      if (++spins > 2000) {
        sched_yield();
        if ((spins & 1023) == 0 && now_ms() - t0 > timeout_s_ * 1000)
          throw Error("ShmExchanger: timeout waiting for rank " + std::to_string(r));
      }
    }
  }
  std::vector<double> out(static_cast<size_t>(world_) * n);
  for (int r = 0; r < world_; ++r) {
    const double* src = vals + (static_cast<size_t>(buf) * world_ + r) * maxv_;
    for (int i = 0; i < n; ++i) out[static_cast<size_t>(r) * n + i] = src[i];
  }
  return out;
}

// -------------------------------------------------------------------- Comm --

#define CEK_NCCL(expr)                                                             \
  do {                                                                             \
    ncclResult_t _r = (expr);                                                      \
    if (_r != ncclSuccess)                                                         \
      throw Error(std::string("RCCL error in " #expr ": ") + ncclGetErrorString(_r)); \
  } while (0)

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  CEK_NCCL(ncclGetUniqueId(&id));
  return std::string(id.internal, sizeof(id.internal));
}

RcclComm::RcclComm(const std::string& uid, int rank, int world, int device)
    : rank_(rank), world_(world), device_(device) {
  if (uid.size() != sizeof(ncclUniqueId)) throw Error("bad RCCL unique id size");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), sizeof(id.internal));
  CEK_HIP(hipSetDevice(device));
  ncclComm_t c;
  CEK_NCCL(ncclCommInitRank(&c, world, id, rank));
  comm_ = c;
}

RcclComm::~RcclComm() {
  if (comm_) ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void RcclComm::broadcast(void* dptr, uint64_t bytes, int root, hipStream_t s) {
  if (bytes == 0 || world_ == 1) return;
  CEK_NCCL(ncclBroadcast(dptr, dptr, bytes, ncclChar, root, static_cast<ncclComm_t>(comm_), s));
}

void RcclComm::allgatherv(void* dptr, const std::vector<uint64_t>& offsets,
                      const std::vector<uint64_t>& sizes, hipStream_t s) {
  if (world_ == 1) return;
  auto* base = static_cast<char*>(dptr);
  // Equal slices at contiguous offsets: one ring all-gather.
  static const bool direct_always = [] {
    const char* e = std::getenv("CEK_ALLGATHERV");
    return e && std::string(e) == "direct";
  }();
  bool equal = !direct_always;
  for (int r = 0; r < world_; ++r)
    if (sizes[r] != sizes[0] || offsets[r] != offsets[0] + sizes[0] * r) equal = false;
  if (equal && sizes[0] > 0) {
    CEK_NCCL(ncclAllGather(base + offsets[rank_], base + offsets[0], sizes[0], ncclChar,
                           static_cast<ncclComm_t>(comm_), s));
    return;
  }
  // Uneven slices (the balancer moved work): every rank sends its slice
  // straight to each peer (allgatherv_plan).  The MI355X node is a full xGMI
  // mesh — one link per GPU pair — so the N−1 sends of a rank leave on N−1
  // different links at once and each link carries one slice, where a ring (or
  // a group of ring broadcasts) pushes every slice over every link it passes.
  auto* comm = static_cast<ncclComm_t>(comm_);
  const auto plan = allgatherv_plan(rank_, world_, offsets, sizes);
  if (plan.empty()) return;
  // A throw between ncclGroupStart and ncclGroupEnd must still close the
  // group: an open group turns every later call on this communicator into a
  // confusing failure.
  struct Group {
    bool open = false;
    void start() {
      CEK_NCCL(ncclGroupStart());
      open = true;
    }
    void end() {
      open = false;
      CEK_NCCL(ncclGroupEnd());
    }
    ~Group() {
      if (open) (void)ncclGroupEnd();
    }
  } group;
  group.start();
  for (const auto& op : plan) {
    if (op.send)
      CEK_NCCL(ncclSend(base + op.offset, op.bytes, ncclChar, op.peer, comm, s));
    else
      CEK_NCCL(ncclRecv(base + op.offset, op.bytes, ncclChar, op.peer, comm, s));
  }
  group.end();
}

std::vector<P2POp> allgatherv_plan(int rank, int world, const std::vector<uint64_t>& offsets,
                                   const std::vector<uint64_t>& sizes) {
  if (world < 1 || rank < 0 || rank >= world) throw Error("allgatherv_plan: bad rank / world");
  if (static_cast<int>(offsets.size()) != world || static_cast<int>(sizes.size()) != world)
    throw Error("allgatherv_plan: one offset and one size per rank");
  std::vector<P2POp> plan;
  // step k: send to rank+k, receive from rank−k (every rank's k-th pair is a
  // matched shift, so no link carries two slices in one step)
  for (int k = 1; k < world; ++k) {
    const int to = (rank + k) % world, from = (rank - k + world) % world;
    if (sizes[rank] > 0) plan.push_back({true, to, offsets[rank], sizes[rank]});
    if (sizes[from] > 0) plan.push_back({false, from, offsets[from], sizes[from]});
  }
  return plan;
}

void RcclComm::allreduce_sum_f32(void* dptr, uint64_t count, hipStream_t s) {
  CEK_NCCL(ncclAllReduce(dptr, dptr, count, ncclFloat32, ncclSum, static_cast<ncclComm_t>(comm_), s));
}

void RcclComm::allreduce_sum_f64(void* dptr, uint64_t count, hipStream_t s) {
  CEK_NCCL(ncclAllReduce(dptr, dptr, count, ncclFloat64, ncclSum, static_cast<ncclComm_t>(comm_), s));
}

}  // namespace cek
