// Multi-process (one process per MI355X) support.
//
// The reference drives every device from one process (Cores.cs:156-344) and
// balances them with per-device timings it holds in memory.  On MI355X the
// idiomatic layout is one process per GPU, so the balancer's input — every
// device's time for the previous call of a compute id — is exchanged across
// ranks:
//   * ShmExchanger: node-local control plane in POSIX shared memory
//     (double-buffered slots + per-rank epoch words; ~µs per exchange),
//   * Comm: RCCL communicator (xGMI) used for the data plane — broadcast of
//     `read` arrays and all-gather(v) of written slices so device replicas
//     stay coherent without a host bounce.
#pragma once
#include "common.h"

namespace cek {

class Exchanger {
 public:
  virtual ~Exchanger() = default;
  // Gather `n` doubles from every rank; returns world*n values, rank-major.
  virtual std::vector<double> allgather(const std::vector<double>& local) = 0;
  virtual void barrier() { allgather(std::vector<double>(1, 0.0)); }
  virtual int rank() const = 0;
  virtual int world() const = 0;
};

class ShmExchanger : public Exchanger {
 public:
  // Rank 0 creates the segment, the others attach (retrying up to timeout).
  ShmExchanger(const std::string& name, int rank, int world, int max_values = 64,
               double timeout_s = 300.0);
  ~ShmExchanger() override;
  std::vector<double> allgather(const std::vector<double>& local) override;
  void unlink();  // remove the name (segment lives until every rank unmaps)
  int rank() const override { return rank_; }
  int world() const override { return world_; }

 private:
  std::string name_;
  int rank_, world_, maxv_;
  double timeout_s_;
  void* base_ = nullptr;
  size_t size_ = 0;
  uint64_t epoch_ = 0;
};

// Data plane of a distributed job: broadcast / all-gather-v / all-reduce on
// device (or, for CPU devices, host) memory, ordered on stream s.
class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // In-place broadcast of `bytes` at dptr from root.
  virtual void broadcast(void* dptr, uint64_t bytes, int root, hipStream_t s) = 0;
  // In-place all-gather-v: rank r owns [offsets[r], offsets[r]+sizes[r]) bytes.
  virtual void allgatherv(void* dptr, const std::vector<uint64_t>& offsets,
                          const std::vector<uint64_t>& sizes, hipStream_t s) = 0;
  virtual void allreduce_sum_f32(void* dptr, uint64_t count, hipStream_t s) = 0;
  virtual void allreduce_sum_f64(void* dptr, uint64_t count, hipStream_t s) = 0;
};

// One point-to-point transfer of an uneven all-gather-v, from this rank's
// point of view: send this rank's slice to `peer`, or receive `peer`'s.
struct P2POp {
  bool send;
  int peer;
  uint64_t offset, bytes;
};

// The grouped sends/receives rank `rank` issues for an uneven all-gather-v
// (RcclComm::allgatherv).  Pure function of the (identical on every rank)
// offsets/sizes, so the pairing — every send matched by exactly one receive
// of the same bytes at the peer, zero-byte pairs skipped on both sides — is
// checked on the CPU for every world size (tests/test_allgatherv_plan.py).
std::vector<P2POp> allgatherv_plan(int rank, int world, const std::vector<uint64_t>& offsets,
                                   const std::vector<uint64_t>& sizes);

// RCCL communicator over xGMI (one GPU per rank).
class RcclComm : public Comm {
 public:
  static std::string unique_id();  // bytes of an ncclUniqueId
  RcclComm(const std::string& uid, int rank, int world, int device);
  ~RcclComm() override;
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void broadcast(void* dptr, uint64_t bytes, int root, hipStream_t s) override;
  // Equal contiguous slices: one RCCL all-gather.  Uneven slices (after the
  // balancer moved work): grouped point-to-point sends, each rank's slice
  // straight to every peer over that pair's own xGMI link.
  // CEK_ALLGATHERV=direct uses the sends for equal slices too.
  void allgatherv(void* dptr, const std::vector<uint64_t>& offsets,
                  const std::vector<uint64_t>& sizes, hipStream_t s) override;
  void allreduce_sum_f32(void* dptr, uint64_t count, hipStream_t s) override;
  void allreduce_sum_f64(void* dptr, uint64_t count, hipStream_t s) override;

 private:
  void* comm_ = nullptr;  // ncclComm_t
  int rank_, world_, device_;
};

}  // namespace cek
