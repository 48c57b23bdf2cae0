// Asynchronous copy engine for stage-to-stage transfers (the device→device
// ClPipeline).  The reference moves every stage transition through host
// memory with blocking reads/writes (ClPipeline.cs:1422-1574); here each
// transfer is one async copy on a per-GPU copy stream:
//   * GPU → GPU: hipMemcpyPeerAsync on the DESTINATION GPU's stream (the
//     destination pulls over the xGMI link to the source; on MI355X every
//     pair of GPUs has its own link, so pulls from different sources run on
//     different links),
//   * host ↔ GPU: hipMemcpyAsync on that GPU's stream (PCIe),
//   * host ↔ host (CPU devices): memcpy.
// Copies of one push are enqueued back to back without host syncs; sync()
// waits for all of them once.  Byte counters split the traffic by path so
// tests can assert that a push never bounces through host memory.
#pragma once
#include <mutex>
#include <vector>

#include "common.h"

namespace cek {

class CopyEngine {
 public:
  CopyEngine() = default;
  ~CopyEngine();
  CopyEngine(const CopyEngine&) = delete;
  CopyEngine& operator=(const CopyEngine&) = delete;

  // dst_dev / src_dev: GPU ordinal, or -1 for host memory.
  void copy(void* dst, int dst_dev, const void* src, int src_dev, uint64_t bytes);
  void sync();

  uint64_t p2p_bytes = 0, h2d_bytes = 0, d2h_bytes = 0, host_bytes = 0;
  uint64_t copies = 0;
  void reset_counters() { p2p_bytes = h2d_bytes = d2h_bytes = host_bytes = copies = 0; }

  // Copy timeline: with record_timeline on, every device copy is bracketed
  // by timing events on its stream; timeline() waits for them and returns
  // each copy's span on the host clock (event_host_ms), then clears the list.
  bool record_timeline = false;
  struct Span {
    int ordinal;       // the GPU whose stream ran the copy
    std::string kind;  // p2p | h2d | d2h
    uint64_t bytes;
    double abs_begin_ms, abs_end_ms;
  };
  std::vector<Span> timeline();

 private:
  struct Pending {
    int ordinal;
    std::string kind;
    uint64_t bytes;
    hipEvent_t b, e;
  };
  std::vector<Pending> pending_;
  std::vector<std::pair<int, hipEvent_t>> free_events_;
  hipEvent_t timing_event(int ordinal);
  hipStream_t stream(int ordinal);
  std::mutex mu_;
  std::vector<hipStream_t> streams_;
};

}  // namespace cek
