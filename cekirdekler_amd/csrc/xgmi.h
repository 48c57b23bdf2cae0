// Device→device copy engines and xGMI link evidence.
//
// The reference has no device→device path at all (every transition bounces
// through host memory, ClPipeline.cs:1422-1574; Worker.cs:833-860).  Here a
// GPU→GPU copy is either
//   * SDMA: hipMemcpyPeerAsync / hipMemcpyAsync(D2D) — the DMA engines,
//     no compute units used, or
//   * kernel: a 16-byte-per-lane copy kernel on the stream's GPU that reads
//     (pull) or writes (push) the peer's memory over xGMI with peer access
//     on — several CUs keep many requests in flight per link.
// Which one is faster depends on the pair and the size (the PCIe probe of
// profiles/hostres_streaming.md saw the same choice double or halve the
// rate), so it is measured, not assumed: measure_copy() times one engine on
// one pair, calibrate() fills a per-(pair, size class) table, and
// peer_copy() — used by Cores' read fan-out / keep-resident gather /
// copy_between and by the pipeline CopyEngine — takes the faster engine
// from that table (SDMA until a pair is calibrated).
#pragma once
#include "common.h"

namespace cek {

enum CopyKind : int { kCopySdma = 0, kCopyKernel = 1 };

struct CopyMeasure {
  int src = -1, dst = -1, engine = 0;
  int stream_ordinal = -1;  // the GPU whose stream ran the copy (kernel: its CUs)
  uint64_t bytes = 0;
  int reps = 0;
  double ms = 0;    // per copy
  double gbps = 0;  // bytes / ms
  bool verified = false;  // destination equal to the source, byte for byte
};

// Time `reps` copies of `bytes` from GPU src to GPU dst (src == dst: a copy
// inside one GPU) with one engine, on a stream of `stream_ordinal` (-1: the
// destination's, i.e. a pull), after one untimed copy; then compare the
// destination with the source byte for byte.
CopyMeasure measure_copy(int src, int dst, uint64_t bytes, int engine, int reps, int stream_ordinal = -1);

// Every ordered pair of `ordinals` at once (each destination pulls from every
// source on its own stream): aggregate GB/s over the wall time.
struct ConcurrentMeasure {
  int gpus = 0, copies = 0, engine = 0;
  uint64_t bytes_per_copy = 0;
  double wall_ms = 0, aggregate_gbps = 0, per_copy_gbps = 0;
  bool verified = false;
};
ConcurrentMeasure measure_all_pairs(const std::vector<int>& ordinals, uint64_t bytes, int engine, int reps);

// Engine table: calibrate() measures both engines for every ordered pair of
// `ordinals` (and each GPU with itself) at each size and records the faster
// one per size class; choose_engine() looks it up (SDMA for an unknown pair,
// the nearest calibrated size class otherwise).
void calibrate(const std::vector<int>& ordinals, const std::vector<uint64_t>& sizes, int reps);
int choose_engine(int src, int dst, uint64_t bytes);
void set_engine_override(int engine);  // -1: table, 0/1: force (tests, env CEK_D2D_ENGINE)
void record_engine(int src, int dst, uint64_t bytes, int engine);  // one measured winner
std::vector<std::vector<double>> engine_table();  // rows: src, dst, bytes, engine

// One GPU→GPU copy on stream s of GPU stream_ordinal with the chosen engine.
// Returns the engine used.
int peer_copy(void* dst, int dst_dev, const void* src, int src_dev, uint64_t bytes, hipStream_t s,
              int stream_ordinal);

}  // namespace cek
