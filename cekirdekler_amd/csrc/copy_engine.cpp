#include "copy_engine.h"

#include "xgmi.h"

#include <cstring>

#include "device.h"

namespace cek {

CopyEngine::~CopyEngine() {
  for (size_t i = 0; i < streams_.size(); ++i) {
    if (!streams_[i]) continue;
    (void)hipSetDevice(static_cast<int>(i));
    (void)hipStreamSynchronize(streams_[i]);
    (void)hipStreamDestroy(streams_[i]);
  }
  for (auto& p : pending_) free_events_.push_back({p.ordinal, p.b}), free_events_.push_back({p.ordinal, p.e});
  for (auto& fe : free_events_) {
    (void)hipSetDevice(fe.first);
    (void)hipEventDestroy(fe.second);
  }
}

hipEvent_t CopyEngine::timing_event(int ordinal) {
  for (size_t i = 0; i < free_events_.size(); ++i)
    if (free_events_[i].first == ordinal) {
      hipEvent_t e = free_events_[i].second;
      free_events_.erase(free_events_.begin() + static_cast<long>(i));
      return e;
    }
  hipEvent_t e;
  CEK_HIP(hipEventCreateWithFlags(&e, kTimingEventFlags));
  return e;
}

std::vector<CopyEngine::Span> CopyEngine::timeline() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Span> out;
  for (auto& p : pending_) {
    CEK_HIP(hipSetDevice(p.ordinal));
    CEK_HIP(hipEventSynchronize(p.e));
    out.push_back({p.ordinal, p.kind, p.bytes, event_host_ms(p.ordinal, p.b), event_host_ms(p.ordinal, p.e)});
    free_events_.push_back({p.ordinal, p.b});
    free_events_.push_back({p.ordinal, p.e});
  }
  pending_.clear();
  return out;
}

hipStream_t CopyEngine::stream(int ordinal) {
  if (ordinal < 0) throw Error("copy engine: no stream for host memory");
  if (static_cast<int>(streams_.size()) <= ordinal) streams_.resize(ordinal + 1, nullptr);
  if (!streams_[ordinal]) {
    CEK_HIP(hipSetDevice(ordinal));
    CEK_HIP(hipStreamCreateWithFlags(&streams_[ordinal], hipStreamNonBlocking));
  }
  return streams_[ordinal];
}

void CopyEngine::copy(void* dst, int dst_dev, const void* src, int src_dev, uint64_t bytes) {
  if (bytes == 0 || dst == src) return;
  std::lock_guard<std::mutex> g(mu_);
  ++copies;
  if (dst_dev < 0 && src_dev < 0) {
    std::memcpy(dst, src, bytes);
    host_bytes += bytes;
    return;
  }
  const int on = dst_dev >= 0 ? dst_dev : src_dev;  // the GPU whose stream runs the copy
  hipStream_t s = stream(on);
  CEK_HIP(hipSetDevice(on));
  Pending p{on, "", bytes, nullptr, nullptr};
  if (record_timeline) {
    p.b = timing_event(on);
    p.e = timing_event(on);
    CEK_HIP(hipEventRecord(p.b, s));
  }
  if (dst_dev >= 0 && src_dev >= 0) {
    // SDMA or a pull kernel on the destination, by the calibrated table (xgmi.h)
    peer_copy(dst, dst_dev, src, src_dev, bytes, s, on);
    p2p_bytes += bytes;
    p.kind = "p2p";
  } else if (dst_dev >= 0) {
    CEK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    h2d_bytes += bytes;
    p.kind = "h2d";
  } else {
    CEK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    d2h_bytes += bytes;
    p.kind = "d2h";
  }
  if (record_timeline) {
    CEK_HIP(hipEventRecord(p.e, s));
    pending_.push_back(p);
  }
}

void CopyEngine::sync() {
  std::lock_guard<std::mutex> g(mu_);
  for (size_t i = 0; i < streams_.size(); ++i) {
    if (!streams_[i]) continue;
    CEK_HIP(hipSetDevice(static_cast<int>(i)));
    CEK_HIP(hipStreamSynchronize(streams_[i]));
  }
}

}  // namespace cek
