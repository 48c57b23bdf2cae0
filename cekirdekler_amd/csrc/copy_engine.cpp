#include "copy_engine.h"

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
  if (dst_dev >= 0 && src_dev >= 0) {
    hipStream_t s = stream(dst_dev);
    CEK_HIP(hipSetDevice(dst_dev));
    CEK_HIP(hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, s));
    p2p_bytes += bytes;
  } else if (dst_dev >= 0) {
    hipStream_t s = stream(dst_dev);
    CEK_HIP(hipSetDevice(dst_dev));
    CEK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    h2d_bytes += bytes;
  } else {
    hipStream_t s = stream(src_dev);
    CEK_HIP(hipSetDevice(src_dev));
    CEK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    d2h_bytes += bytes;
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
