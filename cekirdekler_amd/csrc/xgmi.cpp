#include "xgmi.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>

#include "device.h"
#include "jit.h"
#include "memory.h"

namespace cek {

namespace {

// 16 bytes per lane, grid-stride: the kernel engine.  Launched on the GPU of
// the stream; with peer access on, either pointer may live on another GPU.
const char* kCopy16 = R"CEK(
typedef unsigned int cek_u32x4 __attribute__((ext_vector_type(4)));
__global__ void cek_copy16_d2d(const cek_u32x4* src, cek_u32x4* dst, long long n16) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (; i < n16; i += stride) dst[i] = src[i];
}
)CEK";

std::mutex g_mu;
std::map<int, std::shared_ptr<Program>> g_prog;
std::map<std::pair<int, int>, std::map<uint64_t, int>> g_table;  // (src, dst) -> bytes -> engine
int g_override = [] {
  const char* e = std::getenv("CEK_D2D_ENGINE");
  return e ? std::atoi(e) : -1;
}();

hipFunction_t copy_fn(int ordinal) {
  std::lock_guard<std::mutex> g(g_mu);
  auto& p = g_prog[ordinal];
  if (!p) {
    p = Program::build(gpu_info(ordinal), kCopy16, {}, {});
    if (!p->ok()) throw Error("device copy kernel failed to build: " + p->log());
  }
  return p->gpu_fn("cek_copy16_d2d");
}

std::map<std::pair<int, int>, bool> g_access;  // (accessing GPU, owning GPU) -> peer access on

// Whether a kernel on GPU `a` may dereference memory of GPU `b`: peer access
// enabled (once per pair).  A copy kernel that touched another GPU's memory
// without it would fault, and a fault can reset every GPU of the node.
bool kernel_can_reach(int a, int b) {
  if (a == b) return true;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_access.find({a, b});
    if (it != g_access.end()) return it->second;
  }
  const auto m = enable_peer_access_among({a, b});
  const bool ok = m[0][1] != 0;
  std::lock_guard<std::mutex> g(g_mu);
  g_access[{a, b}] = ok;
  g_access[{b, a}] = m[1][0] != 0;
  return ok;
}

bool kernel_engine_ok(int ordinal, int src_dev, int dst_dev) {
  return kernel_can_reach(ordinal, src_dev) && kernel_can_reach(ordinal, dst_dev);
}

void launch_copy(int ordinal, void* dst, const void* src, uint64_t bytes, hipStream_t s) {
  // whole 16-byte vectors by the kernel, a ragged tail (if any) by SDMA
  const uint64_t body = bytes & ~uint64_t(15);
  if (body && ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0) {
    hipFunction_t f = copy_fn(ordinal);
    long long n16 = static_cast<long long>(body / 16), off = 0, gs = n16;
    void* params[] = {&src, &dst, &n16, &off, &gs};
    // 8 work-groups per CU of 256 lanes: enough requests in flight to fill a
    // link; fewer for small copies
    const long long per_group = 256ll * 8;
    const unsigned groups = static_cast<unsigned>(std::max(1ll, std::min(2048ll, (n16 + per_group - 1) / per_group)));
    CEK_HIP(hipModuleLaunchKernel(f, groups, 1, 1, 256, 1, 1, 0, s, params, nullptr));
  } else {
    CEK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
    return;
  }
  if (bytes > body)
    CEK_HIP(hipMemcpyAsync(static_cast<char*>(dst) + body, static_cast<const char*>(src) + body, bytes - body,
                           hipMemcpyDeviceToDevice, s));
}

void sdma_copy(void* dst, int dst_dev, const void* src, int src_dev, uint64_t bytes, hipStream_t s) {
  if (src_dev == dst_dev)
    CEK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
  else
    CEK_HIP(hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, s));
}

// deterministic, position-dependent bytes (an offset error shows)
void fill_pattern(std::vector<uint32_t>& v, uint32_t seed) {
  uint32_t x = seed * 2654435761u + 1u;
  for (auto& w : v) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    w = x;
  }
}

struct DevBuf {
  int ordinal = -1;
  void* p = nullptr;
  DevBuf(int o, uint64_t bytes) : ordinal(o) {
    CEK_HIP(hipSetDevice(o));
    CEK_HIP(hipMalloc(&p, bytes));
  }
  ~DevBuf() {
    if (p) {
      (void)hipSetDevice(ordinal);
      (void)hipFree(p);
    }
  }
};

}  // namespace

int peer_copy(void* dst, int dst_dev, const void* src, int src_dev, uint64_t bytes, hipStream_t s,
              int stream_ordinal) {
  if (!bytes) return kCopySdma;
  int e = choose_engine(src_dev, dst_dev, bytes);
  // the kernel runs on the stream's GPU and dereferences both ends
  if (e == kCopyKernel && !kernel_engine_ok(stream_ordinal, src_dev, dst_dev)) e = kCopySdma;
  if (e == kCopyKernel)
    launch_copy(stream_ordinal, dst, src, bytes, s);
  else
    sdma_copy(dst, dst_dev, src, src_dev, bytes, s);
  return e;
}

CopyMeasure measure_copy(int src, int dst, uint64_t bytes, int engine, int reps, int stream_ordinal) {
  if (bytes == 0 || bytes % 4) throw Error("measure_copy: bytes must be a positive multiple of 4");
  if (engine != kCopySdma && engine != kCopyKernel) throw Error("measure_copy: engine is 0 (SDMA) or 1 (kernel)");
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (src != dst) enable_peer_access_among({src, dst});
  const int so = stream_ordinal >= 0 ? stream_ordinal : dst;
  if (engine == kCopyKernel && !kernel_engine_ok(so, src, dst))
    throw Error("measure_copy: no peer access for a copy kernel on GPU " + std::to_string(so) + " between GPUs " +
                std::to_string(src) + " and " + std::to_string(dst));
  CopyMeasure m;
  m.src = src;
  m.dst = dst;
  m.engine = engine;
  m.stream_ordinal = so;
  m.bytes = bytes;
  m.reps = std::max(1, reps);
  {
    DevBuf sb(src, bytes), db(dst, bytes);
    std::vector<uint32_t> pat(bytes / 4), back(bytes / 4);
    fill_pattern(pat, static_cast<uint32_t>(src * 31 + dst + 7));
    CEK_HIP(hipSetDevice(src));
    CEK_HIP(hipMemcpy(sb.p, pat.data(), bytes, hipMemcpyHostToDevice));
    CEK_HIP(hipSetDevice(dst));
    CEK_HIP(hipMemset(db.p, 0, bytes));
    CEK_HIP(hipSetDevice(so));
    hipStream_t s;
    CEK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CEK_HIP(hipEventCreate(&e0));
    CEK_HIP(hipEventCreate(&e1));
    auto one = [&] {
      if (engine == kCopyKernel)
        launch_copy(so, db.p, sb.p, bytes, s);
      else
        sdma_copy(db.p, dst, sb.p, src, bytes, s);
    };
    one();  // untimed (first-touch, page tables, module load)
    CEK_HIP(hipEventRecord(e0, s));
    for (int r = 0; r < m.reps; ++r) one();
    CEK_HIP(hipEventRecord(e1, s));
    CEK_HIP(hipEventSynchronize(e1));
    float ms = 0;
    CEK_HIP(hipEventElapsedTime(&ms, e0, e1));
    m.ms = ms / m.reps;
    m.gbps = static_cast<double>(bytes) / (m.ms * 1e6);
    CEK_HIP(hipSetDevice(dst));
    CEK_HIP(hipMemcpy(back.data(), db.p, bytes, hipMemcpyDeviceToHost));
    m.verified = std::memcmp(back.data(), pat.data(), bytes) == 0;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
  }
  if (cur >= 0) (void)hipSetDevice(cur);
  return m;
}

ConcurrentMeasure measure_all_pairs(const std::vector<int>& ords, uint64_t bytes, int engine, int reps) {
  ConcurrentMeasure cm;
  cm.gpus = static_cast<int>(ords.size());
  cm.engine = engine;
  cm.bytes_per_copy = bytes;
  if (ords.size() < 2 || bytes == 0 || bytes % 4) return cm;
  int cur = -1;
  (void)hipGetDevice(&cur);
  enable_peer_access_among(ords);
  const int n = static_cast<int>(ords.size());
  if (engine == kCopyKernel)
    for (int d = 0; d < n; ++d)
      for (int s = 0; s < n; ++s)
        if (!kernel_can_reach(ords[d], ords[s])) return cm;  // not measurable: verified stays false
  reps = std::max(1, reps);
  std::vector<std::unique_ptr<DevBuf>> src(n);
  std::vector<std::vector<std::unique_ptr<DevBuf>>> dst(n);
  std::vector<std::vector<hipStream_t>> st(n, std::vector<hipStream_t>(n, nullptr));
  std::vector<std::vector<uint32_t>> pat(n, std::vector<uint32_t>(bytes / 4));
  for (int i = 0; i < n; ++i) {
    src[i].reset(new DevBuf(ords[i], bytes));
    fill_pattern(pat[i], static_cast<uint32_t>(ords[i] + 101));
    CEK_HIP(hipMemcpy(src[i]->p, pat[i].data(), bytes, hipMemcpyHostToDevice));
  }
  for (int d = 0; d < n; ++d) {
    dst[d].resize(n);
    for (int s = 0; s < n; ++s) {
      if (s == d) continue;
      dst[d][s].reset(new DevBuf(ords[d], bytes));
      CEK_HIP(hipSetDevice(ords[d]));
      CEK_HIP(hipStreamCreateWithFlags(&st[d][s], hipStreamNonBlocking));
    }
  }
  auto issue = [&](int times) {
    for (int r = 0; r < times; ++r)
      for (int d = 0; d < n; ++d)
        for (int s = 0; s < n; ++s) {
          if (s == d) continue;
          CEK_HIP(hipSetDevice(ords[d]));
          if (engine == kCopyKernel)
            launch_copy(ords[d], dst[d][s]->p, src[s]->p, bytes, st[d][s]);
          else
            sdma_copy(dst[d][s]->p, ords[d], src[s]->p, ords[s], bytes, st[d][s]);
        }
  };
  auto drain = [&] {
    for (int d = 0; d < n; ++d)
      for (int s = 0; s < n; ++s)
        if (st[d][s]) {
          CEK_HIP(hipSetDevice(ords[d]));
          CEK_HIP(hipStreamSynchronize(st[d][s]));
        }
  };
  issue(1);
  drain();
  const double t0 = now_ms();
  issue(reps);
  drain();
  cm.wall_ms = now_ms() - t0;
  cm.copies = n * (n - 1) * reps;
  cm.aggregate_gbps = static_cast<double>(bytes) * cm.copies / (cm.wall_ms * 1e6);
  cm.per_copy_gbps = cm.aggregate_gbps / (n * (n - 1));
  bool ok = true;
  std::vector<uint32_t> back(bytes / 4);
  for (int d = 0; d < n && ok; ++d)
    for (int s = 0; s < n && ok; ++s) {
      if (s == d) continue;
      CEK_HIP(hipSetDevice(ords[d]));
      CEK_HIP(hipMemcpy(back.data(), dst[d][s]->p, bytes, hipMemcpyDeviceToHost));
      ok = std::memcmp(back.data(), pat[s].data(), bytes) == 0;
    }
  cm.verified = ok;
  for (int d = 0; d < n; ++d)
    for (int s = 0; s < n; ++s)
      if (st[d][s]) {
        (void)hipSetDevice(ords[d]);
        (void)hipStreamDestroy(st[d][s]);
      }
  src.clear();
  dst.clear();
  if (cur >= 0) (void)hipSetDevice(cur);
  return cm;
}

void calibrate(const std::vector<int>& ords, const std::vector<uint64_t>& sizes, int reps) {
  std::map<std::pair<int, int>, std::map<uint64_t, int>> t;
  for (int s : ords)
    for (int d : ords)
      for (uint64_t b : sizes) {
        const CopyMeasure a = measure_copy(s, d, b, kCopySdma, reps);
        if (!a.verified) throw Error("calibrate: a measured copy did not verify");
        if (!kernel_engine_ok(d, s, d)) {  // no peer access: SDMA only
          t[{s, d}][b] = kCopySdma;
          continue;
        }
        const CopyMeasure k = measure_copy(s, d, b, kCopyKernel, reps);
        if (!k.verified) throw Error("calibrate: a measured copy did not verify");
        t[{s, d}][b] = k.gbps > a.gbps ? kCopyKernel : kCopySdma;
      }
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& kv : t) g_table[kv.first] = kv.second;
}

int choose_engine(int src, int dst, uint64_t bytes) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_override == kCopySdma || g_override == kCopyKernel) return g_override;
  auto it = g_table.find({src, dst});
  if (it == g_table.end() || it->second.empty()) return kCopySdma;
  // nearest calibrated size class (log scale)
  const auto& m = it->second;
  auto hi = m.lower_bound(bytes);
  if (hi == m.end()) return std::prev(hi)->second;
  if (hi == m.begin()) return hi->second;
  auto lo = std::prev(hi);
  const double l = std::log2(static_cast<double>(bytes) / lo->first), h = std::log2(static_cast<double>(hi->first) / bytes);
  return l <= h ? lo->second : hi->second;
}

void record_engine(int src, int dst, uint64_t bytes, int engine) {
  if (engine != kCopySdma && engine != kCopyKernel) throw Error("record_engine: engine is 0 or 1");
  std::lock_guard<std::mutex> g(g_mu);
  g_table[{src, dst}][bytes] = engine;
}

void set_engine_override(int engine) {
  std::lock_guard<std::mutex> g(g_mu);
  g_override = engine;
}

std::vector<std::vector<double>> engine_table() {
  std::lock_guard<std::mutex> g(g_mu);
  std::vector<std::vector<double>> out;
  for (auto& kv : g_table)
    for (auto& e : kv.second)
      out.push_back({double(kv.first.first), double(kv.first.second), double(e.first), double(e.second)});
  return out;
}

}  // namespace cek
