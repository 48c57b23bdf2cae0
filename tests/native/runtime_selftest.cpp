// Native self-test of the C++ runtime on the host CPU device, built with
// AddressSanitizer + UndefinedBehaviorSanitizer (sanitizers on
// the host runtime).  Exercises the balancer law, the JIT front end, and
// Cores::compute on logical CPU devices: plain, event/driver pipelines,
// repeats + sync kernel, phase separation, failover.  Exit code 0 = pass.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "balancer.h"
#include "cores.h"
#include "device.h"
#include "jit.h"

using namespace cek;

static int failures = 0;
#define CHECK(cond)                                                      \
  do {                                                                   \
    if (!(cond)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                        \
    }                                                                    \
  } while (0)

static const char* kSrc = R"(
__global__ void inc(float* x) { x[get_global_id(0)] += 1.0f; }
__global__ void saxpy(const float* a, const float* x, float* y) {
  long long i = get_global_id(0); y[i] = a[0] * x[i] + y[i]; }
__global__ void count(float* x, int* c) { if (get_global_id(0) == 0) c[0] += 1; }
__global__ void incc(float* x, int* c) { x[get_global_id(0)] += 1.0f; }
__global__ void groupsum(const float* x, float* out) {
  __shared__ float s[64];
  int l = (int)get_local_id(0);
  s[l] = x[get_global_id(0)];
  __syncthreads();
  for (int w = 32; w > 0; w >>= 1) { if (l < w) s[l] += s[l + w]; __syncthreads(); }
  if (l == 0) out[get_global_id(0) / 64] = s[0];
}
)";

static ArraySpec spec(uint64_t uid, void* p, uint64_t bytes, int esize) {
  ArraySpec a;
  a.uid = uid;
  a.host = p;
  a.bytes = bytes;
  a.elem_size = esize;
  return a;
}

static void test_balancer() {
  for (int trial = 0; trial < 50; ++trial) {
    const int n = 2 + trial % 5;
    const long long step = 64 * (1 + trial % 3), total = step * (40 + trial);
    std::vector<std::vector<double>> hist(kHistoryDepth, std::vector<double>(n, 0.0));
    std::vector<long long> r;
    initial_split(n, true, hist, total, r, step);
    for (int call = 0; call < 20; ++call) {
      std::vector<double> bench(n);
      for (int i = 0; i < n; ++i) bench[i] = static_cast<double>(r[i]) / (1.0 + i) + 0.1;
      load_balance(bench, true, hist, total, r, step);
      CHECK(std::accumulate(r.begin(), r.end(), 0LL) == total);
      for (long long x : r) CHECK(x % step == 0 && x >= 0);
    }
  }
}

static void test_jit() {
  auto ks = parse_kernels(kSrc);
  CHECK(ks.size() == 5);
  for (auto& k : ks) {
    if (k.name == "saxpy") CHECK(k.arity == 3);
    if (k.name == "inc") CHECK(k.arity == 1);
  }
  const std::string g = gpu_rewrite(kSrc);
  CHECK(g.find("__cek_off") != std::string::npos);
  CHECK(is_opencl_dialect("__kernel void k(__global float* a) { a[0] = 1; }"));
}

static void test_cores() {
  DeviceInfo cpu = cpu_info(2);
  std::vector<DeviceInfo> devs = {cpu, cpu};  // two logical CPU devices
  CoresConfig cfg;
  Cores cores(devs, kSrc, cfg);
  CHECK(cores.error_code() == 0);
  if (cores.error_code()) {
    std::fprintf(stderr, "%s\n", cores.error_message().c_str());
    return;
  }
  const long long n = 64 * 64;
  std::vector<float> a(1, 3.0f), x(n), y(n, 1.0f);
  for (long long i = 0; i < n; ++i) x[i] = static_cast<float>(i % 97);

  // plain + event pipeline + driver pipeline
  for (int mode = 0; mode < 3; ++mode) {
    std::fill(y.begin(), y.end(), 1.0f);
    ComputeCall c;
    c.kernels = {"saxpy"};
    ArraySpec sa = spec(1, a.data(), 4, 4), sx = spec(2, x.data(), n * 4, 4), sy = spec(3, y.data(), n * 4, 4);
    sa.write = false;
    sx.write = false;
    sx.partial = mode > 0;
    sy.partial = mode > 0;
    c.arrays = {sa, sx, sy};
    c.global_range = n;
    c.local_range = 64;
    c.compute_id = 10 + mode;
    c.pipeline = mode > 0;
    c.pipeline_event = mode == 1;
    c.blobs = 4;
    cores.record_schedule = true;
    for (int it = 0; it < 3; ++it) {
      std::fill(y.begin(), y.end(), 1.0f);
      cores.compute(c);
    }
    for (long long i = 0; i < n; ++i) CHECK(y[i] == 3.0f * x[i] + 1.0f);
  }
  CHECK(!cores.schedule().empty());

  // repeat + sync kernel
  {
    std::vector<float> v(1024, 0.0f);
    std::vector<int> cnt(1, 0);
    ComputeCall c;
    c.kernels = {"incc"};
    c.repeats = 5;
    c.repeat_kernel = "count";
    ArraySpec sv = spec(4, v.data(), v.size() * 4, 4), sc = spec(5, cnt.data(), 4, 4);
    sc.write_all = true;
    c.arrays = {sv, sc};
    c.global_range = 1024;
    c.local_range = 64;
    c.compute_id = 20;
    cores.compute(c);
    for (float f : v) CHECK(f == 5.0f);
  }

  // barrier kernel (fibers) with per-group outputs
  {
    std::vector<float> v(n), out(n / 64, 0.0f);
    for (long long i = 0; i < n; ++i) v[i] = 1.0f;
    ComputeCall c;
    c.kernels = {"groupsum"};
    ArraySpec sv = spec(6, v.data(), n * 4, 4), so = spec(7, out.data(), out.size() * 4, 4);
    sv.write = false;
    so.read = false;
    so.epg = 1;
    c.arrays = {sv, so};
    c.global_range = n;
    c.local_range = 64;
    c.compute_id = 21;
    cores.compute(c);
    for (float f : out) CHECK(f == 64.0f);
  }

  // arity mismatch is rejected before any launch
  {
    std::vector<float> v(256, 0.0f);
    std::vector<int> cnt(1, 0);
    ComputeCall c;
    c.kernels = {"inc"};
    ArraySpec sv = spec(8, v.data(), 1024, 4), sc = spec(9, cnt.data(), 4, 4);
    sc.write = false;
    c.arrays = {sv, sc};
    c.global_range = 256;
    c.local_range = 64;
    bool threw = false;
    try {
      cores.compute(c);
    } catch (const std::exception&) {
      threw = true;
    }
    CHECK(threw);
  }

  // failover: device 1 fails once, its slice is recomputed on device 0
  {
    std::vector<float> v(1024, 0.0f);
    ComputeCall c;
    c.kernels = {"inc"};
    c.arrays = {spec(10, v.data(), v.size() * 4, 4)};
    c.global_range = 1024;
    c.local_range = 64;
    c.compute_id = 22;
    cores.auto_failover = true;
    cores.inject_failure(1, 1);
    cores.compute(c);
    for (float f : v) CHECK(f == 1.0f);
    CHECK(!cores.device_enabled(1) && cores.failovers() == 1);
    cores.set_device_enabled(1, true);
  }
  cores.finish();
}

int main() {
  test_balancer();
  test_jit();
  test_cores();
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("runtime self-test passed\n");
  return 0;
}
