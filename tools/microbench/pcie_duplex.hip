// PCIe duplex microbenchmark: 256 MiB host→device and 256 MiB device→host
// at the same time on two streams, by each combination of mechanism:
//   sdma  hipMemcpyAsync (pinned host memory; the runtime picks SDMA or a blit)
//   kern  a copy kernel that reads / writes the mapped host pages directly
// Build: hipcc --offload-arch=gfx950 -O3 -o pcie_duplex pcie_duplex.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void copy16(const u32x4* __restrict__ src, u32x4* __restrict__ dst, long long n16) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (; i < n16; i += stride) dst[i] = src[i];
}

static const size_t kBytes = 256ull << 20;

static void launch_copy(void* dst, const void* src, hipStream_t s, int groups) {
  const long long n16 = kBytes / 16;
  copy16<<<groups, 256, 0, s>>>(static_cast<const u32x4*>(src), static_cast<u32x4*>(dst), n16);
  CHECK(hipGetLastError());
}

int main() {
  void *d_up, *d_dn, *h_up, *h_dn;
  CHECK(hipMalloc(&d_up, kBytes));
  CHECK(hipMalloc(&d_dn, kBytes));
  CHECK(hipHostMalloc(&h_up, kBytes, hipHostMallocMapped | hipHostMallocPortable));
  CHECK(hipHostMalloc(&h_dn, kBytes, hipHostMallocMapped | hipHostMallocPortable));
  CHECK(hipMemset(d_dn, 1, kBytes));
  std::fill_n(static_cast<char*>(h_up), kBytes, 2);
  void *hd_up, *hd_dn;  // device views of the host pages
  CHECK(hipHostGetDevicePointer(&hd_up, h_up, 0));
  CHECK(hipHostGetDevicePointer(&hd_dn, h_dn, 0));
  hipStream_t s_up, s_dn;
  CHECK(hipStreamCreateWithFlags(&s_up, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s_dn, hipStreamNonBlocking));

  // modes: 0 none, 1 sdma (hipMemcpyAsync), 2 kernel with G groups
  struct Case {
    const char* name;
    int up, dn, groups;
  };
  const Case cases[] = {
      {"up sdma", 1, 0, 0},          {"dn sdma", 0, 1, 0},          {"up kern64", 2, 0, 64},
      {"up kern256", 2, 0, 256},     {"dn kern64", 0, 2, 64},       {"dn kern256", 0, 2, 256},
      {"both sdma/sdma", 1, 1, 0},   {"both sdma/kern64", 1, 2, 64}, {"both sdma/kern256", 1, 2, 256},
      {"both kern64/sdma", 2, 1, 64}, {"both kern256/sdma", 2, 1, 256}, {"both kern128/kern128", 2, 2, 128},
  };
  for (const Case& c : cases) {
    std::vector<double> ms;
    for (int rep = 0; rep < 6; ++rep) {
      CHECK(hipDeviceSynchronize());
      auto t0 = std::chrono::steady_clock::now();
      if (c.up == 1) CHECK(hipMemcpyAsync(d_up, h_up, kBytes, hipMemcpyHostToDevice, s_up));
      if (c.up == 2) launch_copy(d_up, hd_up, s_up, c.groups);
      if (c.dn == 1) CHECK(hipMemcpyAsync(h_dn, d_dn, kBytes, hipMemcpyDeviceToHost, s_dn));
      if (c.dn == 2) launch_copy(hd_dn, d_dn, s_dn, c.groups);
      CHECK(hipStreamSynchronize(s_up));
      CHECK(hipStreamSynchronize(s_dn));
      ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    const double moved = kBytes * double((c.up ? 1 : 0) + (c.dn ? 1 : 0));
    std::printf("%-22s %8.3f ms  %6.1f GB/s aggregate\n", c.name, med, moved / (med * 1e-3) / 1e9);
  }
  // D2H by hipMemcpyAsync into each kind of pinned host memory, as one copy
  // and as 16 copies of 16 MiB
  {
    void* h_def = nullptr;
    CHECK(hipHostMalloc(&h_def, kBytes, hipHostMallocDefault));
    void* h_reg = std::malloc(kBytes);
    std::fill_n(static_cast<char*>(h_reg), kBytes, 0);
    CHECK(hipHostRegister(h_reg, kBytes, hipHostRegisterDefault));
    struct Kind {
      const char* name;
      void* p;
    };
    const Kind kinds[] = {{"hipHostMalloc(mapped|portable)", h_dn}, {"hipHostMalloc(default)", h_def},
                          {"hipHostRegister(malloc)", h_reg}};
    for (const Kind& k : kinds)
      for (int pieces : {1, 16}) {
        std::vector<double> ms;
        for (int rep = 0; rep < 6; ++rep) {
          CHECK(hipDeviceSynchronize());
          auto t0 = std::chrono::steady_clock::now();
          const size_t piece = kBytes / pieces;
          for (int i = 0; i < pieces; ++i)
            CHECK(hipMemcpyAsync(static_cast<char*>(k.p) + i * piece, static_cast<char*>(d_dn) + i * piece, piece,
                                 hipMemcpyDeviceToHost, s_dn));
          CHECK(hipStreamSynchronize(s_dn));
          ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2];
        std::printf("d2h %-32s x%-2d %8.3f ms  %6.1f GB/s\n", k.name, pieces, med, kBytes / (med * 1e-3) / 1e9);
      }
    // both directions, hipMemcpyAsync, into / from default-flag and registered memory
    for (const Kind& k : kinds) {
      std::vector<double> ms;
      for (int rep = 0; rep < 6; ++rep) {
        CHECK(hipDeviceSynchronize());
        auto t0 = std::chrono::steady_clock::now();
        CHECK(hipMemcpyAsync(d_up, h_up, kBytes, hipMemcpyHostToDevice, s_up));
        CHECK(hipMemcpyAsync(k.p, d_dn, kBytes, hipMemcpyDeviceToHost, s_dn));
        CHECK(hipStreamSynchronize(s_up));
        CHECK(hipStreamSynchronize(s_dn));
        ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
      }
      std::sort(ms.begin(), ms.end());
      const double med = ms[ms.size() / 2];
      std::printf("both sdma up, d2h into %-32s %8.3f ms  %6.1f GB/s aggregate\n", k.name, med,
                  2.0 * kBytes / (med * 1e-3) / 1e9);
    }
    CHECK(hipHostUnregister(h_reg));
    std::free(h_reg);
    CHECK(hipHostFree(h_def));
  }
  // correctness of the kernel paths
  CHECK(hipMemset(d_up, 0, kBytes));
  launch_copy(d_up, hd_up, s_up, 64);
  CHECK(hipStreamSynchronize(s_up));
  std::vector<char> back(4096);
  CHECK(hipMemcpy(back.data(), static_cast<char*>(d_up) + kBytes - 4096, 4096, hipMemcpyDeviceToHost));
  bool ok = std::all_of(back.begin(), back.end(), [](char v) { return v == 2; });
  launch_copy(hd_dn, d_dn, s_dn, 64);
  CHECK(hipStreamSynchronize(s_dn));
  ok = ok && static_cast<char*>(h_dn)[kBytes - 1] == 1;
  std::printf("kernel copies %s\n", ok ? "ok" : "WRONG");
  CHECK(hipFree(d_up));
  CHECK(hipFree(d_dn));
  CHECK(hipHostFree(h_up));
  CHECK(hipHostFree(h_dn));
  return ok ? 0 : 1;
}
