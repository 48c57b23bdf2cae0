// Can downloads by a copy kernel run beside a GEMM that fills every CU?
// A CU-masked stream (hipExtStreamCreateWithCUMask) keeps R CUs out of the
// "GEMM" (a busy kernel holding one 512-thread, 160 KiB-LDS work-group per
// CU, like the bf16 tile kernels) and gives them to the D2H copy kernel,
// while the uploads run on SDMA: 256 MiB each way, pinned host memory.
// Reserved CUs are chosen two ways: the last R CU bits, or R bits spread
// evenly over the 256 (every 256/R-th).
// Build: hipcc --offload-arch=gfx950 -O3 -o pcie_cumask pcie_cumask.hip
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

// one 512-thread work-group per CU (160 KiB LDS), FMA-bound for `iters`
__global__ __launch_bounds__(512) void busy(float* out, int iters) {
  __shared__ float lds[40960];
  float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.9999f, d = blockIdx.x * 1e-4f;
  for (int i = 0; i < iters; ++i) {
    a = fmaf(a, b, c);
    d = fmaf(d, c, b);
    b = fmaf(b, 0.99999f, 1e-6f);
  }
  lds[threadIdx.x] = a + d;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = lds[(blockIdx.x * 7) & 511];
}

static const size_t kBytes = 256ull << 20;

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000000;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  void *d_up, *d_dn, *h_up, *h_dn;
  float* d_out;
  CHECK(hipMalloc(&d_up, kBytes));
  CHECK(hipMalloc(&d_dn, kBytes));
  CHECK(hipMalloc(&d_out, 4096 * sizeof(float)));
  CHECK(hipHostMalloc(&h_up, kBytes, hipHostMallocMapped | hipHostMallocPortable));
  CHECK(hipHostMalloc(&h_dn, kBytes, hipHostMallocMapped | hipHostMallocPortable));
  CHECK(hipMemset(d_dn, 1, kBytes));
  std::fill_n(static_cast<char*>(h_up), kBytes, 2);
  void* hd_dn;
  CHECK(hipHostGetDevicePointer(&hd_dn, h_dn, 0));
  hipStream_t s_up;
  CHECK(hipStreamCreateWithFlags(&s_up, hipStreamNonBlocking));

  auto mask_of = [&](int reserved, bool spread, bool want_reserved) {
    std::vector<uint32_t> m((ncu + 31) / 32, 0);
    for (int cu = 0; cu < ncu; ++cu) {
      bool r = spread ? (reserved > 0 && (cu % (ncu / reserved)) == (ncu / reserved) - 1) : cu >= ncu - reserved;
      if (r == want_reserved) m[cu / 32] |= 1u << (cu % 32);
    }
    return m;
  };
  struct Case {
    const char* name;
    int reserved;  // 0: no masks
    bool spread, busy_on, dn_kernel;
  };
  const Case cases[] = {
      {"no busy, up sdma | dn sdma", 0, false, false, false},
      {"no busy, up sdma | dn kern(all CUs)", 0, false, false, true},
      {"busy all CUs, up sdma | dn sdma", 0, false, true, false},
      {"busy all CUs, up sdma | dn kern", 0, false, true, true},
      {"busy 248 CUs, dn kern on last 8", 8, false, true, true},
      {"busy 248 CUs, dn kern on 8 spread", 8, true, true, true},
      {"busy 240 CUs, dn kern on 16 spread", 16, true, true, true},
      {"busy 224 CUs, dn kern on 32 spread", 32, true, true, true},
      {"no busy, dn kern on 8 spread", 8, true, false, true},
      {"busy 248 CUs (8 spread free), up sdma | dn sdma", 8, true, true, false},
  };
  std::printf("{\"cus\": %d, \"iters\": %d, \"cases\": [\n", ncu, iters);
  bool first = true;
  for (const Case& c : cases) {
    for (int rep = 0; rep < 3; ++rep) {
      hipStream_t s_busy, s_dn;
      if (c.reserved > 0) {
        auto mb = mask_of(c.reserved, c.spread, false), md = mask_of(c.reserved, c.spread, true);
        CHECK(hipExtStreamCreateWithCUMask(&s_busy, static_cast<uint32_t>(mb.size()), mb.data()));
        CHECK(hipExtStreamCreateWithCUMask(&s_dn, static_cast<uint32_t>(md.size()), md.data()));
      } else {
        CHECK(hipStreamCreateWithFlags(&s_busy, hipStreamNonBlocking));
        CHECK(hipStreamCreateWithFlags(&s_dn, hipStreamNonBlocking));
      }
      hipEvent_t u0, u1, d0, d1, b1;
      CHECK(hipEventCreate(&u0));
      CHECK(hipEventCreate(&u1));
      CHECK(hipEventCreate(&d0));
      CHECK(hipEventCreate(&d1));
      CHECK(hipEventCreate(&b1));
      CHECK(hipDeviceSynchronize());
      const double t0 = now_ms();
      if (c.busy_on) {
        busy<<<ncu * 2, 512, 0, s_busy>>>(d_out, iters);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(b1, s_busy));
      }
      CHECK(hipEventRecord(u0, s_up));
      CHECK(hipMemcpyAsync(d_up, h_up, kBytes, hipMemcpyHostToDevice, s_up));
      CHECK(hipEventRecord(u1, s_up));
      CHECK(hipEventRecord(d0, s_dn));
      if (c.dn_kernel) {
        const int groups = c.reserved > 0 ? c.reserved * 8 : 64;
        copy16<<<groups, 256, 0, s_dn>>>(static_cast<const u32x4*>(d_dn), static_cast<u32x4*>(hd_dn), kBytes / 16);
        CHECK(hipGetLastError());
      } else {
        CHECK(hipMemcpyAsync(h_dn, d_dn, kBytes, hipMemcpyDeviceToHost, s_dn));
      }
      CHECK(hipEventRecord(d1, s_dn));
      CHECK(hipEventSynchronize(u1));
      CHECK(hipEventSynchronize(d1));
      const double copies_wall = now_ms() - t0;
      float up_ms = 0, dn_ms = 0, busy_ms = -1;
      CHECK(hipEventElapsedTime(&up_ms, u0, u1));
      CHECK(hipEventElapsedTime(&dn_ms, d0, d1));
      CHECK(hipDeviceSynchronize());
      if (c.busy_on) busy_ms = static_cast<float>(now_ms() - t0);
      std::printf("%s{\"case\": \"%s\", \"rep\": %d, \"up_ms\": %.3f, \"dn_ms\": %.3f, \"copies_wall_ms\": %.3f, "
                  "\"busy_wall_ms\": %.3f}",
                  first ? "" : ",\n", c.name, rep, up_ms, dn_ms, copies_wall, busy_ms);
      first = false;
      std::fflush(stdout);
      CHECK(hipEventDestroy(u0));
      CHECK(hipEventDestroy(u1));
      CHECK(hipEventDestroy(d0));
      CHECK(hipEventDestroy(d1));
      CHECK(hipEventDestroy(b1));
      CHECK(hipStreamDestroy(s_busy));
      CHECK(hipStreamDestroy(s_dn));
    }
  }
  std::printf("\n]}\n");
  return 0;
}
