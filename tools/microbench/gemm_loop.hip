// Main-loop probe of the production bf16 GEMM kernels, outside the runtime:
// times cek_sgemm_bf16_256x256pb (8192³) and an 8-GPU slice kernel
// (1024 × 8192 × 8192) with hipEvents: argv[3] = sw (256x256pbw, default),
// sh (256x256pbh) or ss (256x256pbs).
// Built twice by tools/microbench/build_gemm_loop.sh:
//   gemm_loop      the kernels as shipped
//   gemm_loop_l2   -DCEK_KTILE: every stage load re-reads K-tiles 0/1 of its
//                  tile (the operand stream hits L2), same instruction stream
// The difference between the two is what operand latency/bandwidth costs the
// ping-pong schedule.
#ifdef CEK_PROBE_L2
#define CEK_KTILE(ks, kt) ((ks) + ((kt) & 1))
#endif
#ifdef CEK_PROBE_TS
// timeline build: work-group thread 0 stamps the 100 MHz realtime counter at
// entry (0), prologue done (1), main loop done (2), hand-over steps (3, 4) and
// after its C stores have completed (5); slot 6 holds the XCD id
#include <hip/hip_runtime.h>
__device__ unsigned long long cek_ts[4096 * 8];
__device__ unsigned long long cek_clk[4096 * 8];  // s_memtime (shader clock) at the same points
__device__ __forceinline__ void cek_stamp(int k) {
  if (threadIdx.x == 0) {
    cek_ts[blockIdx.x * 8 + k] = __builtin_amdgcn_s_memrealtime();
    cek_clk[blockIdx.x * 8 + k] = __builtin_amdgcn_s_memtime();
    if (k == 0) {
      unsigned x;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
      cek_ts[blockIdx.x * 8 + 6] = x & 15u;
    }
  }
}
#define CEK_TS(k) cek_stamp(k)
#define CEK_TS_END                                \
  do {                                            \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
    __syncthreads();                              \
    cek_stamp(5);                                 \
  } while (0)
#endif
#include "../../cekirdekler_amd/kernels/sgemm_bf16.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

static float time_kernel(void (*launch)(hipStream_t), int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) launch(0);
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) launch(0);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

static int *g_dims, *g_dims_slice, *g_cnt;
static uint16_t *g_A, *g_B;
static float *g_C, *g_W;
static const int N = 8192, SLICE = 1024;

static void launch_full(hipStream_t s) {
  hipLaunchKernelGGL(cek_sgemm_bf16_256x256pb, dim3((N / 256) * (N / 256)), dim3(512), 0, s, g_dims, g_A, g_B, g_C,
                     0LL, (long long)(N / 256) * (N / 256) * 512);
}

static char g_slice = 'w';  // w: pb_sw, h: pb_sh, s: pb_ss
static void launch_slice(hipStream_t s) {
  const int tiles = (SLICE / 256) * (N / 256);
  if (g_slice == 'h')
    hipLaunchKernelGGL(cek_sgemm_bf16_256x256pb_sh, dim3(2 * tiles), dim3(512), 0, s, g_dims_slice, g_A, g_B, g_C, g_W,
                       g_cnt, 0LL, (long long)2 * tiles * 512);
  else if (g_slice == 's')
    hipLaunchKernelGGL(cek_sgemm_bf16_256x256pb_ss, dim3(2 * tiles), dim3(512), 0, s, g_dims_slice, g_A, g_B, g_C, g_W,
                       g_cnt, 0LL, (long long)2 * tiles * 512);
  else
    hipLaunchKernelGGL(cek_sgemm_bf16_256x256pb_sw, dim3(2 * tiles), dim3(512), 0, s, g_dims_slice, g_A, g_B, g_C, g_W,
                       g_cnt, 0LL, (long long)2 * tiles * 512);
}

#ifdef CEK_PROBE_TS
// host copy of cek_xcd_remap (kernels/cek_kernel.h)
static unsigned host_xcd_remap(unsigned b, unsigned nwg) {
  const unsigned xcd = b & 7u, q = nwg >> 3, r = nwg & 7u;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

static double pct(std::vector<double> v, double q) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[(size_t)(q * (v.size() - 1))];
}

// one launch, then per-stamp distributions (µs after the earliest entry) for
// the owner (even u) and helper (odd u) work-groups
static void timeline(const char* name, void (*launch)(hipStream_t), int grid) {
  std::vector<unsigned long long> ts((size_t)grid * 8, 0);
  CK(hipMemcpyToSymbol(HIP_SYMBOL(cek_ts), ts.data(), ts.size() * 8));
  launch(0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpyFromSymbol(ts.data(), HIP_SYMBOL(cek_ts), ts.size() * 8));
  std::vector<unsigned long long> clk((size_t)grid * 8, 0);
  CK(hipMemcpyFromSymbol(clk.data(), HIP_SYMBOL(cek_clk), clk.size() * 8));
  unsigned long long t0 = ~0ull, tend = 0;
  for (int b = 0; b < grid; ++b) {
    t0 = std::min(t0, ts[b * 8]);
    for (int k = 1; k < 6; ++k) tend = std::max(tend, ts[b * 8 + k]);
  }
  printf("{\"timeline\": \"%s\", \"span_us\": %.2f", name, (tend - t0) / 100.0);
  for (int role = 0; role < 2; ++role) {
    for (int k = 0; k < 6; ++k) {
      std::vector<double> v;
      for (int b = 0; b < grid; ++b) {
        const unsigned u = host_xcd_remap((unsigned)b, (unsigned)grid);
        if ((int)(u & 1) != role || !ts[b * 8 + k]) continue;
        v.push_back((ts[b * 8 + k] - t0) / 100.0);
      }
      if (v.empty()) continue;
      printf(", \"%s_t%d\": [%.2f, %.2f, %.2f, %.2f]", role ? "odd" : "even", k, pct(v, 0), pct(v, 0.5), pct(v, 0.9),
             pct(v, 1.0));
    }
  }
  printf("}\n");
  // per XCD: work-groups run, median main-loop time (t2 - t1) and median end (t5 or t4)
  printf("{\"timeline_by_xcd\": \"%s\"", name);
  for (int x = 0; x < 8; ++x) {
    std::vector<double> loop, end, ghz;
    for (int b = 0; b < grid; ++b) {
      if ((int)ts[b * 8 + 6] != x || !ts[b * 8 + 2]) continue;
      loop.push_back((ts[b * 8 + 2] - ts[b * 8 + 1]) / 100.0);
      // s_memtime ticks per µs over the main loop (the realtime counter is 100 MHz)
      ghz.push_back((double)(clk[b * 8 + 2] - clk[b * 8 + 1]) / ((ts[b * 8 + 2] - ts[b * 8 + 1]) * 10.0));
      const unsigned long long e = ts[b * 8 + 5] ? ts[b * 8 + 5] : ts[b * 8 + 4];
      end.push_back((e - t0) / 100.0);
    }
    printf(", \"xcd%d\": {\"wgs\": %zu, \"loop_us\": [%.2f, %.2f, %.2f], \"end_us\": [%.2f, %.2f], \"memtime_ghz\": [%.3f, %.3f, %.3f]}",
           x, loop.size(), pct(loop, 0), pct(loop, 0.5), pct(loop, 1.0), pct(end, 0.5), pct(end, 1.0), pct(ghz, 0),
           pct(ghz, 0.5), pct(ghz, 1.0));
  }
  printf("}\n");
}
#endif

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const int shift = argc > 2 ? atoi(argv[2]) : 4;  // the slice helper's K-tile deficit (dims[5])
  if (argc > 3) g_slice = argv[3][1];  // "sw" / "sh" / "ss"
  const char* slice_name = g_slice == 'h' ? "256x256pbh" : g_slice == 's' ? "256x256pbs" : "256x256pbw";
  const size_t nab = (size_t)N * N;
  CK(hipMalloc(&g_A, nab * 2));
  CK(hipMalloc(&g_B, nab * 2));
  CK(hipMalloc(&g_C, nab * 4));
  CK(hipMalloc(&g_W, (size_t)SLICE * N * 4));
  const int tiles_slice = (SLICE / 256) * (N / 256);
  CK(hipMalloc(&g_cnt, (4 * tiles_slice + 1) * sizeof(int)));
  CK(hipMemset(g_cnt, 0, (4 * tiles_slice + 1) * sizeof(int)));
  // uniform bf16 values in [-1, 1): 0x3f80 bias + random mantissa, random sign
  std::vector<uint16_t> h(nab);
  unsigned x = 12345u;
  for (size_t i = 0; i < nab; ++i) {
    x = x * 1664525u + 1013904223u;
    h[i] = (uint16_t)(0x3e00u + ((x >> 9) & 0x1ffu)) | (uint16_t)((x >> 31) << 15);
  }
  CK(hipMemcpy(g_A, h.data(), nab * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(g_B, h.data(), nab * 2, hipMemcpyHostToDevice));
  int dims[8] = {N, N, N, 4, 1, 0, 0, 0};
  int dims_s[8] = {SLICE, N, N, 4, 2, shift, 0, 0};
  CK(hipMalloc(&g_dims, sizeof dims));
  CK(hipMalloc(&g_dims_slice, sizeof dims_s));
  CK(hipMemcpy(g_dims, dims, sizeof dims, hipMemcpyHostToDevice));
  CK(hipMemcpy(g_dims_slice, dims_s, sizeof dims_s, hipMemcpyHostToDevice));
#ifdef CEK_PROBE_L2
  const char* variant = "l2_operands";
#else
  const char* variant = "shipped";
#endif
  for (int round = 0; round < 2; ++round) {
    float ms = time_kernel(launch_full, reps);
    printf("{\"variant\": \"%s\", \"kernel\": \"256x256pb\", \"shape\": \"8192^3\", \"ms\": %.4f, \"tflops\": %.1f}\n",
           variant, ms, 2.0 * N * N * (double)N / ms / 1e9);
    ms = time_kernel(launch_slice, reps);
    printf("{\"variant\": \"%s\", \"kernel\": \"%s\", \"shift\": %d, \"shape\": \"1024x8192x8192\", \"ms\": %.4f, \"tflops\": %.1f}\n",
           variant, slice_name, shift, ms, 2.0 * SLICE * N * (double)N / ms / 1e9);
  }
#ifdef CEK_PROBE_TS
  timeline("256x256pb 8192^3", launch_full, (N / 256) * (N / 256));
  char tl[64];
  snprintf(tl, sizeof tl, "%s 1024x8192x8192", slice_name);
  timeline(tl, launch_slice, 2 * tiles_slice);
#endif
  int err = 0;
  CK(hipMemcpy(&err, g_cnt + 4 * tiles_slice, sizeof(int), hipMemcpyDeviceToHost));
  printf("{\"spin_timeouts\": %d}\n", err);
  return 0;
}
