// VALU issue-rate microbenchmark for gfx950: FLOP/s of dependent-chain FMA
// streams, scalar (v_fma_f32) vs packed (v_pk_fma_f32), by the number of
// independent chains per wave and the number of waves per SIMD.
// build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int CH>
__global__ __launch_bounds__(256) void scalar_fma(float* out, int iters, float k) {
  float a[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) a[c] = threadIdx.x * 1e-3f + c;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = __builtin_fmaf(a[c], k, 0.5f);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CH>
__global__ __launch_bounds__(256) void packed_fma(float* out, int iters, float k) {
  f32x2 a[CH];
  const f32x2 kk = {k, k}, h = {0.5f, 0.5f};
#pragma unroll
  for (int c = 0; c < CH; ++c) a[c] = f32x2{threadIdx.x * 1e-3f + c, threadIdx.x * 2e-3f + c};
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = __builtin_elementwise_fma(a[c], kk, h);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += a[c].x + a[c].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static void run(const char* name, K kern, int chains, int lanes_per_op, int waves_per_simd, float* out) {
  const int iters = 4096;
  const int blocks = 256 * waves_per_simd;  // 256 threads = 4 waves = 1 per SIMD
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  ms /= 5;
  const double flop = 2.0 * lanes_per_op * chains * (double)iters * blocks * 256;
  printf("{\"kernel\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, \"tflops\": %.1f}\n", name,
         chains, waves_per_simd, ms, flop / ms / 1e9);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 256 * 16 * sizeof(float));
  for (int w : {1, 2, 4, 8}) {
    run("scalar_fma", scalar_fma<1>, 1, 1, w, out);
    run("scalar_fma", scalar_fma<4>, 4, 1, w, out);
    run("scalar_fma", scalar_fma<8>, 8, 1, w, out);
    run("packed_fma", packed_fma<1>, 1, 2, w, out);
    run("packed_fma", packed_fma<4>, 4, 2, w, out);
    run("packed_fma", packed_fma<8>, 8, 2, w, out);
  }
  hipFree(out);
  return 0;
}
