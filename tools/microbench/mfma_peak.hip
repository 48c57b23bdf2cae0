// Matrix-core ceiling on gfx950 under a full-chip load: back-to-back
// v_mfma_f32_16x16x32_bf16 from registers (no memory in the loop), with the
// GEMM kernel's register shape (8×4 accumulators per wave, 512-thread
// work-groups, one per CU) — the rate the 256x256pb main loop is measured
// against, at whatever clock the chip holds under that load.
// build: hipcc --offload-arch=gfx950 -O3 mfma_peak.hip -o mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <int FM, int FN, bool TOGGLE>
__global__ __launch_bounds__(512) void mfma_loop(float* out, int iters) {
  f32x4 acc[FM][FN];
  bf16x8 a[FM], b[FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
    for (int e = 0; e < 8; ++e) a[i][e] = (short)(0x3c00 + threadIdx.x + i + e);
#pragma unroll
  for (int j = 0; j < FN; ++j)
    for (int e = 0; e < 8; ++e) b[j][e] = (short)(0x3c00 + threadIdx.x + 3 * j + e);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  unsigned x = threadIdx.x * 2654435761u;
  for (int it = 0; it < iters; ++it) {
    if constexpr (TOGGLE) {
      // fresh mantissa bits every iteration (operand switching activity of
      // a real GEMM; the exponents stay put)
      x = x * 1664525u + 1013904223u;
      const short m = (short)(x & 0x007f);
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] ^= m;
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] ^= (short)(m << 1);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* out;
  const int blocks = 256 * 4;
  (void)hipMalloc(&out, (size_t)blocks * 512 * sizeof(float));
  const int iters = 2048;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int r = 0; r < 6; ++r) {
    auto kern = r < 3 ? mfma_loop<8, 4, false> : mfma_loop<8, 4, true>;
    kern<<<blocks, 512>>>(out, iters);
    (void)hipEventRecord(a);
    for (int k = 0; k < 5; ++k) kern<<<blocks, 512>>>(out, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    // per wave per iteration: 2·8·4 MFMAs of 16·16·32·2 FLOP
    const double flop = 2.0 * 8 * 4 * 16 * 16 * 32 * 2.0 * iters * blocks * 8;
    printf("{\"kernel\": \"mfma_16x16x32_bf16_regs\", \"operands\": \"%s\", \"ms\": %.4f, \"tflops\": %.1f}\n",
           r < 3 ? "constant" : "toggled", ms, flop / ms / 1e9);
  }
  (void)hipFree(out);
  return 0;
}
