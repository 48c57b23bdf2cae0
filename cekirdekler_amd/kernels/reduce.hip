// Sum reduction: each work-group of L threads reduces L·8 floats (two
// dwordx4 loads per lane) with a 64-lane DPP/shuffle tree per wave, then one
// LDS exchange across waves; partials[group] gets the block sum (absolute
// group id, so the device slices of a range-partitioned call write disjoint
// partials).  cek_reduce_sum_f32_final folds a partials array in one group.
#include "cek_kernel.h"

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

extern "C" __global__ __launch_bounds__(256) void cek_reduce_sum_f32(const float4* x, float* partials,
                                                                   CEK_HIDDEN) {
  __shared__ float ws[4];
  const long long g = cek_global_group_id();
  const long long base = g * (long long)blockDim.x * 2 + threadIdx.x;
  const float4 a = x[base], b = x[base + blockDim.x];
  float v = (a.x + a.y) + (a.z + a.w) + (b.x + b.y) + (b.z + b.w);
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) ws[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += ws[i];
    partials[g] = s;
  }
}

// Same, 32 floats per lane (8 dwordx4 loads in flight per lane, 8192 floats
// per work-group): a quarter of the groups and partials, and deeper memory
// parallelism per wave for HBM-bound sums.
extern "C" __global__ __launch_bounds__(256) void cek_reduce_sum_f32_x32(const float4* x, float* partials,
                                                                       CEK_HIDDEN) {
  __shared__ float ws[4];
  const long long g = cek_global_group_id();
  const long long base = g * (long long)blockDim.x * 8 + threadIdx.x;
  const f32x4* xv = reinterpret_cast<const f32x4*>(x);
  f32x4 r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = __builtin_nontemporal_load(&xv[base + (long long)k * blockDim.x]);
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) v += (r[k].x + r[k].y) + (r[k].z + r[k].w);
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) ws[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += ws[i];
    partials[g] = s;
  }
}

// n = sizes[0] partials -> out[0]; launched with one group (global = local)
extern "C" __global__ __launch_bounds__(256) void cek_reduce_sum_f32_final(const int* sizes,
                                                                         const float* partials,
                                                                         float* out, CEK_HIDDEN) {
  __shared__ float ws[4];
  const int n = sizes[0];
  float v = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) v += partials[i];
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) ws[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += ws[i];
    out[0] = s;
  }
}
