// All-pairs gravitational N-body on CDNA4 (BASELINE config "N-body 1M
// particles"; the reference's test workload is the 2-D O(n²) force loop of
// Tester.cs:7726-7743).
//
// pos  : float4 {x, y, z, m} per body     acc : float4 {ax, ay, az, 0}
// params: {softening², G, n, 0}
//
// One work item = TWO bodies (i and i + half the group's span) so the inner
// loop issues packed f32 ops (v_pk_fma_f32 / v_pk_mul_f32: 2 interactions
// per VALU issue); the j loop streams the bodies through LDS in tiles of
// blockDim bodies — every lane of a wave reads the same LDS address (a
// broadcast, no bank conflicts) — and uses the hardware rsqrt.  20 FLOP per
// interaction is the accounting convention.  Work items are absolute
// (__cek_off), so the body range is load-balanced across devices like any
// other compute().
#include "cek_kernel.h"

extern "C" __global__ __launch_bounds__(256) void cek_nbody_f32(const float4* __restrict__ pos,
                                                              float4* __restrict__ vel,
                                                              float4* __restrict__ acc,
                                                              const float* __restrict__ params,
                                                              CEK_HIDDEN) {
  (void)vel;
  __shared__ float4 tile[256];
  const float eps2 = params[0], gconst = params[1];
  const int n = (int)params[2];
  // work item w handles bodies 2·(w - lane-group base) layout: i0 = base + l, i1 = base + l + L
  const long long w = cek_global_id();
  const int L = blockDim.x;
  const long long grp = w / L, l = w % L;
  const long long i0 = grp * 2 * L + l, i1 = i0 + L;
  const float4 p0 = pos[i0], p1 = pos[i1];
  f32x2 px = {p0.x, p1.x}, py = {p0.y, p1.y}, pz = {p0.z, p1.z};
  f32x2 ax = {0.f, 0.f}, ay = {0.f, 0.f}, az = {0.f, 0.f};
  const f32x2 e2 = {eps2, eps2};
  for (int j0 = 0; j0 < n; j0 += L) {
    __syncthreads();
    tile[threadIdx.x] = pos[j0 + threadIdx.x];
    __syncthreads();
#pragma unroll 8
    for (int j = 0; j < L; ++j) {
      const float4 q = tile[j];
      const f32x2 qx = {q.x, q.x}, qy = {q.y, q.y}, qz = {q.z, q.z}, qm = {q.w, q.w};
      const f32x2 dx = qx - px, dy = qy - py, dz = qz - pz;
      const f32x2 r2 = dx * dx + dy * dy + dz * dz + e2;
      f32x2 inv = {__builtin_amdgcn_rsqf(r2.x), __builtin_amdgcn_rsqf(r2.y)};
      const f32x2 s = qm * inv * inv * inv;
      ax += dx * s;
      ay += dy * s;
      az += dz * s;
    }
  }
  acc[i0] = make_float4(gconst * ax.x, gconst * ay.x, gconst * az.x, 0.f);
  acc[i1] = make_float4(gconst * ax.y, gconst * ay.y, gconst * az.y, 0.f);
}

// Leapfrog kick-drift: v += a·dt; x += v·dt for the same two bodies per
// work item as cek_nbody_f32, so both kernels run in one compute() on the
// same balanced range (same argument list).  params: {softening², G, n, dt}
__device__ __forceinline__ void kick_drift(float4* pos, float4* vel, const float4* acc, long long i,
                                           float dt) {
  float4 p = pos[i], v = vel[i];
  const float4 a = acc[i];
  v.x += a.x * dt;
  v.y += a.y * dt;
  v.z += a.z * dt;
  p.x += v.x * dt;
  p.y += v.y * dt;
  p.z += v.z * dt;
  pos[i] = p;
  vel[i] = v;
}

extern "C" __global__ __launch_bounds__(256) void cek_nbody_integrate_f32(float4* __restrict__ pos,
                                                                       float4* __restrict__ vel,
                                                                       const float4* __restrict__ acc,
                                                                       const float* __restrict__ params,
                                                                       CEK_HIDDEN) {
  const long long w = cek_global_id();
  const int L = blockDim.x;
  const long long i0 = (w / L) * 2 * L + (w % L);
  const float dt = params[3];
  kick_drift(pos, vel, acc, i0, dt);
  kick_drift(pos, vel, acc, i0 + L, dt);
}

// Per-group kinetic energy diagnostic: energy[g] = Σ ½ m |v|² over the
// group's 2·L bodies (same work-item mapping as above).
extern "C" __global__ __launch_bounds__(256) void cek_nbody_energy_f32(const float4* __restrict__ pos,
                                                                     const float4* __restrict__ vel,
                                                                     float* __restrict__ energy,
                                                                     CEK_HIDDEN) {
  __shared__ float ws[4];
  const long long w = cek_global_id();
  const int L = blockDim.x;
  const long long i0 = (w / L) * 2 * L + (w % L), i1 = i0 + L;
  const float4 p0 = pos[i0], v0 = vel[i0], p1 = pos[i1], v1 = vel[i1];
  float e = 0.5f * p0.w * (v0.x * v0.x + v0.y * v0.y + v0.z * v0.z) +
            0.5f * p1.w * (v1.x * v1.x + v1.y * v1.y + v1.z * v1.z);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = e;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += ws[k];
    energy[cek_global_group_id()] = s;
  }
}
