// All-pairs gravitational N-body on CDNA4 (BASELINE config "N-body 1M
// particles"; the reference's test workload is the 2-D O(n²) force loop of
// Tester.cs:7726-7743).
//
// cek-flags: -fno-slp-vectorize
//
// pos  : float4 {x, y, z, m} per body     acc : float4 {ax, ay, az, 0}
// params: {softening², G, n, dt}
//
// One work item = B bodies (B = 2 or 4): in workgroup g (256 work items) the
// item with local id l owns bodies g·256·B + k·256 + l, k < B.  The j loop
// streams all bodies through LDS in tiles of 256 (the next tile is fetched
// into registers while the current one is consumed); every lane of a wave
// reads the same LDS address (a broadcast, no bank conflicts) and applies it
// to its B bodies.  The bodies are processed as packed pairs: measured on
// MI355X a wave64 VALU instruction costs ≈4 cycles of SIMD issue whether it
// is v_fma_f32 or v_pk_fma_f32 (PMC: 4.2 cycles per VALU instruction at two
// waves per SIMD), so FP32 peak needs the packed forms.  Per pair of
// interactions: 3 pk_add, 3 pk_fma (r²), 2 v_rsq_f32, 3 pk_mul, 3 pk_fma =
// 14 instructions for 40 FLOP (20 per interaction, the usual convention);
// with two pairs per work item the rsq results are consumed by the other
// pair's independent work instead of s_nop padding.  Auto-SLP is disabled
// (cek-flags) so only these explicit vectors are packed.
// Work items are absolute (__cek_off), so the body range is load-balanced
// across devices like any other compute().
#include "cek_kernel.h"

namespace {

template <int B>
__device__ __forceinline__ long long first_body(long long w) {
  return (w >> 8) * (256LL * B) + (w & 255);
}

template <int B>
__device__ __forceinline__ void nbody_force(const float4* __restrict__ pos, float4* __restrict__ acc,
                                            const float* __restrict__ params, long long off) {
  static_assert(B % 2 == 0, "bodies are processed in packed pairs");
  constexpr int NP = B / 2;  // packed pairs per work item
  __shared__ float4 tile[256];
  if (blockDim.x != 256) return;  // body mapping assumes 256-item groups
  const float eps2 = params[0], gconst = params[1];
  const int n = (int)params[2];
  const int l = threadIdx.x;
  const long long i0 = first_body<B>((long long)blockIdx.x * 256 + l + off);
  // pair p holds bodies k = 2p (.x) and 2p+1 (.y)
  f32x2 px[NP], py[NP], pz[NP], ax[NP], ay[NP], az[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const float4 b0 = pos[i0 + (2 * p) * 256], b1 = pos[i0 + (2 * p + 1) * 256];
    px[p] = f32x2{b0.x, b1.x};
    py[p] = f32x2{b0.y, b1.y};
    pz[p] = f32x2{b0.z, b1.z};
    ax[p] = ay[p] = az[p] = f32x2{0.f, 0.f};
  }
  const f32x2 e2 = {eps2, eps2};
  float4 next = pos[l];
  for (int j0 = 0; j0 < n; j0 += 256) {
    __syncthreads();
    tile[l] = next;
    __syncthreads();
    if (j0 + 256 < n) next = pos[j0 + 256 + l];
#pragma unroll 4
    for (int j = 0; j < 256; ++j) {
      const float4 q = tile[j];
      const f32x2 qx = {q.x, q.x}, qy = {q.y, q.y}, qz = {q.z, q.z}, qm = {q.w, q.w};
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const f32x2 dx = qx - px[p], dy = qy - py[p], dz = qz - pz[p];
        const f32x2 r2 = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy, __builtin_elementwise_fma(dz, dz, e2)));
        const f32x2 inv = {__builtin_amdgcn_rsqf(r2.x), __builtin_amdgcn_rsqf(r2.y)};
        const f32x2 s = (qm * inv) * (inv * inv);
        ax[p] = __builtin_elementwise_fma(dx, s, ax[p]);
        ay[p] = __builtin_elementwise_fma(dy, s, ay[p]);
        az[p] = __builtin_elementwise_fma(dz, s, az[p]);
      }
    }
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    acc[i0 + (2 * p) * 256] = make_float4(gconst * ax[p].x, gconst * ay[p].x, gconst * az[p].x, 0.f);
    acc[i0 + (2 * p + 1) * 256] = make_float4(gconst * ax[p].y, gconst * ay[p].y, gconst * az[p].y, 0.f);
  }
}

// Leapfrog kick-drift: v += a·dt; x += v·dt for the same bodies per work item
// as the force kernel, so both run in one compute() on the same balanced range
// (same argument list).
template <int B>
__device__ __forceinline__ void nbody_integrate(float4* __restrict__ pos, float4* __restrict__ vel,
                                                const float4* __restrict__ acc, const float* __restrict__ params,
                                                long long off) {
  if (blockDim.x != 256) return;
  const long long i0 = first_body<B>((long long)blockIdx.x * 256 + threadIdx.x + off);
  const float dt = params[3];
#pragma unroll
  for (int k = 0; k < B; ++k) {
    const long long i = i0 + k * 256;
    float4 p = pos[i], v = vel[i];
    const float4 a = acc[i];
    v.x = fmaf(a.x, dt, v.x);
    v.y = fmaf(a.y, dt, v.y);
    v.z = fmaf(a.z, dt, v.z);
    p.x = fmaf(v.x, dt, p.x);
    p.y = fmaf(v.y, dt, p.y);
    p.z = fmaf(v.z, dt, p.z);
    pos[i] = p;
    vel[i] = v;
  }
}

// Per-group kinetic energy diagnostic: energy[g] = Σ ½ m |v|² over the
// group's 256·B bodies (same mapping).
template <int B>
__device__ __forceinline__ void nbody_energy(const float4* __restrict__ pos, const float4* __restrict__ vel,
                                             float* __restrict__ energy, long long off) {
  __shared__ float ws[4];
  if (blockDim.x != 256) return;
  const long long i0 = first_body<B>((long long)blockIdx.x * 256 + threadIdx.x + off);
  float e = 0.f;
#pragma unroll
  for (int k = 0; k < B; ++k) {
    const float4 p = pos[i0 + k * 256], v = vel[i0 + k * 256];
    e += 0.5f * p.w * (v.x * v.x + v.y * v.y + v.z * v.z);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = e;
  __syncthreads();
  if (threadIdx.x == 0) energy[blockIdx.x + off / 256] = ws[0] + ws[1] + ws[2] + ws[3];
}

}  // namespace

#define CEK_NBODY_KERNELS(B)                                                                          \
  extern "C" __global__ __launch_bounds__(256) void cek_nbody_f32_b##B(                               \
      const float4* __restrict__ pos, float4* __restrict__ vel, float4* __restrict__ acc,             \
      const float* __restrict__ params, CEK_HIDDEN) {                                                 \
    (void)vel;                                                                                        \
    nbody_force<B>(pos, acc, params, __cek_off);                                                      \
  }                                                                                                   \
  extern "C" __global__ __launch_bounds__(256) void cek_nbody_integrate_f32_b##B(                     \
      float4* __restrict__ pos, float4* __restrict__ vel, const float4* __restrict__ acc,             \
      const float* __restrict__ params, CEK_HIDDEN) {                                                 \
    nbody_integrate<B>(pos, vel, acc, params, __cek_off);                                             \
  }                                                                                                   \
  extern "C" __global__ __launch_bounds__(256) void cek_nbody_energy_f32_b##B(                        \
      const float4* __restrict__ pos, const float4* __restrict__ vel, float* __restrict__ energy,     \
      CEK_HIDDEN) {                                                                                   \
    nbody_energy<B>(pos, vel, energy, __cek_off);                                                     \
  }

CEK_NBODY_KERNELS(2)
CEK_NBODY_KERNELS(4)
