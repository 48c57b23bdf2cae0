// Shared definitions for the AOT (hipcc --genco) CDNA4 kernel library.
//
// Every library kernel follows the runtime's launch ABI: array parameters
// first, then the two hidden parameters appended by the JIT rewrite
// (`long long __cek_off, long long __cek_gsize`), so library kernels and
// user kernel strings are launched identically by Worker::launch and take
// part in range partitioning / load balancing like any user kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CEK_HIDDEN long long __cek_off, long long __cek_gsize
#define cek_global_id() ((long long)blockIdx.x * (long long)blockDim.x + (long long)threadIdx.x + __cek_off)
#define cek_global_group_id() ((long long)blockIdx.x + __cek_off / (long long)blockDim.x)

// Bijective XCD-aware remap of the device-local block index (guide T1):
// consecutive remapped ids land on the same XCD (blocks b, b+8, ... share one
// under round-robin dispatch), so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ unsigned cek_xcd_remap(unsigned b, unsigned nwg) {
  const unsigned xcd = b & 7u, q = nwg >> 3, r = nwg & 7u;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void glb_cvoid;
