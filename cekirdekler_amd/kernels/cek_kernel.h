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

// Output tile of tile index t (work-group order; C is stored tile-major in
// this order).  P == 0: grouped order — GM tile rows per group, the tiles of
// a group walk down its rows first, so the work-groups an XCD runs at once
// share A and B K-slices through its L2.  P > 0: square shells of P row
// panels (host-resident streaming, Cores event pipeline with explicit
// blobs): shell s = R_s (row panel s × column panels 0..s) then C_s (row
// panels 0..s-1 × column panel s), each block in grouped order — every tile
// of shell s needs only panels 0..s of A and B, and a shell's C is one
// contiguous range.  With pm × pn tiles per panel pair, shells 0..s-1 hold
// pm·pn·s² tiles.
__device__ __forceinline__ void cek_grouped(long long t, int rows, int cols, int GM, int& tm, int& tn) {
  const int per_group = GM * cols, grp = (int)(t / per_group), first = grp * GM;
  const int gsz = min(rows - first, GM), in_g = (int)(t % per_group);
  tm = first + in_g % gsz;
  tn = in_g / gsz;
}

__device__ __forceinline__ void cek_tile_coords(long long t, int ntm, int ntn, int GM, int P, int& tm, int& tn) {
  if (P <= 0) {
    cek_grouped(t, ntm, ntn, GM, tm, tn);
    return;
  }
  const int pm = ntm / P, pn = ntn / P;
  const long long per = (long long)pm * pn;
  int s = (int)__builtin_sqrtf((float)(t / per));
  while ((long long)(s + 1) * (s + 1) * per <= t) ++s;
  while ((long long)s * s * per > t) --s;
  long long r = t - (long long)s * s * per;
  const long long r_tiles = (long long)pm * (s + 1) * pn;
  if (r < r_tiles) {  // R_s: row panel s, columns 0 .. (s+1)·pn
    cek_grouped(r, pm, (s + 1) * pn, GM, tm, tn);
    tm += s * pm;
  } else {  // C_s: rows 0 .. s·pm, column panel s
    cek_grouped(r - r_tiles, s * pm, pn, GM, tm, tn);
    tn += s * pn;
  }
}
