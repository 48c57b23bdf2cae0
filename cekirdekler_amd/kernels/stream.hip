// Streaming kernels (HBM-bound): SAXPY, byte copy (the reference's "test"
// kernel, Tester.cs:35-38), vector add (Tester.cs:7819-7830).  Each work
// item handles `elements per work item` = 4 floats (16-B dwordx4 accesses,
// Guideline 13); byte copy moves 16 B per work item.
#include "cek_kernel.h"

// y = a[0] * x + y       (4 floats per work item)
extern "C" __global__ void cek_saxpy_f32(const float* a, const float4* x, float4* y, CEK_HIDDEN) {
  const long long i = cek_global_id();
  const float s = a[0];
  float4 xv = x[i], yv = y[i];
  yv.x = s * xv.x + yv.x;
  yv.y = s * xv.y + yv.y;
  yv.z = s * xv.z + yv.z;
  yv.w = s * xv.w + yv.w;
  y[i] = yv;
}

// dst = src, 16 bytes per work item
extern "C" __global__ void cek_copy_u8(const uint4* src, uint4* dst, CEK_HIDDEN) {
  const long long i = cek_global_id();
  dst[i] = src[i];
}

// c = a + b               (4 floats per work item)
extern "C" __global__ void cek_vec_add_f32(const float4* a, const float4* b, float4* c, CEK_HIDDEN) {
  const long long i = cek_global_id();
  float4 x = a[i], y = b[i];
  c[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
}
