// Mandelbrot escape-time kernel (BASELINE config "Mandelbrot 4096×4096,
// 1×MI355X, event-driven read/compute/write pipeline").
//
// view = {x0, y0, dx, dy}, size = {width, height, max_iter, 0};
// out[p] = iteration count of pixel p (row-major).  Each work item computes
// 4 horizontally adjacent pixels as two packed pairs (v_pk_fma_f32 issue,
// 64 FLOP/clk/SIMD) and stores them as one int4; the iteration loop exits as
// soon as all four of the lane's pixels escaped, the wave as soon as all 64
// lanes did.  8 FLOP per pixel-iteration is the accounting convention.
#include "cek_kernel.h"

extern "C" __global__ __launch_bounds__(256) void cek_mandelbrot_f32(const float* view, const int* size,
                                                                   int4* out, CEK_HIDDEN) {
  const long long q = cek_global_id();  // quad index
  const int W = size[0], max_iter = size[2];
  const long long p0 = q * 4;
  const int y = (int)(p0 / W), x = (int)(p0 % W);
  const float x0 = view[0], y0 = view[1], dx = view[2], dy = view[3];
  const float ci = y0 + y * dy;
  f32x2 cra = {x0 + x * dx, x0 + (x + 1) * dx};
  f32x2 crb = {x0 + (x + 2) * dx, x0 + (x + 3) * dx};
  f32x2 zra = {0.f, 0.f}, zia = {0.f, 0.f}, zrb = {0.f, 0.f}, zib = {0.f, 0.f};
  int na0 = max_iter, na1 = max_iter, nb0 = max_iter, nb1 = max_iter;
  const f32x2 cic = {ci, ci};
  for (int it = 0; it < max_iter; ++it) {
    f32x2 zr2a = zra * zra, zi2a = zia * zia, zr2b = zrb * zrb, zi2b = zib * zib;
    f32x2 ma = zr2a + zi2a, mb = zr2b + zi2b;
    if (ma.x > 4.f && na0 == max_iter) na0 = it;
    if (ma.y > 4.f && na1 == max_iter) na1 = it;
    if (mb.x > 4.f && nb0 == max_iter) nb0 = it;
    if (mb.y > 4.f && nb1 == max_iter) nb1 = it;
    if ((na0 < max_iter) & (na1 < max_iter) & (nb0 < max_iter) & (nb1 < max_iter)) break;
    f32x2 tza = zra * zia, tzb = zrb * zib;
    zia = tza + tza + cic;
    zib = tzb + tzb + cic;
    zra = zr2a - zi2a + cra;
    zrb = zr2b - zi2b + crb;
  }
  out[q] = make_int4(na0, na1, nb0, nb1);
}
