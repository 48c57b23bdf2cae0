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
  const f32x2 cra = {x0 + x * dx, x0 + (x + 1) * dx};
  const f32x2 crb = {x0 + (x + 2) * dx, x0 + (x + 3) * dx};
  const f32x2 cic = {ci, ci};
  f32x2 zra = {0.f, 0.f}, zia = {0.f, 0.f}, zrb = {0.f, 0.f}, zib = {0.f, 0.f};
  // Escape counting without per-iteration branches: a pixel's count grows
  // while |z|² <= 4; once |z| > max(2, |c|) it never returns (inf/NaN compare
  // false), so the count equals the first escape iteration.  The escape
  // test that ends the loop runs once per 8 unrolled iterations.
  int na0 = 0, na1 = 0, nb0 = 0, nb1 = 0;
  for (int it = 0; it < max_iter; it += 8) {
    f32x2 ma, mb;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const f32x2 zr2a = zra * zra, zi2a = zia * zia, zr2b = zrb * zrb, zi2b = zib * zib;
      ma = zr2a + zi2a;
      mb = zr2b + zi2b;
      na0 += ma.x <= 4.f;
      na1 += ma.y <= 4.f;
      nb0 += mb.x <= 4.f;
      nb1 += mb.y <= 4.f;
      const f32x2 ta = zra * zia, tb = zrb * zib;
      zia = ta + ta + cic;
      zib = tb + tb + cic;
      zra = zr2a - zi2a + cra;
      zrb = zr2b - zi2b + crb;
    }
    if (!(ma.x <= 4.f) && !(ma.y <= 4.f) && !(mb.x <= 4.f) && !(mb.y <= 4.f)) break;
  }
  out[q] = make_int4(min(na0, max_iter), min(na1, max_iter), min(nb0, max_iter), min(nb1, max_iter));
}
