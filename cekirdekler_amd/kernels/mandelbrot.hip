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

// ---------------------------------------------------------------------------
// Packed escape count: every operation of the iteration is a packed-f32
// instruction over a PAIR of pixels (a wave64 VALU instruction costs ~4
// issue cycles packed or not), including the count: each counted iteration
// adds
//     t = clamp(2^20 · (4 − |z|²), 0, 1)        (one v_pk_fma_f32 … clamp)
// which is 1 while |z|² ≤ 4 − 2^-20 and 0 once the pixel escaped (±inf and NaN
// clamp to 0), so the float sum is the escape iteration.  Only pixels whose
// |z|² lands within 2^-20 of 4 can differ by one iteration from a strict
// "|z|² > 4" test.
__device__ __forceinline__ f32x2 pk_fma_clamp(f32x2 a, f32x2 b, f32x2 c) {
  f32x2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 clamp" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// 8×16 pixel block per wave, one packed pair (2 horizontally adjacent
// pixels) per lane: a smaller block keeps the lanes' escape times closer
// (87 % vs 85 % busy lanes on the 4096² view) at half the per-wave ILP,
// which the one-wave work-groups make up with occupancy.  Bands of 8 rows.
extern "C" __global__ __launch_bounds__(64) void cek_mandelbrot_blk8_f32(const float* view, const int* size,
                                                                       int2* out, CEK_HIDDEN) {
  const long long w = cek_global_id();
  const int W = size[0], max_iter = size[2];
  const long long band_items = 4LL * W;  // 8 rows × W px / 2 px per work item
  const long long band = w / band_items;
  const int q = (int)(w - band * band_items);
  const int blk = q >> 6, l = q & 63;
  const int row = (int)band * 8 + (l >> 3), col = blk * 16 + (l & 7) * 2;
  const float x0 = view[0], y0 = view[1], dx = view[2], dy = view[3];
  const float ci = y0 + row * dy;
  const f32x2 cr = {x0 + col * dx, x0 + (col + 1) * dx}, civ = {ci, ci};
  f32x2 zr = {0.f, 0.f}, zi = {0.f, 0.f}, cnt = {0.f, 0.f}, t = {1.f, 1.f};
  const f32x2 nbig = {-1048576.f, -1048576.f}, cbig = {4194304.f, 4194304.f}, two = {2.f, 2.f};
  for (int it = 0; it < max_iter; it += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const f32x2 zi2 = zi * zi;
      const f32x2 m = __builtin_elementwise_fma(zr, zr, zi2);
      t = pk_fma_clamp(m, nbig, cbig);
      cnt += t;
      const f32x2 tz = zr * zi;
      zr = __builtin_elementwise_fma(zr, zr, -zi2) + cr;
      zi = __builtin_elementwise_fma(tz, two, civ);
    }
    if (t.x < 0.5f && t.y < 0.5f) break;
  }
  out[((long long)row * W + col) >> 1] = make_int2(min((int)(cnt.x + 0.5f), max_iter), min((int)(cnt.y + 0.5f), max_iter));
}

// Deferred escape counting with cheap bookkeeping ("blk8h"): the 8-iteration
// blocks run without the per-iteration escape count; at each block's end a pixel
// whose |z|² is still <= 4 records that z and the iteration (it + 8) as its
// last known non-escaped point; an escaped pixel stops recording (escape is
// monotone, inf/NaN fail `m <= 4`).  No start-of-block copies and no "already
// escaped?" tests: 2 compares + 6 selects per block instead of 19 VALU ops.
// The counting pass from the last recorded z adds the non-escaped iterations
// of the escape block; a pixel that never escaped ends at ex = max_iter.
extern "C" __global__ __launch_bounds__(64) void cek_mandelbrot_blk8h_f32(const float* view, const int* size,
                                                                        int2* out, CEK_HIDDEN) {
  const long long w = cek_global_id();
  const int W = size[0], max_iter = size[2];
  const long long band_items = 4LL * W;
  const long long band = w / band_items;
  const int q = (int)(w - band * band_items);
  const int blk = q >> 6, l = q & 63;
  const int row = (int)band * 8 + (l >> 3), col = blk * 16 + (l & 7) * 2;
  const float x0 = view[0], y0 = view[1], dx = view[2], dy = view[3];
  const float ci = y0 + row * dy;
  const f32x2 cr = {x0 + col * dx, x0 + (col + 1) * dx}, civ = {ci, ci};
  const f32x2 two = {2.f, 2.f};
  f32x2 zr = {0.f, 0.f}, zi = {0.f, 0.f};
  f32x2 fr = {0.f, 0.f}, fi = {0.f, 0.f};  // last z with |z|² <= 4 at a block boundary
  int ex = 0, ey = 0;                      // its iteration
  for (int it = 8; it <= max_iter; it += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const f32x2 zi2 = zi * zi;
      const f32x2 tz = zr * zi;
      zr = __builtin_elementwise_fma(zr, zr, cr) - zi2;
      zi = __builtin_elementwise_fma(tz, two, civ);
    }
    const f32x2 m = __builtin_elementwise_fma(zr, zr, zi * zi);
    const bool kx = m.x <= 4.f, ky = m.y <= 4.f;
    if (kx) {
      fr.x = zr.x;
      fi.x = zi.x;
      ex = it;
    }
    if (ky) {
      fr.y = zr.y;
      fi.y = zi.y;
      ey = it;
    }
    if (!kx && !ky) break;
  }
  const f32x2 nbig = {-1048576.f, -1048576.f}, cbig = {4194304.f, 4194304.f};
  f32x2 cnt = {0.f, 0.f};
  zr = fr;
  zi = fi;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const f32x2 zi2 = zi * zi;
    const f32x2 m = __builtin_elementwise_fma(zr, zr, zi2);
    cnt += pk_fma_clamp(m, nbig, cbig);
    const f32x2 tz = zr * zi;
    zr = __builtin_elementwise_fma(zr, zr, cr) - zi2;
    zi = __builtin_elementwise_fma(tz, two, civ);
  }
  out[((long long)row * W + col) >> 1] =
      make_int2(min(ex + (int)(cnt.x + 0.5f), max_iter), min(ey + (int)(cnt.y + 0.5f), max_iter));
}

// blk8h with fewer instructions per useful iteration ("blk8k"):
//  * the iteration is 4 packed instructions instead of 5 —
//      t = zr·zi;  a = fma(zr, zr, cr);  zr' = fma(−zi, zi, a);  zi' = fma(t, 2, ci)
//    (blk8h computed zi² separately because blk8 shared it with |z|²; the
//    8-iteration blocks need |z|² only at the block's end);
//  * the first block counts every iteration (blk8's exact count), so a wave
//    whose pixels all escape within 8 iterations — most of the exterior —
//    stores its counts and ends without the counting pass;
//  * a wave none of whose pixels escaped (set interior) skips the counting
//    pass (wave-uniform branch).
// Same 8×16 block per one-wave work-group and block-end bookkeeping as blk8h.
extern "C" __global__ __launch_bounds__(64) void cek_mandelbrot_blk8k_f32(const float* view, const int* size,
                                                                        int2* out, CEK_HIDDEN) {
  const long long w = cek_global_id();
  const int W = size[0], max_iter = size[2];
  const long long band_items = 4LL * W;
  const long long band = w / band_items;
  const int q = (int)(w - band * band_items);
  const int blk = q >> 6, l = q & 63;
  const int row = (int)band * 8 + (l >> 3), col = blk * 16 + (l & 7) * 2;
  const float x0 = view[0], y0 = view[1], dx = view[2], dy = view[3];
  const float ci = y0 + row * dy;
  const f32x2 cr = {x0 + col * dx, x0 + (col + 1) * dx}, civ = {ci, ci};
  const f32x2 two = {2.f, 2.f};
  const f32x2 nbig = {-1048576.f, -1048576.f}, cbig = {4194304.f, 4194304.f};
  const long long o = ((long long)row * W + col) >> 1;
  f32x2 zr = {0.f, 0.f}, zi = {0.f, 0.f};
  // block 1, counted exactly (blk8's iteration)
  f32x2 cnt = {0.f, 0.f}, tc = {1.f, 1.f};
  const int first = min(8, max_iter);
  for (int u = 0; u < first; ++u) {
    const f32x2 zi2 = zi * zi;
    const f32x2 m = __builtin_elementwise_fma(zr, zr, zi2);
    tc = pk_fma_clamp(m, nbig, cbig);
    cnt += tc;
    const f32x2 tz = zr * zi;
    zr = __builtin_elementwise_fma(zr, zr, -zi2) + cr;
    zi = __builtin_elementwise_fma(tz, two, civ);
  }
  // escaped within block 1 ⇔ the last counted step was already escaped
  const bool dx1 = tc.x < 0.5f, dy1 = tc.y < 0.5f;
  const bool wave_done = __all(dx1 && dy1) || first >= max_iter;
  if (wave_done) {
    out[o] = make_int2(min((int)(cnt.x + 0.5f), max_iter), min((int)(cnt.y + 0.5f), max_iter));
    return;
  }
  // blk8h's bookkeeping from iteration 8 on: the last z with |z|² <= 4 at a
  // block end, and its iteration; a pixel escaped in block 1 keeps (0, z=0)
  // and is recounted from the start by the counting pass
  f32x2 fr = {0.f, 0.f}, fi = {0.f, 0.f};
  int ex = 0, ey = 0;
  if (!dx1) {
    fr.x = zr.x;
    fi.x = zi.x;
    ex = 8;
  }
  if (!dy1) {
    fr.y = zr.y;
    fi.y = zi.y;
    ey = 8;
  }
  bool kx = !dx1, ky = !dy1;
  for (int it = 16; it <= max_iter && (kx || ky); it += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const f32x2 tz = zr * zi;
      const f32x2 a = __builtin_elementwise_fma(zr, zr, cr);
      zr = __builtin_elementwise_fma(-zi, zi, a);
      zi = __builtin_elementwise_fma(tz, two, civ);
    }
    const f32x2 m = __builtin_elementwise_fma(zr, zr, zi * zi);
    kx = m.x <= 4.f;
    ky = m.y <= 4.f;
    if (kx) {
      fr.x = zr.x;
      fi.x = zi.x;
      ex = it;
    }
    if (ky) {
      fr.y = zr.y;
      fi.y = zi.y;
      ey = it;
    }
  }
  // counting pass over the escape block, skipped when no pixel of the wave
  // escaped (every lane reached max_iter)
  cnt = f32x2{0.f, 0.f};
  if (!__all(ex >= max_iter && ey >= max_iter)) {
    zr = fr;
    zi = fi;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const f32x2 zi2 = zi * zi;
      const f32x2 m = __builtin_elementwise_fma(zr, zr, zi2);
      cnt += pk_fma_clamp(m, nbig, cbig);
      const f32x2 tz = zr * zi;
      const f32x2 a = __builtin_elementwise_fma(zr, zr, cr);
      zr = a - zi2;
      zi = __builtin_elementwise_fma(tz, two, civ);
    }
  }
  out[o] = make_int2(min(ex + (int)(cnt.x + 0.5f), max_iter), min(ey + (int)(cnt.y + 0.5f), max_iter));
}

// blk8k with fewer instructions per wave ("blk8m": 16-iteration blocks from
// iteration 16; "blk8t": 32-iteration blocks from iteration 32, with the
// iteration and counting streams ordered by hand):
//  * wave-uniform prologue: the wave's band and block come from one scalar
//    32-bit division of the work-group index (one-wave work-groups; the
//    range offset is a multiple of 64), not a per-lane 64-bit division;
//  * block 1 counted exactly from z1 = c, with a wave exit after 4 iterations
//    as well as after 8 (half the exterior waves are done by then);
//  * from iteration S the blocks are BIG iterations long: the block-end
//    bookkeeping (|z|², 2 compares, 6 selects) is paid per BIG iterations;
//  * the loop runs wave-uniformly (exit when no lane is still bounded at a
//    block end), so its counter stays scalar;
//  * the counting pass runs in chunks of 8 counted iterations from the last
//    bounded block end and stops as soon as every lane has escaped, is
//    interior, or has reached max_iter.
// A lane escaped in block 1 keeps (0, z = 0) and is recounted from the start.
// Measured: profiles/mandelbrot_r3.md.

// wave-uniform votes combined from the compare masks on the scalar unit
// (a vote on a combined bool costs a VALU select and compare)
__device__ __forceinline__ unsigned long long ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ bool all_lanes(unsigned long long m) { return m == __builtin_amdgcn_read_exec(); }

// N iterations of the 4-instruction step in one hand-ordered stream:
//   a = zr·zr + cr;  t = zr·zi;  zr' = −zi·zi + a;  zi' = 2t + ci
// Every result is read two instructions after it is written, so the packed
// FP32 read-after-write wait state is filled by the other chain; the
// compiler's order (t, a, zr', zi') puts two s_nop per iteration in a
// wave's stream.  One s_nop pads each end against the surrounding code.
#define CEK_MANDEL_STEP                                                    \
  "v_pk_fma_f32 %2, %0, %0, %4\n\t"                                       \
  "v_pk_mul_f32 %3, %0, %1\n\t"                                           \
  "v_pk_fma_f32 %0, %1, %1, %2 neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"         \
  "v_pk_fma_f32 %1, %3, 2.0, %5 op_sel_hi:[1,0,1]\n\t"
#define CEK_MANDEL_STEP4 CEK_MANDEL_STEP CEK_MANDEL_STEP CEK_MANDEL_STEP CEK_MANDEL_STEP
template <int N>
__device__ __forceinline__ void mandel_steps_asm(f32x2& zr, f32x2& zi, const f32x2 cr, const f32x2 civ) {
  static_assert(N == 8 || N == 16 || N == 32, "8, 16 or 32 steps");
  f32x2 a, t;
  if constexpr (N == 8)
    asm volatile("s_nop 0\n\t" CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 "s_nop 0"
                 : "+v"(zr), "+v"(zi), "=&v"(a), "=&v"(t) : "v"(cr), "v"(civ));
  else if constexpr (N == 16)
    asm volatile("s_nop 0\n\t" CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 "s_nop 0"
                 : "+v"(zr), "+v"(zi), "=&v"(a), "=&v"(t) : "v"(cr), "v"(civ));
  else
    asm volatile("s_nop 0\n\t" CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 CEK_MANDEL_STEP4
                 CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 "s_nop 0"
                 : "+v"(zr), "+v"(zi), "=&v"(a), "=&v"(t) : "v"(cr), "v"(civ));
}

// N steps from (sr, si) into (dr, di), leaving (sr, si) intact: the first
// step reads the source pair and writes the destination pair, the other
// N − 1 run in place on the destination (same hand order and spacing as
// above).  The all-bounded fast path ping-pongs between two pairs with it, so
// the block's start z stays available as the checkpoint without a copy.
#define CEK_MANDEL_STEP_FROM                                               \
  "v_pk_fma_f32 %2, %6, %6, %4\n\t"                                       \
  "v_pk_mul_f32 %3, %6, %7\n\t"                                           \
  "v_pk_fma_f32 %0, %7, %7, %2 neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"         \
  "v_pk_fma_f32 %1, %3, 2.0, %5 op_sel_hi:[1,0,1]\n\t"
#define CEK_MANDEL_STEP2 CEK_MANDEL_STEP CEK_MANDEL_STEP
#define CEK_MANDEL_STEP7 CEK_MANDEL_STEP4 CEK_MANDEL_STEP2 CEK_MANDEL_STEP
template <int N>
__device__ __forceinline__ void mandel_steps_from_asm(const f32x2 sr, const f32x2 si, f32x2& dr, f32x2& di,
                                                      const f32x2 cr, const f32x2 civ) {
  static_assert(N == 8 || N == 32, "8 or 32 steps");
  f32x2 a, t;
  if constexpr (N == 8)
    asm volatile("s_nop 0\n\t" CEK_MANDEL_STEP_FROM CEK_MANDEL_STEP7 "s_nop 0"
                 : "=&v"(dr), "=&v"(di), "=&v"(a), "=&v"(t) : "v"(cr), "v"(civ), "v"(sr), "v"(si));
  else
    asm volatile("s_nop 0\n\t" CEK_MANDEL_STEP_FROM CEK_MANDEL_STEP7 CEK_MANDEL_STEP4 CEK_MANDEL_STEP4
                 CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 CEK_MANDEL_STEP4 "s_nop 0"
                 : "=&v"(dr), "=&v"(di), "=&v"(a), "=&v"(t) : "v"(cr), "v"(civ), "v"(sr), "v"(si));
}

// N counted iterations (|z|² checked and counted every step), ordered so
// that every result is read at least two instructions after it is written:
//   q = zi·zi; t = zr·zi; m = zr·zr + q; a = zr·zr + cr; tc = clamp(m·nbig + cbig);
//   zr = a − q; zi = 2t + ci; cnt += tc
#define CEK_MANDEL_COUNT                                                   \
  "v_pk_mul_f32 %4, %1, %1\n\t"                                           \
  "v_pk_mul_f32 %5, %0, %1\n\t"                                           \
  "v_pk_fma_f32 %6, %0, %0, %4\n\t"                                       \
  "v_pk_fma_f32 %7, %0, %0, %8\n\t"                                       \
  "v_pk_fma_f32 %3, %6, %10, %11 clamp\n\t"                               \
  "v_pk_add_f32 %0, %7, %4 neg_lo:[0,1] neg_hi:[0,1]\n\t"                 \
  "v_pk_fma_f32 %1, %5, 2.0, %9 op_sel_hi:[1,0,1]\n\t"                    \
  "v_pk_add_f32 %2, %2, %3\n\t"
template <int N>
__device__ __forceinline__ void mandel_counted_asm(f32x2& zr, f32x2& zi, f32x2& cnt, f32x2& tc, const f32x2 cr,
                                                   const f32x2 civ, const f32x2 nbig, const f32x2 cbig) {
  static_assert(N == 3 || N == 4 || N == 8, "3, 4 or 8 counted steps");
  f32x2 q, t, m, a;
#define CEK_MANDEL_COUNT_ARGS                                              \
  : "+v"(zr), "+v"(zi), "+v"(cnt), "=&v"(tc), "=&v"(q), "=&v"(t), "=&v"(m), "=&v"(a) \
  : "v"(cr), "v"(civ), "v"(nbig), "v"(cbig)
  if constexpr (N == 3)
    asm volatile("s_nop 0\n\t" CEK_MANDEL_COUNT CEK_MANDEL_COUNT CEK_MANDEL_COUNT "s_nop 0" CEK_MANDEL_COUNT_ARGS);
  else if constexpr (N == 4)
    asm volatile("s_nop 0\n\t" CEK_MANDEL_COUNT CEK_MANDEL_COUNT CEK_MANDEL_COUNT CEK_MANDEL_COUNT
                 "s_nop 0" CEK_MANDEL_COUNT_ARGS);
  else
    asm volatile("s_nop 0\n\t" CEK_MANDEL_COUNT CEK_MANDEL_COUNT CEK_MANDEL_COUNT CEK_MANDEL_COUNT
                 CEK_MANDEL_COUNT CEK_MANDEL_COUNT CEK_MANDEL_COUNT CEK_MANDEL_COUNT "s_nop 0" CEK_MANDEL_COUNT_ARGS);
#undef CEK_MANDEL_COUNT_ARGS
}

// FAST: 0 = per-lane checkpoints after every block; 1 = none while every
// lane is bounded (blk8y)
template <int BIG, int S, bool ASM, int FAST = 0>
__device__ __forceinline__ int2 mandel_blk8_core(const f32x2 cr, const f32x2 civ, const int max_iter) {
  static_assert(BIG % 8 == 0 && S % 8 == 0 && S >= 8, "block lengths are multiples of 8");
  static_assert(!FAST || ASM, "the all-bounded fast path uses the hand-ordered blocks");
  const f32x2 two = {2.f, 2.f};
  const f32x2 nbig = {-1048576.f, -1048576.f}, cbig = {4194304.f, 4194304.f};
  f32x2 zr = {0.f, 0.f}, zi = {0.f, 0.f}, cnt = {0.f, 0.f}, tc = {1.f, 1.f};
  auto counted = [&]() {
    const f32x2 zi2 = zi * zi;
    const f32x2 m = __builtin_elementwise_fma(zr, zr, zi2);
    tc = pk_fma_clamp(m, nbig, cbig);
    cnt += tc;
    const f32x2 tz = zr * zi;
    zr = __builtin_elementwise_fma(zr, zr, cr) - zi2;
    zi = __builtin_elementwise_fma(tz, two, civ);
  };
  if (max_iter <= 8) {  // uniform: the whole range is one counted block
    for (int u = 0; u < max_iter; ++u) counted();
    return make_int2((int)(cnt.x + 0.5f), (int)(cnt.y + 0.5f));
  }
  // z0 = 0 is always bounded and z1 = c: start counted from there
  zr = cr;
  zi = civ;
  cnt = f32x2{1.f, 1.f};
  if constexpr (ASM) {
    mandel_counted_asm<3>(zr, zi, cnt, tc, cr, civ, nbig, cbig);
  } else {
#pragma unroll
    for (int u = 1; u < 4; ++u) counted();
  }
  if (all_lanes(ballot(tc.x < 0.5f) & ballot(tc.y < 0.5f))) return make_int2((int)(cnt.x + 0.5f), (int)(cnt.y + 0.5f));
  if constexpr (ASM) {
    mandel_counted_asm<4>(zr, zi, cnt, tc, cr, civ, nbig, cbig);
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) counted();
  }
  const bool dx1 = tc.x < 0.5f, dy1 = tc.y < 0.5f;
  if (all_lanes(ballot(dx1) & ballot(dy1))) return make_int2((int)(cnt.x + 0.5f), (int)(cnt.y + 0.5f));
  f32x2 fr = {0.f, 0.f}, fi = {0.f, 0.f};
  int ex = 0, ey = 0;
  if (!dx1) {
    fr.x = zr.x;
    fi.x = zi.x;
    ex = 8;
  }
  if (!dy1) {
    fr.y = zr.y;
    fi.y = zi.y;
    ey = 8;
  }
  auto block_end = [&](int it) -> bool {  // true while some lane is still bounded
    const f32x2 m = __builtin_elementwise_fma(zr, zr, zi * zi);
    const bool kx = m.x <= 4.f, ky = m.y <= 4.f;
    if (kx) {
      fr.x = zr.x;
      fi.x = zi.x;
      ex = it;
    }
    if (ky) {
      fr.y = zr.y;
      fi.y = zi.y;
      ey = it;
    }
    return (ballot(kx) | ballot(ky)) != 0;
  };
  auto step = [&]() {
    const f32x2 tz = zr * zi;
    const f32x2 a = __builtin_elementwise_fma(zr, zr, cr);
    zr = __builtin_elementwise_fma(-zi, zi, a);
    zi = __builtin_elementwise_fma(tz, two, civ);
  };
  int it = 8;
  bool live = true;
  if constexpr (FAST == 1) {
    // While EVERY lane is still bounded (set-interior waves: ~90 % of the
    // work on views centred on the set) no lane needs a checkpoint of its
    // own: the blocks alternate between two z pairs, so the block's start z
    // is the checkpoint without a copy, and the block start is every lane's
    // last bounded iteration.  Per block that is |z|² and two compares
    // instead of |z|², two compares, a move and six selects.  The first
    // escape hands per-lane checkpoints to the general loops below, which go
    // on from the same block boundary.
    if ((ballot(dx1) | ballot(dy1)) == 0) {
      // the loop carries (ar, ai) only; (br, bi) lives between its halves
      f32x2 ar = zr, ai = zi, br, bi;
      bool rem = false, second = false;
      for (;;) {
        int L = it < S ? 8 : BIG;
        if (it + L > max_iter) {
          rem = true;
          break;
        }
        if (L == 8)
          mandel_steps_from_asm<8>(ar, ai, br, bi, cr, civ);
        else
          mandel_steps_from_asm<BIG>(ar, ai, br, bi, cr, civ);
        f32x2 m = __builtin_elementwise_fma(br, br, bi * bi);
        it += L;
        if (!all_lanes(ballot(m.x <= 4.f) & ballot(m.y <= 4.f))) break;
        L = it < S ? 8 : BIG;
        if (it + L > max_iter) {
          rem = second = true;
          break;
        }
        if (L == 8)
          mandel_steps_from_asm<8>(br, bi, ar, ai, cr, civ);
        else
          mandel_steps_from_asm<BIG>(br, bi, ar, ai, cr, civ);
        m = __builtin_elementwise_fma(ar, ar, ai * ai);
        it += L;
        if (!all_lanes(ballot(m.x <= 4.f) & ballot(m.y <= 4.f))) {
          second = true;
          break;
        }
      }
      // `second`: the last block ran from (br, bi) into (ar, ai)
      const f32x2 sr = second ? br : ar, si = second ? bi : ai;  // the block's start z
      const f32x2 dr = second ? ar : br, di = second ? ai : bi;  // its end z
      if (rem) {  // every lane bounded at `it` (= the block start here); the rest is counted below
        fr = zr = second ? br : ar;  // the z every lane has at `it`
        fi = zi = second ? bi : ai;
        ex = ey = it;
        live = false;
      } else {  // the first escapes: per-lane checkpoints from here on
        const int L = (it - 8) < S ? 8 : BIG;  // the length of the block that just ran
        const f32x2 m = __builtin_elementwise_fma(dr, dr, di * di);
        const bool kx = m.x <= 4.f, ky = m.y <= 4.f;
        fr.x = kx ? dr.x : sr.x;
        fi.x = kx ? di.x : si.x;
        ex = kx ? it : it - L;
        fr.y = ky ? dr.y : sr.y;
        fi.y = ky ? di.y : si.y;
        ey = ky ? it : it - L;
        zr = dr;
        zi = di;
        live = (ballot(kx) | ballot(ky)) != 0;
      }
    }
  }
  for (; live && it < S && it + 8 <= max_iter; it += 8) {
    if constexpr (ASM) {
      mandel_steps_asm<8>(zr, zi, cr, civ);
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) step();
    }
    live = block_end(it + 8);
  }
  for (; live && it + BIG <= max_iter; it += BIG) {
    if constexpr (ASM) {
      mandel_steps_asm<BIG>(zr, zi, cr, civ);
    } else {
#pragma unroll
      for (int u = 0; u < BIG; ++u) step();
    }
    live = block_end(it + BIG);
  }
  // counting pass from the last bounded block end; the remainder after the
  // loop is shorter than BIG, so BIG counted iterations always suffice
  cnt = f32x2{0.f, 0.f};
  if (!all_lanes(ballot(ex >= max_iter) & ballot(ey >= max_iter))) {
    zr = fr;
    zi = fi;
    for (int k = 0; k < BIG; k += 8) {
      if constexpr (ASM) {
        mandel_counted_asm<8>(zr, zi, cnt, tc, cr, civ, nbig, cbig);
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) counted();
      }
      const unsigned long long doneX = ballot(tc.x < 0.5f) | ballot(ex + k + 8 >= max_iter);
      const unsigned long long doneY = ballot(tc.y < 0.5f) | ballot(ey + k + 8 >= max_iter);
      if (all_lanes(doneX & doneY)) break;
    }
  }
  return make_int2(min(ex + (int)(cnt.x + 0.5f), max_iter), min(ey + (int)(cnt.y + 0.5f), max_iter));
}

// one 8×16 block of an 8-row band per one-wave work-group.  CENTER: the
// launch's bands run from its middle band outwards (middle, middle − 1,
// middle + 1, …), a longest-first order for views centred on the set: the
// set-interior waves (~20× an exterior wave's work) start early and the
// cheap exterior bands fill the end of the launch instead of a tail of
// interior waves sharing a few SIMDs.  The order stays inside the launch's
// own bands (device ranges and pipeline chunks are whole bands), so every
// write stays in the launch's range.
// FASTPRO: a shorter serial prologue per wave.  The view and size loads
// are issued together (one wait instead of two dependent ones), and a
// power-of-two blocks-per-band count (any width 16·2^k, e.g. 4096) maps the
// work-group index with shifts instead of three scalar integer divisions
// (~100 dependent SALU instructions per wave in the compiler's expansion);
// other widths keep the division.
template <int BIG, int S, bool ASM, bool CENTER = false, bool FASTPRO = false, int FAST = 0>
__device__ __forceinline__ void mandel_blk8m(const float* view, const int* size, int2* out, long long off) {
  const int W = size[0], max_iter = size[2];
  const float x0 = view[0], y0 = view[1], dx = view[2], dy = view[3];
  if constexpr (FASTPRO) asm volatile("" ::"s"(W), "s"(max_iter), "s"(x0), "s"(y0), "s"(dx), "s"(dy));
  const int bpb = W >> 4;  // blocks per band
  int band, blk;
  if (FASTPRO && (bpb & (bpb - 1)) == 0) {
    const int sh = __builtin_ctz((unsigned)bpb);
    if constexpr (CENTER) {
      const int b0 = (int)(off >> (6 + sh));
      const int nbl = (int)gridDim.x >> sh;  // bands in this launch
      const int kb = (int)blockIdx.x >> sh;
      blk = (int)blockIdx.x & (bpb - 1);
      const int c = nbl >> 1;
      band = b0 + ((kb & 1) ? c - ((kb + 1) >> 1) : c + (kb >> 1));
    } else {
      const int wv = (int)(((long long)blockIdx.x * 64 + off) >> 6);
      band = wv >> sh;
      blk = wv & (bpb - 1);
    }
  } else if constexpr (CENTER) {
    const int b0 = __builtin_amdgcn_readfirstlane((int)((off >> 6) / bpb));
    const int nbl = (int)gridDim.x / bpb;  // bands in this launch
    const int kb = (int)blockIdx.x / bpb;
    blk = (int)blockIdx.x - kb * bpb;
    const int c = nbl >> 1;
    band = b0 + ((kb & 1) ? c - ((kb + 1) >> 1) : c + (kb >> 1));
  } else {
    const int wv = __builtin_amdgcn_readfirstlane((int)(((long long)blockIdx.x * 64 + off) >> 6));
    band = wv / bpb;
    blk = wv - band * bpb;
  }
  const int l = threadIdx.x;
  const int r = l >> 3, c2 = (l & 7) * 2;
  const float ci = y0 + (float)(band * 8 + r) * dy;
  const float crx = x0 + (float)(blk * 16 + c2) * dx;
  const f32x2 cr = {crx, crx + dx}, civ = {ci, ci};
  out[((long long)band * 4 * W + blk * 8) + r * (W >> 1) + (l & 7)] = mandel_blk8_core<BIG, S, ASM, FAST>(cr, civ, max_iter);
}

extern "C" __global__ __launch_bounds__(64) void cek_mandelbrot_blk8m_f32(const float* view, const int* size,
                                                                        int2* out, CEK_HIDDEN) {
  mandel_blk8m<16, 16, false>(view, size, out, __cek_off);
}

extern "C" __global__ __launch_bounds__(64) void cek_mandelbrot_blk8t_f32(const float* view, const int* size,
                                                                        int2* out, CEK_HIDDEN) {
  mandel_blk8m<32, 32, true>(view, size, out, __cek_off);
}

// blk8t with the launch's bands in centre-out order
extern "C" __global__ __launch_bounds__(64) void cek_mandelbrot_blk8u_f32(const float* view, const int* size,
                                                                        int2* out, CEK_HIDDEN) {
  mandel_blk8m<32, 32, true, true>(view, size, out, __cek_off);
}

// blk8u with the short prologue (FASTPRO)
extern "C" __global__ __launch_bounds__(64) void cek_mandelbrot_blk8r_f32(const float* view, const int* size,
                                                                        int2* out, CEK_HIDDEN) {
  mandel_blk8m<32, 32, true, true, true>(view, size, out, __cek_off);
}

// blk8r with the all-bounded fast path (FAST)
extern "C" __global__ __launch_bounds__(64) void cek_mandelbrot_blk8y_f32(const float* view, const int* size,
                                                                        int2* out, CEK_HIDDEN) {
  mandel_blk8m<32, 32, true, true, true, 1>(view, size, out, __cek_off);
}

