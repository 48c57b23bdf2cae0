// Host loops the reference runs WITHOUT its runtime, kept as baselines for
// the claims it makes against them.
//
// wave_reference_scalar: the CPU-only strategy of the Unity wave example
// (Kamera.cs:208-218, `strategy = true`): one thread, one vertex at a time,
// Vector3 arithmetic with double-precision Math.Sqrt / Math.Sin, which is
// the denominator of the example's "CPU+GPU 3x as fast" comment
// (Kamera.cs:266).  Compiled scalar (no auto-vectorisation, as the .NET JIT
// emits it) so the baseline is the reference's loop, not this framework's
// vectorised CPU device.
#include <cmath>

#include "refloops.h"

namespace cek {

__attribute__((optimize("no-tree-vectorize"))) void wave_reference_scalar(const float* base, const float* normals,
                                                                          float* out, long long n, float ctr,
                                                                          float t) {
  if (n <= 0) return;
  const float x = base[0], y = base[1];
  for (long long i = 0; i < n; ++i) {
    const float* b = base + 3 * i;
    const float* nr = normals + 3 * i;
    float* o = out + 3 * i;
    const float dx = b[0] - x, dy = b[1] - y;
    // C#: (float)Math.Sin(40.0f * t + 100.0f * Math.Sqrt(dx * dx + dy * dy))
    const float s = static_cast<float>(std::sin(static_cast<double>(40.0f * t) +
                                                100.0 * std::sqrt(static_cast<double>(dx * dx + dy * dy))));
    // C#: verticesBase[i] + 0.02f * normals[i] * ctr * s (left to right)
    for (int c = 0; c < 3; ++c) o[c] = b[c] + ((0.02f * nr[c]) * ctr) * s;
  }
}

}  // namespace cek
