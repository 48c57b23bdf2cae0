#pragma once

namespace cek {

// The reference wave example's single-threaded scalar CPU loop
// (Kamera.cs:208-218); base / normals / out are n packed Vector3 (x, y, z).
void wave_reference_scalar(const float* base, const float* normals, float* out, long long n, float ctr, float t);

}  // namespace cek
