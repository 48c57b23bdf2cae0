// Host-resident GEMM C = A·Bᵀ streamed in square shells over one GPU.
//
// The 1-D event pipeline (Cores::run_event_pipeline) must upload all of B
// before the first blob can run, so a host-resident call costs at least
// B's upload plus the whole C download.  Here A and B are cut into P row
// panels each and uploaded in the order A0 B0 A1 B1 …; shell s is every
// C block that needs panel s and no later one:
//
//   R_s = A_s · B[0..s]ᵀ      (PM rows × (s+1)·PN cols)
//   C_s = A[0..s-1] · B_sᵀ    (s·PM rows × PN cols)
//
// Both are plain GEMMs on contiguous sub-matrices (a row prefix of a
// row-major [rows][K] operand is contiguous), so the ordinary tile kernel
// runs them with pointer offsets.  Shell s's kernels start as soon as
// panels s have landed, and its C comes down while later panels go up:
// uploads, kernels and downloads of consecutive shells overlap on the
// main (upload) stream, two compute streams and two download streams.
//
// Host C layout: shell by shell, R_s then C_s, each tile-major in the
// kernel's grouped tile order (ops/gemm.py untiles it).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "cores.h"
#include "memory.h"

namespace cek {

void Cores::gemm_host_shells(int local_dev, const std::string& kernel, const ArraySpec& A, const ArraySpec& B,
                             const ArraySpec& C, int M, int N, int K, int panels, int group_m, int BM, int BN,
                             int L) {
  std::lock_guard<std::recursive_mutex> call_guard(call_mu_);
  if (local_dev < 0 || local_dev >= static_cast<int>(workers_.size())) throw Error("gemm_host_shells: bad device");
  Worker& w = *workers_[local_dev];
  if (!w.gpu()) throw Error("gemm_host_shells: GPU devices only");
  if (capturing_) throw Error("gemm_host_shells: not inside a graph capture");
  if (panels < 1 || M % panels || N % panels) throw Error("gemm_host_shells: M and N must split into panels");
  const int PM = M / panels, PN = N / panels;
  const int es = A.elem_size;  // 2: bf16 operands (BK = 64), 4: fp32 operands (BK = 32)
  if (PM % BM || PN % BN || L <= 0 || (es != 2 && es != 4) || K % (es == 2 ? 64 : 32))
    throw Error("gemm_host_shells: panel sizes must be whole tiles and K whole K-tiles");
  if (B.elem_size != es || A.bytes != 1ull * es * M * K || B.bytes != 1ull * es * N * K ||
      C.bytes != 4ull * M * N || C.elem_size != 4)
    throw Error("gemm_host_shells: A, B must be [M][K], [N][K] of one element type and C fp32 [M][N]");
  hipFunction_t fn = w.program().gpu_fn(kernel);
  w.wait();
  w.set_device();

  // per-kernel dims ([M', N', K, group_m, split_k, 0, 0, 0]) in device memory
  if (shell_dims_.size() < workers_.size()) shell_dims_.resize(workers_.size(), nullptr);
  if (shell_dims_cap_.size() < workers_.size()) shell_dims_cap_.resize(workers_.size(), 0);
  std::vector<int> dims(static_cast<size_t>(2 * panels) * 8, 0);
  for (int s = 0; s < panels; ++s) {
    int* r = &dims[static_cast<size_t>(2 * s) * 8];
    r[0] = PM, r[1] = (s + 1) * PN, r[2] = K, r[3] = group_m, r[4] = 1;
    int* c = r + 8;
    c[0] = s * PM, c[1] = PN, c[2] = K, c[3] = group_m, c[4] = 1;
  }
  const size_t dims_bytes = dims.size() * sizeof(int);
  if (shell_dims_host_.size() < workers_.size()) shell_dims_host_.resize(workers_.size());
  hipStream_t up = w.main_stream();
  if (shell_dims_host_[local_dev] != dims) {
    // the dims change only with the shape: uploaded (asynchronously, ahead of
    // the first panel on the upload stream the kernels wait on) when they do
    if (shell_dims_cap_[local_dev] < dims_bytes) {
      if (shell_dims_[local_dev]) {
        CEK_HIP(hipStreamSynchronize(up));  // a previous call's kernels may still read the old block
        (void)hipFree(shell_dims_[local_dev]);
      }
      shell_dims_[local_dev] = nullptr;
      CEK_HIP(hipMalloc(&shell_dims_[local_dev], dims_bytes));
      shell_dims_cap_[local_dev] = dims_bytes;
      if (shell_dims_pin_.size() < workers_.size()) shell_dims_pin_.resize(workers_.size(), nullptr);
      if (shell_dims_pin_[local_dev]) host_free(shell_dims_pin_[local_dev]);
      shell_dims_pin_[local_dev] = host_alloc(dims_bytes, 4096, nullptr);
    }
    CEK_HIP(hipStreamSynchronize(up));  // the staging buffer may still feed an earlier copy
    std::memcpy(shell_dims_pin_[local_dev], dims.data(), dims_bytes);
    CEK_HIP(hipMemcpyAsync(shell_dims_[local_dev], shell_dims_pin_[local_dev], dims_bytes, hipMemcpyHostToDevice, up));
    shell_dims_host_[local_dev] = dims;
  }
  char* dA = static_cast<char*>(w.buffer(A));
  char* dB = static_cast<char*>(w.buffer(B));
  char* dC = static_cast<char*>(w.buffer(C));
  int* dd = static_cast<int*>(shell_dims_[local_dev]);

  const uint64_t a_panel = static_cast<uint64_t>(PM) * K, b_panel = static_cast<uint64_t>(PN) * K;  // elements
  uint64_t c_off = 0;  // elements of C before shell s
  int slot = 0;
  for (int s = 0; s < panels; ++s) {
    w.h2d(up, A, s * a_panel, a_panel);
    w.h2d(up, B, s * b_panel, b_panel);
    hipEvent_t landed = w.event(slot++);
    CEK_HIP(hipEventRecord(landed, up));
    hipStream_t ks = w.pipe_stream(s & 1, 1);
    hipStream_t ws = pipeline_writes_on_compute_stream ? ks : w.pipe_stream(s & 1, 2);
    CEK_HIP(hipStreamWaitEvent(ks, landed, 0));
    const uint64_t shell_begin = c_off;
    for (int part = 0; part < 2; ++part) {
      const int* d = &dims[static_cast<size_t>(2 * s + part) * 8];
      const long long tiles = static_cast<long long>(d[0] / BM) * (d[1] / BN);
      if (tiles == 0) continue;
      const void* pd = dd + (2 * s + part) * 8;
      const void* pa = dA + es * (part == 0 ? s * a_panel : 0);
      const void* pb = dB + es * (part == 0 ? 0 : s * b_panel);
      void* pc = dC + 4 * c_off;
      long long off = 0, gs = tiles * L;
      void* params[] = {&pd, &pa, &pb, &pc, &off, &gs};
      CEK_HIP(hipModuleLaunchKernel(fn, static_cast<unsigned>(tiles), 1, 1, static_cast<unsigned>(L), 1, 1, 0, ks,
                                    params, nullptr));
      c_off += static_cast<uint64_t>(d[0]) * d[1];
    }
    if (ws != ks) {
      hipEvent_t done = w.event(slot++);
      CEK_HIP(hipEventRecord(done, ks));
      CEK_HIP(hipStreamWaitEvent(ws, done, 0));
    }
    w.d2h(ws, C, shell_begin, c_off - shell_begin);
  }
  for (int h = 0; h < 2 && h < panels; ++h) {
    CEK_HIP(hipStreamSynchronize(w.pipe_stream(h, 1)));
    CEK_HIP(hipStreamSynchronize(w.pipe_stream(h, 2)));
  }
  CEK_HIP(hipStreamSynchronize(up));
}

}  // namespace cek
