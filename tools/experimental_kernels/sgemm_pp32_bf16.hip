// bf16 GEMM, ping-pong wave groups with a 4-deep BK = 32 LDS ring — same
// contract as sgemm_bf16.hip (C = A·Bᵀ, fp32 tile-major C in grouped tile
// order, one work-group per BM×BN tile, range-partitionable by compute()).
//
// Why: the BK = 64 ping-pong kernel (MODE 2) keeps one K-tile of DMA in
// flight; PMC on 8192³ shows the matrix pipe 61 % busy with 30 % of wave time
// parked at barriers/vmcnt.  Splitting the same 128 KiB of LDS into four
// 32 KiB stages lets the loader run three K-tiles ahead (≈3 MFMA sections of
// latency cover instead of ≈2).
//
// Per K-tile (BK = 32): A 256×32 and Bt BN×32 bf16 rows of 64 B, staged by
// the first wave group (G0) with global_load_lds (16 B per lane, lane-linear
// LDS image); the 16-byte chunk (4 per row) is XOR-swizzled with
// (row >> 2) & 3 on the global source and on the ds_read_b128 address, so
// each 16-lane fragment read touches 16 distinct bank slots.  G0 and G1 (one
// wave of each per SIMD) alternate an LDS-read section and an MFMA section,
// one barrier apart.
//
// Ordering: stage k+3 is issued at the start of G0's read section of K-tile
// k into the buffer of K-tile k−1, whose last reader (G1's read section of
// k−1) retired its reads (lgkmcnt(0)) before the barrier that opened this
// section.  G0's MFMA section of k ends with a vmcnt that retires stage k+1
// before the barrier after which it is read.
#include "cek_kernel.h"

namespace {

template <int N>
__device__ __forceinline__ void vmcnt_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int WM, int WN, int FM, int FN>
__device__ __forceinline__ void gemm_pp32(const int* __restrict__ dims, const uint16_t* __restrict__ A,
                                          const uint16_t* __restrict__ Bt, float* __restrict__ C, char* smem,
                                          long long off) {
  constexpr int BM = WM * 16 * FM, BN = WN * 16 * FN, BK = 32, NST = 4;
  constexpr int NWAVES = WM * WN, NT = 64 * NWAVES, STAGERS = NWAVES / 2;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = A_BYTES / 1024 / STAGERS, B_INSTR = B_BYTES / 1024 / STAGERS;
  constexpr int LOADS = A_INSTR + B_INSTR;  // glds per staging wave per K-tile
  static_assert(A_INSTR * STAGERS * 1024 == A_BYTES && B_INSTR * STAGERS * 1024 == B_BYTES, "staging split");
  if (blockDim.x != NT) return;

  const int M = dims[0], N = dims[1], K = dims[2], GM = dims[3] > 0 ? dims[3] : 1;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const long long t = (long long)cek_xcd_remap(blockIdx.x, gridDim.x) + off / NT;
  const int ntn = N / BN, ntm = M / BM;
  const int per_group = GM * ntn, grp = (int)(t / per_group), first = grp * GM;
  const int gsz = min(ntm - first, GM), in_g = (int)(t % per_group);
  const int tm = first + in_g % gsz, tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  const bool g1 = wave >= STAGERS;

  // staging: one wave-instruction = 1 KiB = 16 rows × 64 B; lane l → row l/4,
  // physical chunk l%4 holding logical chunk (l%4) ^ ((row >> 2) & 3)
  const int lrow = lane >> 2, lchunk = (lane & 3) ^ ((lrow >> 2) & 3);
  const unsigned lane_off = (unsigned)(lrow * K + lchunk * 8) * 2u;
  const int sw = wave % STAGERS;
  const char* a_wave = (const char*)(A + (size_t)(m0 + sw * A_INSTR * 16) * K);
  const char* b_wave = (const char*)(Bt + (size_t)(n0 + sw * B_INSTR * 16) * K);
  auto stage = [&](int kt) {
    char* base = smem + (kt % NST) * STAGE;
#pragma unroll
    for (int j = 0; j < A_INSTR; ++j) {
      const char* src = a_wave + ((size_t)j * 16 * K + (size_t)kt * BK) * 2;
      __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off), (lds_void*)(base + (sw * A_INSTR + j) * 1024),
                                       16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < B_INSTR; ++j) {
      const char* src = b_wave + ((size_t)j * 16 * K + (size_t)kt * BK) * 2;
      __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off),
                                       (lds_void*)(base + A_BYTES + (sw * B_INSTR + j) * 1024), 16, 0, 0);
    }
  };

  // fragment reads: row (group rows + frag·16 + l%16), logical chunk l/16,
  // physical = chunk ^ ((row >> 2) & 3) = (l/16) ^ ((l%16) >> 2)
  const int fr = lane & 15, fq = lane >> 4;
  const int pc = fq ^ ((fr >> 2) & 3);
  const int a_off = (wr * 16 * FM + fr) * 64 + pc * 16;
  const int b_off = A_BYTES + (wc * 16 * FN + fr) * 64 + pc * 16;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[FM], fb[FN];

  const int nk = K / BK;
  if (!g1) {
    for (int s = 0; s < NST - 1; ++s)
      if (s < nk) stage(s);
    if (nk >= 3)
      vmcnt_wait<2 * LOADS>();
    else
      vmcnt_wait<0>();
  }
  bar();
  if (g1) bar();  // G1 runs one section behind
  for (int kt = 0; kt < nk; ++kt) {
    const char* base = smem + (kt % NST) * STAGE;
    if (!g1 && kt + NST - 1 < nk) stage(kt + NST - 1);
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j] = *(const bf16x8*)(base + b_off + j * 1024);
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = *(const bf16x8*)(base + a_off + i * 1024);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (!g1) {  // retire stage kt+1 (issued stages run up to min(kt+3, nk-1))
      const int ahead = min(kt + NST - 1, nk - 1) - (kt + 1);
      if (ahead >= 2)
        vmcnt_wait<2 * LOADS>();
      else if (ahead == 1)
        vmcnt_wait<LOADS>();
      else
        vmcnt_wait<0>();
    }
    bar();
  }
  if (!g1) bar();  // equal barrier counts for both groups

  float* ct = C + (size_t)t * BM * BN;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ct[(size_t)(wr * 16 * FM + i * 16 + fq * 4 + r) * BN + wc * 16 * FN + j * 16 + fr] = acc[i][j][r];
}

}  // namespace

#define CEK_GEMM_PP32_KERNEL(NAME, WM, WN, FM, FN)                                                        \
  extern "C" __global__ __launch_bounds__(64 * WM * WN) void NAME(const int* dims, const uint16_t* A,        \
                                                                  const uint16_t* Bt, float* C, CEK_HIDDEN) { \
    __shared__ __attribute__((aligned(16))) char smem[4 * (WM * 16 * FM + WN * 16 * FN) * 32 * 2];         \
    gemm_pp32<WM, WN, FM, FN>(dims, A, Bt, C, smem, __cek_off);                                           \
  }

CEK_GEMM_PP32_KERNEL(cek_sgemm_bf16_256x256q, 2, 4, 8, 4)
CEK_GEMM_PP32_KERNEL(cek_sgemm_bf16_256x128q, 4, 2, 4, 4)
