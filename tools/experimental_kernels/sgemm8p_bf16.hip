// bf16 GEMM, 256×256 tiles, 8-phase half-tile pipeline (cdna_hip_programming.md
// §5 "The 256² 8-phase template"), same contract as sgemm_bf16.hip:
//
//   C = A · Bᵀ      A: [M][K] bf16, Bt: [N][K] bf16 (row-major), C fp32
//   C tile-major in the grouped tile order, one work-group (512 threads) per
//   256×256 tile, range-partitionable by compute().
//
// Geometry: 8 waves as 2 (M) × 4 (N), each wave owns 128×64 of C = 8×4
// v_mfma_f32_16x16x32_bf16 accumulators.  A K-tile (BK = 64) is split into
// four 16 KiB HALF-TILES, in the order the waves first read them:
//   0: A rows of quadrant-row 0 (rows wr·128 + 0..63 for both wr)
//   1: Bt rows of quadrant-column 0 (rows wc·64 + 0..31 for all wc)
//   2: Bt rows of quadrant-column 1 (wc·64 + 32..63)
//   3: A rows of quadrant-row 1 (wr·128 + 64..127)
// Each PHASE computes one 64×32 quadrant of every wave's C over K = 64
// (16 MFMAs) — quadrants (0,0) (0,1) (1,1) (1,0) per K-tile — reading only
// the half-tile(s) it needs, and issues the global_load_lds of ONE half-tile
// D = R − 4 items ahead into a ring of R half-tile slots in LDS.  The two wave
// groups (wr = 0 / 1, one wave of each per SIMD) run one barrier apart, so
// while one group issues its MFMAs the other reads LDS and issues DMA.
//
// Ordering (barriers B1, B2, …; group 0's phase p = reads B(2p−1) MFMA B(2p),
// group 1 one barrier later):
//   RAW  an item retired by the vmcnt before phase p's first barrier is read
//        in phase p+1 or later;
//   WAR  a slot is restaged ≥ 2 phases after its last read: item s+R is
//        issued in phase s+R−D = s+4 and the last read of item s is in phase
//        ≤ s+2 (half-tile 1 is re-read by quadrant (1,0)).
// The vmcnt allowance per phase follows from which items the next phase
// reads (see `wait_for_next`).  LDS rows are 128 B with the 16-byte chunk
// XOR-swizzled by (row & 7) on the global source and on the read (rule 21).
#include "cek_kernel.h"

namespace {

template <int Q>
struct QTag {
  static constexpr int value = Q;
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void block_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int R>
__device__ __forceinline__ void gemm8p(const int* __restrict__ dims, const uint16_t* __restrict__ A,
                                       const uint16_t* __restrict__ Bt, float* __restrict__ C, char* smem,
                                       long long off) {
  constexpr int BM = 256, BN = 256, BK = 64, NT = 512, HT = 16384, D = R - 4;
  static_assert(D >= 4, "ring needs at least 8 slots");
  if (blockDim.x != NT) return;  // 8 waves assumed by every index below (uniform exit)
  const int M = dims[0], N = dims[1], K = dims[2], GM = dims[3] > 0 ? dims[3] : 1;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const long long t = (long long)cek_xcd_remap(blockIdx.x, gridDim.x) + off / NT;
  const int ntn = N / BN, ntm = M / BM;
  const int per_group = GM * ntn, grp = (int)(t / per_group), first = grp * GM;
  const int gsz = min(ntm - first, GM), in_g = (int)(t % per_group);
  const int tm = first + in_g % gsz, tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  // Staging: wave w fills half-tile rows [16w, 16w+16) with two 1 KiB
  // wave-instructions (8 rows × 128 B each); lane l → row +l/8, physical
  // chunk l%8 holding logical chunk (l%8) ^ (l/8).
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ (lrow & 7);
  const unsigned lane_off = (unsigned)(lrow * K + lchunk * 8) * 2u;
  const char* a_src = (const char*)(A + (size_t)(m0 + (wave >> 2) * 128 + (wave & 3) * 16) * K);
  const char* b_src = (const char*)(Bt + (size_t)(n0 + (wave >> 1) * 64 + (wave & 1) * 16) * K);
  const size_t row8 = (size_t)8 * K * 2;  // 8 rows, bytes

  auto slot_of = [](int s) { return s - (s / R) * R; };
  auto issue = [&](int s) {
    const int kt = s >> 2, j = s & 3;
    char* dst = smem + slot_of(s) * HT + wave * 2048;
    const char* src;
    if (j == 0 || j == 3)
      src = a_src + (size_t)(j == 3 ? 64 : 0) * K * 2;
    else
      src = b_src + (size_t)(j == 2 ? 32 : 0) * K * 2;
    src += (size_t)kt * BK * 2;
    __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off), (lds_void*)dst, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + row8 + lane_off), (lds_void*)(dst + 1024), 16, 0, 0);
  };

  // Fragment read offsets inside a half-tile: row (group·rows + frag·16 + l%16),
  // logical chunk s·4 + l/16, physical = logical ^ (l & 7).
  const int fr = lane & 15, fq = lane >> 4;
  int a_off[2], b_off[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int pc = (s * 4 + fq) ^ (lane & 7);
    a_off[s] = (wr * 64 + fr) * 128 + pc * 16;
    b_off[s] = (wc * 32 + fr) * 128 + pc * 16;
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[4][2], fb[2][2];

  const int nk = K / BK, total = 4 * nk;

  // RAW wait at the end of phase p (quadrant Q) for the items phase p+1
  // reads: steady state leaves D−2 items (2 loads each) in flight, D−1
  // before quadrant (1,0), whose only new half-tile was already needed.
  auto wait_for_next = [&](int p, auto q_tag) {
    constexpr int Q = decltype(q_tag)::value;
    if (p + 1 >= total) return;
    if (p + D < total) {
      if constexpr (Q == 2)
        wait_vmcnt<2 * (D - 1)>();
      else
        wait_vmcnt<2 * (D - 2)>();
    } else {
      wait_vmcnt<0>();
    }
  };

  auto phase = [&](int k, auto q_tag) {
    constexpr int Q = decltype(q_tag)::value;
    constexpr int MI = (Q == 0 || Q == 1) ? 0 : 1;
    constexpr int NI = (Q == 0 || Q == 3) ? 0 : 1;
    const int p = 4 * k + Q;
    if constexpr (Q != 2) {  // B half-tile of this quadrant column
      const char* hb = smem + slot_of(4 * k + (NI ? 2 : 1)) * HT;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[j][s] = *(const bf16x8*)(hb + b_off[s] + j * 2048);
    }
    if constexpr (Q == 0 || Q == 2) {  // A half-tile of this quadrant row
      __builtin_amdgcn_sched_barrier(0);
      const char* ha = smem + slot_of(4 * k + (MI ? 3 : 0)) * HT;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i][s] = *(const bf16x8*)(ha + a_off[s] + i * 2048);
    }
    if (p + D < total) issue(p + D);
    wait_for_next(p, q_tag);
    block_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          acc[MI * 4 + i][NI * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[j][s], acc[MI * 4 + i][NI * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    block_barrier();
  };

  // prologue: D items in flight, items 0 and 1 (phase 0's reads) retired
  for (int s = 0; s < D; ++s)
    if (s < total) issue(s);
  if (total >= D)
    wait_vmcnt<2 * (D - 2)>();
  else
    wait_vmcnt<0>();
  block_barrier();
  if (wr == 1) block_barrier();  // group 1 runs one barrier behind

  for (int k = 0; k < nk; ++k) {
    phase(k, QTag<0>{});
    phase(k, QTag<1>{});
    phase(k, QTag<2>{});
    phase(k, QTag<3>{});
  }
  if (wr == 0) block_barrier();  // equal barrier counts for both groups

  // Epilogue: acc[i][j][r] is C(row = wr·128 + i·16 + fq·4 + r, col = wc·64 + j·16 + fr)
  float* ct = C + (size_t)t * BM * BN;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ct[(size_t)(wr * 128 + i * 16 + fq * 4 + r) * BN + wc * 64 + j * 16 + fr] = acc[i][j][r];
}

}  // namespace

#define CEK_GEMM8P_KERNEL(NAME, R)                                                        \
  extern "C" __global__ __launch_bounds__(512) void NAME(const int* dims, const uint16_t* A, \
                                                         const uint16_t* Bt, float* C, CEK_HIDDEN) { \
    __shared__ __attribute__((aligned(16))) char smem[R * 16384];                         \
    gemm8p<R>(dims, A, Bt, C, smem, __cek_off);                                           \
  }

CEK_GEMM8P_KERNEL(cek_sgemm8p_bf16_r8, 8)
CEK_GEMM8P_KERNEL(cek_sgemm8p_bf16_r10, 10)
