// fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_16x16x4_f32), fp32 in / out:
// the single-precision member of the range-partitioned GEMM family.
//
//   C = A · Bᵀ      A: [M][K] f32 row-major, Bt: [N][K] f32 row-major
//   C is written TILE-MAJOR in the grouped tile order of kernels/sgemm_bf16.hip,
//   so a device's contiguous range of tiles is one contiguous slice of C.
//
// Structure: BK = 32 floats = 128 B per row, the same byte geometry as the
// bf16 kernels (BK = 64 bf16).  Both operands go global→LDS with
// global_load_lds_dwordx4 (16 B per lane, 8 rows × 128 B per wave
// instruction) into two LDS stages, XOR-swizzling the 16-B chunk index with
// (row & 7) on the global source and on the ds_read_b128 address
// (conflict-free fragment reads).
//
// Fragments: v_mfma_f32_16x16x4_f32 takes one float of A per lane
// (A[row = l%16][k = l/16]) and one of B.  A lane instead reads 16 B —
// A[row][4·(l/16) .. 4·(l/16)+3] of a 16-deep k block — and feeds element t
// to the t-th of four MFMAs: MFMA t then sums over k ∈ {t, 4+t, 8+t, 12+t}
// for A and B alike, and the four together cover the k block exactly.
// One ds_read_b128 per operand fragment per 16 k, four MFMAs per read.
#include "cek_kernel.h"

namespace {

template <int WM, int WN, int FM, int FN, int PIPE>
__device__ __forceinline__ void gemm_f32_tile(const int* __restrict__ dims, const float* __restrict__ A,
                                              const float* __restrict__ Bt, float* __restrict__ C, char* smem,
                                              long long off) {
  constexpr int BM = WM * 16 * FM, BN = WN * 16 * FN, BK = 32;
  constexpr int NWAVES = WM * WN, NT = 64 * NWAVES;
  constexpr int A_BYTES = BM * BK * 4, B_BYTES = BN * BK * 4, STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = A_BYTES / 1024 / NWAVES, B_INSTR = B_BYTES / 1024 / NWAVES;
  static_assert(A_INSTR * NWAVES * 1024 == A_BYTES && B_INSTR * NWAVES * 1024 == B_BYTES, "staging split");

  const int M = dims[0], N = dims[1], K = dims[2], GM = dims[3] > 0 ? dims[3] : 1;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const long long t = (long long)cek_xcd_remap(blockIdx.x, gridDim.x) + off / NT;
  const int ntn = N / BN, ntm = M / BM;
  int tm, tn;
  // a launch wider than the tile grid (a host-side range error) must not
  // read or write past A, B or C: surplus work-groups leave at once
  if (t >= (long long)ntm * ntn) return;
  cek_tile_coords(t, ntm, ntn, GM, dims[6], tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  // staging: lane l of a wave instruction lands at row ins·8 + l/8, physical
  // 16-B chunk l%8, which holds logical chunk (l%8) ^ (row & 7)
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ (lrow & 7);
  const unsigned lane_off = (unsigned)(lrow * K + lchunk * 4) * 4u;
  const char* a_wave = (const char*)(A + (size_t)(m0 + wave * A_INSTR * 8) * K);
  const char* b_wave = (const char*)(Bt + (size_t)(n0 + wave * B_INSTR * 8) * K);
  auto stage = [&](int buf, int kt) {
    char* base = smem + buf * STAGE;
#pragma unroll
    for (int j = 0; j < A_INSTR; ++j) {
      const char* src = a_wave + ((size_t)j * 8 * K + (size_t)kt * BK) * 4;
      __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off),
                                       (lds_void*)(base + (wave * A_INSTR + j) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < B_INSTR; ++j) {
      const char* src = b_wave + ((size_t)j * 8 * K + (size_t)kt * BK) * 4;
      __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off),
                                       (lds_void*)(base + A_BYTES + (wave * B_INSTR + j) * 1024), 16, 0, 0);
    }
  };

  // fragment offsets: row (wr·16FM + i·16 + l%16), logical chunk s·4 + l/16
  const int fr = lane & 15, fq = lane >> 4;
  int a_off[2], b_off[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int pc = (s * 4 + fq) ^ (lane & 7);
    a_off[s] = (wr * 16 * FM + fr) * 128 + pc * 16;
    b_off[s] = A_BYTES + (wc * 16 * FN + fr) * 128 + pc * 16;
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  auto ld = [&](f32x4(&a)[FM], f32x4(&b)[FN], const char* base, int s) {
#pragma unroll
    for (int j = 0; j < FN; ++j) b[j] = *(const f32x4*)(base + b_off[s] + j * 2048);
#pragma unroll
    for (int i = 0; i < FM; ++i) a[i] = *(const f32x4*)(base + a_off[s] + i * 2048);
  };
  auto mma = [&](const f32x4(&a)[FM], const f32x4(&b)[FN]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (PIPE == 3 || PIPE == 4 || PIPE == 5) {
    // one wave per SIMD: both k blocks' fragments read up front, then the
    // next K-tile's LDS-DMA pieces issued one by one between groups of
    // MFMAs, so their issue cost hides in the MFMA stream instead of
    // stalling the only wave on the SIMD before it
    // PIPE 3: spread over all 8 (block, q) MFMA groups; PIPE 4: all within
    // block 0's four groups, so the pieces have block 1's MFMAs to land
    // before the vmcnt(0) that closes the K-tile
    constexpr int NGLDS = A_INSTR + B_INSTR;
    constexpr int NGROUPS = PIPE == 4 ? 4 : 8;  // PIPE 5 spreads like PIPE 3
    constexpr int PER_GROUP = (NGLDS + NGROUPS - 1) / NGROUPS;
    auto stage_one = [&](int buf, int kt, int g) {
      char* base = smem + buf * STAGE;
      if (g < A_INSTR) {
        const char* src = a_wave + ((size_t)g * 8 * K + (size_t)kt * BK) * 4;
        __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off),
                                         (lds_void*)(base + (wave * A_INSTR + g) * 1024), 16, 0, 0);
      } else {
        const int j = g - A_INSTR;
        const char* src = b_wave + ((size_t)j * 8 * K + (size_t)kt * BK) * 4;
        __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off),
                                         (lds_void*)(base + A_BYTES + (wave * B_INSTR + j) * 1024), 16, 0, 0);
      }
    };
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const char* base = smem + cur * STAGE;
      const bool pre = kt + 1 < nk;
      f32x4 fa[2][FM], fb[2][FN];
      ld(fa[0], fb[0], base, 0);
      if constexpr (PIPE != 5) ld(fa[1], fb[1], base, 1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int sq = 0; sq < 8; ++sq) {
        const int sb = sq / 4, q = sq % 4;
        if constexpr (PIPE == 5) {
          // block 1's fragment reads ride between block 0's MFMA groups
          constexpr int NRD = FM + FN, PER_RD = (NRD + 3) / 4;
          if (sq < 4) {
#pragma unroll
            for (int r = 0; r < PER_RD; ++r) {
              const int x = sq * PER_RD + r;
              if (x < FN)
                fb[1][x] = *(const f32x4*)(base + b_off[1] + x * 2048);
              else if (x < NRD)
                fa[1][x - FN] = *(const f32x4*)(base + a_off[1] + (x - FN) * 2048);
            }
          }
        }
        if (pre && sq < NGROUPS) {
#pragma unroll
          for (int p2 = 0; p2 < PER_GROUP; ++p2)
            if (sq * PER_GROUP + p2 < NGLDS) stage_one(cur ^ 1, kt + 1, sq * PER_GROUP + p2);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[sb][i][q], fb[sb][j][q], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else if constexpr (PIPE >= 6 && PIPE <= 8) {
    // PIPE 5 with the K-tile's barrier moved in front of its last MFMA
    // group(s) (BARG): every fragment of this K-tile is in registers by then,
    // so the next K-tile's block-0 fragment reads fly under those MFMAs
    // instead of stalling both waves of the SIMD after the barrier.  The
    // LDS-DMA pieces are spread over groups 0..DMAG-1 (piece p in group
    // p·DMAG/NGLDS), leaving BARG-DMAG groups for them to land.
    // PIPE 6: BARG 7, DMAG 4; PIPE 7: BARG 6, DMAG 4; PIPE 8: BARG 7, DMAG 7
    constexpr int NGLDS = A_INSTR + B_INSTR;
    constexpr int BARG = PIPE == 7 ? 6 : 7;
    constexpr int DMAG = PIPE == 8 ? 7 : 4;
    constexpr int NRD = FM + FN, PER_RD = (NRD + 3) / 4;
    auto stage_one = [&](int buf, int kt, int g) {
      char* base = smem + buf * STAGE;
      if (g < A_INSTR) {
        const char* src = a_wave + ((size_t)g * 8 * K + (size_t)kt * BK) * 4;
        __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off),
                                         (lds_void*)(base + (wave * A_INSTR + g) * 1024), 16, 0, 0);
      } else {
        const int j = g - A_INSTR;
        const char* src = b_wave + ((size_t)j * 8 * K + (size_t)kt * BK) * 4;
        __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off),
                                         (lds_void*)(base + A_BYTES + (wave * B_INSTR + j) * 1024), 16, 0, 0);
      }
    };
    f32x4 fa[2][FM], fb[2][FN];
    ld(fa[0], fb[0], smem, 0);
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const char* base = smem + cur * STAGE;
      const bool pre = kt + 1 < nk;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int sq = 0; sq < 8; ++sq) {
        const int sb = sq / 4, q = sq % 4;
        if (sq < 4) {
#pragma unroll
          for (int r = 0; r < PER_RD; ++r) {
            const int x = sq * PER_RD + r;
            if (x < FN)
              fb[1][x] = *(const f32x4*)(base + b_off[1] + x * 2048);
            else if (x < NRD)
              fa[1][x - FN] = *(const f32x4*)(base + a_off[1] + (x - FN) * 2048);
          }
        }
        if (pre) {
#pragma unroll
          for (int p = 0; p < NGLDS; ++p)
            if (p * DMAG / NGLDS == sq) stage_one(cur ^ 1, kt + 1, p);
        }
        if (sq == BARG) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (pre) ld(fa[0], fb[0], smem + (cur ^ 1) * STAGE, 0);
        }
        // row-block by row-block (all four k of FM/4 rows per group), so a
        // block's A fragments die group by group and free the registers the
        // other block's fragment reads load into
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
#pragma unroll
          for (int ii = 0; ii < FM / 4; ++ii)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              const int i = q * (FM / 4) + ii;
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[sb][i][qq], fb[sb][j][qq], acc[i][j], 0, 0, 0);
            }
      }
      __builtin_amdgcn_s_setprio(0);
    }
  } else {
    static_assert(PIPE == 0, "PIPE is 0, 3, 4, 5, 6, 7 or 8");
    // one barrier per K-tile; the next K-tile's DMA flies under the MFMAs
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
      const char* base = smem + cur * STAGE;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f32x4 a[FM], b[FN];
        ld(a, b, base, s);
        mma(a, b);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  // acc[i][j][r] is C(row = wr·16FM + i·16 + fq·4 + r, col = wc·16FN + j·16 + fr)
  float* ct = C + (size_t)t * BM * BN;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* dst = &ct[(size_t)(wr * 16 * FM + i * 16 + fq * 4 + r) * BN + wc * 16 * FN + j * 16 + fr];
        *dst = acc[i][j][r];
      }
}


// The same tile with v_mfma_f32_32x32x2_f32 (64 cycles, 32×32 outputs):
// lane l reads A[row = l%32][8·kb + 4·(l/32) .. +3] and feeds element t to
// the t-th of four MFMAs, which then sum over k ∈ {t, 4+t} of the 8-deep
// block kb.  Fragments per 8-deep block are half those of a 16-deep block of
// the 16×16×4 form, so two register sets (double-buffered across the four
// blocks of a K-tile) fit beside the 128 accumulator registers of a 128×64
// wave tile; the 16×16×4 form spills there.
// Output layout: acc[i][j][r] is C(row = 32i + 8·(r/4) + 4·(l/32) + r%4, col = 32j + l%32).
template <int WM, int WN, int FM, int FN>
__device__ __forceinline__ void gemm_f32w_tile(const int* __restrict__ dims, const float* __restrict__ A,
                                               const float* __restrict__ Bt, float* __restrict__ C, char* smem,
                                               long long off) {
  constexpr int BM = WM * 32 * FM, BN = WN * 32 * FN, BK = 32;
  constexpr int NWAVES = WM * WN, NT = 64 * NWAVES;
  constexpr int A_BYTES = BM * BK * 4, B_BYTES = BN * BK * 4, STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = A_BYTES / 1024 / NWAVES, B_INSTR = B_BYTES / 1024 / NWAVES;
  static_assert(A_INSTR * NWAVES * 1024 == A_BYTES && B_INSTR * NWAVES * 1024 == B_BYTES, "staging split");

  const int M = dims[0], N = dims[1], K = dims[2], GM = dims[3] > 0 ? dims[3] : 1;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;
  const long long t = (long long)cek_xcd_remap(blockIdx.x, gridDim.x) + off / NT;
  const int ntn = N / BN, ntm = M / BM;
  int tm, tn;
  // a launch wider than the tile grid (a host-side range error) must not
  // read or write past A, B or C: surplus work-groups leave at once
  if (t >= (long long)ntm * ntn) return;
  cek_tile_coords(t, ntm, ntn, GM, dims[6], tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  const int lrow = lane >> 3, lchunk = (lane & 7) ^ (lrow & 7);
  const unsigned lane_off = (unsigned)(lrow * K + lchunk * 4) * 4u;
  const char* a_wave = (const char*)(A + (size_t)(m0 + wave * A_INSTR * 8) * K);
  const char* b_wave = (const char*)(Bt + (size_t)(n0 + wave * B_INSTR * 8) * K);
  auto stage = [&](int buf, int kt) {
    char* base = smem + buf * STAGE;
#pragma unroll
    for (int j = 0; j < A_INSTR; ++j) {
      const char* src = a_wave + ((size_t)j * 8 * K + (size_t)kt * BK) * 4;
      __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off),
                                       (lds_void*)(base + (wave * A_INSTR + j) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < B_INSTR; ++j) {
      const char* src = b_wave + ((size_t)j * 8 * K + (size_t)kt * BK) * 4;
      __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off),
                                       (lds_void*)(base + A_BYTES + (wave * B_INSTR + j) * 1024), 16, 0, 0);
    }
  };

  // fragment offsets for 8-deep block kb: row (wr·32FM + i·32 + l%32),
  // logical 16-B chunk 2·kb + l/32, physical = logical ^ (row & 7)
  const int fr = lane & 31, fq = lane >> 5;
  int a_off[4], b_off[4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    const int pc = (kb * 2 + fq) ^ (lane & 7);
    a_off[kb] = (wr * 32 * FM + fr) * 128 + pc * 16;
    b_off[kb] = A_BYTES + (wc * 32 * FN + fr) * 128 + pc * 16;
  }
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto ld = [&](f32x4(&a)[FM], f32x4(&b)[FN], const char* base, int kb) {
#pragma unroll
    for (int j = 0; j < FN; ++j) b[j] = *(const f32x4*)(base + b_off[kb] + j * 4096);
#pragma unroll
    for (int i = 0; i < FM; ++i) a[i] = *(const f32x4*)(base + a_off[kb] + i * 4096);
  };
  auto mma = [&](const f32x4(&a)[FM], const f32x4(&b)[FN]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x4 xa[FM], xb[FN], ya[FM], yb[FN];
  ld(xa, xb, smem, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const char* base = smem + cur * STAGE;
    if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
    ld(ya, yb, base, 1);
    mma(xa, xb);
    ld(xa, xb, base, 2);
    mma(ya, yb);
    ld(ya, yb, base, 3);
    mma(xa, xb);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) ld(xa, xb, smem + (cur ^ 1) * STAGE, 0);
    mma(ya, yb);
  }

  float* ct = C + (size_t)t * BM * BN;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        ct[(size_t)(wr * 32 * FM + i * 32 + (r / 4) * 8 + fq * 4 + (r % 4)) * BN + wc * 32 * FN + j * 32 + fr] =
            acc[i][j][r];
}

// Register-direct tiles: fragments loaded global → VGPR, no LDS, no barrier.
//
// Every LDS-staged form above shares each K-tile between the waves of a
// work-group, so every K-tile ends in a barrier; with one wave per SIMD
// nothing covers the wait after it (the q tiles, 134–140 TF/s), and with
// two waves per SIMD both waves of a SIMD stall at the same barrier (89 %
// MFMA-busy).  Here a wave loads its own fragments, 16 B per lane straight
// into the register image ds_read_b128 would have produced: lane l holds
// A[row = 16i + l%16][16kb + 4(l/16) .. +3], element t feeding the t-th of
// four MFMAs.  The next 16-deep block's loads go out before the current
// block's MFMAs (4·FM·FN of them, 32 cycles each), so even an HBM miss lands
// in time, and the waves never wait for each other.  Waves that share A
// rows (or B rows) read the same lines through the CU's L1; the L2 sees at
// most a few times the LDS form's traffic, a few TB/s against its ~30.
//
// Buffer loads: one descriptor per operand over the work-group's rows
// (built from work-group-uniform values only), the lane's row and k chunk in
// the voffset VGPR and fragment i / block kb as a scalar soffset: two
// address VGPRs for all loads.
// VAR 0: sched_barrier between the phases and a memory clobber after each
//        load group;
// VAR 1: each MFMA phase starts with an empty asm that takes its fragments
//        in and out ("+v", with a memory clobber), so the phase cannot start
//        before the loads issued ahead of it, and nothing else is pinned.
template <int N>
__device__ __forceinline__ void cek_tie(f32x4 (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(x[i])::"memory");
}

template <int WM, int WN, int FM, int FN, int VAR>
__device__ __forceinline__ void gemm_f32_direct(const int* __restrict__ dims, const float* __restrict__ A,
                                                const float* __restrict__ Bt, float* __restrict__ C,
                                                long long off) {
  constexpr int BM = WM * 16 * FM, BN = WN * 16 * FN, NT = 64 * WM * WN;
  const int M = dims[0], N = dims[1], K = dims[2], GM = dims[3] > 0 ? dims[3] : 1;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;
  const long long t = (long long)cek_xcd_remap(blockIdx.x, gridDim.x) + off / NT;
  const int ntn = N / BN, ntm = M / BM;
  int tm, tn;
  // a launch wider than the tile grid (a host-side range error) must not
  // read or write past A, B or C: surplus work-groups leave at once
  if (t >= (long long)ntm * ntn) return;
  cek_tile_coords(t, ntm, ntn, GM, dims[6], tm, tn);
  const int fr = lane & 15, fq = lane >> 4;
  const float* a_base = A + (size_t)tm * BM * K;
  const float* b_base = Bt + (size_t)tn * BN * K;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)a_base, 0, (unsigned)(BM * K * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)b_base, 0, (unsigned)(BN * K * 4), 0x00020000);
  const int va = ((wr * 16 * FM + fr) * K + fq * 4) * 4;
  const int vb = ((wc * 16 * FN + fr) * K + fq * 4) * 4;
  const int frag_stride = 16 * K * 4;  // bytes between fragment rows i and i+1

  auto load = [&](f32x4(&a)[FM], f32x4(&b)[FN], int kb) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
      a[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, va, i * frag_stride + kb * 64, 0));
#pragma unroll
    for (int j = 0; j < FN; ++j)
      b[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rb, vb, j * frag_stride + kb * 64, 0));
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const f32x4(&a)[FM], const f32x4(&b)[FN]) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
  };
  // VAR 2: the next block's FM+FN loads spread evenly over the current
  // block's 4·FM groups of FN MFMAs (one load every few groups), each group
  // pinned by a scheduling barrier, instead of one burst of loads
  auto mma_ld = [&](const f32x4(&a)[FM], const f32x4(&b)[FN], f32x4(&na)[FM], f32x4(&nb)[FN], int kb_next) {
    // VAR 2: over all 4·FM groups; VAR 3: over the first half, so the last
    // load has half a block of MFMAs more to land; VAR 4: the first quarter
    constexpr int NL = FM + FN, NG = VAR == 4 ? FM : VAR == 3 ? 2 * FM : 4 * FM;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int g = q * FM + i;
#pragma unroll
        for (int l = 0; l < NL; ++l)
          if (l * NG / NL == g) {
            // B fragments first: the next block's first MFMA group needs
            // every b and only a[0], and waits count loads in issue order
            if (l < FN)
              nb[l] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rb, vb, l * frag_stride + kb_next * 64, 0));
            else
              na[l - FN] = __builtin_bit_cast(
                  f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, va, (l - FN) * frag_stride + kb_next * 64, 0));
            asm volatile("" ::: "memory");
          }
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
  };
  const int nkb = K / 16;  // even: K % 32 == 0
  f32x4 a0[FM], b0[FN], a1[FM], b1[FN];
  load(a0, b0, 0);
  __builtin_amdgcn_s_setprio(1);
  // The last iteration reloads block 0 (in bounds, unused): no branch.
  for (int kb = 0; kb < nkb; kb += 2) {
    if constexpr (VAR == 0) {
      load(a1, b1, kb + 1);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mma(a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      load(a0, b0, kb + 2 < nkb ? kb + 2 : 0);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b1);
      __builtin_amdgcn_sched_barrier(0);
    } else if constexpr (VAR == 1) {
      load(a1, b1, kb + 1);
      cek_tie(a0);
      cek_tie(b0);
      mma(a0, b0);
      load(a0, b0, kb + 2 < nkb ? kb + 2 : 0);
      cek_tie(a1);
      cek_tie(b1);
      mma(a1, b1);
    } else {
      static_assert(VAR >= 2 && VAR <= 4, "VAR is 0 .. 4");
      mma_ld(a0, b0, a1, b1, kb + 1);
      mma_ld(a1, b1, a0, b0, kb + 2 < nkb ? kb + 2 : 0);
    }
  }
  __builtin_amdgcn_s_setprio(0);

  // acc[i][j][r] is C(row = wr·16FM + 16i + 4fq + r, col = wc·16FN + 16j + fr)
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

#define CEK_GEMM_F32G_KERNEL(NAME, WM, WN, FM, FN, VAR)                                            \
  extern "C" __global__ __launch_bounds__(64 * WM * WN) void NAME(                                  \
      const int* dims, const float* A, const float* Bt, float* C, CEK_HIDDEN) {                      \
    gemm_f32_direct<WM, WN, FM, FN, VAR>(dims, A, Bt, C, __cek_off);                                 \
  }
// 256×256: 4 waves of 128×128 (one per SIMD, accumulators in AGPRs: 512
// registers per lane) and 8 waves of 128×64 (two per SIMD)
CEK_GEMM_F32G_KERNEL(cek_sgemm_f32_256x256g, 2, 2, 8, 8, 0)
CEK_GEMM_F32G_KERNEL(cek_sgemm_f32_256x256gt, 2, 2, 8, 8, 1)
CEK_GEMM_F32G_KERNEL(cek_sgemm_f32_256x256gh, 2, 2, 8, 8, 3)
CEK_GEMM_F32G_KERNEL(cek_sgemm_f32_256x256g8, 2, 4, 8, 4, 0)
CEK_GEMM_F32G_KERNEL(cek_sgemm_f32_256x256g8t, 2, 4, 8, 4, 1)
CEK_GEMM_F32G_KERNEL(cek_sgemm_f32_256x256g8i, 2, 4, 8, 4, 2)  // loads spread between MFMA groups
CEK_GEMM_F32G_KERNEL(cek_sgemm_f32_256x256g8h, 2, 4, 8, 4, 3)  // spread over the first half
CEK_GEMM_F32G_KERNEL(cek_sgemm_f32_256x256g8q, 2, 4, 8, 4, 4)  // spread over the first quarter

#define CEK_GEMM_F32_KERNEL(NAME, WM, WN, FM, FN, PIPE)                                           \
  extern "C" __global__ __launch_bounds__(64 * WM * WN) void NAME(                                 \
      const int* dims, const float* A, const float* Bt, float* C, CEK_HIDDEN) {                     \
    __shared__ __attribute__((aligned(16))) char smem[2 * (WM * 16 * FM + WN * 16 * FN) * 32 * 4]; \
    gemm_f32_tile<WM, WN, FM, FN, PIPE>(dims, A, Bt, C, smem, __cek_off);                           \
  }

// 128×128 tiles, 4 waves (2×2, 64×64 each), 64 KiB LDS: two work-groups per CU.
CEK_GEMM_F32_KERNEL(cek_sgemm_f32_128x128, 2, 2, 4, 4, 0)
// 256×128 tiles, 8 waves (4×2, 64×64 each), 96 KiB LDS.
CEK_GEMM_F32_KERNEL(cek_sgemm_f32_256x128, 4, 2, 4, 4, 0)
// 256×256 tiles, 8 waves (2×4, 128×64 each), 128 KiB LDS.
CEK_GEMM_F32_KERNEL(cek_sgemm_f32_256x256, 2, 4, 8, 4, 0)
// fragment reads of k block 1 between block 0's MFMA groups (production:
// profiles/gemm_f32_findings.md); ib7: barrier ahead of the last MFMA groups;
// 256x128ie: every LDS-DMA piece within the first k block's MFMAs
CEK_GEMM_F32_KERNEL(cek_sgemm_f32_256x256ir, 2, 4, 8, 4, 5)
CEK_GEMM_F32_KERNEL(cek_sgemm_f32_256x256ib7, 2, 4, 8, 4, 8)
CEK_GEMM_F32_KERNEL(cek_sgemm_f32_256x128ie, 4, 2, 4, 4, 4)

// 32×32×2 form with register double-buffered fragments (gemm_f32w_tile).
#define CEK_GEMM_F32W_KERNEL(NAME, WM, WN, FM, FN)                                                 \
  extern "C" __global__ __launch_bounds__(64 * WM * WN) void NAME(                                  \
      const int* dims, const float* A, const float* Bt, float* C, CEK_HIDDEN) {                      \
    __shared__ __attribute__((aligned(16))) char smem[2 * (WM * 32 * FM + WN * 32 * FN) * 32 * 4];  \
    gemm_f32w_tile<WM, WN, FM, FN>(dims, A, Bt, C, smem, __cek_off);                                 \
  }

CEK_GEMM_F32W_KERNEL(cek_sgemm_f32_256x256w, 2, 4, 4, 2)  // 8 waves, 128×64 each, 128 KiB LDS
