// bf16 GEMM on CDNA4 matrix cores, fp32 accumulate / fp32 output
// ("SGEMM 8192² bf16" of BASELINE.json), range-partitionable by compute():
//
//   C = A · Bᵀ      A: [M][K] bf16 row-major, Bt: [N][K] bf16 row-major
//   C is written TILE-MAJOR: tile t = (tm, tn) (tn fastest) occupies
//   C[t·BM·BN ...] in MFMA-fragment order inside the tile (epilogue; the
//   host's ops/gemm.py tile_to_rows restores rows), so any contiguous range of
//   tiles — the slice a device gets from the load balancer — is one
//   contiguous byte range (the reference's partial write of
//   [ref·e, (ref+r)·e), Worker.cs:1349-1352, with e = BM·BN / local).
//
// Work decomposition for compute(): one work-group (local = 64·WM·WN threads)
// per BM×BN tile, global range = tiles × local.  The work-group's absolute
// tile is its XCD-remapped local block id + __cek_off / local.
//
// Structure (cdna_hip_programming.md §5): 256×BN tile, BK = 64, 2·WN waves
// (2 along M × WN along N), each wave 128×64 of C as 8×4 tiles of
// v_mfma_f32_16x16x32_bf16; both operands staged global→LDS with
// global_load_lds_dwordx4 (16 B/lane, lane-linear LDS image) into two LDS
// stages — the next K-tile's DMA is issued before the current tile's MFMAs
// and retired by one vmcnt(0)+barrier per K-tile.  LDS rows are 128 B; the
// 16-B chunk index is XOR-swizzled with (row & 7) on the global SOURCE
// address and on the ds_read_b128 address (rule 21), which makes every
// fragment read conflict-free (each 16-lane group hits 16 distinct slots).
#include "cek_kernel.h"

// K-tile index of a stage load; tools/microbench/gemm_loop.hip redefines it
// to re-read two K-tiles (an L2-resident operand stream) as a probe.
#ifndef CEK_KTILE
#define CEK_KTILE(ks, kt) ((ks) + (kt))
#endif
// Per-work-group timeline stamps (tools/microbench/gemm_loop.hip defines it
// in its timeline build; empty in the library).
#ifndef CEK_TS
#define CEK_TS(k)
#endif

namespace {

template <int WM, int WN, int FM, int FN, int MODE, bool SK = false, int XCH = 0, bool ROWC = false>
__device__ __forceinline__ void gemm_tile(const int* __restrict__ dims,
                                          const uint16_t* __restrict__ A,
                                          const uint16_t* __restrict__ Bt, float* __restrict__ C,
                                          char* smem, long long off, float* __restrict__ W = nullptr,
                                          int* __restrict__ tile_cnt = nullptr) {
  constexpr int BM = WM * 16 * FM, BN = WN * 16 * FN, BK = 64;
  constexpr int NREG = WM * WN;
  constexpr int NWAVES = NREG, NT = 64 * NWAVES;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  // MODE 0: one LDS stage in flight, all waves stage.  MODE 2: ping-pong —
  // the two halves of the work-group (waves < NWAVES/2 = G0, the rest = G1,
  // one of each per SIMD) alternate between an LDS-read section and an
  // MFMA section, one s_barrier apart, so each SIMD's matrix pipe always has
  // one wave issuing; G0 issues all LDS-DMA staging.  MODE 4: ping-pong with
  // balanced DMA (G0 stages A, G1 stages Bt two K-tiles ahead).  MODE 6:
  // ping-pong with the K-tile's DMA split evenly by 1 KiB chunk, three stages.
  constexpr int STAGERS = MODE >= 2 ? NWAVES / 2 : NWAVES;
  constexpr int A_INSTR = A_BYTES / 1024 / STAGERS;
  constexpr int B_INSTR = B_BYTES / 1024 / STAGERS;

  const int M = dims[0], N = dims[1], K = dims[2], GM = dims[3] > 0 ? dims[3] : 1;
  const int tid = threadIdx.x, lane = tid & 63;
  CEK_TS(0);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = (wave % NREG) / WN, wc = (wave % NREG) % WN;
  // Split-K (SK): work-group u computes K-tiles [ks, ks + nk) of tile u / S;
  // the S work-groups of a tile are consecutive ids, so the XCD remap keeps
  // them on one XCD and the load balancer (granularity S·local) on one device.
  const long long u = (long long)cek_xcd_remap(blockIdx.x, gridDim.x) + off / NT;
  const int S = SK ? max(dims[4], 1) : 1;
  const long long t = u / S;
  // XCH 3: the K-split of u odd (the helper) takes K/64/2 − dims[5] K-tiles
  // from the start, u even (the owner) the rest
  const int kt_all = dims[2] / 64, shift = XCH >= 3 ? dims[5] : 0;
  int ks = XCH >= 3 ? ((u & 1) ? 0 : kt_all / 2 - shift) : SK ? (int)(u % S) * (kt_all / S) : 0;
  // Grouped tile order (dims[3] = GM row panels per group, tiles walk down
  // the group's rows first): the 32 work-groups an XCD runs at once cover a
  // GM × (32/GM) block of C, so A and B K-slices are shared through that
  // XCD's L2 instead of re-fetched per tile.  C storage stays tile-major by
  // t, so a device's contiguous tile range is still one contiguous slice.
  const int ntn = N / BN, ntm = M / BM;
  int tm, tn;
  // a launch wider than the tile grid (a host-side range error) must not
  // read or write past A, B or C: surplus work-groups leave at once
  if (t >= (long long)ntm * ntn) return;
  cek_tile_coords(t, ntm, ntn, GM, dims[6], tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  // Staging: instruction `ins` of this wave fills LDS bytes [ins·1 KiB, +1 KiB)
  // = 8 rows × 128 B; lane l lands at row ins·8 + l/8, physical chunk l%8,
  // which holds logical chunk (l%8) ^ (row & 7).
  // Within one wave-instruction the 8 rows are ins·8 .. ins·8+7, so the
  // logical chunk (l%8) ^ (row&7) = (l%8) ^ (l/8) is the same for every
  // instruction: one per-lane base pointer plus a uniform row stride.
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ (lrow & 7);
  // per-lane 32-bit byte offset + wave-uniform 64-bit base (saddr form)
  const unsigned lane_off = (unsigned)(lrow * K + lchunk * 8) * 2u;
  const int sw = MODE >= 2 ? wave % (NWAVES / 2) : wave;  // staging wave index
  const char* a_wave = (const char*)(A + (size_t)(m0 + sw * A_INSTR * 8) * K);
  const char* b_wave = (const char*)(Bt + (size_t)(n0 + sw * B_INSTR * 8) * K);

  auto stage_a = [&](int buf, int kt) {
    char* base = smem + buf * STAGE;
#pragma unroll
    for (int j = 0; j < A_INSTR; ++j) {
      const char* src = a_wave + ((size_t)j * 8 * K + (size_t)CEK_KTILE(ks, kt) * BK) * 2;
      __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off),
                                       (lds_void*)(base + (sw * A_INSTR + j) * 1024), 16, 0, 0);
    }
  };
  auto stage_b = [&](int buf, int kt) {
    char* base = smem + buf * STAGE + A_BYTES;
#pragma unroll
    for (int j = 0; j < B_INSTR; ++j) {
      const char* src = b_wave + ((size_t)j * 8 * K + (size_t)CEK_KTILE(ks, kt) * BK) * 2;
      __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off),
                                       (lds_void*)(base + (sw * B_INSTR + j) * 1024), 16, 0, 0);
    }
  };
  auto stage = [&](int buf, int kt) {
    stage_a(buf, kt);
    stage_b(buf, kt);
  };

  // Fragment read offsets (bytes) inside a stage: row (wr·128 + i·16 + l%16),
  // logical chunk s·4 + l/16, physical = logical ^ (l & 7).
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

  int nk = XCH >= 3 ? ((u & 1) ? kt_all / 2 - shift : kt_all / 2 + shift) : K / BK / S;
  unsigned my_xcc = 0;
  // XCH 3 / 4 flags per tile: [4t] hand-over state (0 open, 1 the helper's
  // partial is ready, 2 claimed by the owner), [4t + 1] (XCH 4) the owner's
  // hand-over back (0 open, 1 ready, 2 claimed by the helper), [4t + 2]
  // owner's XCD + 1, [4t + 3] helper's XCD + 1; the word after the last tile
  // counts fall-backs.
  bool claimed = false;  // owner: it will compute the helper's K-range itself
  if constexpr (XCH >= 3) {
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(my_xcc));
    my_xcc &= 15u;
    if (tid == 0)
      __hip_atomic_store(&tile_cnt[4 * t + 2 + (u & 1)], (int)my_xcc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!(u & 1) && dims[7] == -1) {
      // debug (dims[7] == -1): the owner claims the hand-over before its main
      // loop, so the fall-back pass runs (tests of the co-residency-safe path)
      int* st = reinterpret_cast<int*>(smem);
      if (tid == 0) {
        int open = 0;
        st[0] = __hip_atomic_compare_exchange_strong(&tile_cnt[4 * t], &open, 2, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      claimed = st[0] != 0;
      __syncthreads();
    }
  }
  if constexpr (MODE == 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
      const char* base = smem + cur * STAGE;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 a[FM], b[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) b[j] = *(const bf16x8*)(base + b_off[s] + j * 2048);
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = *(const bf16x8*)(base + a_off[s] + i * 2048);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else if constexpr (MODE == 2) {
    // Ping-pong.  Interval n (between two block barriers): one group runs its
    // 4·FM·FN MFMAs of K-tile k while the other reads K-tile k(+1)'s
    // fragments.  G0 stages K-tile k+1 into the free LDS buffer during its
    // read section of K-tile k and retires it (vmcnt(0)) at the end of its
    // MFMA section, one barrier before anyone reads it; every read section
    // ends with lgkmcnt(0) before its barrier, so a buffer is never
    // restaged while still being read.
    const bool g1 = wave >= NWAVES / 2;
    bf16x8 fa[2][FM], fb[2][FN];
    auto ldall = [&](const char* base) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[s][j] = *(const bf16x8*)(base + b_off[s] + j * 2048);
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[s][i] = *(const bf16x8*)(base + a_off[s] + i * 2048);
      }
    };
    auto mmaall = [&]() {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s][i], fb[s][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    auto bar = [] {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    if (!g1) stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    if (g1) bar();  // stagger G1 by one section
    for (int kt = 0; kt < nk; ++kt) {
      const char* base = smem + (kt & 1) * STAGE;
      if (!g1 && kt + 1 < nk) stage((kt + 1) & 1, kt + 1);
      ldall(base);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();
      mmaall();
      if (!g1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
    }
    if (!g1) bar();  // equal barrier counts for both groups
  } else if constexpr (MODE == 6) {
    // Ping-pong with the K-tile's DMA split evenly by 1 KiB chunk: the A and
    // Bt rows of a K-tile are NCH chunks (A first, then Bt, contiguous in a
    // stage); G0 issues the first half for K-tile k+1 in its read section of
    // k, G1 the second half for K-tile k+2 in its own.  Three whole stages.
    //   WAR: a stage is refilled ≥ 2 read sections after its last read.
    //   RAW: G0 retires its half of k+1 (vmcnt(0)) before the barrier ending
    //        its MFMA section; G1 ends its read section k with only its half
    //        of k+2 in flight, so k+1 is complete before G0 reads it.
    constexpr int NCH = (A_BYTES + B_BYTES) / 1024, HALF = NCH / 2, PER_WAVE = HALF / (NWAVES / 2);
    constexpr int A_CH = A_BYTES / 1024;
    static_assert(PER_WAVE * (NWAVES / 2) * 2 == NCH, "even chunk split");
    const bool g1 = wave >= NWAVES / 2;
    const int first_chunk = (g1 ? HALF : 0) + sw * PER_WAVE;
    auto stage6 = [&](int kt) {
      char* base = smem + (kt % 3) * STAGE;
#pragma unroll
      for (int j = 0; j < PER_WAVE; ++j) {
        const int c = first_chunk + j;  // wave-uniform
        const char* src = c < A_CH ? (const char*)(A + (size_t)(m0 + c * 8) * K)
                                   : (const char*)(Bt + (size_t)(n0 + (c - A_CH) * 8) * K);
        src += (size_t)(ks + kt) * BK * 2;
        __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off), (lds_void*)(base + c * 1024), 16, 0, 0);
      }
    };
    bf16x8 fa[2][FM], fb[2][FN];
    auto ldall = [&](int kt) {
      const char* base = smem + (kt % 3) * STAGE;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[s][j] = *(const bf16x8*)(base + b_off[s] + j * 2048);
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[s][i] = *(const bf16x8*)(base + a_off[s] + i * 2048);
      }
    };
    auto mmaall = [&]() {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s][i], fb[s][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    auto bar = [] {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    if (!g1) {
      stage6(0);
    } else {
      stage6(0);
      if (nk > 1) stage6(1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    if (g1) bar();  // G1 runs one section behind
    for (int kt = 0; kt < nk; ++kt) {
      const bool g1_issued = g1 && kt + 2 < nk;
      if (!g1) {
        if (kt + 1 < nk) stage6(kt + 1);
      } else if (g1_issued) {
        stage6(kt + 2);
      }
      ldall(kt);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (g1) {
        if (g1_issued) {
          if constexpr (PER_WAVE == 6)
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
          else if constexpr (PER_WAVE == 8)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      bar();
      mmaall();
      if (!g1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
    }
    if (!g1) bar();  // equal barrier counts for both groups
  } else {
    static_assert(MODE == 4, "MODE is 0, 2, 4 or 6");
    // Ping-pong with balanced DMA: G0 stages the A tile of K-tile k+1 and G1
    // the Bt tile of K-tile k+2, each during its own LDS-read section, so both
    // groups' read sections carry the same DMA issue cost (~60-100 cycles per
    // 1 KiB glds) and stay shorter than the partner's MFMA section.  Bt gets
    // three LDS buffers (A 2 × BM·64·2 B, Bt 3 × BN·64·2 B = 160 KiB at 256²).
    //   WAR: both targets were last read in the previous read sections.
    //   RAW: G0's vmcnt(0) closes its MFMA section (A k+1 before G0 reads it);
    //        G1 ends its read section k with B k+1 retired (only k+2 in flight).
    const bool g1 = wave >= NWAVES / 2;
    char* const a_base = smem;
    char* const b_base = smem + 2 * A_BYTES;
    auto stage_a4 = [&](int kt) {
      char* base = a_base + (kt & 1) * A_BYTES;
#pragma unroll
      for (int j = 0; j < A_INSTR; ++j) {
        const char* src = a_wave + ((size_t)j * 8 * K + (size_t)CEK_KTILE(ks, kt) * BK) * 2;
        __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off), (lds_void*)(base + (sw * A_INSTR + j) * 1024),
                                         16, 0, 0);
      }
    };
    auto stage_b4 = [&](int kt) {
      char* base = b_base + (kt % 3) * B_BYTES;
#pragma unroll
      for (int j = 0; j < B_INSTR; ++j) {
        const char* src = b_wave + ((size_t)j * 8 * K + (size_t)CEK_KTILE(ks, kt) * BK) * 2;
        __builtin_amdgcn_global_load_lds((glb_cvoid*)(src + lane_off), (lds_void*)(base + (sw * B_INSTR + j) * 1024),
                                         16, 0, 0);
      }
    };
    bf16x8 fa[2][FM], fb[2][FN];
    auto ldall = [&](int kt) {
      const char* ab = a_base + (kt & 1) * A_BYTES;
      const char* bb = b_base + (kt % 3) * B_BYTES - A_BYTES;  // b_off includes A_BYTES
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[s][j] = *(const bf16x8*)(bb + b_off[s] + j * 2048);
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[s][i] = *(const bf16x8*)(ab + a_off[s] + i * 2048);
      }
    };
    auto mmaall = [&]() {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s][i], fb[s][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    auto bar = [] {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    if (!g1) {
      stage_a4(0);
    } else {
      stage_b4(0);
      if (nk > 1) stage_b4(1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    CEK_TS(1);
    if (g1) bar();  // G1 runs one section behind
    for (int kt = 0; kt < nk; ++kt) {
      const bool b_issued = g1 && kt + 2 < nk;
      if (!g1) {
        if (kt + 1 < nk) stage_a4(kt + 1);
      } else if (b_issued) {
        stage_b4(kt + 2);
      }
      ldall(kt);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (g1) {
        if (b_issued) {
          if constexpr (B_INSTR == 8)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          else if constexpr (B_INSTR == 4)
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
          else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      bar();
      mmaall();
      if (!g1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
    }
    if (!g1) bar();  // equal barrier counts for both groups
    CEK_TS(2);
  }
  // Epilogue: acc[i][j][r] is C(row = wr·16FM + i·16 + fq·4 + r, col = wc·16FN + j·16 + fr)
  bool store_c = true;
  if constexpr (XCH >= 3) {
    // Uneven split-K = 2: the helper (u odd) ran `shift` K-tiles fewer than
    // half, so its partial is ready while the owner (u even) still
    // multiplies.  XCH 3: the helper hands its whole partial tile over and
    // leaves; the owner adds it and stores all of C.  XCH 4 (halves): the
    // helper hands over its partial of the owner's row half (waves wr == 0)
    // and waits; the owner then hands back its partial of the helper's half
    // (waves wr == 1), and each side adds the other's partial to its own half
    // and stores that half of C — the owner's tail moves 384 KiB instead of
    // 512 KiB, the helper stores the other half beside it.
    // Every wait is bounded and co-residency-safe: a side whose partner is
    // late CLAIMS that hand-over (one CAS against the partner's) and
    // multiplies the partner's K-range itself; the last side to touch a
    // state word re-arms it (0) for the next launch.
    // Partials use the fragment order of the C tile (1 KiB per wave
    // instruction).
    f32x4* wt = reinterpret_cast<f32x4*>(W + (size_t)t * BM * BN) + (wr * WN + wc) * FM * FN * 64 + lane;
    int* st = reinterpret_cast<int*>(smem);
    int rk0 = 0, rcnt = 0;  // a K-range this work-group multiplies in the fall-back loop
    bool read_partial = false;
    __syncthreads();  // every wave is done with LDS before it holds the flags
    if (!(u & 1)) {
      if constexpr (XCH == 5) {
        // XCH 5: hand back the partial of the helper's half FIRST, so the
        // two sides' partial stores overlap instead of the owner's waiting
        // for the helper's before starting its own (with no K-tile shift
        // both sides end their loops together)
        if (!claimed) {
          if (wr == 1) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
              for (int j = 0; j < FN; ++j) wt[(i * FN + j) * 64] = acc[i][j];
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (tid == 0) {
            // the helper published its XCD at its start (0: not started
            // yet, then release through the L2 write-back to be safe)
            const int hx = __hip_atomic_load(&tile_cnt[4 * t + 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (hx != (int)my_xcc + 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            int open = 0;
            if (!__hip_atomic_compare_exchange_strong(&tile_cnt[4 * t + 1], &open, 1, __ATOMIC_RELAXED,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
              tile_cnt[4 * t + 1] = 0;  // the helper claimed it: we are the last to touch the word
          }
        }
      }
      // owner, main loop done: is the helper's partial there?
      if (tid == 0) {
        int v = claimed ? 2 : 0;
        if (!claimed) {
          const int limit = dims[7] > 0 ? dims[7] : (1 << 16);
          for (int spins = 0; (v = __hip_atomic_load(&tile_cnt[4 * t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0;) {
            if (++spins > limit) {
              int open = 0;
              if (__hip_atomic_compare_exchange_strong(&tile_cnt[4 * t], &open, 2, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT))
                v = 2;
              else
                v = open;  // the helper got there first: 1
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
        }
        int same = 0;
        if (v == 2) {
          __hip_atomic_fetch_add(&tile_cnt[(size_t)4 * ntm * ntn], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          // XCH 5: the hand-back published above has no reader now (the
          // helper aborts at its own CAS): re-arm the word
          if constexpr (XCH == 5) tile_cnt[4 * t + 1] = 0;
        } else {  // ready: the helper published its XCD before its partial
          const int hx = __hip_atomic_load(&tile_cnt[4 * t + 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          tile_cnt[4 * t + 3] = 0;
          tile_cnt[4 * t] = 0;  // re-arm: the owner is the last to touch the state
          same = hx == (int)my_xcc + 1;
        }
        tile_cnt[4 * t + 2] = 0;  // this launch's XCD word retires with the owner
        st[0] = v;
        st[1] = same;
      }
      __syncthreads();
      claimed = st[0] == 2;
      const bool same = st[1] != 0;
      __syncthreads();  // st[] read by every wave before LDS is reused
      if (claimed) {
        rk0 = 0;
        rcnt = kt_all / 2 - shift;
      } else {
        if constexpr (XCH == 4) {
          // hand back the partial of the helper's half
          if (wr == 1) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
              for (int j = 0; j < FN; ++j) wt[(i * FN + j) * 64] = acc[i][j];
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (tid == 0) {
            if (!same) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            int open = 0;
            if (!__hip_atomic_compare_exchange_strong(&tile_cnt[4 * t + 1], &open, 1, __ATOMIC_RELAXED,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
              tile_cnt[4 * t + 1] = 0;  // the helper claimed it: we are the last to touch the word
          }
          store_c = wr == 0;
        }
        if constexpr (XCH == 5) store_c = wr == 0;
        if (!same) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        read_partial = XCH == 3 || wr == 0;
      }
    } else {
      // helper: publish the partial (XCH 4: of the owner's half only)
      if (XCH == 3 || wr == 0) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) wt[(i * FN + j) * 64] = acc[i][j];
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      CEK_TS(3);
      if (tid == 0) {
        // the owner's XCD word (0 once the owner has finished or before it
        // started: then release through the L2 write-back to be safe)
        const int px = __hip_atomic_load(&tile_cnt[4 * t + 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (px != (int)my_xcc + 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int open = 0;
        int abort = 0;
        if (!__hip_atomic_compare_exchange_strong(&tile_cnt[4 * t], &open, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT)) {
          // the owner claimed the hand-over and computed our K-range itself:
          // this work-group is the last to touch the tile's words
          tile_cnt[4 * t] = 0;
          tile_cnt[4 * t + 3] = 0;
          abort = 1;
        }
        st[0] = abort;
        st[2] = px == (int)my_xcc + 1;
      }
      __syncthreads();
      const bool abort = st[0] != 0, same_o = st[2] != 0;
      __syncthreads();
      if (abort || XCH == 3) return;
      // XCH 4: wait for the owner's partial of our half
      if (tid == 0) {
        int v = 0;
        const int limit = dims[7] == -2 ? 0 : (1 << 20);
        for (int spins = 0; (v = __hip_atomic_load(&tile_cnt[4 * t + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0;) {
          if (++spins > limit) {
            int open = 0;
            if (__hip_atomic_compare_exchange_strong(&tile_cnt[4 * t + 1], &open, 2, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
              v = 2;
            else
              v = open;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        if (v == 2)
          __hip_atomic_fetch_add(&tile_cnt[(size_t)4 * ntm * ntn], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
          tile_cnt[4 * t + 1] = 0;  // re-arm: the helper is the last to touch it
        st[0] = v;
      }
      __syncthreads();
      const bool fb2 = st[0] == 2;
      __syncthreads();
      if (fb2) {
        rk0 = kt_all / 2 - shift;
        rcnt = kt_all / 2 + shift;
      } else {
        if (!same_o) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        read_partial = wr == 1;
      }
      store_c = wr == 1;
    }
    if (rcnt > 0) {
      // fall-back: the partner's K-tiles [rk0, rk0 + rcnt), one LDS stage in
      // flight, the first half of the waves staging (rare path: kept simple,
      // outside the tuned loop)
      const bool g1 = wave >= NWAVES / 2;
      ks = rk0;
      nk = rcnt;
      if (!g1) stage(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (!g1 && kt + 1 < nk) stage(cur ^ 1, kt + 1);
        const char* base = smem + cur * STAGE;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 a[FM], b[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j) b[j] = *(const bf16x8*)(base + b_off[s2] + j * 2048);
#pragma unroll
          for (int i = 0; i < FM; ++i) a[i] = *(const bf16x8*)(base + a_off[s2] + i * 2048);
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
    CEK_TS(3);
    if (read_partial) {
      f32x4 part[FM][FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) part[i][j] = wt[(i * FN + j) * 64];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] += part[i][j];
    }
    CEK_TS(4);
  } else if constexpr (SK) {
    if (S > 1) {
      // Every split stores its partial tile; the last of the S to arrive
      // (device-scope counter) adds the others' partials to its own and
      // writes C, then re-arms the counter for the next call.  Partials are
      // in fragment order (one dwordx4 per lane per fragment, 1 KiB per wave
      // instruction), so a wave needs one base address, not one per element.
      const int frag0 = (wr * WN + wc) * FM * FN * 64 + lane;
      f32x4* wt = reinterpret_cast<f32x4*>(W + (size_t)u * BM * BN) + frag0;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) wt[(i * FN + j) * 64] = acc[i][j];
      // Each wave waits for its stores to reach L2; ONE release fence (an L2
      // write-back) then covers the whole block before the arrival counter —
      // a fence per wave would write the L2 back eight times.
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* flag = reinterpret_cast<int*>(smem);
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const int old = __hip_atomic_fetch_add(&tile_cnt[t], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = old == S - 1;
        if (old == S - 1) tile_cnt[t] = 0;
      }
      __syncthreads();
      if (*flag == 0) return;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      for (int s2 = 0; s2 < S; ++s2) {
        if (s2 == (int)(u % S)) continue;
        const f32x4* wp = reinterpret_cast<const f32x4*>(W + (size_t)(t * S + s2) * BM * BN) + frag0;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] += wp[(i * FN + j) * 64];
      }
    }
  }
  // C tile in fragment order: wave (wr, wc)'s fragment (i, j) is 64 lanes ×
  // 16 B = 1 KiB contiguous, so every store is one dwordx4 per lane (a
  // row-major tile takes four dword stores per fragment, and with one
  // work-group per CU the store tail is exposed).  Host side: ops/gemm.py
  // tile_to_rows.  Element (row, col) of the tile lives at
  // ((((wr·WN + wc)·FM + i)·FN + j)·64 + fq·16 + fr)·4 + r.
  if constexpr (ROWC) {
    // Row-major C ([M][N], ldc = N): a lane holds 4 consecutive ROWS of one
    // column per fragment, so each wave turns its 16-row strips around in
    // LDS (4 KiB + padding per wave; the main loop is done with LDS): lane
    // (fq, fr) writes fragment j's rows fq·4 + r at column j·16 + fr, then
    // every lane reads 16 B of one row and stores it — 16 lanes cover a
    // 256-B row segment, one dwordx4 per lane per 4 rows.  Row stride 68
    // floats: the two 16-lane halves of a 32-lane write group fall on
    // different banks.
    constexpr int RS = 16 * FN + 4;
    __syncthreads();
    float* strip = reinterpret_cast<float*>(smem) + wave * 16 * RS;
    const int rrow = lane >> 4, rcol = (lane & 15) * 4;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) strip[(fq * 4 + r) * RS + j * 16 + fr] = acc[i][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's strip is written
#pragma unroll
      for (int q = 0; q < 16 / 4; ++q) {
        const int row = q * 4 + rrow;
        const f32x4 v = *reinterpret_cast<const f32x4*>(strip + row * RS + rcol);
        const size_t grow = (size_t)m0 + wr * 16 * FM + i * 16 + row;
        *reinterpret_cast<f32x4*>(C + grow * N + n0 + wc * 16 * FN + rcol) = v;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the strip is rewritten
    }
  } else if (store_c) {
    f32x4* ct = reinterpret_cast<f32x4*>(C + (size_t)t * BM * BN);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) ct[(((wr * WN + wc) * FM + i) * FN + j) * 64 + lane] = acc[i][j];
  }
#ifdef CEK_TS_END
  CEK_TS_END;
#endif
}

}  // namespace

#define CEK_GEMM_KERNEL(NAME, WM, WN, FM, FN, MODE)                                              \
  extern "C" __global__ __launch_bounds__(64 * WM * WN) void NAME(                                \
      const int* dims, const uint16_t* A, const uint16_t* Bt, float* C, CEK_HIDDEN) {              \
    __shared__ __attribute__((aligned(16))) char smem[2 * (WM * 16 * FM + WN * 16 * FN) * 64 * 2]; \
    gemm_tile<WM, WN, FM, FN, MODE>(dims, A, Bt, C, smem, __cek_off);                              \
  }

#define CEK_GEMM_SK_KERNEL(NAME, WM, WN, FM, FN, MODE)                                           \
  extern "C" __global__ __launch_bounds__(64 * WM * WN) void NAME(                                \
      const int* dims, const uint16_t* A, const uint16_t* Bt, float* C, float* W, int* tile_cnt,    \
      CEK_HIDDEN) {                                                                                \
    __shared__ __attribute__((aligned(16))) char smem[2 * (WM * 16 * FM + WN * 16 * FN) * 64 * 2]; \
    gemm_tile<WM, WN, FM, FN, MODE, true>(dims, A, Bt, C, smem, __cek_off, W, tile_cnt);           \
  }

// Split-K ping-pong variants (dims[4] = S splits; K/64 divisible by S):
// strongly scaled slices keep one 256-row tile per CU busy instead of
// leaving CUs idle (8 GPUs × 1024 rows of an 8192² problem = 128 tiles).
CEK_GEMM_SK_KERNEL(cek_sgemm_bf16_256x256pp_sk, 2, 4, 8, 4, 2)
// balanced-DMA split-K (three Bt buffers: 160 KiB LDS)
extern "C" __global__ __launch_bounds__(512) void cek_sgemm_bf16_256x256pb_sk(
    const int* dims, const uint16_t* A, const uint16_t* Bt, float* C, float* W, int* tile_cnt, CEK_HIDDEN) {
  __shared__ __attribute__((aligned(16))) char smem[(2 * 256 + 3 * 256) * 64 * 2];
  gemm_tile<2, 4, 8, 4, 4, true>(dims, A, Bt, C, smem, __cek_off, W, tile_cnt);
}

// uneven split-K = 2 with a one-way hand-over (dims[5] = the helper's
// K-tile deficit): the helper's partial stores overlap the owner's last
// K-tiles instead of both sides' exchange landing at the end of the launch
extern "C" __global__ __launch_bounds__(512) void cek_sgemm_bf16_256x256pb_sw(
    const int* dims, const uint16_t* A, const uint16_t* Bt, float* C, float* W, int* tile_cnt, CEK_HIDDEN) {
  __shared__ __attribute__((aligned(16))) char smem[(2 * 256 + 3 * 256) * 64 * 2];
  gemm_tile<2, 4, 8, 4, 4, true, 3>(dims, A, Bt, C, smem, __cek_off, W, tile_cnt);
}

// the same with the row halves exchanged at the end (XCH 4): the owner's
// tail carries 384 KiB instead of 512, the helper stores half of C
extern "C" __global__ __launch_bounds__(512) void cek_sgemm_bf16_256x256pb_sh(
    const int* dims, const uint16_t* A, const uint16_t* Bt, float* C, float* W, int* tile_cnt, CEK_HIDDEN) {
  __shared__ __attribute__((aligned(16))) char smem[(2 * 256 + 3 * 256) * 64 * 2];
  gemm_tile<2, 4, 8, 4, 4, true, 4>(dims, A, Bt, C, smem, __cek_off, W, tile_cnt);
}

// halves exchanged with both partial stores in flight at once (XCH 5):
// meant for an even split (dims[5] = 0), both sides ending together
extern "C" __global__ __launch_bounds__(512) void cek_sgemm_bf16_256x256pb_ss(
    const int* dims, const uint16_t* A, const uint16_t* Bt, float* C, float* W, int* tile_cnt, CEK_HIDDEN) {
  __shared__ __attribute__((aligned(16))) char smem[(2 * 256 + 3 * 256) * 64 * 2];
  gemm_tile<2, 4, 8, 4, 4, true, 5>(dims, A, Bt, C, smem, __cek_off, W, tile_cnt);
}

#define CEK_GEMM_B3_KERNEL(NAME, WM, WN, FM, FN, MODE)                                              \
  extern "C" __global__ __launch_bounds__(64 * WM * WN) void NAME(                                    \
      const int* dims, const uint16_t* A, const uint16_t* Bt, float* C, CEK_HIDDEN) {                  \
    __shared__ __attribute__((aligned(16))) char smem[(2 * WM * 16 * FM + 3 * WN * 16 * FN) * 64 * 2]; \
    gemm_tile<WM, WN, FM, FN, MODE>(dims, A, Bt, C, smem, __cek_off);                                  \
  }

// Balanced-DMA ping-pong (MODE 4):
// 160 KiB LDS at 256², 128 KiB at 256×128.
CEK_GEMM_B3_KERNEL(cek_sgemm_bf16_256x256pb, 2, 4, 8, 4, 4)
// the same with C row-major ([M][N]) through an LDS turn-around per wave
extern "C" __global__ __launch_bounds__(512) void cek_sgemm_bf16_256x256pbr(
    const int* dims, const uint16_t* A, const uint16_t* Bt, float* C, CEK_HIDDEN) {
  __shared__ __attribute__((aligned(16))) char smem[(2 * 256 + 3 * 256) * 64 * 2];
  gemm_tile<2, 4, 8, 4, 4, false, 0, true>(dims, A, Bt, C, smem, __cek_off);
}
CEK_GEMM_B3_KERNEL(cek_sgemm_bf16_256x128pb, 4, 2, 4, 4, 4)

// Even chunk-split DMA with three whole stages (MODE 6): 144 KiB at 256×128.
extern "C" __global__ __launch_bounds__(512) void cek_sgemm_bf16_256x128pe(
    const int* dims, const uint16_t* A, const uint16_t* Bt, float* C, CEK_HIDDEN) {
  __shared__ __attribute__((aligned(16))) char smem[3 * (256 + 128) * 64 * 2];
  gemm_tile<4, 2, 4, 4, 6>(dims, A, Bt, C, smem, __cek_off);
}

// 256×256 tiles, 8 waves (2×4, 128×64 each), 128 KiB LDS, 1 block/CU.
CEK_GEMM_KERNEL(cek_sgemm_bf16_256x256, 2, 4, 8, 4, 0)
CEK_GEMM_KERNEL(cek_sgemm_bf16_256x256pp, 2, 4, 8, 4, 2)
// 128×128 tiles, 4 waves (2×2, 64×64 each), 64 KiB LDS, 2 blocks/CU.
CEK_GEMM_KERNEL(cek_sgemm_bf16_128x128, 2, 2, 4, 4, 0)
