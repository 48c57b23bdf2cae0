"""Range-partitioned GEMMs: bf16 (the "SGEMM 8192² bf16" config of
BASELINE.json) and fp32 on the fp32 matrix cores.

``C = A · Bᵀ`` with A ``[M][K]`` and Bt ``[N][K]`` bf16 row-major, C fp32 in
tile-major layout (see ``kernels/sgemm_bf16.hip``).  The global range is one
work-group per output tile, so the load balancer splits the problem across
devices in whole tiles and each device's C slice is one contiguous range
(``elements_per_work_item = BM·BN / local``).

``resident=True`` keeps A and B on the devices after the first upload and
leaves C in device memory (the BASELINE "device-resident" number);
``resident=False`` is the reference's host-resident semantics: A and B are
uploaded and every device downloads its C slice on each call.
"""
from __future__ import annotations

import numpy as np

from ..arrays import ClArray
from ..cruncher import ClComputeError, ClNumberCruncher
from .library import library

# tile name -> (BM, BN, work-group size, kernel).  The production tiles and
# at most two tested alternates per dtype; every variant measured and dropped
# in rounds 1-2 is in git history, with its numbers in profiles/gemm_*.md.
TILES = {
    # balanced-DMA ping-pong (G0 stages A, G1 stages Bt two K-tiles ahead):
    # the full-problem tile (1.47-1.50 PF at 8192³)
    "256x256pb": (256, 256, 512, "cek_sgemm_bf16_256x256pb"),
    # the same kernel with C row-major [M][N] (an LDS turn-around per wave in
    # the epilogue): the layout hipBLASLt writes, for like-for-like numbers;
    # device-resident computes only (a device's slice of C is one block of
    # rows only when its tile range is whole tile groups)
    "256x256pbr": (256, 256, 512, "cek_sgemm_bf16_256x256pbr"),
    # uneven split-K = 2 (the helper runs `exchange_shift` K-tiles fewer and
    # hands its whole partial to the owner while the owner still multiplies):
    # the 8-GPU slice (1024 rows of 8192², 128 tiles for 256 CUs).  The
    # hand-over is co-residency-safe: an owner whose helper is late claims
    # the hand-over and multiplies the helper's K-range itself.
    "256x256pbw": (256, 256, 512, "cek_sgemm_bf16_256x256pb_sw"),
    # the same, row halves exchanged at the end: the helper hands over its
    # partial of the owner's half, the owner hands back its partial of the
    # helper's half, each stores one half of C (384 KiB of tail traffic on
    # the owner instead of 512)
    "256x256pbh": (256, 256, 512, "cek_sgemm_bf16_256x256pb_sh"),
    # halves exchanged with an even split: the owner hands its partial back
    # before it waits for the helper's, so both partial stores are in flight
    # together and both sides end their loops together
    "256x256pbs": (256, 256, 512, "cek_sgemm_bf16_256x256pb_ss"),
    # 256×128 fallbacks (twice the tiles): even chunk-split DMA, three stages / balanced DMA
    "256x128pe": (256, 128, 512, "cek_sgemm_bf16_256x128pe"),
    "256x128pb": (256, 128, 512, "cek_sgemm_bf16_256x128pb"),
    # reference structures: one LDS stage in flight / ping-pong wave groups
    # (the latter with a last-arriver split-K variant)
    "256x256": (256, 256, 512, "cek_sgemm_bf16_256x256"),
    "256x256pp": (256, 256, 512, "cek_sgemm_bf16_256x256pp"),
    # small problems: 2 blocks per CU
    "128x128": (128, 128, 256, "cek_sgemm_bf16_128x128"),
}

GEMM_LIBS = ("sgemm_bf16",)

# Wave geometry of every bf16 tile (WM × WN waves, FM × FN 16×16 fragments
# each): the kernels store a C tile in fragment order (one dwordx4 per lane
# per fragment), which tile_to_rows / rows_to_tile convert.
TILE_WAVES = {
    "256x256pb": (2, 4, 8, 4), "256x256pbr": (2, 4, 8, 4), "256x256pbw": (2, 4, 8, 4), "256x256pbh": (2, 4, 8, 4), "256x256pbs": (2, 4, 8, 4), "256x256": (2, 4, 8, 4), "256x256pp": (2, 4, 8, 4),
    "256x128pe": (4, 2, 4, 4), "256x128pb": (4, 2, 4, 4), "128x128": (2, 2, 4, 4),
}


def tile_to_rows(t: np.ndarray, geom) -> np.ndarray:
    """Fragment-ordered C tiles (``[..., BM·BN]``) → row-major ``[..., BM, BN]``.
    In-tile offset of (row, col) = ((((wr·WN + wc)·FM + i)·FN + j)·64 + fq·16 + fr)·4 + r
    with row = wr·16FM + i·16 + fq·4 + r and col = wc·16FN + j·16 + fr."""
    WM, WN, FM, FN = geom
    lead = t.shape[:-1]
    x = t.reshape(lead + (WM, WN, FM, FN, 4, 16, 4))
    n = len(lead)
    perm = list(range(n)) + [n + 0, n + 2, n + 4, n + 6, n + 1, n + 3, n + 5]
    return x.transpose(perm).reshape(lead + (WM * FM * 16, WN * FN * 16))


def rows_to_tile(b: np.ndarray, geom) -> np.ndarray:
    """Inverse of :func:`tile_to_rows`: row-major ``[..., BM, BN]`` → fragment order."""
    WM, WN, FM, FN = geom
    lead = b.shape[:-2]
    x = b.reshape(lead + (WM, FM, 4, 4, WN, FN, 16))  # wr i fq r wc j fr
    n = len(lead)
    perm = list(range(n)) + [n + 0, n + 4, n + 1, n + 5, n + 2, n + 6, n + 3]
    return np.ascontiguousarray(x.transpose(perm)).reshape(lead + (-1,))

# fp32 tiles (kernels/sgemm_f32.hip): v_mfma_f32_16x16x4_f32, BK = 32
F32_TILES = {
    # production: register-direct, 8 waves of 128×64 — fragments loaded
    # global → VGPR, no LDS, no barrier — with the next block's loads spread
    # evenly over the current block's MFMA groups (152.8 TF at 8192³ vs
    # hipBLASLt 152.8 on one box, 152.0 / 151.7 vs 152.0 on another, where
    # the first-half spread g8h ran 151.2 / 150.6; profiles/round4_session5.md,
    # round4_session6.md)
    "256x256g8i": (256, 256, 512, "cek_sgemm_f32_256x256g8i"),
    # the same loads spread over the first half / quarter of the groups
    "256x256g8h": (256, 256, 512, "cek_sgemm_f32_256x256g8h"),
    "256x256g8q": (256, 256, 512, "cek_sgemm_f32_256x256g8q"),
    # burst loads ahead of each block's MFMAs (151.4 TF vs hipBLASLt 153.4 on
    # another box, 256x256ir 138.6 there)
    "256x256g8": (256, 256, 512, "cek_sgemm_f32_256x256g8"),
    # LDS-staged: k block 1's fragment reads between block 0's MFMA groups
    # (146-147 TF at 8192³ on earlier boxes)
    "256x256ir": (256, 256, 512, "cek_sgemm_f32_256x256ir"),
    # alternates: the barrier ahead of the last MFMA groups; v_mfma_f32_32x32x2_f32
    "256x256ib7": (256, 256, 512, "cek_sgemm_f32_256x256ib7"),
    "256x256w": (256, 256, 512, "cek_sgemm_f32_256x256w"),
    # 256×128: every LDS-DMA piece within the first k block's MFMAs
    "256x128ie": (256, 128, 512, "cek_sgemm_f32_256x128ie"),
    # plain one-stage-in-flight structures
    "256x256": (256, 256, 512, "cek_sgemm_f32_256x256"),
    "256x128": (256, 128, 512, "cek_sgemm_f32_256x128"),
    # register-direct: fragments global → VGPR, no LDS, no barrier; 4 waves
    # of 128×128 (one per SIMD) or 8 of 128×64; t = phases ordered by
    # fragment ties instead of scheduling barriers
    "256x256g": (256, 256, 256, "cek_sgemm_f32_256x256g"),
    "256x256gt": (256, 256, 256, "cek_sgemm_f32_256x256gt"),
    "256x256gh": (256, 256, 256, "cek_sgemm_f32_256x256gh"),  # 4-wave form of g8h
    "256x256g8t": (256, 256, 512, "cek_sgemm_f32_256x256g8t"),
    "128x128": (128, 128, 256, "cek_sgemm_f32_128x128"),
}

# tiles whose kernel stores C row-major ([M][N]) instead of tile-major
ROW_MAJOR_TILES = {"256x256pbr"}
# tiles with a split-K kernel variant ("<kernel>_sk", arrays + W + counters)
SPLIT_K_TILES = {"256x256pp", "256x256pb"}
# tiles whose kernel always runs two K-splits with a hand-over (flag words per tile)
EXCHANGE_TILES = {"256x256pbw": 4, "256x256pbh": 4, "256x256pbs": 4}
# K-tile deficit of the helper split (dims[5]): it hands its whole partial
# over and leaves while the owner still multiplies
EXCHANGE_SHIFT = {"256x256pbw": 4, "256x256pbh": 4, "256x256pbs": 0}


def to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """fp32 → bf16 bit patterns (round to nearest even), as uint16."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return r


def from_bf16_bits(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << 16).view(np.float32)


def tile_coords(t: np.ndarray, M: int, N: int, BM: int, BN: int, group_m: int, panels: int = 0):
    """Tile index → (tile row, tile col) under the kernel's order
    (``cek_tile_coords`` in kernels/cek_kernel.h): grouped rows, or square
    shells of ``panels`` row panels (shell s = R_s then C_s)."""
    t = np.asarray(t)
    ntm, ntn = M // BM, N // BN

    def grouped(r, rows, cols):
        gm = max(1, group_m)
        per = gm * cols
        first = (r // per) * gm
        gsz = np.minimum(rows - first, gm)
        in_g = r % per
        return first + in_g % gsz, in_g // gsz

    if panels <= 0:
        return grouped(t, ntm, ntn)
    pm, pn = ntm // panels, ntn // panels
    tm = np.empty_like(t)
    tn = np.empty_like(t)
    s = np.floor(np.sqrt(t // (pm * pn))).astype(np.int64)
    s = np.where((s + 1) ** 2 * pm * pn <= t, s + 1, s)
    s = np.where(s * s * pm * pn > t, s - 1, s)
    r = t - s * s * pm * pn
    r_tiles = pm * (s + 1) * pn
    for sh in np.unique(s):
        sel = s == sh
        rr = r[sel]
        isr = rr < r_tiles[sel]
        a, b = grouped(rr[isr], pm, (sh + 1) * pn)
        c, d = grouped(rr[~isr] - pm * (sh + 1) * pn, max(sh * pm, 1), pn)
        out_m = np.empty(rr.shape, t.dtype)
        out_n = np.empty(rr.shape, t.dtype)
        out_m[isr], out_n[isr] = a + sh * pm, b
        out_m[~isr], out_n[~isr] = c, d + sh * pn
        tm[sel], tn[sel] = out_m, out_n
    return tm, tn


def untile(c: np.ndarray, M: int, N: int, BM: int, BN: int, group_m: int = 1, geom=None,
           panels: int = 0) -> np.ndarray:
    """Tile-major C (the kernel's tile order) → row-major [M][N]; ``geom``:
    the tile's wave geometry when its elements are in fragment order (bf16
    kernels), None for row-major tiles; ``panels``: shell order."""
    ntm, ntn = M // BM, N // BN
    tiles = c.reshape(ntm * ntn, BM, BN) if geom is None else tile_to_rows(c.reshape(ntm * ntn, BM * BN), geom)
    tm, tn = tile_coords(np.arange(ntm * ntn), M, N, BM, BN, group_m, panels)
    out = np.empty((ntm, ntn, BM, BN), c.dtype)
    out[tm, tn] = tiles
    return out.transpose(0, 2, 1, 3).reshape(M, N)


class GemmBf16:
    def __init__(self, M: int, N: int, K: int, devices=None, tile: str = "256x256",
                 cruncher: ClNumberCruncher | None = None, fill: str = "random", seed: int = 0,
                 group_m: int = 4, split_k: int = 1, wave_granularity: bool | None = None,
                 exchange_shift: int | None = None, handover_spin_limit: int = 0):
        BM, BN, L, kname = TILES[tile]
        self.tile = tile
        if M % BM or N % BN or K % 64:
            raise ValueError(f"M%{BM}, N%{BN} and K%64 must be 0 (got {M},{N},{K})")
        if split_k > 1:
            if tile not in SPLIT_K_TILES:
                raise ValueError(f"split-K is available for tiles {sorted(SPLIT_K_TILES)}")
            if (K // 64) % split_k:
                raise ValueError(f"K/64 ({K // 64}) must be divisible by split_k ({split_k})")
            kname = kname + "_sk"
        self.exchange = tile in EXCHANGE_TILES
        shift = 0
        if self.exchange:
            if (K // 64) % 2:
                raise ValueError(f"K/64 ({K // 64}) must be even for tile {tile}")
            split_k = 2
            if tile in EXCHANGE_SHIFT:
                shift = EXCHANGE_SHIFT[tile] if exchange_shift is None else int(exchange_shift)
                shift = max(0, min(shift, K // 128 - 1))  # the helper keeps >= 1 K-tile
        self.exchange_shift = shift
        self.M, self.N, self.K, self.BM, self.BN, self.L, self.kernel = M, N, K, BM, BN, L, kname
        self.geom = TILE_WAVES[tile]  # C tiles in fragment order
        self.row_major_c = tile in ROW_MAJOR_TILES
        self.split_k = max(1, int(split_k))
        self.tiles = (M // BM) * (N // BN)
        self.global_range = self.tiles * self.split_k * L
        self.cr = cruncher or ClNumberCruncher(devices, "", prebuilt=library(*GEMM_LIBS))
        self.group_m = group_m
        # dims[7]: the owner's wait for the helper's partial, in polls (0: the
        # kernel default, 65536; -1: the owner claims at once, -2 (halves
        # tile): the helper claims the hand-back at once — forced fall-backs)
        self.dims = ClArray(np.array([M, N, K, group_m, self.split_k, shift, 0, int(handover_spin_limit)], np.int32))
        self.dims.write = False
        self.A = ClArray(M * K, "bfloat16")
        self.B = ClArray(N * K, "bfloat16")
        self.C = ClArray(M * N, np.float32)
        for a in (self.A, self.B):
            a.write = False
        self.C.read = False
        self.C.elements_per_work_item = BM * BN // (L * self.split_k)
        self.extra = []
        if self.split_k > 1:
            # per-work-group partial tiles (device-only scratch: never transferred;
            # np.empty leaves the host pages untouched) and per-tile arrival counters
            # (exchange tiles: one tile of partial halves per tile, two ready
            # flags per tile and a spin-timeout counter at the end)
            wtiles = self.tiles if self.exchange else self.tiles * self.split_k
            self.W = ClArray(np.empty(wtiles * BM * BN, np.float32))
            self.W.read = self.W.write = False
            nflags = EXCHANGE_TILES[tile] * self.tiles + 1 if self.exchange else self.tiles
            self.counters = ClArray(np.zeros(nflags, np.int32))
            self.counters.write = False
            self.extra = [self.W, self.counters]
        if fill == "random":
            rng = np.random.default_rng(seed)
            self.A.array[:] = to_bf16_bits(rng.uniform(-1, 1, M * K).astype(np.float32))
            self.B.array[:] = to_bf16_bits(rng.uniform(-1, 1, N * K).astype(np.float32))
        self._uploaded = False
        self.wave_granularity = wave_granularity
        self._orders = {}  # compute id -> shell panels of its tile order (0: grouped)

    def granularity(self) -> int:
        """Balancer unit in work items.  One tile (all its K-splits) by
        default.  On identical GPUs whose slices are whole waves of tiles
        (``work-groups % CUs == 0`` and at least one wave per device), the unit
        is one wave: one work-group per CU.  With 256 CUs and exactly one
        wave of tiles per device (8192² at 4 or 8 GPUs), a one-tile step would
        let timing noise hand a device 257 tiles, which costs it a second
        round of tiles and doubles its time.  A split in whole waves cannot do
        that.  ``wave_granularity`` forces the choice (None = auto)."""
        tile_unit = self.L * self.split_k
        devs = [d for d in self.cr.devices]
        if self.wave_granularity is False or not devs:
            return tile_unit
        cus = {d.compute_units for d in devs}
        gpus = all(d.is_gpu for d in devs)
        if self.wave_granularity is None and not (gpus and len(cus) == 1):
            return tile_unit
        cu = min(cus)
        groups = self.tiles * self.split_k
        ndev = self.cr.number_of_devices or len(devs)
        if cu <= 0 or groups % cu or groups // cu < ndev:
            return tile_unit
        # a wave of tiles must keep a tile's K-splits together
        return cu * self.L if cu % self.split_k == 0 else tile_unit

    @property
    def flops(self) -> float:
        return 2.0 * self.M * self.N * self.K

    def _group_work_items(self) -> int:
        """Work items of one tile group (``group_m`` tile rows × every tile
        column): the unit whose A rows form one contiguous panel."""
        return self.group_m * (self.N // self.BN) * self.L * self.split_k

    def can_stream(self) -> bool:
        """Host-resident streaming needs whole tile groups (A row panels) per
        blob and an integral A panel per work item."""
        ntm, ntn = self.M // self.BM, self.N // self.BN
        per_wi = self.BM * self.K
        return (self.split_k == 1 and ntm % self.group_m == 0
                and per_wi % (ntn * self.L) == 0)

    def run(self, compute_id: int = 1, resident: bool = True, stream_blobs: int = 0,
            stream_event: bool = True) -> None:
        """One GEMM through compute().  ``resident``: A/B stay on the devices
        after the first call and C stays in device memory.  ``stream_blobs``
        (host-resident only): run the call through the event-driven
        read/compute/write pipeline (Cores.cs:1197-1367) in that many blobs
        per device — B is a full read, A goes up one row panel per blob
        (``partial``) and every blob's C tiles come down while later blobs'
        panels upload and compute, on the two half-pipelines' streams."""
        if self.row_major_c and not resident:
            raise ValueError("row-major C tiles run device-resident computes only")
        if self.split_k > 1 and self.cr.enqueue_mode and self.cr.enqueue_mode_async_enable:
            # computes on async queues run concurrently; two launches of one
            # split-K GEMM would share its partial tiles and hand-over words
            raise ClComputeError("split-K / exchange GEMM tiles cannot run on async enqueue queues "
                                 "(concurrent launches would share the partial-tile workspace); "
                                 "use a single-pass tile such as 256x256pb")
        first = not self._uploaded
        self._orders[compute_id] = 0
        streamed = bool(stream_blobs) and not resident
        if streamed and not self.can_stream():
            raise ValueError("stream_blobs needs split_k == 1, whole tile groups and an integral A panel "
                             "per work item")
        for a in (self.dims, self.A, self.B):
            a.read = first or not resident
        self.A.partial_read = streamed
        # an A row panel of one tile group spans group_m·BM rows; per work item
        self.A.elements_per_work_item = (self.BM * self.K) // ((self.N // self.BN) * self.L) if streamed else 1
        if self.split_k > 1:
            self.counters.read = first  # zeroed once; the kernel re-arms them
        self.C.write = not resident
        gran = self.granularity()
        if streamed:
            gran = self._group_work_items()
        self.dims.next_param(self.A, self.B, self.C, *self.extra).compute(
            self.cr, compute_id, self.kernel, self.global_range, self.L,
            pipeline=streamed, pipeline_type=stream_event, pipeline_blobs=max(1, stream_blobs),
            granularity=gran)
        self._uploaded = True

    def shell_bounds(self, panels: int, split_last: int = 0):
        """Work-item bounds of the square shells (blob s = shell s) and the
        per-blob row panels of A and B, for :meth:`run_shells`.  The last
        ``split_last`` shells become two blobs each, ``R_s`` (which uploads
        panels A_s and B_s) and ``C_s`` (no upload), so ``R_s``'s C tiles
        come down while ``C_s`` multiplies: the call's tail after the last
        upload is ``C_s`` alone."""
        P = int(panels)
        if self.split_k != 1:
            raise ValueError("shell streaming runs single-pass tiles (split_k == 1)")
        if P < 1 or self.M % P or self.N % P or (self.M // P) % self.BM or (self.N // P) % self.BN:
            raise ValueError(f"M and N must split into {P} panels of whole {self.BM}x{self.BN} tiles")
        pm, pn = self.M // P // self.BM, self.N // P // self.BN
        a_rows, b_rows = self.M // P, self.N // P
        unit = pm * pn * self.L  # work items of one panel × panel block
        bounds, a_sl, b_sl = [0], [], []
        for k in range(P):
            a_panel, b_panel = (k * a_rows * self.K, a_rows * self.K), (k * b_rows * self.K, b_rows * self.K)
            if k >= P - int(split_last) and k > 0:
                bounds += [(k * k + k + 1) * unit, (k + 1) * (k + 1) * unit]  # R_k, then C_k
                a_sl += [a_panel, (0, 0)]
                b_sl += [b_panel, (0, 0)]
            else:
                bounds.append((k + 1) * (k + 1) * unit)
                a_sl.append(a_panel)
                b_sl.append(b_panel)
        return bounds, a_sl, b_sl

    def run_shells(self, panels: int = 16, compute_id: int = 2, split_last: int = 0) -> None:
        """One host-resident call through ``compute()``: the event-driven
        read/compute/write pipeline with explicit, uneven blobs — blob s is
        square shell s (``R_s = A_s·B[0..s]ᵀ`` then ``C_s = A[0..s-1]·B_sᵀ``,
        the kernels' shell tile order, ``dims[6] = panels``), A and B go up
        one row panel per blob (``ClArray.blob_slices``) on the upload stream
        and every shell's C comes down (one contiguous range) while later
        panels go up.  The first kernels need two panels instead of all of
        B.  One device holds the range (several: the plain path)."""
        bounds, a_sl, b_sl = self.shell_bounds(panels, split_last)
        if getattr(self, "_dims_shell", None) is None or int(self._dims_shell.array[6]) != panels:
            d = self.dims.array.copy()
            d[6] = panels
            self._dims_shell = ClArray(d)
            self._dims_shell.write = False
        self._orders[compute_id] = int(panels)
        saved = [(a.read, a.partial_read, a.blob_slices) for a in (self.A, self.B)]
        try:
            for a, sl in ((self.A, a_sl), (self.B, b_sl)):
                a.partial_read = True
                a.blob_slices = sl
            self.C.write = True
            self._dims_shell.read = True
            self._dims_shell.next_param(self.A, self.B, self.C).compute(
                self.cr, compute_id, self.kernel, self.global_range, self.L, pipeline=True,
                pipeline_blobs=bounds, granularity=self.granularity())
        finally:
            for a, (r, pr, bs) in zip((self.A, self.B), saved):
                a.partial_read, a.blob_slices = pr, bs
                a.read = r
        self._uploaded = False  # the device copies of A/B were streamed, not kept whole

    def run_host_shells(self, panels: int = 8, device: int = 0) -> None:
        """One host-resident call streamed in square shells
        (``Cores::gemm_host_shells``, ``csrc/shell_gemm.cpp``): A and B go up
        in ``panels`` row panels each (A0 B0 A1 B1 …), shell s's two GEMMs
        (``A_s·B[0..s]ᵀ`` and ``A[0..s-1]·B_sᵀ``) run once panels s have
        landed, and each shell's C comes down while later panels go up.
        Unlike the 1-D blob pipeline, the first kernels need only two panels
        instead of all of B.  One GPU of the cruncher; the host C is in shell
        layout (:meth:`shells_result`)."""
        if self.split_k != 1:
            raise ValueError("shell streaming runs single-pass tiles (split_k == 1)")
        pm, pn = self.M // max(1, panels), self.N // max(1, panels)
        if panels < 1 or self.M % panels or self.N % panels or pm % self.BM or pn % self.BN:
            raise ValueError(f"M and N must split into {panels} panels of whole {self.BM}x{self.BN} tiles")
        self.cr.cores.gemm_host_shells(device, self.kernel, self.A._spec(), self.B._spec(), self.C._spec(),
                                       self.M, self.N, self.K, panels, self.group_m, self.BM, self.BN, self.L)

    def shells_result(self, panels: int = 8) -> np.ndarray:
        """Row-major fp32 C from the host C of :meth:`run_host_shells`
        (shell by shell: ``R_s`` then ``C_s``, each tile-major)."""
        pm, pn = self.M // panels, self.N // panels
        out = np.empty((self.M, self.N), np.float32)
        c, off = self.C.array, 0
        for s in range(panels):
            m, n = pm, (s + 1) * pn
            out[s * pm:(s + 1) * pm, :n] = untile(c[off:off + m * n], m, n, self.BM, self.BN, self.group_m, self.geom)
            off += m * n
            if s:
                m, n = s * pm, pn
                out[:s * pm, s * pn:(s + 1) * pn] = untile(c[off:off + m * n], m, n, self.BM, self.BN, self.group_m, self.geom)
                off += m * n
        return out

    def verify_shells(self, panels: int = 8, samples: int = 16, seed: int = 2) -> float:
        """Max relative error of sampled 256-row × 256-column blocks of
        :meth:`shells_result` against a float64 host product."""
        c = self.shells_result(panels)
        a, b = self.A.array, self.B.array
        a = (from_bf16_bits(a) if a.dtype == np.uint16 else a).reshape(self.M, self.K)
        b = (from_bf16_bits(b) if b.dtype == np.uint16 else b).reshape(self.N, self.K)
        rng = np.random.default_rng(seed)
        worst = 0.0
        for _ in range(samples):
            r = int(rng.integers(0, self.M // 256)) * 256
            q = int(rng.integers(0, self.N // 256)) * 256
            ref = a[r:r + 256].astype(np.float64) @ b[q:q + 256].astype(np.float64).T
            worst = max(worst, float(np.abs(c[r:r + 256, q:q + 256] - ref).max() / max(np.abs(ref).max(), 1e-30)))
        return worst

    def verify_shells_full(self, panels: int = 8, device=None) -> tuple:
        """Every element of :meth:`shells_result` against a float64 product
        computed by torch on ``device``: ``(max_rel_err, blocks_checked)``,
        the error per BM×BN block relative to that block's ``max |ref|``."""
        import torch

        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else (
                torch.device("cpu"))
        c = torch.from_numpy(self.shells_result(panels)).to(device)
        ref = self._reference_t(device)
        ntm, ntn = self.M // self.BM, self.N // self.BN
        got = c.view(ntm, self.BM, ntn, self.BN).double()
        want = ref.view(ntm, self.BM, ntn, self.BN)
        err = (got - want).abs().amax(dim=(1, 3)) / want.abs().amax(dim=(1, 3)).clamp_min(1e-30)
        return float(err.max()), ntm * ntn

    def _reference_t(self, device):
        """C = A·Bᵀ in float64 on a torch device (row-major [M][N])."""
        import torch

        def operand(arr, rows):
            x = arr.array
            if x.dtype == np.uint16:  # bf16 bit patterns
                t = torch.from_numpy(x.view(np.int16)).to(device).view(torch.bfloat16)
            else:
                t = torch.from_numpy(x).to(device)
            return t.reshape(rows, self.K).double()

        return operand(self.A, self.M) @ operand(self.B, self.N).T

    def result(self, download: bool = True) -> np.ndarray:
        """Row-major fp32 C (downloads every device's slice when resident)."""
        if download:
            rng = self.cr.ranges(self.cr._cores.last_compute_id)
            refs = self.cr.references(self.cr._cores.last_compute_id)
            e = self.C.elements_per_work_item
            for dev in range(self.cr._cores.num_devices):
                g = self.cr._cores.global_base + dev
                lo, n = refs[g] * e, rng[g] * e
                self._download_slice(dev, lo, n)
        if getattr(self, "row_major_c", False):
            return self.C.array.reshape(self.M, self.N).copy()
        return untile(self.C.array, self.M, self.N, self.BM, self.BN, self.group_m, self.geom,
                      self._orders.get(self.cr._cores.last_compute_id, 0))

    def tile_block(self, flat: np.ndarray) -> np.ndarray:
        """One C tile as stored (``BM·BN`` floats) → row-major ``[BM][BN]``."""
        return flat.reshape(self.BM, self.BN) if self.geom is None else tile_to_rows(flat, self.geom)

    def handover_fallbacks(self) -> int:
        """Exchange tiles only: how many owners found their helper's partial
        missing after the bounded wait and multiplied the helper's K-range
        themselves (summed over devices and calls).  C is correct either way;
        a nonzero count means the GPU was shared (helpers not co-resident)
        and those tiles ran at half speed."""
        if not self.exchange:
            return 0
        total = 0
        for dev in range(self.cr._cores.num_devices):
            self.cr.download(self.counters, dev)
            total += int(self.counters.array[-1])
        return total

    spin_timeouts = handover_fallbacks  # round-3 name

    def verify(self, compute_id: int = 1, tiles_per_device: int = 8, seed: int = 1,
               host: bool = False) -> float:
        """Max relative error of the device-resident C of ``compute_id``
        against a float64 host product, over sampled output tiles of this
        process's devices' ranges: the first and last tile of each range plus
        random ones.  Relative to ``max |ref|`` of each tile.  Downloads each
        local device's C replica (device memory is not changed).
        ``host=True`` checks the host C instead (a host-resident call's
        downloaded slices), without downloading."""
        ranges = self.cr.ranges(compute_id)
        refs = self.cr.references(compute_id)
        unit = self.L * self.split_k
        a = from_bf16_bits(self.A.array).reshape(self.M, self.K) if self.A.array.dtype == np.uint16 else (
            self.A.array.reshape(self.M, self.K))
        b = from_bf16_bits(self.B.array).reshape(self.N, self.K) if self.B.array.dtype == np.uint16 else (
            self.B.array.reshape(self.N, self.K))
        rng = np.random.default_rng(seed)
        saved = self.C.array.copy()
        worst = 0.0
        tile = self.BM * self.BN
        for dev in range(self.cr._cores.num_devices):
            g = self.cr._cores.global_base + dev
            t0, nt = refs[g] // unit, ranges[g] // unit
            if nt == 0:
                continue
            if not host:
                self.cr.download(self.C, dev)
            picks = {t0, t0 + nt - 1}
            picks.update((t0 + rng.choice(nt, size=min(nt, tiles_per_device), replace=False)).tolist())
            picks = np.array(sorted(picks))
            tm, tn = tile_coords(picks, self.M, self.N, self.BM, self.BN, self.group_m,
                                 self._orders.get(compute_id, 0))
            for t, r, c in zip(picks, tm, tn):
                if getattr(self, "row_major_c", False):
                    got = self.C.array.reshape(self.M, self.N)[r * self.BM:(r + 1) * self.BM,
                                                               c * self.BN:(c + 1) * self.BN].astype(np.float64)
                else:
                    got = self.tile_block(self.C.array[t * tile:(t + 1) * tile]).astype(np.float64)
                ref = (a[r * self.BM:(r + 1) * self.BM].astype(np.float64)
                       @ b[c * self.BN:(c + 1) * self.BN].astype(np.float64).T)
                worst = max(worst, float(np.max(np.abs(got - ref)) / max(float(np.max(np.abs(ref))), 1e-30)))
        self.C.array[:] = saved
        return worst

    def verify_full(self, compute_id: int = 1, host: bool = False, device=None) -> tuple:
        """Whole-output check: EVERY C tile this process's devices own under
        the split of ``compute_id``, against a float64 product computed by
        torch on ``device`` (default: torch's current GPU, else the CPU).
        Each local device's C replica is downloaded (``host=True``: the host C
        of a host-resident call is checked as it is), untiled on ``device``
        and compared tile by tile.  Returns ``(max_rel_err, tiles_checked)``;
        the error of a tile is ``max |C - ref| / max |ref|`` over the tile."""
        import torch

        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else (
                torch.device("cpu"))
        M, N, BM, BN = self.M, self.N, self.BM, self.BN
        ntm, ntn = M // BM, N // BN
        ref = self._reference_t(device)  # [M][N] float64
        ref_tiles = ref.view(ntm, BM, ntn, BN).permute(0, 2, 1, 3)  # [ntm][ntn][BM][BN]
        del ref
        ranges = self.cr.ranges(compute_id)
        refs = self.cr.references(compute_id)
        unit = self.L * self.split_k
        saved = self.C.array.copy()
        worst, checked = 0.0, 0
        try:
            for dev in range(self.cr._cores.num_devices):
                g = self.cr._cores.global_base + dev
                t0, nt = refs[g] // unit, ranges[g] // unit
                if nt == 0:
                    continue
                if not host:
                    self.cr.download(self.C, dev)
                tm, tn = tile_coords(np.arange(t0, t0 + nt), M, N, BM, BN, self.group_m,
                                     self._orders.get(compute_id, 0))
                tm_t = torch.from_numpy(np.asarray(tm, np.int64)).to(device)
                tn_t = torch.from_numpy(np.asarray(tn, np.int64)).to(device)
                c = torch.from_numpy(self.C.array).to(device)
                if getattr(self, "row_major_c", False):
                    got = c.view(ntm, BM, ntn, BN).permute(0, 2, 1, 3)[tm_t, tn_t]
                else:
                    flat = c.view(-1, BM * BN)[t0:t0 + nt]
                    if self.geom is None:
                        got = flat.view(nt, BM, BN)
                    else:
                        WM, WN, FM, FN = self.geom
                        got = flat.view(nt, WM, WN, FM, FN, 4, 16, 4).permute(0, 1, 3, 5, 7, 2, 4, 6).reshape(nt, BM, BN)
                want = ref_tiles[tm_t, tn_t]
                err = (got.double() - want).abs().amax(dim=(1, 2)) / want.abs().amax(dim=(1, 2)).clamp_min(1e-30)
                worst = max(worst, float(err.max()))
                checked += nt
                del c, got, want, err
        finally:
            self.C.array[:] = saved
        return worst, checked

    def _download_slice(self, dev: int, lo: int, n: int) -> None:
        # a sub-view ClArray sharing the same uid would alias buffers; the
        # native download copies the whole replica, slice afterwards
        tmp = np.empty_like(self.C.array)
        saved = self.C.array.copy()
        self.cr.download(self.C, dev)
        tmp[:] = self.C.array
        self.C.array[:] = saved
        self.C.array[lo:lo + n] = tmp[lo:lo + n]

    def reference(self, rows: slice = slice(None)) -> np.ndarray:
        a = from_bf16_bits(self.A.array).reshape(self.M, self.K)[rows].astype(np.float64)
        b = from_bf16_bits(self.B.array).reshape(self.N, self.K).astype(np.float64)
        return a @ b.T


class GemmF32(GemmBf16):
    """``C = A · Bᵀ`` in fp32 on the fp32 matrix cores (``v_mfma_f32_16x16x4_f32``):
    A ``[M][K]``, Bt ``[N][K]`` and C fp32, C tile-major like :class:`GemmBf16`
    (same grouped tile order, so the same range partitioning and
    wave-quantized balancing apply)."""

    def __init__(self, M: int, N: int, K: int, devices=None, tile: str = "256x256g8i",
                 cruncher: ClNumberCruncher | None = None, fill: str = "random", seed: int = 0,
                 group_m: int = 4, wave_granularity: bool | None = None):
        BM, BN, L, kname = F32_TILES[tile]
        self.tile = tile
        if M % BM or N % BN or K % 32:
            raise ValueError(f"M%{BM}, N%{BN} and K%32 must be 0 (got {M},{N},{K})")
        self.M, self.N, self.K, self.BM, self.BN, self.L, self.kernel = M, N, K, BM, BN, L, kname
        self.geom = None  # the fp32 kernels store C tiles row-major
        self.row_major_c = False
        self.exchange = False
        self.split_k = 1
        self.tiles = (M // BM) * (N // BN)
        self.global_range = self.tiles * L
        self.cr = cruncher or ClNumberCruncher(devices, "", prebuilt=library("sgemm_f32"))
        self.group_m = group_m
        self.dims = ClArray(np.array([M, N, K, group_m, 1, 0, 0, 0], np.int32))
        self.dims.write = False
        self.A = ClArray(M * K, np.float32)
        self.B = ClArray(N * K, np.float32)
        self.C = ClArray(M * N, np.float32)
        for a in (self.A, self.B):
            a.write = False
        self.C.read = False
        self.C.elements_per_work_item = BM * BN // L
        self.extra = []
        if fill == "random":
            rng = np.random.default_rng(seed)
            self.A.array[:] = rng.uniform(-1, 1, M * K).astype(np.float32)
            self.B.array[:] = rng.uniform(-1, 1, N * K).astype(np.float32)
        self._uploaded = False
        self.wave_granularity = wave_granularity
        self._orders = {}

    def reference(self, rows: slice = slice(None)) -> np.ndarray:
        a = self.A.array.reshape(self.M, self.K)[rows].astype(np.float64)
        b = self.B.array.reshape(self.N, self.K).astype(np.float64)
        return a @ b.T
