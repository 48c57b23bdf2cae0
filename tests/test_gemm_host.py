"""Host-side logic of the GEMM ops (no GPU): object set-up for every tile,
the shell decomposition, tile orders and the guards that run before any
kernel does."""
import numpy as np
import pytest

import cekirdekler_amd as ck
from cekirdekler_amd.ops.gemm import F32_TILES, TILES, GemmBf16, GemmF32, tile_coords


@pytest.fixture(scope="module")
def cpu_cr():
    cr = ck.ClNumberCruncher(ck.ClPlatforms.all().cpus(True), "__global__ void nop(float* x) {}")
    yield cr
    cr.dispose()


@pytest.mark.parametrize("tile", sorted(TILES))
def test_bf16_objects(cpu_cr, tile):
    g = GemmBf16(512, 512, 256, cruncher=cpu_cr, tile=tile)
    assert g.row_major_c == (tile == "256x256pbr")
    assert g.global_range == g.tiles * g.split_k * g.L
    if g.row_major_c:
        with pytest.raises(ValueError):
            g.run(resident=False)


@pytest.mark.parametrize("tile", sorted(F32_TILES))
def test_f32_objects(cpu_cr, tile):
    g = GemmF32(512, 512, 256, cruncher=cpu_cr, tile=tile)
    assert not g.row_major_c and not g.exchange


def test_shell_bounds_cover_every_tile(cpu_cr):
    g = GemmBf16(2048, 2048, 256, cruncher=cpu_cr, tile="256x256pb")
    bounds, a_sl, b_sl = g.shell_bounds(4)
    assert bounds[0] == 0 and bounds[-1] == g.global_range
    assert len(a_sl) == len(b_sl) == 4
    assert sum(n for _, n in a_sl) == g.A.N and sum(n for _, n in b_sl) == g.B.N
    # blob s holds exactly the tiles of shell s, which need panels 0..s only
    t = np.arange(g.tiles)
    tm, tn = tile_coords(t, 2048, 2048, 256, 256, g.group_m, 4)
    assert len(set(zip(tm.tolist(), tn.tolist()))) == g.tiles
    for s in range(4):
        lo, hi = bounds[s] // g.L, bounds[s + 1] // g.L
        assert tm[lo:hi].max() < (s + 1) * 2 and tn[lo:hi].max() < (s + 1) * 2
        assert ((tm[lo:hi] // 2 == s) | (tn[lo:hi] // 2 == s)).all()
    with pytest.raises(ValueError):
        g.shell_bounds(3)


@pytest.mark.parametrize("split_last", [1, 2, 4])
def test_shell_bounds_split_last_shells(cpu_cr, split_last):
    """The last shells split into R_s (row panel s, which uploads A_s and B_s)
    and C_s (column panel s above it, no upload); every blob holds exactly
    its part's tiles and only R_s blobs upload."""
    g = GemmBf16(2048, 2048, 256, cruncher=cpu_cr, tile="256x256pb")
    P, pt = 4, 2  # 4 panels of 2 tiles each way
    bounds, a_sl, b_sl = g.shell_bounds(P, split_last)
    nsplit = min(split_last, P - 1)
    assert len(bounds) == P + 1 + nsplit and bounds[-1] == g.global_range
    assert sum(n for _, n in a_sl) == g.A.N and sum(n for _, n in b_sl) == g.B.N
    t = np.arange(g.tiles)
    tm, tn = tile_coords(t, 2048, 2048, 256, 256, g.group_m, P)
    q = 0
    for s in range(P):
        parts = ("R", "C") if s >= P - split_last and s > 0 else ("RC",)
        for part in parts:
            lo, hi = bounds[q] // g.L, bounds[q + 1] // g.L
            rows, cols = tm[lo:hi] // pt, tn[lo:hi] // pt
            if part == "R":
                assert (rows == s).all() and (cols <= s).all() and hi - lo == (s + 1) * pt * pt
                assert a_sl[q][1] > 0 and b_sl[q][1] > 0
            elif part == "C":
                assert (cols == s).all() and (rows < s).all() and hi - lo == s * pt * pt
                assert a_sl[q][1] == 0 and b_sl[q][1] == 0
            else:
                assert ((rows == s) | (cols == s)).all()
            q += 1


def test_explicit_blob_count_does_not_stretch_the_range():
    """Explicit blob bounds whose count does not divide the range (split
    shells: 6 blobs over 16 tiles) leave the one device's range at exactly the
    global range; the equal-blob step (blobs × unit) once rounded it up to
    18 tiles, launching two work-groups past C."""
    src = ("__global__ void cek_sgemm_bf16_256x256pb(const int* d, const unsigned short* a, "
           "const unsigned short* b, float* c) {}")
    cr = ck.ClNumberCruncher(ck.ClPlatforms.all().cpus(True), src)
    g = GemmBf16(1024, 1024, 512, cruncher=cr, tile="256x256pb")
    for split in (0, 2, 3):
        g.run_shells(4, compute_id=3 + split, split_last=split)
        assert cr.ranges(3 + split) == [g.global_range]
    cr.dispose()


@pytest.mark.parametrize("cls,tile", [(GemmBf16, "256x256pb"), (GemmBf16, "256x256pbr"), (GemmBf16, "256x128pe"),
                                      (GemmF32, "256x256g8i")])
def test_verify_full_checks_every_tile(cls, tile):
    """the whole-output check compares every tile a
    process owns (untiled from the kernel's fragment order / tile order on
    the torch device) with a float64 product, and catches one wrong element
    anywhere."""
    from cekirdekler_amd.ops.gemm import rows_to_tile

    cpu = ck.ClPlatforms.all().cpus(True)
    cr = ck.ClNumberCruncher(cpu + cpu, "__global__ void nop(float* x) {}")
    g = cls(512, 768, 256, cruncher=cr, tile=tile)
    unit = g.L * g.split_k
    half = g.tiles // 2 * unit
    cr.cores.set_state(1, [half, g.tiles * unit - half], [[0.0, 0.0] for _ in range(10)], [1.0, 1.0])
    ref = g.reference()
    if g.row_major_c:
        g.C.array[:] = ref.astype(np.float32).ravel()
    else:
        tm, tn = tile_coords(np.arange(g.tiles), g.M, g.N, g.BM, g.BN, g.group_m)
        blocks = [ref[r * g.BM:(r + 1) * g.BM, c * g.BN:(c + 1) * g.BN].astype(np.float32) for r, c in zip(tm, tn)]
        tiles = np.stack(blocks)
        g.C.array[:] = (rows_to_tile(tiles, g.geom) if g.geom is not None else tiles).ravel()
    err, checked = g.verify_full(1, host=True, device="cpu")
    assert checked == g.tiles and err < 1e-6, (err, checked)
    g.C.array[g.C.N - 7] += 0.5  # one element of the last tile
    err, _ = g.verify_full(1, host=True, device="cpu")
    assert err > 1e-4
    cr.dispose()


def test_verify_shells_full_checks_every_block(cpu_cr):
    """The native shell stream's host C (shell layout) checked whole."""
    from cekirdekler_amd.ops.gemm import rows_to_tile, untile  # noqa: F401

    g = GemmBf16(1024, 1024, 256, cruncher=cpu_cr, tile="256x256pb", group_m=2)
    P = 2
    ref = g.reference().astype(np.float32)
    pm, pn = g.M // P, g.N // P
    parts = []
    for s in range(P):  # R_s then C_s, each tile-major in grouped order
        for rows, cols in (((s * pm, (s + 1) * pm), (0, (s + 1) * pn)),
                           ((0, s * pm), (s * pn, (s + 1) * pn))):
            m, n = rows[1] - rows[0], cols[1] - cols[0]
            if m == 0:
                continue
            blk = ref[rows[0]:rows[1], cols[0]:cols[1]]
            tm, tn = tile_coords(np.arange((m // 256) * (n // 256)), m, n, 256, 256, g.group_m)
            tiles = np.stack([blk[r * 256:(r + 1) * 256, c * 256:(c + 1) * 256] for r, c in zip(tm, tn)])
            parts.append(rows_to_tile(tiles, g.geom).ravel())
    g.C.array[:] = np.concatenate(parts)
    np.testing.assert_array_equal(g.shells_result(P), ref)
    err, blocks = g.verify_shells_full(P, device="cpu")
    assert blocks == 16 and err < 1e-6
    g.C.array[5] += 1.0
    assert g.verify_shells_full(P, device="cpu")[0] > 1e-4
