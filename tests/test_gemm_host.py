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
