"""Wave-equation example (Kamera.cs:188-284) and the auxiliary-function
prelude (ClBuiltInAuxilliaryFunctions.cs:28-47) on the host CPU device."""
import numpy as np
import pytest

from cekirdekler_amd import ClArray, ClBuiltInAuxilliaryFunctions, ClNumberCruncher, ClPlatforms
from cekirdekler_amd.models.wave import VERTEX, WaveSurface, grid_mesh, wave_reference


@pytest.fixture(scope="module")
def cpu():
    return ClPlatforms.all().cpus(True)


def test_wave_matches_host_loop(cpu):
    base, nrm = grid_mesh(100, 37)            # 3700 vertices: not a multiple of 64
    w = WaveSurface(base, nrm, devices=cpu)
    for _ in range(6):
        v = w.update()
    ref = w.reference()
    for c in "xyz":
        np.testing.assert_allclose(v[c], ref[c], atol=1e-6)
    assert np.abs(ref["z"]).max() > 0          # the surface actually moved
    # padded tail untouched (the id < arguments[4] guard)
    assert np.all(w.xyzo.array.view(VERTEX)[w.n:]["z"] == 0)


def test_wave_reference_formula():
    base, nrm = grid_mesh(8, 8)
    out = wave_reference(base, nrm, 0.3, 0.5, base["x"][0], base["y"][0])
    r = np.hypot(base["x"] - base["x"][0], base["y"] - base["y"][0])
    np.testing.assert_allclose(out["z"], 0.02 * 0.3 * np.sin(40 * 0.5 + 100 * r), atol=1e-6)
    np.testing.assert_array_equal(out["x"], base["x"])


def test_aux_prelude_selection():
    aux = ClBuiltInAuxilliaryFunctions()
    assert str(aux) == ""
    aux.exampleFunction = True                 # reference spelling
    assert aux.example_function and "exampleFunction" in str(aux)
    with pytest.raises(AttributeError):
        aux.no_such_function = True


def test_aux_functions_run_on_cpu(cpu):
    aux = ClBuiltInAuxilliaryFunctions(example_function=True, block_sum=True, bf16=True, lerp=True)
    src = aux.wrap("""
    __global__ void k(const float* x, float* sums, int* ex, unsigned short* h, float* l) {
        __shared__ float scratch[64];
        long long i = get_global_id(0);
        float s = cek_block_sum(x[i], scratch);
        if (get_local_id(0) == 0) sums[cek_global_group_id()] = s;
        ex[i] = exampleFunction((int)i, 1);
        h[i] = cek_f32_to_bf16(x[i]);
        l[i] = cek_lerp(0.f, x[i], 0.5f);
    }""")
    cr = ClNumberCruncher(cpu, src)
    assert cr.error_code() == 0, cr.error_message()
    n = 256
    x = ClArray(np.linspace(-2, 2, n).astype(np.float32)); x.write = False
    sums = ClArray(np.zeros(n // 64, np.float32)); sums.read = False
    sums.elements_per_group = 1
    ex = ClArray(np.zeros(n, np.int32)); ex.read = False
    h = ClArray(np.zeros(n, np.uint16)); h.read = False
    lv = ClArray(np.zeros(n, np.float32)); lv.read = False
    x.next_param(sums, ex, h, lv).compute(cr, 1, "k", n, 64)
    np.testing.assert_allclose(sums.array, x.array.reshape(-1, 64).sum(1), rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(ex.array, np.arange(n) + 1)
    bits = x.array.view(np.uint32)
    rne = ((bits + 0x7FFF + ((bits >> 16) & 1)) >> 16).astype(np.uint16)
    np.testing.assert_array_equal(h.array, rne)
    np.testing.assert_allclose(lv.array, x.array * 0.5)
    cr.dispose()


def test_mandelbrot_kernel_table_is_consistent():
    """Every Mandelbrot variant maps to a library kernel with a valid range
    decomposition (checked on the host; the kernels run in the GPU tier)."""
    from cekirdekler_amd.models import mandelbrot as mb
    from cekirdekler_amd.ops.library import ARITY, LIBRARY

    for name, (kernel, ppw, local) in mb.KERNELS.items():
        assert kernel in LIBRARY["mandelbrot"] and ARITY[kernel] == 3, name
        assert local in (64, 256) and (local == 256 or name in mb.BAND_KERNELS)
        W, H = 4096, 4096
        G = W * H // ppw
        assert G % local == 0
        if name in mb.BAND_KERNELS:
            band = mb.BAND_ROWS[name] * W // ppw   # work items per band
            assert band % local == 0 and G % band == 0 and (G // band) % 8 == 0


def test_library_arity_covers_every_kernel():
    from cekirdekler_amd.ops.library import ARITY, LIBRARY

    for names in LIBRARY.values():
        for k in names:
            assert k in ARITY, k


def _tile_major(c, M, N, BM, BN, gm, geom=None):
    """Row-major [M][N] → tile-major in the kernels' grouped tile order (each
    tile in fragment order when ``geom`` is given, as the bf16 kernels store it)."""
    from cekirdekler_amd.ops.gemm import rows_to_tile, tile_coords

    ntiles = (M // BM) * (N // BN)
    tm, tn = tile_coords(np.arange(ntiles), M, N, BM, BN, gm)
    blocks = [c[r * BM:(r + 1) * BM, q * BN:(q + 1) * BN] for r, q in zip(tm, tn)]
    return np.concatenate([(b if geom is None else rows_to_tile(b, geom)).ravel() for b in blocks])


@pytest.mark.parametrize("tile", ["256x256pb", "256x128pe", "128x128"])
def test_fragment_order_round_trip(tile):
    """tile_to_rows / rows_to_tile are inverse, and the element the kernel
    epilogue stores at ((((wr·WN + wc)·FM + i)·FN + j)·64 + fq·16 + fr)·4 + r
    comes back at (wr·16FM + i·16 + fq·4 + r, wc·16FN + j·16 + fr)."""
    from cekirdekler_amd.ops.gemm import TILE_WAVES, TILES, rows_to_tile, tile_to_rows

    BM, BN = TILES[tile][:2]
    WM, WN, FM, FN = geom = TILE_WAVES[tile]
    assert (WM * FM * 16, WN * FN * 16) == (BM, BN)
    rows = np.arange(BM * BN, dtype=np.float32).reshape(BM, BN)
    flat = rows_to_tile(rows, geom)
    np.testing.assert_array_equal(tile_to_rows(flat, geom), rows)
    rng = np.random.default_rng(0)
    for _ in range(64):
        wr, wc, i, j = (int(rng.integers(n)) for n in (WM, WN, FM, FN))
        fq, fr, r = int(rng.integers(4)), int(rng.integers(16)), int(rng.integers(4))
        off = ((((wr * WN + wc) * FM + i) * FN + j) * 64 + fq * 16 + fr) * 4 + r
        assert flat[off] == rows[wr * 16 * FM + i * 16 + fq * 4 + r, wc * 16 * FN + j * 16 + fr]


@pytest.mark.parametrize("geom", [None, (2, 2, 4, 4)])
@pytest.mark.parametrize("panels,gm", [(1, 2), (2, 2), (4, 1), (4, 3)])
def test_shell_layout_round_trip(panels, gm, geom):
    """The host C layout of the square-shell stream (Cores::gemm_host_shells:
    shell by shell, R_s = rows of panel s × columns of panels 0..s, then
    C_s = rows of panels 0..s-1 × columns of panel s, each tile-major) is
    undone exactly by GemmBf16.shells_result."""
    from types import SimpleNamespace

    from cekirdekler_amd.ops.gemm import GemmBf16

    M, N, BM, BN = 512, 1024, 128, 128
    full = np.random.default_rng(0).standard_normal((M, N)).astype(np.float32)
    pm, pn = M // panels, N // panels
    parts = []
    for s in range(panels):
        parts.append(_tile_major(full[s * pm:(s + 1) * pm, :(s + 1) * pn], pm, (s + 1) * pn, BM, BN, gm, geom))
        if s:
            parts.append(_tile_major(full[:s * pm, s * pn:(s + 1) * pn], s * pm, pn, BM, BN, gm, geom))
    host = np.concatenate(parts)
    assert host.size == M * N
    g = SimpleNamespace(M=M, N=N, BM=BM, BN=BN, group_m=gm, geom=geom, C=SimpleNamespace(array=host))
    np.testing.assert_array_equal(GemmBf16.shells_result(g, panels), full)
