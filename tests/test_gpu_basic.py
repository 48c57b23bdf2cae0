"""GPU tier: user kernel JIT (hiprtc), library kernels and the multi-device
paths on a real MI355X.  Numerics are checked against plain numpy/fp64."""
import numpy as np
import pytest

import cekirdekler_amd as ck

pytestmark = pytest.mark.gpu


def _gpu():
    return ck.ClPlatforms.all().gpus()


SAXPY = """
__global__ void saxpy(const float* a, const float* x, float* y) {
  long long i = get_global_id(0);
  y[i] = a[0] * x[i] + y[i];
}
"""


def test_jit_saxpy_single_gpu():
    cr = ck.ClNumberCruncher(_gpu()[0], SAXPY)
    assert cr.error_code() == 0, cr.error_message()
    n = 1 << 20
    a = ck.ClArray(np.array([3.0], np.float32))
    x = ck.ClArray(np.random.rand(n).astype(np.float32))
    y = ck.ClArray(np.random.rand(n).astype(np.float32))
    ref = np.float32(3.0) * x.array + y.array
    a.write = False
    x.write = False
    a.next_param(x, y).compute(cr, 1, "saxpy", n, 256)
    np.testing.assert_allclose(y.array, ref, rtol=1e-6)


@pytest.mark.parametrize("pipeline,ptype", [(False, True), (True, ck.PIPELINE_EVENT), (True, ck.PIPELINE_DRIVER)])
def test_logical_devices_pipelines(pipeline, ptype):
    g = _gpu()
    devs = g[0] + g[0] + g[0]
    cr = ck.ClNumberCruncher(devs, SAXPY)
    n = 3 * 256 * 8 * 64
    a = ck.ClArray(np.array([2.0], np.float32))
    x = ck.ClArray(np.arange(n, dtype=np.float32))
    y = ck.ClArray(np.ones(n, np.float32))
    x.partial_read = True
    y.partial_read = True
    a.write = False
    x.write = False
    for it in range(4):
        y.array[:] = 1
        a.next_param(x, y).compute(cr, 5, "saxpy", n, 256, 0, pipeline, ptype, 8)
        np.testing.assert_array_equal(y.array, 2 * x.array + 1)
    assert sum(cr.ranges(5)) == n


@pytest.mark.parametrize("tile", ["256x256", "256x256pp", "256x256pb", "256x128pb", "256x128pe", "128x128"])
def test_gemm_bf16_matches_fp64(tile):
    from cekirdekler_amd.ops.gemm import GemmBf16

    g = GemmBf16(1024, 512, 512, devices=_gpu()[0], tile=tile)
    g.run(resident=False)
    c = g.result(download=False)
    ref = g.reference()
    err = np.abs(c - ref).max()
    assert err < 1e-4 * np.abs(ref).max(), err


@pytest.mark.parametrize("tile", ["256x256pb", "256x128pb", "256x128pe", "256x256pp"])
@pytest.mark.parametrize("shape", [(256, 256, 64), (512, 256, 128), (256, 512, 192), (1024, 768, 320),
                                   (2048, 2048, 1024)])
def test_gemm_8phase_pipeline_tails(tile, shape):
    """The 8-phase ring pipeline at K-tile counts below, at and above its
    prefetch depth (prologue/tail waits), on several grid shapes."""
    from cekirdekler_amd.ops.gemm import GemmBf16

    M, N, K = shape
    g = GemmBf16(M, N, K, devices=_gpu()[0], tile=tile, group_m=2)
    for _ in range(3):                       # repeated runs screen for LDS races
        g.run(resident=False)
        c = g.result(download=False)
        ref = g.reference()
        err = np.abs(c - ref).max()
        assert err < 1e-4 * np.abs(ref).max(), (shape, err)


@pytest.mark.parametrize("tile", ["256x256pp", "256x256pb"])
@pytest.mark.parametrize("split", [2, 4])
def test_gemm_split_k(tile, split):
    """Split-K: partial tiles + last-arrival reduction, counters re-armed
    across calls, K-split work-groups kept on one device by the balancer
    granularity (two logical devices, one made slower)."""
    from cekirdekler_amd.ops.gemm import GemmBf16

    g0 = _gpu()[0]
    cr = ck.ClNumberCruncher(g0 + g0, "", prebuilt=__import__(
        "cekirdekler_amd.ops.library", fromlist=["library"]).library("sgemm_bf16"))
    cr.set_time_scale(1, 2.0)
    g = GemmBf16(1024, 768, 1024, cruncher=cr, tile=tile, split_k=split, group_m=2)
    ref = g.reference()
    for _ in range(4):
        g.run(resident=False)
        c = g.result(download=False)
        err = np.abs(c - ref).max()
        assert err < 1e-4 * np.abs(ref).max(), err
    unit = g.L * split
    assert all(r % unit == 0 for r in cr.ranges(1)) and sum(cr.ranges(1)) == g.global_range
    cr.dispose()


@pytest.mark.parametrize("tile,limit", [("256x256pbw", 0), ("256x256pbw", -1), ("256x256pbw", 1),
                                        ("256x256pbh", 0), ("256x256pbh", -1), ("256x256pbh", -2), ("256x256pbh", 1),
                                        ("256x256pbs", 0), ("256x256pbs", -1), ("256x256pbs", -2), ("256x256pbs", 1)])
def test_gemm_split_k_handover(tile, limit):
    """Uneven split-K = 2 with a one-way hand-over: flags re-armed across
    calls (4 calls), the pair of K-splits kept on one device (two logical
    devices, one slower).  limit -1: every owner claims the hand-over before
    its main loop and multiplies the helper's K-range itself (the
    co-residency-safe fall-back); limit 1: one poll, either path; C is
    right in every case."""
    from cekirdekler_amd.ops.gemm import GemmBf16
    from cekirdekler_amd.ops.library import library

    g0 = _gpu()[0]
    cr = ck.ClNumberCruncher(g0 + g0, "", prebuilt=library("sgemm_bf16"))
    cr.set_time_scale(1, 2.0)
    g = GemmBf16(1024, 768, 1024, cruncher=cr, tile=tile, group_m=2, handover_spin_limit=limit)
    assert g.split_k == 2
    ref = g.reference()
    for _ in range(4):
        g.run(resident=False)
        c = g.result(download=False)
        err = np.abs(c - ref).max()
        assert err < 1e-4 * np.abs(ref).max(), err
    fb = g.handover_fallbacks()
    if limit == 0:
        assert fb == 0
    if limit == -1:
        assert fb == 4 * g.tiles, fb  # every owner of every call fell back
    if limit == -2 and tile != "256x256pbs":
        # helpers claimed the hand-back (race with the owner: not every
        # tile; pbs owners hand back before they wait, so it may be none)
        assert fb > 0, fb
    # the state words are re-armed: only the fall-back counter is nonzero
    for dev in range(2):
        cr.download(g.counters, dev)
        assert not g.counters.array[:-1].any()
    assert all(r % (2 * g.L) == 0 for r in cr.ranges(1)) and sum(cr.ranges(1)) == g.global_range
    cr.dispose()


def test_gemm_two_logical_devices_balanced():
    from cekirdekler_amd.ops.gemm import GemmBf16

    g0 = _gpu()[0]
    g = GemmBf16(1024, 1024, 256, devices=g0 + g0, tile="256x128pe")
    for _ in range(3):
        g.run(resident=False)
    c = g.result(download=False)
    ref = g.reference()
    assert np.abs(c - ref).max() < 1e-4 * np.abs(ref).max()


def test_gemm_wave_granularity_two_logical_devices():
    """Whole waves of tiles per device (one work-group per CU): 512 tiles of
    256² over two logical devices of one 256-CU GPU split 256/256 and stay
    in whole waves under re-balancing; every slice is correct."""
    from cekirdekler_amd.ops.gemm import GemmBf16

    g0 = _gpu()[0]
    cu = g0.device(0).compute_units
    g = GemmBf16(2048, (2 * cu // 8) * 256, 128, devices=g0 + g0, tile="256x256pb")
    unit = g.granularity()
    assert unit == cu * g.L
    for _ in range(4):
        g.run(resident=False)
        assert all(r % unit == 0 for r in g.cr.ranges(1)) and sum(g.cr.ranges(1)) == g.global_range
    c = g.result(download=False)
    ref = g.reference()
    assert np.abs(c - ref).max() < 1e-4 * np.abs(ref).max()
    assert GemmBf16(256, 256, 64, devices=g0, tile="256x256pb").granularity() == 512  # < 1 wave: per tile


@pytest.mark.parametrize("kernel", ["quad", "blk8", "blk8h", "blk8k", "blk8m", "blk8t", "blk8u", "blk8r", "blk8y"])
def test_mandelbrot_event_pipeline_matches_numpy(kernel):
    from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer

    m = MandelbrotRenderer(512, 256, max_iter=64, devices=_gpu()[0], kernel=kernel)
    img = m.render(pipeline=True, blobs=4)
    ref = m.reference()
    mism = np.mean(img != ref)
    assert mism < 0.01, mism


@pytest.mark.parametrize("kernel", ["blk8h", "blk8k", "blk8m", "blk8t", "blk8u", "blk8r", "blk8y"])
@pytest.mark.parametrize("shape", [(1024, 1024, 256), (512, 256, 60), (256, 128, 5), (512, 256, 100),
                                   (768, 128, 60)])
def test_mandelbrot_blk8k_matches_numpy(shape, kernel):
    """blk8k's exactly counted first block, early-exit waves, the 4-op
    iteration and the skipped counting pass (max_iter a multiple of 8, not
    a multiple, and below one block) against the float32 numpy reference;
    width 768 (48 blocks per band, not a power of two) takes blk8r's
    division path."""
    from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer

    w, h, it = shape
    m = MandelbrotRenderer(w, h, max_iter=it, devices=_gpu()[0], kernel=kernel)
    img = m.render(pipeline=False).copy()
    ref = m.reference()
    assert np.mean(img != ref) < 2e-3, np.mean(img != ref)
    m.cr.dispose()


@pytest.mark.parametrize("shape", [(1024, 1024, 256), (1024, 512, 100), (512, 512, 60), (768, 256, 200)])
@pytest.mark.parametrize("view", [(-2.0, -1.5, 3.0, 3.0), (-0.8, -0.2, 0.4, 0.4)])
def test_mandelbrot_fast_path_equals_general(shape, view):
    """blk8y (no per-lane checkpoints while every lane is bounded, z pairs
    ping-ponged) computes the same z sequence and checkpoints as blk8r:
    images bit-identical, on the default view and on a zoom that is mostly
    set interior, with max_iter a multiple of the block, not one, and below
    the first 32-step block."""
    from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer

    w, h, it = shape
    imgs = []
    for k in ("blk8r", "blk8y"):
        m = MandelbrotRenderer(w, h, max_iter=it, view=view, devices=_gpu()[0], kernel=k)
        imgs.append(m.render(pipeline=False).copy())
        m.cr.dispose()
    for img in imgs[1:]:
        assert np.array_equal(imgs[0], img), int((imgs[0] != img).sum())


@pytest.mark.parametrize("kernel,per_item", [("cek_reduce_sum_f32", 8), ("cek_reduce_sum_f32_x32", 32)])
def test_reduce_sum(kernel, per_item):
    from cekirdekler_amd.ops.library import library

    g = _gpu()[0]
    cr = ck.ClNumberCruncher(g + g, "", prebuilt=library("reduce"))  # two slices, disjoint partials
    n = 1 << 22
    x = ck.ClArray(np.random.rand(n).astype(np.float32))
    x.elements_per_work_item = per_item
    x.write = False
    groups = n // (256 * per_item)
    part = ck.ClArray(groups, np.float32)
    part.read = False
    part.elements_per_group = 1
    G = n // per_item
    x.next_param(part).compute(cr, 1, kernel, G, 256)
    np.testing.assert_allclose(part.array.sum(), x.array.astype(np.float64).sum(), rtol=1e-5)


@pytest.mark.parametrize("bpw", [2, 4])
def test_nbody_forces_match_fp64(bpw):
    from cekirdekler_amd.models.nbody import NBodySimulation, nbody_accel_reference

    sim = NBodySimulation(4096, devices=_gpu()[0], resident=False, bodies_per_item=bpw)
    sim.forces()
    sim.cr.sync()
    got = sim.acc.array.reshape(-1, 4)[:, :3]
    ref = nbody_accel_reference(sim.pos.array, 0.01 ** 2)
    err = np.abs(got - ref).max() / np.abs(ref).max()
    assert err < 1e-4, err


@pytest.mark.parametrize("resident", [True, False])
def test_nbody_steps_two_logical_devices(resident):
    from cekirdekler_amd.models.nbody import NBodySimulation

    g0 = _gpu()[0]
    one = NBodySimulation(2048, devices=g0, resident=resident)
    two = NBodySimulation(2048, devices=g0 + g0, resident=resident)
    for _ in range(3):
        one.step()
        two.step()
    one.download()
    two.download()
    np.testing.assert_allclose(two.pos.array, one.pos.array, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("tile", ["128x128", "256x128", "256x256", "256x256w", "256x256ir", "256x256ib7", "256x128ie",
                                  "256x256g", "256x256gt", "256x256gh", "256x256g8", "256x256g8t", "256x256g8i", "256x256g8h", "256x256g8q"])
@pytest.mark.parametrize("shape", [(512, 512, 256), (768, 512, 96), (512, 256, 32)])
def test_gemm_f32_matches_fp64(tile, shape):
    """fp32 matrix-core GEMM (v_mfma_f32_16x16x4_f32) against a float64 host
    product; K = 96 leaves an odd number of 32-deep K-tiles."""
    from cekirdekler_amd.ops.gemm import F32_TILES, GemmF32

    M, N, K = shape
    BM, BN = F32_TILES[tile][:2]
    if M % BM or N % BN:
        pytest.skip("shape not a multiple of the tile")
    g = GemmF32(M, N, K, devices=_gpu()[0], tile=tile, group_m=2)
    g.run(resident=False)
    c = g.result(download=False)
    ref = g.reference()
    assert np.abs(c - ref).max() < 1e-4 * np.sqrt(K) * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("tile,rows", [("256x256pb", 8192), ("256x256pbw", 1024), ("256x256pbh", 1024),
                                      ("256x256pbs", 1024)])
def test_gemm_benchmarked_size_verify(tile, rows):
    """The headline kernels at the benchmarked size: the full 8192³ problem
    (N = 1) and the 1024-row slice one GPU of eight computes, device-resident
    through compute() in enqueue mode as bench.py times it, checked by
    GemmBf16.verify_full (EVERY tile vs a float64 product on the GPU) and
    by the sampled host check."""
    from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16
    from cekirdekler_amd.ops.library import library

    cr = ck.ClNumberCruncher(_gpu()[0], "", prebuilt=library(*GEMM_LIBS))
    g = GemmBf16(rows, 8192, 8192, cruncher=cr, tile=tile)
    g.run(compute_id=1, resident=True)
    cr.enqueue_mode = True
    for _ in range(5):
        g.run(compute_id=1, resident=True)
    cr.enqueue_mode = False
    err = g.verify(compute_id=1, tiles_per_device=6)
    assert err < 1e-4, err
    err_full, tiles = g.verify_full(compute_id=1)
    assert tiles == g.tiles and err_full < 1e-4, (err_full, tiles)
    assert g.spin_timeouts() == 0
    cr.dispose()
    for a in (g.A, g.B, g.C, g.dims):
        a.dispose()


def test_gemm_async_queues_overlap_verified():
    """The bench's async-queue schedule: consecutive single-pass GEMMs on
    async enqueue queues (they overlap on the GPU) leave a correct C; a
    split-K tile refuses that mode (its partial-tile workspace is per GEMM)."""
    from cekirdekler_amd.cruncher import ClComputeError
    from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16
    from cekirdekler_amd.ops.library import library

    cr = ck.ClNumberCruncher(_gpu()[0], "", prebuilt=library(*GEMM_LIBS))
    g = GemmBf16(1024, 8192, 2048, cruncher=cr, tile="256x256pb")
    g.run(compute_id=1, resident=True)
    cr.enqueue_mode = True
    cr.enqueue_mode_async_enable = True
    for _ in range(6):
        g.run(compute_id=1, resident=True)
    cr.enqueue_mode = False
    cr.enqueue_mode_async_enable = False
    assert g.verify(compute_id=1, tiles_per_device=6) < 1e-4
    w = GemmBf16(1024, 1024, 1024, cruncher=cr, tile="256x256pbw")
    w.run(compute_id=2, resident=True)
    cr.enqueue_mode = True
    cr.enqueue_mode_async_enable = True
    try:
        with pytest.raises(ClComputeError):
            w.run(compute_id=2, resident=True)
    finally:
        cr.enqueue_mode = False
        cr.enqueue_mode_async_enable = False
    cr.dispose()


@pytest.mark.parametrize("tile,panels", [("256x256pb", 4), ("256x256pb", 2), ("256x128pe", 4), ("256x256", 1)])
def test_gemm_host_shells_matches_fp64(tile, panels):
    """Host-resident GEMM streamed in square shells (Cores::gemm_host_shells)
    against a float64 host product, every element; repeated calls reuse the
    device buffers."""
    from cekirdekler_amd.ops.gemm import GemmBf16

    g = GemmBf16(2048, 2048, 512, devices=_gpu()[0], tile=tile, group_m=2)
    for _ in range(2):
        g.C.array[:] = 0
        g.run_host_shells(panels)
        got = g.shells_result(panels)
        ref = g.reference()
        assert float(np.abs(got - ref).max() / np.abs(ref).max()) < 1e-5
    g.cr.dispose()


def test_gemm_f32_host_shells_matches_fp64():
    """The square-shell host-resident stream with fp32 operands (GemmF32)."""
    from cekirdekler_amd.ops.gemm import GemmF32

    g = GemmF32(1024, 1024, 256, devices=_gpu()[0], tile="256x256ir", group_m=2)
    g.run_host_shells(2)
    got = g.shells_result(2)
    ref = g.reference()
    assert float(np.abs(got - ref).max() / np.abs(ref).max()) < 1e-5
    assert g.verify_shells(2, samples=4) < 1e-5
    g.cr.dispose()


def test_mandelbrot_two_frames_in_flight_async_enqueue():
    """bench.py's frames_in_flight_2: two renderers on one cruncher, rendered
    alternately in async enqueue mode over 2 queues (launches run side by
    side); both device images equal the numpy reference afterwards."""
    from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer
    from cekirdekler_amd.ops.library import library

    cr = ck.ClNumberCruncher(_gpu()[0], "", prebuilt=library("mandelbrot"), queue_concurrency=2)
    ms = [MandelbrotRenderer(1024, 512, max_iter=100, cruncher=cr, kernel="blk8y") for _ in range(2)]
    for i, m in enumerate(ms):
        m.render(i + 1, pipeline=False)
        m.out.write = False
    ref = ms[0].reference()
    cr.enqueue_mode_async_enable = True
    cr.enqueue_mode = True
    for k in range(8):
        ms[k % 2].render(k % 2 + 1, pipeline=False)
    cr.enqueue_mode = False
    cr.enqueue_mode_async_enable = False
    for m in ms:
        m.out.array[:] = -1
        cr.download(m.out, 0)
        img = m.out.array.reshape(m.height, m.width)
        assert np.mean(img != ref) < 2e-3
    cr.dispose()


@pytest.mark.parametrize("tile,panels,split", [("256x256pb", 4, 0), ("256x256pb", 2, 0), ("256x128pe", 4, 0),
                                               ("256x256pb", 4, 2), ("256x256pb", 4, 4)])
def test_gemm_shells_through_compute(tile, panels, split):
    """Host-resident GEMM streamed in square shells THROUGH compute(): the
    event pipeline with explicit uneven blobs (blob s = shell s), A and B
    uploaded one row panel per blob, C downloaded shell by shell — the
    kernels' shell tile order (dims[6]) untiled on the host."""
    from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16
    from cekirdekler_amd.ops.library import library

    cr = ck.ClNumberCruncher(_gpu()[0], "", prebuilt=library(*GEMM_LIBS))
    g = GemmBf16(1024, 1024, 512, cruncher=cr, tile=tile)
    ref = g.reference()
    for _ in range(2):
        g.C.array[:] = np.nan
        g.run_shells(panels, compute_id=3, split_last=split)
        rec = cr.last_record()
        assert rec["pipelined"], rec
        assert rec["h2d_bytes"] == g.A.array.nbytes + g.B.array.nbytes + g.dims.array.nbytes, rec
        assert rec["d2h_bytes"] == g.C.array.nbytes, rec
        c = g.result(download=False)
        assert np.abs(c - ref).max() < 1e-4 * np.abs(ref).max()
    assert g.verify(compute_id=3, host=True) < 1e-4
    # a resident grouped-order run afterwards is unaffected by the shell dims
    g.run(compute_id=1, resident=True)
    assert g.verify(compute_id=1) < 1e-4
    cr.dispose()


def test_gemm_row_major_c_variant():
    """256x256pbr: the production kernel with a row-major C epilogue (LDS
    turn-around per wave) — bit-identical to the fragment-order kernel's C
    after untiling, and right against float64."""
    from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16
    from cekirdekler_amd.ops.library import library

    cr = ck.ClNumberCruncher(_gpu()[0], "", prebuilt=library(*GEMM_LIBS))
    frag = GemmBf16(1024, 1536, 512, cruncher=cr, tile="256x256pb")
    rowc = GemmBf16(1024, 1536, 512, cruncher=cr, tile="256x256pbr")
    rowc.A.array[:] = frag.A.array
    rowc.B.array[:] = frag.B.array
    frag.run(compute_id=1, resident=True)
    rowc.run(compute_id=2, resident=True)
    a = frag.result()
    b = rowc.result()
    np.testing.assert_array_equal(a, b)
    ref = frag.reference()
    assert np.abs(b - ref).max() < 1e-4 * np.abs(ref).max()
    assert rowc.verify(compute_id=2) < 1e-4
    with pytest.raises(ValueError):
        rowc.run(compute_id=3, resident=False)
    cr.dispose()


def test_gemm_shells_with_reserved_copy_cus():
    """Shell-streamed GEMM with downloads by a copy kernel on 8 reserved CUs
    (CU-masked streams): same C as the plain path, and the masks can be
    turned on and off between calls."""
    from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16
    from cekirdekler_amd.ops.library import library

    cr = ck.ClNumberCruncher(_gpu()[0], "", prebuilt=library(*GEMM_LIBS))
    g = GemmBf16(2048, 2048, 512, cruncher=cr, tile="256x256pb")
    ref = g.reference()
    cr.copy_cus = 8
    cr.kernel_d2h = True
    assert cr.copy_cus == 8
    for _ in range(2):
        g.C.array[:] = np.nan
        g.run_shells(4, compute_id=3)
        c = g.result(download=False)
        assert np.abs(c - ref).max() < 1e-4 * np.abs(ref).max()
    assert cr.cores.kernel_d2h_bytes >= g.C.array.nbytes
    cr.kernel_d2h = False
    cr.copy_cus = 0
    g.C.array[:] = np.nan
    g.run_shells(4, compute_id=3)
    assert np.abs(g.result(download=False) - ref).max() < 1e-4 * np.abs(ref).max()
    cr.dispose()
