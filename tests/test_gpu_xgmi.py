"""xGMI data plane inside one process.  On the one-GPU
box the "peers" are logical devices of GPU 0: hipMemcpyPeerAsync with
source ordinal == destination ordinal is legal, so the peer-copy branch and
its event ordering run exactly as between two MI355X, only without the
link."""
import numpy as np
import pytest

import cekirdekler_amd as ck

pytestmark = pytest.mark.gpu

GATHER = """
__global__ void gather(const float* b, const int* nb, float* y) {
  long long i = get_global_id(0);
  int n = nb[0];
  y[i] = b[(i * 7919) % n] + 2.0f * b[n - 1 - (i % n)];
}
"""


def _ref(b, n_out):
    i = np.arange(n_out)
    n = len(b)
    return b[(i * 7919) % n] + np.float32(2.0) * b[n - 1 - (i % n)]


@pytest.mark.parametrize("ndev", [2, 3, 4])
def test_read_array_fanout_over_peer_copies(ndev):
    g0 = ck.ClPlatforms.all().gpus()[0]
    devs = g0
    for _ in range(ndev - 1):
        devs = devs + g0
    cr = ck.ClNumberCruncher(devs, GATHER)
    assert cr.peer_reads
    nb = (3 << 20) // 4 * ndev  # ≥ 1 MiB per chunk, divisible into 4 KiB chunks
    b = ck.ClArray(np.random.default_rng(0).standard_normal(nb).astype(np.float32))
    b.write = False
    nbv = ck.ClArray(np.array([nb], np.int32))
    nbv.write = False
    n_out = 256 * 64 * ndev
    y = ck.ClArray(np.zeros(n_out, np.float32))
    y.read = False
    for it in range(3):
        b.array[:] = b.array * np.float32(0.5) + np.float32(it)  # new contents every call
        b.next_param(nbv, y).compute(cr, 1, "gather", n_out, 64)
        np.testing.assert_array_equal(y.array, _ref(b.array, n_out))
        rec = cr.last_record()
        # b crosses PCIe once (1/D per GPU); the small nb array goes to every device
        assert rec["h2d_bytes"] == b.array.nbytes + ndev * 4, rec
        assert rec["p2p_bytes"] == (ndev - 1) * b.array.nbytes, rec
    # reference behaviour when off: one whole upload per device
    cr.peer_reads = False
    b.next_param(nbv, y).compute(cr, 1, "gather", n_out, 64)
    np.testing.assert_array_equal(y.array, _ref(b.array, n_out))
    rec = cr.last_record()
    assert rec["p2p_bytes"] == 0 and rec["h2d_bytes"] == ndev * (b.array.nbytes + 4)
    cr.dispose()


def test_fanout_in_enqueue_mode_and_async_queues():
    """Enqueue mode runs computes back to back without host syncs: a GPU's
    next chunk upload must wait until its peers pulled the previous one, and
    kernels on async compute queues must wait for the pulls."""
    g0 = ck.ClPlatforms.all().gpus()[0]
    cr = ck.ClNumberCruncher(g0 + g0, GATHER)
    nb = 1 << 20
    b = ck.ClArray(np.random.default_rng(1).standard_normal(nb).astype(np.float32))
    b.write = False
    nbv = ck.ClArray(np.array([nb], np.int32))
    nbv.write = False
    n_out = 1 << 16
    y = ck.ClArray(np.zeros(n_out, np.float32))
    y.read = False
    b.next_param(nbv, y).compute(cr, 2, "gather", n_out, 64)
    cr.enqueue_mode = True
    cr.enqueue_mode_async_enable = True
    for _ in range(8):
        b.next_param(nbv, y).compute(cr, 2, "gather", n_out, 64)
    cr.enqueue_mode = False
    np.testing.assert_array_equal(y.array, _ref(b.array, n_out))
    assert cr.last_record()["p2p_bytes"] == b.array.nbytes
    cr.dispose()


def test_cl_pipeline_multi_device_stages_stay_on_device():
    """Stage 1 on three logical GPUs (uneven split: one device made slower),
    stage 2 on one GPU, stage 3 on two GPUs.  Every transition is a peer
    copy: PCIe carries only the pushed inputs (to each stage-1 device) and
    the results; nothing is staged through host memory."""
    from cekirdekler_amd.parallel.pipeline import ClPipelineStage

    g0 = ck.ClPlatforms.all().gpus()[0]
    n = 1 << 16
    k1 = "__global__ void f1(const float* x, const float* c, float* y) { long long i = get_global_id(0); y[i] = x[i] * c[0] + (float)i; }"
    k2 = "__global__ void f2(const float* y, float* z) { long long i = get_global_id(0); z[i] = y[i] + y[(i * 31) % 65536]; }"
    k3 = "__global__ void f3(const float* z, float* w) { long long i = get_global_id(0); w[i] = z[i] - 1.0f; }"

    def stage(devs, src, name, ins, hid, outs):
        s = ClPipelineStage()
        s.add_devices(devs)
        s.add_kernels(src, name, [n], [64])
        s.add_input_buffers(*ins)
        if hid:
            s.add_hidden_buffers(*hid)
        s.add_output_buffers(*outs)
        return s

    s1 = stage(g0 + g0 + g0, k1, "f1", [np.zeros(n, np.float32)], [np.array([3.0], np.float32)],
               [np.zeros(n, np.float32)])
    s2 = stage(g0, k2, "f2", [np.zeros(n, np.float32)], None, [np.zeros(n, np.float32)])
    s3 = stage(g0 + g0, k3, "f3", [np.zeros(n, np.float32)], None, [np.zeros(n, np.float32)])
    s1.prepend_to_stage(s2)
    s3.append_to_stage(s2)
    pipe = s1.make_pipeline()
    s1.cruncher.set_time_scale(2, 3.0)  # uneven slices in stage 1
    s3.cruncher.set_time_scale(0, 2.0)
    i = np.arange(n)

    def expect(p):
        y = np.float32(3.0) * np.float32(p) + i.astype(np.float32)
        return (y + y[(i * 31) % n]) - np.float32(1.0)

    res = np.zeros(n, np.float32)
    seen = 0
    pushes = 14
    for p in range(pushes):
        if pipe.push_data([np.full(n, float(p), np.float32)], [res]):
            np.testing.assert_array_equal(res, expect(seen))
            seen += 1
    assert seen == pushes - 6
    st = pipe.transfer_stats()
    assert st["h2d"] == pushes * 3 * n * 4   # inputs to each stage-1 device
    assert st["d2h"] == pushes * n * 4       # results only
    assert st["host"] == 0 and st["p2p"] > 0
    r1 = s1.cruncher.ranges(1)
    assert len(set(r1)) > 1, r1             # the split really was uneven
    pipe.dispose()


def test_cl_pipeline_mixed_cpu_gpu_stage():
    """A stage spanning the CPU device and a GPU: the CPU device's replica
    is the host array itself, the GPU's is device memory; the copy engine
    moves each slice from whichever device computed it (host↔GPU copies
    for the mixed stage, GPU→GPU pulls elsewhere)."""
    from cekirdekler_amd.parallel.pipeline import ClPipelineStage

    plats = ck.ClPlatforms.all()
    g0, cpu = plats.gpus()[0], plats.cpus(True)
    n = 1 << 14
    k1 = "__global__ void f1(const float* x, float* y) { long long i = get_global_id(0); y[i] = x[i] * 2.0f + (float)i; }"
    k2 = "__global__ void f2(const float* y, float* z) { long long i = get_global_id(0); z[i] = y[i] + 1.0f; }"
    s1, s2 = ClPipelineStage(), ClPipelineStage()
    s1.add_devices(g0 + cpu)
    s1.add_kernels(k1, "f1", [n], [64])
    s1.add_input_buffers(np.zeros(n, np.float32))
    s1.add_output_buffers(np.zeros(n, np.float32))
    s2.add_devices(g0)
    s2.add_kernels(k2, "f2", [n], [64])
    s2.add_input_buffers(np.zeros(n, np.float32))
    s2.add_output_buffers(np.zeros(n, np.float32))
    s1.prepend_to_stage(s2)
    pipe = s1.make_pipeline()
    i = np.arange(n, dtype=np.float32)
    res = np.zeros(n, np.float32)
    seen = 0
    for p in range(10):
        if pipe.push_data([np.full(n, float(p), np.float32)], [res]):
            np.testing.assert_array_equal(res, np.float32(seen) * 2 + i + 1)
            seen += 1
    assert seen == 6
    r = s1.cruncher.ranges(1)
    assert all(x > 0 for x in r), r  # both devices computed a slice
    pipe.dispose()


@pytest.mark.parametrize("engine", [0, 1])
@pytest.mark.parametrize("nbytes", [4 << 20, (1 << 20) + 4, 256 << 20])
def test_copy_engines_byte_exact_same_gpu(engine, nbytes):
    """both device→device engines (SDMA, copy kernel) on one
    GPU, byte for byte (a size that is not a multiple of 16 takes the
    kernel's SDMA tail)."""
    from cekirdekler_amd._native import cek

    r = cek.measure_copy(0, 0, nbytes, engine, 2)
    assert r["verified"], r
    assert r["gbps"] > 0


def test_gather_through_kernel_copy_engine():
    """The keep-resident gather with the copy-kernel engine forced: same
    result as with SDMA (Cores::d2d_copy → peer_copy)."""
    from cekirdekler_amd._native import cek

    g0 = ck.ClPlatforms.all().gpus()[0]
    src = """__global__ void hop(const float* x, float* y) {
      long long i = get_global_id(0); long long n = get_global_size(0);
      y[i] = x[(i * 7919) % n] * 0.5f + 1.0f; }"""
    results = []
    for engine in (0, 1):
        cek.set_copy_engine_override(engine)
        try:
            cr = ck.ClNumberCruncher(g0 + g0 + g0, src)
            cr.set_time_scale(2, 1.6)
            n = 3 * (1 << 15)
            x0 = np.random.default_rng(5).standard_normal(n).astype(np.float32)
            a, b = ck.ClArray(x0.copy()), ck.ClArray(np.zeros(n, np.float32))
            a.write = b.write = False
            s, d = a, b
            for it in range(5):
                s.read = it == 0
                d.read = False
                s.gather_resident, d.gather_resident = False, True
                s.next_param(d).compute(cr, 1, "hop", n, 64)
                s, d = d, s
            outs = []
            for dev in range(3):
                s.array[:] = 0
                cr.download(s, dev)
                outs.append(s.array.copy())
            cr.dispose()
        finally:
            cek.set_copy_engine_override(-1)
        for o in outs[1:]:
            np.testing.assert_array_equal(o, outs[0])
        results.append(outs[0])
    np.testing.assert_array_equal(results[0], results[1])


def test_peer_bandwidth_report_on_visible_gpus():
    """The bench's xGMI section on whatever this box has (one GPU: the
    same-GPU rows only, no crash)."""
    from cekirdekler_amd.utils.multigpu import peer_bandwidth_report, visible_gpus

    n = visible_gpus()
    rep = peer_bandwidth_report(list(range(min(n, 8))), pair_bytes=64 << 20, all_bytes=16 << 20, reps=2)
    assert rep["gpus_visible"] == n
    assert rep["all_verified"], rep
    assert set(rep["same_gpu"]) == {"sdma", "kernel", "faster"}
    if n >= 2:
        assert rep["pairs"] and rep["all_pairs"]
