"""Keep-resident gather (``ClArray.gather_resident``) and
the read fan-out's in-place hazard, on logical devices of GPU 0.

The reference makes an iterative kernel's results coherent by downloading
every device's slice and uploading the whole array again on the next call
(Tester.cs:7759-7765).  With the gather flag the slices are copied
device→device after the kernels (peer copies; between logical devices of one
GPU they are D2D copies on the same code path), ordered by events, so after
the first call nothing crosses PCIe.
"""
import numpy as np
import pytest

import cekirdekler_amd as ck

pytestmark = pytest.mark.gpu

SRC = """
__global__ void hop(const float* x, float* y) {
  long long i = get_global_id(0);
  long long n = get_global_size(0);
  y[i] = x[(i * 7919) % n] * 0.5f + 1.0f;
}
__global__ void pick(const float* x, float* tmp) {
  long long i = get_global_id(0);
  long long n = get_global_size(0);
  tmp[i] = x[(i * 7919) % n];
}
__global__ void update(float* x, const float* tmp) {
  long long i = get_global_id(0);
  x[i] = tmp[i] * 0.5f + 1.0f;
}
"""


def _step(x):
    n = len(x)
    return x[(np.arange(n) * 7919) % n] * np.float32(0.5) + np.float32(1.0)


def _gpus(k):
    g0 = ck.ClPlatforms.all().gpus()[0]
    devs = g0
    for _ in range(k - 1):
        devs = devs + g0
    return devs


@pytest.mark.parametrize("ndev", [2, 3])
def test_gather_ping_pong_device_resident(ndev):
    cr = ck.ClNumberCruncher(_gpus(ndev), SRC)
    cr.set_time_scale(ndev - 1, 1.7)  # uneven split after the first call
    n = 1 << 16
    x0 = np.random.default_rng(0).standard_normal(n).astype(np.float32)
    a = ck.ClArray(x0.copy())
    b = ck.ClArray(np.zeros(n, np.float32))
    for arr in (a, b):
        arr.write = False
        arr.gather_resident = True
    ref = x0.copy()
    src, dst = a, b
    for it in range(12):
        src.read = it == 0
        dst.read = False
        src.gather_resident, dst.gather_resident = False, True  # the written array
        src.next_param(dst).compute(cr, 1, "hop", n, 64)
        ref = _step(ref)
        rec = cr.last_record()
        if it > 0:
            assert rec["h2d_bytes"] == 0 and rec["d2h_bytes"] == 0, rec
        assert rec["gather_bytes"] == (ndev - 1) * n * 4, rec
        assert rec["p2p_path"] == "local", rec
        src, dst = dst, src
    assert len(set(cr.ranges(1))) > 1  # the split moved while resident
    for d in range(ndev):  # every replica holds the whole result
        src.array[:] = 0
        cr.download(src, d)
        np.testing.assert_allclose(src.array, ref, rtol=1e-6, atol=1e-6)
    cr.dispose()


@pytest.mark.parametrize("enqueue", [False, True])
def test_gather_in_place_waits_for_every_reader(enqueue):
    """Two kernels in one compute, as in N-body: ``pick`` reads x across
    every slice, ``update`` rewrites this device's slice in place.  A device
    must not push its new slice into a peer's replica while the peer's
    ``pick`` still reads it."""
    cr = ck.ClNumberCruncher(_gpus(2), SRC)
    n = 1 << 18
    x0 = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    x = ck.ClArray(x0.copy())
    tmp = ck.ClArray(np.zeros(n, np.float32))
    x.write = False
    x.gather_resident = True
    tmp.read = False
    tmp.write = False
    ref = x0.copy()
    steps = 16
    x.read = True
    x.next_param(tmp).compute(cr, 2, "pick update", n, 256)
    ref = _step(ref)
    x.read = False
    if enqueue:
        cr.enqueue_mode = True
    for _ in range(steps - 1):
        x.next_param(tmp).compute(cr, 2, "pick update", n, 256)
        ref = _step(ref)
    if enqueue:
        cr.enqueue_mode = False
    for d in range(2):
        x.array[:] = 0
        cr.download(x, d)
        np.testing.assert_allclose(x.array, ref, rtol=1e-5, atol=1e-5)
    cr.dispose()


def test_gather_cpu_and_gpu_devices():
    """The CPU device's replica is the host array: GPU slices are pushed into
    it (D2H) and its slice is pulled into the GPU replica (H2D)."""
    plats = ck.ClPlatforms.all()
    cr = ck.ClNumberCruncher(plats.gpus()[0] + plats.cpus(True), SRC)
    n = 1 << 14
    x0 = np.random.default_rng(2).standard_normal(n).astype(np.float32)
    a = ck.ClArray(x0.copy())
    b = ck.ClArray(np.zeros(n, np.float32))
    for arr in (a, b):
        arr.write = False
        arr.gather_resident = True
    ref = x0.copy()
    src, dst = a, b
    for it in range(6):
        src.read = it == 0
        dst.read = False
        src.gather_resident, dst.gather_resident = False, True  # the written array
        src.next_param(dst).compute(cr, 3, "hop", n, 64)
        ref = _step(ref)
        src, dst = dst, src
    np.testing.assert_allclose(src.array, ref, rtol=1e-6, atol=1e-6)  # host = CPU replica
    src.array[:] = 0
    cr.download(src, 0)
    np.testing.assert_allclose(src.array, ref, rtol=1e-6, atol=1e-6)
    cr.dispose()


def test_share_slices_is_event_ordered():
    """The manual form: share_slices after a compute, no host sync inside
    enqueue mode; the next compute sees every slice."""
    cr = ck.ClNumberCruncher(_gpus(2), SRC)
    n = 1 << 16
    x0 = np.random.default_rng(3).standard_normal(n).astype(np.float32)
    a = ck.ClArray(x0.copy())
    b = ck.ClArray(np.zeros(n, np.float32))
    a.write = b.write = False
    a.next_param(b).compute(cr, 4, "hop", n, 64)
    cr.cores.share_slices(4, b._spec(), 64)
    a.read = b.read = False
    cr.enqueue_mode = True
    b.next_param(a).compute(cr, 4, "hop", n, 64)
    cr.cores.share_slices(4, a._spec(), 64)
    cr.enqueue_mode = False
    ref = _step(_step(x0))
    for d in range(2):
        cr.download(a, d)
        np.testing.assert_allclose(a.array, ref, rtol=1e-6, atol=1e-6)
    cr.dispose()


FANOUT_INPLACE = """
__global__ void clobber(float* b, float* y) {
  long long i = get_global_id(0);
  long long n = get_global_size(0);
  y[i] = b[(i + n / 2) % n];
  b[i] = -1.0f;
}
"""


@pytest.mark.parametrize("enqueue", [False, True])
def test_fanout_waits_for_peers_before_kernels_modify_in_place(enqueue):
    """a `read`, not-`write` array is staged by the xGMI fan-out
    (1/D uploaded per device, the rest pulled from peers).  The kernel
    overwrites its own slice of it in place; a peer that has not pulled that
    chunk yet must still receive the host data."""
    cr = ck.ClNumberCruncher(_gpus(2), FANOUT_INPLACE)
    n = 1 << 20  # 4 MiB: above peer_read_min_bytes
    b = ck.ClArray(np.zeros(n, np.float32))
    b.write = False
    y = ck.ClArray(np.zeros(n, np.float32))
    y.read = False
    rng = np.random.default_rng(4)
    src = (np.arange(n) + n // 2) % n

    def check(host):
        # an item whose source index lies in its OWN device's slice races with
        # that device's own in-place writes (the kernel's business); every
        # source in the OTHER device's slice must hold the host value
        refs, rngs = cr.references(5), cr.ranges(5)
        owner = np.searchsorted(np.array(refs[1:]), np.arange(n), side="right")
        cross = owner != owner[src]
        assert cross.sum() >= n // 4
        np.testing.assert_array_equal(y.array[cross], host[src][cross])

    if enqueue:
        cr.enqueue_mode = True
    outs = []
    for it in range(6):
        b.array[:] = rng.standard_normal(n).astype(np.float32)
        host = b.array.copy()
        b.next_param(y).compute(cr, 5, "clobber", n, 256)
        if not enqueue:
            check(host)
            assert cr.last_record()["p2p_bytes"] > 0
        outs.append(host)
    if enqueue:
        cr.enqueue_mode = False
        check(outs[-1])
    cr.dispose()


def test_graph_capture_pins_small_pageable_arrays():
    """arrays below auto_pin_min_bytes used to stay pageable, and
    their captured copies would replay stale pages.  Inside a capture every
    transferred array is registered first."""
    cr = ck.ClNumberCruncher(_gpus(1), SRC)
    n = 1024  # 4 KiB: below the 64 KiB auto-pin threshold
    a = ck.ClArray(np.arange(n, dtype=np.float32))
    b = ck.ClArray(np.zeros(n, np.float32))
    a.next_param(b).compute(cr, 6, "hop", n, 64)
    with cr.capture() as g:
        a.next_param(b).compute(cr, 6, "hop", n, 64)
    for v in (3.0, -2.0):
        a.array[:] = v  # replay reads the array's current contents
        g.replay(1)
        np.testing.assert_allclose(b.array, np.full(n, v * 0.5 + 1.0, np.float32))
    g.destroy()
    cr.dispose()


def test_graph_exit_keeps_the_user_exception():
    cr = ck.ClNumberCruncher(_gpus(1), SRC)
    with pytest.raises(ZeroDivisionError):
        with cr.capture():
            1 / 0
    assert not cr.cores.capturing
    cr.dispose()


def test_failover_regathers_recomputed_slice():
    """when a device fails, a survivor recomputes its
    slice; with a keep-resident array that slice must still reach every
    surviving replica, or later steps read stale values."""
    cr = ck.ClNumberCruncher(_gpus(3), SRC)
    cr.auto_failover = True
    n = 3 * (1 << 14)
    x0 = np.random.default_rng(7).standard_normal(n).astype(np.float32)
    a = ck.ClArray(x0.copy())
    b = ck.ClArray(np.zeros(n, np.float32))
    for arr in (a, b):
        arr.write = False
    ref = x0.copy()
    src, dst = a, b
    for it in range(6):
        if it == 2:
            cr.cores.inject_failure(2, 1)  # device 2 fails once, is dropped
        src.read = it == 0
        dst.read = False
        src.gather_resident, dst.gather_resident = False, True
        src.next_param(dst).compute(cr, 5, "hop", n, 64)
        ref = _step(ref)
        src, dst = dst, src
    assert cr.cores.failovers == 1
    assert not cr.device_enabled(2)
    for d in (0, 1):  # both survivors hold the whole, current result
        src.array[:] = 0
        cr.download(src, d)
        np.testing.assert_allclose(src.array, ref, rtol=1e-6, atol=1e-6)
    cr.dispose()


COPY_SRC = """
__global__ void slowfill(float* x) {
  long long i = get_global_id(0);
  float v = (float)i;
  for (int k = 0; k < 4000; ++k) v = v * 1.0000001f + 0.0f;
  x[i] = v > -1.0f ? (float)i + 1.0f : 0.0f;
}
__global__ void add1(float* x) { long long i = get_global_id(0); x[i] = x[i] + 1.0f; }
"""


def test_copy_between_orders_against_async_compute_queues():
    """with async enqueue a compute sits on a compute
    queue, not the main stream.  copy_between must wait for it (the source
    is still being written) and later computes on any queue must wait for
    the copy (they read the destination)."""
    g0 = ck.ClPlatforms.all().gpus()[0]
    cr = ck.ClNumberCruncher(g0 + g0, COPY_SRC, queue_concurrency=4)
    n = 1 << 18
    x = ck.ClArray(np.zeros(n, np.float32))
    y = ck.ClArray(np.zeros(n, np.float32))
    x.read = y.read = False
    x.write = y.write = False
    # establish buffers on both devices (one device each, full range)
    x.compute(cr, 11, "add1", n, 256)
    y.compute(cr, 12, "add1", n, 256)
    cr.enqueue_mode = True
    cr.enqueue_mode_async_enable = True
    # device 0: slow fill of x on a compute queue, then copy x(dev0) -> y(dev1)
    cr.cores.set_device_enabled(1, False)
    x.compute(cr, 13, "slowfill", n, 256)
    cr.cores.copy_between(0, x._spec(), 1, y._spec(), n * 4)
    cr.cores.set_device_enabled(1, True)
    cr.cores.set_device_enabled(0, False)
    y.compute(cr, 14, "add1", n, 256)  # on device 1, a compute queue: must see the copy
    cr.cores.set_device_enabled(0, True)
    cr.enqueue_mode = False
    cr.enqueue_mode_async_enable = False
    cr.download(y, 1)
    np.testing.assert_array_equal(y.array, np.arange(n, dtype=np.float32) + 2.0)
    cr.dispose()
