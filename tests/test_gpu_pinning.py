"""Wrapped host arrays are page-locked on first compute (VERDICT r1 item 6;
reference pins every array per compute, Cores.cs:535-541)."""
import time

import numpy as np
import pytest

import cekirdekler_amd as ck
from cekirdekler_amd import cek

pytestmark = pytest.mark.gpu

SPIN = """
__global__ void spin(float* x, const int* it) {
  long long i = get_global_id(0);
  float v = x[i];
  for (int k = 0; k < it[0]; ++k) v = v * 0.9999f + 0.5f;
  x[i] = v;
}
"""


def test_wrapped_numpy_array_is_registered_and_unregistered():
    cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], SPIN)
    host = np.ones(1 << 16, np.float32)
    x = ck.ClArray(host)
    it = ck.ClArray(np.array([4], np.int32))
    it.write = False
    assert not cek.host_is_pinned(host.ctypes.data)
    x.next_param(it).compute(cr, 1, "spin", len(host), 256)
    assert x.pinned and cek.host_is_pinned(host.ctypes.data)
    assert not it.pinned  # below auto_pin_min_bytes: left pageable
    x.dispose()
    assert not cek.host_is_pinned(host.ctypes.data)
    cr.dispose()


def test_pinned_wrapped_d2h_does_not_block_enqueue_mode():
    """A D2H from pageable memory blocks the host until the stream drains;
    from the registered array, compute() returns while the kernel runs."""
    cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], SPIN)
    n = 1 << 18
    it = ck.ClArray(np.array([1000000], np.int32))  # a kernel of ~20 ms
    it.write = False

    def host_ms(pin_threshold):
        ck.ClArray.auto_pin_min_bytes = pin_threshold
        try:
            x = ck.ClArray(np.ones(n, np.float32))
            x.read = False
            x.next_param(it).compute(cr, 2, "spin", n, 256)  # warm: buffers, JIT, registration
            cr.enqueue_mode = True
            t = time.perf_counter()
            x.next_param(it).compute(cr, 2, "spin", n, 256)
            dt = (time.perf_counter() - t) * 1e3
            t = time.perf_counter()
            cr.enqueue_mode = False
            total = (time.perf_counter() - t) * 1e3 + dt
            pinned = x.pinned
            x.dispose()
            return dt, total, pinned
        finally:
            ck.ClArray.auto_pin_min_bytes = 64 * 1024

    dt_pin, total_pin, pinned = host_ms(64 * 1024)
    dt_page, total_page, pinned_page = host_ms(0)
    assert pinned and not pinned_page
    assert total_pin > 10.0, total_pin           # the kernel really runs long
    assert dt_pin < 0.25 * total_pin, (dt_pin, total_pin)
    assert dt_page > 0.5 * total_page, (dt_page, total_page)  # pageable: blocked
    cr.dispose()


@pytest.mark.parametrize("pipeline", [False, True])
def test_kernel_d2h_downloads_match(pipeline):
    """``kernel_d2h``: slices of registered (and hipHostMalloc) host arrays
    come down through the runtime's copy kernel, on two logical devices,
    serial and through the event pipeline; unaligned or small copies fall
    back to hipMemcpyAsync."""
    src = "__global__ void k(float* y) { long long i = get_global_id(0); y[i] = (float)(i % 9973) + 0.5f; }"
    g0 = ck.ClPlatforms.all().gpus()[0]
    cr = ck.ClNumberCruncher(g0 + g0, src)
    cr.kernel_d2h = True
    assert cr.kernel_d2h
    n = 1 << 22  # 16 MiB
    for y in (ck.ClArray(np.zeros(n, np.float32)), ck.ClArray(n, np.float32)):
        y.read = False
        y.compute(cr, 1, "k", n, 256, pipeline=pipeline, pipeline_blobs=4)
        np.testing.assert_array_equal(y.array, (np.arange(n) % 9973).astype(np.float32) + 0.5)
        y.dispose()
    assert cr.cores.kernel_d2h_bytes >= 2 * n * 4
    cr.dispose()
