"""Compute graphs: a sequence of compute() calls captured into one hipGraph
per GPU and replayed (MI355X-native: launch-bound loops as graphs instead
of one host call per kernel and copy)."""
import time

import numpy as np
import pytest

import cekirdekler_amd as ck

pytestmark = pytest.mark.gpu

SRC = """
__global__ void inc(float* x) { x[get_global_id(0)] += 1.0f; }
__global__ void axpy(const float* a, float* x) { long long i = get_global_id(0); x[i] = x[i] * 0.5f + a[i]; }
"""


def test_captured_sequence_replays_on_two_logical_gpus():
    g0 = ck.ClPlatforms.all().gpus()[0]
    cr = ck.ClNumberCruncher(g0 + g0, SRC)
    n = 1 << 16
    x = ck.ClArray(np.zeros(n, np.float32))
    x.compute(cr, 1, "inc", n, 256)              # buffers exist, split decided
    x.read = x.write = False                     # device-resident from here on
    with cr.capture() as g:
        for _ in range(3):
            x.compute(cr, 1, "inc", n, 256)      # recorded, not run
    g.replay(10)
    for d in range(2):                           # each device's slice got 30 more increments
        cr.download(x, d)
        refs, rng = cr.references(1), cr.ranges(1)
        lo, hi = refs[d], refs[d] + rng[d]
        np.testing.assert_array_equal(x.array[lo:hi], 31.0)
    g.destroy()
    cr.dispose()


def test_captured_transfers_read_host_memory_at_replay():
    """H2D / D2H inside a graph move the host arrays' current contents."""
    cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], SRC)
    n = 1 << 16
    a = ck.ClArray(np.ones(n, np.float32))        # auto-registered (256 KiB)
    a.write = False
    x = ck.ClArray(np.zeros(n, np.float32))
    a.next_param(x).compute(cr, 2, "axpy", n, 256)
    with cr.capture() as g:
        a.next_param(x).compute(cr, 2, "axpy", n, 256)
    a.array[:] = 4.0
    x.array[:] = 0.0
    g.replay(1)
    # x is read (host 0.0 goes up at replay), a is read (4.0), x comes back
    np.testing.assert_array_equal(x.array, np.float32(0.0 * 0.5 + 4.0))
    g.destroy()
    cr.dispose()


def test_graph_replay_beats_per_call_issue():
    """A launch-bound loop: 64 tiny computes per replay."""
    cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], SRC)
    n = 1 << 12
    x = ck.ClArray(np.zeros(n, np.float32))
    x.compute(cr, 3, "inc", n, 256)
    x.read = x.write = False
    with cr.capture() as g:
        for _ in range(64):
            x.compute(cr, 3, "inc", n, 256)
    g.replay(2)
    t = time.perf_counter()
    g.replay(10)
    graph_us = (time.perf_counter() - t) * 1e6 / 640
    cr.enqueue_mode = True
    t = time.perf_counter()
    for _ in range(640):
        x.compute(cr, 3, "inc", n, 256)
    cr.enqueue_mode = False
    call_us = (time.perf_counter() - t) * 1e6 / 640
    cr.download(x, 0)
    np.testing.assert_array_equal(x.array, 1.0 + 64 * 12 + 640)
    assert graph_us < call_us, (graph_us, call_us)
    g.destroy()
    cr.dispose()


def test_capture_refuses_cpu_device():
    plats = ck.ClPlatforms.all()
    cr = ck.ClNumberCruncher(plats.gpus()[0] + plats.cpus(True), SRC)
    with pytest.raises(Exception, match="GPU devices only"):
        with cr.capture():
            pass
    cr.dispose()


def test_replay_refuses_a_graph_whose_buffers_were_released():
    """A graph replays the device pointers it captured: once an array it
    uses is disposed, replay must raise instead of touching freed memory."""
    cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], SRC)
    n = 1 << 16
    x = ck.ClArray(np.zeros(n, np.float32))
    x.compute(cr, 3, "inc", n, 256)
    x.read = x.write = False
    with cr.capture() as g:
        x.compute(cr, 3, "inc", n, 256)
    g.replay(2)
    x.dispose()
    with pytest.raises(Exception, match="stale"):
        g.replay(1)
    g.destroy()
    cr.dispose()
