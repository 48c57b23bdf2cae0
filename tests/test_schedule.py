"""Recorded-schedule checks of the event-driven and driver pipelines
(SURVEY §7.4 item 5), on logical CPU devices; the GPU tier repeats them."""
import numpy as np
import pytest

import cekirdekler_amd as ck
from cekirdekler_amd.utils.schedule import check_pipeline_schedule

SRC = "__global__ void k(const float* x, float* y) { long long i = get_global_id(0); y[i] = x[i] * 2.0f; }"


def _record(devices, ptype, blobs, **layout):
    cr = ck.ClNumberCruncher(devices, SRC)
    cr.cores.record_schedule = True
    for k, v in layout.items():
        setattr(cr.cores, k, v)
    n = 64 * blobs * len(devices) * 4
    x = ck.ClArray(np.arange(n, dtype=np.float32)); x.partial_read = True; x.write = False
    y = ck.ClArray(np.zeros(n, np.float32)); y.read = False
    x.next_param(y).compute(cr, 1, "k", n, 64, 0, True, ptype, blobs)
    np.testing.assert_array_equal(y.array, 2 * x.array)
    sched = cr.cores.schedule()
    cr.dispose()
    return sched


@pytest.mark.parametrize("ptype,blobs", [(ck.PIPELINE_EVENT, 4), (ck.PIPELINE_EVENT, 3), (ck.PIPELINE_EVENT, 8),
                                         (ck.PIPELINE_DRIVER, 8)])
def test_pipeline_schedule_dependencies(ptype, blobs):
    cpu = ck.ClPlatforms.all().cpus(True)
    sched = _record(cpu + cpu, ptype, blobs)
    assert {o[1] for o in sched} >= {"h2d", "kernel", "d2h"}
    assert check_pipeline_schedule(sched) == 2 * blobs


def test_checker_detects_a_missing_edge():
    cpu = ck.ClPlatforms.all().cpus(True)
    sched = _record(cpu, ck.PIPELINE_EVENT, 4)
    # drop the wait that orders chunk 1's kernel after its H2D
    kern = [o for o in sched if o[1] == "kernel"][1]
    broken = [o for o in sched if not (o[1] == "wait" and o[2] == kern[2] and o[3] == kern[3] and o[4] == kern[4])]
    with pytest.raises(AssertionError):
        check_pipeline_schedule(broken)


@pytest.mark.parametrize("layout", [{"pipeline_reads_on_main_stream": False},
                                    {"pipeline_writes_one_stream": True},
                                    {"pipeline_writes_on_compute_stream": True}])
def test_pipeline_schedule_stream_layouts(layout):
    """Every stream layout of the event pipeline keeps H2D → kernel → D2H per
    chunk (the log names the streams the copies actually run on)."""
    cpu = ck.ClPlatforms.all().cpus(True)
    sched = _record(cpu + cpu, ck.PIPELINE_EVENT, 4, **layout)
    assert check_pipeline_schedule(sched) == 8


def test_explicit_uneven_blobs_with_array_slices():
    """Explicit pipeline blobs (compute(..., pipeline_blobs=[0, b1, ..., G])):
    uneven work-item ranges, alternating half-pipelines, and per-blob array
    slices that are NOT proportional to the blob's work items (blob k of a
    shell-streamed GEMM uploads row panel k of A and B).  The recorded
    schedule keeps H2D → kernel → D2H per blob, and the result is right."""
    src = """__global__ void k(const float* x, const float* w, float* y) {
      long long i = get_global_id(0); y[i] = x[i] * 2.0f + w[i % 64]; }"""
    cpu = ck.ClPlatforms.all().cpus(True)
    cr = ck.ClNumberCruncher(cpu, src)
    cr.cores.record_schedule = True
    cr.cores.pipeline_reads_two_streams = True  # the optional second upload stream, checked below
    bounds = [0, 64, 256, 576, 1024]  # 1, 3, 5, 7 work-groups of 64: a shell-like progression
    n = bounds[-1]
    x = ck.ClArray(np.arange(n, dtype=np.float32))
    x.partial_read = True
    x.write = False
    w = ck.ClArray(np.arange(256, dtype=np.float32))  # 4 panels of 64: blob k uploads panel k
    w.partial_read = True
    w.write = False
    w.blob_slices = [(64 * k, 64) for k in range(4)]
    y = ck.ClArray(np.zeros(n, np.float32))
    y.read = False
    x.next_param(w, y).compute(cr, 1, "k", n, 64, 0, True, ck.PIPELINE_EVENT, bounds)
    np.testing.assert_array_equal(y.array, 2 * x.array + w.array[np.arange(n) % 64])
    sched = cr.cores.schedule()
    kernels = [(o[3], o[4], o[2]) for o in sched if o[1] == "kernel"]
    assert [(b, c) for b, c, _ in kernels] == [(0, 64), (64, 192), (256, 320), (576, 448)]
    assert [s for _, _, s in kernels] == [18, 21, 18, 21]  # halves alternate
    # the two partial arrays go up on two streams (main, and upload stream 17)
    assert {o[2] for o in sched if o[1] == "h2d" and o[3] >= 0} == {0, 17}
    assert check_pipeline_schedule(sched) == 4
    # a kernel that does not wait for the second upload stream is caught
    k1 = [o for o in sched if o[1] == "kernel"][1]
    ev = [o[5] for o in sched if o[1] == "rec" and o[2] == 17 and o[3] == k1[3]][0]
    broken = [o for o in sched if not (o[1] == "wait" and o[5] == ev and o[2] == k1[2])]
    with pytest.raises(AssertionError):
        check_pipeline_schedule(broken)
    assert cr.last_record()["pipelined"]
    cr.dispose()


def test_explicit_blob_bounds_validated():
    cpu = ck.ClPlatforms.all().cpus(True)
    cr = ck.ClNumberCruncher(cpu, SRC)
    x = ck.ClArray(np.zeros(256, np.float32))
    y = ck.ClArray(np.zeros(256, np.float32))
    with pytest.raises(Exception):
        x.next_param(y).compute(cr, 1, "k", 256, 64, 0, True, ck.PIPELINE_EVENT, [0, 100, 256])
    cr.dispose()


@pytest.mark.parametrize("hwq,want", [("4", 3), ("2", 1), ("1", 1), ("", 3), ("64", 15)])
def test_queue_concurrency_follows_hw_queues(monkeypatch, hwq, want):
    """the default async / driver-pipeline queue count
    follows the GPU's hardware queue count (GPU_MAX_HW_QUEUES, 4 by default):
    one compute stream per queue the main stream leaves free, so no two
    compute streams share a queue (hardware.async_queue_count); the driver
    pipeline maps blob k to queue k mod that count."""
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", hwq)
    cpu = ck.ClPlatforms.all().cpus(True)
    cr = ck.ClNumberCruncher(cpu, SRC)
    assert cr.compute_queue_concurrency == want
    cr.dispose()
    blobs = 8
    sched = _record(cpu, ck.PIPELINE_DRIVER, blobs)
    kern = [o for o in sched if o[1] == "kernel"]
    assert len(kern) == blobs  # one kernel op per blob
    assert [o[2] for o in kern] == [1 + (k % want) for k in range(len(kern))]
    assert check_pipeline_schedule(sched) == len(kern)
    # an explicit count still wins
    cr = ck.ClNumberCruncher(cpu, SRC, queue_concurrency=16)
    assert cr.compute_queue_concurrency == 16
    cr.dispose()


@pytest.mark.parametrize("reads_main", [True, False])
def test_explicit_blobs_order_every_earlier_upload(reads_main):
    """with explicit blobs, blob q's kernels may read
    panels uploaded by earlier blobs of the other half-pipeline.  Whatever
    the read-stream setting, every blob's kernels are ordered after every
    earlier blob's uploads."""
    src = """__global__ void k(const float* x, const float* w, float* y) {
      long long i = get_global_id(0); y[i] = x[i] * 2.0f + w[i % 64]; }"""
    cpu = ck.ClPlatforms.all().cpus(True)
    cr = ck.ClNumberCruncher(cpu, src)
    cr.cores.record_schedule = True
    cr.cores.pipeline_reads_on_main_stream = reads_main
    bounds = [0, 64, 256, 576, 1024]
    n = bounds[-1]
    x = ck.ClArray(np.arange(n, dtype=np.float32))
    x.partial_read = True
    x.write = False
    w = ck.ClArray(np.arange(256, dtype=np.float32))
    w.partial_read = True
    w.write = False
    w.blob_slices = [(64 * k, 64) for k in range(4)]
    y = ck.ClArray(np.zeros(n, np.float32))
    y.read = False
    x.next_param(w, y).compute(cr, 1, "k", n, 64, 0, True, ck.PIPELINE_EVENT, bounds)
    np.testing.assert_array_equal(y.array, 2 * x.array + w.array[np.arange(n) % 64])
    assert check_pipeline_schedule(cr.cores.schedule(), prefix_uploads=True) == 4
    cr.dispose()
