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
