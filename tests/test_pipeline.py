"""Stage pipelines on the CPU device: device→device ClPipeline with double
buffers (results appear after 2·stages pushes, like ClPipeline.cs:114-124)
and the single-device multi-stream DevicePipeline."""
import numpy as np

import cekirdekler_amd as ck
from cekirdekler_amd.parallel.pipeline import (ClPipelineStage, DevicePipeline, DevicePipelineArray,
                                               DevicePipelineArrayType, DevicePipelineStage)

N = 1024
K1 = "__global__ void add1(const float* x, float* y) { long long i = get_global_id(0); y[i] = x[i] + 1.0f; }"
K2 = "__global__ void mul2(const float* y, float* t, float* z) { long long i = get_global_id(0); t[i] = y[i]; z[i] = t[i] * 2.0f; }"
K3 = "__global__ void sub3(const float* z, float* w) { long long i = get_global_id(0); w[i] = z[i] - 3.0f; }"


def _stage(devs, src, name, ins, hid, outs):
    s = ClPipelineStage()
    s.add_devices(devs)
    s.add_kernels(src, name, [N], [64])
    s.add_input_buffers(*ins)
    if hid:
        s.add_hidden_buffers(*hid)
    s.add_output_buffers(*outs)
    return s


def test_three_stage_pipeline_latency_and_values():
    cpu = ck.ClPlatforms.all().cpus(True)
    x, y1, y2, t, z1, z2, w = (np.zeros(N, np.float32) for _ in range(7))
    s1 = _stage(cpu, K1, "add1", [x], None, [y1])
    s2 = _stage(cpu, K2, "mul2", [y2], [t], [z1])
    s3 = _stage(cpu, K3, "sub3", [z2], None, [w])
    s1.prepend_to_stage(s2)
    s3.append_to_stage(s2)
    pipe = s1.make_pipeline()
    res = np.zeros(N, np.float32)
    seen = []
    for p in range(12):
        data = np.full(N, float(p), np.float32)
        ready = pipe.push_data([data], [res])
        if ready:
            seen.append(float(res[0]))
            assert np.all(res == res[0])
    # f(p) = (p + 1) * 2 - 3, emitted with a lag of 2·stages = 6 pushes
    assert seen == [(p + 1) * 2 - 3 for p in range(len(seen))]
    assert len(seen) == 12 - 6
    pipe.dispose()


def test_device_pipeline_transition_double_buffer():
    cpu = ck.ClPlatforms.all().cpus(True)
    src = K1 + "\n" + K3
    dp = DevicePipeline(cpu, src)
    inp = DevicePipelineArray(DevicePipelineArrayType.INPUT, np.zeros(N, np.float32))
    mid = DevicePipelineArray(DevicePipelineArrayType.TRANSITION, np.zeros(N, np.float32))
    out = DevicePipelineArray(DevicePipelineArrayType.OUTPUT, np.zeros(N, np.float32))
    a = DevicePipelineStage("add1", N, 64)
    a.bind_array(inp)
    a.bind_array(mid)
    b = DevicePipelineStage("sub3", N, 64)
    b.bind_array(mid)
    b.bind_array(out)
    dp.add_stage(a)
    dp.add_stage(b)
    got = []
    for p in range(6):
        dp.input_buffer(inp).array[:] = p
        dp.feed()
        got.append(float(dp.output_buffer(out).array[0]))
    # value p enters at feed p+1, passes stage a at p+1, stage b at p+2
    assert got[3:] == [(p + 1) - 3 for p in range(1, 4)]
    dp.dispose()


def test_multi_device_stage_sees_hidden_constants():
    """A stage on several devices (range-split, host-staged) reads its hidden
    buffers' initial host contents on every device."""
    cpu = ck.ClPlatforms.all().cpus(True)
    ks = "__global__ void scale(const float* x, const float* c, float* y) { long long i = get_global_id(0); y[i] = x[i] * c[0]; }"
    x, y = np.zeros(N, np.float32), np.zeros(N, np.float32)
    c = np.array([3.0], np.float32)
    s1 = _stage(cpu + cpu, ks, "scale", [x], [c], [y])
    s2 = _stage(cpu, K3, "sub3", [np.zeros(N, np.float32)], None, [np.zeros(N, np.float32)])
    s1.prepend_to_stage(s2)
    pipe = s1.make_pipeline()
    res = np.zeros(N, np.float32)
    seen = []
    for p in range(8):
        if pipe.push_data([np.full(N, float(p), np.float32)], [res]):
            assert np.all(res == res[0])
            seen.append(float(res[0]))
    assert seen == [3.0 * p - 3.0 for p in range(len(seen))] and len(seen) == 8 - 4
    pipe.dispose()


def test_timeline_coverage_helpers():
    from cekirdekler_amd.parallel.pipeline import _coverage, _intersection

    busy, multi = _coverage([(0, 4), (2, 6), (10, 11)])
    assert busy == 7 and multi == 2
    assert _intersection(0, 10, [(2, 3), (2.5, 5), (8, 20)]) == 5


def test_device_pipeline_timeline_on_cpu():
    """Serial mode runs the stages one after another: spans are recorded per
    stage and no two stages overlap."""
    cpu = ck.ClPlatforms.all().cpus(True)
    N = 1 << 12
    src = ("__global__ void add1(const float* x, float* y) { long long i = get_global_id(0); y[i] = x[i] + 1.0f; }\n"
           "__global__ void sub3(const float* z, float* w) { long long i = get_global_id(0); w[i] = z[i] - 3.0f; }")
    dp = DevicePipeline(cpu, src)
    inp = DevicePipelineArray(DevicePipelineArrayType.INPUT, np.zeros(N, np.float32))
    mid = DevicePipelineArray(DevicePipelineArrayType.TRANSITION, np.zeros(N, np.float32))
    out = DevicePipelineArray(DevicePipelineArrayType.OUTPUT, np.zeros(N, np.float32))
    a = DevicePipelineStage("add1", N, 256)
    a.bind_array(inp)
    a.bind_array(mid)
    b = DevicePipelineStage("sub3", N, 256)
    b.bind_array(mid)
    b.bind_array(out)
    dp.add_stage(a)
    dp.add_stage(b)
    dp.enable_serial_mode()
    dp.record_timeline = True
    for _ in range(4):
        dp.feed()
    spans = dp._collect()
    assert sorted({st for st, _, _ in spans}) == [0, 1] and len(spans) == 8
    assert all(e >= b for _, b, e in spans)
    assert dp.query_timeline_overlap_percentage() == 0.0
    assert dp.stages_overlapping_percentages() == [0.0, 0.0]
    dp.dispose()


def test_stage_enqueue_mode_runs_its_kernels_back_to_back():
    """ClPipelineStage.enqueueMode (ClPipeline.cs:212): a stage with two
    kernels runs them without a host sync between them and gives the same
    results as the synchronous stage."""
    cpu = ck.ClPlatforms.all().cpus(True)
    outs = []
    for enq in (False, True):
        x, w = np.zeros(N, np.float32), np.zeros(N, np.float32)
        s = ClPipelineStage()
        s.add_devices(cpu)
        s.add_kernels(K1, "add1", [N], [64])
        s.add_kernels("__global__ void dbl(const float* x, float* y) { long long i = get_global_id(0); y[i] = y[i] * 2.0f; }",
                      "dbl", [N], [64])
        s.add_input_buffers(x)
        s.add_output_buffers(w)
        s.enqueueMode = enq
        assert s.enqueue_mode is enq
        pipe = s.make_pipeline()
        res = np.zeros(N, np.float32)
        got = []
        for p in range(6):
            if pipe.push_data([np.full(N, float(p), np.float32)], [res]):
                got.append(float(res[0]))
        outs.append(got)
        assert not s.cruncher.enqueue_mode  # left after every run
        pipe.dispose()
    assert outs[0] == outs[1] == [(p + 1) * 2.0 for p in range(len(outs[0]))]


def test_device_pipeline_stage_queries_and_user_event_counter():
    """DevicePipelineStage.hasInput / hasOutput (ClPipeline.cs:2812-2840), the
    stopHostDeviceTransmission switch (its effect on copies is checked on a
    GPU: a CPU device computes in host memory) and the ClUserEvent counter."""
    cpu = ck.ClPlatforms.all().cpus(True)
    dp = DevicePipeline(cpu, K1)
    inp = DevicePipelineArray(DevicePipelineArrayType.INPUT, np.zeros(N, np.float32))
    out = DevicePipelineArray(DevicePipelineArrayType.OUTPUT, np.zeros(N, np.float32))
    a = DevicePipelineStage("add1", N, 64)
    a.bind_array(inp)
    a.bind_array(out)
    assert a.hasInput and a.hasOutput
    assert not DevicePipelineStage("add1", N, 64).has_input
    dp.add_stage(a)
    a.stopHostDeviceTransmission = True
    assert a.stop_host_device_transmission
    dp.feed()
    a.stop_host_device_transmission = False
    dp.input_buffer(inp).array[:] = 7
    dp.feed()
    dp.feed()
    assert float(dp.output_buffer(out).array[0]) == 8.0
    dp.async_host_work()
    dp.dispose()
    ev = ck.ClUserEvent()
    ev.inc()
    ev.inc()
    ev.dec()
    assert ev.count == 1
    ev.dec()
    assert ev.count == 0
    import pytest
    with pytest.raises(RuntimeError):
        ev.dec()
    ev.dispose()
