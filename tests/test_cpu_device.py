"""compute() on the CPU device (the reference's de-facto fake backend,
SURVEY §4): flag semantics, logical multi-device splits, pipelines, repeats,
enqueue mode, barrier kernels (fibers) and the usage-type-2 Cores API.  The
SAXPY 1M config of BASELINE.json must match numpy bit-for-bit."""
import numpy as np
import pytest

import cekirdekler_amd as ck

SRC = """
__global__ void saxpy(const float* a, const float* x, float* y) {
  long long i = get_global_id(0);
  y[i] = a[0] * x[i] + y[i];
}
__global__ void copy2(const float* src, float* dst) {
  long long i = get_global_id(0);
  dst[2 * i] = src[2 * i];
  dst[2 * i + 1] = src[2 * i + 1];
}
__global__ void inc(float* x) { x[get_global_id(0)] += 1.0f; }
__global__ void count(float* x, int* c) { if (get_global_id(0) == 0) c[0] += 1; }
__global__ void incc(float* x, int* c) { x[get_global_id(0)] += 1.0f; }
__global__ void groupsum(const float* x, float* out) {
  __shared__ float s[64];
  int l = (int)get_local_id(0);
  s[l] = x[get_global_id(0)];
  __syncthreads();
  for (int w = 32; w > 0; w >>= 1) { if (l < w) s[l] += s[l + w]; __syncthreads(); }
  if (l == 0) out[get_global_id(0) / 64] = s[0];
}
"""


@pytest.fixture(scope="module")
def cpu():
    return ck.ClPlatforms.all().cpus(True)


@pytest.fixture(scope="module")
def cr(cpu):
    c = ck.ClNumberCruncher(cpu, SRC)
    assert c.error_code() == 0, c.error_message()
    return c


def test_saxpy_1m_bit_exact(cr):
    n = 1 << 20
    a = ck.ClArray(np.array([1.7], np.float32))
    a.write = False
    x = ck.ClArray(np.random.rand(n).astype(np.float32))
    y0 = np.random.rand(n).astype(np.float32)
    y = ck.ClArray(y0.copy())
    a.next_param(x, y).compute(cr, 1, "saxpy", n, 256)
    np.testing.assert_array_equal(y.array, np.float32(1.7) * x.array + y0)


def test_kernel_with_inner_loop_vectorized_runner_exact(cpu):
    """The CPU runner vectorizes across work-items ("omp simd") also when the
    kernel body has a loop of its own; every item must still follow its own
    scalar fp32 chain (fmaf per step, no contraction or reassociation)."""
    src = """__global__ void poly(const float* x, float* y) {
      long long i = get_global_id(0);
      float v = x[i], acc = y[i];
      for (int k = 0; k < 24; ++k) acc = fmaf(acc, v, 0.25f);
      if (i % 7 == 3) acc = -acc;
      y[i] = acc;
    }"""
    c = ck.ClNumberCruncher(cpu + cpu, src)
    n = 256 * 40
    rng = np.random.default_rng(5)
    x = ck.ClArray(rng.uniform(-0.9, 0.9, n).astype(np.float32))
    y0 = rng.uniform(-1, 1, n).astype(np.float32)
    y = ck.ClArray(y0.copy())
    x.partial_read = y.partial_read = True
    x.next_param(y).compute(c, 1, "poly", n, 256)
    acc = y0.copy()
    for _ in range(24):  # fmaf: one rounding of the exact a·b + c
        acc = (acc.astype(np.float64) * x.array + 0.25).astype(np.float32)
    acc[np.arange(n) % 7 == 3] *= -1
    np.testing.assert_array_equal(y.array, acc)


def test_repeated_compute_reuses_the_built_call(cpu):
    """A repeated compute reuses its native call; any flag or storage change
    of an array, or another range, builds a new one — and the results follow
    the new flags."""
    c = ck.ClNumberCruncher(cpu, SRC)
    x = ck.ClArray(np.zeros(256, np.float32))
    g = ck.ClParameterGroup([x])
    first = c._build_call(g, 1, "inc", 256, 64)
    assert c._build_call(g, 1, "inc", 256, 64) is first
    assert c._build_call(g, 1, "inc", 128, 64) is not first  # another range
    x.write = False  # another flag: another spec, another call
    assert c._build_call(g, 1, "inc", 256, 64) is not first
    x.write = True
    x.elements_per_work_item = 2
    assert c._build_call(g, 1, "inc", 128, 64) is not first
    x.elements_per_work_item = 1
    for _ in range(3):
        x.compute(c, 1, "inc", 256, 64)
    np.testing.assert_array_equal(x.array, np.full(256, 3.0, np.float32))
    x.compute(c, 1, "inc", 128, 64)  # half the range: only the first half moves
    np.testing.assert_array_equal(x.array[:128], np.full(128, 4.0, np.float32))
    np.testing.assert_array_equal(x.array[128:], np.full(128, 3.0, np.float32))


@pytest.mark.parametrize("pipeline", [False, True])
def test_guarded_loop_kernel_exact_and_bounded(cpu, pipeline):
    """A guard ("if (i >= n) return;") ahead of a loop: the vectorized
    runner must leave the items past the guard untouched and match the
    scalar fp32 chain on the others."""
    src = """__global__ void gpoly(const float* x, float* y, const int* n) {
      long long i = get_global_id(0);
      if (i >= n[0]) return;
      float v = x[i], acc = y[i];
      for (int k = 0; k < 16; ++k) acc = fmaf(acc, v, 0.25f);
      y[i] = acc;
    }"""
    c = ck.ClNumberCruncher(cpu + cpu, src)
    g, lim = 256 * 24, 256 * 24 - 77
    rng = np.random.default_rng(9)
    x = ck.ClArray(rng.uniform(-0.9, 0.9, g).astype(np.float32))
    y0 = rng.uniform(-1, 1, g).astype(np.float32)
    y = ck.ClArray(y0.copy())
    nn = ck.ClArray(np.array([lim], np.int32))
    nn.write = False
    x.next_param(y, nn).compute(c, 1, "gpoly", g, 256, pipeline=pipeline, pipeline_blobs=4)
    acc = y0[:lim].copy()
    for _ in range(16):
        acc = (acc.astype(np.float64) * x.array[:lim] + 0.25).astype(np.float32)
    np.testing.assert_array_equal(y.array[:lim], acc)
    np.testing.assert_array_equal(y.array[lim:], y0[lim:])


def test_kernel_that_cannot_be_inlined_still_builds(cpu):
    """Kernels are force-inlined into their runner; one the compiler cannot
    inline (here: non-tail recursion, which g++ refuses as "recursive
    inlining") is rebuilt as a plain call."""
    src = """__global__ void rec(float* x, int* d) {
      long long i = get_global_id(0);
      if (d[i] <= 0) return;
      d[i] -= 1;
      x[i] += 1.0f;
      rec(x, d);
      x[i] += 0.5f;
    }"""
    c = ck.ClNumberCruncher(cpu, src)
    assert c.error_code() == 0, c.error_message()
    depth = np.arange(256, dtype=np.int32) % 4
    x = ck.ClArray(np.zeros(256, np.float32))
    d = ck.ClArray(depth.copy())
    x.next_param(d).compute(c, 1, "rec", 256, 64)
    np.testing.assert_array_equal(x.array, 1.5 * depth.astype(np.float32))


def test_elements_per_work_item_and_partial(cpu):
    devs = cpu + cpu + cpu
    cr = ck.ClNumberCruncher(devs, SRC)
    n = 3 * 64 * 16
    src = ck.ClArray(np.arange(2 * n, dtype=np.float32))
    dst = ck.ClArray(np.zeros(2 * n, np.float32))
    src.partial_read = True
    src.elements_per_work_item = 2
    dst.elements_per_work_item = 2
    dst.read = False
    for _ in range(3):
        src.next_param(dst).compute(cr, 2, "copy2", n, 64)
    np.testing.assert_array_equal(dst.array, src.array)
    r = cr.ranges(2)
    assert len(r) == 3 and sum(r) == n and all(x % 64 == 0 for x in r)


@pytest.mark.parametrize("ptype", [ck.PIPELINE_EVENT, ck.PIPELINE_DRIVER])
def test_pipelines_on_cpu(cpu, ptype):
    cr = ck.ClNumberCruncher(cpu + cpu, SRC)
    n = 2 * 256 * 8 * 4
    x = ck.ClArray(np.zeros(n, np.float32))
    x.partial_read = True
    for k in range(3):
        x.compute(cr, 3, "inc", n, 256, 0, True, ptype, 8)
    np.testing.assert_array_equal(x.array, 3.0)
    assert cr.last_record()["pipelined"]


def test_repeat_with_sync_kernel(cr):
    x = ck.ClArray(np.zeros(1024, np.float32))
    c = ck.ClArray(np.zeros(1, np.int32))
    c.write_all = True
    cr.repeat_count = 5
    cr.repeat_kernel_name = "count"
    try:
        x.next_param(c).compute(cr, 4, "incc", 1024, 64)
    finally:
        cr.repeat_count = 1
        cr.repeat_kernel_name = ""
    np.testing.assert_array_equal(x.array, 5.0)
    assert c.array[0] == 5  # sync kernel (global=local, offset 0) runs after each repeat


def test_barrier_kernel_uses_fibers(cr):
    n = 64 * 32
    x = ck.ClArray(np.random.rand(n).astype(np.float32))
    out = ck.ClArray(np.zeros(n // 64, np.float32))
    out.elements_per_work_item = 1
    out.write_all = True
    x.next_param(out).compute(cr, 5, "groupsum", n, 64)
    np.testing.assert_allclose(out.array, x.array.reshape(-1, 64).sum(1), rtol=1e-5)


def test_validation_errors(cr):
    x = ck.ClArray(np.zeros(100, np.float32))
    with pytest.raises(ck.ClComputeError):
        x.compute(cr, 6, "inc", 100, 64)        # not a multiple of local
    with pytest.raises(ck.ClComputeError):
        x.compute(cr, 6, "inc", 128, 64)        # array shorter than G*epw
    assert cr.number_of_errors_happened >= 2


def test_enqueue_mode_and_markers(cr):
    x = ck.ClArray(np.zeros(4096, np.float32))
    cr.fine_grained_queue_control = True
    cr.enqueue_mode = True
    for _ in range(10):
        x.compute(cr, 8, "inc", 4096, 256)
    cr.enqueue_mode = False
    cr.fine_grained_queue_control = False
    np.testing.assert_array_equal(x.array, 10.0)
    assert cr.count_markers_reached() >= 10
    assert cr.count_markers_remaining() == 0


def test_usage_type_2_cores_api():
    cores = ck.Cores("cpu", SRC, local_range=64)
    n = 1024
    a = np.array([2.0], np.float32)
    x = np.arange(n, dtype=np.float32)
    y = np.ones(n, np.float32)
    cores.compute("saxpy", 1, "", [a, x, y], [" read ", " partial read ", " partial read write "], [1, 1, 1],
                  n, 1)
    np.testing.assert_array_equal(y, 2 * x + 1)
    rep = cores.performance_report(1)
    assert "Compute-ID: 1" in rep and "workitems" in rep


def test_load_balancer_with_injected_imbalance(cpu):
    cr = ck.ClNumberCruncher(cpu + cpu, SRC)
    cr.set_time_scale(1, 3.0)
    n = 1 << 16
    x = ck.ClArray(np.zeros(n, np.float32))
    for _ in range(25):
        x.compute(cr, 9, "inc", n, 256)
    r = cr.ranges(9)
    assert r[0] > r[1] * 1.5
    assert cr.normalized_global_ranges_of_devices(9)[0] > 0.55
    hist = cr.performance_history(9)     # 10-deep window, rows sum to 1 once filled
    assert len(hist) == 10 and all(len(h) == 2 for h in hist)
    assert abs(sum(hist[-1]) - 1.0) < 1e-6 and hist[-1][0] > hist[-1][1]


def test_kernel_arity_mismatch_is_rejected(cr):
    # inc takes one array; passing two would shift the hidden offset argument
    x = ck.ClArray(np.zeros(256, np.float32))
    c = ck.ClArray(np.zeros(1, np.int32))
    c.write = False
    with pytest.raises(Exception, match="array parameter"):
        x.next_param(c).compute(cr, 40, "inc", 256, 64)


def test_granularity_quantizes_device_ranges(cpu):
    c = ck.ClNumberCruncher(cpu + cpu, SRC)
    c.set_time_scale(1, 3.0)
    x = ck.ClArray(np.zeros(64 * 40, np.float32))
    for _ in range(6):
        x.compute(c, 1, "inc", 64 * 40, 64, granularity=64 * 4)
        assert all(r % 256 == 0 for r in c.ranges(1)), c.ranges(1)
    np.testing.assert_array_equal(x.array, 6.0)
    assert c.ranges(1)[0] > c.ranges(1)[1]
    with pytest.raises(ck.ClComputeError):
        x.compute(c, 2, "inc", 64 * 40, 64, granularity=96)
    c.dispose()


def test_user_event_on_cpu_device_is_a_no_op_gate(cr):
    ev = ck.ClUserEvent()
    ev.add_cruncher(cr)
    assert ev.armed
    x = ck.ClArray(np.zeros(256, np.float32))
    x.compute(cr, 41, "inc", 256, 64)   # CPU streams are not gated
    ev.trigger()
    assert not ev.armed
    np.testing.assert_array_equal(x.array, 1.0)


def test_disable_device_rebalances_over_the_others(cpu):
    c = ck.ClNumberCruncher(cpu + cpu + cpu, SRC)
    x = ck.ClArray(np.zeros(64 * 30, np.float32))
    x.compute(c, 1, "inc", 64 * 30, 64)
    c.disable_device(1)
    x.compute(c, 1, "inc", 64 * 30, 64)
    r = c.ranges(1)
    assert r[1] == 0 and sum(r) == 64 * 30 and r[0] > 0 and r[2] > 0
    c.enable_device(1)
    for _ in range(3):
        x.compute(c, 1, "inc", 64 * 30, 64)
    assert c.ranges(1)[1] > 0
    np.testing.assert_array_equal(x.array, 5.0)
    c.dispose()


def test_injected_failure_and_auto_failover(cpu):
    c = ck.ClNumberCruncher(cpu + cpu, SRC)
    x = ck.ClArray(np.zeros(64 * 16, np.float32))
    c.cores.inject_failure(1, 1)
    with pytest.raises(Exception, match="injected failure"):
        x.compute(c, 1, "inc", 64 * 16, 64)
    assert c.device_enabled(1)                 # without failover nothing changes
    x.array[:] = 0
    c.auto_failover = True
    c.cores.inject_failure(1, 1)
    x.compute(c, 2, "inc", 64 * 16, 64)        # device 1 fails; its slice reruns on device 0
    assert not c.device_enabled(1) and c.cores.failovers == 1
    np.testing.assert_array_equal(x.array, 1.0)
    x.compute(c, 2, "inc", 64 * 16, 64)        # later calls skip the dropped device
    assert c.ranges(2) == [64 * 16, 0]
    np.testing.assert_array_equal(x.array, 2.0)
    c.dispose()


def test_record_log_json_lines(cpu, tmp_path, monkeypatch):
    import json

    import cekirdekler_amd.cruncher as crm

    path = tmp_path / "records.jsonl"
    monkeypatch.setattr(crm, "_RECORD_LOG", str(path))
    c = ck.ClNumberCruncher(cpu, SRC)
    x = ck.ClArray(np.zeros(256, np.float32))
    for _ in range(3):
        x.compute(c, 5, "inc", 256, 64)
    lines = [json.loads(l) for l in path.read_text().splitlines()]
    assert len(lines) == 3 and lines[-1]["compute_id"] == 5 and lines[-1]["kernels"] == ["inc"]
    assert sum(lines[-1]["ranges"]) == 256 and lines[-1]["h2d_bytes"] == 1024
    c.dispose()


def test_devices_ranked_by_nbody_time(cpu):
    """ClDevices.devicesWithHighestDirectNbodyPerformance (ClObjectApi.cs:1222-1244):
    every device runs the N-body test alone; the list comes back fastest first
    (here: two copies of the CPU device, so only the shape is checked)."""
    plats = ck.ClPlatforms.all()
    ranked = (plats.cpus(True) + plats.cpus(True)).devices_with_highest_direct_nbody_performance(n=1024)
    assert len(ranked) == 2 and all(d.is_cpu for d in ranked)


def test_debug_checks_flag_and_env(cpu, monkeypatch):
    """debug_checks round-trips (host buffers on the CPU device are the
    user's arrays, so only GPU buffers get guard tails) and CEK_DEBUG=1
    turns it on at construction."""
    c = ck.ClNumberCruncher(cpu, SRC)
    assert not c.debug_checks
    c.debug_checks = True
    x = ck.ClArray(np.zeros(256, np.float32))
    x.compute(c, 1, "inc", 256, 64)
    np.testing.assert_array_equal(x.array, np.ones(256, np.float32))
    c.dispose()
    monkeypatch.setenv("CEK_DEBUG", "1")
    c2 = ck.ClNumberCruncher(cpu, SRC)
    assert c2.debug_checks
    c2.dispose()


def test_license_text_names_gpl():
    """Reference ``License.cs:58``: the library exposes its license notice."""
    import cekirdekler_amd
    text = cekirdekler_amd.license_text()
    assert "GNU General Public License" in text
    assert "Cekirdekler" in text


def test_usable_cpus_respects_share(monkeypatch):
    """The CPU device's pool is sized to the CPUs the process may use
    (affinity, cgroup quota, OMP_NUM_THREADS), not the machine's count."""
    import os

    from cekirdekler_amd.hardware import usable_cpus

    n = usable_cpus()
    assert 1 <= n <= (os.cpu_count() or 1)
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    assert usable_cpus() <= 2
    dev = ck.ClPlatforms.all().cpus(True).device(0)
    monkeypatch.delenv("CEK_CPU_THREADS", raising=False)
    assert dev.native_info().cpu_threads <= 2


def test_array_release_inside_locked_region_does_not_deadlock():
    """A garbage collection inside ``_release_uid``'s locked region runs
    ``ClArray.__del__`` on the same thread, which releases its own uid: the
    registry lock must be re-entrant (this hung a GPU test run)."""
    import threading

    from cekirdekler_amd import arrays

    done = threading.Event()

    def nested():
        with arrays._live_lock:
            arrays._release_uid(-1)
        done.set()

    t = threading.Thread(target=nested, daemon=True)
    t.start()
    t.join(10)
    assert done.is_set()


def test_queue_concurrency_and_last_used_compute_id(cpu):
    cr = ck.ClNumberCruncher(cpu, "__global__ void k(float* x) { x[get_global_id(0)] += 1.0f; }",
                             queue_concurrency=40)
    assert cr.computeQueueConcurrency == 16  # clamped like the reference's ≤ 16
    x = ck.ClArray(np.zeros(256, np.float32))
    x.compute(cr, 7, "k", 256, 64)
    assert cr.lastUsedComputeId == 7 and cr.numberOfDevices == cr.number_of_devices
    cr.dispose()


def test_cpu_pool_shared_between_crunchers_and_safe_concurrently(cpu):
    """Crunchers whose CPU device has the same thread count run on one
    process-wide pool (CpuPool::shared); two CPU devices of one set keep two
    pools, and two crunchers computing at once from two threads take turns
    on the shared pool with correct results."""
    import threading

    a = ck.ClNumberCruncher(cpu, SRC)
    b = ck.ClNumberCruncher(cpu, SRC)
    two = ck.ClNumberCruncher(cpu + cpu, SRC)
    try:
        pa, pb = a._cores.cpu_pool_id(0), b._cores.cpu_pool_id(0)
        assert pa != 0 and pa == pb
        assert two._cores.cpu_pool_id(0) == pa
        assert two._cores.cpu_pool_id(1) not in (0, pa)
        n = 1 << 18
        errs = []

        def run(cr, seed):
            try:
                rng = np.random.default_rng(seed)
                av = ck.ClArray(np.array([1.5], np.float32))
                av.write = False
                x = ck.ClArray(rng.random(n, dtype=np.float32))
                for _ in range(20):
                    y0 = rng.random(n, dtype=np.float32)
                    y = ck.ClArray(y0.copy())
                    av.next_param(x, y).compute(cr, 7, "saxpy", n, 256)
                    np.testing.assert_array_equal(y.array, np.float32(1.5) * x.array + y0)
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        ts = [threading.Thread(target=run, args=(c, s)) for s, c in enumerate((a, b, two))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs, errs
    finally:
        for c in (a, b, two):
            c.dispose()


def test_cpu_pool_not_reused_across_fork(cpu):
    """A process forked after a CPU cruncher exists builds its own pool: the
    parent's pool threads do not exist in the child (a shared pool reused
    there would wait for them forever)."""
    import os

    cr = ck.ClNumberCruncher(cpu, SRC)
    x = ck.ClArray(np.zeros(1 << 14, np.float32))
    x.compute(cr, 1, "inc", 1 << 14, 256)
    pid = os.fork()
    if pid == 0:  # child: a new cruncher of the same size, one compute
        code = 3
        try:
            c2 = ck.ClNumberCruncher(cpu, SRC)
            y = ck.ClArray(np.zeros(1 << 14, np.float32))
            y.compute(c2, 1, "inc", 1 << 14, 256)
            code = 0 if float(y.array.sum()) == float(1 << 14) else 4
        finally:
            os._exit(code)
    import time

    t_end = time.time() + 60
    while True:
        done, status = os.waitpid(pid, os.WNOHANG)
        if done:
            break
        if time.time() > t_end:
            os.kill(pid, 9)
            os.waitpid(pid, 0)
            raise AssertionError("forked child hung on the CPU pool")
        time.sleep(0.05)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status
    assert float(x.array.sum()) == float(1 << 14)
    cr.dispose()
