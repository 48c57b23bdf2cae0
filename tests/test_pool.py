"""Task pool × device pool on logical CPU devices (the reference allows the
same device several times, ClPipeline.cs:4337)."""
import threading

import numpy as np
import pytest

import cekirdekler_amd as ck
from cekirdekler_amd.parallel.pool import ClDevicePool, ClDevicePoolType, ClTaskPool, ClTaskType

SRC = """
__global__ void fill(float* x, float* v) { x[get_global_id(0)] = v[0]; }
__global__ void add(float* x, float* v) { x[get_global_id(0)] += v[0]; }
"""


def _task(kernel, n, value, arr=None):
    x = arr if arr is not None else ck.ClArray(np.zeros(n, np.float32))
    v = ck.ClArray(np.array([value], np.float32))
    v.write = False
    return x, x.next_param(v).task(1, kernel, n, 64)


@pytest.mark.parametrize("fine", [False, True])
def test_pool_runs_every_task_once(fine):
    cpu = ck.ClPlatforms.all().cpus(True)
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, fine, 3)
    pool.add_device(cpu + cpu + cpu)
    tp = ClTaskPool()
    arrays, done = [], []
    lock = threading.Lock()
    for i in range(48):
        x, t = _task("fill", 256, float(i))
        t.set_callback(lambda i=i: (lock.acquire(), done.append(i), lock.release()))
        tp.feed(t)
        arrays.append(x)
    pool.enqueue_task_pool(tp)
    pool.finish()
    for i, x in enumerate(arrays):
        np.testing.assert_array_equal(x.array, float(i))
    assert sorted(done) == list(range(48))
    assert sum(pool.device_task_counts()) == 48
    pool.dispose()


def test_frozen_flags_and_serial_group():
    cpu = ck.ClPlatforms.all().cpus(True)
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, True, 4)
    pool.add_device(cpu + cpu)
    x = ck.ClArray(np.zeros(128, np.float32))
    tp = ClTaskPool()
    # a serial group of 10 "add 1" tasks on one shared array must run in order on one device
    for k in range(10):
        _, t = _task("add", 128, 1.0, x)
        if k == 0:
            t.type = ClTaskType.TASK_MESSAGE_SERIAL_MODE_BEGIN
        if k == 9:
            t.type = ClTaskType.TASK_MESSAGE_SERIAL_MODE_END
        tp.feed(t)
    pool.enqueue_task_pool(tp)
    pool.finish()
    np.testing.assert_array_equal(x.array, 10.0)
    pool.dispose()


def test_global_sync_orders_phases():
    cpu = ck.ClPlatforms.all().cpus(True)
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, True, 3)
    pool.add_device(cpu + cpu)
    order = []
    lock = threading.Lock()
    tp = ClTaskPool()
    for i in range(12):
        _, t = _task("fill", 256, 1.0)
        if i == 6:
            t.type = ClTaskType.TASK_MESSAGE_GLOBAL_SYNCHRONIZATION_FIRST
        t.set_callback(lambda i=i: (lock.acquire(), order.append(i), lock.release()))
        tp.feed(t)
    pool.enqueue_task_pool(tp)
    pool.finish()
    assert sorted(order) == list(range(12))
    assert set(order[:6]) == set(range(6))  # everything before the barrier finished first
    pool.dispose()


def test_broadcast_runs_on_every_device_and_select_group_pins():
    cpu = ck.ClPlatforms.all().cpus(True)
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, True, 3)
    pool.add_device(cpu + cpu + cpu)
    tp = ClTaskPool()
    seen = []
    lock = threading.Lock()
    _, b = _task("fill", 256, 7.0)
    b.type = ClTaskType.TASK_MESSAGE_BROADCAST
    b.set_callback(lambda: (lock.acquire(), seen.append("b"), lock.release()))
    tp.feed(b)
    # a device-select group: every task of it runs on one device
    group = []
    for k in range(6):
        _, t = _task("fill", 256, float(k))
        if k == 0:
            t.type = ClTaskType.TASK_MESSAGE_DEVICE_SELECT_BEGIN
        if k == 5:
            t.type = ClTaskType.TASK_MESSAGE_DEVICE_SELECT_END
        group.append(t)
        tp.feed(t)
    pool.enqueue_task_pool(tp)
    pool.finish()
    assert seen == ["b"] * 3  # one callback per device copy
    assert len({t.device_index for t in group}) == 1 and group[0].device_index is not None
    assert sum(pool.device_task_counts()) == 3 + 6
    pool.dispose()


def test_task_error_is_reported_by_finish():
    cpu = ck.ClPlatforms.all().cpus(True)
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, True, 2)
    pool.add_device(cpu)
    tp = ClTaskPool()
    _, t = _task("fill", 256, 1.0)
    t.kernels = "no_such_kernel"
    tp.feed(t)
    _, ok = _task("fill", 256, 2.0)
    tp.feed(ok)
    pool.enqueue_task_pool(tp)
    with pytest.raises(ck.ClComputeError, match="no_such_kernel"):
        pool.finish()
    assert sum(pool.device_task_counts()) == 2  # the failing task retired too
    pool.dispose()


def test_tasks_without_callback_retire_natively_and_report_device():
    """only tasks with a callback cross back into Python
    one by one; every other task's device and time are read for the whole
    batch at finish() (and reach the caller's object, not only the pool's
    copy).  A raising callback is reported by finish()."""
    cpu = ck.ClPlatforms.all().cpus(True, max_cpu_cores=1)
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, True, 2)
    pool.add_device(cpu + cpu)
    tp = ClTaskPool()
    plain = []
    for i in range(40):
        _, t = _task("fill", 256, float(i))
        plain.append(t)
        tp.feed(t)
    _, bad = _task("fill", 256, 1.0)
    bad.set_callback(lambda: 1 / 0)
    tp.feed(bad)
    pool.enqueue_task_pool(tp)
    with pytest.raises(ck.ClComputeError, match="ZeroDivisionError"):
        pool.finish()
    assert all(t.device_index in (0, 1) for t in plain)
    assert all(t.elapsed_ms >= 0 for t in plain)
    assert not pool._notify and not pool._live  # nothing held after finish
    assert len(pool._templates) == 1  # one shape, one template for the pool's lifetime
    pool.dispose()


SPIN = """
__global__ void spin(float* x, int* it) {
  long long i = get_global_id(0);
  float v = x[i];
  for (int k = 0; k < it[0]; ++k) v = v * 0.999f + 0.5f;
  x[i] = v;
}
__global__ void fill(float* x, int* it) { x[get_global_id(0)] = (float)it[0]; }
"""


def _spin_task(kernel, n, iters):
    x = ck.ClArray(np.zeros(n, np.float32))
    it = ck.ClArray(np.array([iters], np.int32))
    it.write = False
    return x, x.next_param(it).task(1, kernel, n, 64)


def test_select_group_lands_on_least_loaded_device():
    """A device-select group goes to the device with the fewest tasks in
    flight (ClPipeline.cs:4100-4127), not to whichever consumer grabs it."""
    cpu = ck.ClPlatforms.all().cpus(True)
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SPIN, True, 3)
    pool.add_device(cpu + cpu)
    busy = ClTaskPool()
    xb, tb = _spin_task("spin", 64 * 8, 3_000_000)  # one long task keeps its device busy
    busy.feed(tb)
    pool.enqueue_task_pool(busy)
    import time
    for _ in range(200):  # wait until a consumer has taken it
        if sum(pool.device_in_flight()) == 1:
            break
        time.sleep(0.005)
    busy_dev = pool.device_in_flight().index(1)
    grp = ClTaskPool()
    tasks = []
    for k in range(4):
        _, t = _spin_task("fill", 64, k)
        t.type = (ClTaskType.TASK_MESSAGE_DEVICE_SELECT_BEGIN if k == 0 else
                  ClTaskType.TASK_MESSAGE_DEVICE_SELECT_END if k == 3 else ClTaskType.TASK_MESSAGE_DEFAULT)
        grp.feed(t)
        tasks.append(t)
    pool.enqueue_task_pool(grp)
    pool.finish()
    assert {t.device_index for t in tasks} == {1 - busy_dev}
    assert tb.device_index == busy_dev
    pool.dispose()


def test_queue_limit_shrinks_as_pool_drains():
    """Per-device queue depth follows pool progress (ClPipeline.cs:4178-4236):
    N/10 → N/20 → N/33 → N/50 → 2 → 1 tasks over the device count."""
    cpu = ck.ClPlatforms.all().cpus(True)
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SPIN, True, 16)
    pool.add_device(cpu + cpu)
    tp = ClTaskPool()
    for _ in range(400):
        _, t = _spin_task("spin", 64, 2000)
        tp.feed(t)
    pool.enqueue_task_pool(tp)
    pool.finish()
    h = pool.queue_limit_history()
    # 400 tasks / 2 devices: 20 → 10 → 6 → 4 → 1, floored at 2 in flight
    assert h[0] == 16 and h[-1] == 2, h          # N/10/2 = 20 clamped to 16 queues
    assert all(a >= b for a, b in zip(h, h[1:])), h
    assert {10, 6, 4}.issubset(h), h
    assert len(pool.marker_reach_speeds()) == 2
    pool.dispose()


def test_task_kernel_repeats():
    """ClTask.kernelRepeats / kernelRepeatName (stubs in the reference,
    ClPipeline.cs:3368-3373): one task runs its kernel list that many times,
    through the device pool and through task.compute(cruncher)."""
    cpu = ck.ClPlatforms.all().cpus(True)
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, False, 2)
    pool.add_device(cpu + cpu)
    tp = ClTaskPool()
    arrays = []
    for reps in (1, 2, 5):
        x, t = _task("add", 256, 1.0)
        t.kernelRepeats = reps
        assert t.kernel_repeats == reps and t.kernelRepeatName == ""
        tp.feed(t)
        arrays.append((reps, x))
    pool.enqueue_task_pool(tp)
    pool.finish()
    for reps, x in arrays:
        np.testing.assert_array_equal(x.array, float(reps))
    pool.dispose()
    cr = ck.ClNumberCruncher(cpu, SRC)
    x, t = _task("add", 256, 2.0)
    t.kernel_repeats = 3
    t.compute(cr)
    np.testing.assert_array_equal(x.array, 6.0)
    assert cr.repeat_count == 1  # the cruncher's own setting is restored
    cr.dispose()


@pytest.mark.parametrize("fine", [False, True])
def test_round_robin_rotates_tasks(fine):
    """ClDevicePoolType.DEVICE_ROUND_ROBIN (ClPipeline.cs:3801-3806): task k
    runs on device k mod D; a serial group takes one rotation slot as a
    whole and stays in order on its device; a global barrier is untargeted."""
    cpu = ck.ClPlatforms.all().cpus(True)
    D = 3
    pool = ClDevicePool(ClDevicePoolType.DEVICE_ROUND_ROBIN, SRC, fine, 3)
    pool.add_device(cpu + cpu + cpu)
    tp = ClTaskPool()
    tasks, arrays = [], []
    for i in range(12):
        x, t = _task("fill", 256, float(i))
        tp.feed(t)
        tasks.append(t)
        arrays.append(x)
    shared = ck.ClArray(np.zeros(128, np.float32))
    group = []
    for k in range(4):  # serial group: rotation slot 12 -> device 0
        _, t = _task("add", 128, 1.0, shared)
        t.type = (ClTaskType.TASK_MESSAGE_SERIAL_MODE_BEGIN if k == 0 else
                  ClTaskType.TASK_MESSAGE_SERIAL_MODE_END if k == 3 else ClTaskType.TASK_MESSAGE_DEFAULT)
        tp.feed(t)
        group.append(t)
    x, t = _task("fill", 256, 99.0)  # rotation slot 13 -> device 1
    tp.feed(t)
    tasks.append(t)
    arrays.append(x)
    pool.enqueue_task_pool(tp)
    pool.finish()
    for i, t in enumerate(tasks[:12]):
        assert t.device_index == i % D, (i, t.device_index)
    assert {t.device_index for t in group} == {12 % D}
    assert tasks[12].device_index == 13 % D
    np.testing.assert_array_equal(shared.array, 4.0)
    for i, x in enumerate(arrays[:12]):
        np.testing.assert_array_equal(x.array, float(i))
    assert pool.device_task_counts() == [8, 5, 4]
    pool.dispose()


@pytest.mark.parametrize("fine", [False, True])
def test_round_robin_group_with_barrier_flags(fine):
    """a serial group whose BEGIN carries a global barrier
    (its own flag, or inherited from the previous task's SYNC_LAST) and whose
    END carries one too must still take one rotation slot as a whole, stay in
    order on its device, and release the rotation afterwards."""
    cpu = ck.ClPlatforms.all().cpus(True)
    D = 3
    pool = ClDevicePool(ClDevicePoolType.DEVICE_ROUND_ROBIN, SRC, fine, 3)
    pool.add_device(cpu + cpu + cpu)
    tp = ClTaskPool()
    before = []
    for i in range(2):  # slots 0, 1; the second one's SYNC_LAST is inherited by the group's BEGIN
        x, t = _task("fill", 256, float(i))
        if i == 1:
            t.type = ClTaskType.TASK_MESSAGE_GLOBAL_SYNCHRONIZATION_LAST
        tp.feed(t)
        before.append(t)
    shared = ck.ClArray(np.zeros(128, np.float32))
    group = []
    for k in range(5):  # slot 2 -> device 2, as a whole
        _, t = _task("add", 128, 1.0, shared)
        if k == 0:
            t.type = ClTaskType.TASK_MESSAGE_SERIAL_MODE_BEGIN | ClTaskType.TASK_MESSAGE_GLOBAL_SYNCHRONIZATION_FIRST
        elif k == 4:
            t.type = ClTaskType.TASK_MESSAGE_SERIAL_MODE_END | ClTaskType.TASK_MESSAGE_GLOBAL_SYNCHRONIZATION_FIRST
        tp.feed(t)
        group.append(t)
    after = []
    for i in range(4):  # slots 3.. -> devices 0, 1, 2, 0: the rotation was released
        _, t = _task("fill", 256, 5.0)
        tp.feed(t)
        after.append(t)
    pool.enqueue_task_pool(tp)
    pool.finish()
    assert [t.device_index for t in before] == [0, 1]
    assert {t.device_index for t in group} == {2}
    np.testing.assert_array_equal(shared.array, 5.0)
    assert [t.device_index for t in after] == [i % D for i in range(3, 7)]
    pool.dispose()


def test_task_with_kernel_list():
    """ClTask kernels given as a list of names (accepted by
    the cruncher's name splitter) also go through the pool's template key."""
    cpu = ck.ClPlatforms.all().cpus(True)
    pool = ClDevicePool(ClDevicePoolType.DEVICE_COMPUTE_AT_WILL, SRC, False, 2)
    pool.add_device(cpu + cpu)
    tp = ClTaskPool()
    arrays = []
    for i in range(4):
        x = ck.ClArray(np.zeros(256, np.float32))
        v = ck.ClArray(np.array([float(i)], np.float32))
        v.write = False
        t = x.next_param(v).task(1, ["fill", "add"], 256, 64)
        tp.feed(t)
        arrays.append(x)
    pool.enqueue_task_pool(tp)
    pool.finish()
    for i, x in enumerate(arrays):
        np.testing.assert_array_equal(x.array, 2.0 * i)
    pool.dispose()
