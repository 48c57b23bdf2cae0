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
