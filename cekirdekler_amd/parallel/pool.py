"""Task pool × device pool greedy scheduling (reference ``ClTask``,
``ClTaskPool``, ``ClDevicePool``; ClPipeline.cs:3247-5077).

A :class:`ClTask` freezes one ``compute()`` call — the arrays, their flags at
freeze time and the launch parameters (ClArray.cs:1552-1583).  Tasks are fed
to a :class:`ClTaskPool` (FIFO); pools are enqueued into a
:class:`ClDevicePool`, which runs one consumer thread per device: an idle
device takes the next task immediately ("compute at will", the reference's
greedy default).  Each device keeps up to ``max_queues_per_device`` tasks in
flight on its own HIP streams (enqueue mode + round-robin queues) and tracks
completion with stream-written marker words (``hipStreamWriteValue64``), the
µs-cheap counterpart of the reference's 150–300 µs marker callbacks
(Cores.cs:447).

Task type flags (ClTaskType, :3247-3321): DEVICE_SELECT_BEGIN/END and
SERIAL_MODE_BEGIN/END pin a group of tasks to one device (in order),
GLOBAL_SYNCHRONIZATION_FIRST/LAST act as pool-wide barriers before/after a
task, BROADCAST runs a task on every device.
"""
from __future__ import annotations

import collections
import enum
import threading
import time
from typing import Callable, Deque, List, Optional

from .._native import cek
from ..arrays import ClParameterGroup
from ..cruncher import PIPELINE_EVENT, ClNumberCruncher
from ..hardware import ClDevices


class ClTaskType(enum.IntFlag):
    TASK_MESSAGE_DEFAULT = 0
    TASK_MESSAGE_DEVICE_SELECT_BEGIN = 1
    TASK_MESSAGE_DEVICE_SELECT_END = 2
    TASK_MESSAGE_GLOBAL_SYNCHRONIZATION_FIRST = 4
    TASK_MESSAGE_GLOBAL_SYNCHRONIZATION_LAST = 8
    TASK_MESSAGE_BROADCAST = 16
    TASK_MESSAGE_NO_COMPUTE = 32
    TASK_MESSAGE_SERIAL_MODE_BEGIN = 64
    TASK_MESSAGE_SERIAL_MODE_END = 128


class ClDevicePoolType(enum.IntEnum):
    DEVICE_COMPUTE_AT_WILL = 0


class ClTask:
    """A frozen compute (reference ``ClTask``)."""

    def __init__(self, group: Optional[ClParameterGroup], compute_id: int = 0, kernels: str = "",
                 global_range: int = 0, local_range: int = 256, global_offset: int = 0,
                 pipeline: bool = False, pipeline_type: bool = PIPELINE_EVENT, pipeline_blobs: int = 4):
        self.group = group
        # freeze array flags now: later flag changes do not affect the task
        self.specs = [a._spec() for a in group.arrays] if group is not None else []
        self.compute_id = compute_id
        self.kernels = kernels
        self.global_range = global_range
        self.local_range = local_range
        self.global_offset = global_offset
        self.pipeline = pipeline
        self.pipeline_type = pipeline_type
        self.pipeline_blobs = pipeline_blobs
        self.type = ClTaskType.TASK_MESSAGE_DEFAULT
        self.callback: Optional[Callable[[], None]] = None
        self._callback_ran = False
        self.device_index: Optional[int] = None  # which device computed it (set by the pool)
        self.elapsed_ms = 0.0

    def compute(self, cruncher: ClNumberCruncher) -> None:
        if self.group is None or self.type & ClTaskType.TASK_MESSAGE_NO_COMPUTE and not self.kernels:
            return
        cruncher._compute_group(self.group, self.compute_id, self.kernels, self.global_range, self.local_range,
                                self.global_offset, self.pipeline, self.pipeline_type, self.pipeline_blobs,
                                specs=self.specs)

    def set_callback(self, fn: Callable[[], None]) -> None:
        self.callback = fn
        self._callback_ran = False

    setCallBack = set_callback

    def _run_callback(self) -> None:
        if self.callback is not None and not self._callback_ran:
            self._callback_ran = True
            self.callback()

    def duplicate(self) -> "ClTask":
        t = ClTask(None)
        t.__dict__.update(self.__dict__)
        t._callback_ran = False
        return t

    @staticmethod
    def device_barrier() -> "ClTask":
        """Stub kept for parity: a plain task (reference returns a plain task
        too, ClPipeline.cs:3502)."""
        return ClTask(None)

    @staticmethod
    def global_barrier() -> "ClTask":
        t = ClTask(None)
        t.type = ClTaskType.TASK_MESSAGE_GLOBAL_SYNCHRONIZATION_FIRST
        return t

    deviceBarrier = device_barrier
    globalBarrier = global_barrier


class ClTaskGroup:
    """Reference stub (ClPipeline.cs:3526-3599): a list of tasks that a pool
    feeds as one device-select group."""

    def __init__(self, type_=None):
        self.tasks: List[ClTask] = []
        self.type = type_

    def add(self, task: ClTask) -> None:
        self.tasks.append(task)


class ClTaskPool:
    """FIFO of tasks (reference ``ClTaskPool``)."""

    def __init__(self):
        self.tasks: Deque[ClTask] = collections.deque()
        self.total = 0

    def feed(self, task) -> None:
        if isinstance(task, ClTaskGroup):
            ts = [t.duplicate() for t in task.tasks]
            if ts:
                ts[0].type |= ClTaskType.TASK_MESSAGE_DEVICE_SELECT_BEGIN
                ts[-1].type |= ClTaskType.TASK_MESSAGE_DEVICE_SELECT_END
            for t in ts:
                self.tasks.append(t)
            self.total += len(ts)
            return
        self.tasks.append(task.duplicate())
        self.total += 1

    def reset(self) -> None:
        self.tasks.clear()
        self.total = 0

    def remaining_task_groups_or_tasks(self) -> int:
        return len(self.tasks)

    remainingTaskGroupsOrTasks = remaining_task_groups_or_tasks

    def next_task(self) -> Optional[ClTask]:
        return self.tasks.popleft() if self.tasks else None

    nextTask = next_task


class _DeviceWorker(threading.Thread):
    """Consumer thread of one device.  Keeps up to ``max_queues`` tasks in
    flight; each issued task carries a marker ticket (stream slot, value)
    written by the device when the task's commands complete, so completion
    is detected per task, in any order, without host callbacks."""

    def __init__(self, pool: "ClDevicePool", index: int, cruncher: ClNumberCruncher):
        super().__init__(daemon=True)
        self.pool, self.index, self.cruncher = pool, index, cruncher
        self.inflight: List[tuple] = []  # (task, slot, value)
        self.completed = 0
        self.busy_ms = 0.0

    def _retire(self) -> int:
        cores = self.cruncher.cores
        keep, done = [], 0
        for t, slot, val in self.inflight:
            if cores.marker_word(0, slot) >= val:
                self.completed += 1
                done += 1
                self.pool._task_done(self, t)
            else:
                keep.append((t, slot, val))
        self.inflight = keep
        return done

    def _wait_one(self) -> None:
        while self.inflight and self._retire() == 0:
            time.sleep(0.00002)

    def _drain(self) -> None:
        cr = self.cruncher
        if cr.enqueue_mode:
            cr.enqueue_mode = False  # synchronises every stream of the device
        self._retire()
        for t, _, _ in self.inflight:  # (defensive) all commands are complete now
            self.completed += 1
            self.pool._task_done(self, t)
        self.inflight = []

    def run(self) -> None:
        cr = self.cruncher
        asynchronous = self.pool.max_queues > 1
        if asynchronous:
            cr.fine_grained_queue_control = True
        while True:
            t = self.pool._take(self)
            if t is None:
                if self.inflight:
                    if asynchronous:
                        self._wait_one()
                    continue
                if cr.enqueue_mode:
                    cr.enqueue_mode = False
                if self.pool._closed:
                    break
                self.pool._wait_for_work(self)
                continue
            t.device_index = self.index
            t0 = time.perf_counter()
            if asynchronous:
                if not cr.enqueue_mode:
                    cr.enqueue_mode = True
                cr.enqueue_mode_async_enable = not t._serial
                t.compute(cr)
                slot, val = cr.cores.last_marker(0)
                self.inflight.append((t, slot, val))
                self._retire()
                while len(self.inflight) >= self.pool.max_queues:
                    self._wait_one()
            else:
                t.compute(cr)
                self.completed += 1
                self.pool._task_done(self, t)
            self.busy_ms += (time.perf_counter() - t0) * 1e3
        if cr.enqueue_mode:
            cr.enqueue_mode = False


class ClDevicePool:
    """Greedy device pool (reference ``ClDevicePool``)."""

    def __init__(self, pool_type: ClDevicePoolType = ClDevicePoolType.DEVICE_COMPUTE_AT_WILL,
                 kernel_source: str = "", fine_grained_queue_control: bool = False,
                 max_queues_per_device: int = 3, prebuilt=None):
        self.pool_type = pool_type
        self.kernel_source = kernel_source
        self.prebuilt = prebuilt
        self.max_queues = max(1, min(16, int(max_queues_per_device))) if fine_grained_queue_control else 1
        self.workers: List[_DeviceWorker] = []
        self._lock = threading.Condition()
        self._queue: Deque[ClTask] = collections.deque()
        self._outstanding = 0
        self._closed = False
        self._owner: Optional[_DeviceWorker] = None  # device-select group owner
        self._blocked = False

    def add_device(self, devices: ClDevices) -> None:
        """Adds each device (the same device may be added several times)."""
        for i in range(len(devices)):
            cr = ClNumberCruncher(devices[i], self.kernel_source, prebuilt=self.prebuilt,
                                  queue_concurrency=max(1, self.max_queues))
            if cr.error_code():
                raise RuntimeError(cr.error_message())
            w = _DeviceWorker(self, len(self.workers), cr)
            self.workers.append(w)
            w.start()

    addDevice = add_device

    def enqueue_task_pool(self, pool: ClTaskPool) -> None:
        with self._lock:
            sync_next = False
            while pool.tasks:
                t = pool.tasks.popleft()
                if sync_next:  # GLOBAL_SYNC_LAST of the previous task = barrier before this one
                    t.type |= ClTaskType.TASK_MESSAGE_GLOBAL_SYNCHRONIZATION_FIRST
                sync_next = bool(t.type & ClTaskType.TASK_MESSAGE_GLOBAL_SYNCHRONIZATION_LAST)
                t._serial = bool(t.type & (ClTaskType.TASK_MESSAGE_SERIAL_MODE_BEGIN |
                                           ClTaskType.TASK_MESSAGE_SERIAL_MODE_END))
                if t.type & ClTaskType.TASK_MESSAGE_BROADCAST:
                    for w in self.workers:
                        d = t.duplicate()
                        d._serial = t._serial
                        d._broadcast_target = w
                        self._queue.append(d)
                        self._outstanding += 1
                else:
                    self._queue.append(t)
                    self._outstanding += 1
            self._lock.notify_all()

    enqueueTaskPool = enqueue_task_pool

    # ---- consumer protocol --------------------------------------------------
    def _take(self, w: _DeviceWorker) -> Optional[ClTask]:
        with self._lock:
            while True:
                if not self._queue:
                    return None
                t = self._queue[0]
                target = getattr(t, "_broadcast_target", None)
                if target is not None and target is not w:
                    # find a task this worker may take; broadcast copies wait for their device
                    for j, u in enumerate(self._queue):
                        if getattr(u, "_broadcast_target", None) in (None, w):
                            if self._owner is not None and self._owner is not w and getattr(u, "_broadcast_target", None) is None:
                                return None
                            del self._queue[j]
                            return self._after_take(w, u)
                    return None
                if self._owner is not None and self._owner is not w and target is None:
                    return None  # a device-select group is pinned to another device
                if t.type & ClTaskType.TASK_MESSAGE_GLOBAL_SYNCHRONIZATION_FIRST:
                    if self._running > 0:
                        self._blocked = True
                        return None
                self._queue.popleft()
                return self._after_take(w, t)

    _running = 0

    def _after_take(self, w: _DeviceWorker, t: ClTask) -> ClTask:
        if t.type & (ClTaskType.TASK_MESSAGE_DEVICE_SELECT_BEGIN | ClTaskType.TASK_MESSAGE_SERIAL_MODE_BEGIN):
            self._owner = w
        if t.type & (ClTaskType.TASK_MESSAGE_DEVICE_SELECT_END | ClTaskType.TASK_MESSAGE_SERIAL_MODE_END):
            if self._owner is w:
                self._owner = None
        self._running += 1
        return t

    def _wait_for_work(self, w: _DeviceWorker) -> None:
        with self._lock:
            if not self._queue and not self._closed:
                self._lock.wait(0.01)
            elif self._queue:
                self._lock.wait(0.0005)

    def _task_done(self, w: _DeviceWorker, t: ClTask) -> None:
        try:
            t._run_callback()
        finally:
            with self._lock:
                self._outstanding -= 1
                self._running -= 1
                self._lock.notify_all()

    def finish(self) -> int:
        """Block until every enqueued task has completed; returns 0."""
        with self._lock:
            while self._outstanding > 0:
                self._lock.wait(0.01)
        return 0

    def device_task_counts(self) -> List[int]:
        return [w.completed for w in self.workers]

    def dispose(self) -> None:
        self.finish()
        with self._lock:
            self._closed = True
            self._lock.notify_all()
        for w in self.workers:
            w.join(5.0)
            w.cruncher.dispose()
