"""Task pool × device pool greedy scheduling (reference ``ClTask``,
``ClTaskPool``, ``ClDevicePool``; ClPipeline.cs:3247-5077).

A :class:`ClTask` freezes one ``compute()`` call — the arrays, their flags at
freeze time and the launch parameters (ClArray.cs:1552-1583).  Tasks are fed
to a :class:`ClTaskPool` (FIFO); pools are enqueued into a
:class:`ClDevicePool`, whose scheduler is native (``cek.DevicePool``,
``csrc/pool.cpp``): one C++ consumer thread per device takes the next task
the moment its device has room ("compute at will", the reference's greedy
default), with no Python and no GIL per task.  With fine-grained queue
control each device keeps several tasks in flight — the reference's
adaptive per-device limit (N/10 … N/50 tasks over the devices, at most 16,
ClPipeline.cs:4178-4236) — spread over ``max_queues_per_device`` HIP
streams (enqueue mode + round-robin queues), and retires them through
stream markers (fence-less events, recorded after each task and polled with
``hipEventQuery``), the µs-cheap counterpart of the reference's 150–300 µs
marker callbacks (Cores.cs:447).
The in-flight depth is not tied to the stream count: tasks queued in order
on one stream still keep the device busy while the host prepares the next.
A CU-partitioned device (``ClDevices.cu_partitions``) gets one stream: each
CU-masked stream owns a hardware queue, and 8 partitions × several streams
oversubscribe the GPU's queue slots (measured: 4096 one-work-group tasks
over 8 partitions ran at 38 k tasks/s with 4 streams per partition against
95 k with one; profiles/r5/README.md).  User callbacks run on
a dispatcher thread as completions arrive.

Task type flags (ClTaskType, :3247-3321): DEVICE_SELECT_BEGIN/END and
SERIAL_MODE_BEGIN/END pin a group of tasks to one device (in order),
GLOBAL_SYNCHRONIZATION_FIRST/LAST act as pool-wide barriers before/after a
task, BROADCAST runs a task on every device.
"""
from __future__ import annotations

import collections
import enum
import threading
from typing import Callable, Deque, List, Optional

from .._native import cek
from ..arrays import ClParameterGroup
from ..cruncher import PIPELINE_EVENT, ClComputeError, ClNumberCruncher
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
    """ClPipeline.cs:3792-3806: an idle device takes the next task (at will),
    or tasks go to the devices in strict rotation (round robin: the
    reference's stub "better for identical devices", e.g. 8 MI355X)."""
    DEVICE_COMPUTE_AT_WILL = 0
    DEVICE_ROUND_ROBIN = 1


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
        # run the task's kernels this many times, with kernel_repeat_name
        # between repeats (the cruncher's repeatCount / repeatKernelName for
        # one task; NotImplementedException stubs in ClPipeline.cs:3368-3373)
        self.kernel_repeats = 1
        self.kernel_repeat_name = ""

    kernelRepeats = property(lambda self: self.kernel_repeats,
                             lambda self, v: setattr(self, "kernel_repeats", int(v)))
    kernelRepeatName = property(lambda self: self.kernel_repeat_name,
                                lambda self, v: setattr(self, "kernel_repeat_name", str(v)))

    def _apply_repeats(self, call) -> None:
        call.repeats = max(1, int(self.kernel_repeats))
        call.repeat_kernel = self.kernel_repeat_name if self.kernel_repeats > 1 else ""

    def compute(self, cruncher: ClNumberCruncher) -> None:
        if self.group is None or self.type & ClTaskType.TASK_MESSAGE_NO_COMPUTE and not self.kernels:
            return
        saved = cruncher.repeat_count, cruncher.repeat_kernel_name
        cruncher.repeat_count, cruncher.repeat_kernel_name = max(1, int(self.kernel_repeats)), self.kernel_repeat_name
        try:
            cruncher._compute_group(self.group, self.compute_id, self.kernels, self.global_range, self.local_range,
                                    self.global_offset, self.pipeline, self.pipeline_type, self.pipeline_blobs,
                                    specs=self.specs)
        finally:
            cruncher.repeat_count, cruncher.repeat_kernel_name = saved

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
            for d, o in zip(ts, task.tasks):
                d._origin = o
            if ts:
                ts[0].type |= ClTaskType.TASK_MESSAGE_DEVICE_SELECT_BEGIN
                ts[-1].type |= ClTaskType.TASK_MESSAGE_DEVICE_SELECT_END
            for t in ts:
                self.tasks.append(t)
            self.total += len(ts)
            return
        d = task.duplicate()
        d._origin = task  # the caller's object learns where (and how long) it ran
        self.tasks.append(d)
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


class ClDevicePool:
    """Greedy device pool (reference ``ClDevicePool``, ClPipeline.cs:3891).

    Devices are fixed per native pool: :meth:`add_device` after tasks were
    enqueued first waits for them (``finish``) and then rebuilds the pool."""

    def __init__(self, pool_type: ClDevicePoolType = ClDevicePoolType.DEVICE_COMPUTE_AT_WILL,
                 kernel_source: str = "", fine_grained_queue_control: bool = False,
                 max_queues_per_device: int = 3, prebuilt=None):
        self.pool_type = pool_type
        self.kernel_source = kernel_source
        self.prebuilt = prebuilt
        self.max_queues = max(1, min(16, int(max_queues_per_device))) if fine_grained_queue_control else 1
        # tasks in flight per device: the adaptive limit decides, up to 16
        # (without fine-grained control: one at a time, synchronously)
        self.max_in_flight = 16 if fine_grained_queue_control else 1
        self.crunchers: List[ClNumberCruncher] = []
        self._native = None
        self._counts_base: List[int] = []
        self._cv = threading.Condition()
        self._notify = {}  # id -> [task, completions still expected]: tasks with a callback
        self._live = []  # (first id, tasks) per enqueued batch: keeps the arrays alive until finish()
        self._templates = {}  # template key -> validated ComputeCall (per device pool)
        self._next_id = 0
        self._expected = 0
        self._handled = 0
        self._errors: List[str] = []
        self._closed = False
        self._dispatcher: Optional[threading.Thread] = None

    def add_device(self, devices: ClDevices) -> None:
        """Adds each device (the same device may be added several times)."""
        for i in range(len(devices)):
            part = devices.device(i).cu_partition is not None
            cr = ClNumberCruncher(devices[i], self.kernel_source, prebuilt=self.prebuilt,
                                  queue_concurrency=1 if part else max(1, self.max_queues))
            if cr.error_code():
                raise RuntimeError(cr.error_message())
            self.crunchers.append(cr)
        self._rebuild()

    addDevice = add_device

    def _rebuild(self) -> None:
        counts = [0] * len(self.crunchers)
        if self._native is not None:
            self.finish()
            for i, c in enumerate(self.device_task_counts()):
                counts[i] = c
            self._native.close()
        self._counts_base = counts
        self._native = cek.DevicePool([c.cores for c in self.crunchers], self.max_in_flight, int(self.pool_type))
        if self._dispatcher is None:
            self._dispatcher = threading.Thread(target=self._dispatch_loop, daemon=True)
            self._dispatcher.start()

    # ---- completions / callbacks -------------------------------------------
    # Only tasks with a callback come back to Python one by one (the native
    # pool records them as notify tasks); every other task retires natively,
    # and its device and time are read for the whole batch in finish().
    def _dispatch_loop(self) -> None:
        while not self._closed:
            nat = self._native
            if nat is None:
                break
            self._handle(nat.completions(20.0))

    def _handle(self, comps) -> None:
        if not comps:
            return
        for c in comps:
            with self._cv:
                entry = self._notify.get(c.id)
            err = c.error
            if entry is not None:
                t = entry[0]
                for u in (t, getattr(t, "_origin", None)):
                    if u is not None:
                        u.device_index = c.device
                        u.elapsed_ms = c.ms
                if not err and t.callback is not None:
                    try:
                        t.callback()
                    except Exception as e:  # reported by finish()
                        self._errors.append(f"task {c.id} on device {c.device}: callback: {e!r}")
            with self._cv:
                if entry is not None:
                    entry[1] -= 1
                    if entry[1] <= 0:
                        self._notify.pop(c.id, None)
                self._handled += 1
                self._cv.notify_all()

    # ---- producer -------------------------------------------------------------
    def enqueue_task_pool(self, pool: ClTaskPool) -> None:
        """Hand every task of ``pool`` to the native device pool, in FIFO
        order.  Tasks that share a compute shape (compute id, kernels,
        ranges, pipeline, repeats) share one validated template call, built
        once per device pool (``_templates``); the native side gets one batch
        (``DevicePool.enqueue_batch``) holding one copy of each template."""
        if self._native is None:
            raise RuntimeError("device pool has no devices (add_device first)")
        cr0 = self.crunchers[0]
        ndev = len(self.crunchers)
        cache = self._templates
        tasks = list(pool.tasks)
        pool.tasks.clear()
        with self._cv:
            first_id = self._next_id
            self._next_id += len(tasks)
            self._live.append((first_id, tasks))
        # handed over in chunks: the consumers start on the first chunk while
        # this thread prepares the next (one pool for the queue-depth policy)
        for c0 in range(0, max(1, len(tasks)), self.ENQUEUE_CHUNK):
            self._enqueue_chunk(tasks, c0, min(len(tasks), c0 + self.ENQUEUE_CHUNK), first_id, cr0, ndev, cache)

    ENQUEUE_CHUNK = 256

    def _enqueue_chunk(self, tasks, c0, c1, first_id, cr0, ndev, cache) -> None:
        local = {}  # template key -> index into this chunk's template list
        templates = []
        which, arrays, types = [], [], []
        notify = []  # (id, [task, copies]) of tasks with a callback
        expected = 0
        NO_COMPUTE, BROADCAST = int(ClTaskType.TASK_MESSAGE_NO_COMPUTE), int(ClTaskType.TASK_MESSAGE_BROADCAST)
        NOTIFY = int(cek.DevicePool.NOTIFY)
        for k in range(c0, c1):
            t = tasks[k]
            ty = int(t.type)
            kn = t.kernels
            if t.group is not None and kn and not (ty & NO_COMPUTE and not kn):
                bl = t.pipeline_blobs
                key = (t.compute_id, kn if isinstance(kn, str) else tuple(kn), t.global_range, t.local_range,
                       t.global_offset, bool(t.pipeline), bool(t.pipeline_type),
                       bl if isinstance(bl, int) else tuple(bl), int(t.kernel_repeats), t.kernel_repeat_name)
                j = local.get(key)
                if j is None:
                    call = cache.get(key)
                    if call is None:
                        try:
                            call = cr0._build_call(ClParameterGroup(), t.compute_id, t.kernels, t.global_range,
                                                   t.local_range, t.global_offset, t.pipeline, t.pipeline_type,
                                                   t.pipeline_blobs, specs=[])
                            t._apply_repeats(call)
                        except ClComputeError as e:
                            raise ClComputeError(f"task {first_id + k}: {e}") from None
                        cache[key] = call
                    j = local[key] = len(templates)
                    templates.append(call)
                which.append(j)
                arrays.append(t.specs)
            else:
                j = local.get(None)
                if j is None:
                    j = local[None] = len(templates)
                    templates.append(cek.ComputeCall())  # barrier / message tasks: no kernels
                which.append(j)
                arrays.append([])
            if t.callback is not None:
                copies = ndev if ty & BROADCAST else 1
                notify.append((first_id + k, [t, copies]))
                expected += copies
                ty |= NOTIFY
            types.append(ty)
        with self._cv:
            self._notify.update(notify)
            self._expected += expected
        if c1 > c0:
            self._native.enqueue_batch(templates, which, arrays, types, list(range(first_id + c0, first_id + c1)),
                                       len(tasks), c0 > 0)

    enqueueTaskPool = enqueue_task_pool

    def finish(self) -> int:
        """Block until every enqueued task has completed and its callback has
        run; raises if a task failed.  Returns 0."""
        if self._native is None:
            return 0
        self._native.finish()
        while True:
            self._handle(self._native.completions(0.0))
            with self._cv:
                if self._handled >= self._expected:
                    break
                self._cv.wait(0.005)
        with self._cv:
            live, self._live = self._live, []
        for first, tasks in live:  # where and how long every task ran
            devs, mss = self._native.results(first, len(tasks))
            for t, d, m in zip(tasks, devs, mss):
                if d >= 0:
                    t.device_index = d
                    t.elapsed_ms = m
                    o = t.__dict__.get("_origin")
                    if o is not None:
                        o.device_index = d
                        o.elapsed_ms = m
        errs = [f"task {e.id} on device {e.device}: {e.error}" for e in self._native.take_errors()]
        with self._cv:
            errs, self._errors = self._errors + errs, []
        if errs:
            raise ClComputeError("device pool: " + "; ".join(errs))
        return 0

    def device_task_counts(self) -> List[int]:
        if self._native is None:
            return []
        return [int(b + c) for b, c in zip(self._counts_base, self._native.device_task_counts())]

    def device_busy_ms(self) -> List[float]:
        return list(self._native.device_busy_ms()) if self._native is not None else []

    # ---- scheduling policy (ClPipeline.cs:4100-4236, :4788-4817) --------------
    def queue_limit(self) -> int:
        """Current per-device queue-depth limit: follows the head pool's
        progress (N/10 → N/20 → N/33 → N/50 → 2 → 1 tasks, over the device
        count, at most 16)."""
        return int(self._native.queue_limit()) if self._native is not None else 0

    def queue_limit_history(self) -> List[int]:
        """Every distinct limit the consumers have applied, in order."""
        return list(self._native.queue_limit_history()) if self._native is not None else []

    def marker_reach_speeds(self) -> List[float]:
        """Per device: markers retired per ms, 15-sample moving average
        (reference ``markerReachSpeed``)."""
        return list(self._native.marker_speeds()) if self._native is not None else []

    markerReachSpeed = marker_reach_speeds

    def device_in_flight(self) -> List[int]:
        """Per device: tasks taken and not yet retired (the load measure a
        select/serial group is placed by)."""
        return list(self._native.device_in_flight()) if self._native is not None else []

    def dispose(self) -> None:
        if self._native is not None:
            try:
                self.finish()
            finally:
                self._closed = True
                self._native.close()
                if self._dispatcher is not None:
                    self._dispatcher.join(5.0)
        for cr in self.crunchers:
            cr.dispose()
        self.crunchers = []
