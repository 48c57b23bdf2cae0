"""Stage pipelines.

**Device→device stage pipeline** (reference ``ClPipeline`` /
``ClPipelineStage``, ClPipeline.cs:41-1874).  A linear chain of stages, each
with its own device set, kernels and input/hidden/output buffers.  Inputs and
outputs are double-buffered: on every :meth:`ClPipeline.push_data` all stages
compute concurrently on their current buffers while the previous results move
one stage forward through the duplicates; then current and duplicate swap.
Results appear after ~2·stages pushes (same ready-counter rule as the
reference, :114-124).

MI355X-native difference: the reference moves every stage transition
device→host→device (ClPipeline.cs:1422-1574).  Here every stage keeps its
buffers resident on each of its devices (a CPU device's "replica" is the
host array itself).  A stage transition is a set of async copies on the
native :class:`CopyEngine`: each device of the next stage pulls every slice
of the previous stage's output straight from the device that computed it
(``hipMemcpyPeerAsync`` over that GPU pair's xGMI link), so a multi-device
stage never bounces through host memory.  Slice ownership follows the
balancer split of the stage's last kernel, snapshotted when the push that
wrote the output ended.  Only pipeline inputs and results cross PCIe.

**Single-device multi-queue pipeline** (reference ``DevicePipeline`` /
``DevicePipelineStage`` / ``DevicePipelineArray(Type)``,
ClPipeline.cs:2363-3234).  N stages on one device, each launched on its own
HIP stream (enqueue mode + async queues) so their kernels overlap;
TRANSITION arrays are double-buffered between neighbouring stages,
INPUT/OUTPUT arrays double-buffered towards the host.
"""
from __future__ import annotations

import enum
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, List, Optional, Sequence

import numpy as np

from .._native import cek, gpu_available
from ..arrays import ClArray, ClParameterGroup, as_clarray
from ..cruncher import ClNumberCruncher
from ..hardware import ClDevices

_peer_enabled = False
_peer_lock = threading.Lock()


def _enable_peers() -> None:
    global _peer_enabled
    with _peer_lock:
        if not _peer_enabled and gpu_available():
            cek.enable_peer_access()
            _peer_enabled = True


def _clone(a: ClArray) -> ClArray:
    d = ClArray(a.N, a.dtype if not a.is_bf16 else "bfloat16")
    d.array[:] = a.array
    d.elements_per_work_item = a.elements_per_work_item
    d.elements_per_group = a.elements_per_group
    return d


# =========================================================================== device → device


class ClPipelineStage:
    """One stage: devices + kernels + input/hidden/output buffers."""

    def __init__(self, debug: bool = False):
        self.debug = debug
        self.devices: Optional[ClDevices] = None
        self.kernel_source = ""
        self.kernel_names: List[str] = []
        self.global_ranges: List[int] = []
        self.local_ranges: List[int] = []
        self.init_names: List[str] = []
        self.init_globals: List[int] = []
        self.init_locals: List[int] = []
        self.inputs: List[ClArray] = []
        self.hiddens: List[ClArray] = []
        self.outputs: List[ClArray] = []
        self._in_dup: List[ClArray] = []
        self._out_dup: List[ClArray] = []
        self.previous: Optional["ClPipelineStage"] = None
        self.next: Optional["ClPipelineStage"] = None
        self.cruncher: Optional[ClNumberCruncher] = None
        self.elapsed_time = 0.0
        self.stage_id = 0
        self._resident = False
        # run this stage's kernels back to back without a host sync between
        # them (ClPipelineStage.enqueueMode, ClPipeline.cs:212); the stage
        # still drains before its outputs move on
        self.enqueue_mode = False

    # ---- building -----------------------------------------------------------
    def add_devices(self, devices: ClDevices) -> None:
        self.devices = devices if self.devices is None else self.devices + devices

    def add_kernels(self, kernels: str, kernel_names: str, global_ranges: Sequence[int],
                    local_ranges: Sequence[int]) -> None:
        self.kernel_source += "\n" + kernels
        names = kernel_names.split() if isinstance(kernel_names, str) else list(kernel_names)
        if len(names) != len(global_ranges) or len(names) != len(local_ranges):
            raise ValueError("one global and one local range per kernel name")
        self.kernel_names += names
        self.global_ranges += list(global_ranges)
        self.local_ranges += list(local_ranges)

    def initializer_kernel(self, names: str, global_ranges: Sequence[int], local_ranges: Sequence[int]) -> None:
        """Kernels run once on both buffer sets when the pipeline is built
        (reference initializerKernel, ClPipeline.cs:1678)."""
        self.init_names = names.split()
        self.init_globals = list(global_ranges)
        self.init_locals = list(local_ranges)

    def add_input_buffers(self, *arrays) -> None:
        self.inputs += [as_clarray(a) for a in arrays]

    def add_hidden_buffers(self, *arrays) -> None:
        self.hiddens += [as_clarray(a) for a in arrays]

    def add_output_buffers(self, *arrays) -> None:
        self.outputs += [as_clarray(a) for a in arrays]

    def prepend_to_stage(self, stage: "ClPipelineStage") -> None:
        """This stage runs before ``stage``."""
        self.next, stage.previous = stage, self

    def append_to_stage(self, stage: "ClPipelineStage") -> None:
        """This stage runs after ``stage``."""
        stage.next, self.previous = self, stage

    addDevices = add_devices
    addKernels = add_kernels
    initializerKernel = initializer_kernel
    addInputBuffers = add_input_buffers
    addHiddenBuffers = add_hidden_buffers
    addOutputBuffers = add_output_buffers
    prependToStage = prepend_to_stage
    appendToStage = append_to_stage
    enqueueMode = property(lambda self: self.enqueue_mode,
                           lambda self, v: setattr(self, "enqueue_mode", bool(v)))

    def make_pipeline(self) -> "ClPipeline":
        head = self
        while head.previous is not None:
            head = head.previous
        stages = []
        s = head
        while s is not None:
            stages.append(s)
            s = s.next
        for i, st in enumerate(stages):
            st.stage_id = i
            st._setup()
        for st in stages:
            st._run_initializers()
        return ClPipeline(stages, self.debug)

    makePipeline = make_pipeline

    # ---- runtime --------------------------------------------------------------
    def _setup(self) -> None:
        if self.devices is None or len(self.devices) == 0:
            raise ValueError(f"stage {self.stage_id} has no devices")
        self.cruncher = ClNumberCruncher(self.devices, self.kernel_source, no_pipelining=True)
        if self.cruncher.error_code():
            raise RuntimeError(f"stage {self.stage_id} build failed:\n{self.cruncher.error_message()}")
        self._resident = True
        self._ordinals = [d.info.ordinal if d.is_gpu else -1 for d in self.devices]
        if any(o >= 0 for o in self._ordinals):
            _enable_peers()
        self._in_dup = [_clone(a) for a in self.inputs]
        self._out_dup = [_clone(a) for a in self.outputs]
        for a in self.inputs + self._in_dup + self.outputs + self._out_dup + self.hiddens:
            a.read, a.partial_read, a.write = False, False, False
        # materialise every replica with the host contents once (constants,
        # initial state); from here on nothing moves except by the pipeline
        for a in self.inputs + self._in_dup + self.outputs + self._out_dup + self.hiddens:
            for d in range(len(self._ordinals)):
                self.cruncher.upload(a, d)
        self._owner = None      # (refs, ranges, local) of the output's writer
        self._owner_next = None

    def _snapshot_owner(self) -> None:
        """Record which device computed which slice of this push's outputs
        (the split of the stage's last kernel, compute id ``len(kernels)``)."""
        if len(self._ordinals) == 1 or not self.kernel_names:
            self._owner_next = None
            return
        cid = len(self.kernel_names)
        self._owner_next = (self.cruncher.references(cid), self.cruncher.ranges(cid), self.local_ranges[-1])

    def _slices(self, a: ClArray):
        """(device, byte offset, bytes) of every device's slice of output
        ``a`` as last written; one whole-array slice from device 0 for a
        single-device stage or before the first push."""
        if self._owner is None:
            return [(0, 0, a.nbytes)]
        refs, ranges, local = self._owner
        item = a.nbytes // max(a.N, 1)
        out = []
        for d, (r, n) in enumerate(zip(refs, ranges)):
            if a.elements_per_group:
                b, c = (r // local) * a.elements_per_group, (n // local) * a.elements_per_group
            else:
                b, c = r * a.elements_per_work_item, n * a.elements_per_work_item
            b, c = min(b * item, a.nbytes), c * item
            c = max(0, min(c, a.nbytes - b))
            if c:
                out.append((d, b, c))
        return out

    def _group(self, dup: bool) -> ClParameterGroup:
        ins = self._in_dup if dup else self.inputs
        outs = self._out_dup if dup else self.outputs
        return ClParameterGroup(ins + self.hiddens + outs)

    def _run_initializers(self) -> None:
        for dup in (False, True):
            g = self._group(dup)
            for k, G, L in zip(self.init_names, self.init_globals, self.init_locals):
                g.compute(self.cruncher, 1000 + self.stage_id, k, G, L)

    def run(self) -> None:
        t0 = time.perf_counter()
        g = self._group(False)
        enqueue = self.enqueue_mode and len(self.kernel_names) > 1
        if enqueue:
            self.cruncher.enqueue_mode = True
        try:
            for i, (k, G, L) in enumerate(zip(self.kernel_names, self.global_ranges, self.local_ranges)):
                g.compute(self.cruncher, 1 + i, k, G, L)
        finally:
            if enqueue:
                self.cruncher.enqueue_mode = False  # drains the stage's queues
        self.elapsed_time = (time.perf_counter() - t0) * 1e3

    def _replica_ptr(self, a: ClArray, device: int = 0) -> int:
        return self.cruncher.device_pointer(a, device)

    def switch_input_buffers(self) -> None:
        self.inputs, self._in_dup = self._in_dup, self.inputs

    def switch_output_buffers(self) -> None:
        self.outputs, self._out_dup = self._out_dup, self.outputs


def _transfer(engine, dst_stage: Optional[ClPipelineStage], dst: ClArray, src_stage: Optional[ClPipelineStage],
              src: ClArray) -> None:
    """Enqueue the copies that move src's data into dst on ``engine``.
    Stage sides are device-resident replicas (every device of the
    destination stage receives every slice, pulled from the source device
    that owns it); a ``None`` stage is the host array itself."""
    n = min(src.nbytes, dst.nbytes)
    if src_stage is None:
        srcs = [(-1, src.host_pointer(), 0, n)]
    else:
        srcs = [(src_stage._ordinals[d], src_stage._replica_ptr(src, d), b, min(c, n - b))
                for d, b, c in src_stage._slices(src) if b < n]
    if dst_stage is None:
        dsts = [(-1, dst.host_pointer())]
    else:
        dsts = [(dst_stage._ordinals[d], dst_stage._replica_ptr(dst, d)) for d in range(len(dst_stage._ordinals))]
    for dd, dp in dsts:
        for sd, sp, b, c in srcs:
            engine.copy(dp + b, dd, sp + b, sd, c)


class ClPipeline:
    """A built device-to-device pipeline (reference ``ClPipeline``)."""

    def __init__(self, stages: List[ClPipelineStage], debug: bool = False):
        self.stages = stages
        self.debug = debug
        self.counter = 0
        self._pool = ThreadPoolExecutor(max_workers=max(1, len(stages)))
        self.engine = cek.CopyEngine()

    def _forward(self, data, results) -> None:
        """Enqueue every transfer of this push (no host sync): host data into
        stage 0's spare inputs, each stage's previous outputs into the next
        stage's spare inputs, the last stage's previous outputs to the host."""
        e = self.engine
        last = len(self.stages) - 1
        if data is not None:
            st = self.stages[0]
            for dst, d in zip(st._in_dup, data):
                _transfer(e, st, dst, None, as_clarray(d))
        for k in range(last):
            st, nxt = self.stages[k], self.stages[k + 1]
            for dst, src in zip(nxt._in_dup, st._out_dup):
                _transfer(e, nxt, dst, st, src)
        self._wrapped = []
        if results is not None:
            st = self.stages[last]
            for r, src in zip(results, st._out_dup):
                w = as_clarray(r)
                _transfer(e, None, w, st, src)
                if not isinstance(r, ClArray):
                    self._wrapped.append((r, w))

    def transfer_stats(self) -> dict:
        """Bytes moved by the stage transitions so far, by path: ``p2p``
        (GPU↔GPU peer copies), ``h2d``/``d2h`` (PCIe, pipeline inputs and
        results only) and ``host`` (CPU-device memcpy)."""
        e = self.engine
        return {"p2p": e.p2p_bytes, "h2d": e.h2d_bytes, "d2h": e.d2h_bytes, "host": e.host_bytes,
                "copies": e.copies}

    def push_data(self, data: Optional[Sequence] = None, results: Optional[Sequence] = None) -> bool:
        """Advance the pipeline one step; returns True once results are
        flowing out (reference pushData, ClPipeline.cs:49-125).  Every stage
        computes on its current buffers (one host thread per stage) while
        the transfers of the previous step's buffers run on the copy
        engine's streams; one sync joins them."""
        S = len(self.stages)
        futs = [self._pool.submit(st.run) for st in self.stages]
        try:
            self._forward(data, results)
            self.engine.sync()
        finally:
            for f in futs:
                f.result()
        for r, w in self._wrapped:  # a non-contiguous result was wrapped through a copy
            view = np.asarray(r)
            if not np.shares_memory(view, w.array):
                np.copyto(view.reshape(-1), w.array[:view.size].reshape(-1))
        for i, st in enumerate(self.stages):
            st._snapshot_owner()
            if data is not None or i != 0:
                st.switch_input_buffers()
            if results is not None or i != S - 1:
                st.switch_output_buffers()
                st._owner = st._owner_next
        self.counter += 1
        if data is None and results is None:
            return self.counter > 2 * S - 2
        if data is not None and results is not None:
            return self.counter > 2 * S
        return self.counter > 2 * S - 1

    pushData = push_data

    def elapsed_times(self) -> List[float]:
        return [s.elapsed_time for s in self.stages]

    # ---- measured overlap (stage kernels vs stage-transition copies) ---------
    @property
    def record_timeline(self) -> bool:
        return bool(self.engine.record_timeline)

    @record_timeline.setter
    def record_timeline(self, on: bool) -> None:
        """Time every stage's kernels (hipEvents on each device) and every
        copy of the stage transitions (hipEvents on the copy streams), all
        on one host-anchored clock."""
        self.engine.record_timeline = bool(on)
        for st in self.stages:
            st.cruncher.record_timeline = bool(on)

    def timeline(self) -> dict:
        """``{"kernels": [(stage, device, begin, end)], "copies": [(kind,
        device, bytes, begin, end)], "t0": origin}`` in host-clock ms since
        the first recorded event (``t0`` on the runtime clock,
        ``cek.now_ms()``); waits for the recorded work and clears it."""
        ks = [(i, t["device"], t["abs_begin_ms"], t["abs_end_ms"])
              for i, st in enumerate(self.stages) for t in st.cruncher.timeline()]
        cs = [(c["kind"], c["device"], c["bytes"], c["abs_begin_ms"], c["abs_end_ms"]) for c in self.engine.timeline()]
        t0 = min([k[2] for k in ks] + [c[3] for c in cs], default=0.0)
        return {"kernels": [(i, d, b - t0, e - t0) for i, d, b, e in ks],
                "copies": [(k, d, n, b - t0, e - t0) for k, d, n, b, e in cs], "t0": t0}

    @staticmethod
    def copy_overlap(tl: dict, stage: Optional[int] = None) -> dict:
        """How much of the stage-transition copy time ran while kernels of
        ``stage`` (default: every stage) were executing: ``copy_ms`` (busy
        time of the copies, union), ``hidden_ms`` and ``fraction`` =
        hidden / copy (1.0: transfers fully overlapped with compute)."""
        ks = [(b, e) for i, _, b, e in tl["kernels"] if stage is None or i == stage]
        cs = [(b, e) for _, _, _, b, e in tl["copies"]]
        copy_ms = _coverage(cs)[0]
        # hidden = |union(copies) ∩ union(kernels)|
        union, cur = [], None
        for b, e in sorted(cs):
            if cur and b <= cur[1]:
                cur[1] = max(cur[1], e)
            else:
                if cur:
                    union.append(tuple(cur))
                cur = [b, e]
        if cur:
            union.append(tuple(cur))
        hidden = sum(_intersection(b, e, ks) for b, e in union)
        return {"copy_ms": copy_ms, "hidden_ms": hidden, "fraction": hidden / copy_ms if copy_ms > 0 else 1.0}

    def dispose(self) -> None:
        self._pool.shutdown(wait=True)
        for s in self.stages:
            if s.cruncher:
                s.cruncher.dispose()


# =========================================================================== single device


class DevicePipelineArrayType(enum.IntEnum):
    INPUT = 0
    OUTPUT = 1
    INTERNAL = 2
    TRANSITION = 3


class DevicePipelineArray:
    """An array bound to device-pipeline stages with a role."""

    def __init__(self, type_: DevicePipelineArrayType, array):
        self.type = DevicePipelineArrayType(type_)
        self.array = as_clarray(array)
        if self.type != DevicePipelineArrayType.INTERNAL:
            # Double buffers live in pinned memory: a copy from or to pageable
            # memory would block the host until the stream drains, and stage
            # k+1 could not be enqueued while stage k runs.
            self.array.fast_arr = True
        self.dup = _clone(self.array) if self.type != DevicePipelineArrayType.INTERNAL else None
        self.stages: List["DevicePipelineStage"] = []

    def buffers(self):
        return (self.array, self.dup)


class DevicePipelineStage:
    def __init__(self, kernel_names: str, global_range: int, local_range: int):
        self.kernel_names = kernel_names
        self.global_range = global_range
        self.local_range = local_range
        self.arrays: List[DevicePipelineArray] = []
        self.index = 0
        # skip this stage's host↔device copies of its INPUT / OUTPUT arrays
        # from now on (stopHostDeviceTransmission, ClPipeline.cs:2678): the
        # stage keeps computing on what its device buffers hold
        self.stop_host_device_transmission = False

    def bind_array(self, arr: DevicePipelineArray) -> None:
        self.arrays.append(arr)
        arr.stages.append(self)

    @property
    def has_input(self) -> bool:
        """True if any bound array is an INPUT (ClPipeline.cs:2812)."""
        return any(a.type == DevicePipelineArrayType.INPUT for a in self.arrays)

    @property
    def has_output(self) -> bool:
        """True if any bound array is an OUTPUT (ClPipeline.cs:2829)."""
        return any(a.type == DevicePipelineArrayType.OUTPUT for a in self.arrays)

    bindArray = bind_array
    hasInput, hasOutput = has_input, has_output
    stopHostDeviceTransmission = property(
        lambda self: self.stop_host_device_transmission,
        lambda self, v: setattr(self, "stop_host_device_transmission", bool(v)))


def _coverage(intervals):
    """(time covered by ≥1 interval, time covered by ≥2 intervals)."""
    ev = sorted([(b, 1) for b, _ in intervals] + [(e, -1) for _, e in intervals])
    busy = multi = 0.0
    depth, last = 0, None
    for t, d in ev:
        if last is not None:
            if depth >= 1:
                busy += t - last
            if depth >= 2:
                multi += t - last
        depth += d
        last = t
    return busy, multi


def _intersection(b, e, intervals) -> float:
    """Length of [b, e) covered by the union of ``intervals``."""
    cut = sorted((max(b, x), min(e, y)) for x, y in intervals if min(e, y) > max(b, x))
    total, end = 0.0, b
    for x, y in cut:
        x = max(x, end)
        if y > x:
            total += y - x
            end = y
    return total


class DevicePipeline:
    """N stages on one device, overlapped on separate HIP streams."""

    def __init__(self, device: ClDevices, kernel_source: str, queue_concurrency: Optional[int] = None):
        if len(device) != 1:
            raise ValueError("DevicePipeline runs on exactly one device")
        self.cruncher = ClNumberCruncher(device, kernel_source, queue_concurrency=queue_concurrency)
        if self.cruncher.error_code():
            raise RuntimeError(self.cruncher.error_message())
        self.stages: List[DevicePipelineStage] = []
        self.serial = False
        self._parity = 0
        self._async = None

    def add_stage(self, stage: DevicePipelineStage) -> None:
        stage.index = len(self.stages)
        self.stages.append(stage)

    addStage = add_stage

    def enable_serial_mode(self) -> None:
        self.serial = True

    def enable_parallel_mode(self) -> None:
        self.serial = False

    enableSerialMode = enable_serial_mode
    enableParallelMode = enable_parallel_mode

    # Timeline queries (declared but not implemented in the reference,
    # ClPipeline.cs:2391-2399): every feed with ``record_timeline`` on leaves
    # one hipEvent-timed kernel span per stage (compute id 100 + stage).
    @property
    def record_timeline(self) -> bool:
        return self.cruncher.record_timeline

    @record_timeline.setter
    def record_timeline(self, on: bool) -> None:
        self.cruncher.record_timeline = on
        self._spans = []

    def _collect(self) -> List[tuple]:
        spans = getattr(self, "_spans", [])
        spans += [(t["compute_id"] - 100, t["begin_ms"], t["end_ms"]) for t in self.cruncher.timeline()]
        self._spans = spans
        return spans

    def query_timeline_overlap_percentage(self) -> float:
        """Share (%) of the recorded busy time during which two or more stages
        ran at once (0 for a fully serial pipeline)."""
        spans = self._collect()
        busy, multi = _coverage([(b, e) for _, b, e in spans])
        return 100.0 * multi / busy if busy > 0 else 0.0

    def stages_overlapping_percentages(self) -> List[float]:
        """Per stage: share (%) of its own kernel time that overlapped any
        other stage's kernels."""
        spans = self._collect()
        out = []
        for i in range(len(self.stages)):
            mine = [(b, e) for st, b, e in spans if st == i]
            others = [(b, e) for st, b, e in spans if st != i]
            own = sum(e - b for b, e in mine)
            shared = sum(_intersection(b, e, others) for b, e in mine)
            out.append(100.0 * shared / own if own > 0 else 0.0)
        return out

    queryTimelineOverlapPercentage = query_timeline_overlap_percentage
    stagesOverlappingPercentages = stages_overlapping_percentages

    def _args(self, st: DevicePipelineStage) -> ClParameterGroup:
        p = self._parity
        out = []
        for a in st.arrays:
            if a.type == DevicePipelineArrayType.INTERNAL:
                buf = a.array
                buf.read = buf.write = buf.partial_read = False
            elif a.type == DevicePipelineArrayType.INPUT:
                buf = a.buffers()[p]          # host fills the other one meanwhile
                buf.read, buf.write, buf.partial_read = not st.stop_host_device_transmission, False, False
            elif a.type == DevicePipelineArrayType.OUTPUT:
                buf = a.buffers()[p]
                buf.read, buf.write, buf.partial_read = False, not st.stop_host_device_transmission, False
            else:  # TRANSITION: producer (first bound stage) writes p, consumer reads 1-p
                producer = a.stages[0] is st
                buf = a.buffers()[p if producer else 1 - p]
                buf.read = buf.write = buf.partial_read = False
            out.append(buf)
        return ClParameterGroup(out)

    def _enqueue(self) -> None:
        cr = self.cruncher
        if not self.serial:
            cr.enqueue_mode = True
            cr.enqueue_mode_async_enable = True
        for st in self.stages:
            self._args(st).compute(cr, 100 + st.index, st.kernel_names, st.global_range, st.local_range)

    def _finish(self) -> None:
        cr = self.cruncher
        if not self.serial:
            cr.enqueue_mode = False
            cr.enqueue_mode_async_enable = False
        self._parity ^= 1

    def feed(self) -> None:
        """One pipeline step: every stage runs once (concurrently)."""
        self._enqueue()
        self._finish()

    def feed_async_begin(self) -> None:
        self._enqueue()

    def feed_async_end(self) -> None:
        self._finish()

    def feed_async(self, callback: Callable[[], None]) -> None:
        """Enqueue a step, run ``callback`` (host work) while devices compute,
        then complete the step."""
        self._enqueue()
        try:
            callback()
        finally:
            self._finish()

    feedAsync = feed_async
    feedAsyncBegin = feed_async_begin
    feedAsyncEnd = feed_async_end

    def async_host_work(self) -> None:
        """Reference placeholder with an empty body (ClPipeline.cs:2663); host
        work beside a step is :meth:`feed_async`'s callback here."""

    asyncHostWork = async_host_work

    def input_buffer(self, arr: DevicePipelineArray) -> ClArray:
        """The host-side INPUT buffer the host may fill for the next feed."""
        return arr.buffers()[1 - self._parity]

    def output_buffer(self, arr: DevicePipelineArray) -> ClArray:
        """The OUTPUT buffer holding the last completed feed's results."""
        return arr.buffers()[1 - self._parity]

    def dispose(self) -> None:
        self.cruncher.dispose()
