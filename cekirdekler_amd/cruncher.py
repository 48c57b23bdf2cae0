"""``ClNumberCruncher`` — the entry API (reference ClNumberCruncher.cs:56-415)
and ``Cores`` usage-type-2 API (reference Cores.cs:37-1982).

A cruncher JIT-compiles one HIP C++ (or OpenCL-C dialect) kernel string for
every selected device (hiprtc → gfx950 code object per GPU, host compiler for
the CPU device), owns a native ``Cores`` scheduler, and executes
``ClArray``/``ClParameterGroup.compute(...)`` calls: the global range is split
across devices by the iterative load balancer per compute id.
"""
from __future__ import annotations

import enum
import json
import logging
import os
import re
import threading
import time
from typing import List, Optional, Sequence

import numpy as np

from ._native import cek, kernel_dir
from .arrays import ClArray, ClParameterGroup, _register_cores, as_clarray
from .hardware import ClDevices, ClPlatforms, async_queue_count, mixed_cpu_policy

PIPELINE_EVENT = True    # Cores.PIPELINE_EVENT (Cores.cs:416-423)
PIPELINE_DRIVER = False  # Cores.PIPELINE_DRIVER

_SPLIT = re.compile(r"[ ,;\-\n@]+")


class AcceleratorType(enum.IntFlag):
    """Device classes (reference ``AcceleratorType``, ClNumberCruncher.cs:32-49)."""
    CPU = 1
    GPU = 2
    ACC = 4


# Structured observability: with CEK_RECORD_LOG=<path> every
# compute() appends one JSON line {time, devices, compute_id, kernels, ranges,
# device_ms, bytes, pipelined, wall_ms}; the "cekirdekler_amd" logger gets the
# same record at DEBUG level.
_logger = logging.getLogger("cekirdekler_amd")
_RECORD_LOG = os.environ.get("CEK_RECORD_LOG") or None
_record_lock = threading.Lock()


def _log_record(cr, kernels) -> None:
    rec = cr.last_record()
    rec.update(time=time.time(), kernels=list(kernels), devices=cr.device_names())
    line = json.dumps(rec)
    _logger.debug(line)
    with _record_lock, open(_RECORD_LOG, "a") as f:
        f.write(line + "\n")


class ClUserEvent:
    """Host-triggered start gate for device streams (reference ClUserEvent,
    ClUserEvent.cs:28-117; "development cancelled" there, Worker.cs:487-560).

    ``add_cruncher(cr)`` makes every stream of the cruncher's devices wait
    (``hipStreamWaitValue32`` on a pinned host word) until :meth:`trigger`;
    work enqueued meanwhile — e.g. in enqueue mode — starts on all devices at
    once when triggered.  An armed event left untriggered is triggered when it
    is garbage collected, so no stream stays blocked."""

    def __init__(self):
        self._ev = cek.UserEvent()
        self._holds = 0
        self._lock = threading.Lock()

    def add_cruncher(self, cruncher: "ClNumberCruncher", device: int = -1) -> None:
        cruncher.cores.gate(self._ev, int(device))

    addCommandQueue = add_cruncher

    def trigger(self) -> None:
        self._ev.trigger()

    # Counter form (ClUserEvent.inc / dec, ClUserEvent.cs:66-84): every inc()
    # is a hold on the gated streams, every dec() releases one; the streams
    # start when the last hold is released.
    def inc(self) -> None:
        with self._lock:
            self._holds += 1

    def dec(self) -> None:
        with self._lock:
            if self._holds <= 0:
                raise RuntimeError("ClUserEvent.dec() without a matching inc()")
            self._holds -= 1
            release = self._holds == 0
        if release:
            self.trigger()

    @property
    def count(self) -> int:
        return self._holds

    def dispose(self) -> None:
        """Releases any stream still gated (never leaves a queue blocked)."""
        if self.armed:
            self.trigger()

    @property
    def armed(self) -> bool:
        return bool(self._ev.armed)


class ClComputeError(ValueError):
    """A compute() call was rejected by validation (work-size/array-size)."""


def split_kernel_names(kernels) -> List[str]:
    if isinstance(kernels, (list, tuple)):
        return [k for k in kernels if k]
    return [k for k in _SPLIT.split(kernels.strip()) if k]


def select_devices(types, num_gpus: int = -1, cpu_cores: int = -1, stream: bool = True) -> ClDevices:
    """Device discovery from an AcceleratorType (reference Cores ctor,
    Cores.cs:156-273: CPUs partitioned to N-1 cores, GPUs capped by
    numberOfGPUsToUse)."""
    if isinstance(types, str):
        t = 0
        low = types.lower()
        t |= AcceleratorType.CPU if "cpu" in low else 0
        t |= AcceleratorType.GPU if "gpu" in low else 0
        t |= AcceleratorType.ACC if "acc" in low else 0
        types = AcceleratorType(t)
    plats = ClPlatforms.all()
    devs = ClDevices([])
    if types & AcceleratorType.CPU:
        devs = devs + plats.cpus(True, stream, cpu_cores)
    if types & AcceleratorType.GPU:
        g = plats.gpus(False)
        if num_gpus is not None and num_gpus > 0:
            g = g[:num_gpus]
        devs = devs + g
    return devs


class ClNumberCruncher:
    """Compiles a kernel string for a device set and runs computes on it.

    ``ClNumberCruncher(AcceleratorType.GPU, src)`` or
    ``ClNumberCruncher(ClPlatforms.all().gpus(), src)``.  ``prebuilt`` adds
    AOT code objects (``[(path, [names])]``) — the library kernels of
    :mod:`cekirdekler_amd.ops` use this.
    """

    def __init__(self, devices, kernel_source: str = "", cpu_cores: int = -1, num_gpus: int = -1,
                 stream: bool = True, no_pipelining: bool = False, queue_concurrency: Optional[int] = None,
                 prebuilt: Optional[Sequence] = None, options: Optional[Sequence[str]] = None,
                 smooth: bool = True):
        if isinstance(devices, (AcceleratorType, int, str)):
            devices = select_devices(devices, num_gpus, cpu_cores, stream)
        if not isinstance(devices, ClDevices):
            devices = ClDevices(list(devices))
        self.devices = devices
        self.kernel_source = kernel_source or ""
        if "enqueue_kernel" in self.kernel_source:
            raise NotImplementedError(
                "OpenCL 2.0 enqueue_kernel (blocks) has no HIP equivalent; use cek_enqueue(child, n, param) "
                "with `__cek_child__ void child(long long id, long long param, <parent's params>)` "
                "(GPU-resident child levels, see ClNumberCruncher.device_enqueue_errors)")
        cfg = cek.CoresConfig()
        # async-enqueue / driver-pipeline streams per device: one per hardware
        # queue the main stream leaves free, unless asked (the reference's
        # fixed 16 aliases onto 4 queues; hardware.async_queue_count)
        if queue_concurrency is None:
            queue_concurrency = async_queue_count()
        cfg.queue_concurrency = int(queue_concurrency)
        self._queue_concurrency = max(1, min(16, int(queue_concurrency)))
        cfg.no_pipelining = bool(no_pipelining)
        cfg.smooth = bool(smooth)
        cfg.options = list(options or [])
        cfg.prebuilt = [p if isinstance(p, str) else f"{p[0]}|{','.join(p[1])}" for p in (prebuilt or [])]
        self.repeat_count = 1
        self.repeat_kernel_name = ""
        self.performance_feed = False
        self.number_of_errors_happened = 0
        self._call_cache = {}
        self._cores = None
        if len(devices) == 0:
            self._error_code, self._error_message = 1, "no device selected"
            return
        # A CPU device next to GPUs shares the host with the GPU workers'
        # threads: see mixed_cpu_policy
        n_gpu = sum(1 for d in devices if d.is_gpu)
        policy = mixed_cpu_policy() if (n_gpu and any(d.is_cpu for d in devices)) else "none"
        reserve = n_gpu if policy in ("reserve", "both") else 0
        self.mixed_cpu_policy = policy
        self._cores = cek.Cores([d.native_info(reserve_threads=reserve) for d in devices], self.kernel_source, cfg)
        if policy in ("sleep", "both"):
            self._cores.sleep_waits = True
        self._error_code = self._cores.error_code
        self._error_message = self._cores.error_message
        if self._error_code:
            self.number_of_errors_happened += 1
        elif os.environ.get("CEK_DEBUG", "") not in ("", "0"):
            self.debug_checks = True
        _register_cores(self)

    # ------------------------------------------------------------ status
    def error_code(self) -> int:
        return self._error_code

    def error_message(self) -> str:
        return self._error_message

    errorCode = error_code
    errorMessage = error_message

    @property
    def cores(self):
        if self._cores is None:
            raise RuntimeError("cruncher has no native core (disposed or failed)")
        return self._cores

    @property
    def kernel_names(self) -> List[str]:
        return [k.name for k in self._cores.kernels] if self._cores else []

    def device_names(self) -> List[str]:
        return [self._cores.device(i).name for i in range(self._cores.num_devices)]

    deviceNames = device_names

    @property
    def number_of_devices(self) -> int:
        return self._cores.num_global_devices if self._cores else 0

    @property
    def compute_queue_concurrency(self) -> int:
        """Streams per device that async enqueue rotates over
        (``computeQueueConcurrency``, ClNumberCruncher.cs:313, ≤ 16)."""
        return self._queue_concurrency

    @property
    def last_used_compute_id(self) -> int:
        """Compute id of the latest compute() (Cores.cs:961); -1 before any."""
        return int(self._cores.last_compute_id) if self._cores else -1

    computeQueueConcurrency = compute_queue_concurrency
    lastUsedComputeId = last_used_compute_id
    numberOfDevices = number_of_devices

    # ------------------------------------------------------------ modes
    def _prop(name):  # noqa: N805
        def get(self):
            return getattr(self._cores, name) if self._cores else False

        def set_(self, v):
            if self._cores:
                setattr(self._cores, name, bool(v))
        return property(get, set_)

    @property
    def repeat_graph_threshold(self) -> int:
        """Repeat loops with at least this many kernel launches per device are
        captured into a hipGraph and replayed (0 = never)."""
        return int(self._cores.graph_min_launches) if self._cores else 0

    @repeat_graph_threshold.setter
    def repeat_graph_threshold(self, n: int) -> None:
        if self._cores:
            self._cores.graph_min_launches = int(n)

    # ------------------------------------------------------------ failure handling
    def disable_device(self, device: int) -> None:
        """Drop a local device: later computes re-balance over the others
        (SURVEY §5.3 "drop device and re-balance")."""
        self._cores.set_device_enabled(int(device), False)

    def enable_device(self, device: int) -> None:
        self._cores.set_device_enabled(int(device), True)

    def device_enabled(self, device: int) -> bool:
        return bool(self._cores.device_enabled(int(device)))

    auto_failover = _prop("auto_failover")

    no_compute_mode = _prop("no_compute")
    fine_grained_queue_control = _prop("fine_grained")
    enqueue_mode_async_enable = _prop("async_enqueue")
    enqueue_mode = _prop("enqueue_mode")
    smooth_load_balancer = _prop("smooth")
    noComputeMode = no_compute_mode
    fineGrainedQueueControl = fine_grained_queue_control
    enqueueModeAsyncEnable = enqueue_mode_async_enable
    enqueueMode = enqueue_mode
    smoothLoadBalancer = smooth_load_balancer
    del _prop

    @property
    def repeatCount(self) -> int:  # noqa: N802
        return self.repeat_count

    @repeatCount.setter
    def repeatCount(self, v: int) -> None:  # noqa: N802
        self.repeat_count = int(v)

    @property
    def repeatKernelName(self) -> str:  # noqa: N802
        return self.repeat_kernel_name

    @repeatKernelName.setter
    def repeatKernelName(self, v: str) -> None:  # noqa: N802
        self.repeat_kernel_name = v or ""

    @property
    def performanceFeed(self) -> bool:  # noqa: N802
        return self.performance_feed

    @performanceFeed.setter
    def performanceFeed(self, v: bool) -> None:  # noqa: N802
        self.performance_feed = bool(v)

    def flush_last_used_command_queue(self) -> None:
        """HIP submits at enqueue time; kept for API parity (clFlush)."""

    flushLastUsedCommandQueue = flush_last_used_command_queue

    def sync(self) -> None:
        """Wait for every queued operation on every device."""
        if self._cores:
            self._cores.finish()

    def count_markers_reached(self) -> int:
        return int(self._cores.markers_reached()) if self._cores else 0

    def count_markers_remaining(self) -> int:
        return int(self._cores.markers_issued() - self._cores.markers_reached()) if self._cores else 0

    countMarkersReached = count_markers_reached
    countMarkersRemaining = count_markers_remaining

    # ------------------------------------------------------------ balancer state
    def ranges(self, compute_id: int) -> List[int]:
        return list(self._cores.ranges(compute_id))

    def references(self, compute_id: int) -> List[int]:
        return list(self._cores.references(compute_id))

    def benchmarks(self, compute_id: int) -> List[float]:
        return list(self._cores.benchmarks(compute_id))

    def performance_history(self, compute_id: int) -> List[List[float]]:
        """The balancer's moving-average window for ``compute_id``: 10 rows
        (oldest first) of normalized per-device throughputs (≙
        ``Cores.performanceHistory``, reference src/Cores.cs:1075)."""
        return [list(h) for h in self._cores.history(compute_id)]

    performanceHistory = performance_history

    def normalized_compute_powers_of_devices(self, compute_id: Optional[int] = None):
        c = self._cores
        cid = c.last_compute_id if compute_id is None else compute_id
        if not c or not c.has_state(cid):
            return None
        b, r = c.benchmarks(cid), c.ranges(cid)
        tot = sum(b) + 0.01 * len(b)
        thr = [(tot / (bi + 0.01)) * (ri + 1) for bi, ri in zip(b, r)]
        s = sum(thr) or 1.0
        return [x / s for x in thr]

    def normalized_global_ranges_of_devices(self, compute_id: int):
        c = self._cores
        if not c or not c.has_state(compute_id):
            return None
        r = c.ranges(compute_id)
        s = float(sum(r)) or 1.0
        return [x / s for x in r]

    normalizedComputePowersOfDevices = normalized_compute_powers_of_devices
    normalizedGlobalRangesOfDevices = normalized_global_ranges_of_devices

    def performance_report(self, compute_id: int = 0) -> str:
        """Console table of load distribution and per-device times
        (reference Cores.performanceReport, Cores.cs:994-1063)."""
        c = self._cores
        if compute_id == 0:
            ids = c.compute_ids()
            if not ids:
                s = "Needs one more compute to profile. Load balancer needs multiple iterations to be useful."
                print(s)
                return s
            compute_id = ids[0]
        if not c.has_state(compute_id):
            s = "Error: Global range array is not ready."
            print(s)
            return s
        r = c.ranges(compute_id)
        b = c.benchmarks(compute_id)
        tot = float(sum(r)) or 1.0
        pct = "----- Load Distributions: " + "".join(f" [{100.0 * x / tot:.1f}%] -" for x in r)
        pct += "-" * max(0, 50 - len(pct))
        lines = ["", "", f"Compute-ID: {compute_id}  {pct}" + "-" * 48]
        base = c.global_base
        for i in range(len(r)):
            if 0 <= i - base < c.num_devices:
                d = c.device(i - base)
                kind = "gddr" if (d.dedicated_memory and not d.streaming) else "stream"
                name = d.name.strip()
            else:
                kind, name = "remote", f"rank-device {i}"
            head = f"Device {i}({kind}): {name}"
            head = head[:50].ljust(50)
            lines.append(f"{head} ||| time: {b[i]:,.2f}ms, workitems: {r[i]:,}")
        lines.append("-" * 113)
        s = "\n".join(lines) + "\n"
        print(s)
        return s

    performanceReport = performance_report

    def last_compute_performance_report(self) -> str:
        return self.performance_report(self._cores.last_compute_id)

    lastComputePerformanceReport = last_compute_performance_report

    # ------------------------------------------------------------ device-side enqueue
    def device_enqueue_errors(self) -> int:
        """Child launches dropped so far by ``cek_enqueue`` (a queue level
        full, or an enqueue deeper than the supported levels), summed over
        devices.  Waits for the devices.  Device-side enqueue replaces the
        reference's OpenCL 2.0 default-queue ``enqueue_kernel``
        (ClNumberCruncher.cs:203-205, Worker.cs:224-227): a kernel appends
        ``{child, n, param}`` records to its device's queue, and generated
        dispatcher launches run each child level right after the parent on
        the same stream, with no host round trip."""
        return int(self._cores.device_enqueue_errors()) if self._cores else 0

    def set_device_enqueue_levels(self, levels: int) -> None:
        """Child levels run after each parent launch (0..3, default 3)."""
        self._cores.set_device_enqueue_levels(int(levels))

    # ------------------------------------------------------------ debug checks
    @property
    def debug_checks(self) -> bool:
        """Debug mode (the reference has none and lists
        out-of-bounds native access as a known issue, README.md:40-45).
        While on, GPU buffers allocated from then on get a 4 KiB guard tail,
        every kernel launch is synchronised so a fault names its kernel, and
        a kernel that wrote past the end of one of its arrays fails the
        compute with the array index and the first corrupted byte.  Costs a
        sync and a 4 KiB read-back per array per launch.  ``CEK_DEBUG=1``
        turns it on for every cruncher.  Graph-replayed repeat loops are not
        checked."""
        return bool(self._cores.debug_checks) if self._cores else False

    @debug_checks.setter
    def debug_checks(self, on: bool) -> None:
        self._cores.debug_checks = bool(on)

    # ------------------------------------------------------------ device timeline
    @property
    def record_timeline(self) -> bool:
        return bool(self._cores.record_timeline) if self._cores else False

    @record_timeline.setter
    def record_timeline(self, on: bool) -> None:
        self._cores.record_timeline = bool(on)

    def timeline(self) -> List[dict]:
        """Kernel spans recorded while ``record_timeline`` was on: one dict per
        compute per device (``device``, ``compute_id``, ``begin_ms``,
        ``end_ms``), timed by hipEvents on the stream the kernels ran on and
        relative to that device's first span; ``abs_begin_ms``/``abs_end_ms``
        put every device on the host clock (each GPU's event clock anchored
        once), so spans of different GPUs can be compared.  Waits for the
        recorded work and clears the list."""
        return [{"device": d, "compute_id": cid, "begin_ms": b, "end_ms": e, "abs_begin_ms": ab, "abs_end_ms": ae}
                for d, cid, b, e, ab, ae in self._cores.timeline()]

    @property
    def record_kernel_times(self) -> bool:
        """Kernel profiling timestamps (OpenCL's CL_PROFILING_COMMAND_START /
        END): while on, every kernel launch carries a start and a stop event
        stamped by the dispatch itself (``hipExtModuleLaunchKernel``), so
        :meth:`kernel_times` gives each kernel's own execution time — without
        the gap between back-to-back launches that stream events and host
        clocks include."""
        return bool(self._cores.kernel_times_on) if self._cores else False

    @record_kernel_times.setter
    def record_kernel_times(self, on: bool) -> None:
        self._cores.kernel_times_on = bool(on)

    def kernel_times(self, device: int = 0) -> List[tuple]:
        """(kernel name, ms) of every launch on local ``device`` recorded
        while :attr:`record_kernel_times` was on, in launch order; waits for
        them and clears the list."""
        return [(k, float(ms)) for k, ms in self._cores.kernel_times(device)]

    recordKernelTimes = record_kernel_times
    kernelTimes = kernel_times

    def last_record(self) -> dict:
        """Structured record of the last compute (observability)."""
        r = self._cores.last_record()
        return {"compute_id": r.compute_id, "wall_ms": r.wall_ms, "ranges": list(r.ranges),
                "references": list(r.references), "device_ms": list(r.device_ms),
                "h2d_bytes": r.h2d_bytes, "d2h_bytes": r.d2h_bytes, "p2p_bytes": r.p2p_bytes,
                "gather_bytes": r.gather_bytes, "staged_bytes": r.staged_bytes, "p2p_path": r.p2p_path,
                "pipelined": r.pipelined}

    # ------------------------------------------------------------ peer topology
    def peer_topology(self) -> dict:
        """The device set's GPU-to-GPU links: the
        distinct GPU ordinals, ``hipDeviceCanAccessPeer`` among them (peer
        access is enabled at construction when they span two or more GPUs)
        and the resulting path — ``none`` (one GPU), ``xgmi`` (every pair
        peers) or ``staged`` (some pair cannot; the read fan-out then uploads
        over PCIe per device)."""
        if self._cores is None:
            return {"ordinals": [], "matrix": [], "path": "none"}
        return {"ordinals": list(self._cores.peer_ordinals),
                "matrix": [list(r) for r in self._cores.peer_matrix],
                "path": self._cores.p2p_path}

    # ------------------------------------------------------------ compute graphs
    def capture(self) -> "ComputeGraph":
        """Record the computes issued inside ``with cr.capture() as g:`` into
        one hipGraph per GPU instead of running them; ``g.replay(n)``
        launches the whole sequence n times back to back (one
        ``hipGraphLaunch`` per GPU per replay).  The split of every compute
        id is frozen at its current value, host transfers happen at replay
        time (pinned / registered host arrays), and the computes must have
        run once before (buffers exist).  GPU devices only."""
        return ComputeGraph(self)

    # ------------------------------------------------------------ kernel downloads
    @property
    def kernel_d2h(self) -> bool:
        """Download slices of pinned / registered host arrays (≥ 1 MiB,
        16-byte aligned) with a copy kernel that writes straight into the host
        pages, instead of ``hipMemcpyAsync``.  Keeps downloads off the SDMA
        engines the uploads use, so a download waiting for its kernel never
        holds up an upload queued behind it (streamed host-resident calls;
        ``profiles/hostres_streaming.md``).  Env ``CEK_KERNEL_D2H=1``."""
        return bool(self._cores.kernel_d2h) if self._cores else False

    @kernel_d2h.setter
    def kernel_d2h(self, on: bool) -> None:
        self._cores.kernel_d2h = bool(on)

    @property
    def copy_cus(self) -> int:
        """CUs per GPU reserved for copy kernels (0: none): the pipeline's
        write streams run on those CUs only (CU-masked HIP streams) and
        every other stream on the rest, so downloads by copy kernel
        (``kernel_d2h``) never wait for a compute work-group to leave a CU
        and overlap the SDMA uploads.  Setting it drains and re-creates the
        streams."""
        return int(self._cores.copy_cus) if self._cores else 0

    @copy_cus.setter
    def copy_cus(self, n: int) -> None:
        self._cores.copy_cus = int(n)

    # ------------------------------------------------------------ xGMI read fan-out
    @property
    def peer_reads(self) -> bool:
        """Full ``read`` arrays (≥ ``peer_read_min_bytes``, not written by the
        kernels) are uploaded 1/D per local GPU and all-gathered GPU↔GPU
        with peer copies over xGMI instead of D whole PCIe uploads (default
        on; reference behaviour — one upload per device — when off)."""
        return bool(self._cores.peer_reads) if self._cores else False

    @peer_reads.setter
    def peer_reads(self, on: bool) -> None:
        self._cores.peer_reads = bool(on)

    @property
    def peer_read_min_bytes(self) -> int:
        return int(self._cores.peer_read_min_bytes) if self._cores else 0

    @peer_read_min_bytes.setter
    def peer_read_min_bytes(self, n: int) -> None:
        self._cores.peer_read_min_bytes = int(n)

    def calibrate_peer_reads(self, sizes=None, calls: int = 5, cached: bool = True) -> dict:
        """Measure where the xGMI read fan-out starts to beat per-GPU uploads
        on this cruncher's GPUs and set :attr:`peer_read_min_bytes` to it
        (the broadcast / per-GPU upload choice by a
        measured size threshold; the built-in 1 MiB is only the default).
        The measurement runs on a temporary cruncher over the same devices
        (``utils.multigpu.measure_peer_read_threshold``); the result is kept
        per device set for the process (``cached``).  Fewer than two GPUs:
        nothing to choose, the threshold is left as it is.  A fan-out that
        never wins sets the threshold past every measured size."""
        from .utils import multigpu

        gpus = [d for d in self.devices if d.is_gpu]
        if len(gpus) < 2:
            return {"skipped": "fewer than two GPU devices", "peer_read_min_bytes": self.peer_read_min_bytes}
        key = multigpu.device_set_key(gpus)
        res = multigpu._PEER_READ_CACHE.get(key) if cached else None
        if res is None:
            res = multigpu.measure_peer_read_threshold(ClDevices(gpus), sizes or multigpu.PEER_READ_SIZES, calls)
            if not res["exact"]:
                raise RuntimeError("calibrate_peer_reads: a measured call produced a wrong output")
            multigpu._PEER_READ_CACHE[key] = res
        cross = res["crossover_bytes"]
        self.peer_read_min_bytes = int(cross) if cross is not None else 2 * max(res["sizes"])
        return {**res, "peer_read_min_bytes": self.peer_read_min_bytes}

    calibratePeerReads = calibrate_peer_reads

    # ------------------------------------------------------------ compute
    def _validate(self, group: ClParameterGroup, names, G, L, pipeline, blobs) -> None:
        D = self.number_of_devices
        if self._error_code:
            raise ClComputeError("Number-cruncher device compile error:\n" + self._error_message)
        if G % L != 0:
            raise ClComputeError(
                f"Work-size error: global range({G}) is not an integer multiple of local range({L}).")
        if pipeline and G % (L * blobs) != 0:
            raise ClComputeError(
                f"Work-size error: global range({G}) is not an integer multiple of "
                f"(local range)*(number of pipeline blobs)=({L * blobs}).")
        need = L * D * (blobs if pipeline else 1)
        if G < need:
            raise ClComputeError(
                f"Work-size error: global work size({G}) must be equal to or greater than "
                f"(number of selected devices)*(local worksize){'*(blobs)' if pipeline else ''}=({need})")
        if not names:
            raise ClComputeError("no kernel name given")
        for a in group.arrays:
            if a.blob_slices is not None:  # explicit per-blob slices: checked natively
                if any(b < 0 or n < 0 or b + n > a.N for b, n in a.blob_slices):
                    raise ClComputeError(f"Array-size error: a blob slice exceeds the array length ({a.N}).")
                continue
            if a._partial or (a._write and not a._write_all):
                if a.elements_per_group > 0:
                    if a.N < (G // L) * a.elements_per_group:
                        raise ClComputeError(
                            f"Array-size error: (number of groups)*(elements per group)="
                            f"({(G // L) * a.elements_per_group}) must be <= array length ({a.N}).")
                elif a.N < G * a.elements_per_work_item:
                    raise ClComputeError(
                        f"Array-size error: (global range)*(number of array elements per work item)="
                        f"({G * a.elements_per_work_item}) must be equal to or less than array length ({a.N}).")

    def _compute_group(self, group: ClParameterGroup, compute_id: int, kernels, global_range: int,
                       local_range: int = 256, global_offset: int = 0, pipeline: bool = False,
                       pipeline_type: bool = PIPELINE_EVENT, pipeline_blobs: int = 4, specs=None,
                       granularity: int = 0) -> None:
        call = self._build_call(group, compute_id, kernels, global_range, local_range, global_offset,
                                pipeline, pipeline_type, pipeline_blobs, specs, granularity)
        self._cores.compute(call)
        if specs is None:
            me = id(self)
            for a in group.arrays:
                if not a._ro:
                    a._split_log[me] = (int(compute_id), int(a.elements_per_work_item), int(a.elements_per_group),
                                        int(local_range))
        if self.performance_feed:
            self.performance_report(compute_id)
        if _RECORD_LOG is not None:
            _log_record(self, kernels=list(call.kernels))

    def _build_call(self, group: ClParameterGroup, compute_id: int, kernels, global_range: int,
                    local_range: int = 256, global_offset: int = 0, pipeline: bool = False,
                    pipeline_type: bool = PIPELINE_EVENT, pipeline_blobs: int = 4, specs=None,
                    granularity: int = 0):
        """Validate a compute and freeze it into a native ComputeCall.

        A repeated compute (same id, kernels, ranges, pipeline settings,
        repeat settings and the same native array specs — a spec changes with
        any flag or storage change) reuses the call built the first time:
        validation and the native struct's construction are ~5-8 µs of the
        host's per-compute cost, which is most of a small kernel's."""
        cache_key = None
        if specs is None and isinstance(pipeline_blobs, (int, np.integer)):
            pin = bool(self._cores is not None and self._cores.capturing)
            arr_specs = [a._spec(pin=pin) for a in group.arrays]
            cache_key = (int(compute_id), kernels if isinstance(kernels, str) else tuple(kernels),
                         int(global_range), int(local_range), int(global_offset), bool(pipeline),
                         bool(pipeline_type), int(pipeline_blobs), int(granularity), int(self.repeat_count),
                         self.repeat_kernel_name, pin, tuple(map(id, arr_specs)))
            hit = self._call_cache.get(cache_key)
            if hit is not None:
                return hit[0]
        names = split_kernel_names(kernels)
        G, L = int(global_range), int(local_range)
        # pipeline_blobs: a count (equal blobs), or explicit work-item bounds
        # [0, b1, ..., G] of uneven blobs (one device; ClArray.blob_slices)
        bounds = None
        if not isinstance(pipeline_blobs, (int, np.integer)):
            bounds = [int(x) for x in pipeline_blobs]
            pipeline_blobs = max(1, len(bounds) - 1)
        try:
            self._validate(group if specs is None else ClParameterGroup(), names, G, L,
                           pipeline and bounds is None, int(pipeline_blobs))
        except ClComputeError:
            self.number_of_errors_happened += 1
            raise
        call = cek.ComputeCall()
        call.kernels = names
        call.repeats = max(1, int(self.repeat_count))
        call.repeat_kernel = self.repeat_kernel_name if self.repeat_count > 1 else ""
        if specs is not None:
            call.arrays = specs
        else:
            pin = bool(self._cores is not None and self._cores.capturing)
            arr_specs = [a._spec(pin=pin) for a in group.arrays]
            call.arrays = arr_specs
        call.global_range = G
        call.local_range = L
        call.global_offset = int(global_offset)
        call.compute_id = int(compute_id)
        call.pipeline = bool(pipeline)
        call.pipeline_event = bool(pipeline_type)
        call.blobs = int(pipeline_blobs)
        if bounds is not None:
            call.blob_bounds = bounds
        if granularity:
            if granularity % L or G % granularity:
                self.number_of_errors_happened += 1
                raise ClComputeError(f"granularity({granularity}) must be a multiple of the local range({L}) "
                                     f"and divide the global range({G})")
            call.granularity = int(granularity)
        if cache_key is not None:
            if len(self._call_cache) >= 64:
                self._call_cache.clear()
            # the entry holds the spec objects its key names by id(), so no
            # id is reused while the entry lives
            self._call_cache[cache_key] = (call, arr_specs)
        return call

    def compute(self, arrays, compute_id: int, kernels, global_range: int, local_range: int = 256,
                global_offset: int = 0, pipeline: bool = False, pipeline_type: bool = PIPELINE_EVENT,
                pipeline_blobs: int = 4, granularity: int = 0) -> None:
        """Functional form: ``cr.compute([a, b, c], 1, "k", G, L)``."""
        group = arrays if isinstance(arrays, ClParameterGroup) else ClParameterGroup(arrays)
        self._compute_group(group, compute_id, kernels, global_range, local_range, global_offset,
                            pipeline, pipeline_type, pipeline_blobs, granularity=granularity)

    # ------------------------------------------------------------ device data access
    def upload(self, array: ClArray, device: int = 0) -> None:
        self._cores.upload(device, as_clarray(array)._spec())

    def download(self, array: ClArray, device: int = 0) -> None:
        self._cores.download(device, as_clarray(array)._spec())

    def device_pointer(self, array: ClArray, device: int = 0) -> int:
        return int(self._cores.device_pointer(device, as_clarray(array)._spec()))

    def _release_array(self, uid: int) -> None:
        if self._cores is not None:
            self._cores.release_array(uid)

    def set_time_scale(self, device: int, scale: float) -> None:
        """Test/bench hook: multiply a device's measured time (injected
        heterogeneity for load-balancer convergence measurements)."""
        self._cores.set_time_scale(device, float(scale))

    def set_time_offset(self, device: int, ms: float) -> None:
        """Test/bench hook: a fixed cost of ``ms`` host milliseconds per
        compute on a device (spent before its work, counted in its time)."""
        self._cores.set_time_offset(device, float(ms))

    @property
    def overhead_aware_balancer(self) -> bool:
        """Opt-in balancing that models each device's time as fixed cost +
        per-item cost (t = a + b·range, fitted from this compute id's
        history) instead of the reference's proportional law, and leaves a
        device out when its share would not pay for its fixed cost — so
        adding a device never makes a compute slower (the predictor slot
        the reference stubs out, HelperFunctions.cs:163-178).  The exact law
        stays the default; single-process crunchers only."""
        return bool(self._cores.balancer_predictor) if self._cores else False

    @overhead_aware_balancer.setter
    def overhead_aware_balancer(self, on: bool) -> None:
        self._cores.balancer_predictor = bool(on)

    def balancer_predictor_info(self, compute_id: int) -> dict:
        """The predictor's last decision for a compute id (``law`` while it
        gathers samples, ``multi``, ``single`` or ``probe``), its fits and
        the measured multi-/single-device overheads."""
        return dict(self._cores.predictor_info(int(compute_id)))

    # ------------------------------------------------------------ lifecycle
    def dispose(self) -> None:
        if self._cores is not None:
            try:
                self._cores.finish()
            except Exception:
                pass
            self._cores = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.dispose()

    def __repr__(self) -> str:
        return f"<ClNumberCruncher devices={self.device_names() if self._cores else []} kernels={self.kernel_names}>"


class Cores:
    """Reference "usage type 2" API: ``Cores(types, src, names, ...)`` then
    ``compute(names, repeats, syncKernel, arrays, readWrite, epw, G, id, ...)``
    with the readWrite token strings ``partial read write all ro wo zc``
    (plus the extension token ``gather``: keep-resident all-gather)
    (ClArray.cs:611-629, Cores.cs:471)."""

    PIPELINE_EVENT = PIPELINE_EVENT    # Cores.cs:416-423
    PIPELINE_DRIVER = PIPELINE_DRIVER

    def __init__(self, device_types, kernel_source: str, kernel_names=None, default_queue: bool = False,
                 local_range: int = 256, num_gpus: int = -1, stream: bool = True, max_cpu: int = -1,
                 no_pipelining: bool = False, devices: Optional[ClDevices] = None):
        devs = devices if devices is not None else select_devices(device_types, num_gpus, max_cpu, stream)
        self.local_range = local_range
        self.cruncher = ClNumberCruncher(devs, kernel_source, no_pipelining=no_pipelining)
        self.kernel_names = kernel_names or self.cruncher.kernel_names

    @property
    def number_of_devices(self) -> int:
        return self.cruncher.number_of_devices

    numberOfDevices = number_of_devices

    def compute(self, kernel_names, repeats: int, repeat_kernel: str, arrays, read_writes: Sequence[str],
                elements_per_item: Sequence[int], global_range: int, compute_id: int,
                global_offset: int = 0, pipeline: bool = False, blobs: int = 4,
                pipeline_type: bool = PIPELINE_EVENT, local_range: Optional[int] = None) -> None:
        group = ClParameterGroup()
        for arr, rw, e in zip(arrays, read_writes, elements_per_item):
            a = as_clarray(arr)
            toks = set(rw.split())
            a._partial = "partial" in toks
            a._read = "read" in toks
            a._write = "write" in toks
            a._write_all = "all" in toks
            a.gather_resident = "gather" in toks
            a._ro = "ro" in toks
            a._wo = "wo" in toks
            a.zero_copy = "zc" in toks
            a.elements_per_work_item = int(e)
            group.arrays.append(a)
        self.cruncher.repeat_count = repeats
        self.cruncher.repeat_kernel_name = repeat_kernel or ""
        self.cruncher._compute_group(group, compute_id, kernel_names, global_range,
                                     local_range or self.local_range, global_offset, pipeline,
                                     pipeline_type, blobs)

    def performance_report(self, compute_id: int = 0) -> str:
        return self.cruncher.performance_report(compute_id)

    performanceReport = performance_report

    def benchmarks(self, compute_id: int):
        return self.cruncher.benchmarks(compute_id)

    def performance_history(self, compute_id: int):
        return self.cruncher.performance_history(compute_id)

    performanceHistory = performance_history

    def global_ranges(self, compute_id: int):
        return self.cruncher.ranges(compute_id)

    def global_references(self, compute_id: int):
        return self.cruncher.references(compute_id)

    def device_names(self):
        return self.cruncher.device_names()

    deviceNames = device_names

    # The reference Cores' mode switches and error state (Cores.cs:80-140),
    # forwarded to the cruncher that runs this Cores.
    def _fwd(name):  # noqa: N805
        return property(lambda self: getattr(self.cruncher, name),
                        lambda self, v: setattr(self.cruncher, name, v))

    enqueue_mode = _fwd("enqueue_mode")
    enqueue_mode_async_enable = _fwd("enqueue_mode_async_enable")
    fine_grained_queue_control = _fwd("fine_grained_queue_control")
    no_compute_mode = _fwd("no_compute_mode")
    smooth_load_balancer = _fwd("smooth_load_balancer")
    del _fwd
    enqueueMode, enqueueModeAsyncEnable = enqueue_mode, enqueue_mode_async_enable
    fineGrainedQueueControl, noComputeMode, smoothLoadBalancer = (
        fine_grained_queue_control, no_compute_mode, smooth_load_balancer)

    def error_code(self) -> int:
        return self.cruncher.error_code()

    def error_message(self) -> str:
        return self.cruncher.error_message()

    errorCode, errorMessage = error_code, error_message

    @property
    def all_errors_string(self) -> str:
        """Every initialisation / build error so far (Cores.allErrorsString)."""
        return self.cruncher.error_message()

    allErrorsString = all_errors_string

    def dispose(self) -> None:
        self.cruncher.dispose()


class ComputeGraph:
    """A captured sequence of computes (see :meth:`ClNumberCruncher.capture`)."""

    def __init__(self, cruncher: "ClNumberCruncher"):
        self.cruncher = cruncher
        self.id: Optional[int] = None

    def __enter__(self) -> "ComputeGraph":
        self.cruncher.cores.capture_begin()
        return self

    def __exit__(self, exc_type, exc, tb) -> None:
        if exc_type is not None:
            # the body failed: end the capture, but never let a capture error
            # replace the user's exception
            try:
                self.cruncher.cores.graph_destroy(self.cruncher.cores.capture_end())
            except Exception:
                pass
            return
        self.id = self.cruncher.cores.capture_end()

    def replay(self, times: int = 1, sync: bool = True) -> None:
        if self.id is None:
            raise RuntimeError("graph was not captured")
        self.cruncher.cores.graph_launch(self.id, int(times), bool(sync))

    def destroy(self) -> None:
        if self.id is not None:
            self.cruncher.cores.graph_destroy(self.id)
            self.id = None
