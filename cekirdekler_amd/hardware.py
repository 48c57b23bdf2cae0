"""Device query and selection (reference ``ClPlatforms`` / ``ClDevices``,
ClObjectApi.cs:158-1272).

Platforms on an MI355X node: one "AMD ROCm HIP" platform holding every
visible GPU, and one "Host CPU" platform holding the CPU device (a native
thread pool; "partition" keeps one core free like the reference's N-1 core
fission, ClDevice.cs:85-95).  ``ClDevices`` lists may contain the same
physical device several times (logical devices), which the reference allows
(ClPipeline.cs:1728, :4337; ``operator +`` ClObjectApi.cs:813).
"""
from __future__ import annotations

import os
from typing import Iterable, List, Optional

from ._native import cek

GPU_PLATFORM = "AMD ROCm HIP"
CPU_PLATFORM = "Host CPU"


def usable_cpus() -> int:
    """CPUs this process may actually use: the smallest of its affinity
    mask, the cgroup CPU quota (v2 ``cpu.max``, v1 ``cfs_quota_us``) and
    ``OMP_NUM_THREADS`` when set.  ``os.cpu_count()`` reports the whole
    machine, and a pool sized to it on a container with a CPU share
    oversubscribes the share many times over."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0 and per > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota:
        n = min(n, max(1, int(quota + 0.999)))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def hw_queue_count() -> int:
    """Hardware queues HIP gives this process per GPU: ``GPU_MAX_HW_QUEUES``
    (HIP's default, and the MI355X box's setting, is 4), clamped to 1..16.

    Streams beyond this count alias onto shared hardware queues and pick up
    false dependencies (one stream's copy waits behind another stream's
    kernel): on one box 4 async GEMM queues gave 1399 TF/s against 1329 with
    16 (profiles/round4_session4.md).  So the default async-enqueue and
    driver-pipeline queue count is this, not the reference's 16
    (Worker.cs:435-458, Cores.cs:1383-1855)."""
    v = os.environ.get("GPU_MAX_HW_QUEUES", "").strip()
    n = int(v) if v.isdigit() and int(v) > 0 else 4
    return max(1, min(16, n))


def async_queue_count() -> int:
    """Default async-enqueue / driver-pipeline compute streams per device:
    one per hardware queue the device's main stream leaves free,
    ``hw_queue_count() - 1`` (at least 1).

    HIP binds each new stream to a hardware queue: a new queue while the
    pool has fewer than GPU_MAX_HW_QUEUES, afterwards an existing one.  The
    main stream takes one, so with 4 queues a fourth compute stream lands on
    the queue of a busy compute stream and the computes on those two run one
    after the other — measured on MI355X (``tools/queue_map_probe.py``,
    ``profiles/r5/README.md``): with 4 compute streams the computes on
    streams 2 and 3 serialise, with 3 every consecutive pair runs side by
    side, and a two-stage DevicePipeline overlaps its stages in every
    window instead of in none."""
    return max(1, hw_queue_count() - 1)


def mixed_cpu_policy() -> str:
    """How a device set that mixes a CPU device with GPUs shares the host
    (``CEK_MIXED_CPU``): the reference sizes its CPU device to every core but
    one, the caller's (ClDevice.cs:85-95); here each GPU worker is a host
    thread too, waiting on its streams.

    * ``reserve`` — the CPU pool gives up one thread per GPU worker
      (``usable_cpus() - 1 - #GPUs`` with the partition flag);
    * ``sleep`` — GPU workers sleep on blocking events instead of spinning;
    * ``both`` / ``none``.
    """
    v = os.environ.get("CEK_MIXED_CPU", "").strip().lower()
    return v if v in ("reserve", "sleep", "both", "none") else MIXED_CPU_DEFAULT


MIXED_CPU_DEFAULT = "reserve"


class ClDevice:
    """One selectable device plus its selection flags."""

    def __init__(self, info, partition: bool = False, streaming: bool = False, max_cpu_cores: int = -1,
                 cu_partition: Optional[tuple] = None):
        self.info = info
        self.partition = bool(partition)
        self.streaming = bool(streaming)
        self.max_cpu_cores = int(max_cpu_cores)
        # (p, k): this logical GPU device runs on CU partition p of k
        # (ClDevices.cu_partitions); None = every CU of the GPU
        self.cu_partition = tuple(cu_partition) if cu_partition else None

    @property
    def is_gpu(self) -> bool:
        return self.info.type == cek.DevType.GPU.value

    @property
    def is_cpu(self) -> bool:
        return self.info.type == cek.DevType.CPU.value

    @property
    def name(self) -> str:
        return self.info.name

    @property
    def vendor(self) -> str:
        return self.info.vendor

    @property
    def compute_units(self) -> int:
        if self.cu_partition:
            return self.info.compute_units // self.cu_partition[1]
        return self.info.compute_units

    numberOfComputeUnits = compute_units

    @property
    def memory_bytes(self) -> int:
        return self.info.mem_bytes

    def is_gddr(self) -> bool:
        """Dedicated device memory; the "stream" flag turns it off
        (reference ClDevice.isGddr, ClDevice.cs:161)."""
        return bool(self.info.dedicated_memory) and not self.streaming

    isGddr = is_gddr

    def native_info(self, reserve_threads: int = 0):
        """DeviceInfo handed to the native runtime (CPU pool sized here).
        ``reserve_threads``: host threads the device set's GPU workers keep
        busy, taken off the CPU pool (``mixed_cpu_policy``) unless the core
        count was given explicitly (``max_cpu_cores``, ``CEK_CPU_THREADS``)."""
        if not self.is_cpu:
            if not self.cu_partition:
                return self.info
            info = cek.gpu_info(self.info.ordinal)
            info.cu_part, info.cu_parts = self.cu_partition
            return info
        hw = usable_cpus()
        threads = hw - 1 if (self.partition and hw > 1) else hw
        if self.max_cpu_cores > 0:
            threads = min(threads, self.max_cpu_cores)
        else:
            threads -= max(0, int(reserve_threads))
        env = os.environ.get("CEK_CPU_THREADS")
        if env:
            threads = int(env)
        info = cek.cpu_info(max(1, threads))
        info.streaming = True
        return info

    def copy(self, partition=None, streaming=None, max_cpu_cores=None) -> "ClDevice":
        return ClDevice(self.info, self.partition if partition is None else partition,
                        self.streaming if streaming is None else streaming,
                        self.max_cpu_cores if max_cpu_cores is None else max_cpu_cores, self.cu_partition)

    def __repr__(self) -> str:
        part = f" cu-part={self.cu_partition[0]}/{self.cu_partition[1]}" if self.cu_partition else ""
        return f"<ClDevice {self.info.describe()}{part}>"


class ClDevices:
    """An ordered list of devices (duplicates allowed)."""

    def __init__(self, devices: Optional[Iterable[ClDevice]] = None):
        self.devices: List[ClDevice] = list(devices or [])

    def __getitem__(self, i):
        if isinstance(i, slice):
            return ClDevices(self.devices[i])
        return ClDevices([self.devices[i]])

    def device(self, i: int) -> ClDevice:
        return self.devices[i]

    def __len__(self) -> int:
        return len(self.devices)

    @property
    def Length(self) -> int:  # noqa: N802
        return len(self.devices)

    def __iter__(self):
        return iter(self.devices)

    def __add__(self, other: "ClDevices") -> "ClDevices":
        return ClDevices(self.devices + list(other.devices))

    def cu_partitions(self, parts: int) -> "ClDevices":
        """Every GPU of the list as ``parts`` logical devices, each running on
        its own 1/parts of the GPU's CUs (CU-masked streams,
        ``hipExtStreamCreateWithCUMask``; every partition holds CUs of every
        XCD, ``cek.partition_cus``).  The reference lets one device be added
        to a pool or a stage several times (ClPipeline.cs:1728, :4337) and
        then shares it whole; partitions make the same logical devices run
        side by side on disjoint CUs, so a one-GPU box can stand in for
        ``parts`` smaller GPUs.  Non-GPU devices are kept as they are."""
        parts = int(parts)
        out = []
        for d in self.devices:
            if not d.is_gpu or parts <= 1:
                out.append(d)
                continue
            if d.info.compute_units % parts:
                raise ValueError(f"{d.info.compute_units} CUs do not split into {parts} partitions")
            out += [ClDevice(d.info, d.partition, d.streaming, d.max_cpu_cores, (p, parts)) for p in range(parts)]
        return ClDevices(out)

    cuPartitions = cu_partitions

    def _copy(self, devs, partition, streaming, max_cpu_cores) -> "ClDevices":
        return ClDevices(d.copy(partition, streaming, max_cpu_cores) for d in devs)

    # ---- filters ----
    def cpus(self, device_partition: bool = False, streaming: bool = False, max_cpu_cores: int = -1) -> "ClDevices":
        return self._copy([d for d in self.devices if d.is_cpu], device_partition, streaming, max_cpu_cores)

    def gpus(self, streaming: bool = False) -> "ClDevices":
        return self._copy([d for d in self.devices if d.is_gpu], False, streaming, -1)

    def accelerators(self, streaming: bool = False) -> "ClDevices":
        return ClDevices([])  # no ACC-class devices on an MI355X node

    def devices_with_dedicated_memory(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        r = [d for d in self.devices if d.info.dedicated_memory]
        return self._copy(r, device_partition, streaming, max_cpu_cores) if r else None

    def devices_with_host_memory_sharing(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        r = [d for d in self.devices if not d.info.dedicated_memory]
        return self._copy(r, device_partition, streaming, max_cpu_cores) if r else None

    def devices_with_most_compute_units(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        r = sorted(self.devices, key=lambda d: -d.compute_units)
        return self._copy(r, device_partition, streaming, max_cpu_cores)

    def devices_with_highest_memory_available(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        r = sorted(self.devices, key=lambda d: -d.memory_bytes)
        return self._copy(r, device_partition, streaming, max_cpu_cores)

    def _vendor(self, keys, device_partition, streaming, max_cpu_cores):
        keys = (keys,) if isinstance(keys, str) else keys
        r = [d for d in self.devices if any(k in (d.vendor + " " + d.name).lower() for k in keys)]
        return self._copy(r, device_partition, streaming, max_cpu_cores)

    def devices_amd(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._vendor(("amd", "advanced micro"), device_partition, streaming, max_cpu_cores)

    def devices_nvidia(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._vendor("nvidia", device_partition, streaming, max_cpu_cores)

    def devices_intel(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._vendor("intel", device_partition, streaming, max_cpu_cores)

    def devices_altera(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._vendor("altera", device_partition, streaming, max_cpu_cores)

    def devices_xilinx(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._vendor("xilinx", device_partition, streaming, max_cpu_cores)

    def devices_with_highest_direct_nbody_performance(self, device_partition=False, streaming=False,
                                                      max_cpu_cores=-1, n: int = 16 * 1024,
                                                      iterations: int = 5):
        """Rank devices, fastest first, by the N-body test (n=16384 per device,
        ClObjectApi.cs:1222-1244).  The reference's stopwatch also spans the
        kernel build and the host reference loop; here only the device's
        compute iterations are timed (after one warm-up compute), so the
        ranking measures the devices, not the JIT."""
        from .utils.tester import nbody

        timed = []
        for d in self.devices:
            dd = ClDevices([d.copy(device_partition, streaming, max_cpu_cores)])
            ms: list = []
            if nbody(n, dd, streaming, log=False, iterations=iterations, check=False, timing=ms):
                ms = [float("inf")]  # a device that cannot build the test ranks last
            timed.append((ms[0], d))
        timed.sort(key=lambda x: x[0])
        return self._copy([d for _, d in timed], device_partition, streaming, max_cpu_cores)

    def devices_with_highest_intrapolated_nbody_performance(self, *a, **k):
        raise NotImplementedError("not implemented in the reference either (ClObjectApi.cs:1254)")

    def devices_with_highest_least_oscillated_nbody_performance(self, *a, **k):
        raise NotImplementedError("not implemented in the reference either (ClObjectApi.cs:1267)")

    # camelCase aliases
    devicesWithDedicatedMemory = devices_with_dedicated_memory
    devicesWithHostMemorySharing = devices_with_host_memory_sharing
    devicesWithMostComputeUnits = devices_with_most_compute_units
    devicesWithHighestMemoryAvailable = devices_with_highest_memory_available
    devicesAmd = devices_amd
    devicesNvidia = devices_nvidia
    devicesIntel = devices_intel
    devicesAltera = devices_altera
    devicesXilinx = devices_xilinx
    devicesWithHighestDirectNbodyPerformance = devices_with_highest_direct_nbody_performance

    def log_info(self) -> str:
        lines = []
        for i, d in enumerate(self.devices):
            lines.append(f"Device {i}: {d.info.describe()}")
        s = "\n".join(lines)
        print(s)
        return s

    logInfo = log_info

    def __repr__(self) -> str:
        return "ClDevices[" + ", ".join(d.name for d in self.devices) + "]"


class ClPlatform:
    def __init__(self, name: str, vendor: str, devices: List[ClDevice]):
        self.name = name
        self.vendor = vendor
        self.devices = devices

    def number_of_gpus(self) -> int:
        return sum(d.is_gpu for d in self.devices)

    def number_of_cpus(self) -> int:
        return sum(d.is_cpu for d in self.devices)

    def number_of_accelerators(self) -> int:
        return 0

    numberOfGpus = number_of_gpus
    numberOfCpus = number_of_cpus
    numberOfAccelerators = number_of_accelerators

    def __repr__(self) -> str:
        return f"<ClPlatform {self.name} ({self.vendor}) devices={len(self.devices)}>"


class ClPlatforms:
    """All platforms of this host (reference ``ClPlatforms.all()``)."""

    def __init__(self, platforms: List[ClPlatform]):
        self.platforms = platforms

    @staticmethod
    def all() -> "ClPlatforms":
        infos = cek.enumerate_devices()
        gpus = [ClDevice(i) for i in infos if i.type == cek.DevType.GPU.value]
        cpus = [ClDevice(i) for i in infos if i.type == cek.DevType.CPU.value]
        plats = []
        if gpus:
            plats.append(ClPlatform(GPU_PLATFORM, "Advanced Micro Devices, Inc. (AMD)", gpus))
        if cpus:
            plats.append(ClPlatform(CPU_PLATFORM, cpus[0].name, cpus))
        return ClPlatforms(plats)

    def __getitem__(self, i):
        return ClPlatforms([self.platforms[i]])

    def __len__(self) -> int:
        return len(self.platforms)

    @property
    def Length(self) -> int:  # noqa: N802
        return len(self.platforms)

    def _all_devices(self) -> ClDevices:
        return ClDevices(d for p in self.platforms for d in p.devices)

    def platform_vendor_names(self) -> List[List[str]]:
        return [[p.name, p.vendor] for p in self.platforms]

    platformVendorNames = platform_vendor_names

    def platforms_with_most_devices(self) -> "ClPlatforms":
        return ClPlatforms(sorted(self.platforms, key=lambda p: -len(p.devices)))

    def _by_vendor(self, key: str) -> "ClPlatforms":
        return ClPlatforms([p for p in self.platforms if key in (p.vendor + p.name).lower()])

    def platforms_amd(self):
        return self._by_vendor("amd")

    def platforms_intel(self):
        return self._by_vendor("intel")

    def platforms_nvidia(self):
        return self._by_vendor("nvidia")

    def platforms_altera(self):
        return self._by_vendor("altera")

    def platforms_xilinx(self):
        return self._by_vendor("xilinx")

    platformsWithMostDevices = platforms_with_most_devices
    platformsAmd = platforms_amd
    platformsIntel = platforms_intel
    platformsNvidia = platforms_nvidia
    platformsAltera = platforms_altera
    platformsXilinx = platforms_xilinx

    def cpus(self, device_partition=False, streaming=False, max_cpu_cores=-1) -> ClDevices:
        return self._all_devices().cpus(device_partition, streaming, max_cpu_cores)

    def gpus(self, streaming=False) -> ClDevices:
        return self._all_devices().gpus(streaming)

    def accelerators(self, streaming=False) -> ClDevices:
        return ClDevices([])

    def devices_with_most_compute_units(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._all_devices().devices_with_most_compute_units(device_partition, streaming, max_cpu_cores)

    def devices_with_dedicated_memory(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._all_devices().devices_with_dedicated_memory(device_partition, streaming, max_cpu_cores)

    def devices_with_host_memory_sharing(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._all_devices().devices_with_host_memory_sharing(device_partition, streaming, max_cpu_cores)

    def devices_with_highest_memory_available(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._all_devices().devices_with_highest_memory_available(device_partition, streaming, max_cpu_cores)

    def devices_amd(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._all_devices().devices_amd(device_partition, streaming, max_cpu_cores)

    def devices_intel(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._all_devices().devices_intel(device_partition, streaming, max_cpu_cores)

    def devices_nvidia(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._all_devices().devices_nvidia(device_partition, streaming, max_cpu_cores)

    def devices_altera(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._all_devices().devices_altera(device_partition, streaming, max_cpu_cores)

    def devices_xilinx(self, device_partition=False, streaming=False, max_cpu_cores=-1):
        return self._all_devices().devices_xilinx(device_partition, streaming, max_cpu_cores)

    devicesWithMostComputeUnits = devices_with_most_compute_units
    devicesWithDedicatedMemory = devices_with_dedicated_memory
    devicesWithHostMemorySharing = devices_with_host_memory_sharing
    devicesWithHighestMemoryAvailable = devices_with_highest_memory_available
    devicesAmd = devices_amd
    devicesIntel = devices_intel
    devicesNvidia = devices_nvidia
    devicesAltera = devices_altera
    devicesXilinx = devices_xilinx

    def log_info(self) -> str:
        lines = []
        for i, p in enumerate(self.platforms):
            lines.append(f"Platform {i}: {p.name} / {p.vendor}")
            for j, d in enumerate(p.devices):
                lines.append(f"  Device {j}: {d.info.describe()}")
        s = "\n".join(lines)
        print(s)
        return s

    logInfo = log_info
