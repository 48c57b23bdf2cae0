"""One process per MI355X: range partitioning across ranks.

The reference drives all devices from one process (Cores.cs:156-344).  On an
MI355X node the idiomatic layout is one process per GPU (torchrun /
``torch.distributed``), so :class:`DistributedCruncher` runs the same
``compute()`` API with:

* the balancer over the *global* device list (``world × local devices``),
  each rank executing only its own devices' ranges;
* the per-device times of every call exchanged through the native
  node-local shared-memory control plane (``ShmExchanger``; ~µs), or through
  ``torch.distributed`` for multi-node jobs — every rank then computes the
  identical next split, so no split is ever communicated;
* an optional native RCCL communicator (xGMI) for the data plane:
  ``broadcast_reads`` (rank 0 uploads ``read`` arrays, RCCL broadcasts them),
  ``split_reads`` (each rank uploads 1/N, RCCL all-gathers) and ``gather_writes`` (written slices all-gathered into every rank's device
  replica — the "keep resident" iterative mode of SURVEY §5.8 item 5).
"""
from __future__ import annotations

import os
import socket
import uuid
import warnings
from dataclasses import dataclass
from typing import Optional

from .._native import cek, gpu_available
from ..cruncher import ClNumberCruncher
from ..hardware import ClDevices, ClPlatforms


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"

    @property
    def is_distributed(self) -> bool:
        return self.world > 1


def env_context() -> DistContext:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return DistContext(rank, world, local)


def init_distributed(backend: Optional[str] = None) -> DistContext:
    """Initialise torch.distributed from the torchrun environment (no-op for
    a single process).  Uses 127.0.0.1 when MASTER_ADDR is unset."""
    ctx = env_context()
    if ctx.world <= 1:
        return ctx
    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if not dist.is_initialized():
        if backend is None:
            # RCCL needs one GPU per rank; ranks sharing a GPU use gloo
            backend = "nccl" if (gpu_available() and torch.cuda.is_available()
                                 and torch.cuda.device_count() >= ctx.world) else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(ctx.local_rank)
        dist.init_process_group(backend=backend, rank=ctx.rank, world_size=ctx.world)
    ctx.backend = dist.get_backend()
    return ctx


class TorchExchanger(cek.Exchanger):
    """Exchanger over torch.distributed (gloo/nccl) — multi-node fallback."""

    def __init__(self, rank: int, world: int, group=None):
        super().__init__()
        self._rank, self._world, self._group = rank, world, group

    def allgather(self, local):
        import torch.distributed as dist

        out = [None] * self._world
        dist.all_gather_object(out, list(local), group=self._group)
        return [float(v) for part in out for v in part]

    def rank(self) -> int:
        return self._rank

    def world(self) -> int:
        return self._world


class TorchComm(cek.Comm):
    """The data plane of :class:`DistributedCruncher` over ``torch.distributed``
    (gloo) on HOST memory: the broadcast of ``read`` arrays, the split-read
    all-gather and the all-gather of written slices for ranks whose devices
    are CPU devices (their "device replica" is the host array itself).  The
    native scheduler calls it exactly where it calls RCCL on GPUs, so the
    whole keep-resident / broadcast-reads protocol — including which ranks
    must join which collective — runs in the GPU-less test tier."""

    def __init__(self, rank: int, world: int, group=None):
        super().__init__()
        self._rank, self._world, self._group = rank, world, group

    def rank(self) -> int:
        return self._rank

    def world(self) -> int:
        return self._world

    @staticmethod
    def _view(ptr: int, nbytes: int, dtype=None):
        import ctypes

        import numpy as np
        import torch

        buf = (ctypes.c_uint8 * nbytes).from_address(ptr)
        a = np.frombuffer(buf, dtype=np.uint8)
        if dtype is not None:
            a = a.view(dtype)
        return torch.from_numpy(a)

    def broadcast(self, ptr: int, nbytes: int, root: int, stream: int) -> None:
        import torch.distributed as dist

        if nbytes and self._world > 1:
            dist.broadcast(self._view(ptr, nbytes), src=root, group=self._group)

    def allgatherv(self, ptr: int, offsets, sizes, stream: int) -> None:
        import torch.distributed as dist

        if self._world <= 1:
            return
        for r in range(self._world):  # every rank joins every owner's broadcast
            if sizes[r]:
                dist.broadcast(self._view(ptr + offsets[r], sizes[r]), src=r, group=self._group)

    def _allreduce(self, ptr: int, count: int, dtype) -> None:
        import numpy as np
        import torch.distributed as dist

        if count and self._world > 1:
            dist.all_reduce(self._view(ptr, count * np.dtype(dtype).itemsize, dtype), group=self._group)

    def allreduce_sum_f32(self, ptr: int, count: int, stream: int) -> None:
        import numpy as np

        self._allreduce(ptr, count, np.float32)

    def allreduce_sum_f64(self, ptr: int, count: int, stream: int) -> None:
        import numpy as np

        self._allreduce(ptr, count, np.float64)


def _broadcast_object(obj, ctx: DistContext):
    import torch.distributed as dist

    lst = [obj]
    dist.broadcast_object_list(lst, src=0)
    return lst[0]


def _same_node(ctx: DistContext) -> bool:
    import torch.distributed as dist

    names = [None] * ctx.world
    dist.all_gather_object(names, socket.gethostname())
    return len(set(names)) == 1


class DistributedCruncher(ClNumberCruncher):
    """ClNumberCruncher whose device set spans the ranks of a job."""

    def __init__(self, kernel_source: str = "", ctx: Optional[DistContext] = None,
                 devices: Optional[ClDevices] = None, comm: bool = False, exchanger: str = "auto",
                 **kwargs):
        self.ctx = ctx or init_distributed()
        if devices is None:
            plats = ClPlatforms.all()
            gpus = plats.gpus()
            if len(gpus):
                devices = gpus[self.ctx.local_rank % len(gpus)]
            else:
                devices = plats.cpus(True)
        super().__init__(devices, kernel_source, **kwargs)
        self._exchanger = None
        self._comm = None
        self._warned_incoherent = False
        if self._cores is None:
            return
        if not self.ctx.is_distributed:
            if comm and self._cores.num_devices == 1 and self.devices.device(0).is_gpu:
                # a one-rank RCCL communicator: the data-plane code path (broadcast
                # of reads, all-gather of written slices) runs exactly as at N ranks
                self._comm = cek.RcclComm(cek.RcclComm.unique_id(), 0, 1, self.devices.device(0).info.ordinal)
                self._cores.set_distributed(None, self._comm, 1, 0)
            return
        import torch.distributed as dist

        nloc = self._cores.num_devices
        kind = exchanger
        if kind == "auto":
            kind = "shm" if _same_node(self.ctx) else "torch"
        if kind == "shm":
            token = _broadcast_object(uuid.uuid4().hex[:16] if self.ctx.rank == 0 else None, self.ctx)
            name = f"/cek_{token}"
            if self.ctx.rank == 0:
                self._exchanger = cek.ShmExchanger(name, 0, self.ctx.world, max(64, nloc))
            dist.barrier()
            if self.ctx.rank != 0:
                self._exchanger = cek.ShmExchanger(name, self.ctx.rank, self.ctx.world, max(64, nloc))
            dist.barrier()
            if self.ctx.rank == 0:
                self._exchanger.unlink()  # nothing left in /dev/shm once every rank exits
        else:
            self._exchanger = TorchExchanger(self.ctx.rank, self.ctx.world)
        if comm and nloc == 1 and self.devices.device(0).is_gpu:
            uid = _broadcast_object(cek.RcclComm.unique_id() if self.ctx.rank == 0 else None, self.ctx)
            self._comm = cek.RcclComm(uid, self.ctx.rank, self.ctx.world, self.devices.device(0).info.ordinal)
        elif comm and nloc == 1 and not self.devices.device(0).is_gpu:
            # CPU devices compute on the host arrays: the collectives run over
            # torch.distributed (gloo) on host memory
            self._comm = TorchComm(self.ctx.rank, self.ctx.world)
        self._cores.set_distributed(self._exchanger, self._comm, self.ctx.world * nloc, self.ctx.rank * nloc)

    @property
    def gather_writes(self) -> bool:
        return self._cores.dist_gather_writes

    @gather_writes.setter
    def gather_writes(self, v: bool) -> None:
        if v and self._comm is None and self.ctx.is_distributed:
            raise RuntimeError("gather_writes needs DistributedCruncher(comm=True)")
        self._cores.dist_gather_writes = bool(v)

    @property
    def broadcast_reads(self) -> bool:
        return self._cores.dist_broadcast_reads

    @broadcast_reads.setter
    def broadcast_reads(self, v: bool) -> None:
        if v and self._comm is None and self.ctx.is_distributed:
            raise RuntimeError("broadcast_reads needs DistributedCruncher(comm=True)")
        self._cores.dist_broadcast_reads = bool(v)

    @property
    def split_reads(self) -> bool:
        """Full ``read`` arrays are uploaded 1/N per rank (each over its own
        PCIe link) and completed by one RCCL all-gather over xGMI.  Requires
        identical host copies on every rank (e.g. inputs generated from the
        same seed); ``broadcast_reads`` is the variant where only rank 0's
        host copy counts."""
        return self._cores.dist_split_reads

    @split_reads.setter
    def split_reads(self, v: bool) -> None:
        if v and self._comm is None and self.ctx.is_distributed:
            raise RuntimeError("split_reads needs DistributedCruncher(comm=True)")
        self._cores.dist_split_reads = bool(v)

    def _build_call(self, *args, **kwargs):
        call = super()._build_call(*args, **kwargs)
        if self.ctx.is_distributed and not self._warned_incoherent and not (
                self._comm is not None and self._cores.dist_gather_writes):
            for a in call.arrays:
                if a.read and not a.partial and a.write and not a.write_all and not a.zc:
                    self._warned_incoherent = True
                    warnings.warn(
                        "DistributedCruncher: an array is read whole and written by slices. Each rank's "
                        "host copy receives only that rank's slices, and re-balancing moves work items "
                        "between ranks, so later reads see stale values from the other ranks. Use "
                        "comm=True with gather_writes (RCCL all-gather over xGMI), partial_read, or read=False.",
                        RuntimeWarning, stacklevel=4)
                    break
        return call

    def barrier(self) -> None:
        if self._exchanger is not None:
            self._exchanger.allgather([0.0])
