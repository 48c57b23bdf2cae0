"""Checkpoint / resume in the reference's only serialised layout.

The reference has no checkpointing; the state that survives
between its computes is the device buffer cache, the arg-binding cache and
the per-compute-id range/offset tables + timing history (Cores.cs:130-135,
:1065-1098).  A checkpoint here is one :class:`NetworkBuffer` (command
``CHECKPOINT``) holding

* every array's contents as a typed record whose ``hash`` is the array's
  position in the checkpoint (bf16 travels as the 16-bit ``char`` type), and
* per compute id: an int record ``[id, devices, depth]``, an int64 record of
  the ranges, a double record of the last benchmarks and a double record of
  the flattened smoothing history,

so a resumed cruncher re-balances from where it stopped instead of from the
equal split.

Device-resident arrays (``write=False``) are saved as the devices hold them:
each device's replica is authoritative only for the slice of the split it
computed (Worker.cs:1349-1352 — the reference's slice ownership; the split is
the per-compute-id state of Cores.cs:130-135).  ``save`` assembles every such
array from each device's own slice, by the split of the last compute the
array took part in (``ClArray._split_log``; override per array with
``compute_ids``).  A keep-resident (``gather_resident``) array is whole in
any replica.  In a :class:`DistributedCruncher` job every rank contributes
its devices' slices and rank 0 writes the one file.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional

import numpy as np

from ..arrays import ClArray
from .netbuf import CHECKPOINT, NetworkBuffer, TYPE_INT

_ARRAY_TAG = 0x41525200  # "ARR\0"
_STATE_TAG = 0x53544100  # "STA\0"


def _owned_slices(a: ClArray, cruncher, compute_id: Optional[int] = None) -> Optional[List[tuple]]:
    """(local device, first element, end element) of every slice this
    process's devices own in ``a``, or None when the array's device replicas
    are whole (gathered) or it never took part in a compute of ``cruncher``."""
    if a.gather_resident:
        return None
    log = a._split_log.get(id(cruncher))
    if log is None and compute_id is None:
        return None
    cid, epw, epg, L = log if log is not None else (compute_id, a.elements_per_work_item, a.elements_per_group, 0)
    if compute_id is not None:
        cid = compute_id
    cores = cruncher.cores
    ranges, refs = cores.ranges(cid), cores.references(cid)
    if not ranges:
        return None
    L = L or 1
    out = []
    for dev in range(cores.num_devices):
        g = cores.global_base + dev
        if epg > 0:
            lo, n = refs[g] // L * epg, ranges[g] // L * epg
        else:
            lo, n = refs[g] * epw, ranges[g] * epw
        lo, hi = min(lo, a.N), min(lo + n, a.N)
        if hi > lo:
            out.append((dev, lo, hi))
    return out


def _assemble(a: ClArray, cruncher, compute_id: Optional[int]) -> List[tuple]:
    """Fill ``a``'s host copy from the device replicas: device 0's whole
    replica, then every other local device's own slice from its replica.
    Returns the (first, end) element ranges this process owns: the whole
    array when the replicas are whole (``owned is None``), nothing when the
    split left every local device an empty range (``owned == []``: the
    reference law does give a slow device range 0, HelperFunctions.cs:190-280,
    and such a replica holds stale data everywhere)."""
    cores = cruncher.cores
    owned = _owned_slices(a, cruncher, compute_id)
    cruncher.download(a, 0)
    if owned is None:
        return [(0, a.N)]
    if not owned:
        return []
    host = a.array
    if any(dev != 0 for dev, _, _ in owned):
        base = host.copy()
        for dev in range(1, cores.num_devices):
            mine = [(lo, hi) for d, lo, hi in owned if d == dev]
            if not mine:
                continue
            cruncher.download(a, dev)
            for lo, hi in mine:
                base[lo:hi] = host[lo:hi]
        host[:] = base
    return [(lo, hi) for _, lo, hi in owned]


def save(path: str, arrays: Dict[str, ClArray], cruncher=None, download: bool = True,
         compute_ids: Optional[Dict[str, int]] = None) -> int:
    """Write arrays (+ the cruncher's balancer state) to ``path``.  With
    ``download``, device-resident arrays (``write=False``) are assembled from
    the devices first: each device contributes the slice it owns under the
    split of the array's last compute (``compute_ids`` names another compute
    id per array).  In a distributed job every rank must call ``save``; rank
    0 gathers the other ranks' slices and writes the file.  Returns bytes
    written (on every rank)."""
    compute_ids = compute_ids or {}
    names = list(arrays)
    ctx = getattr(cruncher, "ctx", None)
    dist_job = ctx is not None and ctx.is_distributed
    pieces: Dict[str, list] = {}
    for name in names:
        a = arrays[name]
        if download and cruncher is not None and not a.write and not a.zero_copy:
            owned = _assemble(a, cruncher, compute_ids.get(name))
            # a rank ships only the slices its devices computed (possibly
            # none); a whole replica (gathered / keep-resident) is never
            # shipped: rank 0's own copy is already whole
            if dist_job and _owned_slices(a, cruncher, compute_ids.get(name)) is not None:
                pieces[name] = [(lo, hi, a.array[lo:hi].tobytes()) for lo, hi in owned]
    if dist_job:
        import torch.distributed as dist

        got = [None] * ctx.world if ctx.rank == 0 else None
        dist.gather_object(pieces, got, dst=0)
        if ctx.rank == 0:
            for r, part in enumerate(got):
                if r == 0:
                    continue
                for name, segs in part.items():
                    host = arrays[name].array
                    for lo, hi, raw in segs:
                        host[lo:hi] = np.frombuffer(raw, dtype=host.dtype, count=hi - lo)
    nbytes = 0
    if not dist_job or ctx.rank == 0:
        nb = NetworkBuffer(CHECKPOINT)
        nb.add_string("\n".join(names), _STATE_TAG - 1)
        for i, name in enumerate(names):
            nb.add_array(arrays[name].array, _ARRAY_TAG + i)
        if cruncher is not None:
            c = cruncher.cores
            for cid in c.compute_ids():
                rng = np.asarray(c.ranges(cid), np.int64)
                hist = np.asarray(c.history(cid), np.float64)
                nb.add_ints([cid, len(rng), hist.shape[0]], _STATE_TAG)
                nb.add_array(rng, _STATE_TAG + 1)
                nb.add_doubles(c.benchmarks(cid), _STATE_TAG + 2)
                nb.add_doubles(hist.reshape(-1), _STATE_TAG + 3)
        data = nb.to_bytes()
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
        nbytes = len(data)
    if dist_job:
        import torch.distributed as dist

        box = [nbytes]
        dist.broadcast_object_list(box, src=0)
        nbytes = int(box[0])
    return nbytes


def load(path: str, arrays: Optional[Dict[str, ClArray]] = None, cruncher=None) -> Dict[str, np.ndarray]:
    """Read a checkpoint.  Arrays given in ``arrays`` are filled in place;
    with a ``cruncher`` they are also uploaded to every local device replica
    (device-resident arrays resume where they stopped, their flags
    untouched), without one they are re-uploaded on their next compute.
    Balancer state is restored into ``cruncher``.  Returns every array by
    name.  In a distributed job every rank loads the same file."""
    with open(path, "rb") as f:
        data = f.read()
    cmd, recs = NetworkBuffer.parse(data)
    if cmd != CHECKPOINT:
        raise ValueError(f"{path}: not a checkpoint (command {cmd})")
    names = NetworkBuffer.record_string(recs[0]).split("\n") if recs[0].data.size else []
    out: Dict[str, np.ndarray] = {}
    i = 1
    for name in names:
        r = recs[i]
        out[name] = r.data.copy()
        i += 1
        if arrays is not None and name in arrays:
            dst = arrays[name].array
            dst[:] = r.data.view(dst.dtype) if r.data.dtype.itemsize == dst.dtype.itemsize else r.data
            if cruncher is not None and not arrays[name].zero_copy:
                for dev in range(cruncher.cores.num_devices):
                    cruncher.upload(arrays[name], dev)
            else:
                arrays[name].read = True
    while i + 3 < len(recs) + 1 and i < len(recs):
        head = recs[i]
        if head.type != TYPE_INT or head.hash != _STATE_TAG:
            break
        cid, ndev, depth = (int(x) for x in head.data[:3])
        rng = [int(x) for x in recs[i + 1].data]
        bench = [float(x) for x in recs[i + 2].data]
        hist = np.asarray(recs[i + 3].data, np.float64).reshape(depth, ndev).tolist()
        if cruncher is not None:
            cruncher.cores.set_state(cid, rng, hist, bench)
        i += 4
    return out
