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
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional

import numpy as np

from ..arrays import ClArray
from .netbuf import CHECKPOINT, NetworkBuffer, TYPE_INT

_ARRAY_TAG = 0x41525200  # "ARR\0"
_STATE_TAG = 0x53544100  # "STA\0"


def save(path: str, arrays: Dict[str, ClArray], cruncher=None, download: bool = True) -> int:
    """Write arrays (+ the cruncher's balancer state) to ``path``.  With
    ``download`` the device replicas of device 0 are read back first for
    arrays that are device-resident (``write=False``).  Returns bytes."""
    nb = NetworkBuffer(CHECKPOINT)
    names = list(arrays)
    nb.add_string("\n".join(names), _STATE_TAG - 1)
    for i, name in enumerate(names):
        a = arrays[name]
        if download and cruncher is not None and not a.write:
            cruncher.download(a, 0)
        nb.add_array(a.array, _ARRAY_TAG + i)
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
    return len(data)


def load(path: str, arrays: Optional[Dict[str, ClArray]] = None, cruncher=None) -> Dict[str, np.ndarray]:
    """Read a checkpoint.  Arrays given in ``arrays`` are filled in place
    (and re-uploaded on their next compute); balancer state is restored into
    ``cruncher``.  Returns every array by name."""
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
