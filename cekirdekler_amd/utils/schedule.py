"""Dependency checker for the recorded pipeline schedule (SURVEY §7.4 item 5:
"unit-test the event pipeline's dependency DAG with a recorded-schedule
checker").

``Cores.record_schedule = True`` makes every pipeline append the operations
it issues — transfers, kernels, event records and waits, each with its
logical stream — in issue order.  :func:`check_pipeline_schedule` rebuilds
the happens-before relation the device would enforce (program order inside a
stream + record→wait event edges) and verifies for every device:

* each chunk's kernels run after the full reads and after that chunk's H2D;
* each chunk's D2H runs after that chunk's kernels;
* the final synchronisation point (last op on the main stream) is reached
  only after every kernel and D2H.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Sequence, Tuple

Op = Tuple[int, str, int, int, int, int]  # device, op, stream, begin, count, event


def happens_before(ops: Sequence[Op]) -> List[set]:
    """Transitive successor sets of the schedule's happens-before graph."""
    n = len(ops)
    succ: List[set] = [set() for _ in range(n)]
    last_on_stream: Dict[int, int] = {}
    last_rec: Dict[int, int] = {}
    for i, (_, op, stream, _, _, ev) in enumerate(ops):
        if stream in last_on_stream:
            succ[last_on_stream[stream]].add(i)
        last_on_stream[stream] = i
        if op == "rec":
            last_rec[ev] = i
        elif op == "wait":
            if ev not in last_rec:
                raise AssertionError(f"op {i}: wait on event {ev} that was never recorded")
            succ[last_rec[ev]].add(i)
    # reachability (ops are issued in order, so edges only point forward)
    reach: List[set] = [set() for _ in range(n)]
    for i in range(n - 1, -1, -1):
        for j in succ[i]:
            reach[i].add(j)
            reach[i] |= reach[j]
    return reach


def check_pipeline_schedule(schedule: Sequence[Op], prefix_uploads: bool = False) -> int:
    """Raises AssertionError on a missing dependency; returns the number of
    checked (kernel, transfer) pairs.

    ``prefix_uploads``: every chunk's kernels must also run after the H2D of
    every EARLIER chunk (explicit blobs of a shell-streamed GEMM: shell s
    reads the row panels uploaded by blobs 0..s, which alternate between the
    two half-pipelines)."""
    by_dev: Dict[int, List[Op]] = defaultdict(list)
    for op in schedule:
        by_dev[op[0]].append(tuple(op))
    checked = 0
    for dev, ops in by_dev.items():
        reach = happens_before(ops)
        full = [i for i, o in enumerate(ops) if o[1] == "h2d" and o[3] < 0]
        h2d: Dict[Tuple[int, int], List[int]] = defaultdict(list)  # a chunk may upload on two streams
        for i, o in enumerate(ops):
            if o[1] == "h2d" and o[3] >= 0:
                h2d[(o[3], o[4])].append(i)
        kern = {(o[3], o[4]): i for i, o in enumerate(ops) if o[1] == "kernel"}
        d2h = {(o[3], o[4]): i for i, o in enumerate(ops) if o[1] == "d2h"}
        main_ops = [i for i, o in enumerate(ops) if o[2] == 0]
        final = main_ops[-1] if main_ops else None
        for chunk, k in kern.items():
            for f in full:
                if k not in reach[f]:
                    raise AssertionError(f"device {dev}: kernel {chunk} may start before the full reads")
            for u in h2d.get(chunk, []):
                if k not in reach[u]:
                    raise AssertionError(f"device {dev}: kernel {chunk} may start before its H2D")
            if prefix_uploads:
                for other, ups in h2d.items():
                    if other[0] < chunk[0] and any(k not in reach[u] for u in ups):
                        raise AssertionError(f"device {dev}: kernel {chunk} may start before the H2D of "
                                             f"earlier blob {other}")
            if chunk in d2h and d2h[chunk] not in reach[k]:
                raise AssertionError(f"device {dev}: D2H {chunk} may start before its kernels")
            checked += 1
        if final is not None:
            for i in list(kern.values()) + list(d2h.values()):
                if final != i and final not in reach[i]:
                    raise AssertionError(f"device {dev}: op {ops[i]} is not ordered before the final sync")
    return checked
