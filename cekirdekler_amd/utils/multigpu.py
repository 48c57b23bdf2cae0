"""Helpers for the multi-GPU test tier: how many physical GPUs
this process sees, why a test needing N of them is skipped, and the
``torch.distributed.run`` command line for a child job of N ranks.

The child job is always started as a separate process (``subprocess``),
never by replacing the current one: the parent may already have initialised
the GPU runtime.
"""
from __future__ import annotations

import os
import socket
import sys
from typing import List, Optional, Sequence


def visible_gpus() -> int:
    """Physical GPUs visible to this process (0 without a HIP runtime)."""
    try:
        from .._native import cek

        return int(cek.gpu_count())
    except Exception:
        return 0


def multi_gpu_skip_reason(need: int, have: Optional[int] = None) -> Optional[str]:
    """None when ``need`` distinct GPUs are visible, else the skip reason."""
    have = visible_gpus() if have is None else int(have)
    if need < 2:
        raise ValueError("the multi-GPU tier needs at least 2 GPUs per test")
    if have >= need:
        return None
    return f"needs {need} physical GPUs, {have} visible"


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def torchrun_cmd(script: str, nproc: int, args: Sequence[str] = (), port: Optional[int] = None) -> List[str]:
    """``python -m torch.distributed.run`` for ``nproc`` ranks on this node,
    rendezvous on 127.0.0.1 (the container hostname may not resolve)."""
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port or free_port()}", os.path.abspath(script),
            *[str(a) for a in args]]


def child_env() -> dict:
    """The parent's environment minus any torchrun variables of its own, with
    the repository on PYTHONPATH."""
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


# ---------------------------------------------------------------- xGMI evidence
ENGINES = {"sdma": 0, "kernel": 1}


def peer_pairs(n: int) -> List[tuple]:
    """The GPU pairs a bandwidth report times one by one: neighbours 0→1,
    the farthest ordinal 0→n-1 and 1→2 (distinct pairs only)."""
    cand = [(0, 1), (0, n - 1), (1, 2), (n - 1, 0)]
    out = []
    for p in cand:
        if p[0] != p[1] and max(p) < n and p not in out:
            out.append(p)
    return out


def peer_bandwidth_report(ordinals: Sequence[int], pair_bytes: int = 256 << 20, all_bytes: int = 64 << 20,
                          reps: int = 5) -> dict:
    """Device→device copy bandwidth by engine:
    SDMA (hipMemcpyPeerAsync) and a pull copy kernel on the destination, for
    a few GPU pairs one at a time, every ordered pair at once, and inside
    GPU 0.  Every copy is checked byte for byte.  The per-pair winner is
    entered into the runtime's engine table (Cores / CopyEngine use it for
    that pair from then on)."""
    from .._native import cek

    ords = [int(o) for o in ordinals]
    out = {"gpus_visible": visible_gpus(), "job_gpus": len(ords), "pair_bytes": pair_bytes,
           "same_gpu": {}, "pairs": [], "all_pairs": {}}
    if not ords:
        return out
    g0 = ords[0]
    for name, e in ENGINES.items():
        out["same_gpu"][name] = cek.measure_copy(g0, g0, pair_bytes, e, reps)
    out["same_gpu"]["faster"] = max(ENGINES, key=lambda k: out["same_gpu"][k]["gbps"])
    for i, j in peer_pairs(len(ords)):
        s, d = ords[i], ords[j]
        row = {"src": s, "dst": d}
        for name, e in ENGINES.items():
            row[name] = cek.measure_copy(s, d, pair_bytes, e, reps)
        row["faster"] = max(ENGINES, key=lambda k: row[k]["gbps"])
        if hasattr(cek, "record_copy_engine") and all(row[k]["verified"] for k in ENGINES):
            cek.record_copy_engine(s, d, pair_bytes, ENGINES[row["faster"]])
        out["pairs"].append(row)
    if len(ords) >= 2:
        for name, e in ENGINES.items():
            out["all_pairs"][name] = cek.measure_all_pairs(ords, all_bytes, e, 2)
    checks = [out["same_gpu"][k]["verified"] for k in ENGINES]
    checks += [r[k]["verified"] for r in out["pairs"] for k in ENGINES]
    checks += [v["verified"] for v in out["all_pairs"].values()]
    out["all_verified"] = all(checks)
    if out["pairs"]:
        out["min_pair_gbps"] = min(max(r[k]["gbps"] for k in ENGINES) for r in out["pairs"])
    return out


# --------------------------------------------- broadcast vs per-GPU upload threshold
PEER_READ_SIZES = (65536, 262144, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20)
_TOUCH_SRC = """
__global__ void cek_touch(const float* x, float* y) {
    long long i = get_global_id(0);
    y[i] = x[i] * 2.0f + 1.0f;
}
"""
# measured thresholds per device set (ordinals, CU partitions), for the process
_PEER_READ_CACHE: dict = {}


def pick_crossover(sizes: Sequence[int], direct_ms: Sequence[float], staged_ms: Sequence[float]) -> Optional[int]:
    """The smallest size from which the staged fan-out stays faster than the
    direct uploads at every larger size measured (None: never)."""
    for i in range(len(sizes)):
        if all(s < d for s, d in zip(staged_ms[i:], direct_ms[i:])):
            return int(sizes[i])
    return None


def measure_peer_read_threshold(devices, sizes: Sequence[int] = PEER_READ_SIZES, calls: int = 5) -> dict:
    """Time the two ways a full ``read`` array reaches every GPU of
    ``devices`` ("choose by size threshold, measured"):
    ``direct`` — every GPU uploads the whole array over its own PCIe link
    (the reference, Worker.cs:833-860) — and ``staged`` — 1/D uploaded per
    GPU, the rest pulled from the peers' replicas over xGMI
    (``Cores::stage_peer_reads``).  A tiny kernel reads the array on every
    GPU, so a call's time is the transfer; modes interleaved, median of
    ``calls``, every output checked.  Returns the sizes, both timings,
    ``crossover_bytes`` (:func:`pick_crossover`) and ``exact``."""
    import statistics
    import time

    import numpy as np

    from ..arrays import ClArray
    from ..cruncher import ClNumberCruncher

    cr = ClNumberCruncher(devices, _TOUCH_SRC)
    if cr.error_code():
        raise RuntimeError(cr.error_message())
    D = cr.number_of_devices
    try:
        cr.peer_read_min_bytes = 0
        G = 256 * D * 4
        y = ClArray(np.zeros(G, np.float32))
        y.read = False
        out = {"devices": D, "calls": int(calls), "sizes": [], "direct_ms": [], "staged_ms": [],
               "staged_path": [], "exact": True}
        cid = 1
        for size in sizes:
            n = max(G, int(size) // 4)
            x = ClArray(n, np.float32)
            x.array[:] = np.arange(n, dtype=np.float32) % 1000
            x.write = False
            want = x.array[:G] * 2.0 + 1.0
            times = {"direct": [], "staged": []}
            for mode in ("direct", "staged"):  # untimed first calls: buffers, balancer state
                cr.peer_reads = mode == "staged"
                x.next_param(y).compute(cr, cid + (mode == "staged"), "cek_touch", G, 256)
            for _ in range(max(1, int(calls))):
                for mode in ("direct", "staged"):
                    cr.peer_reads = mode == "staged"
                    y.array[:] = 0
                    t0 = time.perf_counter()
                    x.next_param(y).compute(cr, cid + (mode == "staged"), "cek_touch", G, 256)
                    times[mode].append((time.perf_counter() - t0) * 1e3)
                    out["exact"] &= bool(np.array_equal(y.array, want))
            out["sizes"].append(4 * n)
            out["direct_ms"].append(round(statistics.median(times["direct"]), 4))
            out["staged_ms"].append(round(statistics.median(times["staged"]), 4))
            out["staged_path"].append(cr.last_record()["p2p_path"])
            x.dispose()
            cid += 2
        y.dispose()
    finally:
        cr.dispose()
    out["crossover_bytes"] = pick_crossover(out["sizes"], out["direct_ms"], out["staged_ms"])
    return out


def device_set_key(devices) -> tuple:
    """(ordinal, CU partition) of every GPU in ``devices``: the cache key of a
    measured threshold."""
    return tuple((d.info.ordinal, d.cu_partition) for d in devices if d.is_gpu)
