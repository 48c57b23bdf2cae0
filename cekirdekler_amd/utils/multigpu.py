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
