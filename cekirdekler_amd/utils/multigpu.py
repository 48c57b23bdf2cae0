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
