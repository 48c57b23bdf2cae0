"""bench.py --gpus N without a torchrun environment starts N rank processes
itself (torch.distributed.run as a child process) and every rank derives the
same split.  CPU rehearsal: each rank's device is the CPU
device, the control plane is gloo + the shared-memory exchanger."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_n_ranks_with_identical_splits(n):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["CEK_CPU_THREADS"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "2",
                        "--warmup", "1", "--size", "128", "--device", "cpu"],
                       cwd="/tmp", env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["config"]["parallelism"] == f"range-partition dp{n}"
    ex = out["extra"]
    assert len(ex["sgemm_ranges"]) == n and sum(ex["sgemm_ranges"]) == 128 * 128
    assert all(x % 64 == 0 for x in ex["sgemm_ranges"])  # whole work-groups
    assert ex["sgemm_ranges_identical_on_all_ranks"] is True
    assert ex["sgemm_max_rel_err"] < 1e-5
    assert out["steps"] == 2 and out["warmup"] == 1


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--size", "64", "--steps", "1", "--warmup", "0"],
                       cwd="/tmp", env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "ranks" in (r.stderr + r.stdout)
