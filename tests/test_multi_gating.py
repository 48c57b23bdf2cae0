"""CPU tier for the multi-GPU tier's plumbing: the skip gate, the peer-path
classification, the torchrun command line, and the rank worker's control
plane (2 gloo ranks on CPU devices: identical, uneven splits)."""
import json
import os
import subprocess

import pytest

from cekirdekler_amd._native import cek
from cekirdekler_amd.utils.multigpu import child_env, multi_gpu_skip_reason, torchrun_cmd

HERE = os.path.dirname(os.path.abspath(__file__))


def test_skip_gate():
    assert multi_gpu_skip_reason(2, have=0) == "needs 2 physical GPUs, 0 visible"
    assert multi_gpu_skip_reason(2, have=1)
    assert multi_gpu_skip_reason(2, have=2) is None
    assert multi_gpu_skip_reason(8, have=4)
    assert multi_gpu_skip_reason(4, have=8) is None
    with pytest.raises(ValueError):
        multi_gpu_skip_reason(1, have=8)


def test_multi_tier_skips_without_gpus():
    """On this container (no GPU) every multi-GPU test is skipped, not failed."""
    r = subprocess.run(["python", "-m", "pytest", "-q", "-m", "gpu", os.path.join(HERE, "test_gpu_multi.py"),
                        "-p", "no:cacheprovider"], cwd=os.path.dirname(HERE), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "skipped" in r.stdout and "failed" not in r.stdout


def test_peer_path_classification():
    assert cek.peer_path([]) == "none"
    assert cek.peer_path([[1]]) == "none"
    assert cek.peer_path([[1, 1], [1, 1]]) == "xgmi"
    assert cek.peer_path([[1, 0], [1, 1]]) == "staged"
    full = [[1] * 8 for _ in range(8)]
    assert cek.peer_path(full) == "xgmi"
    full[3][5] = 0
    assert cek.peer_path(full) == "staged"
    assert cek.enable_peer_access_among([]) == []


def test_torchrun_cmd():
    cmd = torchrun_cmd("x.py", 4, ["--a", 1], port=12345)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=12345" in cmd
    assert cmd[-2:] == ["--a", "1"]
    env = child_env()
    assert "RANK" not in env and env["PYTHONPATH"].split(os.pathsep)[0] == os.path.dirname(HERE)


def test_cores_peer_topology_on_cpu_devices():
    import cekirdekler_amd as ck

    cpu = ck.ClPlatforms.all().cpus(True)
    cr = ck.ClNumberCruncher(cpu + cpu, "__global__ void k(float* x) { x[get_global_id(0)] += 1.0f; }")
    assert cr.peer_topology() == {"ordinals": [], "matrix": [], "path": "none"}
    cr.dispose()


def test_rank_worker_control_plane_two_gloo_ranks():
    cmd = torchrun_cmd(os.path.join(HERE, "rccl_worker.py"), 2, ["--cpu", "--elems", str(256 * 64)])
    r = subprocess.run(cmd, cwd=HERE, env=child_env(), capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.stdout[-2000:], r.stderr[-2000:])
    out = json.loads(lines[-1])
    assert out["ok"] and out["splits_identical"] and out["ranks"] == 2, out
    assert out["per_rank"][0]["uneven"], out


@pytest.mark.parametrize("world", [2, 4])
def test_rank_worker_data_plane_torchcomm(world):
    """the RCCL worker's data-plane checks (broadcast of
    reads from rank 0, split reads, all-gather of written slices with uneven
    splits, keep-resident gather ping-pong with no host traffic) over
    TorchComm / gloo on CPU devices, at world 2 and 4."""
    cmd = torchrun_cmd(os.path.join(HERE, "rccl_worker.py"), world, ["--torchcomm", "--elems", str(256 * 256)])
    env = child_env()
    env["CEK_CPU_THREADS"] = "1"
    r = subprocess.run(cmd, cwd=HERE, env=env, capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.stdout[-2000:], r.stderr[-2000:])
    out = json.loads(lines[-1])
    assert out["ok"] and out["splits_identical"] and out["ranks"] == world, json.dumps(out)[:3000]
    per = out["per_rank"]
    assert per[0]["uneven"] and all(o["comm"] == "TorchComm" for o in per), per[0]
    assert all(set(o["checks"]) >= {"host_replica_all", "split_reads_slice", "gather_flag_replica",
                                    "gather_flag_no_host_traffic"} for o in per)
    # rank 0 alone uploads for the broadcast of reads
    assert per[0]["broadcast_h2d_bytes"] > 0 and all(o["broadcast_h2d_bytes"] == 0 for o in per[1:])


def test_peer_pairs_and_report_shape(monkeypatch):
    """The xGMI bandwidth report's structure, on a fake measurement backend
    (the real one needs GPUs): pairs chosen, both engines per pair, the
    faster one named, verification folded into all_verified."""
    from cekirdekler_amd.utils import multigpu

    assert multigpu.peer_pairs(1) == []
    assert multigpu.peer_pairs(2) == [(0, 1), (1, 0)]
    assert multigpu.peer_pairs(8) == [(0, 1), (0, 7), (1, 2), (7, 0)]

    class Fake:
        @staticmethod
        def measure_copy(s, d, b, e, reps=5, stream_ordinal=-1):
            return {"src": s, "dst": d, "engine": ["sdma", "kernel"][e], "bytes": b, "gbps": 50.0 + 10 * e,
                    "ms": 1.0, "verified": True}

        @staticmethod
        def measure_all_pairs(ords, b, e, reps=3):
            return {"gpus": len(ords), "aggregate_gbps": 1000.0, "verified": True}

    import cekirdekler_amd._native as nat

    monkeypatch.setattr(nat, "cek", Fake)
    monkeypatch.setattr(multigpu, "visible_gpus", lambda: 4)
    rep = multigpu.peer_bandwidth_report([0, 1, 2, 3])
    assert rep["gpus_visible"] == 4 and rep["job_gpus"] == 4
    assert [(r["src"], r["dst"]) for r in rep["pairs"]] == [(0, 1), (0, 3), (1, 2), (3, 0)]
    assert all(r["faster"] == "kernel" for r in rep["pairs"])
    assert rep["all_verified"] and rep["min_pair_gbps"] == 60.0
    assert set(rep["all_pairs"]) == {"sdma", "kernel"}
