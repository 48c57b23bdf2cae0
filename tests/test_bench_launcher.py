"""bench.py --gpus N without a torchrun environment starts N rank processes
itself (torch.distributed.run as a child process) and every rank derives the
same split.  CPU rehearsal: each rank's device is the CPU
device, the control plane is gloo + the shared-memory exchanger.  N = 8 is
the node the driver's scaling run uses."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINE_LIMIT = 6000  # the driver keeps the tail of stdout: the whole line must fit


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_spawns_n_ranks_with_identical_splits(n, tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["CEK_CPU_THREADS"] = "1" if n >= 8 else "2"
    detail = tmp_path / "detail.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "2",
                        "--warmup", "1", "--size", "128", "--device", "cpu", "--detail", str(detail)],
                       cwd="/tmp", env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    assert len(lines[0]) < LINE_LIMIT, len(lines[0])
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["config"]["parallelism"] == f"range-partition dp{n}"
    sg = out["extra"]["sgemm"]
    assert list(out["extra"])[-3:] == ["load_balance_iters", "mandelbrot_4k", "sgemm"]  # metric components last
    assert len(sg["ranges"]) == n and sum(sg["ranges"]) == 128 * 128
    assert all(x % 64 == 0 for x in sg["ranges"])  # whole work-groups
    assert sg["ranges_identical_on_all_ranks"] is True
    assert sg["max_rel_err_full"] < 1e-5 and sg["tiles_checked"] == sg["tiles_total"]
    assert out["steps"] == 2 and out["warmup"] == 1
    full = json.loads(detail.read_text())
    assert full["sgemm"]["ranges"] == sg["ranges"] and len(full["sgemm_ranges_all_ranks"]) == n


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--size", "64", "--steps", "1", "--warmup", "0"],
                       cwd="/tmp", env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "ranks" in (r.stderr + r.stdout)


def _bench_module():
    spec = importlib.util.spec_from_file_location("bench_main", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("world", [1, 8])
def test_compact_line_fits_with_a_real_gpu_run(world):
    """the line printed from a full GPU run's results
    (round 4's session-22 line, every config present, with an 8-rank split
    for world 8) stays under the limit and carries every metric component."""
    bench = _bench_module()
    old = json.loads(open(os.path.join(ROOT, "profiles", "r4", "bench_session22.json")).read())
    ex = old["extra"]
    ranges = [65536] * world if world > 1 else ex["sgemm_ranges"]
    sg = {"gflops": 1.5e6, "ms": 0.72, "tile": "256x256pb", "single_queue": ex["sgemm_single_queue"],
          "async_queues": ex["sgemm_async_queues"], "sync_per_step_gflops": ex["sgemm_sync_per_step_gflops"],
          "ranges": ranges, "balancer_setup_calls": 6, "max_rel_err": 1.5e-6, "tiles_checked": 1024,
          "tiles_total": 1024, "host_resident_ms": 7.09, "host_resident_mode": ex["sgemm_host_resident_mode"],
          "max_rel_err_host_resident": 1.5e-6, "handover_fallbacks": 0}
    full = {"sgemm": sg, "sgemm_ranges_all_ranks": [ranges] * world, "sgemm_row_major_c": ex["sgemm_row_major_c"],
            "mandelbrot_4k": ex["mandelbrot_4k"], "load_balance_iters": ex["load_balance_iters"],
            **{k: ex[k] for k in ("nbody_pipeline", "task_pool", "saxpy_1m_cpu", "wave_cpu_gpu",
                                  "sgemm_host_resident_rccl", "hetero_stream")},
            "pipeline_overlap": {"read_compute_write_ms": [4.9, 4.8, 4.7], "ideal_speedup_sum_over_max": 2.9,
                                 "ms": {"3phase": 15.0}, "pipeline_speedup_event": 2.1,
                                 "pipeline_speedup_driver": 2.0, "best_event": "event_b8",
                                 "best_event_4streams": "event_b8_4streams", "best_driver_q4": "driver_b8_q4",
                                 "best_driver_q16": "driver_b8_q16", "event_5_vs_4_streams": [7.1, 7.0],
                                 "driver_q4_vs_q16": [7.5, 7.9], "outputs_exact": True, "lcg_iters": 4000},
            "peer_topology": ex["peer_topology"]}
    extra = bench.compact_extra(full, "gpurun_out/bench_detail_n1.json")
    line = json.dumps({"metric": bench.METRIC, "value": 1.5e6, "unit": "GFLOPS", "n_gpus": world, "steps": 20,
                       "warmup": 3, "ms_per_step": 0.72, "higher_is_better": True, "scaling": "strong",
                       "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
                       "config": {"model": "SGEMM 8192x8192x8192 bf16 (fp32 acc/out), range-partitioned + "
                                           "load-balanced, tile 256x256pb", "global_batch": 1, "seq_len": 8192,
                                  "parallelism": f"range-partition dp{world}", "timing": "enqueue mode, one queue",
                                  "device": "gpu"},
                       "extra": extra}, separators=(",", ":"))
    assert len(line) < LINE_LIMIT, len(line)
    out = json.loads(line)["extra"]
    assert out["mandelbrot_4k"]["ms"] > 0 and out["mandelbrot_4k"]["kernel_only"]["pct_fp32_peak_157_3"] > 0
    assert out["load_balance_iters"]["iters"] == 5
    assert out["sgemm"]["gflops_single_queue"] > 0 and out["sgemm"]["tiles_checked"] == 1024
    assert out["task_pool"]["dispatch_tasks_per_s"] > 0
    assert out["nbody_pipeline"]["force_stage_pct_fp32_peak"] > 0
    assert out["pipeline_overlap"]["pipeline_speedup_event"] == 2.1
    assert out["hetero_stream"]["iters_1"]["x_cpu"] > 1
    assert list(out)[-3:] == ["load_balance_iters", "mandelbrot_4k", "sgemm"]


def test_run_child_reports_errors_and_kills_hung_children(tmp_path):
    """The node configs and the peer topology run as children with their own
    time limit: a child that fails or hangs becomes an ``error`` field (the
    headline line is still printed), a hung child's whole process group is
    killed, and the last JSON line of a good child is returned."""
    bench = _bench_module()
    env = bench._child_env()
    good = bench._run_child([sys.executable, "-c", "print('noise'); print('{\"a\": 1}')"], env, 30)
    assert good == {"a": 1}
    bad = bench._run_child([sys.executable, "-c", "import sys; sys.exit(3)"], env, 30)
    assert "exit 3" in bad["error"]
    pidfile = tmp_path / "grandchild.pid"
    hung = [sys.executable, "-c",
            "import subprocess, sys, time; "
            f"p = subprocess.Popen([sys.executable, '-c', 'import time; time.sleep(60)']); "
            f"open({str(pidfile)!r}, 'w').write(str(p.pid)); time.sleep(60)"]
    out = bench._run_child(hung, env, 3)
    assert "error" in out and "Timeout" in out["error"]
    pid = int(pidfile.read_text())
    # the grandchild was in the child's session: killed with it
    import time

    def alive(p):
        try:
            with open(f"/proc/{p}/status") as f:  # a killed, not yet reaped process is a zombie
                return not any(ln.startswith("State:") and "Z" in ln.split()[1] for ln in f)
        except FileNotFoundError:
            return False

    for _ in range(50):
        if not alive(pid):
            break
        time.sleep(0.1)
    else:
        pytest.fail("the hung child's grandchild survived")


def test_wait_for_exit_waits_for_live_ranks_only():
    """Rank 0 starts its timing extras once the other ranks' processes are
    gone (bench._wait_for_exit): it returns at once for PIDs that do not
    exist, waits for a live one, and gives up after its time limit."""
    import time

    bench = _bench_module()
    t = time.time()
    bench._wait_for_exit([2 ** 22 + 12345], timeout_s=5.0)  # no such process
    assert time.time() - t < 1.0
    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(1.0)"])
    t = time.time()
    bench._wait_for_exit([p.pid], timeout_s=10.0)
    waited = time.time() - t
    p.wait()
    assert 0.5 < waited < 8.0, waited
    q = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"])
    try:
        t = time.time()
        bench._wait_for_exit([q.pid], timeout_s=0.5)
        assert 0.4 < time.time() - t < 3.0
    finally:
        q.kill()
        q.wait()
