#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): node GFLOPS of the range-partitioned,
load-balanced bf16 SGEMM 8192³ across N MI355X (one process per GPU), plus the
Mandelbrot 4096² event-pipeline number and the load-balancer convergence
count ("load-balance iters") as extra fields.

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...   (N > 1)

A step is one ``compute()`` of the whole 8192×8192×8192 GEMM through the
framework: the balancer splits the 1024 (or 2048) output tiles across the
ranks, every rank runs the hand-written CDNA4 MFMA kernel on its slice, the
per-device times are exchanged and the next split is computed.  Inputs are
device-resident after the first call and C stays in device memory
(BASELINE.md "device-resident"); the host-resident variant (A/B uploaded and
C slices downloaded each call) is reported separately.  Data: synthetic
uniform [-1, 1) bf16.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

METRIC = "GFLOPS (node) SGEMM-8k + mandelbrot-4k at 1/2/4/8 MI355X; load-balance iters"


def _sync():
    import torch

    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _barrier(ctx):
    if ctx.is_distributed:
        import torch.distributed as dist

        dist.barrier()


def _max_over_ranks(ctx, v: float) -> float:
    if not ctx.is_distributed:
        return v
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device()) if (
        dist.get_backend() == "nccl") else torch.device("cpu")
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _sum_over_ranks(ctx, v: float) -> float:
    if not ctx.is_distributed:
        return v
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device()) if (
        dist.get_backend() == "nccl") else torch.device("cpu")
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def timed(ctx, fn, steps: int, warmup: int, enter=None, leave=None) -> float:
    """W untimed calls, then K timed calls bracketed by barrier + device sync
    on both sides; the max over ranks.  ``enter``/``leave`` run inside the
    timed bracket around the K calls (enqueue mode on/off: leaving drains
    every queue, so all K computes are inside the measurement)."""
    for _ in range(warmup):
        fn()
    _barrier(ctx)
    _sync()
    t0 = time.perf_counter()
    if enter:
        enter()
    for _ in range(steps):
        fn()
    if leave:
        leave()
    _sync()
    # each rank's clock stops once its own device has drained; the closing
    # barrier only lines the ranks up for the max (it is not work)
    ms = (time.perf_counter() - t0) * 1e3 / steps
    _barrier(ctx)
    return _max_over_ranks(ctx, ms)


def _converge(ctx, cr, step, compute_id: int, max_calls: int = 40, stable: int = 5) -> int:
    """Calls ``step`` until the split has not changed for ``stable``
    consecutive calls (identical on every rank: the splits are derived from
    exchanged timings), at most ``max_calls``; returns the calls made."""
    last, same = None, 0
    for n in range(1, max_calls + 1):
        step()
        r = cr.ranges(compute_id)
        same = same + 1 if r == last else 0
        last = r
        if same >= stable:
            return n
    return max_calls


def bench_sgemm(ctx, steps, warmup, size=8192, tile=None):
    from cekirdekler_amd.ops.gemm import GemmBf16
    from cekirdekler_amd.ops.library import library
    from cekirdekler_amd.parallel.distributed import DistributedCruncher

    if tile is None:
        # 256² tiles while every CU still gets one (balanced-DMA ping-pong,
        # ~1.45 PF at 8192³).  Once a GPU's slice has fewer 256² tiles than
        # CUs (8 GPUs × 1024 rows: 128 tiles), the split-K = 2 kernel whose
        # two K-splits exchange row halves through their XCD's L2 keeps every
        # CU busy: 1.22 PF at 1024 rows vs 1.08 for the 256×128 tile on the
        # same box (profiles/gemm_scaling_slices.md)
        tile = "256x256pb" if (size // 256) ** 2 // ctx.world >= 256 else (
            "256x256pby" if (size // 64) % 2 == 0 else "256x128pe")
    from cekirdekler_amd.ops.gemm import GEMM_LIBS

    cr = DistributedCruncher("", ctx=ctx, prebuilt=library(*GEMM_LIBS))
    g = GemmBf16(size, size, size, cruncher=cr, tile=tile)
    step = lambda: g.run(compute_id=1, resident=True)  # noqa: E731
    # Setup (untimed): run the iterative load balancer to convergence — the
    # config is "balancer to convergence" — and bring the clocks up.
    converge = _converge(ctx, cr, step, compute_id=1)
    # Warm-up computes run the load balancer to its split; the K timed
    # computes run in enqueue mode (reference ClNumberCruncher.enqueueMode:
    # no host sync between computes, split frozen, timings gathered when the
    # mode is left) — every step still runs the whole GEMM on every device.
    ms_sync = timed(ctx, step, steps, warmup)  # one host sync + time exchange per compute
    ms = timed(ctx, step, steps, 1,
               enter=lambda: setattr(cr, "enqueue_mode", True),
               leave=lambda: setattr(cr, "enqueue_mode", False))
    host_steps = max(2, min(steps, 5))
    ms_host = timed(ctx, lambda: g.run(compute_id=2, resident=False), host_steps, 1)
    ranges = cr.ranges(1)
    timeouts = g.spin_timeouts()
    if timeouts:
        raise RuntimeError(f"GEMM {tile}: {timeouts} work-groups timed out waiting for their K-split partner")
    cr.dispose()
    for a in (g.A, g.B, g.C, g.dims):
        a.dispose()  # release 0.5 GB of pinned host memory before the next config
    return {"ms": ms, "gflops": g.flops / (ms * 1e-3) / 1e9, "tile": tile, "balancer_setup_calls": converge,
            "sync_per_step_ms": ms_sync, "sync_per_step_gflops": g.flops / (ms_sync * 1e-3) / 1e9,
            "host_resident_ms": ms_host, "host_resident_gflops": g.flops / (ms_host * 1e-3) / 1e9,
            "ranges": ranges}


def bench_mandelbrot(ctx, steps, warmup):
    try:
        from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer
        from cekirdekler_amd.parallel.distributed import DistributedCruncher
        from cekirdekler_amd.ops.library import library
    except Exception as e:  # pragma: no cover
        return {"error": f"unavailable: {e}"}
    cr = DistributedCruncher("", ctx=ctx, prebuilt=library("mandelbrot"))
    m = MandelbrotRenderer(4096, 4096, max_iter=256, cruncher=cr)
    ms = timed(ctx, lambda: m.render(compute_id=3, pipeline=True), max(3, steps // 2), warmup)
    flops = _sum_over_ranks(ctx, m.flops())
    out = {"ms": ms, "gflops": flops / (ms * 1e-3) / 1e9, "flop_per_iter": 8, "kernel": m.kernel,
           "image_pinned": m.out.fast_arr and m.out._fast.pinned}
    cr.dispose()
    return out


def bench_lb_iters():
    """Computes until every device share is within 5% of steady state, on two
    logical devices of this GPU with an injected 2:1 slowdown (the reference
    law converges as 0.7^k)."""
    import cekirdekler_amd as ck

    plats = ck.ClPlatforms.all()
    gpus = plats.gpus()
    devs = (gpus[0] + gpus[0]) if len(gpus) else (plats.cpus(True) + plats.cpus(True))
    # compute-heavy kernel so a device's time is proportional to its range
    # (fixed launch/sync overheads would otherwise bias the steady state)
    src = """__global__ void k(float* x){ long long i = get_global_id(0); float v = x[i];
        for (int j = 0; j < 2048; ++j) v = v * 0.999f + 1.0f; x[i] = v; }"""
    cr = ck.ClNumberCruncher(devs, src)
    cr.cores.serial = True  # logical devices share one GPU: time them in isolation
    cr.set_time_scale(1, 2.0)
    n = 1 << 22
    x = ck.ClArray(n, np.float32)
    x.read = False
    x.write = False
    shares = []
    for _ in range(40):
        x.compute(cr, 7, "k", n, 256)
        r = cr.ranges(7)
        shares.append(r[0] / sum(r))
    steady = shares[-1]
    it = next(i for i in range(len(shares)) if all(abs(s - steady) <= 0.05 * steady for s in shares[i:]))
    cr.dispose()
    return {"iters": it + 1, "steady_share_dev0": steady}


ROOT = os.path.dirname(os.path.abspath(__file__))


def bench_node_configs(world: int) -> dict:
    """BASELINE configs 4 and 5 on this job's GPUs (0 .. world-1), run by
    rank 0 after every other rank has left: the N-body 3-stage
    device→device pipeline (stage transitions over xGMI) and the 256-task
    pool over a device pool.  Both are single-process multi-GPU programs (the
    reference's model), so each runs as a child process with its own time
    limit; a failure is reported in its field and cannot stop the headline."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    out = {}
    for name, script, args in (("nbody_pipeline", "nbody_pipeline.py", ["--pushes", "8"]),
                               ("task_pool", "task_pool.py", [])):
        try:
            r = subprocess.run([sys.executable, script, "--gpus", str(world), *args], cwd=os.path.join(ROOT, "bench"),
                               env=env, capture_output=True, text=True, timeout=180)
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            out[name] = json.loads(lines[-1]) if (r.returncode == 0 and lines) else {
                "error": f"exit {r.returncode}: {(r.stderr or r.stdout)[-300:]}"}
        except Exception as e:  # timeout or parse failure
            out[name] = {"error": repr(e)[:300]}
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--tile", default=None)
    ap.add_argument("--skip-mandelbrot", action="store_true")
    ap.add_argument("--skip-node-configs", action="store_true",
                    help="skip the N-body pipeline and task-pool configs (rank 0, after the headline)")
    args = ap.parse_args(argv)

    from cekirdekler_amd.parallel.distributed import init_distributed

    ctx = init_distributed()
    sg = bench_sgemm(ctx, args.steps, args.warmup, args.size, args.tile)
    mb = {} if args.skip_mandelbrot else bench_mandelbrot(ctx, args.steps, args.warmup)
    lb = bench_lb_iters() if ctx.rank == 0 else {}
    if ctx.is_distributed:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()  # the other ranks exit here; rank 0 goes on alone
    node = {} if (ctx.rank != 0 or args.skip_node_configs) else bench_node_configs(ctx.world)
    if ctx.rank == 0:
        out = {
            "metric": METRIC,
            "value": round(sg["gflops"], 1),
            "unit": "GFLOPS",
            "n_gpus": ctx.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(sg["ms"], 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"model": f"SGEMM {args.size}x{args.size}x{args.size} bf16 (fp32 acc/out), "
                                f"range-partitioned + load-balanced, tile {sg['tile']}",
                       "global_batch": 1, "seq_len": args.size,
                       "parallelism": f"range-partition dp{ctx.world}"},
            "extra": {
                "sgemm_device_resident_gflops": round(sg["gflops"], 1),
                "sgemm_sync_per_step_gflops": round(sg["sync_per_step_gflops"], 1),
                "sgemm_host_resident_gflops": round(sg["host_resident_gflops"], 1),
                "sgemm_host_resident_ms": round(sg["host_resident_ms"], 3),
                "sgemm_ranges": sg["ranges"],
                "mandelbrot_4k": mb,
                "load_balance_iters": lb,
                "nbody_pipeline": node.get("nbody_pipeline"),
                "task_pool": node.get("task_pool"),
            },
        }
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
