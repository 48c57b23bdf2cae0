#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): node GFLOPS of the range-partitioned,
load-balanced bf16 SGEMM 8192³ across N MI355X (one process per GPU), plus the
Mandelbrot 4096² event-pipeline number and the load-balancer convergence
count ("load-balance iters") as extra fields.

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...   (N > 1)

Without a torchrun environment, ``--gpus N > 1`` starts the N rank processes
itself: ``torch.distributed.run`` runs as a child process of this one, which
never imports the runtime or touches a GPU, and this process exits with the
launcher's code (no exec).

A step is one ``compute()`` of the whole 8192×8192×8192 GEMM through the
framework: the balancer splits the 1024 (or 2048) output tiles across the
ranks, every rank runs the hand-written CDNA4 MFMA kernel on its slice, the
per-device times are exchanged and the next split is computed.  Inputs are
device-resident after the first call and C stays in device memory
(BASELINE.md "device-resident"); the host-resident variant (A/B uploaded and
C slices downloaded each call) is reported separately.  Data: synthetic
uniform [-1, 1) bf16.  After the timed loops every rank downloads its device
replica of C and compares EVERY tile of its own range with a float64 product
computed by torch on its GPU (``GemmBf16.verify_full``); the bench exits
non-zero when the relative error exceeds 1e-4 (measured: ~1.5e-6).

Rank 0 prints ONE compact JSON line (< 6 KB, so a log tail keeps it whole):
the headline fields, then ``extra`` with one short summary per config and
the metric's own components LAST (``load_balance_iters``,
``mandelbrot_4k``, ``sgemm``).  Everything measured — per-round arrays,
predictor fits, placements — goes to ``--detail`` (default
``gpurun_out/bench_detail_n{N}.json`` and ``profiles/bench_detail_n{N}.json``).

In a container without a GPU the headline runs a plain kernel-string GEMM on
each rank's CPU device instead (``"device": "cpu"`` in the config): that is
the launcher / control-plane rehearsal the CPU tests use, not a number.
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
        # CUs (8 GPUs × 1024 rows: 128 tiles), the uneven split-K = 2 kernel
        # keeps every CU busy: its helper split runs 4 K-tiles fewer and hands
        # its whole partial over while the owner still multiplies, 1.22 PF at
        # 1024 rows vs 1.18 for the exchanged-halves split and 1.07 for
        # hipBLASLt (fp32 out) on the same box (profiles/gemm_exchange_splitk.md)
        tile = "256x256pb" if (size // 256) ** 2 // ctx.world >= 256 else (
            "256x256pbw" if (size // 64) % 2 == 0 else "256x128pe")
    from cekirdekler_amd.ops.gemm import GEMM_LIBS

    # 4 async enqueue queues per device, one per hardware queue
    # (GPU_MAX_HW_QUEUES=4): 1399 TF/s at 1024 rows against 1376 with 2 and
    # 1329 with 16 on one box (profiles/round4_session4.md)
    cr = DistributedCruncher("", ctx=ctx, prebuilt=library(*GEMM_LIBS), queue_concurrency=4)
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
    ranges = cr.ranges(1)
    # the same computes once more with dispatch-stamped kernel times: the
    # GEMM kernel alone, without the gap between back-to-back launches that
    # the per-step time includes (informative; not the headline)
    cr.record_kernel_times = True
    cr.enqueue_mode = True
    for _ in range(steps):
        step()
    cr.enqueue_mode = False
    cr.record_kernel_times = False
    kt = sorted(t for name, t in cr.kernel_times(0) if name.startswith("cek_sgemm"))
    kernel_ms = _max_over_ranks(ctx, kt[len(kt) // 2] if kt else 0.0)
    # the benchmarked output itself: EVERY tile of this rank's C replica
    # against a float64 product on its GPU (before the host-resident run
    # below re-splits compute id 2 and overwrites the host copy)
    err, tiles_checked = g.verify_full(compute_id=1)
    err = _max_over_ranks(ctx, err)
    tiles_checked = int(_sum_over_ranks(ctx, tiles_checked))
    # owners that found their split-K helper late and multiplied its K-range
    # themselves (C correct either way; nonzero = a shared GPU)
    fallbacks = int(_sum_over_ranks(ctx, g.handover_fallbacks()))
    # The same K computes on async enqueue queues (reference
    # enqueueModeAsyncEnable, Cores.cs:80-83 and :858-935: each compute goes
    # to the next of the device's queues, with no order between them):
    # consecutive GEMMs overlap on the
    # GPU, so the CUs that finish a launch's tiles early start the next
    # launch's instead of idling through its tail.  Every step still computes
    # the whole GEMM.  A slice with fewer tiles than CUs then needs no
    # split-K: two launches in flight fill the chip with whole tiles.
    # Split-K tiles cannot run this way (their partial-tile workspace is
    # per GEMM), so a split-K bench tile gets a single-pass twin here.
    ga, cid_a = (g, 1) if g.split_k == 1 else (GemmBf16(size, size, size, cruncher=cr, tile="256x256pb"), 5)
    step_a = lambda: ga.run(compute_id=cid_a, resident=True)  # noqa: E731
    converge_a = _converge(ctx, cr, step_a, compute_id=cid_a) if cid_a != 1 else 0

    def enter_async():
        cr.enqueue_mode = True
        cr.enqueue_mode_async_enable = True

    def leave_async():
        cr.enqueue_mode = False
        cr.enqueue_mode_async_enable = False

    # untimed: one pass over every async queue, so the queues' HIP streams
    # exist before the timed loop (creating one costs ~1 ms)
    enter_async()
    for _ in range(cr.compute_queue_concurrency + 1):
        step_a()
    leave_async()
    ms_async = timed(ctx, step_a, steps, 0, enter=enter_async, leave=leave_async)
    err_async, tiles_async = ga.verify_full(compute_id=cid_a)
    err_async = _max_over_ranks(ctx, err_async)
    tiles_async = int(_sum_over_ranks(ctx, tiles_async))
    if ga is not g:
        for a in (ga.A, ga.B, ga.C, ga.dims):
            a.dispose()
    host_steps = max(2, min(steps, 5))
    # host-resident: A and B uploaded and C downloaded on every call, through
    # the event-driven read/compute/write pipeline in 8 blobs (B a full
    # read, A row panels and C tiles streamed; profiles/hostres_streaming.md).
    # Falls back to the serial 3-phase path when the tile cannot stream.
    # a blob holds whole tile groups (A row panels), and the runtime pipelines
    # only when every rank's range splits into whole blobs: at N ranks each
    # holds groups/N of them
    groups = (g.M // g.BM) // max(1, g.group_m)
    blobs = max(1, min(HOST_RESIDENT_BLOBS, groups // ctx.world)) if g.can_stream() else 0
    host_calls = []

    host_piped = []

    def host_step():
        t = time.perf_counter()
        g.run(compute_id=2, resident=False, stream_blobs=blobs)
        host_calls.append((time.perf_counter() - t) * 1e3)
        host_piped.append(cr.last_record()["pipelined"])

    ms_host = timed(ctx, host_step, host_steps, 2)
    # the streamed host-resident output: this rank's tiles of the host C
    err_host = _max_over_ranks(ctx, g.verify_full(compute_id=2, host=True)[0])
    ms_blobs, mode = ms_host, f"compute() event pipeline, {blobs} equal blobs" if blobs else "compute() serial 3-phase"
    ms_shells = ms_native_shells = ms_shells_cu = None
    panels = HOST_RESIDENT_PANELS
    if ctx.world == 1 and g.split_k == 1 and size % panels == 0 and (size // panels) % max(g.BM, g.BN) == 0:
        # one GPU holds the whole problem: the square-shell stream through
        # compute() — the event pipeline with explicit, uneven blobs (blob s =
        # shell s; A and B go up one row panel per blob), whose first kernels
        # need two panels instead of all of B
        ms_shells = timed(ctx, lambda: g.run_shells(panels, compute_id=3), host_steps, 2)
        err_shells = g.verify_full(compute_id=3, host=True)[0]
        err_host = max(err_host, err_shells)
        if ms_shells < ms_host:
            ms_host, mode = ms_shells, f"compute() event pipeline, {panels} shell blobs"
        # the same with downloads by a copy kernel on CUs reserved for it
        # (CU-masked streams): the downloads never wait for a GEMM
        # work-group to leave a CU, so they run beside the SDMA uploads
        try:
            cr.copy_cus, cr.kernel_d2h = HOST_RESIDENT_COPY_CUS, True
            ms_shells_cu = timed(ctx, lambda: g.run_shells(panels, compute_id=4), host_steps, 2)
            err_host = max(err_host, g.verify_full(compute_id=4, host=True)[0])
        finally:
            cr.kernel_d2h, cr.copy_cus = False, 0
        if ms_shells_cu < ms_host:
            ms_host, mode = ms_shells_cu, (f"compute() event pipeline, {panels} shell blobs, downloads by a copy "
                                           f"kernel on {HOST_RESIDENT_COPY_CUS} reserved CUs")
        # the same schedule through its dedicated native entry point, for comparison
        ms_native_shells = timed(ctx, lambda: g.run_host_shells(panels), host_steps, 2)
        err_host = max(err_host, g.verify_shells_full(panels)[0])
    cr.dispose()
    for a in (g.A, g.B, g.C, g.dims):
        a.dispose()  # release 0.5 GB of pinned host memory before the next config
    single = {"ms": ms, "gflops": g.flops / (ms * 1e-3) / 1e9, "tile": tile, "max_rel_err": err,
              "tiles_checked": tiles_checked}
    overlapped = {"ms": ms_async, "gflops": g.flops / (ms_async * 1e-3) / 1e9, "tile": ga.tile,
                  "max_rel_err": err_async, "tiles_checked": tiles_async, "balancer_setup_calls": converge_a}
    # headline: the latency of ONE GEMM at a time (one queue, each compute
    # drains before the next starts on the device) — the strong-scaled
    # number.  The async-queue schedule overlaps
    # consecutive GEMMs: throughput of back-to-back GEMMs, reported beside
    # it as sgemm.gflops_async_queues, never as the headline.
    best = single
    timing = "enqueue mode, one queue (one GEMM in flight)"
    return {"ms": best["ms"], "gflops": best["gflops"], "tile": best["tile"], "timing": timing,
            "single_queue": single, "async_queues": overlapped, "balancer_setup_calls": converge,
            "sync_per_step_ms": ms_sync, "sync_per_step_gflops": g.flops / (ms_sync * 1e-3) / 1e9,
            "host_resident_ms": ms_host, "host_resident_gflops": g.flops / (ms_host * 1e-3) / 1e9,
            "host_resident_blobs": blobs, "host_resident_calls_ms": [round(x, 3) for x in host_calls],
            "host_resident_pipelined": host_piped, "host_resident_mode": mode,
            "host_resident_blob_pipeline_ms": ms_blobs, "host_resident_shells_ms": ms_shells,
            "host_resident_native_shells_ms": ms_native_shells, "host_resident_shells_copy_cus_ms": ms_shells_cu,
            "ranges": ranges, "max_rel_err": max(err, err_async, err_host), "max_rel_err_host_resident": err_host,
            "tiles_checked": tiles_checked, "tiles_total": g.tiles,
            "kernel_ms": kernel_ms, "kernel_gflops": g.flops / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else None,
            "handover_fallbacks": fallbacks, "device": "gpu"}


CPU_GEMM_SRC = """
__global__ void gemm_nt(const int* d, const float* a, const float* b, float* c) {
  long long i = get_global_id(0);
  int n = d[1], k = d[2];
  long long r = i / n, col = i % n;
  float s = 0.0f;
  for (int j = 0; j < k; ++j) s += a[r * k + j] * b[col * k + j];
  c[i] = s;
}
"""


def bench_sgemm_cpu(ctx, steps, warmup, size=256):
    """GPU-less rehearsal of the headline: the same range-partitioned,
    balanced compute() over one CPU device per rank (plain fp32 kernel
    string, one work item per output element, C device-resident after the
    first call).  Exercises the rank launcher, the shared-memory control
    plane and the identical-split property, not the MI355X kernel."""
    import cekirdekler_amd as ck
    from cekirdekler_amd.parallel.distributed import DistributedCruncher

    cr = DistributedCruncher(CPU_GEMM_SRC, ctx=ctx, devices=ck.ClPlatforms.all().cpus(True))
    rng = np.random.default_rng(0)
    dims = ck.ClArray(np.array([size, size, size, 0], np.int32))
    a = ck.ClArray(rng.uniform(-1, 1, size * size).astype(np.float32))
    b = ck.ClArray(rng.uniform(-1, 1, size * size).astype(np.float32))
    c = ck.ClArray(np.zeros(size * size, np.float32))
    for x in (dims, a, b):
        x.write = False
    c.read = False
    n, local = size * size, 64

    def step():
        dims.next_param(a, b, c).compute(cr, 1, "gemm_nt", n, local)

    converge = _converge(ctx, cr, step, compute_id=1)
    ms = timed(ctx, step, steps, warmup)
    ranges = cr.ranges(1)
    lo = cr.references(1)[ctx.rank]
    hi = lo + ranges[ctx.rank]
    ref = (a.array.reshape(size, size).astype(np.float64) @ b.array.reshape(size, size).astype(np.float64).T).ravel()
    err = float(np.max(np.abs(c.array[lo:hi] - ref[lo:hi])) / max(np.max(np.abs(ref)), 1e-30)) if hi > lo else 0.0
    err = _max_over_ranks(ctx, err)
    cr.dispose()
    flops = 2.0 * size ** 3
    return {"ms": ms, "gflops": flops / (ms * 1e-3) / 1e9, "tile": "cpu-naive", "balancer_setup_calls": converge,
            "sync_per_step_ms": ms, "sync_per_step_gflops": flops / (ms * 1e-3) / 1e9,
            "host_resident_ms": ms, "host_resident_gflops": flops / (ms * 1e-3) / 1e9,
            "ranges": ranges, "max_rel_err": err, "handover_fallbacks": 0, "device": "cpu",
            "tiles_checked": size * size, "tiles_total": size * size}


def _all_ranges(ctx, ranges):
    """Every rank's view of the split (they must be identical: each rank
    derives it from the same exchanged timings)."""
    if not ctx.is_distributed:
        return [list(ranges)]
    import torch.distributed as dist

    out = [None] * ctx.world
    dist.all_gather_object(out, list(ranges))
    return out


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
           "image_pinned": m.out.pinned}
    cr.dispose()
    if ctx.rank == 0:
        try:  # an extra: a failure is reported in its field, never stops the headline
            out["kernel_only"] = _mandelbrot_kernel_only()
        except Exception as e:  # pragma: no cover
            out["kernel_only"] = {"error": repr(e)[:300]}
    return out


def _row_major_comparison(steps: int) -> dict:
    """Like-for-like layout check: the headline kernel with a
    row-major C epilogue (``256x256pbr``) at 8192³ through compute() in
    enqueue mode, and hipBLASLt (torch.mm, bf16 in, fp32 out, row-major C)
    at the same shape on the same GPU, each the median of 5 timed runs."""
    import statistics

    import torch

    import cekirdekler_amd as ck
    from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16
    from cekirdekler_amd.ops.library import library

    size = 8192
    flops = 2.0 * size ** 3
    cr = ck.ClNumberCruncher(ck.ClPlatforms.all().gpus()[0], "", prebuilt=library(*GEMM_LIBS))
    g = GemmBf16(size, size, size, cruncher=cr, tile="256x256pbr")
    g.run(compute_id=1, resident=True)
    runs = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cr.enqueue_mode = True
        for _ in range(steps):
            g.run(compute_id=1, resident=True)
        cr.enqueue_mode = False
        torch.cuda.synchronize()
        runs.append((time.perf_counter() - t0) / steps)
    err, tiles = g.verify_full(compute_id=1)
    cr.dispose()
    for arr in (g.A, g.B, g.C, g.dims):
        arr.dispose()
    out = {"tile": "256x256pbr", "gflops": round(flops / statistics.median(runs) / 1e9, 1), "max_rel_err": err,
           "tiles_checked": tiles}
    try:
        a = torch.randn(size, size, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(size, size, device="cuda", dtype=torch.bfloat16).T
        for _ in range(3):
            c = torch.mm(a, b, out_dtype=torch.float32)
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                c = torch.mm(a, b, out_dtype=torch.float32)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / steps)
        out["hipblaslt_fp32_out_gflops"] = round(flops / statistics.median(ts) / 1e9, 1)
        out["vs_hipblaslt"] = round(out["gflops"] / out["hipblaslt_fp32_out_gflops"], 4)
        del a, b, c
        torch.cuda.empty_cache()
    except Exception as e:  # pragma: no cover
        out["hipblaslt_error"] = repr(e)[:200]
    return out


def _mandelbrot_kernel_only(kernel: str = "blk8y", reps: int = 40) -> dict:
    """The fastest Mandelbrot kernel alone on this rank's GPU (image left in
    device memory, no D2H, calls enqueued back to back in enqueue mode):
    BASELINE's "kernel >= 50 % of FP32 peak" target.
    The end-to-end number above is PCIe-bound and runs blk8 (the kernel does
    not change it, tools/mandel_ab_probe.py).

    Two numbers: ``ms`` renders one image over and over on one stream (each
    launch drains before the next starts); ``frames_in_flight_2`` renders
    two images alternately in the reference's async enqueue mode
    (enqueueModeAsyncEnable over 2 queues): the two frames' launches run side
    by side, so the SIMDs stay full through each launch's ramp-up and drain
    (double-buffered frames of an animation; every frame is computed whole,
    tools/mandel_async_probe.py, profiles/mandelbrot_r3.md)."""
    import torch

    from cekirdekler_amd.models.mandelbrot import MandelbrotRenderer
    from cekirdekler_amd.ops.library import library
    import cekirdekler_amd as ck

    gpus = ck.ClPlatforms.all().gpus()
    cr = ck.ClNumberCruncher(gpus[0], "", prebuilt=library("mandelbrot"), queue_concurrency=2)
    ms = [MandelbrotRenderer(4096, 4096, max_iter=256, cruncher=cr, kernel=kernel) for _ in range(2)]
    for i, m in enumerate(ms):
        m.render(i + 1, pipeline=False)  # image downloaded once: its counts give the FLOPs
    flops = ms[0].flops()
    for m in ms:
        m.out.write = False

    def batch(frames_in_flight: int) -> float:
        """One timed run of `reps` calls enqueued back to back (no host sync
        per call), ms per call."""
        cr.enqueue_mode_async_enable = frames_in_flight > 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cr.enqueue_mode = True
        for k in range(reps):
            ms[k % frames_in_flight].render(k % frames_in_flight + 1, pipeline=False)
        cr.enqueue_mode = False
        torch.cuda.synchronize()
        cr.enqueue_mode_async_enable = False
        return (time.perf_counter() - t0) * 1e3 / reps

    for k in range(500):  # ~45 ms: the clock settles (the first runs read up to 10 % slower)
        ms[0].render(1, pipeline=False)
    batch(2)
    # 9 rounds, the two modes taking turns (clock drift hits both alike);
    # each mode's median
    runs = {1: [], 2: []}
    for _ in range(9):
        for f in (1, 2):
            runs[f].append(batch(f))

    def summary(runs):
        ms_ = sorted(runs)[len(runs) // 2]
        tf = flops / (ms_ * 1e-3) / 1e12
        return {"ms": round(ms_, 4), "ms_runs": [round(x, 4) for x in runs], "tflops": round(tf, 2),
                "pct_fp32_peak_157_3": round(100 * tf / 157.3, 1)}

    out = {"kernel": ms[0].kernel, **summary(runs[1])}
    # the same launches with dispatch-stamped start/stop events: each
    # kernel's own execution time, without the gap between back-to-back
    # launches that the wall-clock number above includes
    cr.record_kernel_times = True
    cr.enqueue_mode = True
    for k in range(reps):
        ms[0].render(1, pipeline=False)
    cr.enqueue_mode = False
    cr.record_kernel_times = False
    kt = sorted(t for name, t in cr.kernel_times(0) if "mandelbrot" in name)
    if kt:
        kt_ms = kt[len(kt) // 2]
        out["kernel_timestamps"] = {"ms": round(kt_ms, 4), "launches": len(kt),
                                    "pct_fp32_peak_157_3": round(100 * flops / (kt_ms * 1e-3) / 1e12 / 157.3, 1)}
    two = summary(runs[2])
    # both device images (last written by the overlapped frames) are whole
    # and equal to the image downloaded before the timed runs
    ref = ms[0].out.array.copy()
    equal = True
    for m in ms:
        m.out.array[:] = -1
        cr.download(m.out, 0)
        equal = equal and bool((m.out.array == ref).all())
    two["images_equal"] = equal
    out["frames_in_flight_2"] = two
    cr.dispose()
    return out


def bench_sgemm_slices(steps: int, rows=(4096, 2048, 1024), size: int = 8192) -> dict:
    """The per-GPU share of the strongly scaled headline, measured on this
    GPU: at N = 2 / 4 / 8 GPUs a rank computes 4096 /
    2048 / 1024 rows of the 8192³ GEMM.  Each slice runs as bench_sgemm
    times it (one GEMM in flight, enqueue mode, the tile bench_sgemm picks
    at that N) and its whole output is checked against a float64 product."""
    import torch

    from cekirdekler_amd.ops.gemm import GEMM_LIBS, GemmBf16
    from cekirdekler_amd.ops.library import library
    import cekirdekler_amd as ck

    gpu = ck.ClPlatforms.all().gpus()[0]
    out = {}
    for m in rows:
        tile = "256x256pb" if (m // 256) * (size // 256) >= 256 else "256x256pbw"
        cr = ck.ClNumberCruncher(gpu, "", prebuilt=library(*GEMM_LIBS))
        g = GemmBf16(m, size, size, cruncher=cr, tile=tile)
        # warm-up until the clocks have settled: the first rounds after a
        # new GEMM object run up to 12 % slow (rounds of one process:
        # 1278 → 1469 TF/s at 4096 rows, profiles/r6/README.md)
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < SLICE_WARMUP_S:
            for _ in range(10):
                g.run(compute_id=1, resident=True)
            torch.cuda.synchronize()
        rounds = []
        for _ in range(SLICE_ROUNDS):  # the median round: one cold round cannot set the number
            torch.cuda.synchronize()
            cr.enqueue_mode = True
            t0 = time.perf_counter()
            for _ in range(steps):
                g.run(compute_id=1, resident=True)
            cr.enqueue_mode = False
            torch.cuda.synchronize()
            rounds.append((time.perf_counter() - t0) * 1e3 / steps)
        ms = sorted(rounds)[len(rounds) // 2]
        rounds_tf = [round(g.flops / r / 1e9, 1) for r in rounds]
        err, tiles = g.verify_full(compute_id=1)
        out[str(m)] = {"tflops": round(g.flops / ms / 1e9, 1), "ms": round(ms, 4), "tile": tile, "rounds_tflops": rounds_tf,
                       "max_rel_err": err, "tiles_checked": tiles, "tiles_total": g.tiles,
                       "handover_fallbacks": g.handover_fallbacks()}
        cr.dispose()
        for a in (g.A, g.B, g.C, g.dims, *g.extra):
            a.dispose()
    return out


def bench_lb_iters():
    """Computes until device 0's share stays within 5% of its steady state
    (the median of the last 10 of 40 calls), on two logical devices of this
    GPU with an injected 2:1 slowdown (the reference law converges as 0.7^k;
    SURVEY §7.4 item 3).  Run by rank 0 alone after the other ranks have
    left, so no other process shares the host or the GPU
    (``parallel.balancer.measure_lb_convergence``; the whole trajectory goes
    to the detail file)."""
    import cekirdekler_amd as ck
    from cekirdekler_amd.parallel.balancer import measure_lb_convergence

    plats = ck.ClPlatforms.all()
    gpus = plats.gpus()
    devs = (gpus[0] + gpus[0]) if len(gpus) else (plats.cpus(True) + plats.cpus(True))
    return measure_lb_convergence(devs, calls=40, slow_device=1, slowdown=2.0)


ROOT = os.path.dirname(os.path.abspath(__file__))


def _child_env() -> dict:
    """This environment without the rank variables: a child program is a
    job of its own (or starts its own torchrun)."""
    return {k: v for k, v in os.environ.items()
            if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                         "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}


def _run_child(cmd, env, timeout: float) -> dict:
    """Run one bench/ program as a child process in its own session and
    return the last JSON line it printed; a failure or a timeout (which
    kills the whole process group, torchrun's ranks too) is reported in the
    returned dict instead."""
    p = subprocess.Popen(cmd, cwd=os.path.join(ROOT, "bench"), env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True, start_new_session=True)
    try:
        so, se = p.communicate(timeout=timeout)
        lines = [ln for ln in so.splitlines() if ln.startswith("{")]
        return json.loads(lines[-1]) if (p.returncode == 0 and lines) else {
            "error": f"exit {p.returncode}: {(se or so)[-300:]}"}
    except Exception as e:  # timeout or parse failure
        try:
            os.killpg(p.pid, 9)
        except OSError:
            pass
        p.communicate()
        return {"error": repr(e)[:300]}


def bench_node_configs(world: int) -> dict:
    """BASELINE configs 4 and 5 on this job's GPUs (0 .. world-1), run by
    rank 0 after every other rank has left: the N-body 3-stage
    device→device pipeline (stage transitions over xGMI) and the 256-task
    pool over a device pool; plus config 1, SAXPY 1M on the CPU device, the
    wave example and CPU + GPU co-execution on host-resident data.  They are
    single-process programs (the reference's model), so each runs as a child
    process with its own time limit; a failure is reported in its field and
    cannot stop the headline."""
    env = _child_env()
    out = {}
    rccl = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
            "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "rccl_gemm.py",
            "--expect-world", str(world)]
    import torch

    # config 4 is specified on 4 GPUs (2 + 1 + 1 placement); on fewer GPUs the
    # same placement is rehearsed on 4 logical devices of GPU 0
    nb_args = ["--gpus", str(min(world, 4))] if world >= 4 else ["--gpus", "4", "--logical", "4"]
    configs = [("nbody_pipeline", [sys.executable, "nbody_pipeline.py", *nb_args, "--pushes", "14"]),
               ("task_pool", [sys.executable, "task_pool.py", "--gpus", str(world)]),
               ("saxpy_1m_cpu", [sys.executable, "saxpy_cpu.py"]),
               ("wave_cpu_gpu", [sys.executable, "wave_cpu_gpu.py"])]
    if world <= torch.cuda.device_count():
        configs.append(("sgemm_host_resident_rccl", rccl))
    else:
        # a launcher rehearsal with ranks sharing a GPU: RCCL refuses two
        # ranks on one device
        out["sgemm_host_resident_rccl"] = {"skipped": f"{world} ranks on {torch.cuda.device_count()} GPU(s); "
                                                      "RCCL needs one GPU per rank"}
    configs.append(("hetero_stream", [sys.executable, "hetero_stream.py"]))
    # the reference's read/compute/write overlap claim on a balanced workload
    configs.append(("pipeline_overlap", [sys.executable, "pipeline_overlap.py"]))
    # the reference's async-queue timeline: four independent computes on the
    # async enqueue queues against one at a time
    configs.append(("async_queues", [sys.executable, "async_queues.py"]))
    # xGMI fan-out vs per-GPU uploads of read arrays, by size
    configs.append(("broadcast_threshold", [sys.executable, "broadcast_threshold.py", "--gpus", str(world)]))
    t_start = time.monotonic()
    for name, cmd in configs:
        # the extras share one time budget, so a hung config cannot push the
        # whole run (headline included) past the driver's limit
        left = NODE_CONFIGS_BUDGET_S - (time.monotonic() - t_start)
        if left < 30:
            out[name] = {"skipped": f"node-config time budget ({NODE_CONFIGS_BUDGET_S} s) spent"}
            continue
        out[name] = _run_child(cmd, env, min(180, left))
    return out


SLICE_ROUNDS = 5  # bench_sgemm_slices: timed rounds per slice (median)
SLICE_WARMUP_S = 0.3  # bench_sgemm_slices: untimed GEMMs per slice before timing
MAX_REL_ERR = 1e-4  # bf16 inputs, fp32 accumulation: measured ~1.5e-6 relative to max |ref| per tile
NODE_CONFIGS_BUDGET_S = 360  # all of bench_node_configs' child processes together
PEER_TOPOLOGY_TIMEOUT_S = 90
HOST_RESIDENT_BLOBS = 8
HOST_RESIDENT_PANELS = 16
HOST_RESIDENT_COPY_CUS = 8


def write_detail(full: dict, world: int, path=None, gpu: bool = True) -> str:
    """Everything the run measured, as one JSON file (the printed line only
    summarises it): ``path``, else ``gpurun_out/bench_detail_n{N}.json`` and,
    for a GPU run, ``profiles/bench_detail_n{N}.json``.  Returns the path the
    line cites."""
    paths = [path] if path else [os.path.join(ROOT, "gpurun_out", f"bench_detail_n{world}.json")] + (
        [os.path.join(ROOT, "profiles", f"bench_detail_n{world}.json")] if gpu else [])
    written = None
    for p in paths:
        try:
            os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
            with open(p, "w") as f:
                json.dump(full, f, indent=1, default=str)
            written = written or os.path.relpath(p, ROOT)
        except OSError:
            pass
    return written or ""


def _r(x, nd=3):
    """Round a number for the summary line: ints and non-numbers pass, small
    magnitudes (errors) keep 3 significant digits."""
    if isinstance(x, (bool, int)) or not isinstance(x, float):
        return x
    if x != 0 and abs(x) < 0.1:
        return float(f"{x:.3g}")
    return round(x, nd)


def _pick(d, keys, nd=3):
    """{key: rounded value} for the keys of ``d`` that exist (an error or
    skip note passes through whole, cut to 160 characters)."""
    if not isinstance(d, dict):
        return d
    if "error" in d or "skipped" in d:
        return {k: str(d[k])[:160] for k in ("error", "skipped") if k in d}
    return {k: _r(d[k], nd) for k in keys if k in d}


def compact_extra(full: dict, detail: str) -> dict:
    """The printed line's ``extra``: one short summary per config, with the
    headline metric's own components last (load-balance iters,
    Mandelbrot-4k, SGEMM), so even a truncated log keeps them (VERDICT r4
    next #1).  ``full`` is what :func:`write_detail` writes."""
    ex = {"detail_file": detail}
    peers = full.get("peer_topology") or {}
    if "error" in peers:
        ex["peer"] = _pick(peers, [])
    elif peers:
        bw = peers.get("bandwidth") or {}
        same = (bw.get("same_gpu") or {}).get("sdma") or {}
        pairs = bw.get("pairs") or []
        ex["peer"] = {"gpus_visible": peers.get("gpus_visible"), "path": peers.get("path"),
                      "same_gpu_sdma_gbps": _r(same.get("gbps"), 1),
                      "pair_gbps_max": _r(max((q.get("gbps", 0) for q in pairs if isinstance(q, dict)), default=None), 1),
                      "all_verified": bw.get("all_verified")}
    if full.get("sgemm_host_resident_rccl") is not None:
        ex["rccl_host_resident"] = _pick(full["sgemm_host_resident_rccl"],
                                         ["ranks", "split_reads_ms", "max_rel_err_split_reads",
                                          "max_rel_err_gathered_replicas"], 7)
    hs = full.get("hetero_stream")
    if isinstance(hs, dict):
        if "error" in hs or "skipped" in hs:
            ex["hetero_stream"] = _pick(hs, [])
        else:
            ex["hetero_stream"] = {k: {**{c: _r((v.get(c) or {}).get("ms")) for c in ("cpu", "gpu", "gpu+cpu", "gpu+cpu_fit")
                                           if isinstance(v.get(c), dict)},
                                       "x_cpu": _r(v.get("speedup_over_cpu")), "x_gpu": _r(v.get("speedup_over_gpu"))}
                                   for k, v in hs.items() if k.startswith("iters_") and isinstance(v, dict)}
    wv = full.get("wave_cpu_gpu")
    if isinstance(wv, dict):
        w = _pick(wv, ["reference_cpu_ms_per_frame", "cpu_ms_per_frame", "gpu_ms_per_frame", "gpu+cpu_ms_per_frame",
                       "gpu+cpu_fit_ms_per_frame", "speedup_gpu+cpu_over_reference_cpu",
                       "speedup_gpu_over_reference_cpu", "speedup_gpu+cpu_over_cpu", "speedup_gpu_over_cpu",
                       "speedup_gpu+cpu_fit_over_cpu"], 4)
        pred = wv.get("gpu+cpu_fit_predictor")
        if isinstance(pred, dict):
            w["fit_decision"] = pred.get("decision")
        ex["wave_cpu_gpu"] = w
    if full.get("saxpy_1m_cpu") is not None:
        ex["saxpy_1m_cpu"] = _pick(full["saxpy_1m_cpu"], ["ms", "GBps", "bit_exact_vs_numpy"], 4)
    po = full.get("pipeline_overlap")
    if isinstance(po, dict):
        p = _pick(po, ["read_compute_write_ms", "ideal_speedup_sum_over_max", "pipeline_speedup_event",
                       "pipeline_speedup_driver", "pipeline_speedup_driver_in_queue",
                       "pipeline_speedup_driver_reads_in_queue", "best_event", "best_event_4streams", "default_compute_streams",
                       "best_driver_default", "best_driver_q4", "best_driver_q16", "event_5_vs_4_streams",
                       "driver_default_q4_q16", "outputs_exact", "lcg_iters"])
        if isinstance(po.get("ms"), dict):
            p["3phase_ms"] = po["ms"].get("3phase")
        ex["pipeline_overlap"] = p
    aq = full.get("async_queues")
    if isinstance(aq, dict):
        ex["async_queues"] = _pick(aq, ["compute_streams", "ms_per_round_of_4", "async_speedup_over_sync",
                                        "deferred_vs_inorder", "outputs_checked"])
    bt = full.get("broadcast_threshold")
    if isinstance(bt, dict):
        ex["broadcast_threshold"] = _pick(bt, ["devices", "logical", "crossover_bytes", "runtime_adopted_min_bytes",
                                               "sizes", "direct_ms", "staged_ms", "exact"], 4)
    tp = full.get("task_pool")
    if isinstance(tp, dict):
        t = _pick(tp, ["tasks", "pool_devices", "cu_partitioned", "makespan_ms", "ideal_ms_sum_over_devices",
                       "makespan_over_ideal", "makespan_over_ideal_cu_partitioned", "dispatch_tasks_per_s", "host_us_per_task", "median_task_device_us",
                       "serial_group_in_order", "gemm_task_max_rel_err", "reduce_task_rel_err"])
        rr = tp.get("round_robin")
        if isinstance(rr, dict):
            t["round_robin_makespan_over_ideal"] = _r(rr.get("makespan_over_ideal"))
        cs = tp.get("concurrent_spans")
        if isinstance(cs, dict):
            t["makespan_over_concurrent_ideal"] = _r(cs.get("makespan_over_ideal"))
            t["contention_factor"] = _r(cs.get("contention_factor"))
        t["makespan_over_greedy_sim"] = _r(tp.get("makespan_over_greedy_sim"))
        pj = tp.get("projected_8gpu")
        if isinstance(pj, dict):
            t["projected_8gpu_makespan_over_ideal"] = _r(pj.get("makespan_over_ideal"))
            t["projected_8gpu_serial_host_over_ideal"] = _r(pj.get("makespan_serial_host_over_ideal"))
            t["dispatch_tasks_per_s_one_device"] = pj.get("dispatch_tasks_per_s_one_device")
            t["dispatch_tasks_per_s_8_logical_whole_gpu"] = pj.get("dispatch_tasks_per_s_8_whole_gpu_logical_devices")
            sb = pj.get("schedule_bounds") or {}
            t["projected_8gpu_fifo_zero_host_cost"] = _r(sb.get("fifo_no_host_cost"))
            t["projected_8gpu_lpt_zero_host_cost"] = _r(sb.get("lpt_no_host_cost"))
            t["projected_8gpu_without_barrier_task"] = _r(pj.get("makespan_no_barrier_over_ideal"))
        ex["task_pool"] = t
    nb = full.get("nbody_pipeline")
    if isinstance(nb, dict):
        n = _pick(nb, ["n", "gpus_used", "cu_partitioned", "push_ms_median", "force_stage_pct_fp32_peak",
                       "min_device_busy_fraction", "device_busy_fraction", "overlap_efficiency",
                       "step_check_max_rel_err"], 4)
        co = nb.get("copy_overlap")
        if isinstance(co, dict):
            n["copy_overlap_with_force"] = co.get("with_force_stage")
        ex["nbody_pipeline"] = n
    # ---- the headline metric's components, last ----
    lb = full.get("load_balance_iters") or {}
    ex["load_balance_iters"] = _pick(lb, ["iters", "steady_share_dev0", "calls"], 4) if lb else None
    mb = full.get("mandelbrot_4k") or {}
    if mb:
        m = _pick(mb, ["ms", "gflops", "kernel"], 4)
        ko = mb.get("kernel_only")
        if isinstance(ko, dict):
            m["kernel_only"] = _pick(ko, ["kernel", "ms", "pct_fp32_peak_157_3"], 4)
            kts = ko.get("kernel_timestamps")
            if isinstance(kts, dict):
                m["kernel_only"]["pct_kernel_timestamps"] = kts.get("pct_fp32_peak_157_3")
            two = ko.get("frames_in_flight_2")
            if isinstance(two, dict):
                m["kernel_only"]["pct_2_frames"] = two.get("pct_fp32_peak_157_3")
                m["kernel_only"]["images_equal"] = two.get("images_equal")
        ex["mandelbrot_4k"] = m
    else:
        ex["mandelbrot_4k"] = None
    sl = full.get("sgemm_slices") or {}
    if isinstance(sl, dict) and sl:
        if "error" in sl:
            ex["sgemm_slices"] = _pick(sl, [])
        else:  # TF/s per slice (rows), the worst error over all of them
            ex["sgemm_slices"] = {k: v.get("tflops") for k, v in sl.items() if isinstance(v, dict)}
            ex["sgemm_slices"]["max_rel_err"] = _r(max((v.get("max_rel_err", 0) for v in sl.values()
                                                        if isinstance(v, dict)), default=None), 9)
            ex["sgemm_slices"]["all_tiles_checked"] = all(v.get("tiles_checked") == v.get("tiles_total")
                                                          for v in sl.values() if isinstance(v, dict))
    sg = full.get("sgemm") or {}
    rc = full.get("sgemm_row_major_c") or {}
    all_ranges = full.get("sgemm_ranges_all_ranks") or [sg.get("ranges")]
    sq, aq = sg.get("single_queue") or {}, sg.get("async_queues") or {}
    ex["sgemm"] = {
        "gflops_single_queue": _r(sq.get("gflops"), 1), "gflops_async_queues": _r(aq.get("gflops"), 1),
        "gflops_sync_per_step": _r(sg.get("sync_per_step_gflops"), 1),
        "kernel_ms": _r(sg.get("kernel_ms"), 4), "gflops_kernel_timestamps": _r(sg.get("kernel_gflops"), 1),
        "tile": sg.get("tile"), "ranges": sg.get("ranges"),
        "ranges_identical_on_all_ranks": all(r == all_ranges[0] for r in all_ranges),
        "balancer_setup_calls": sg.get("balancer_setup_calls"),
        "max_rel_err_full": _r(sg.get("max_rel_err"), 9),
        "tiles_checked": sg.get("tiles_checked"), "tiles_total": sg.get("tiles_total"),
        "host_resident_ms": _r(sg.get("host_resident_ms")),
        "host_resident_mode": sg.get("host_resident_mode"),
        "host_resident_max_rel_err": _r(sg.get("max_rel_err_host_resident"), 9),
        "row_major_c_gflops": _r(rc.get("gflops"), 1), "hipblaslt_fp32_out_gflops": rc.get("hipblaslt_fp32_out_gflops"),
        "vs_hipblaslt": rc.get("vs_hipblaslt"), "handover_fallbacks": sg.get("handover_fallbacks"),
    }
    return ex


def _peer_topology(world: int) -> dict:
    """hipDeviceCanAccessPeer among this job's GPUs, the device-to-device
    path between them and measured copy bandwidth by engine
    (``bench/peer_topology.py``), in a child process with its own time limit
    so that the peer paths cannot hold the headline line back."""
    return _run_child([sys.executable, "peer_topology.py", "--gpus", str(world)], _child_env(), PEER_TOPOLOGY_TIMEOUT_S)


def _free_port() -> int:
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """Start ``n`` rank processes of this script through
    ``torch.distributed.run`` (a child process, rendezvous on 127.0.0.1) and
    return its exit code.  Called before anything imports the runtime, so
    this process never initialises a GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--tile", default=None)
    ap.add_argument("--device", choices=("auto", "gpu", "cpu"), default="auto",
                    help="cpu: kernel-string GEMM on each rank's CPU device (launcher rehearsal)")
    ap.add_argument("--skip-mandelbrot", action="store_true")
    ap.add_argument("--skip-node-configs", action="store_true",
                    help="skip the N-body pipeline and task-pool configs (rank 0, after the headline)")
    ap.add_argument("--detail", default=None,
                    help="path of the full results JSON (default: gpurun_out/ and profiles/bench_detail_n{N}.json)")
    return ap.parse_args(argv)


def _wait_for_exit(pids, timeout_s: float = 60.0) -> None:
    """Until every process in ``pids`` has exited (or is a zombie waiting
    for its parent), at most ``timeout_s``."""
    def alive(pid: int) -> bool:
        try:
            with open(f"/proc/{pid}/stat") as f:
                return f.read().rsplit(")", 1)[1].split()[0] != "Z"
        except (OSError, IndexError):
            return False

    t_end = time.time() + timeout_s
    while time.time() < t_end and any(alive(p) for p in pids):
        time.sleep(0.05)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, argv)

    from cekirdekler_amd._native import gpu_available
    from cekirdekler_amd.parallel.distributed import init_distributed

    ctx = init_distributed()
    if ctx.world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the job has {ctx.world} ranks")
    use_gpu = args.device == "gpu" or (args.device == "auto" and gpu_available())
    if use_gpu:
        sg = bench_sgemm(ctx, args.steps, args.warmup, args.size, args.tile)
    else:
        sg = bench_sgemm_cpu(ctx, args.steps, args.warmup, min(args.size, 512))
    all_ranges = _all_ranges(ctx, sg["ranges"])
    mb = {} if (args.skip_mandelbrot or not use_gpu) else bench_mandelbrot(ctx, args.steps, args.warmup)
    rowc = {}
    if ctx.rank == 0 and use_gpu and args.size == 8192:
        try:  # an extra: a failure is reported in its field
            rowc = _row_major_comparison(args.steps)
        except Exception as e:  # pragma: no cover
            rowc = {"error": repr(e)[:300]}
    others = []
    if ctx.is_distributed:
        import torch.distributed as dist

        pids = [None] * ctx.world
        dist.all_gather_object(pids, os.getpid())
        others = [p for r, p in enumerate(pids) if r != ctx.rank]
        dist.barrier()
        dist.destroy_process_group()  # the other ranks exit here; rank 0 goes on alone
    if ctx.rank == 0 and others:
        # the timing measurements below start once the other ranks have gone
        # (their teardown, 7 GPU contexts when ranks share a GPU, disturbed
        # 10 calls of the load-balance measurement in an 8-rank rehearsal)
        _wait_for_exit(others, timeout_s=60.0)
    lb = bench_lb_iters() if (ctx.rank == 0 and use_gpu) else {}
    slices = {}
    if ctx.rank == 0 and use_gpu and args.size == 8192:
        try:  # an extra: a failure is reported in its field
            slices = bench_sgemm_slices(args.steps)
        except Exception as e:  # pragma: no cover
            slices = {"error": repr(e)[:300]}
    node = {} if (ctx.rank != 0 or args.skip_node_configs or not use_gpu) else bench_node_configs(ctx.world)
    peers = _peer_topology(ctx.world) if (ctx.rank == 0 and use_gpu) else {}
    ok = sg["max_rel_err"] <= MAX_REL_ERR
    if ctx.rank == 0:
        size = args.size if use_gpu else min(args.size, 512)
        full = {
            "sgemm": sg, "sgemm_ranges_all_ranks": all_ranges,
            "sgemm_row_major_c": rowc, "sgemm_slices": slices, "mandelbrot_4k": mb, "load_balance_iters": lb,
            **node,
            "peer_topology": peers,
        }
        detail = write_detail(full, ctx.world, args.detail, gpu=use_gpu)
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
            "dtype": "bf16" if use_gpu else "fp32",
            "data": "synthetic",
            "config": {"model": f"SGEMM {size}x{size}x{size} {'bf16' if use_gpu else 'fp32'} (fp32 acc/out), "
                                f"range-partitioned + load-balanced, tile {sg['tile']}",
                       "global_batch": 1, "seq_len": size,
                       "parallelism": f"range-partition dp{ctx.world}",
                       "timing": sg.get("timing", "enqueue mode, one queue"),
                       "device": sg["device"]},
            "extra": compact_extra(full, detail),
        }
        print(json.dumps(out, separators=(",", ":")), flush=True)
        if not ok:
            print(f"bench.py: SGEMM output check failed: max rel err {sg['max_rel_err']:.3e} "
                  f"(limit {MAX_REL_ERR})", file=sys.stderr, flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
