"""The reference's async-queue timeline (async.png, README: "queue-overlapped
vecAdd / vecMul / vecDiv / vecAddInt kernels ≈ 3 ms each, buffer transfers
≈ 1-2 ms"), measured: four independent computes, each uploading its two
inputs, running its kernel and downloading its result, issued

* ``sync``        — one compute() at a time, host sync after each;
* ``enqueue``     — enqueue mode on one queue (no host syncs, in order);
* ``async``       — enqueue mode + ``enqueue_mode_async_enable``: each
  compute on the next compute stream (Cores.cs:80-83, :858-935), the
  downloads issued after the next compute's uploads (the streams share an
  SDMA queue, see ``Cores::flush_downloads``);
* ``async_inorder`` — the same with each compute's downloads in its own
  order (``Cores.deferred_downloads = False``).

The kernels carry ``--iters`` dependent multiply-adds per element so a
kernel takes about as long as its transfers, as in the reference's
picture.  Every result is checked exactly against numpy (integer kernel) or
to float tolerance (the GPU fuses the multiply-add), and every mode must
produce the same bits; modes are interleaved over rounds (median ms per
round of four computes)."""
import argparse
import statistics
import time

import numpy as np

from common import emit, sync

import cekirdekler_amd as ck

SRC = """
__global__ void vecAdd(const float* a, const float* b, const int* it, float* c) {
    long long i = get_global_id(0); float v = a[i] + b[i];
    for (int k = 0; k < it[0]; ++k) v = v * 0.999f + 0.001f;
    c[i] = v;
}
__global__ void vecMul(const float* a, const float* b, const int* it, float* c) {
    long long i = get_global_id(0); float v = a[i] * b[i];
    for (int k = 0; k < it[0]; ++k) v = v * 0.999f + 0.001f;
    c[i] = v;
}
__global__ void vecDiv(const float* a, const float* b, const int* it, float* c) {
    long long i = get_global_id(0); float v = a[i] / b[i];
    for (int k = 0; k < it[0]; ++k) v = v * 0.999f + 0.001f;
    c[i] = v;
}
__global__ void vecAddInt(const int* a, const int* b, const int* it, int* c) {
    long long i = get_global_id(0); unsigned int v = (unsigned int)(a[i] + b[i]);
    for (int k = 0; k < it[0]; ++k) v = v * 1664525u + 1013904223u;
    c[i] = (int)v;
}
"""


def float_ref(v: np.ndarray, iters: int) -> np.ndarray:
    v = v.astype(np.float32)
    for _ in range(iters):
        v = v * np.float32(0.999) + np.float32(0.001)
    return v


def int_ref(v: np.ndarray, iters: int) -> np.ndarray:
    a, c = 1664525, 1013904223
    A, C = 1, 0
    pa, pc, n = a, c, iters
    while n:  # f^iters in closed form (mod 2^32)
        if n & 1:
            A, C = (pa * A) & 0xFFFFFFFF, (pa * C + pc) & 0xFFFFFFFF
        pa, pc = (pa * pa) & 0xFFFFFFFF, (pa * pc + pc) & 0xFFFFFFFF
        n >>= 1
    u = v.astype(np.uint32).astype(np.uint64)
    return ((u * np.uint64(A) + np.uint64(C)) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4 << 20)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    gpu = ck.ClPlatforms.all().gpus()
    if not len(gpu):
        raise SystemExit("async_queues.py needs a GPU")
    cr = ck.ClNumberCruncher(gpu[0], SRC)
    if cr.error_code():
        raise SystemExit(cr.error_message())
    n = a.n
    rng = np.random.default_rng(1)
    it = ck.ClArray(np.array([a.iters], np.int32))
    it.write = False
    jobs = []
    for k, name in enumerate(("vecAdd", "vecMul", "vecDiv", "vecAddInt")):
        if name == "vecAddInt":
            x = ck.ClArray(n, np.int32)
            y = ck.ClArray(n, np.int32)
            z = ck.ClArray(n, np.int32)
            x.array[:] = rng.integers(-1000, 1000, n)
            y.array[:] = rng.integers(-1000, 1000, n)
            want = int_ref(x.array + y.array, a.iters)
        else:
            x = ck.ClArray(n, np.float32)
            y = ck.ClArray(n, np.float32)
            z = ck.ClArray(n, np.float32)
            x.array[:] = rng.random(n, dtype=np.float32) + 0.5
            y.array[:] = rng.random(n, dtype=np.float32) + 0.5
            op = {"vecAdd": np.add, "vecMul": np.multiply, "vecDiv": np.divide}[name]
            want = float_ref(op(x.array, y.array), a.iters)
        x.write = y.write = False
        z.read = False
        jobs.append((name, 10 + k, x.next_param(y, it, z), z, want))

    def round_(mode):
        if mode != "sync":
            cr.enqueue_mode = True
            cr.enqueue_mode_async_enable = mode.startswith("async")
        cr.cores.deferred_downloads = mode != "async_inorder"
        for name, cid, grp, _, _ in jobs:
            grp.compute(cr, cid, name, n, 256)
        if mode != "sync":
            cr.enqueue_mode = False
            cr.enqueue_mode_async_enable = False

    modes = ("sync", "enqueue", "async", "async_inorder")
    for m in modes:  # untimed: buffers, streams, balancer state
        round_(m)
    times = {m: [] for m in modes}
    exact = True
    bad = {}
    firsts = {}
    for _ in range(a.rounds):
        for m in modes:
            for _, _, _, z, _ in jobs:
                z.array[:] = 0
            sync()
            t = time.perf_counter()
            round_(m)
            sync()
            times[m].append((time.perf_counter() - t) * 1e3)
            for name, _, _, z, want in jobs:
                if name == "vecAddInt":
                    ok = bool(np.array_equal(z.array, want))
                    err = float(np.mean(z.array != want))
                else:  # the GPU contracts v * 0.999 + 0.001 into one FMA; numpy rounds twice
                    ok = bool(np.allclose(z.array, want, rtol=1e-4, atol=1e-5))
                    err = float(np.max(np.abs(z.array - want)))
                first = firsts.setdefault(name, z.array.copy())
                ok &= bool(np.array_equal(z.array, first))  # every mode: the same bits
                exact &= ok
                if not ok:
                    bad[f"{m}/{name}"] = err
    med = {m: round(statistics.median(v), 3) for m, v in times.items()}
    # the parts of one compute, timed alone (sync, one compute)
    out = {"config": "async_queues", "n": n, "iters": a.iters, "kernels": [j[0] for j in jobs],
           "compute_streams": cr.compute_queue_concurrency, "ms_per_round_of_4": med,
           "async_speedup_over_sync": round(med["sync"] / med["async"], 3),
           "async_speedup_over_enqueue": round(med["enqueue"] / med["async"], 3),
           "deferred_vs_inorder": [med["async"], med["async_inorder"]],
           "outputs_checked": exact, **({"failed": bad} if bad else {}),
           "timing": f"median of {a.rounds} interleaved rounds"}
    cr.dispose()
    emit(out)


if __name__ == "__main__":
    main()
