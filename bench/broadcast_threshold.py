"""Size threshold between the two ways a `read` array reaches every GPU
("Choose by size threshold, measured").

* ``direct``: the reference's way (Worker.cs:833-860) — every GPU uploads the
  whole array over its own PCIe link;
* ``staged``: the runtime's xGMI fan-out (``Cores::stage_peer_reads``) —
  every GPU uploads 1/D of it, then pulls the other D−1 chunks from its
  peers' replicas (``hipMemcpyPeerAsync`` over the point-to-point links),
  event-ordered, no host sync.

For each size a compute() reads the array whole on every GPU (a tiny
kernel, so the call time is the transfer); both modes are timed as the
median of ``--calls`` calls, interleaved, and every call's output is
checked.  ``crossover_bytes`` is the smallest size from which ``staged``
stays faster: the value for ``Cores.peer_read_min_bytes``.

With one GPU the D devices are logical devices of it (``"logical": true``):
every copy then shares one PCIe link and one GPU, so the numbers rehearse
the code path only; the driver's multi-GPU run measures the real threshold.
"""
import argparse
import statistics
import time

import numpy as np

from common import emit, sync

import cekirdekler_amd as ck

SRC = """
__global__ void touch(const float* x, float* y) {
    long long i = get_global_id(0);
    y[i] = x[i] * 2.0f + 1.0f;
}
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=0, help="GPUs to use (0: all visible)")
    ap.add_argument("--calls", type=int, default=7)
    ap.add_argument("--sizes", default="65536,262144,1048576,4194304,16777216,67108864,268435456")
    a = ap.parse_args()
    g = ck.ClPlatforms.all().gpus()
    ng = len(g) if a.gpus <= 0 else min(a.gpus, len(g))
    logical = ng < 2
    devs = (g[0] + g[0]) if logical else g[0:ng]
    D = len(devs)
    cr = ck.ClNumberCruncher(devs, SRC)
    if cr.error_code():
        raise SystemExit(cr.error_message())
    cr.cores.peer_read_min_bytes = 0
    G = 256 * D * 4
    y = ck.ClArray(np.zeros(G, np.float32))
    y.read = False
    out = {"config": "broadcast_threshold", "devices": D, "logical": logical, "calls": a.calls,
           "sizes": [], "direct_ms": [], "staged_ms": [], "staged_path": [], "exact": True}
    cid = 1
    for size in (int(s) for s in a.sizes.split(",")):
        n = max(G, size // 4)
        x = ck.ClArray(n, np.float32)
        x.array[:] = np.arange(n, dtype=np.float32) % 1000
        x.write = False
        want = x.array[:G] * 2.0 + 1.0
        times = {"direct": [], "staged": []}
        for mode in ("direct", "staged"):  # untimed first calls: buffers, balancer state
            cr.cores.peer_reads = mode == "staged"
            x.next_param(y).compute(cr, cid + (mode == "staged"), "touch", G, 256)
        for _ in range(a.calls):
            for mode in ("direct", "staged"):
                cr.cores.peer_reads = mode == "staged"
                y.array[:] = 0
                sync()
                t0 = time.perf_counter()
                x.next_param(y).compute(cr, cid + (mode == "staged"), "touch", G, 256)
                sync()
                times[mode].append((time.perf_counter() - t0) * 1e3)
                out["exact"] &= bool(np.array_equal(y.array, want))
        rec = cr.last_record()
        out["sizes"].append(4 * n)
        out["direct_ms"].append(round(statistics.median(times["direct"]), 4))
        out["staged_ms"].append(round(statistics.median(times["staged"]), 4))
        out["staged_path"].append(rec["p2p_path"])
        x.dispose()
        cid += 2
    cross = None
    for i in range(len(out["sizes"])):
        if all(s < d for s, d in zip(out["staged_ms"][i:], out["direct_ms"][i:])):
            cross = out["sizes"][i]
            break
    out["crossover_bytes"] = cross
    out["runtime_default_min_bytes"] = 1 << 20
    cr.dispose()
    emit(out)


if __name__ == "__main__":
    main()
