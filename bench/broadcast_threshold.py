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
stays faster; ``ClNumberCruncher.calibrate_peer_reads`` (which this runs)
adopts it as the runtime's ``peer_read_min_bytes``.

With one GPU the D devices are logical devices of it (``"logical": true``):
every copy then shares one PCIe link and one GPU, so the numbers rehearse
the code path only; the driver's multi-GPU run measures the real threshold.
"""
import argparse

from common import emit

import cekirdekler_amd as ck
from cekirdekler_amd.utils.multigpu import PEER_READ_SIZES


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=0, help="GPUs to use (0: all visible)")
    ap.add_argument("--calls", type=int, default=7)
    ap.add_argument("--sizes", default=",".join(str(s) for s in PEER_READ_SIZES))
    a = ap.parse_args()
    g = ck.ClPlatforms.all().gpus()
    ng = len(g) if a.gpus <= 0 else min(a.gpus, len(g))
    logical = ng < 2
    devs = (g[0] + g[0]) if logical else g[0:ng]
    # the runtime's own calibration (ClNumberCruncher.calibrate_peer_reads):
    # measures both modes by size and adopts the crossover as
    # peer_read_min_bytes for this device set
    cr = ck.ClNumberCruncher(devs, "")
    default = cr.peer_read_min_bytes
    res = cr.calibrate_peer_reads(sizes=[int(s) for s in a.sizes.split(",")], calls=a.calls)
    out = {"config": "broadcast_threshold", "logical": logical, **res,
           "runtime_default_min_bytes": default, "runtime_adopted_min_bytes": cr.peer_read_min_bytes}
    cr.dispose()
    emit(out)


if __name__ == "__main__":
    main()
