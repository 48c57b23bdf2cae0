"""Peer topology of the job's GPUs (bench.py's ``peer_topology`` field):
hipDeviceCanAccessPeer among GPUs 0 .. world-1, the device-to-device path
the runtime takes between them, and measured copy bandwidth by engine (SDMA
vs copy kernel; a few pairs, every pair at once, inside GPU 0), every copy
checked byte for byte (``utils/multigpu.peer_bandwidth_report``).

A child process of bench.py with its own time limit, like the node configs:
the first run of the peer paths on a real multi-GPU node cannot hold the
headline line back."""
import argparse

from common import emit

from cekirdekler_amd._native import cek
from cekirdekler_amd.utils.multigpu import peer_bandwidth_report

ap = argparse.ArgumentParser()
ap.add_argument("--gpus", type=int, default=1)
a = ap.parse_args()
full = cek.can_access_peer_matrix()
ngpu = min(a.gpus, len(full))  # ranks may share a GPU (one-GPU rehearsals)
m = [row[:ngpu] for row in full[:ngpu]]
out = {"gpus_visible": len(full), "job_gpus": a.gpus, "can_access_peer": m, "path": cek.peer_path(m)}
try:  # an extra: a failure is reported in its field
    out["bandwidth"] = peer_bandwidth_report(list(range(ngpu)))
except Exception as e:  # pragma: no cover
    out["bandwidth"] = {"error": repr(e)[:300]}
emit(out)
