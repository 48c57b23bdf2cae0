#!/bin/bash
# Seventeenth GPU session: the reused native call (host cost per compute):
# the GPU tier, the wave example, the fan-out probe.  Each step has its own
# time limit; a failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/runo}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/gputests.log" 2>&1 || exit $?
(cd bench && timeout -k 10 200 python wave_cpu_gpu.py) > "$out/wave.json" 2> "$out/wave.err" || exit $?
timeout -k 10 200 python tools/fanout_probe.py > "$out/fanout.json" 2> "$out/fanout.err" || exit $?
