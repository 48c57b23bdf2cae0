#!/bin/bash
# Fifteenth GPU session: the wave example with the vectorized CPU math, the
# GPU tier.  Each step has its own time limit; a failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/runn}
mkdir -p "$out"
export TMPDIR=/tmp
(cd bench && timeout -k 10 200 python wave_cpu_gpu.py) > "$out/wave.json" 2> "$out/wave.err" || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/gputests.log" 2>&1 || exit $?
