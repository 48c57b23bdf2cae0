#!/bin/bash
# Ninth GPU session: the GPU tier (with the CPU + GPU co-execution test) and
# the Mandelbrot end-to-end time against the blob count.  Each step has its
# own time limit; a failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/runi}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/gputests.log" 2>&1 || exit $?
timeout -k 10 200 python tools/mandel_e2e_probe.py blobs=1,2,4,8 > "$out/mandel_e2e.json" 2> "$out/mandel_e2e.err" || exit $?
