#!/bin/bash
# Fourth GPU session: async-queue count at the slice sizes, host-resident
# shells with two upload streams, the GPU tier, the bench.  Each step has its
# own time limit; a failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/rund}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python tools/scale_probe.py 1024,2048,4096 256x256pb:a:q2,256x256pb:a:q4,256x256pb:a,256x256pb 3 20 \
  > "$out/scale_async.json" 2> "$out/scale_async.err" || exit $?
timeout -k 10 240 python tools/hostres_probe.py 16,8 4 > "$out/hostres_two_streams.json" 2> "$out/hostres.err" || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/gputests.log" 2>&1 || exit $?
timeout -k 10 400 python bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
