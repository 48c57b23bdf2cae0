#!/bin/bash
# One GPU session: the GPU test tier, then (only if it passed) the bench,
# then (time permitting) the round's probes.  Every GPU step has its own
# time limit; a failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/run}
mkdir -p "$out"
start=$(date +%s)
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gputests.log" 2>&1
rc=$?
echo "tests rc=$rc" >> "$out/gputests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$out/bench.json" 2> "$out/bench.err"
rc=$?
echo "bench rc=$rc" >> "$out/bench.err"
[ $rc -eq 0 ] || exit $rc
if [ -n "$CEK_SKIP_PROBES" ] || [ $(( $(date +%s) - start )) -gt 600 ]; then exit 0; fi
bash tools/gpu_probes_r4.sh "$out/probes"
