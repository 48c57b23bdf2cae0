#!/bin/bash
# Seventh GPU session: the GPU tier, smoke(), the bench with every node
# config, and the bench's kernel trace.  Each step has its own time limit; a
# failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/rung}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/gputests.log" 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
timeout -k 10 500 python bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o bench -- python3 bench.py --steps 10 --warmup 2 \
  --skip-node-configs > "$out/prof_bench.json" 2> "$out/prof_bench.err" || exit $?
