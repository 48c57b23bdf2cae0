#!/bin/bash
# Twenty-third GPU session: device-pool dispatch with 1 µs timer slack on the
# consumer threads (default now) against the kernel's 50 µs default
# (CEK_POOL_SLACK_NS=0), alternating.
set -o pipefail
out=${1:-gpurun_out/runr}
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2; do
  for m in 1000 0; do
    CEK_POOL_SLACK_NS=$m timeout -k 10 200 python tools/fanout_probe.py > "$out/fanout_${m}_$r.json" 2> "$out/fanout_${m}_$r.err" || exit $?
    (cd bench && CEK_POOL_SLACK_NS=$m timeout -k 10 200 python task_pool.py --gpus 1) > "$out/pool_${m}_$r.json" 2> "$out/pool_${m}_$r.err" || exit $?
  done
done
