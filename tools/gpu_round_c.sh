#!/bin/bash
# Third GPU session: the GPU tier on the current tree, the j-split N-body
# pipeline (four logical devices), PCIe issue-pattern and host-resident
# panel-count probes, the headline bench.  Each step has its own time limit;
# a failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/runc}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/gputests.log" 2>&1 || exit $?
timeout -k 10 240 python bench/nbody_pipeline.py --gpus 4 --logical 4 --pushes 12 > "$out/nbody_shared.json" \
  2> "$out/nbody_shared.err" || exit $?
timeout -k 10 300 python tools/scale_probe.py 1024,2048,4096 256x256pb:a:q2,256x256pb:a:q4,256x256pb:a,256x256pb 3 20 \
  > "$out/scale_async.json" 2> "$out/scale_async.err" || exit $?
timeout -k 10 120 python tools/h2d_chunks_probe.py "$out/h2d_chunks.json" > /dev/null 2> "$out/h2d_chunks.err" || exit $?
timeout -k 10 240 python tools/hostres_probe.py 8,16,32 4 > "$out/hostres_panels.json" 2> "$out/hostres_panels.err" || exit $?
CEK_DEVICE_SPANS=0 timeout -k 10 180 python tools/fanout_probe.py "$out/fanout_nospans.json" > "$out/fanout_nospans.log" 2>&1 || exit $?
timeout -k 10 400 python bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
