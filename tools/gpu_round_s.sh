#!/bin/bash
# Twenty-fourth GPU session: 2-rank bench rehearsal on one GPU (the
# distributed path with the reused native call) and the 8-GPU slice
# schedules once more.  Each step has its own time limit; a failing step
# ends the call.
set -o pipefail
out=${1:-gpurun_out/runs}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --skip-node-configs --skip-mandelbrot \
  > "$out/bench_2r.json" 2> "$out/bench_2r.err" || exit $?
timeout -k 10 300 python tools/scale_probe.py 1024,8192 256x256pbw,256x256pb:a:q4,256x256pb 3 20 \
  > "$out/scale.json" 2> "$out/scale.err" || exit $?
