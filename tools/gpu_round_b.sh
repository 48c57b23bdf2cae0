#!/bin/bash
# Second GPU session of the round: a kernel trace of the headline bench, then
# multi-rank rehearsals of the bench on the one GPU (ranks share GPU 0; the
# 8-GPU run is the driver's).  Every step has its own time limit; a failing
# step ends the call.
set -o pipefail
out=${1:-gpurun_out/runb}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/prof" -o bench -- python3 bench.py --steps 10 --warmup 2 \
  --skip-node-configs > "$out/prof_bench.json" 2> "$out/prof_bench.err" || exit $?
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --skip-node-configs --skip-mandelbrot \
  > "$out/bench_2r.json" 2> "$out/bench_2r.err" || exit $?
timeout -k 10 400 python bench.py --gpus 4 --size 4096 --steps 5 --warmup 2 --skip-node-configs --skip-mandelbrot \
  > "$out/bench_4r_4096.json" 2> "$out/bench_4r_4096.err" || exit $?
