#!/bin/bash
# Fifth GPU session: fp32 load-spreading variants, the 8-GPU slice kernels
# against 4 async queues on one box, host-resident shells (one upload
# stream again), the bench.  Each step has its own time limit; a failing
# step ends the call.
set -o pipefail
out=${1:-gpurun_out/rune}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 240 python tools/gemm_f32_probe.py 8192 256x256g8,256x256g8i,256x256g8h 3 5 \
  > "$out/f32_spread.json" 2> "$out/f32_spread.err" || exit $?
timeout -k 10 300 python tools/scale_probe.py 1024,8192 256x256pbw,256x256pbs,256x256pb:a:q4,256x256pb 3 20 \
  > "$out/scale.json" 2> "$out/scale.err" || exit $?
timeout -k 10 240 python tools/hostres_probe.py 16 4 > "$out/hostres.json" 2> "$out/hostres.err" || exit $?
timeout -k 10 400 python bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
