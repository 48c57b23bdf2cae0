#!/bin/bash
# Twentieth GPU session: the wave frame and co-execution with GPU workers
# spinning (CEK_SLEEP_WAITS=0, the old behaviour) or sleeping on a
# blocking-sync event (the default now for GPU+CPU crunchers), alternating.
set -o pipefail
out=${1:-gpurun_out/runq}
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2 3; do
  for m in 0 1; do
    export CEK_SLEEP_WAITS=$m
    (cd bench && timeout -k 10 200 python wave_cpu_gpu.py) > "$out/wave_s${m}_$r.json" 2> "$out/wave_s${m}_$r.err" || exit $?
  done
done
for m in 0 1; do
  export CEK_SLEEP_WAITS=$m
  (cd bench && timeout -k 10 200 python hetero_stream.py --iters 1,16 --rounds 3) > "$out/hetero_s$m.json" 2> "$out/hetero_s$m.err" || exit $?
done
