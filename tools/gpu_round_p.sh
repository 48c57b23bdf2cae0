#!/bin/bash
# Nineteenth GPU session: how host threads wait for the GPU (CEK_HIP_SYNC)
# against the wave frame and the co-execution case.  Each step has its own
# time limit; a failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/runp}
mkdir -p "$out"
export TMPDIR=/tmp
for m in default spin yield blocking; do
  if [ "$m" = default ]; then unset CEK_HIP_SYNC; else export CEK_HIP_SYNC=$m; fi
  (cd bench && timeout -k 10 200 python wave_cpu_gpu.py) > "$out/wave_$m.json" 2> "$out/wave_$m.err" || exit $?
  (cd bench && timeout -k 10 200 python hetero_stream.py --iters 16 --rounds 3) > "$out/hetero_$m.json" 2> "$out/hetero_$m.err" || exit $?
done
