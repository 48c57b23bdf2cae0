#!/bin/bash
# Twentieth GPU session: the wave frame with HIP's default host wait and with
# blocking waits (CEK_HIP_SYNC=blocking), three alternating runs each.
set -o pipefail
out=${1:-gpurun_out/runq}
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2 3; do
  for m in default blocking; do
    if [ "$m" = default ]; then unset CEK_HIP_SYNC; else export CEK_HIP_SYNC=$m; fi
    (cd bench && timeout -k 10 200 python wave_cpu_gpu.py) > "$out/wave_${m}_$r.json" 2> "$out/wave_${m}_$r.err" || exit $?
  done
done
