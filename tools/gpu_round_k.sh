#!/bin/bash
# Eleventh GPU session: CPU + GPU co-execution against the CPU device's
# thread count (does the CPU share slow down beside the GPU's DMA and host
# thread?).  Each step has its own time limit; a failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/runk}
mkdir -p "$out"
export TMPDIR=/tmp
for t in 15 12 8; do
  (cd bench && timeout -k 10 200 python hetero_stream.py --iters 1,16 --cpu-threads $t) \
    > "$out/hetero_t$t.json" 2> "$out/hetero_t$t.err" || exit $?
done
