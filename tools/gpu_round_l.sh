#!/bin/bash
# Thirteenth GPU session: fp32 load spreading, half vs quarter vs all, twice.
set -o pipefail
out=${1:-gpurun_out/runl}
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 240 python tools/gemm_f32_probe.py 8192 256x256g8h,256x256g8q,256x256g8i 3 5 \
    > "$out/f32_$r.json" 2> "$out/f32_$r.err" || exit $?
done
