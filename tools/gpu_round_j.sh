#!/bin/bash
# Tenth GPU session: the bench with every node config (co-execution included).
set -o pipefail
out=${1:-gpurun_out/runj}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
