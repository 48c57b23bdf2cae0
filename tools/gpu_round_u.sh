#!/bin/bash
# Examples on the GPU box: CPU + GPU co-execution, hello SAXPY.
set -o pipefail
out=${1:-gpurun_out/runu}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python examples/cpu_gpu_coexecution.py > "$out/coexec.log" 2>&1 || exit $?
timeout -k 10 200 python examples/hello_saxpy.py > "$out/saxpy.log" 2>&1 || exit $?
