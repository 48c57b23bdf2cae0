#!/bin/bash
# Eighth GPU session: PCIe download patterns (the Mandelbrot image's 64 MiB),
# N-body force j-loop unroll variants.  Each step has its own time limit; a
# failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/runh}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python tools/h2d_chunks_probe.py "$out/pcie.json" > "$out/pcie.log" 2>&1 || exit $?
timeout -k 10 300 python tools/nbody_force_variants.py 1048576 1,0.25 "$out/nbody_unroll.json" \
  b2_js2,b2_js2u4,b2_js2u16,b2_js2u32,b4_js2 > "$out/nbody_unroll.log" 2>&1 || exit $?
