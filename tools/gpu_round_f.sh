#!/bin/bash
# Sixth GPU session: CPU + GPU co-execution on host-resident data, the fp32
# default tile (spread loads) against hipBLASLt with one counter pass, the
# N-body force kernel with masses in LDS, CPU-device n-body, the GPU tier.
# Each step has its own time limit; a failing step ends the call.
set -o pipefail
out=${1:-gpurun_out/runf}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python bench/hetero_stream.py > "$out/hetero.json" 2> "$out/hetero.err" || exit $?
timeout -k 10 240 python tools/gemm_f32_probe.py 8192 256x256g8h,256x256g8,256x256gh 3 5 \
  > "$out/f32.json" 2> "$out/f32.err" || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d "$out/f32_pmc" -o run --output-format csv -- python3 tools/gemm_f32_pmc.py 256x256g8h,256x256g8 torch \
  > "$out/f32_pmc.log" 2>&1 || exit $?
timeout -k 10 240 python tools/nbody_force_variants.py 1048576 1,0.25 "$out/nbody_m.json" b2_js2,b2_js2m,b4_js2,b4_js2m \
  > "$out/nbody_m.log" 2>&1 || exit $?
(cd bench && timeout -k 10 240 python nbody_pipeline.py --gpus 4 --logical 4 --pushes 12) \
  > "$out/nbody_pipeline.json" 2> "$out/nbody_pipeline.err" || exit $?
timeout -k 10 200 python tools/cpu_nbody_probe.py 8192 > "$out/cpu_nbody.json" 2> "$out/cpu_nbody.err" || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/gputests.log" 2>&1 || exit $?
