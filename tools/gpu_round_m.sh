#!/bin/bash
# Fourteenth GPU session: counters of the fp32 default tile against hipBLASLt.
set -o pipefail
out=${1:-gpurun_out/runm}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d "$out/f32_pmc" -o run --output-format csv -- python3 tools/gemm_f32_pmc.py 256x256g8i,256x256g8h torch \
  > "$out/f32_pmc.log" 2>&1 || exit $?
