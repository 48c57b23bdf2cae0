#!/bin/bash
# PMC passes over a few 8192³ GEMM dispatches (tile list in $1); each pass
# has its own time limit; a counter the tool rejects ends only that pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
TILES=${1:-256x256pp}
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/gemm_pmc$i -o run --output-format csv \
      -- python3 tools/gemm_pmc.py "$TILES" > gpurun_out/gemm_pmc$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
