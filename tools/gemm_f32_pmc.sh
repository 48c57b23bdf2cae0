#!/bin/bash
# PMC passes over fp32 GEMM dispatches (ours + hipBLASLt via torch): MFMA
# busy, wait/issue split, clock.  Each pass has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/f32_pmc$i -o run --output-format csv \
      -- python3 tools/gemm_f32_pmc.py 256x256,256x256pb torch > gpurun_out/f32_pmc$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
