#!/bin/bash
# PMC passes over a few 4096² Mandelbrot dispatches of the kernels in $1
# (comma list); each pass has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export MANDEL_KERNELS=${1:-blk8h,blk8k} NBODY=0
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set -d gpurun_out/mandel_pmc$i -o run --output-format csv \
      -- python3 tools/valu_pmc.py > gpurun_out/mandel_pmc$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  python3 tools/pmc_table.py gpurun_out/mandel_pmc$i mandelbrot >> gpurun_out/mandel_pmc.txt
done
exit 0
