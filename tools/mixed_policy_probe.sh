#!/bin/bash
# CPU + GPU co-execution under each host-sharing policy (CEK_MIXED_CPU,
# hardware.mixed_cpu_policy): the wave example and the host-resident
# co-execution sweep, one child per policy, outputs under gpurun_out/.
# usage: tools/mixed_policy_probe.sh [policies] [tag] [extra env assignment]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}/bench"
pols="${1:-none reserve sleep both}"
tag="${2:-mp}"
extra="${3:-}"
for p in $pols; do
  env CEK_MIXED_CPU=$p $extra timeout -k 10 120 python wave_cpu_gpu.py > ../gpurun_out/${tag}_wave_$p.json || exit $?
  env CEK_MIXED_CPU=$p $extra timeout -k 10 200 python hetero_stream.py --rounds 3 --calls 4 > ../gpurun_out/${tag}_hetero_$p.json || exit $?
  echo "policy $p done"
done
