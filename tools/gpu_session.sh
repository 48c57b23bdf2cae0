#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; each step has its own time
# limit.  Test failures (exit 1) do not stop the session; a crash, abort,
# fault or timeout does (no further GPU work after those).
# usage: tools/gpu_session.sh "name:seconds:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc elapsed=$(( $(date +%s) - start ))s"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ -n "$CEK_STOP_ON_FAIL" ]; }; then
    echo "=== stopping: $name exited with $rc"
    exit $rc
  fi
done
exit 0
