#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first
# step that faults, aborts or times out (rc >= 2, pytest's "tests failed" = 1
# continues).  Usage: scripts/gpu_step.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($to s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -5 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ge 2 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
