#!/bin/bash
# One GPU session: GPU tests, smoke, default bench line. Stops at the first
# GPU fault / abort / timeout (exit codes other than 0 and pytest's 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  return $rc
}
step pytest_gpu ${PYTEST_TO:-1000} python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
[ -n "$NO_BENCH" ] && exit $rc
step bench 600 python bench.py || exit $?  # the driver's command
exit $rc
