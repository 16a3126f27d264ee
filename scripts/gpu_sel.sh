#!/bin/bash
# One GPU session over a selection: TESTS="tests/a.py tests/b.py::t" (pytest, -m gpu and CPU
# tests alike), then optionally the default bench line (BENCH=1, extra args in BENCH_ARGS).
# Stops at the first GPU fault / abort / timeout (exit codes other than 0 and pytest's 1).
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
rc=0
if [ -n "$TESTS" ]; then
  step sel_tests ${TEST_TIMEOUT:-700} python -u -m pytest $TESTS -q -p no:cacheprovider -rf -s --timeout 240 --timeout-method thread
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$BENCH" ]; then
  step bench ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS} || exit $?
  grep '^{' gpurun_out/bench.log > gpurun_out/bench.json || true
fi
exit $rc
