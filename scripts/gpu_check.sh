#!/bin/bash
# One GPU session: GPU tests, smoke, short bench. Stops at the first GPU
# fault / abort / timeout (exit codes other than 0 and pytest's 1).
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
step pytest_gpu 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rA
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py --steps 20 --warmup 3 || exit $?
step bench_fast 600 python bench.py --steps 20 --warmup 3 --parity --no-cpu-baseline || exit $?
step bench_b100 600 python bench.py --steps 200 --warmup 10 --minibatch 100 --no-cpu-baseline || exit $?
step bench_b100_fast 600 python bench.py --steps 200 --warmup 10 --minibatch 100 --parity --no-cpu-baseline || exit $?
