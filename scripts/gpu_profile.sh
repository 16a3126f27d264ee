#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench (fast = the headline, and parity),
# then separate PMC passes for FETCH_SIZE and WRITE_SIZE (never combined with
# other tracing), plus the LR (config 3) leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
R=$(pwd)
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"
  return $rc
}
B="$R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity-leg"
# the PMC window: warmup 3 launches, then the 20 timed ones
run prof_fast 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fast -o run -- python3 $B || exit $?
run prof_parity 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_parity -o run -- python3 $B --parity || exit $?
run pmc_fetch_fast 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_fast -o run -- python3 $B || exit $?
run pmc_write_fast 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_fast -o run -- python3 $B || exit $?
run prof_lr 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lr -o run -- python3 $R/bench.py --app lr --steps 20 --warmup 3 || exit $?
