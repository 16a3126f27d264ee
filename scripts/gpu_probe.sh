#!/bin/bash
# Round-2 probe: GPU tests, the default bench, the B=100 bench and a
# kernel-trace profile of the B=100 bench (per-step fixed cost breakdown).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
R=$(pwd)
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
step bench 300 python bench.py --steps 20 --warmup 5 --no-parity-leg || exit $?
step bench_b100 300 python bench.py --steps 200 --warmup 10 --minibatch 100 --no-cpu-baseline --no-parity-leg || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$R"
step prof_b100 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b100 -o run -- python3 $R/bench.py --steps 200 --warmup 10 --minibatch 100 --no-cpu-baseline --no-parity-leg || exit $?
