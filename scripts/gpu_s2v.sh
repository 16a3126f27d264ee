#!/bin/bash
# sent2vec GPU tests + the config-5 bench leg
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"; return $rc; }
step pytest_s2v 600 python -u -m pytest tests/test_s2v_gpu.py -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread || exit $?
step bench_s2v 600 python bench.py --app s2v --steps 20 --warmup 3 --no-cpu-baseline || exit $?
