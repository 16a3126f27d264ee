#!/bin/bash
# w2v GPU tests, the default bench line, then the rocprof passes (scripts/gpu_profile.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"; return $rc; }
step pytest_w2v 400 python -u -m pytest tests/test_w2v_gpu.py tests/test_snapshot_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread || exit $?
step bench 400 python bench.py || exit $?
bash scripts/gpu_profile.sh
