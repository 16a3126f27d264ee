#!/bin/bash
# tests + the two bench modes (no rocprof)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step pytest_gpu 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rA -s
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench 600 python bench.py --steps 20 --warmup 3 || exit $?
step bench_parity 600 python bench.py --steps 20 --warmup 3 --parity --no-cpu-baseline || exit $?
