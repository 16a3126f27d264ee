#!/bin/bash
# Round-end rehearsal: the GPU suite, smoke() and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 400 python bench.py || exit $?
