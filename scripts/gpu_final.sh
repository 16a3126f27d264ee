#!/bin/bash
# Round-end refresh: the whole GPU suite, smoke(), the default bench line, the
# rocprof passes (scripts/gpu_profile.sh) and the LR / sent2vec bench legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 400 python bench.py || exit $?
bash scripts/gpu_profile.sh || exit $?
step bench_lr 400 python bench.py --app lr || exit $?
step bench_s2v 400 python bench.py --app s2v || exit $?
