#!/bin/bash
# LR + compat GPU tests, then the three bench legs (w2v headline, LR config 3, sent2vec config 5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"; return $rc; }
step pytest_lr 600 python -u -m pytest tests/test_lr_gpu.py tests/test_compat.py -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread || exit $?
step bench_lr 600 python bench.py --app lr --steps 20 --warmup 3 || exit $?
step bench_s2v 600 python bench.py --app s2v --steps 20 --warmup 3 || exit $?
step bench_w2v 600 python bench.py --steps 20 --warmup 3 --no-parity-leg || exit $?
