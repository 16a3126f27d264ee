#!/bin/bash
# Round-4 batch.  PART=tests: the prep-kernel variants' bit-identity tests.  PART=ab: same-box A/B (old
# prep = iota/seg4/tok_local off vs the defaults; sort tile shapes), LR tile chunks, SQ counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "$PART" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests/test_bench_shape_gpu.py -k "SORT_IOTA or SORT_CFG or SEG4 or TOK_LOCAL or ITEM_HEADS" -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/r4b_tests.log; exit $rc
fi
VARIANTS="SWPS_SORT_IOTA=0 SWPS_SEG4=0 SWPS_TOK_LOCAL=0 SWPS_ITEM_HEADS=0;SWPS_NOP=1;SWPS_SORT_CFG=1;SWPS_SORT_CFG=2;SWPS_SORT_CFG=3" REPS=2 BENCH_ARGS="--config1-steps 0 --no-app-legs" bash scripts/gpu_ab.sh || exit $?
NO_TESTS=1 AB_VAR=SWPS_LR_TILE_CHUNK VARIANTS="1024 1280 1536" bash scripts/lr_fwdc_ab.sh
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
NAME=bfp32 N=20 bash scripts/gpu_sq.sh bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity-leg --b100-steps 0 --config1-steps 0 --no-app-legs || exit $?
NAME=b100 N=200 bash scripts/gpu_sq.sh bench.py --steps 200 --warmup 10 --minibatch 100 --no-cpu-baseline --no-parity-leg --config1-steps 0 --b100-steps 0 --no-app-legs || exit $?
exit 0
