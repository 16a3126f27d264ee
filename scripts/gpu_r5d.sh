#!/bin/bash
# LR GPU suite + the lr leg (plan none / load) + a rocprof kernel summary of the default lr leg
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_lr_gpu.py tests/test_compat.py -m gpu -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/r5d_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5d_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r5d_lr_none.log 2>&1 || { tail -20 gpurun_out/r5d_lr_none.log; exit 1; }
grep '^{' gpurun_out/r5d_lr_none.log > gpurun_out/r5d_lr_none.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5d_prof -o run -- python3 bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r5d_prof.log 2>&1 || exit 1
f=$(find gpurun_out/r5d_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5d_lr_kernel_stats.csv
grep '^{' gpurun_out/r5d_prof.log > gpurun_out/r5d_lr_traced.json
exit $rc
