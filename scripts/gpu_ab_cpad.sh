#!/bin/bash
# w2v/snapshot/quality/compat GPU tests, then same-box A/B of SWPS_CACHE_PAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_w2v_gpu.py tests/test_snapshot_gpu.py tests/test_quality_gpu.py tests/test_compat.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_w2v.log 2>&1 || { tail -30 gpurun_out/pytest_w2v.log; exit 1; }
tail -1 gpurun_out/pytest_w2v.log
AB_NAME=SWPS_CACHE_PAD AB_VALS="0 1" bash scripts/gpu_ab_vars.sh || exit $?
AB_NAME=SWPS_CACHE_PAD AB_VALS="0 1" bash scripts/gpu_ab_vars.sh || exit $?
