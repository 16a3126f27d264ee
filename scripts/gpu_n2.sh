#!/bin/bash
# the driver's multi-GPU command shape at N=2 (two ranks on the one GPU: the library's TCP transport)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python bench.py --gpus 2 > gpurun_out/n2_bench.log 2>&1; rc=$?
grep '^{' gpurun_out/n2_bench.log | tail -1 > gpurun_out/n2_bench.json
tail -3 gpurun_out/n2_bench.log | cut -c1-300
exit $rc
