#!/bin/bash
# the driver's own bench command (no flags), its JSON line kept
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python bench.py > gpurun_out/default_bench.log 2>&1 || { tail -30 gpurun_out/default_bench.log; exit 1; }
grep '^{' gpurun_out/default_bench.log | tail -1 > gpurun_out/default_bench.json
cut -c1-400 gpurun_out/default_bench.json
