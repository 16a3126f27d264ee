#!/bin/bash
# same-box A/B of the gather knobs (rows in flight per wave, grid cap)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB_NAME=SWPS_GATHER_UNR AB_VALS="4 8 16" bash scripts/gpu_ab_vars.sh || exit $?
AB_NAME=SWPS_GATHER_GRID AB_VALS="2048 4096 8192 16384 65536" bash scripts/gpu_ab_vars.sh || exit $?
