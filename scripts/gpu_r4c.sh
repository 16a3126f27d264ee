#!/bin/bash
# Per-feature A/B of the round-4 prep changes at B = 100 and B = 5000, and LR tile chunks 1536-2048.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
VARIANTS="SWPS_NOP=1;SWPS_ITEM_HEADS=0;SWPS_TOK_LOCAL=0;SWPS_ITEM_HEADS=0 SWPS_TOK_LOCAL=0;SWPS_SORT_IOTA=0 SWPS_SEG4=0 SWPS_TOK_LOCAL=0 SWPS_ITEM_HEADS=0" REPS=2 BENCH_ARGS="--config1-steps 0 --no-app-legs" bash scripts/gpu_ab.sh || exit $?
AB_VAR=SWPS_LR_TILE_CHUNK VARIANTS="1536 1792 2048" bash scripts/lr_fwdc_ab.sh
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
exit 0
