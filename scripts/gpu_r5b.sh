#!/bin/bash
# round 5: LR fixed-point step variants, sent2vec (tests + leg), the compat suite incl. sent2vec.cpp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYTEST_K=fixed bash scripts/gpu_lrplan.sh || exit $?
bash scripts/gpu_s2v.sh || exit $?
