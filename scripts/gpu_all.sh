#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_dist.sh || exit $?
bash scripts/gpu_quick.sh || exit $?
