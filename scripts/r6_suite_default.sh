#!/bin/bash
# the GPU suite + smoke, then the driver's default line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_suite.sh || exit $?
bash scripts/r6_default.sh
