#!/bin/bash
# Targeted GPU step: pytest on the given test files / -k filter, output to
# gpurun_out/$NAME.log; then optional extra commands ($EXTRA, run only when
# the tests did not fault).  Usage: NAME=t6 K="alias" bash scripts/gpu_t.sh tests/x.py ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
NAME=${NAME:-t}
timeout -k 10 ${TO:-500} python -u -m pytest "$@" -m gpu -q -p no:cacheprovider -rf -s --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/$NAME.log 2>&1
rc=$?
grep -h "passed\|failed\|FAILED\|analogy\|ingest" gpurun_out/$NAME.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$EXTRA" ]; then bash -c "$EXTRA" || exit $?; fi
exit $rc
