#!/bin/bash
# every GPU test (not -x: the whole list of failures), then smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1050 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/suite_tests.log 2>&1
rc=$?; tail -15 gpurun_out/suite_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/suite_smoke.log 2>&1 || { tail -20 gpurun_out/suite_smoke.log; exit 1; }
tail -1 gpurun_out/suite_smoke.log
exit $rc
