#!/bin/bash
# the compat suite (incl. sent2vec.cpp unchanged) and the word2vec GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_compat.py tests/test_w2v_gpu.py -m gpu -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/r5c_tests.log 2>&1
rc=$?; tail -8 gpurun_out/r5c_tests.log; exit $rc
