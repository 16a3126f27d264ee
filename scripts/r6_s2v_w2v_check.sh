#!/bin/bash
# sent2vec tests + phases, and the w2v tests of the push variants (split push)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_w2v_gpu.py tests/test_bench_shape_gpu.py -m gpu -x -q -p no:cacheprovider -k "split or variant or push" --timeout 300 --timeout-method thread > gpurun_out/w2vs_tests.log 2>&1 || { tail -30 gpurun_out/w2vs_tests.log; exit 1; }
tail -1 gpurun_out/w2vs_tests.log
bash scripts/r6_s2v_check.sh
