#!/bin/bash
# sent2vec: GPU tests (incl. the unchanged sent2vec.cpp) and the s2v leg with its load phases
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_s2v_gpu.py tests/test_compat.py -m gpu -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread -k "s2v or sent2vec" > gpurun_out/s2v2_tests.log 2>&1
rc=$?; tail -4 gpurun_out/s2v2_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SWPS_S2V_LOAD_TIMES=1 timeout -k 10 300 python bench.py --app s2v --steps 31 --warmup 31 --no-cpu-baseline > gpurun_out/s2v2_bench.log 2>&1 || { tail -20 gpurun_out/s2v2_bench.log; exit 1; }
grep "s2v load" gpurun_out/s2v2_bench.log
grep '^{' gpurun_out/s2v2_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['setup_s'], d['config']['end_to_end'])"
exit $rc
