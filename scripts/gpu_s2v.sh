#!/bin/bash
# sent2vec: the GPU tests and the s2v leg (its load time / single-pass end to end)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_s2v_gpu.py tests/test_compat.py tests/test_host.py -m gpu -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/s2v_tests.log 2>&1
rc=$?; tail -8 gpurun_out/s2v_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --app s2v --steps 31 --warmup 31 --no-cpu-baseline > gpurun_out/s2v_bench.log 2>&1 || { tail -20 gpurun_out/s2v_bench.log; exit 1; }
grep '^{' gpurun_out/s2v_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['setup_s'], d['config']['end_to_end'])"
exit $rc
