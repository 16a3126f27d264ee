#!/bin/bash
# the default line's s2v leg alone (31 minibatches of 8,193 docs), twice; then the tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  SWPS_S2V_LOAD_TIMES=1 timeout -k 10 300 python bench.py --app s2v --steps 31 --warmup 0 --no-cpu-baseline > gpurun_out/r6_s2v_dl.json 2> gpurun_out/r6_s2v_dl.err || { tail -20 gpurun_out/r6_s2v_dl.err; exit 1; }
  grep "of which" gpurun_out/r6_s2v_dl.err | tail -1
  python3 -c "
import json; d = json.load(open('gpurun_out/r6_s2v_dl.json')); c = d['config']
print('31-batch leg value %.4g single pass %.3f s steady %.4g' % (d['value'], c['setup_s']['single_pass'], c['steady_state']['value']))"
done
K=single_pass timeout -k 10 300 python -u -m pytest tests/test_s2v_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "single_pass or full_rank or short" 2>&1 | tail -2
