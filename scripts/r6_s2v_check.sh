#!/bin/bash
# sent2vec: the GPU tests, then the single pass's phases on the 62-minibatch leg (2 reps)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_s2v_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s2vc_tests.log 2>&1 || { tail -30 gpurun_out/s2vc_tests.log; exit 1; }
tail -2 gpurun_out/s2vc_tests.log
for rep in 1 2; do
  SWPS_S2V_LOAD_TIMES=1 timeout -k 10 300 python bench.py --app s2v --steps 31 --warmup 31 --no-cpu-baseline > gpurun_out/s2vc_$rep.json 2> gpurun_out/s2vc_$rep.err || { tail -20 gpurun_out/s2vc_$rep.err; exit 1; }
  python3 -c "
import json; d = json.load(open('gpurun_out/s2vc_$rep.json')); print('value %.4g steady %.4g' % (d['value'], d['config']['steady_state']['value']))"
  grep "of which" gpurun_out/s2vc_$rep.err | tail -1
done
