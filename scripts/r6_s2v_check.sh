#!/bin/bash
# round 6: sent2vec tests, then the s2v leg (single pass) with its load phases
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_s2v_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread ${K:+-k "$K"} > gpurun_out/r6_s2v_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r6_s2v_tests.log | tail -30
[ $rc -ne 0 ] && exit $rc
for args in "--app s2v --steps 31 --warmup 31" "--app s2v --steps 62 --warmup 62 --s2v-docs 8192"; do
  SWPS_S2V_LOAD_TIMES=1 timeout -k 10 300 python bench.py $args --no-cpu-baseline > gpurun_out/r6_s2v_leg.json 2> gpurun_out/r6_s2v_leg.err || { tail -20 gpurun_out/r6_s2v_leg.err; exit 1; }
  grep "s2v load" gpurun_out/r6_s2v_leg.err | tail -4
  python3 -c "
import json; d = json.load(open('gpurun_out/r6_s2v_leg.json')); c = d['config']
print('$args', 'value %.4g ms/step %.3f setup %s steady %.4g frac %.3f' % (d['value'], d['ms_per_step'], c['setup_s'], c['steady_state']['value'], d['roofline']['frac']))"
done
