#!/bin/bash
# round 6: sent2vec load phases (SWPS_S2V_LOAD_TIMES) on the bench's s2v leg shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
SWPS_S2V_LOAD_TIMES=1 timeout -k 10 300 python bench.py --app s2v --steps 31 --warmup 31 --no-cpu-baseline > gpurun_out/r6_s2v_phases.json 2> gpurun_out/r6_s2v_phases.err || { tail -20 gpurun_out/r6_s2v_phases.err; exit 1; }
grep "s2v load" gpurun_out/r6_s2v_phases.err
python3 -c "
import json; d = json.load(open('gpurun_out/r6_s2v_phases.json')); c = d['config']
print('value %.4g setup %s e2e %.4g' % (d['value'], c['setup_s'], c['end_to_end']['value']))"
