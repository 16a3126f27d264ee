#!/bin/bash
# sent2vec single pass, 62- and the line's 31-minibatch legs, 3 reps (SWPS_S2V_LOAD_TIMES phases)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3; do
  SWPS_S2V_LOAD_TIMES=1 timeout -k 10 300 python bench.py --app s2v --steps 31 --warmup 31 --no-cpu-baseline > gpurun_out/s2vab_$rep.json 2> gpurun_out/s2vab_$rep.err || { tail -20 gpurun_out/s2vab_$rep.err; exit 1; }
  python3 -c "
import json; d = json.load(open('gpurun_out/s2vab_$rep.json')); print('rep $rep value %.4g' % d['value'])"
  grep "plans 0..15" gpurun_out/s2vab_$rep.err | tail -1 | cut -c1-160
done
