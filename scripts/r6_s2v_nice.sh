#!/bin/bash
# sent2vec single pass: plan workers' niceness A/B (SWPS_S2V_NICE), interleaved, on the 62-minibatch leg
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do for n in 0 10 19; do
  SWPS_S2V_NICE=$n SWPS_S2V_LOAD_TIMES=1 timeout -k 10 300 python bench.py --app s2v --steps 31 --warmup 31 --no-cpu-baseline > gpurun_out/s2vn_$n.json 2> gpurun_out/s2vn_$n.err || { tail -20 gpurun_out/s2vn_$n.err; exit 1; }
  python3 -c "
import json; d = json.load(open('gpurun_out/s2vn_$n.json')); print('nice $n value %.4g' % d['value'])"
  grep "of which" gpurun_out/s2vn_$n.err | tail -1
done; done
