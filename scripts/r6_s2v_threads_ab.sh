#!/bin/bash
# sent2vec single pass: plan workers A/B (SWPS_S2V_THREADS), interleaved, 62-minibatch leg
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do for n in 8 12 16; do
  SWPS_S2V_THREADS=$n timeout -k 10 300 python bench.py --app s2v --steps 31 --warmup 31 --no-cpu-baseline > gpurun_out/s2vt_$n.json 2> gpurun_out/s2vt_$n.err || { tail -20 gpurun_out/s2vt_$n.err; exit 1; }
  python3 -c "
import json; d = json.load(open('gpurun_out/s2vt_$n.json')); print('threads $n rep $rep value %.4g' % d['value'])"
done; done
