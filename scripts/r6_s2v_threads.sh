#!/bin/bash
# the s2v single pass at several plan-worker counts (SWPS_S2V_THREADS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
for th in ${THREADS:-16 14 12 8}; do
  SWPS_S2V_THREADS=$th SWPS_S2V_LOAD_TIMES=1 timeout -k 10 300 python bench.py --app s2v --steps 31 --warmup 31 --no-cpu-baseline > gpurun_out/r6_s2v_th.json 2> gpurun_out/r6_s2v_th.err || { tail -20 gpurun_out/r6_s2v_th.err; exit 1; }
  grep "of which" gpurun_out/r6_s2v_th.err | tail -1
  python3 -c "
import json; d = json.load(open('gpurun_out/r6_s2v_th.json')); c = d['config']
print('threads $th value %.4g single pass %.3f s' % (d['value'], c['setup_s']['single_pass']))"
done
