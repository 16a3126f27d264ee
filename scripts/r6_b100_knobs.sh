#!/bin/bash
# B = 100: existing knobs re-measured on the final code (2 interleaved reps)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
CMD="bench.py --gpus 1 --steps 200 --warmup 10 --minibatch 100 --no-cpu-baseline --no-parity-leg --config1-steps 0 --no-app-legs --b100-steps 0"
for rep in 1 2; do
  for v in "default:" "ov2:SWPS_OVERLAP=2" "prio0:SWPS_PREP_PRIO=0" "small:SWPS_SORT_SMALL=1" "wpe1:SWPS_PUSH_WPE=1" "fwdg8:SWPS_FWD_G=8"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python $CMD > gpurun_out/b100k_$name.log 2>&1 || { tail -5 gpurun_out/b100k_$name.log; exit 1; }
    grep '^{' gpurun_out/b100k_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name rep $rep %.4g %.4f ms' % (d['value'], d['ms_per_step']))"
  done
done
