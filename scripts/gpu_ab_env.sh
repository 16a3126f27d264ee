#!/bin/bash
# same-box A/B of one environment knob on the headline and B = 100 legs: AB_VAR, AB_VALUES, AB_REPS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in $(seq 1 ${AB_REPS:-2}); do
  for v in ${AB_VALUES}; do
    env ${AB_VAR}=$v timeout -k 10 300 python bench.py --no-app-legs --no-parity-leg --config1-steps 0 \
      --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab_$v.$rep.json 2> gpurun_out/ab_$v.$rep.log || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/ab_$v.$rep.json').read().strip().splitlines()[-1]); b=d.get('minibatch_100') or {}; print('${AB_VAR}=$v rep $rep', d['value'], d['ms_per_step'], b.get('value'), b.get('ms_per_step'), d['kernel_ms'].get('push'), d['kernel_ms'].get('gather'))"
  done
done
