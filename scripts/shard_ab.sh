#!/bin/bash
# Same-box A/B: unsharded vs the sharded world-1 path (library driver, RCCL), REPS rounds interleaved;
# VARIANTS: ';'-separated env settings for extra sharded runs (e.g. "SWPS_PULL_IN_PLACE=0")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A="--steps 20 --warmup 5 --no-cpu-baseline --no-parity-leg --b100-steps 0 --config1-steps 0"
IFS=';' read -ra VS <<< "${VARIANTS:-}"
for r in $(seq 1 ${REPS:-2}); do
  i=0
  for v in "plain" "sharded" "${VS[@]}"; do
    i=$((i + 1))
    if [ "$v" = plain ]; then args="$A"; envs=""; elif [ "$v" = sharded ]; then args="$A --sharded"; envs=""; else args="$A --sharded"; envs="$v"; fi
    env $envs timeout -k 10 300 python bench.py $args > gpurun_out/shab_${r}_${i}.log 2>&1 || exit $?
    python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); x=d.get('exchange') or {}
print('%-28s %.4g w/s %.3f ms exch %.3f ms' % (sys.argv[2], d['value'], d['ms_per_step'], x.get('ms_per_step') or 0))" gpurun_out/shab_${r}_${i}.log "$v"
  done
done
