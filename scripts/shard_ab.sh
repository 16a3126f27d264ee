#!/bin/bash
# Same-box A/B: unsharded vs the sharded world-1 path (library driver, RCCL), REPS rounds interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A="--steps 20 --warmup 5 --no-cpu-baseline --no-parity-leg --b100-steps 0 --config1-steps 0"
for r in $(seq 1 ${REPS:-2}); do
  for v in "" "--sharded"; do
    timeout -k 10 300 python bench.py $A $v > gpurun_out/shab_${r}_${v:-plain}.log 2>&1 || exit $?
    python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); x=d.get('exchange') or {}
print('%-10s %.4g w/s %.3f ms exch %.3f ms' % (sys.argv[2] or 'plain', d['value'], d['ms_per_step'], x.get('ms_per_step') or 0))" gpurun_out/shab_${r}_${v:-plain}.log "$v"
  done
done
