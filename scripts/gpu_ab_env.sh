#!/bin/bash
# A/B of an env-var-selected variant ($AB_VAR=1) on one box, alternating runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-leg $AB_ARGS > gpurun_out/ab_base_$i.log 2>&1 || exit $?
  env ${AB_ENV:-$AB_VAR=1} timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-leg $AB_ARGS > gpurun_out/ab_var_$i.log 2>&1 || exit $?
done
for f in gpurun_out/ab_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel_ms"]; print(round(d["value"]/1e6,1), round(d["ms_per_step"],2), {a: round(b/d["steps"],3) for a,b in k.items()})')"; done
