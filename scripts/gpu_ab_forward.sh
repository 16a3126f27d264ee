#!/bin/bash
# A/B of forward-kernel variants selected by env var $AB_VAR, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-leg > gpurun_out/ab_base_$i.log 2>&1 || exit $?
  env $AB_VAR=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-leg > gpurun_out/ab_var_$i.log 2>&1 || exit $?
done
for f in gpurun_out/ab_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), round(d["ms_per_step"],2), round(d["roofline"]["avg_launch_ms"],3))')"; done
