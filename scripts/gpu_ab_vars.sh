#!/bin/bash
# A/B over values of an env var: AB_NAME=<var> AB_VALS="0 1 2 ..." (one bench run each, same box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in $AB_VALS; do
  env $AB_NAME=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity-leg $AB_ARGS > gpurun_out/abv_$v.log 2>&1 || exit $?
done
for v in $AB_VALS; do echo "$AB_NAME=$v $(tail -1 gpurun_out/abv_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel_ms"]; print(round(d["value"]/1e6,1), round(d["ms_per_step"],2), {a: round(b/d["steps"],3) for a,b in k.items()})')"; done
