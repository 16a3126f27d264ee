#!/bin/bash
# words/s and per-kernel ms per step vs minibatch size (lines of 1000 tokens)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mb in ${MBS:-100 500 1000 2000 5000}; do
  timeout -k 10 300 python bench.py --steps $((40000/mb)) --warmup 2 --minibatch $mb --no-cpu-baseline --no-parity-leg $EXTRA > gpurun_out/mb_$mb.log 2>&1 || exit $?
  echo "mb=$mb $(tail -1 gpurun_out/mb_$mb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "Mw/s", round(d["ms_per_step"],3), "ms frac", round(d["roofline"]["frac"],3), {k: round(v/d["steps"],3) for k,v in d["kernel_ms"].items()})')"
done
