#!/bin/bash
# Same-box A/B of LR env settings on the config-3 bench: VARIANTS="A=0;A=1" REPS=2 bash scripts/lr_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS}"
for r in $(seq 1 ${REPS:-1}); do
  i=0
  for v in "${VS[@]}"; do
    i=$((i + 1))
    env $v timeout -k 10 200 python bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrab_${r}_${i}.log 2>&1 || exit $?
    V="$v" python3 - gpurun_out/lrab_${r}_${i}.log <<'PY'
import json, os, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
o = r["other"]
print("%-28s %.4g ex/s %.4f ms | %s %.4f ms | %s %.4f ms" % (os.environ["V"], d["value"], d["ms_per_step"], r["kernel"][:24],
      r["avg_launch_ms"], o["kernel"][:24], o["avg_launch_ms"]), flush=True)
PY
  done
done
