#!/bin/bash
# rocprof kernel stats of the LR leg with the per-step plan
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lrplan_prof -o lrplan -- python3 bench.py --app lr --lr-plan step --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/lrplan_prof.log 2>&1 || { tail -20 gpurun_out/lrplan_prof.log; exit 1; }
f=$(find gpurun_out/lrplan_prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/lrplan_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/lrplan_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:30]:
    print("%-90s %6s %10.1f us avg" % (r["Name"][:90], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
