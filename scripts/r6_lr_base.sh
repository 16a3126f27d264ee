#!/bin/bash
# round 6: LR baseline on the current tree — the lr leg twice and a rocprof kernel summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  timeout -k 10 300 python bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r6_lr_base_$i.log 2>&1 || { tail -20 gpurun_out/r6_lr_base_$i.log; exit 1; }
  grep '^{' gpurun_out/r6_lr_base_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$i', '%.4g' % d['value'], '%.4f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['kernel_ms'].items()})"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6lrb -o run -- python3 bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r6_lr_prof.log 2>&1 || exit 1
f=$(find gpurun_out/r6lrb -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/r6_lr_base_kernel_stats.csv
rm -rf gpurun_out/r6lrb
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r6_lr_base_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:10]:
    print("%-70s %6s %8.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
