#!/bin/bash
# the world-1 sharded LR step in its two forms (in place, default; the full protocol,
# SWPS_PULL_IN_PLACE=0): rocprof kernel summaries + the bench lines they come from
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles_r06
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for form in inplace protocol; do
  if [ $form = protocol ]; then export SWPS_PULL_IN_PLACE=0; else export SWPS_PULL_IN_PLACE=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lrsh_$form -o run -- python3 bench.py --app lr --sharded --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrsh_$form.log 2>&1 || exit 1
  cp gpurun_out/lrsh_$form/run_kernel_stats.csv gpurun_out/profiles_r06/r06_lr_sharded_w1_${form}_kernel_stats.csv
  grep '^{' gpurun_out/lrsh_$form.log | tail -1 > gpurun_out/profiles_r06/r06_bench_lr_sharded_w1_${form}_traced.json
  rm -rf gpurun_out/lrsh_$form
  python3 - $form <<'PY'
import csv, json, sys
f = sys.argv[1]
rows = list(csv.DictReader(open("gpurun_out/profiles_r06/r06_lr_sharded_w1_%s_kernel_stats.csv" % f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
d = json.load(open("gpurun_out/profiles_r06/r06_bench_lr_sharded_w1_%s_traced.json" % f))
print(f, "%.4g ex/s %.4f ms" % (d["value"], d["ms_per_step"]))
for r in rows[:10]:
    print("  %-70s %6s %8.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
