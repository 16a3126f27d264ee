#!/bin/bash
# round 6: the LR leg's rocprof summary + PMC passes (final kernels), then the world-1 sharded LR step's
# kernel summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r06 LEGS=lr bash scripts/gpu_profile.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lrsh -o run -- python3 bench.py --app lr --sharded --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrsh.log 2>&1 || exit 1
cp gpurun_out/lrsh/run_kernel_stats.csv gpurun_out/profiles_r06/r06_lr_sharded_w1_kernel_stats.csv
grep '^{' gpurun_out/lrsh.log | tail -1 > gpurun_out/profiles_r06/r06_bench_lr_sharded_w1_traced.json
rm -rf gpurun_out/lrsh
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/profiles_r06/r06_lr_sharded_w1_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print("%-70s %6s %8.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
