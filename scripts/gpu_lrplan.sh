#!/bin/bash
# LR: the plan / fixed-point tests, then the lr leg per mode, and a kernel summary of the fixed-point step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_lr_gpu.py -m gpu -v -x -p no:cacheprovider -rf --timeout 300 --timeout-method thread -k "${PYTEST_K:-plan or fixed or fast_sums or config3}" > gpurun_out/lrplan_tests.log 2>&1
rc=$?; tail -6 gpurun_out/lrplan_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run() {  # tag plan [VAR=value ...]
  tag=$1; plan=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --app lr --lr-plan $plan --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrplan_bench_$tag.log 2>&1 || { tail -20 gpurun_out/lrplan_bench_$tag.log; exit 1; }
  grep '^{' gpurun_out/lrplan_bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', '%.4g' % d['value'], '%.4f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['kernel_ms'].items()}, d['config']['setup_s'], d['config']['end_to_end']['value'])"
}
run none none SWPS_X=1
run place1 none SWPS_LR_PLACE=1
run place2 none SWPS_LR_PLACE=2
run none_b none SWPS_X=2
run place1b none SWPS_LR_PLACE=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lrplan_prof -o run -- python3 bench.py --app lr --lr-plan none --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/lrplan_prof.log 2>&1 || exit 1
f=$(find gpurun_out/lrplan_prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/lrplan_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/lrplan_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print("%-70s %6s %8.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
exit $rc
