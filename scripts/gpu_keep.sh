#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_w2v_gpu.py tests/test_ingest_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/keep_tests.log 2>&1 || { tail -20 gpurun_out/keep_tests.log; exit 1; }
tail -1 gpurun_out/keep_tests.log
for r in 1 2; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-leg --b100-steps 0 --config1-steps 0 --no-app-legs > gpurun_out/keep_bench.log 2>&1 || { tail -20 gpurun_out/keep_bench.log; exit 1; }
grep '^{' gpurun_out/keep_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('headline', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/keep_prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-leg --b100-steps 0 --config1-steps 0 --no-app-legs > gpurun_out/keep_prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/keep_prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_keep" in r["Name"]: print(r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3, "us")
PY
