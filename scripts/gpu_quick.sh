#!/bin/bash
# Quick GPU check of a kernel change: the w2v GPU tests, then the default
# bench line (with its B = 100 leg).  Stops at the first GPU fault / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_w2v_gpu.py tests/test_bench_shape_gpu.py tests/test_snapshot_gpu.py -m gpu -q -p no:cacheprovider -rf --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/quick_bench.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/quick_bench.log") if l.startswith("{")][-1])
print("value %.4g ms/step %.3f frac %.3f" % (d["value"], d["ms_per_step"], d["roofline"]["frac"]), "traffic", d["roofline"].get("traffic"))
print("b100", d.get("minibatch_100", {}).get("value"), d.get("minibatch_100", {}).get("ms_per_step"))
print("kernel_ms", d.get("kernel_ms"))
PY
exit $rc
