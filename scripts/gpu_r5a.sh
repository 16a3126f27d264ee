#!/bin/bash
# Round 5: the N>1 legs / RCCL guard / ADVICE fixes on the GPU, then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_bench_gpu.py tests/test_compat.py tests/test_route_gpu.py tests/test_lr_gpu.py -m gpu -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r5a_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r5a_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python bench.py > gpurun_out/r5a_bench.log 2>&1 || { tail -30 gpurun_out/r5a_bench.log; exit 1; }
grep '^{' gpurun_out/r5a_bench.log | tail -1 > gpurun_out/r5a_bench.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5a_bench.json"))
print("value %.4g ms/step %.3f frac %.3f" % (d["value"], d["ms_per_step"], d["roofline"]["frac"]))
for k in ("config4", "lr", "s2v"):
    v = d.get(k) or {}
    print(k, "%.4g" % v.get("value", 0), v.get("ms_per_step"), (v.get("config") or {}).get("setup_s"), (v.get("config") or {}).get("end_to_end", {}).get("value"))
print("b100", (d.get("minibatch_100") or {}).get("value"))
PY
exit $rc
