#!/bin/bash
# Same-box A/B of library env settings: the GPU tests named in $TESTS (if any),
# then the default bench (B = 5000 + its B = 100 leg) once per variant, REPS
# rounds interleaved.  Variants are ';'-separated env assignments:
#   VARIANTS="SWPS_FUSED_PUSH=0;SWPS_FUSED_PUSH=1" REPS=2 bash scripts/gpu_ab.sh
# (an unused name such as SWPS_NOP=1 stands for the defaults)
# Stops at the first GPU fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rc=0
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TO:-500} python -u -m pytest $TESTS -m gpu -q -p no:cacheprovider -rf --timeout 240 --timeout-method thread ${K:+-k "$K"} > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
IFS=';' read -ra VS <<< "${VARIANTS:-SWPS_FUSED_PUSH=1}"
for r in $(seq 1 ${REPS:-1}); do
  i=0
  for v in "${VS[@]}"; do
    i=$((i + 1))
    env $v timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-parity-leg ${BENCH_ARGS} > gpurun_out/ab_${r}_${i}.log 2>&1 || exit $?
    V="$v" python3 - gpurun_out/ab_${r}_${i}.log <<'PY'
import json, os, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
b = d.get("minibatch_100") or {}
r = d["roofline"]
km = d.get("kernel_ms", {})
n = max(r.get("launches", 1), 1)
print("%-40s %.4g w/s %.3f ms | b100 %s %s | frac %.3f sum %.3f ms (g %.3f p %.3f) sort %.3f rec %.3f fwd %.3f" % (
    os.environ["V"], d["value"], d["ms_per_step"], b.get("value") and "%.4g" % b["value"],
    b.get("ms_per_step") and "%.4f" % b["ms_per_step"], r["frac"], r["avg_launch_ms"],
    r.get("gather_ms_per_launch", 0), r.get("push_ms_per_launch", 0), km.get("sort", 0) / n,
    km.get("records", 0) / n, km.get("forward", 0) / n), flush=True)
PY
  done
done
exit $rc
