#!/bin/bash
# LR: the GPU tests named in $TESTS (default: the LR tests), then a same-box A/B of library env
# settings on the Criteo bench step, REPS interleaved repetitions.  Variants are ';'-separated
# env assignments ("-" = none):
#   VARIANTS="SWPS_LR_PLACE=0 SWPS_LR_XCD=0;-" REPS=2 bash scripts/lr_env_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rc=0
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TO:-600} python -u -m pytest ${TESTS:-tests/test_lr_gpu.py tests/test_order_fixture.py} -q -p no:cacheprovider -rf --timeout 240 --timeout-method thread ${K:+-k "$K"} > gpurun_out/lr_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/lr_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
IFS=';' read -ra VS <<< "${VARIANTS:--}"
for r in $(seq 1 ${REPS:-2}); do
  i=0
  for v in "${VS[@]}"; do
    i=$((i + 1))
    e=$v; [ "$v" = "-" ] && e=""
    env $e timeout -k 10 200 python bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrab_${i}_${r}.json 2>/dev/null || exit $?
    python3 -c "
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']; o = r['other']
print('%-40s value %.4g ms %.4f push %.2f us fwd %.2f us' % (sys.argv[2], d['value'], d['ms_per_step'], r['avg_launch_ms'] * 1e3, o['avg_launch_ms'] * 1e3))
" gpurun_out/lrab_${i}_${r}.json "$v rep $r"
  done
done
exit $rc
