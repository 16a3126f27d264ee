#!/bin/bash
# LR: the forward's bit-identity tests, then a same-box A/B of k_lr_forward_c (SWPS_LR_FWD_C=1) vs
# k_lr_forward_g (=0), two interleaved repetitions each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
[ -z "$NO_TESTS" ] && timeout -k 10 600 python -u -m pytest tests/test_lr_gpu.py tests/test_order_fixture.py -q -p no:cacheprovider -rf --timeout 240 --timeout-method thread > gpurun_out/lr_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lr_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do
  for v in ${VARIANTS:-1 0}; do
    env ${AB_VAR:-SWPS_LR_FWD_C}=$v timeout -k 10 200 python bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrab_${v}_${r}.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; o=r['other']; print(sys.argv[2], 'value %.4g ms %.4f push %.2f us fwd %.2f us' % (d['value'], d['ms_per_step'], r['avg_launch_ms']*1e3 if 'tiles' in r['kernel'] else o['avg_launch_ms']*1e3, o['avg_launch_ms']*1e3 if 'tiles' in r['kernel'] else r['avg_launch_ms']*1e3))" gpurun_out/lrab_${v}_${r}.json "${AB_VAR:-SWPS_LR_FWD_C}=$v rep $r"
  done
done
exit $rc
