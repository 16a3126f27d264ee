#!/bin/bash
# LR per-step plan: its bit-identity tests, the LR GPU suite, then the lr bench leg both ways
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_lr_gpu.py tests/test_order_fixture.py -m gpu -v -x -p no:cacheprovider -rf --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/lrplan_tests.log 2>&1
rc=$?; tail -12 gpurun_out/lrplan_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for plan in step load; do
  timeout -k 10 300 python bench.py --app lr --lr-plan $plan --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrplan_bench_$plan.log 2>&1 || { tail -20 gpurun_out/lrplan_bench_$plan.log; exit 1; }
  grep '^{' gpurun_out/lrplan_bench_$plan.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$plan', '%.4g' % d['value'], d['ms_per_step'], d['kernel_ms'], d['config']['setup_s'], d['config']['end_to_end']['value'])"
done
exit $rc
