#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_w2v_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k overlapped > gpurun_out/ov2_tests.log 2>&1 || { tail -20 gpurun_out/ov2_tests.log; exit 1; }
tail -1 gpurun_out/ov2_tests.log
H="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-leg --b100-steps 0 --config1-steps 0 --no-app-legs"
B="--gpus 1 --steps 200 --warmup 10 --minibatch 100 --no-cpu-baseline --no-parity-leg --config1-steps 0 --no-app-legs"
for rep in 1 2; do
for ov in 0 2 1; do
SWPS_OVERLAP=$ov timeout -k 10 300 python bench.py $H > gpurun_out/ov2_h.log 2>&1 || { tail -20 gpurun_out/ov2_h.log; exit 1; }
grep '^{' gpurun_out/ov2_h.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B5000 ov$ov', '%.4g' % d['value'], '%.3f' % d['ms_per_step'])"
done
for ov in 1 2; do
SWPS_OVERLAP=$ov timeout -k 10 300 python bench.py $B > gpurun_out/ov2_b.log 2>&1 || { tail -20 gpurun_out/ov2_b.log; exit 1; }
grep '^{' gpurun_out/ov2_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B100 ov$ov', '%.4g' % d['value'], '%.4f' % d['ms_per_step'])"
done
done
