#!/bin/bash
# the owner's push fused with its next serve (swps_lr_serve_push_pull): LR sharded tests, the 2-rank
# IPC/TCP check, the 4-rank IPC test, then the world-1 protocol step with and without the fusion
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_lr_gpu.py -m gpu -x -q -p no:cacheprovider -k "sharded or fixed_point or shard" --timeout 200 --timeout-method thread > gpurun_out/ps_tests.log 2>&1 || { tail -30 gpurun_out/ps_tests.log; exit 1; }
tail -1 gpurun_out/ps_tests.log
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 tests/dist_ipc_check.py --tcp-port 29581 > gpurun_out/ps_ipc.log 2>&1 || { tail -30 gpurun_out/ps_ipc.log; exit 1; }
grep -E "lr|IPC OK" gpurun_out/ps_ipc.log | tail -6
timeout -k 10 600 python -u -m pytest tests/test_route_gpu.py tests/test_bench_gpu.py -m gpu -x -q -p no:cacheprovider -k "ipc or every_leg or gpus1" --timeout 450 --timeout-method thread > gpurun_out/ps_route.log 2>&1 || { tail -30 gpurun_out/ps_route.log; exit 1; }
tail -1 gpurun_out/ps_route.log
for f in 1 0 1 0; do
  SWPS_PULL_IN_PLACE=0 SWPS_LR_PUSH_SERVE=$f timeout -k 10 300 python bench.py --app lr --sharded --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ps_b$f.log 2>&1 || { tail -20 gpurun_out/ps_b$f.log; exit 1; }
  grep '^{' gpurun_out/ps_b$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('push_serve=$f', '%.4g' % d['value'], '%.4f' % d['ms_per_step'])"
done
