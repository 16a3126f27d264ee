#!/bin/bash
# world-1 sharded LR in place: the LR GPU tests touching the sharded step, the 2-rank IPC check
# (sharded fixed point over TCP / IPC, dense install), and the world-1 sharded leg in both forms
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_lr_gpu.py -m gpu -x -q -p no:cacheprovider -k "sharded or fixed_point or shard" --timeout 200 --timeout-method thread > gpurun_out/inpl_tests.log 2>&1 || { tail -30 gpurun_out/inpl_tests.log; exit 1; }
tail -2 gpurun_out/inpl_tests.log
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 tests/dist_ipc_check.py --tcp-port 29581 > gpurun_out/inpl_ipc.log 2>&1 || { tail -30 gpurun_out/inpl_ipc.log; exit 1; }
grep -E "ok|IPC OK" gpurun_out/inpl_ipc.log | tail -12
for f in 1 0 1 0; do
  SWPS_PULL_IN_PLACE=$f timeout -k 10 300 python bench.py --app lr --sharded --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/inpl_b$f.log 2>&1 || { tail -20 gpurun_out/inpl_b$f.log; exit 1; }
  grep '^{' gpurun_out/inpl_b$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('inplace=$f', '%.4g' % d['value'], '%.4f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['kernel_ms'].items()})"
done
