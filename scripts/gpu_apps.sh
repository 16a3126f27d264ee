#!/bin/bash
# LR / sent2vec paths: GPU tests, multi-rank sharded LR parity, config-3/5 bench legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step dist2_lr 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 tests/dist_lr_check.py --backend gloo || exit $?
step dist3_lr 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29522 tests/dist_lr_check.py --backend gloo || exit $?
step dist1_lr_nccl 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29523 tests/dist_lr_check.py --backend nccl || exit $?
step pytest_apps 600 python -m pytest tests/test_lr_gpu.py tests/test_s2v_gpu.py -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread -rA
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench_lr 600 python bench.py --app lr --steps 20 --warmup 3 || exit $?
step bench_lr_sharded1 600 python bench.py --app lr --sharded --steps 20 --warmup 3 || exit $?
step bench_s2v 600 python bench.py --app s2v --steps 10 --warmup 2 || exit $?
