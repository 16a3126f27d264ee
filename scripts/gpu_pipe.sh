#!/bin/bash
# sharded w2v: lockstep + pipelined parity/determinism, multi-rank gloo, RCCL world-1 bench both drivers.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step pytest_w2v 600 python -m pytest tests/test_w2v_gpu.py -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread -s -k "pipelined or sharded or single_batch or train_f"
step dist2_fast 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29515 tests/dist_w2v_check.py --backend gloo --dtype f32 --fast || exit $?
step dist3_pipe 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29516 tests/dist_w2v_check.py --backend gloo --dtype f32 --fast --pipeline || exit $?
step dist2_lr 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 tests/dist_lr_check.py --backend gloo || exit $?
step bench_sharded1_lock 600 python bench.py --sharded --steps 20 --warmup 3 --no-cpu-baseline --no-parity-leg || exit $?
step bench_sharded1_pipe 600 python bench.py --sharded --pipeline --steps 20 --warmup 3 --no-cpu-baseline --no-parity-leg || exit $?
