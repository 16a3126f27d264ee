#!/bin/bash
# multi-rank checks that must not run inside a process that already touched the GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step dist2_f64 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tests/dist_w2v_check.py --backend gloo --dtype f64 || exit $?
step dist3_f32 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29512 tests/dist_w2v_check.py --backend gloo --dtype f32 || exit $?
step dist2_fast 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29515 tests/dist_w2v_check.py --backend gloo --dtype f32 --fast || exit $?
step bench_n2_gloo 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 10 --warmup 2 || exit $?
step dist1_nccl 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29514 tests/dist_w2v_check.py --backend nccl --dtype f64 || exit $?
step bench_sharded1_nccl 600 python bench.py --sharded --steps 20 --warmup 3 --no-cpu-baseline --no-parity-leg || exit $?
