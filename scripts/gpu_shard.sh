#!/bin/bash
# sharded-path checks: multi-rank gloo parity (fp64, fp32 parity, fp32 fast),
# world-1 RCCL parity, and the sharded bench at N=1 over RCCL.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step dist2_fast 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29515 tests/dist_w2v_check.py --backend gloo --dtype f32 --fast || exit $?
step dist2_f64 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tests/dist_w2v_check.py --backend gloo --dtype f64 || exit $?
step bench_sharded1_nccl 600 python bench.py --sharded --steps 20 --warmup 3 --no-cpu-baseline --no-parity-leg || exit $?
step pytest_w2v 600 python -m pytest tests/test_w2v_gpu.py tests/test_table_gpu.py tests/test_compat.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread
