#!/bin/bash
# Sharded-path bench lines on one GPU: world 1 over RCCL (Python driver and
# the library's own driver), then 2 ranks sharing the GPU (gloo / the
# library's TCP transport).  Output: gpurun_out/sh_*.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="--steps 10 --warmup 2 --no-cpu-baseline --no-parity-leg --b100-steps 0"
run() { local n=$1; shift; echo "== $n"; timeout -k 10 400 "$@" > gpurun_out/sh_$n.log 2>&1; local rc=$?; grep -h '^{' gpurun_out/sh_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(n if False else '', '%.4g words/s %.2f ms/step' % (d['value'], d['ms_per_step']), d['config']['parallelism'], d.get('exchange'))" 2>/dev/null; return $rc; }
run py1 python bench.py --sharded $B || exit $?
run nat1 python bench.py --sharded --driver native $B || exit $?
run nat2 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --driver native $B || exit $?
run py2 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 2 $B || exit $?
