#!/bin/bash
# Diagnostics (one GPU session): B = 100 host-API + kernel trace (is the GPU waiting for the host?),
# LR kernel trace, SQ counters of the LR and B = 100 kernels.  Outputs under gpurun_out/diag/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/diag
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$R"
B100="bench.py --steps 30 --warmup 5 --minibatch 100 --no-cpu-baseline --no-parity-leg --config1-steps 0 --b100-steps 0 --no-app-legs"
LR="bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline"
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 $to "$@" > gpurun_out/diag/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; return $rc; }
if [ -z "$SKIP_API" ]; then
step b100_api 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/diag/b100api -o run -- python3 $B100 || exit $?
python3 scripts/api_timeline.py gpurun_out/diag/b100api > gpurun_out/diag/b100_api_timeline.txt 2>&1 || exit $?
rm -rf gpurun_out/diag/b100api
fi
if [ -z "$SKIP_LR" ]; then
step lr_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/diag/lrt -o run -- python3 $LR || exit $?
python3 scripts/trace_summary.py gpurun_out/diag/lrt > gpurun_out/diag/lr_timeline.txt 2>&1 || exit $?
cp gpurun_out/diag/lrt/run_kernel_stats.csv gpurun_out/diag/lr_kernel_stats.csv 2>/dev/null
rm -rf gpurun_out/diag/lrt
NAME=lr N=20 bash scripts/gpu_sq.sh $LR || exit $?
fi
if [ -z "$SKIP_SQB" ]; then
NAME=b100 N=30 bash scripts/gpu_sq.sh $B100 || exit $?
fi
ls gpurun_out/diag gpurun_out/sq_*.json
