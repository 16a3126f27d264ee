#!/bin/bash
# SQ wave-state counters (one --pmc pass, 8 SQ counters) of a bench command, per
# kernel (last N launches), into gpurun_out/sq_<name>.json.  WAIT_ANY (parked on
# s_waitcnt / barrier), WAIT_INST_ANY (issue stall) and ACTIVE_INST_ANY partition
# WAVE_CYCLES (MI355X_MICROARCH.md, PMC table), so the summary's parked_frac says
# how much of a wave's life is spent waiting on memory:
#   NAME=lr N=20 bash scripts/gpu_sq.sh bench.py --app lr ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
timeout -k 10 600 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/sq_$NAME -o run -- python3 "$@" > gpurun_out/sq_$NAME.log 2>&1 || exit $?
python3 scripts/pmc_summary.py gpurun_out/sq_$NAME.json gpurun_out/sq_$NAME --last ${N:-20} --cmd "python3 $*" || exit $?
rm -rf gpurun_out/sq_$NAME
