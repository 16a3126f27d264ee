#!/bin/bash
# SQ wave-state summaries (scripts/gpu_sq.sh) of the LR, headline and B = 100 bench
# commands, copied to profiles/${TAG}_sq_<leg>.json.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04}
mkdir -p gpurun_out/profiles_$TAG
W2V="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-leg --b100-steps 0 --config1-steps 0 --no-app-legs"
for L in ${LEGS:-lr w2v_bfp32 w2v_b100}; do
  case $L in
    lr) NAME=lr N=20 bash scripts/gpu_sq.sh bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline || exit $? ;;
    w2v_bfp32) NAME=w2v_bfp32 N=20 bash scripts/gpu_sq.sh $W2V || exit $? ;;
    w2v_b100) NAME=w2v_b100 N=200 bash scripts/gpu_sq.sh bench.py --gpus 1 --steps 200 --warmup 10 --minibatch 100 \
                --no-cpu-baseline --no-parity-leg --config1-steps 0 --no-app-legs || exit $? ;;
    *) echo "unknown leg $L"; exit 2 ;;
  esac
  cp gpurun_out/sq_$L.json gpurun_out/profiles_$TAG/${TAG}_sq_$L.json
done
