#!/bin/bash
# LR push row prefetch: the default (dense buckets only) vs every bucket (SWPS_LR_FX_PF=2), on the
# default line's lr leg (10-batch corpus) and --app lr (43 batches), 2 interleaved reps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LINE="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity-leg --b100-steps 0 --config1-steps 0 --config4-steps 0 --no-lr-sharded-base"
for rep in 1 2; do for pf in 1 2; do
  SWPS_LR_FX_PF=$pf timeout -k 10 400 python $LINE > gpurun_out/pf_line_$pf.log 2>&1 || { tail -5 gpurun_out/pf_line_$pf.log; exit 1; }
  SWPS_LR_FX_PF=$pf timeout -k 10 300 python bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/pf_app_$pf.log 2>&1 || { tail -5 gpurun_out/pf_app_$pf.log; exit 1; }
  python3 - $pf $rep <<'PY'
import json, sys
pf, rep = sys.argv[1], sys.argv[2]
a = json.loads([l for l in open("gpurun_out/pf_line_%s.log" % pf) if l.startswith("{")][-1])["lr"]
b = json.loads([l for l in open("gpurun_out/pf_app_%s.log" % pf) if l.startswith("{")][-1])
print("pf %s rep %s: line lr %.2f us, --app lr %.2f us" % (pf, rep, a["ms_per_step"] * 1e3, b["ms_per_step"] * 1e3))
PY
done; done
