#!/bin/bash
# A/B of two in-tree builds on one box: swiftmpi_amd/lib/ab/libswps_base.so
# (baseline) vs swiftmpi_amd/lib/libswps.so (current), alternating runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  SWPS_LIB=$PWD/swiftmpi_amd/lib/ab/libswps_base.so timeout -k 10 300 python bench.py --no-cpu-baseline $AB_ARGS > gpurun_out/ab_base_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-cpu-baseline $AB_ARGS > gpurun_out/ab_cur_$i.log 2>&1 || exit $?
done
for f in gpurun_out/ab_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel_ms"]; print(round(d["value"]/1e6,1), round(d["ms_per_step"],2), "fwd", round(d["roofline"]["avg_launch_ms"],3), "gather", round(k["gather"]/d["steps"],3), "parity", round((d.get("parity_mode") or {}).get("value",0)/1e6,1))')"; done
