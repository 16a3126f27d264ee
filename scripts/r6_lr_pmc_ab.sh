#!/bin/bash
# LR fixed-point step: PMC traffic (read requests by size + WRITE_SIZE) and step time per variant
# of the push's row prefetch (SWPS_LR_FX_PF) and the dense weight copy (SWPS_LR_FX_MIRROR)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lrab
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$R"
READS="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
CMD="bench.py --app lr --steps 20 --warmup 3 --no-cpu-baseline"
for v in "default:" "pf0:SWPS_LR_FX_PF=0" "pf2:SWPS_LR_FX_PF=2" "nomir:SWPS_LR_FX_MIRROR=0"; do
  name=${v%%:*}; envs=${v#*:}
  export SWPS_LR_FX_PF= SWPS_LR_FX_MIRROR=
  unset SWPS_LR_FX_PF SWPS_LR_FX_MIRROR
  [ -n "$envs" ] && export $envs
  timeout -k 10 300 rocprofv3 --pmc $READS --kernel-trace --output-format csv -d gpurun_out/lrab/rd_$name -o run -- python3 $CMD > gpurun_out/lrab/rd_$name.log 2>&1 || { tail -5 gpurun_out/lrab/rd_$name.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/lrab/wr_$name -o run -- python3 $CMD > gpurun_out/lrab/wr_$name.log 2>&1 || { tail -5 gpurun_out/lrab/wr_$name.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/lrab/pmc_$name.json gpurun_out/lrab/rd_$name gpurun_out/lrab/wr_$name --last 20 --cmd "python3 $CMD" --config '{"app": "lr"}' > /dev/null || exit 1
  for rep in 1 2; do
    timeout -k 10 300 python3 $CMD > gpurun_out/lrab/b_${name}_$rep.log 2>&1 || { tail -5 gpurun_out/lrab/b_${name}_$rep.log; exit 1; }
  done
  python3 - $name <<'PY'
import json, sys
n = sys.argv[1]
p = json.load(open("gpurun_out/lrab/pmc_%s.json" % n))["kernels"]
ms = []
for rep in (1, 2):
    d = json.loads([l for l in open("gpurun_out/lrab/b_%s_%d.log" % (n, rep)) if l.startswith("{")][-1])
    ms.append(d["ms_per_step"] * 1e3)
r = d["roofline"]
def find(sub):
    for k, v in p.items():
        if sub in k:
            return v["hbm_bytes"]
    return float("nan")
st, pu = find("k_lr_fxr_step"), find("k_lr_fxb_push")
print("%-8s step %.1f/%.1f us  fxr PMC %.1f MB (%.2fx of %.1f)  push PMC %.1f MB (%.2fx of %.1f)  kernel ms fwd %.3f push %.3f" % (
    n, ms[0], ms[1], st / 1e6, st / r["bytes_per_launch"], r["bytes_per_launch"] / 1e6, pu / 1e6,
    pu / r["other"]["bytes_per_launch"], r["other"]["bytes_per_launch"] / 1e6, d["kernel_ms"]["forward"], d["kernel_ms"]["push"]))
PY
  rm -rf gpurun_out/lrab/rd_$name gpurun_out/lrab/wr_$name
done
