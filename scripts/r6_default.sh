#!/bin/bash
# the driver's own command (python bench.py, no flags), its JSON line kept under gpurun_out/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python bench.py > gpurun_out/r6_default.out 2> gpurun_out/r6_default.err || { tail -30 gpurun_out/r6_default.err; exit 1; }
grep '^{' gpurun_out/r6_default.out | tail -1 > gpurun_out/r06_bench_default.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r06_bench_default.json"))
print("headline %.4g words/s  %.3f ms  frac %.3f" % (d["value"], d["ms_per_step"], d["roofline"]["frac"]))
print("b100 %.4g  config4 %.4g  config1 gpu %.4g" % (d["minibatch_100"]["value"], d["config4"]["value"], d["config1"]["gpu"]["value"]))
lr = d["lr"]; s = d["s2v"]
q = lr["sharded_world1"]
print("lr %.4g ex/s %.4f ms  sharded_w1 protocol %.4g %.4f ms  in place %.4g %.4f ms" % (lr["value"], lr["ms_per_step"], q["value"], q["ms_per_step"], q["in_place"]["value"], q["in_place"]["ms_per_step"]))
print("s2v single pass %.4g words/s, steady %.4g" % (s["value"], s["config"]["steady_state"]["value"]))
print("cpu", d["cpu_baseline"]["value"], {k: v["value"] for k, v in (d.get("other_modes") or {}).items()})
PY
