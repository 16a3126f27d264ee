#!/bin/bash
# the B = 100 timeline: mean step and the time no kernel runs on any queue, per step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/b100_trace.sh || exit 1
python3 - <<'PY'
import csv, json
rows = list(csv.DictReader(open("gpurun_out/b100_timeline.csv")))
iv = sorted((int(r["start"]), int(r["end"]), r["name"]) for r in rows)
fw = [i for i, x in enumerate(iv) if "k_forward" in x[2]]
tot_gap = tot_span = 0; steps = 0; gaps = []
for s0, s1 in zip(fw[:-1], fw[1:]):
    t0, t1 = iv[s0][0], iv[s1][0]
    seg = sorted((max(a, t0), min(b, t1)) for a, b, n in iv if b > t0 and a < t1)
    busy = 0; cur = t0
    for a, b in seg:
        if b <= cur: continue
        busy += b - max(a, cur); cur = b
    gaps.append(((t1 - t0) - busy) / 1e3)
    tot_gap += (t1 - t0) - busy; tot_span += t1 - t0; steps += 1
out = {"steps": steps, "mean_step_us": tot_span / max(steps, 1) / 1e3, "idle_us_per_step": tot_gap / max(steps, 1) / 1e3,
       "launches_per_step": (fw[-1] - fw[0]) / max(steps, 1), "idle_us": gaps}
print("B=100 traced:", json.dumps({k: v for k, v in out.items() if k != "idle_us"}))
json.dump(out, open("gpurun_out/r06_b100_gaps.json", "w"))
PY
