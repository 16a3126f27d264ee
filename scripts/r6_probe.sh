#!/bin/bash
# round 6: the world-1 sharded LR step (the N > 1 base point), then the B = 100 kernel timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  timeout -k 10 300 python bench.py --app lr --sharded --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r6_lr_sh_$i.json 2> gpurun_out/r6_lr_sh_$i.err || { tail -20 gpurun_out/r6_lr_sh_$i.err; exit 1; }
  python3 -c "
import json; d = json.load(open('gpurun_out/r6_lr_sh_$i.json'))
print('sharded w1', '%.4g' % d['value'], '%.4f ms' % d['ms_per_step'], {k: round(v, 3) for k, v in d['kernel_ms'].items()})"
done
bash scripts/b100_trace.sh || exit 1
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/b100_timeline.csv")))
iv = sorted((int(r["start"]), int(r["end"]), r["name"]) for r in rows)
fw = [i for i, x in enumerate(iv) if "k_forward" in x[2]]
tot_gap = tot_span = 0; steps = 0
for s0, s1 in zip(fw[:-1], fw[1:]):
    t0, t1 = iv[s0][0], iv[s1][0]
    seg = sorted((max(a, t0), min(b, t1)) for a, b, n in iv if b > t0 and a < t1)
    busy = 0; cur = t0
    for a, b in seg:
        if b <= cur: continue
        busy += b - max(a, cur); cur = b
    tot_gap += (t1 - t0) - busy; tot_span += t1 - t0; steps += 1
print("B=100 traced: steps %d mean step %.1f us, GPU idle (no kernel on any queue) %.1f us per step, launches/step %.1f"
      % (steps, tot_span / steps / 1e3, tot_gap / steps / 1e3, (fw[-1] - fw[0]) / steps))
PY
