#!/bin/bash
# the world-1 sharded LR step's dispatch timeline (last 120 dispatches of every kind, by start)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/lrsht -o run -- python3 bench.py --app lr --sharded --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lrsht.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
ev = []
for f in glob.glob("gpurun_out/lrsht/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60], "K", r.get("Queue_Id", "")))
for f in glob.glob("gpurun_out/lrsht/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "copy") + " " + r.get("Bytes", r.get("Size", "")), "M", ""))
ev.sort()
tail = ev[-160:]
t0 = tail[0][0]
with open("gpurun_out/r06_lr_sharded_w1_timeline.csv", "w") as o:
    w = csv.writer(o)
    w.writerow(["t_us", "dur_us", "kind", "name", "queue"])
    for a, b, n, k, q in tail:
        w.writerow(["%.2f" % ((a - t0) / 1e3), "%.2f" % ((b - a) / 1e3), k, n, q])
for a, b, n, k, q in tail[-40:]:
    print("%9.2f %7.2f %s %-60s %s" % ((a - t0) / 1e3, (b - a) / 1e3, k, n, q))
PY
rm -rf gpurun_out/lrsht
