#!/bin/bash
# sent2vec single pass: kernel + copy timeline (rocprofv3), GPU busy / idle during the last pass
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/s2vt -o run -- python3 bench.py --app s2v --steps 31 --warmup 31 --no-cpu-baseline > gpurun_out/s2vt.log 2>&1 || { tail -20 gpurun_out/s2vt.log; exit 1; }
python3 - <<'PY'
import csv, glob
ev = []
for f in glob.glob("gpurun_out/s2vt/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:40], r.get("Queue_Id", "")))
for f in glob.glob("gpurun_out/s2vt/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M", r.get("Direction", "copy") + " " + str(r.get("Size", r.get("Bytes", ""))), ""))
ev.sort()
# the single passes: k_s2v_docs launches; find the 2nd pass (the timed one) = docs launches between the
# first two large gaps; simpler: print per docs launch its start, dur and the gap since the previous docs end
docs = [e for e in ev if e[2] == "K" and "k_s2v_docs" in e[3]]
print("docs launches", len(docs))
prev = None
for a, b, k, n, q in docs:
    print("%12.3f ms dur %7.3f gap %7.3f" % (a / 1e6, (b - a) / 1e6, 0 if prev is None else (a - prev) / 1e6))
    prev = b
# copies summary
cp = [e for e in ev if e[2] == "M"]
tot = sum(b - a for a, b, *_ in cp) / 1e6
print("copies", len(cp), "total ms %.2f" % tot)
with open("gpurun_out/r06_s2v_timeline.csv", "w") as o:
    w = csv.writer(o); w.writerow(["t_ms", "dur_ms", "kind", "name", "queue"])
    t0 = ev[0][0]
    for a, b, k, n, q in ev:
        w.writerow(["%.4f" % ((a - t0) / 1e6), "%.4f" % ((b - a) / 1e6), k, n, q])
PY
rm -rf gpurun_out/s2vt
