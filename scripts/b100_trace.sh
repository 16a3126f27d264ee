# B = 100 kernel timeline (start / end of every dispatch) for the concurrency analysis in DESIGN.md
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b100t -o run -- python3 bench.py --gpus 1 --steps 30 --warmup 5 --minibatch 100 --no-cpu-baseline --no-parity-leg --config1-steps 0 --b100-steps 0 --no-app-legs > gpurun_out/b100t.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/b100t/**/run_kernel_trace.csv", recursive=True) or glob.glob("gpurun_out/b100t/run_kernel_trace.csv")
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
keep = rows[-400:]
with open("gpurun_out/b100_timeline.csv", "w") as o:
    w = csv.writer(o)
    w.writerow(["name", "start", "end", "queue"])
    for r in keep:
        w.writerow([r["Kernel_Name"][:80], r["Start_Timestamp"], r["End_Timestamp"], r.get("Queue_Id", r.get("Stream_Id", ""))])
PY
rm -rf gpurun_out/b100t
