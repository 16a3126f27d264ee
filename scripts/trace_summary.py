"""Per-kernel summary and one steady-state step timeline of a rocprofv3
--kernel-trace CSV (gaps between kernels show where the host, not the GPU,
is the bottleneck).  python scripts/trace_summary.py DIR [first_kernel_index]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
start = int(sys.argv[2]) if len(sys.argv) > 2 else None
st = glob.glob(os.path.join(d, "*kernel_stats.csv"))
if st:
    rows = list(csv.DictReader(open(st[0])))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:24]:
        print("%-70s %7s %10.1f us avg %6.1f%%" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                   float(r["Percentage"])))
tr = glob.glob(os.path.join(d, "*kernel_trace.csv"))
if tr:
    rows = sorted(csv.DictReader(open(tr[0])), key=lambda r: int(r["Start_Timestamp"]))
    s0 = start if start is not None else len(rows) * 3 // 4
    seg = rows[s0:s0 + 40]
    t0 = prev = int(seg[0]["Start_Timestamp"])
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("%8.1f %7.1f gap %5.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, r["Kernel_Name"][:60]))
        prev = e
