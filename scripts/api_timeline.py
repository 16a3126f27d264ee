"""Host API calls beside the kernels they launch, for one steady-state stretch of a
`rocprofv3 --hip-trace --kernel-trace --output-format csv` run: for each kernel its
launch call's host timestamp, its GPU start, and the lag between them (a GPU start
right at its launch call means the GPU was waiting for the host).  Long host calls
(> 20 us) are listed too.   python scripts/api_timeline.py DIR [first_kernel_index]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
ht = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0]
ks = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
api = sorted(csv.DictReader(open(ht)), key=lambda r: int(r["Start_Timestamp"]))
by_corr = {r.get("Correlation_Id"): r for r in api}
s0 = int(sys.argv[2]) if len(sys.argv) > 2 else len(ks) * 3 // 4
seg = ks[s0:s0 + 60]
t0 = int(seg[0]["Start_Timestamp"])
print("kernel start  dur   launch-call(host)  lag   name")
for r in seg:
    a = by_corr.get(r.get("Correlation_Id"))
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    hs = int(a["Start_Timestamp"]) if a else None
    print("%9.1f %6.1f %9s %7s  q%s %s" % ((s - t0) / 1e3, (e - s) / 1e3,
                                         "%.1f" % ((hs - t0) / 1e3) if hs else "-",
                                         "%.1f" % ((s - hs) / 1e3) if hs else "-",
                                         r.get("Queue_Id", r.get("Stream_Id", "")), r["Kernel_Name"][:70]))
t1 = int(seg[-1]["End_Timestamp"])
print("\nhost calls > 20 us in the same stretch:")
for a in api:
    s, e = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
    if t0 <= s <= t1 and e - s > 20000:
        print("%9.1f %8.1f us  %s" % ((s - t0) / 1e3, (e - s) / 1e3, a.get("Function", a.get("Operation", ""))))

print("\nevery host call in the first 1.2 ms of the stretch (start, duration, function, stream/kernel):")
for a in api:
    s, e = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
    if t0 - 400000 <= s <= t0 + 800000:
        print("%9.1f %7.1f  %s %s" % ((s - t0) / 1e3, (e - s) / 1e3, a.get("Function", a.get("Operation", "")),
                                     (a.get("Args", "") or "")[:80]))
