"""Recompute each committed bench line's roofline fraction from the rocprof
kernel-stats CSV of the same leg (profiles/rNN_<leg>_kernel_stats.csv):
algorithmic bytes per launch (the line's bytes_per_launch) / the summed
average durations of the group's kernels / 8 TB/s, against the line's frac.

    python scripts/check_frac.py [profiles/rNN_bench_<leg>.json ...]"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GROUPS = {  # kernel base names of each roofline group
    "w2v": ("k_gather_b", "k_combine_b", "k_push_b", "k_gather_t", "k_combine", "k_push_thp", "k_gather", "k_push",
            "k_push_tg"),
    "lr_forward": ("k_lr_forward_r", "k_lr_forward", "k_lr_forward_l", "k_lr_forward_g", "k_lr_forward_c"),
    "lr_push": ("k_lr_records", "k_lr_reduce_fused", "k_lr_reduce_short", "k_lr_reduce_long", "k_lr_reduce_long_fast",
                "k_lr_tiles", "k_lr_tiles_fin"),
    "s2v": ("k_s2v_docs",),
}


def base(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0].strip()


def main(paths):
    bad = 0
    for p in paths:
        tag = os.path.basename(p)[:3]  # rNN
        leg = os.path.basename(p)[len("r03_bench_"):-len(".json")]
        if leg.endswith("_traced"):  # the line of the traced process itself
            leg = leg[:-len("_traced")]
        csvp = os.path.join(os.path.dirname(p), "%s_%s_kernel_stats.csv" % (tag, leg))
        if not os.path.exists(csvp):
            continue
        b = json.load(open(p))
        r = b["roofline"]
        rows = {}
        for row in csv.DictReader(open(csvp)):
            rows.setdefault(base(row["Name"]), []).append(float(row["AverageNs"]))
        if leg == "lr":
            grp = GROUPS["lr_push"] if ("reduce" in r["kernel"] or "tiles" in r["kernel"]) else GROUPS["lr_forward"]
        elif leg == "s2v":
            grp = GROUPS["s2v"]
        else:
            grp = GROUPS["w2v"]
            if r["kernel"].startswith("k_gather + "):
                grp = ("k_gather", "k_combine")
            elif "k_gather_b" in r["kernel"]:
                grp = ("k_gather_b", "k_combine_b", "k_push_b")
            elif "k_gather_t" in r["kernel"]:
                grp = ("k_gather_t", "k_combine", "k_push_thp", "k_push_tg")
        ns = sum(sum(v) for k, v in rows.items() if k in grp)
        if ns <= 0:
            print("%-16s no group kernels in the CSV" % leg)
            continue
        frac = r["bytes_per_launch"] / (ns * 1e-9) / 1e9 / 8000.0
        rel = abs(frac - r["frac"]) / r["frac"]
        bad += rel > 0.05
        print("%-16s line frac %.3f  csv frac %.3f  (%+.1f %%)  group %s" % (leg, r["frac"], frac, 100 * (frac / r["frac"] - 1),
                                                                       "+".join(k for k in grp if k in rows)))
    return bad


if __name__ == "__main__":
    tag = max(os.path.basename(x)[:3] for x in glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_bench_*.json")))
    ps = sys.argv[1:] or sorted(x for x in glob.glob(os.path.join(ROOT, "profiles", tag + "_bench_*.json"))
                                if not x.endswith("_traced.json"))
    sys.exit(1 if main(ps) else 0)
