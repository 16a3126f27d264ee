"""Summarise rocprofv3 PMC passes of one bench command (each pass a separate
run of the same command, never combined with other tracing) into a
per-kernel, per-launch JSON under profiles/.

    python scripts/pmc_summary.py OUT.json --last N --cmd "..." --config '{...}' DIR [DIR ...]

Each DIR is one `rocprofv3 --pmc ... --kernel-trace --output-format csv`
pass.  The last N launches of each kernel are averaged: bench.py runs W
warmup steps, K timed steps, then K profiled steps whose HIP-event kernel
times give `roofline.achieved`, so N = K makes the counters and the achieved
bandwidth describe the same launches.

HBM bytes per launch (the `hbm_bytes` field, what bench.py reports as
`roofline.traffic`):

* reads: 32 * TCC_EA0_RDREQ_32B + 64 * TCC_EA0_RDREQ_64B + 128 *
  TCC_EA0_RDREQ_128B — the L2's memory-side read requests by size, which
  gfx950 counts separately.  rocprofv3's FETCH_SIZE formula for gfx950 charges
  every request that is not a TCC_BUBBLE or 32-B request 64 B, so a 128-B
  request is tallied at half its size (MI355X_MICROARCH.md §HBM: FETCH_SIZE =
  1/2 of a 16-B/lane streaming read; other widths uncalibrated).  Counting
  the requests by size needs no per-width calibration; when a FETCH_SIZE pass
  is present too, `fetch_ratio` = exact read bytes / FETCH_SIZE bytes is
  printed as the cross-check (2.0 for pure 16-B/lane streaming reads).
* writes: WRITE_SIZE (64-B and 32-B write requests; exact).
Infinity-Cache (MALL) hits are counted by these L2-miss counters, so the
figure is an upper bound on DRAM bytes."""
import argparse
import collections
import csv
import json
import os

READ_SIZES = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_128B_sum": 128}


def load(d):
    path = [os.path.join(d, f) for f in os.listdir(d) if f.endswith("counter_collection.csv")][0]
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(path) as f:
        for r in csv.DictReader(f):
            out[r["Counter_Name"]][r["Kernel_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return {c: {k: [v for _, v in sorted(vs)] for k, vs in ks.items()} for c, ks in out.items()}


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--last", type=int, required=True)
    ap.add_argument("--cmd", default="")
    ap.add_argument("--config", default="{}")
    a = ap.parse_args()
    counters = {}
    for d in a.dirs:
        counters.update(load(d))
    per = collections.defaultdict(dict)  # kernel -> counter -> mean of its last N launches
    for c, ks in counters.items():
        for k, vs in ks.items():
            if len(vs) >= a.last:  # per-step kernels only
                per[short(k)][c] = sum(vs[-a.last:]) / a.last
    kernels = {}
    for k, cs in per.items():
        e = dict(cs)
        rd = sum(cs[c] * s for c, s in READ_SIZES.items()) if all(c in cs for c in READ_SIZES) else None
        wr = cs["WRITE_SIZE"] * 1024.0 if "WRITE_SIZE" in cs else None
        e["read_bytes"] = rd
        e["write_bytes"] = wr
        if rd is not None and "FETCH_SIZE" in cs and cs["FETCH_SIZE"] > 0:
            e["fetch_ratio"] = rd / (cs["FETCH_SIZE"] * 1024.0)
        e["hbm_bytes"] = rd + wr if rd is not None and wr is not None else None
        if cs.get("SQ_WAVE_CYCLES"):  # MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ≈ WAVE_CYCLES
            wc = cs["SQ_WAVE_CYCLES"]
            for c, name in (("SQ_WAIT_ANY", "parked_frac"), ("SQ_WAIT_INST_ANY", "issue_stall_frac"),
                            ("SQ_ACTIVE_INST_ANY", "active_frac")):
                if c in cs:
                    e[name] = cs[c] / wc  # parked = s_waitcnt / barrier (memory latency); issue stall = pipe
            if cs.get("SQ_WAVES"):
                e["quad_cycles_per_wave"] = wc / cs["SQ_WAVES"]
                for c in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                    if c in cs:
                        e[c.replace("SQ_INSTS_", "").lower() + "_per_wave"] = cs[c] / cs["SQ_WAVES"]
        kernels[k] = e
    out = {"source": "rocprofv3 --pmc <pass> --kernel-trace (one run per pass) -- " + a.cmd,
           "passes": [sorted(load(d).keys()) for d in a.dirs],
           "config": json.loads(a.config),
           "window": "the last %d launches of each kernel = bench.py's profiled pass" % a.last,
           "units": "per launch; read_bytes / write_bytes / hbm_bytes in bytes, raw counters as rocprofv3 reports "
                    "them (FETCH_SIZE, WRITE_SIZE in KiB; request counters in requests)",
           "method": "read_bytes = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B (L2 memory-side read requests by "
                     "size); write_bytes = WRITE_SIZE; hbm_bytes = read + write (includes Infinity-Cache hits)",
           "kernels": kernels}
    with open(a.out, "w") as fo:
        json.dump(out, fo, indent=1)
    for k, v in sorted(kernels.items(), key=lambda kv: -(kv[1]["hbm_bytes"] or kv[1].get("SQ_WAVE_CYCLES", 0)))[:10]:
        if "parked_frac" in v:
            print("%-44s waves %d  parked %.2f  issue-stall %.2f  active %.2f  qcyc/wave %.0f" % (
                k, v.get("SQ_WAVES", 0), v["parked_frac"], v.get("issue_stall_frac", 0), v.get("active_frac", 0),
                v.get("quad_cycles_per_wave", 0)))
            continue
        print("%-44s hbm %.4g GB  read %s  write %s  fetch_ratio %s" % (
            k, (v["hbm_bytes"] or 0) / 1e9, v["read_bytes"], v["write_bytes"], v.get("fetch_ratio")))


if __name__ == "__main__":
    main()
