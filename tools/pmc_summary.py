"""Summarise a rocprofv3 collection of profiles/run_profile.sh into profiles/select_pmc.json.

Per select launch (the k_select kernels of both node storage classes of one step), from the PMC passes:
  FETCH_SIZE (KB)  -> doubled per MI355X_MICROARCH.md § HBM (gfx950 reports 1/2 of wide streaming reads)
  WRITE_SIZE (KB)
  hbm_bytes_per_launch = 1024 * (2 * FETCH_SIZE + WRITE_SIZE), summed over the class kernels
plus the kernel-trace average durations and the SQ instruction counts per kernel.
Usage: python tools/pmc_summary.py gpurun_out/prof_<tag> [out.json]
"""
import collections
import csv
import json
import os
import sys


def per_kernel(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main(prof, out):
    stats = {}
    for r in csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_stats.csv"))):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    counters = collections.defaultdict(dict)
    for d in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_clk"):
        p = os.path.join(prof, d, "run_counter_collection.csv")
        if os.path.exists(p):
            for k, v in per_kernel(p).items():
                counters[k].update(v)
    sel = {k: v for k, v in counters.items() if "k_select" in k}
    fetch_kb = sum(v.get("FETCH_SIZE", 0.0) for v in sel.values())
    write_kb = sum(v.get("WRITE_SIZE", 0.0) for v in sel.values())
    res = {
        "source": prof,
        "note": "per select launch = the k_select kernels of both storage classes of one step; "
                "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 counts 1/2 of wide reads; scalar-load "
                "and 8-B/lane access widths are uncalibrated), KB = 1024 B",
        "fetch_kb_raw": fetch_kb,
        "write_kb": write_kb,
        "hbm_bytes_per_launch": 1024.0 * (2.0 * fetch_kb + write_kb),
        "kernels": {k: {"trace": stats.get(k), "counters": v} for k, v in sel.items()},
        "select_avg_ns_sum": sum((stats.get(k) or {}).get("avg_ns", 0.0) for k in sel),
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: res[k] for k in ("hbm_bytes_per_launch", "select_avg_ns_sum")}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "profiles/select_pmc.json")
