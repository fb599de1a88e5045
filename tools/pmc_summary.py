"""Summarise a rocprofv3 collection of profiles/run_profile.sh into profiles/<out>.json.

Per select step (the kernels of one step's bracket: the k_select kernels of both node storage classes for
configs 1-4; for config 5 every kernel of the step: DevSum / restore codes, pass 1, the one-pass select and its
re-run, the general records, the plain pods' k_select), summed over a step's dispatches, from the PMC passes:
  FETCH_SIZE (KB)  -> doubled per MI355X_MICROARCH.md § HBM (gfx950 reports 1/2 of wide streaming reads)
  WRITE_SIZE (KB)
  hbm_bytes_per_launch  = 1024 * (2 * FETCH_SIZE + WRITE_SIZE), summed over the bracket's kernels
  valu_insts_per_launch = SQ_INSTS_VALU summed over the bracket's kernels (per launch)
  salu_insts_per_launch = SQ_INSTS_SALU, likewise
plus the kernel-trace average durations and every SQ counter per kernel. The summary is stamped with the
hash of the kernel sources it was taken on (bench.kernel_source_hash); bench.py ignores a summary whose
stamp differs from the sources it runs.
Usage: python tools/pmc_summary.py gpurun_out/prof_<tag> [profiles/select_pmc.json] [kernel substring ...]
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_kernel(path):
    """{kernel: {counter: sum over its dispatches}}, {kernel: dispatches}."""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ids = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
        ids[r["Kernel_Name"]].add(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(ids[r["Kernel_Name"]]))
    return {k: dict(d) for k, d in agg.items()}, {k: len(v) for k, v in ids.items()}


def per_kernel_issue(name, trace, counters, tsteps):
    """One bracket kernel: its trace entry, counters per step, its time per step (average duration x dispatches per
    step: config 5's k_ext_select runs twice a step, the guess launch and a short re-run) and its VALU issue fraction
    with the instruction costs of profiles/valu_mix.json (the kernel's loop priced per opcode; 4.1 cycles without one)."""
    import bench
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from valu_mix import canon_demangled
    out = {"trace": trace, "counters": counters}
    if not trace:
        return out
    ns = trace["avg_ns"] * trace["calls"] / max(tsteps, 1)
    out["ns_per_step"] = ns
    mix = bench.load_pmc("valu_mix.json")
    m = (mix or {}).get("kernels", {}).get(canon_demangled(name) or "")
    cyc = m["cyc_per_valu"] if m else 4.1
    v = counters.get("SQ_INSTS_VALU", 0.0)
    if ns > 0:
        out["issue"] = {"cycles_per_valu": cyc, "frac": v * cyc / (ns * 1e-9 * bench.SIMD_CYCLES),
                        "priced_by": "profiles/valu_mix.json" if m else "4.1 cycles (no ISA mix)"}
    return out


def main(prof, out, names):
    import bench

    stats = {}
    for r in csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_stats.csv"))):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    # per step: a bracket kernel may run more than once a step (config 5's k_ext_select: the guess launch and the
    # re-run), so counters are summed over dispatches and divided by the step count of the pass (the fewest
    # dispatches of any bracket kernel: each runs at least once a step)
    counters = collections.defaultdict(dict)
    for d in sorted(os.listdir(prof)):
        p = os.path.join(prof, d, "run_counter_collection.csv")
        if d.startswith("pmc") and os.path.exists(p):
            sums, calls = per_kernel(p)
            steps = min([c for k, c in calls.items() if any(n in k for n in names)] or [1])
            for k, v in sums.items():
                counters[k].update({c: x / steps for c, x in v.items()})
    sel = {k: v for k, v in counters.items() if any(n in k for n in names)}
    tsteps = min([v["calls"] for k, v in stats.items() if any(n in k for n in names)] or [1])

    def total(c):
        return sum(v.get(c, 0.0) for v in sel.values())

    res = {
        "source": prof,
        "kernel_source_hash": bench.kernel_source_hash(),
        "bracket": names,
        "note": "per select launch = the bracket's kernels of one step; FETCH_SIZE doubled per "
                "MI355X_MICROARCH.md (gfx950 counts 1/2 of wide reads; scalar-load and 8-B/lane access widths "
                "are uncalibrated), KB = 1024 B",
        "fetch_kb_raw": total("FETCH_SIZE"),
        "write_kb": total("WRITE_SIZE"),
        "hbm_bytes_per_launch": 1024.0 * (2.0 * total("FETCH_SIZE") + total("WRITE_SIZE")),
        "valu_insts_per_launch": total("SQ_INSTS_VALU"),
        "salu_insts_per_launch": total("SQ_INSTS_SALU"),
        "kernels": {k: per_kernel_issue(k, stats.get(k), v, tsteps) for k, v in sel.items()},
        "select_avg_ns_sum": sum((stats.get(k) or {}).get("avg_ns", 0.0) * (stats.get(k) or {}).get("calls", 0) / tsteps
                                 for k in sel),
        "all_kernels_trace": stats,
        "all_kernels_counters": counters,
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: res[k] for k in ("hbm_bytes_per_launch", "valu_insts_per_launch", "salu_insts_per_launch",
                                          "select_avg_ns_sum")}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "select_pmc.json"),
         sys.argv[3:] or ["k_select<"])
