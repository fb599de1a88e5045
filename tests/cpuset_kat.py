"""Runs the cpuset accumulator KATs (tests/golden/cpuset_kat.json, transcribed from
nodenumaresource/cpu_accumulator_test.go) against a `take(topo, max_ref, avail, alloc, needed, bind, excl,
strategy, preferred)` backend: the CPU oracle here, the device accumulator with -m gpu."""
import json
import os

import numpy as np

from koordinator_amd import abi

KAT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cpuset_kat.json")


def load():
    with open(KAT) as f:
        return json.load(f)


def take_case_args(c):
    topo = abi.cpu_topo_for_test(*c["topo"])
    alloc = abi.KgCpuAlloc()
    for cpu in c["allocated"]:
        alloc.ref[cpu] = 0  # KeepOnly(allocated): RefCount 0 in these KATs (maxRefCount 1 ignores it)
        if c["alloc_excl"]:
            alloc.excl[cpu] = abi.KG_CPU_EXCL[c["alloc_excl"]]
    avail = abi.cpu_mask(sorted(set(range(topo.n_cpus)) - set(c["allocated"])))
    return (topo, c["max_ref"], avail, alloc, c["needed"], abi.KG_CPU_BIND[c["bind"]], abi.KG_CPU_EXCL[c["excl"]],
            abi.KG_NUMA_STRATEGY[c["strategy"]])


def check_take(take, c):
    rc, got = take(*take_case_args(c))
    if c["error"]:
        assert rc != 0, c["name"]
    else:
        assert rc == 0, (c["name"], rc)
        assert got == c["want"], (c["source"], c["name"], got, c["want"])


def run_sequence(take, s):
    """getAvailableCPUs (node_allocation.go:192-220) -> takeCPUs -> addCPUs (:103-130), repeated."""
    topo = abi.cpu_topo_for_test(*s["topo"])
    n = topo.n_cpus
    ref = np.zeros(n, np.int64)
    excl = np.zeros(n, np.int64)
    for k, st in enumerate(s["steps"]):
        alloc = abi.KgCpuAlloc()
        for cpu in range(n):
            alloc.ref[cpu] = int(ref[cpu])
            alloc.excl[cpu] = int(excl[cpu]) if ref[cpu] else 0
        avail = abi.cpu_mask([c for c in range(n) if ref[c] < s["max_ref"]])
        rc, got = take(topo, s["max_ref"], avail, alloc, st["needed"], abi.KG_CPU_BIND[st["bind"]],
                       abi.KG_CPU_EXCL[s["excl"]], abi.KG_NUMA_STRATEGY[s["strategy"]], None)
        assert rc == 0 and got == st["want"], (s["name"], k, got, st["want"])
        for cpu in got:
            ref[cpu] += 1
            excl[cpu] = abi.KG_CPU_EXCL[s["add_excl"]]
    if "final_available" in s:
        assert [c for c in range(n) if ref[c] < s["max_ref"]] == s["final_available"]


def run_preferred(take, p):
    topo = abi.cpu_topo_for_test(*p["topo"])
    everything = list(range(topo.n_cpus))
    for call in p["calls"]:
        avail = everything if call["avail"] == "all" else [c for c in everything if c not in (0, 2)]
        pref = None if call["preferred"] is None else abi.cpu_mask(call["preferred"])
        rc, got = take(topo, 1, abi.cpu_mask(avail), None, call["needed"], abi.KG_CPU_BIND[p["bind"]], 0,
                       abi.KG_NUMA_STRATEGY[p["strategy"]], pref)
        assert rc == 0 and got == call["want"], (call, got)
