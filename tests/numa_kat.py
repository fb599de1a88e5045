"""Builders for the NodeNUMAResource known-answer cases of tests/golden/numa_kat.json."""
import json
import os

from koordinator_amd import abi
from koordinator_amd.config import SchedulerConfig

HERE = os.path.dirname(os.path.abspath(__file__))
GI = 1 << 30


def load():
    with open(os.path.join(HERE, "golden", "numa_kat.json")) as f:
        return json.load(f)


def _cfg(hint="LeastAllocated", score="LeastAllocated"):
    cfg = SchedulerConfig(plugins=abi.KG_PLUGIN_NUMA, numa_strategy=score, numa_hint_strategy=hint)
    return cfg.kg_config()


def _node(t, i, cpu, mem, zones, policy):
    t["alloc_cpu"][i] = cpu * 1000
    t["alloc_mem"][i] = mem * GI
    t["alloc_pods"][i] = 110
    t["numa_policy"][i] = getattr(abi, "KG_NUMA_" + policy)
    t["numa_zones"][i] = zones
    for z in range(zones):
        t[f"zone_cpu{z}"][i] = cpu * 1000 // zones
        t[f"zone_mem{z}"][i] = mem * GI // zones


def _pod(cpu, mem):
    p = abi.empty_pods(1)
    p["req_cpu"][0], p["req_mem"][0] = cpu * 1000, mem * GI
    p["nz_cpu"][0], p["nz_mem"][0] = cpu * 1000, mem * GI
    p["flags"][0] = abi.KG_POD_HAS_CPU | abi.KG_POD_HAS_MEM | abi.KG_POD_PROD
    return p


def affinity(case):
    t = abi.empty_nodes(1)
    _node(t, 0, *case["node"], case["zones"], case["policy"])
    for z, pods in case["used"].items():
        for cpu, mem in pods:
            t[f"zone_cpu_used{z}"][0] += cpu * 1000
            t[f"zone_mem_used{z}"][0] += mem * GI
            t["req_cpu"][0] += cpu * 1000
            t["req_mem"][0] += mem * GI
    return _cfg(hint=case["hint"]), t, _pod(*case["pod"])


def score(case):
    n = len(case["nodes"])
    t = abi.empty_nodes(n)
    for i, nd in enumerate(case["nodes"]):
        _node(t, i, *nd["node"], nd["zones"], case["policy"])
        for cpu, mem in case["existing"][i]:
            t["zone_cpu_used0"][i] += cpu * 1000
            t["zone_mem_used0"][i] += mem * GI
            t["req_cpu"][i] += cpu * 1000
            t["req_mem"][i] += mem * GI
    return _cfg(score="MostAllocated"), t, _pod(*case["pod"])
