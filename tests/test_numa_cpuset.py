"""f3 part 2: cpusets under a NUMA affinity (nodenumaresource/resource_manager.go:132-463) and the amplified zone
accounting of getAvailableNUMANodeResources (node_allocation.go:221-243).

- resourceManager.Allocate in the oracle (kgo_numa_allocate) against TestResourceManagerAllocate
  (resource_manager_test.go:35-598): topology buildCPUTopologyForTest(2, 1, 26, 2) (104 CPUs, NUMA node 0 = CPUs 0-51),
  NUMANodeResources 52 cpu / 128Gi per node, an optional existing PodAllocation (Update), the options' requests.
  The existing allocations name CPU 104, outside the topology (cpuset "4-104"): it enters allocatedCPUs under NUMA
  node 0 there; no case's outcome depends on it (only the amplified case reads per-node CPU counts, and there the
  split fits either way), so the transcription drops it.
- Oracle-level properties of the topology manager with cpuset-binding pods on NUMA-policy nodes.
"""
import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi


def _cpus(spec: str):
    out = []
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return [c for c in out if c < 104]


# (line, name, requests cpu (options.requests), original cpu, bind ("" | "FullPCPUs" | "SpreadByPCPUs"), required,
#  ratio, allocated (cpuset, {numa: cpu}), mask, want (cpus or None, {numa: cpu}) or "error")
CASES = [
    (46, "non-existing resources in NUMA", 4, 4, "", False, None, None, [0], ("", {0: 4})),
    (75, "insufficient resources", 54, 54, "", False, None, None, [0], "error"),
    (94, "required FullPCPUs", 4, 4, "FullPCPUs", True, None, None, [0], ("0-3", {0: 4})),
    (125, "required FullPCPUs and allocated", 4, 4, "FullPCPUs", True, None, ("4-104", {0: 48, 1: 52}), [0],
     ("0-3", {0: 4})),
    (176, "failed required FullPCPUs and allocated", 4, 4, "FullPCPUs", True, None, ("1,3,5,7-104", {0: 48, 1: 52}),
     [0], "error"),
    (217, "required SpreadByPCPUs", 4, 4, "SpreadByPCPUs", True, None, None, [0], ("0,2,4,6", {0: 4})),
    (248, "required SpreadByPCPUs and allocated", 4, 4, "SpreadByPCPUs", True, None, ("1,3,5,7-104", {0: 48, 1: 52}),
     [0], ("0,2,4,6", {0: 4})),
    (299, "failed required SpreadByPCPUs and allocated", 4, 4, "SpreadByPCPUs", True, None, ("4-104", {0: 48, 1: 52}),
     [0], "error"),
    (340, "required SpreadByPCPUs amplified", 6, 4, "SpreadByPCPUs", True, 1.5, None, [0], ("0,2,4,6", {0: 4})),
    (377, "required SpreadByPCPUs allocated amplified", 6, 4, "SpreadByPCPUs", True, 1.5,
     ("1,3,5,7-104", {0: 48, 1: 52}), [0], ("0,2,4,6", {0: 4})),
    (434, "CPU share allocated amplified", 4, 4, "", False, 1.5, ("0-49,52-101", {0: 50, 1: 50}), [0], "error"),
    (480, "numa hint on mixed cpuset/share node", 8, 8, "FullPCPUs", True, None, ("0-43,53-96", {0: 48, 1: 48}),
     [0, 1], ("44-47,98-101", {0: 4, 1: 4})),
]


def _case_tables(req_cpu, bind, required, ratio, allocated):
    t = abi.empty_nodes(1)
    r = ratio or 1.0
    t["alloc_cpu"][:] = abi_amplify(104000, r)
    t["alloc_mem"][:] = 256 << 30
    t["alloc_pods"][:] = 110
    t["cpu_amp_ratio"][:] = r
    t["numa_zones"][:] = 2
    t["numa_policy"][:] = abi.KG_NUMA_RESTRICTED
    for z in range(2):
        t[f"zone_cpu{z}"][:] = abi_amplify(52000, r)  # amplifyNUMANodeResources
        t[f"zone_mem{z}"][:] = 128 << 30
    t["cpu_topo"] = np.zeros(1, np.int32)
    t["cpu_topos"] = abi.cpu_topos_array([abi.cpu_topo_for_test(2, 1, 26, 2)])
    alloc = np.zeros((1, 2 * abi.KG_MAX_CPUS), np.uint8)
    status = 0
    if allocated:
        spec, numa = allocated
        for c in _cpus(spec):
            alloc[0, c] = 1
        for z, cpu in numa.items():
            t[f"zone_cpu_used{z}"][:] = cpu * 1000
            status |= 1 << (abi.KG_ZONE_RECORD_SHIFT + z)
        t["cpuset_alloc_milli"][:] = 1000 * len(_cpus(spec))
    t["cpu_alloc"] = alloc
    t["cpu_max_ref"] = np.ones(1, np.uint8)
    t["numa_zone_status"] = np.array([status], np.uint32)
    p = abi.empty_pods(1)
    p["req_cpu"][:] = req_cpu * 1000
    p["nz_cpu"][:] = req_cpu * 1000
    f = abi.KG_POD_HAS_CPU
    if bind:
        f |= abi.KG_POD_CPU_BIND | (abi.KG_CPU_BIND[bind] << abi.KG_POD_CPU_POLICY_SHIFT)
        f |= abi.KG_POD_CPU_REQUIRED if required else 0
    p["flags"][:] = f
    return t, p


def abi_amplify(v, ratio):
    import math
    return v if ratio <= 1 else int(math.ceil(float(v) * ratio))


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-{c[1]}" for c in CASES])
def test_resource_manager_allocate_kat(case):
    line, name, req, orig, bind, required, ratio, allocated, mask, want = case
    nodes, pods = _case_tables(orig, bind, required, ratio, allocated)
    m = sum(1 << z for z in mask)
    ok, cpus, al = oracle_lib.numa_allocate(nodes, pods, m)
    if want == "error":
        assert not ok
        return
    assert ok
    spec, numa = want
    assert cpus == _cpus(spec)
    assert {z: int(al[0, z]) // 1000 for z in range(2) if al[0, z]} == numa


# TestResourceManagerGetTopologyHint (resource_manager_test.go:1279-1679, BestEffort, no NUMA scorer): (line, name,
# cpu, bind, required, ratio, allocated, want cpu hints [(NUMA nodes, preferred)]). The hugepages case (:1581-1620)
# requests a resource the device tables do not hold (parity unpinned for hugepages).
HINT_CASES = [
    (1290, "required FullPCPUs", 4, "FullPCPUs", True, None, None, [([0], True), ([1], True), ([0, 1], False)]),
    (1329, "required FullPCPUs and allocated", 4, "FullPCPUs", True, None, ("4-104", {0: 48, 1: 52}), [([0], True)]),
    (1374, "failed required FullPCPUs and allocated", 4, "FullPCPUs", True, None, ("1,3,5,7-104", {0: 48, 1: 52}), []),
    (1411, "required SpreadByPCPUs", 4, "SpreadByPCPUs", True, None, None,
     [([0], True), ([1], True), ([0, 1], False)]),
    (1450, "required SpreadByPCPUs and allocated", 4, "SpreadByPCPUs", True, None, ("1,3,5,7-104", {0: 48, 1: 52}),
     [([0], True)]),
    (1495, "failed required SpreadByPCPUs and allocated", 4, "SpreadByPCPUs", True, None, ("4-104", {0: 48, 1: 52}), []),
    (1532, "CPU share allocated amplified", 4, "", False, 1.5, ("0-49,52-101", {0: 50, 1: 50}), [([0, 1], True)]),
]


@pytest.mark.parametrize("case", HINT_CASES, ids=[f"{c[0]}-{c[1]}" for c in HINT_CASES])
def test_resource_manager_hints_kat(case):
    from koordinator_amd.config import config5_profile
    line, name, cpu, bind, required, ratio, allocated, want = case
    nodes, pods = _case_tables(cpu, bind, required, ratio, allocated)
    kc = config5_profile().kg_config()
    lists = oracle_lib.numa_hints(kc, nodes, pods, abi.KG_NUMA_BEST_EFFORT)
    assert len(lists) == 1  # cpu only
    got = [([z for z in range(4) if (m >> z) & 1], pref) for m, pref in lists[0]]
    assert got == want


def test_mixed_cluster_cpusets_under_numa_policies_oracle():
    """Bench config 6's shape (synth.mixed): LSR pods and pods on CPU-bind-policy nodes under SingleNUMANode /
    Restricted / BestEffort policies are evaluated (no pair left to the host), some are admitted with a NUMA
    affinity, and a BestEffort Reserve can fail on its CPUs (zone code 0x28)."""
    from koordinator_amd import synth
    cfg, nodes, pods = synth.mixed(1500, 600, seed=6)
    kc = cfg.kg_config()
    v = oracle_lib.eval_verify(kc, nodes, pods)
    assert not (v.status & abi.KG_ST_UNSUPPORTED).any()
    bind = (pods["flags"] & abi.KG_POD_CPU_BIND) != 0
    pol = nodes["numa_policy"]
    topo = nodes["cpu_topo"] >= 0
    for p in (abi.KG_NUMA_SINGLE_NODE, abi.KG_NUMA_RESTRICTED):
        sel = bind[:, None] & ((pol == p) & topo)[None, :]
        ok = sel & (v.status == 0)
        assert ok.sum() > 20, p
        assert (v.numa_zone[ok] >= 0).any()
    be = bind[:, None] & ((pol == abi.KG_NUMA_BEST_EFFORT) & topo)[None, :] & (v.status == 0)
    assert be.sum() > 20


def test_oracle_replay_matches_verify_cpusets():
    """The oracle replay of a cpuset cluster with NUMA policies places each pod on the argmax of the verify row computed
    on the state after the pods before it (Reserve under the NUMA affinity: CPUs, split and records consistent)."""
    from koordinator_amd import synth
    cfg, nodes, pods = synth.mixed(300, 200, seed=9)
    kc = cfg.kg_config()
    bind = np.flatnonzero((pods["flags"] & abi.KG_POD_CPU_BIND) != 0)[:5]
    for k in bind:
        st = oracle_lib.OracleState(kc, nodes)
        rnode, _ = st.replay(abi.take(pods, np.arange(k + 1)))
        st2 = oracle_lib.OracleState(kc, nodes)
        if k:
            st2.replay(abi.take(pods, np.arange(k)))
        t = dict(nodes)
        t.update(st2.table())
        v = oracle_lib.eval_verify(kc, t, abi.take(pods, np.array([k])))
        tot = np.where(v.status[0] == 0, v.total[0], -1)
        want = int(np.argmax(tot)) if tot.max() >= 0 else -1
        if want >= 0 and 0x20 <= int(v.numa_zone[0, want]) < 0x40:
            want = -1  # the winner's Reserve fails
        assert rnode[k] == want, (k, rnode[k], want)
