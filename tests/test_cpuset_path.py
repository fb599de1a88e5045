"""cpuset binding on the device path: NodeNUMAResource Filter / Score of LSE/LSR pods and
of pods on nodes with a CPU bind policy (plugin.go:388-440, util.go:101-138, scoring.go:132-151), and the
Reserve through the device accumulator (resource_manager.go:197-499, node_allocation.go:103-130), against the
oracle (oracle/kg_oracle.c cpuset_filter / cpuset_reserve over oracle/kg_cpuset.c). Bit-exact: status bits,
scores, keys, replay placements, allocated CPUs per node (RefCount and exclusive policy) and
cpuset_alloc_milli."""
import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, cluster, synth


# ---------------------------------------------------------------------------------------------- CPU

def test_oracle_cpuset_verify_outcomes():
    cfg, nodes, pods = synth.cpuset_cluster(300, 160, seed=1)
    kc = cfg.kg_config()
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    bind = (pods["flags"] & abi.KG_POD_CPU_BIND) != 0
    st = ref.status
    assert (st[bind] & abi.KG_ST_NUMA_CPU_TOPO).any()   # nodes without a CPU topology
    assert (st & abi.KG_ST_NUMA_CPU_BIND).any()          # conflicts / SMT / fractional cpus on bind-policy nodes
    assert (st[bind] & abi.KG_ST_NUMA_CPUS).any()        # the required policy's CPUs do not cover the pod
    assert ((st[bind] == 0)).any()                        # and cpuset pods that fit


def test_oracle_cpuset_replay_allocations_respect_policies():
    """Every Reserve of the oracle replay hands out free CPUs (RefCount < maxRefCount), counted into
    cpuset_alloc_milli; required FullPCPUs allocations are whole cores."""
    cfg, nodes, pods = synth.cpuset_cluster(120, 200, seed=2)
    kc = cfg.kg_config()
    st = oracle_lib.OracleState(kc, nodes)
    node, _ = st.replay(pods)
    t = st.table()
    ref = t["cpu_alloc"][:, :abi.KG_MAX_CPUS].astype(np.int64)
    before = nodes["cpu_alloc"][:, :abi.KG_MAX_CPUS].astype(np.int64)
    assert (ref >= before).all()
    assert (ref <= nodes["cpu_max_ref"][:, None]).all()
    assert np.array_equal(t["cpuset_alloc_milli"], 1000 * (ref > 0).sum(axis=1))
    bind = (pods["flags"] & abi.KG_POD_CPU_BIND) != 0
    # cpuset pods on every NUMA policy (under a NUMA affinity the CPUs come from the allocated NUMA nodes)
    placed = bind & (node >= 0)
    assert placed.sum() > 10
    assert (placed & (nodes["numa_policy"][np.maximum(node, 0)] != abi.KG_NUMA_NONE)).any()
    assert (ref.sum() - before.sum()) == int((pods["req_cpu"][placed] // 1000).sum()) + \
        int(sum(pods["req_cpu"][j] // 1000 for j in range(len(node)) if not bind[j] and node[j] >= 0
                and nodes["cpu_bind_policy"][node[j]] != 0 and nodes["cpu_topo"][node[j]] >= 0
                and pods["req_cpu"][j] > 0))


def _cpu_zone(nodes, i):
    topo = abi.KgCpuTopo.from_buffer_copy(nodes["cpu_topos"][nodes["cpu_topo"][i]].tobytes())
    return {c: int(topo.numa[c]) for c in range(int(topo.n_cpus))}


def test_oracle_cpuset_reserve_updates_zone_status():
    """A cpuset Reserve puts the pod's uid in singleNUMANode / sharedNode of the NUMA nodes of its CPUs
    (node_allocation.go:111-143): the oracle's per-zone status after every Reserve equals a host
    NodeAllocation (cluster.py) fed the same allocations, seeded with the node's existing pods."""
    cfg, nodes, pods = synth.cpuset_cluster(60, 120, seed=8)
    nodes["numa_zone_status"] = np.zeros(60, np.uint32)
    kc = cfg.kg_config()
    st = oracle_lib.OracleState(kc, nodes)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    host = {}
    changed = 0
    for j in np.flatnonzero((pods["flags"] & abi.KG_POD_CPU_BIND) != 0):
        ok = np.flatnonzero((ref.status[j] == 0) & (nodes["cpu_topo"] >= 0) & (nodes["numa_policy"] == 0))
        if not len(ok):
            continue
        i = int(ok[j % len(ok)])
        before = st.table()
        st.assume(i, pods, int(j))
        after = st.table()
        took = np.flatnonzero(after["cpu_alloc"][i, :abi.KG_MAX_CPUS] != before["cpu_alloc"][i, :abi.KG_MAX_CPUS])
        alloc = host.setdefault(i, cluster.NodeAllocation())
        alloc.add(f"pod-{j}", cluster._PodAllocation(set(int(c) for c in took), []), _cpu_zone(nodes, i))
        want = alloc.zone_status(abi.KG_MAX_ZONES)
        assert after["numa_zone_status"][i] == want, (j, i, after["numa_zone_status"][i], want)
        changed += int(before["numa_zone_status"][i] != want)
    assert changed >= 3


def _unallocatable_pairs(nodes, pods, ref):
    """(pod, node) pairs of cpuset pods on policy-None nodes with a topology whose accumulator fails
    (Filter status NUMA_CPUS for a required policy, UNSUPPORTED for a preferred one)."""
    bind = (pods["flags"] & abi.KG_POD_CPU_BIND) != 0
    ok_node = (nodes["cpu_topo"] >= 0) & (nodes["numa_policy"] == abi.KG_NUMA_NONE)
    hit = bind[:, None] & ok_node[None, :] & ((ref.status & (abi.KG_ST_NUMA_CPUS | abi.KG_ST_UNSUPPORTED)) != 0) & \
        ((ref.status & np.uint32(~(abi.KG_ST_NUMA_CPUS | abi.KG_ST_UNSUPPORTED) & 0xFFFFFFFF)) == 0)
    return np.argwhere(hit)


def test_oracle_cpuset_reserve_failure_applies_nothing():
    """Reserve of a cpuset pod whose accumulator finds too few CPUs (resource_manager.go:385,427
    ErrNotEnoughCPUs -> the Reserve error): kgo_assume reports the failure and no column moves."""
    cfg, nodes, pods = synth.cpuset_cluster(200, 160, seed=11)
    kc = cfg.kg_config()
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    pairs = _unallocatable_pairs(nodes, pods, ref)
    assert len(pairs) >= 3
    st = oracle_lib.OracleState(kc, nodes)
    before = st.table()
    for j, i in pairs[:8]:
        assert not st.assume(int(i), pods, int(j))
    after = st.table()
    for k in before:
        assert np.array_equal(before[k], after[k]), k


# ---------------------------------------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def ctx():
    from koordinator_amd import engine
    c = engine.Context(0)
    yield c
    c.close()


FIELDS = ("status", "score_nrf", "score_la", "score_numa", "total", "numa_zone")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 4])
def test_cpuset_verify_select(ctx, seed):
    from koordinator_amd import engine
    cfg, nodes, pods = synth.cpuset_cluster(700, 256, seed=seed)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    got = engine.eval_verify(snap, batch)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    for f in FIELDS:
        a, b = getattr(got, f), getattr(ref, f)
        if not np.array_equal(a, b):
            j, i = np.argwhere(a != b)[0]
            raise AssertionError(f"{f} pod {j} node {i}: gpu {a[j, i]} oracle {b[j, i]} status {ref.status[j, i]:#x}")
    for k in (1, 3):
        assert np.array_equal(engine.eval_select(snap, batch, k), oracle_lib.select(kc, nodes, pods, k))
    want = np.bitwise_or.reduce(ref.status & abi.KG_ST_UNSUPPORTED, axis=1)
    assert np.array_equal(engine.result_status(batch), want)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [5, 6])
def test_cpuset_replay(ctx, seed):
    """One pod per cycle with the cpuset Reserve on the device between steps (k_cpuset_reserve before each
    k_replay step): placements, reasons, NodeInfo columns, allocated CPUs and cpuset_alloc_milli."""
    from koordinator_amd import engine
    cfg, nodes, pods = synth.cpuset_cluster(500, 600, seed=seed)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    node, total, why = engine.replay(snap, batch, reasons=True)
    st = oracle_lib.OracleState(kc, nodes)
    rn, rt, rwhy = st.replay(pods, reasons=True)
    bad = np.flatnonzero(node != rn)
    assert not len(bad), (bad[:5], node[bad[:5]], rn[bad[:5]])
    assert np.array_equal(total, rt) and np.array_equal(why, rwhy)
    got, want = snap.read_state(), st.table()
    for k in ("req_cpu", "req_mem", "num_pods", "nz_cpu", "cpuset_alloc_milli", "numa_zone_status"):
        assert np.array_equal(got[k], want[k]), k
    assert np.array_equal(got["cpu_alloc"], want["cpu_alloc"])
    moved = (got["cpu_alloc"][:, :abi.KG_MAX_CPUS] != nodes["cpu_alloc"][:, :abi.KG_MAX_CPUS]).any(axis=1)
    assert moved.sum() > 20


@pytest.mark.gpu
def test_cpuset_assume_and_forget(ctx):
    from koordinator_amd import engine
    cfg, nodes, pods = synth.cpuset_cluster(200, 64, seed=7)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    st = oracle_lib.OracleState(kc, nodes)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    bind = np.flatnonzero((pods["flags"] & abi.KG_POD_CPU_BIND) != 0)
    done = 0
    for j in bind:
        ok = np.flatnonzero((ref.status[j] == 0) & (nodes["cpu_topo"] >= 0) & (nodes["numa_policy"] == 0))
        if not len(ok):
            continue
        i = int(ok[j % len(ok)])
        engine.assume(snap, batch, int(j), i)
        st.assume(i, pods, int(j))
        with pytest.raises(engine.Unsupported):
            engine.forget(snap, batch, int(j), i, -1)
        done += 1
        if done == 12:
            break
    assert done >= 8
    got, want = snap.read_state(), st.table()
    assert np.array_equal(got["cpu_alloc"], want["cpu_alloc"])
    assert np.array_equal(got["cpuset_alloc_milli"], want["cpuset_alloc_milli"])
    assert np.array_equal(got["req_cpu"], want["req_cpu"])
    assert np.array_equal(got["numa_zone_status"], want["numa_zone_status"])


@pytest.mark.gpu
def test_cpuset_then_pod_numa_policy_sees_zone_status(ctx):
    """A cpuset pod Reserved on a policy-None node marks the zones of its CPUs single / shared; a later pod
    with its own SingleNUMANode policy on that node (exclusive Required by default) reads the new status in
    its Filter. Device and oracle agree on the statuses and on the later pods' whole verify matrix."""
    from koordinator_amd import engine
    cfg, nodes, pods = synth.cpuset_cluster(120, 96, seed=9)
    nodes["numa_zone_status"] = np.zeros(120, np.uint32)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    st = oracle_lib.OracleState(kc, nodes)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    done = 0
    for j in np.flatnonzero((pods["flags"] & abi.KG_POD_CPU_BIND) != 0):
        ok = np.flatnonzero((ref.status[j] == 0) & (nodes["cpu_topo"] >= 0) & (nodes["numa_policy"] == 0))
        if not len(ok):
            continue
        i = int(ok[j % len(ok)])
        # a pod without a required policy passes Filter whatever the free CPUs; its Reserve can fail (zone 0x28)
        try:
            engine.assume(snap, batch, int(j), i)
            placed = True
        except engine.ReserveFailed:
            placed = False
        assert st.assume(i, pods, int(j)) == placed
        done += placed
    assert done >= 8
    got, want = snap.read_state(), st.table()
    assert np.array_equal(got["numa_zone_status"], want["numa_zone_status"])
    assert (want["numa_zone_status"] != 0).sum() >= 5
    # later pods: plain (no cpuset) pods carrying their own SingleNUMANode / Restricted policy
    later = synth.pods(160, 77, scale=2.0)
    later["numa_policy"] = np.where(np.arange(160) % 2 == 0, abi.KG_NUMA_SINGLE_NODE,
                                    abi.KG_NUMA_RESTRICTED).astype(np.uint32)
    lb = engine.PodBatch(ctx, later)
    gv = engine.eval_verify(snap, lb)
    rv = oracle_lib.eval_verify(kc, {**nodes, **want}, later)
    for f in FIELDS:
        a, b = getattr(gv, f), getattr(rv, f)
        assert np.array_equal(a, b), f


@pytest.mark.gpu
def test_cpuset_reserve_failure(ctx):
    """kg_assume of a cpuset pod whose accumulator fails: KG_RESERVE_FAILED (ReserveFailed), nothing applied on
    the device (k_cpuset_reserve flags the failure, k_assume skips the NodeInfo Reserve)."""
    from koordinator_amd import engine
    cfg, nodes, pods = synth.cpuset_cluster(200, 160, seed=11)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    pairs = _unallocatable_pairs(nodes, pods, ref)
    before = snap.read_state()
    for j, i in pairs[:8]:
        with pytest.raises(engine.ReserveFailed):
            engine.assume(snap, batch, int(j), int(i))
    after = snap.read_state()
    for k in before:
        assert np.array_equal(before[k], after[k]), k
