"""NodeNUMAResource topology manager on mixed-policy clusters: nodes with 1-4 NUMA
zones under None / BestEffort / Restricted / SingleNUMANode, zone statuses for the Required exclusive
policy, pods with and without their own NUMA policy, LeastAllocated and MostAllocated strategies.

CPU tests (-m "not gpu") check oracle properties every admitted pair must have; the -m gpu tests
compare the HIP engine (through the C ABI) with the oracle bit for bit: filter status bits, NUMA score,
the affinity / zone code of every pair, selections, replay placements and the final zone state
(multi-zone allocations split exactly as tryBestToDistributeEvenly splits them)."""
import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, engine, synth

FIELDS = ("status", "score_nrf", "score_la", "score_numa", "total", "numa_zone")
STRATEGIES = [("LeastAllocated", "LeastAllocated"), ("MostAllocated", "LeastAllocated"),
              ("LeastAllocated", "MostAllocated"), ("MostAllocated", "MostAllocated")]


def workload(seed, n_nodes, n_pods, score="LeastAllocated", hint="LeastAllocated"):
    cfg, nodes, pods = synth.topology(n_nodes, n_pods, seed=seed)
    cfg.numa_strategy, cfg.numa_hint_strategy = score, hint
    return cfg.kg_config(), nodes, pods


def zone_mask(code):
    if code < 0 or abi.ZONE_RESERVE_FAIL <= code < 0x40:  # none, or a BestEffort Reserve that fails
        return 0
    return code & 0xF if code >= 0x40 else 1 << code


# ---- oracle properties (CPU) -----------------------------------------------------------------------

def test_oracle_affinities_are_consistent():
    kc, nodes, pods = workload(1, 400, 160)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    npol, Z = nodes["numa_policy"], nodes["numa_zones"]
    ppol = pods["numa_policy"]
    ok = ref.status == 0
    for j, i in zip(*np.nonzero(ok)):
        pol = ppol[j] if ppol[j] != abi.KG_NUMA_NONE else npol[i]
        if abi.ZONE_RESERVE_FAIL <= int(ref.numa_zone[j, i]) < 0x40:
            assert pol == abi.KG_NUMA_BEST_EFFORT, (j, i)  # only a BestEffort Reserve can fail after Filter
            continue
        m = zone_mask(int(ref.numa_zone[j, i]))
        assert m >> int(Z[i]) == 0, (j, i)
        if pol == abi.KG_NUMA_NONE:
            assert m == 0
        if pol == abi.KG_NUMA_SINGLE_NODE:
            assert bin(m).count("1") <= 1  # one zone, or no allocation (single-zone node / no request)
        if m:
            # the split is feasible: every requested resource fits in the chosen zones
            for res, key in ((0, "cpu"), (1, "mem")):
                req = pods[f"req_{key}"][j]
                avail = sum(max(0, int(nodes[f"zone_{key}{z}"][i]) - int(nodes[f"zone_{key}_used{z}"][i]))
                            for z in range(int(Z[i])) if (m >> z) & 1)
                assert req <= avail, (j, i, key)
    # the workload reaches every outcome of the topology manager
    st = ref.status
    for bit in (abi.KG_ST_NUMA_UNSATISFIED, abi.KG_ST_NUMA_ALIGN, abi.KG_ST_NUMA_NO_RES, abi.KG_ST_NUMA_CONFLICT):
        assert (st & bit).any(), hex(bit)
    codes = ref.numa_zone[ok]
    assert (codes >= 0x40).any() and ((codes >= 0) & (codes < 4)).any()


def best_effort_workload(seed=7, n_nodes=600, n_pods=200):
    """synth.topology plus a few BestEffort two-zone nodes whose zones are fuller than the node-level
    requested (the NRT view can lag the NodeInfo): pods pass their Filter, score them high, and the
    allocation over their zones falls short at Reserve."""
    kc, nodes, pods = workload(seed, n_nodes, n_pods)
    tight = np.flatnonzero((nodes["numa_policy"] == abi.KG_NUMA_BEST_EFFORT) & (nodes["numa_zones"] == 2))[:40]
    for z in range(2):
        nodes[f"zone_cpu_used{z}"][tight] = nodes[f"zone_cpu{z}"][tight] - 1500
        nodes[f"zone_mem_used{z}"][tight[::2]] = nodes[f"zone_mem{z}"][tight[::2]] - (1 << 30)
    nodes["req_cpu"][tight] = nodes["alloc_cpu"][tight] // 4
    nodes["nz_cpu"][tight] = np.maximum(nodes["nz_cpu"][tight], nodes["req_cpu"][tight])
    return kc, nodes, pods


def test_oracle_best_effort_admits_in_reserve_only():
    """BestEffort runs no FilterByNUMANode in Filter (plugin.go:446-455): its pairs carry no NUMA admit
    reason and score node allocatable / requested; the Reserve's topology manager decides the zone, and
    a failing allocation ("Insufficient NUMA cpu / memory") or a node without NUMA resources ("node(s)
    Insufficient NUMA Node resources") shows as a Reserve-failure zone code on a feasible pair."""
    kc, nodes, pods = best_effort_workload()
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    npol, ppol = nodes["numa_policy"], pods["numa_policy"]
    be = (npol[None, :] == abi.KG_NUMA_BEST_EFFORT) & ((ppol[:, None] == abi.KG_NUMA_NONE) |
                                                       (ppol[:, None] == abi.KG_NUMA_BEST_EFFORT))
    admit = abi.KG_ST_NUMA_UNSATISFIED | abi.KG_ST_NUMA_ALIGN | abi.KG_ST_NUMA_NO_RES
    assert not (ref.status[be] & admit).any()
    codes = ref.numa_zone[be & (ref.status == 0)]
    fails = codes[(codes >= abi.ZONE_RESERVE_FAIL) & (codes < 0x40)]
    assert len(fails) > 0 and ((fails & 4) != 0).any() and ((fails & 3) != 0).any()
    # the Reserve of a failing pair fails in the oracle too, and nothing changes
    st = oracle_lib.OracleState(kc, nodes)
    j, i = np.argwhere(be & (ref.status == 0) & (ref.numa_zone >= abi.ZONE_RESERVE_FAIL) & (ref.numa_zone < 0x40))[0]
    before = st.table()
    assert not st.assume(int(i), pods, int(j))
    after = st.table()
    for k in before:
        assert np.array_equal(before[k], after[k]), k


def test_oracle_exclusive_policy_respects_zone_status():
    """Pods carrying their own policy run the Required exclusive policy: a single-zone affinity never
    lands on a shared zone, a multi-zone one never spans a zone held by a single-NUMA pod."""
    kc, nodes, pods = workload(2, 400, 160)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    status = nodes["numa_zone_status"]
    for j, i in zip(*np.nonzero((ref.status == 0) & (pods["numa_policy"][:, None] != abi.KG_NUMA_NONE))):
        if pods["numa_policy"][j] == abi.KG_NUMA_BEST_EFFORT:
            continue  # BestEffort admits non-preferred hints
        m = zone_mask(int(ref.numa_zone[j, i]))
        zs = [(int(status[i]) >> (2 * z)) & 3 for z in range(4) if (m >> z) & 1]
        if len(zs) == 1:
            assert zs[0] != 2, (j, i)
        elif len(zs) > 1:
            assert 1 not in zs, (j, i)


def test_oracle_strategies_change_scores():
    kc0, nodes, pods = workload(3, 200, 64)
    kc1, _, _ = workload(3, 200, 64, score="MostAllocated")
    a = oracle_lib.eval_verify(kc0, nodes, pods)
    b = oracle_lib.eval_verify(kc1, nodes, pods)
    ok = (a.status == 0) & (b.status == 0)
    assert np.array_equal(a.status, b.status)
    assert (a.score_numa[ok] != b.score_numa[ok]).any()


# ---- device parity (GPU) ---------------------------------------------------------------------------

@pytest.fixture(scope="module")
def ctx():
    c = engine.Context(0)
    yield c
    c.close()


def assert_equal(got, ref, what=""):
    for name in FIELDS:
        a, b = getattr(got, name), getattr(ref, name)
        if not np.array_equal(a, b):
            bad = np.argwhere(a != b)
            j, i = bad[0]
            raise AssertionError(f"{what}: {name} differs at {len(bad)} pairs, first pod {j} node {i}: "
                                 f"gpu={a[j, i]} oracle={b[j, i]}")


@pytest.mark.gpu
@pytest.mark.parametrize("score,hint", STRATEGIES)
@pytest.mark.parametrize("seed", [1, 2])
def test_topology_verify(ctx, seed, score, hint):
    kc, nodes, pods = workload(seed, 700, 192, score, hint)
    got = engine.eval_verify(engine.Snapshot(ctx, kc, nodes), engine.PodBatch(ctx, pods))
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    assert_equal(got, ref, f"seed {seed} {score}/{hint}")
    assert (ref.numa_zone >= 0x40).any()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 3])
def test_topology_select(ctx, k):
    kc, nodes, pods = workload(4, 3000, 256)
    got = engine.eval_select(engine.Snapshot(ctx, kc, nodes), engine.PodBatch(ctx, pods), k)
    want = oracle_lib.select(kc, nodes, pods, k)
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("score", ["LeastAllocated", "MostAllocated"])
def test_topology_replay(ctx, score):
    """Sequential placement with multi-zone allocations applied between pods."""
    kc, nodes, pods = workload(5, 1200, 2500, score=score)
    snap = engine.Snapshot(ctx, kc, nodes)
    node, total = engine.replay(snap, engine.PodBatch(ctx, pods))
    ost = oracle_lib.OracleState(kc, nodes)
    onode, ototal = ost.replay(pods)
    assert np.array_equal(node, onode)
    assert np.array_equal(total, ototal)
    state, want = snap.read_state(), ost.table()
    for z in range(abi.KG_MAX_ZONES):
        for k in (f"zone_cpu_used{z}", f"zone_mem_used{z}"):
            assert np.array_equal(state[k], want[k]), k
    for k in ("req_cpu", "req_mem", "num_pods"):
        assert np.array_equal(state[k], want[k]), k
    assert (node < 0).any() and (node >= 0).any()


@pytest.mark.gpu
def test_topology_assume_forget(ctx):
    """Reserve through the C ABI (zone chosen on the device, split over several zones where the hint
    spans them) equals the oracle's Reserve; Unreserve restores single-zone allocations and refuses a
    multi-zone one (not restated)."""
    kc, nodes, pods = workload(6, 300, 96)
    snap, batch = engine.Snapshot(ctx, kc, nodes), engine.PodBatch(ctx, pods)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    ost = oracle_lib.OracleState(kc, nodes)
    before = snap.read_state()
    ok = np.argwhere(ref.status == 0)
    multi = [tuple(x) for x in ok if ref.numa_zone[x[0], x[1]] >= 0x40][:3]
    single = [tuple(x) for x in ok if 0 <= ref.numa_zone[x[0], x[1]] < 4 and tuple(x)[1] not in
              {m[1] for m in multi}][:3]
    assert multi and single
    for j, i in single:
        engine.assume(snap, batch, int(j), int(i))
        ost.assume(int(i), pods, int(j))
    for j, i in single[::-1]:
        engine.forget(snap, batch, int(j), int(i), int(ref.numa_zone[j, i]))
    oracle_lib.assert_state_restored(before, snap.read_state())
    for j, i in multi:
        engine.assume(snap, batch, int(j), int(i))
    for j, i in single[::-1]:
        ost.forget(int(i), pods, int(j), int(ref.numa_zone[j, i]))
    for j, i in multi:
        ost.assume(int(i), pods, int(j))
    state, want = snap.read_state(), ost.table()
    for z in range(abi.KG_MAX_ZONES):
        assert np.array_equal(state[f"zone_cpu_used{z}"], want[f"zone_cpu_used{z}"])
        assert np.array_equal(state[f"zone_mem_used{z}"], want[f"zone_mem_used{z}"])
    j, i = multi[0]
    with pytest.raises(engine.Unsupported):
        engine.forget(snap, batch, int(j), int(i), int(ref.numa_zone[j, i]))


@pytest.mark.gpu
def test_topology_multi_zone_unreserve(ctx):
    """kg_assume_numa returns the allocation the Reserve made (per-zone cpu / memory; a split over several zones for
    0x40 | mask codes) and kg_forget_numa releases exactly it (resource_manager.go:478-483 Release): Reserve of
    several multi-zone and single-zone pods, their Unreserve in another order, every column back to the start. The
    amounts of each split cover the pod's request and sit on the zones of its mask; the zone state after the
    Reserves equals the oracle's."""
    kc, nodes, pods = workload(6, 300, 96)
    snap, batch = engine.Snapshot(ctx, kc, nodes), engine.PodBatch(ctx, pods)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    ost = oracle_lib.OracleState(kc, nodes)
    before = snap.read_state()
    ok = np.argwhere(ref.status == 0)
    multi, used = [], set()
    for j, i in ok:
        if ref.numa_zone[j, i] >= 0x40 and i not in used:
            multi.append((int(j), int(i)))
            used.add(i)
        if len(multi) == 4:
            break
    single = [(int(j), int(i)) for j, i in ok if 0 <= ref.numa_zone[j, i] < 4 and i not in used][:2]
    assert len(multi) >= 2 and single
    made = []
    for j, i in multi + single:
        zone, amounts = engine.assume_numa(snap, batch, j, i)
        assert zone == int(ref.numa_zone[j, i])
        ost.assume(i, pods, j)
        mask = zone & 0xF if zone >= 0x40 else 1 << zone
        off = [z for z in range(abi.KG_MAX_ZONES) if not (mask >> z) & 1]
        assert not amounts[:, off].any()
        if pods["flags"][j] & abi.KG_POD_HAS_CPU:
            assert amounts[0].sum() == pods["req_cpu"][j]
        if pods["flags"][j] & abi.KG_POD_HAS_MEM:
            assert amounts[1].sum() == pods["req_mem"][j]
        made.append((j, i, zone, amounts))
    state, want = snap.read_state(), ost.table()
    for z in range(abi.KG_MAX_ZONES):
        assert np.array_equal(state[f"zone_cpu_used{z}"], want[f"zone_cpu_used{z}"])
        assert np.array_equal(state[f"zone_mem_used{z}"], want[f"zone_mem_used{z}"])
    for j, i, zone, amounts in made[1::2] + made[0::2]:
        engine.forget_numa(snap, batch, j, i, zone, amounts)
    oracle_lib.assert_state_restored(before, snap.read_state())


@pytest.mark.gpu
def test_best_effort_reserve_failures(ctx):
    """The BestEffort semantics on the device: Filter / Score / select without the topology manager, the
    Reserve's zone (or failure) in verify, replays that leave a pod unscheduled when its selected node's
    Reserve fails (reasons carry KG_ST_NUMA_INSUF_*), and kg_assume refusing with KG_RESERVE_FAILED."""
    kc, nodes, pods = best_effort_workload(8, 700, 400)
    snap, batch = engine.Snapshot(ctx, kc, nodes), engine.PodBatch(ctx, pods)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    assert_equal(engine.eval_verify(snap, batch), ref, "verify")
    for k in (1, 3):
        assert np.array_equal(engine.eval_select(snap, batch, k), oracle_lib.select(kc, nodes, pods, k)), k
    onode, ototal, owhy = oracle_lib.OracleState(kc, nodes).replay(pods, reasons=True)
    failed = (onode < 0) & ((owhy & abi.KG_ST_NUMA_RESERVE) != 0)
    assert failed.any()
    node, total, why = engine.replay(snap, batch, reasons=True)
    assert np.array_equal(node, onode) and np.array_equal(total, ototal) and np.array_equal(why, owhy)
    snap.upload(nodes)
    node2, total2 = engine.replay(snap, batch)  # window replay (no reasons)
    assert np.array_equal(node2, onode) and np.array_equal(total2, ototal)
    snap.upload(nodes)
    j, i = np.argwhere((ref.status == 0) & (ref.numa_zone >= abi.ZONE_RESERVE_FAIL) & (ref.numa_zone < 0x40))[0]
    before = snap.read_state()
    with pytest.raises(engine.ReserveFailed):
        engine.assume(snap, batch, int(j), int(i))
    oracle_lib.assert_state_restored(before, snap.read_state())
