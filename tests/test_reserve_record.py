"""kg_reserve / kg_unreserve (ABI 11): the Unreserve of every plugin from the record its Reserve left
(nodenumaresource/plugin.go:700-720 -> resource_manager.go:478-483 Release, node_allocation.go:164-200;
reservation/plugin.go:1409-1460 forgetPods; deviceshare / elasticquota Unreserve; load_aware.go:231-233).

- Known answers (CPU oracle and GPU device): node_allocation_test.go:99-124 TestNodeAllocationStateReleaseCPUs,
  :126-150 Test_cpuAllocation_getAvailableCPUs (two pods sharing CPUs under maxRefCount 2, release of one), and
  plugin_test.go:2203-2240 TestPlugin_Unreserve (a Release gives every CPU back).
- Round trips: Reserve then Unreserve restores the node state exactly (CPU RefCounts, exclusive policies, the NUMA
  single / shared pod counts and statuses, zone used, NodeInfo, LoadAware bases, GPU minors, quota used, and the
  reservation views / infos), apart from the zones' allocation records, which a Release keeps.
- Device parity: interleaved Reserves and Unreserves on cpuset clusters equal the oracle's state after every step."""
import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, synth
from koordinator_amd.config import bench_profile

TOPO = (2, 1, 4, 2)  # buildCPUTopologyForTest(2, 1, 4, 2): 16 CPUs, NUMA node 0 = CPUs 0-7


def _one_node(pods_cpus, max_ref=1, excl=abi.KG_CPU_EXCL["PCPULevel"]):
    """One node with the CPU topology and the given pods' cpusets allocated (addCPUs), and one batch pod per cpuset
    (a cpuset-binding pod requesting that many CPUs)."""
    cfg, t, p = synth.small(1, len(pods_cpus), seed=3, numa=True)
    t["numa_policy"][:] = abi.KG_NUMA_NONE
    t["cpu_topo"] = np.zeros(1, np.int32)
    t["cpu_topos"] = abi.cpu_topos_array([abi.cpu_topo_for_test(*TOPO)])
    alloc = np.zeros((1, 2 * abi.KG_MAX_CPUS), np.uint8)
    single = shared = 0
    for cpus in pods_cpus:
        used = set()
        for c in cpus:
            alloc[0, c] += 1
            alloc[0, abi.KG_MAX_CPUS + c] = excl
            used.add(c // 8)
        for z in used:
            if len(used) > 1:
                shared += 1 << (8 * (abi.KG_MAX_ZONES + z))
            else:
                single += 1 << (8 * z)
    t["cpu_alloc"] = alloc
    t["cpu_max_ref"] = np.full(1, max_ref, np.uint8)
    t["cpuset_alloc_milli"] = np.array([1000 * int((alloc[0, :abi.KG_MAX_CPUS] > 0).sum())], np.int64)
    t["numa_zone_pods"] = np.array([single + shared], np.uint64)
    st = 0
    for z in range(2):
        s1 = (single >> (8 * z)) & 0xFF
        s2 = (shared >> (8 * (abi.KG_MAX_ZONES + z))) & 0xFF
        st |= (2 if s2 else 1 if s1 else 0) << (2 * z)
    t["numa_zone_status"] = np.array([st], np.uint32)
    t["req_cpu"][:] = 1000 * sum(len(c) for c in pods_cpus)
    p["req_cpu"] = np.array([1000 * len(c) for c in pods_cpus], np.int64)
    p["nz_cpu"] = p["req_cpu"].copy()
    p["flags"] = (p["flags"] | abi.KG_POD_CPU_BIND | (1 << abi.KG_POD_CPU_POLICY_SHIFT)).astype(np.uint32)
    return cfg, t, p


def _record(cpus):
    rec = abi.KgReserveRecord()
    rec.numa_zone = -1
    rec.rsv_rid = -1
    rec.flags = abi.KG_RECORD_CPUSET
    m = abi.cpu_mask(cpus)
    for w in range(4):
        rec.cpus[w] = int(m[w])
    return rec


# (reference case, allocated pods' cpusets, maxRefCount, pod released, expected RefCounts, NUMA node 0 status)
RELEASE_KATS = [
    ("node_allocation_test.go:99 TestNodeAllocationStateReleaseCPUs", [range(1, 5)], 1, 0, {}, 0),
    ("node_allocation_test.go:126 Test_cpuAllocation_getAvailableCPUs", [range(1, 5), range(2, 6)], 2, 0,
     {2: 1, 3: 1, 4: 1, 5: 1}, 1),
    ("plugin_test.go:2203 TestPlugin_Unreserve", [range(0, 4)], 1, 0, {}, 0),
]


def _check_release(state, want_refs, want_status):
    refs = state["cpu_alloc"][0, :abi.KG_MAX_CPUS]
    excl = state["cpu_alloc"][0, abi.KG_MAX_CPUS:]
    got = {c: int(refs[c]) for c in range(16) if refs[c]}
    assert got == want_refs
    assert all(excl[c] == 0 for c in range(16) if refs[c] == 0)  # a CPU at RefCount 0 leaves allocatedCPUs
    assert int(state["cpuset_alloc_milli"][0]) == 1000 * len(want_refs)
    assert int(state["numa_zone_status"][0]) & 3 == want_status
    assert (int(state["numa_zone_pods"][0]) & 0xFF) == (1 if want_status == 1 else 0)


@pytest.mark.parametrize("case", RELEASE_KATS, ids=[c[0].split()[1] for c in RELEASE_KATS])
def test_cpuset_release_kat_oracle(case):
    _, sets, max_ref, pod, want_refs, want_status = case
    cfg, t, p = _one_node([list(s) for s in sets], max_ref)
    st = oracle_lib.OracleState(cfg.kg_config(), t)
    st.unreserve(0, p, pod, _record(list(sets[pod])))
    _check_release(st.table(), want_refs, want_status)


@pytest.mark.gpu
@pytest.mark.parametrize("case", RELEASE_KATS, ids=[c[0].split()[1] for c in RELEASE_KATS])
def test_cpuset_release_kat_device(case):
    from koordinator_amd import engine
    _, sets, max_ref, pod, want_refs, want_status = case
    cfg, t, p = _one_node([list(s) for s in sets], max_ref)
    ctx = engine.Context(0)
    snap = engine.Snapshot(ctx, cfg.kg_config(), t)
    batch = engine.PodBatch(ctx, p)
    engine.unreserve(snap, batch, pod, 0, _record(list(sets[pod])))
    _check_release(snap.read_state(), want_refs, want_status)
    ctx.close()


def _winners(kc, nodes, pods):
    """Each pod's best node on the untouched cluster (the round trips Reserve every pod there independently)."""
    keys = oracle_lib.select(kc, nodes, pods, 1)[:, 0]
    return np.where(keys != 0, abi.key_node(keys), -1)


def test_reserve_unreserve_round_trip_oracle():
    """Reserve then Unreserve of each pod on its best node of the mixed cluster (cpusets under every NUMA policy, LSR
    pods, CPU-bind-policy nodes) restores the oracle state exactly."""
    cfg, nodes, pods = synth.mixed(300, 150, seed=21)
    kc = cfg.kg_config()
    st = oracle_lib.OracleState(kc, nodes)
    before = st.table()
    best = _winners(kc, nodes, pods)
    n_cpuset = 0
    for j in range(abi.table_len(pods)):
        if best[j] < 0:
            continue
        ok, rec = st.reserve(int(best[j]), pods, j)
        if not ok:
            continue
        n_cpuset += bool(rec.flags & abi.KG_RECORD_CPUSET)
        st.unreserve(int(best[j]), pods, j, rec)
        oracle_lib.assert_state_restored(before, st.table())
    assert n_cpuset >= 5


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [22, 23])
def test_interleaved_reserve_unreserve_device_vs_oracle(seed):
    """A sequence of kg_reserve / kg_unreserve on the mixed cluster (every third Reserve undone two steps later, so
    Releases land between other pods' allocations on shared nodes) equals the oracle's kgo_reserve / kgo_unreserve
    after every step: records, NodeInfo, zones, CPU RefCounts and exclusive policies, single / shared counts."""
    from koordinator_amd import engine
    cfg, nodes, pods = synth.mixed(200, 90, seed=seed)
    # crowd the pods onto a few nodes so that cpusets of different pods meet there
    kc = cfg.kg_config()
    best = _winners(kc, nodes, pods)
    ctx = engine.Context(0)
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    st = oracle_lib.OracleState(kc, nodes)
    held = []
    keys = ("req_cpu", "req_mem", "num_pods", "cpuset_alloc_milli", "numa_zone_status", "numa_zone_pods", "cpu_alloc",
            "zone_cpu_used0", "zone_cpu_used1", "zone_mem_used0", "zone_mem_used1", "la_fbase_np0")
    n_cpuset = 0
    for j in range(abi.table_len(pods)):
        node = int(best[j]) if best[j] >= 0 else int(best[best >= 0][0])
        node = node % 12  # a dozen nodes take every pod
        ok, orec = st.reserve(node, pods, j)
        try:
            drec = engine.reserve(snap, batch, j, node)
            dok = True
        except engine.ReserveFailed:
            dok = False
        assert ok == dok, j
        if ok:
            assert drec.numa_zone == orec.numa_zone and list(drec.cpus) == list(orec.cpus), j
            assert list(drec.zone_amounts) == list(orec.zone_amounts), j
            n_cpuset += bool(orec.flags & abi.KG_RECORD_CPUSET)
            held.append((j, node, drec, orec))
        if j % 3 == 2 and len(held) >= 2:
            k, kn, dr, orr = held.pop(-2)
            engine.unreserve(snap, batch, k, kn, dr)
            st.unreserve(kn, pods, k, orr)
        dev, want = snap.read_state(), st.table()
        for c in keys:
            assert np.array_equal(dev[c], want[c]), (j, c)
    assert n_cpuset >= 3
    ctx.close()


@pytest.mark.gpu
def test_reserve_unreserve_round_trip_config5_views():
    """Config 5 with reservation views, quotas, GPU minors and cpuset pods: kg_reserve of pods on their best nodes
    (many into reservations) and kg_unreserve of all of them in reverse order leave the device as it was: node state,
    GPU minors, quota used, the views and reservation infos (read back), and the select of the batch."""
    from koordinator_amd import engine
    cfg, nodes, pods, quotas, rsv = synth.cluster5(800, 200, seed_config=95, numa="mix", usage="u01", rsv_gpu=False,
                                                   rsv_frac=0.3)
    pods = {k: v.copy() for k, v in pods.items()}
    nodes, pods = synth.add_cpusets(nodes, pods, 95, bind_frac=0.15)
    rng = np.random.default_rng(95)
    pods["rsv_class"] = np.where(rng.random(len(pods["rsv_class"])) < 0.7,
                                 rng.integers(0, synth.N_RSV_CLASSES, len(pods["rsv_class"])), -1).astype(np.int32)
    kc = cfg.kg_config()
    ctx = engine.Context(0)
    snap = engine.Snapshot(ctx, kc, nodes)
    snap.upload_quotas(quotas)
    snap.upload_reservations(rsv)
    batch = engine.PodBatch(ctx, pods)
    keys0 = engine.eval_select(snap, batch, 1)
    state0 = snap.read_state()
    q0 = snap.read_quotas()
    r0 = snap.read_reservations(rsv)
    best = np.where(keys0[:, 0] != 0, abi.key_node(keys0[:, 0]), -1)
    done = []
    for j in range(abi.table_len(pods)):
        if best[j] < 0:
            continue
        try:
            done.append((j, int(best[j]), engine.reserve(snap, batch, j, int(best[j]))))
        except engine.ReserveFailed:
            pass
    assert sum(1 for _, _, r in done if r.rsv_rid >= 0) >= 10  # pods joined reservations
    assert sum(1 for _, _, r in done if r.flags & abi.KG_RECORD_CPUSET) >= 3
    assert sum(1 for _, _, r in done if r.gpu_minors) >= 10
    mid = snap.read_reservations(rsv)
    assert any(mid.infos[x].allocated_pods != r0.infos[x].allocated_pods for x in range(rsv.n_infos))
    for j, node, rec in reversed(done):
        engine.unreserve(snap, batch, j, node, rec)
    oracle_lib.assert_state_restored(state0, snap.read_state())
    q1 = snap.read_quotas()
    for a, b in zip(q0, q1):
        assert np.array_equal(a, b)
    r1 = snap.read_reservations(rsv)
    for x in range(rsv.n_views):
        for f in ("req", "pod_requested", "r_allocated"):
            assert list(getattr(r1.views[x], f)) == list(getattr(r0.views[x], f)), (x, f)
        for f in ("nz_cpu", "nz_mem", "num_pods"):
            assert getattr(r1.views[x], f) == getattr(r0.views[x], f), (x, f)
    for x in range(rsv.n_infos):
        assert list(r1.infos[x].allocated) == list(r0.infos[x].allocated), x
        assert r1.infos[x].allocated_pods == r0.infos[x].allocated_pods, x
    assert np.array_equal(engine.eval_select(snap, batch, 1), keys0)
    ctx.close()


@pytest.mark.gpu
def test_reserve_unreserve_round_trip_gpu_reservations():
    """Reservations that hold GPUs (restore inputs uploaded): kg_reserve of GPU pods on their best nodes (into the
    reservations' minors where nominated) and kg_unreserve in reverse order restore the GPU tables, views, infos and the
    select of the batch exactly; the Reserves matched the oracle replay's first placements."""
    from koordinator_amd import engine
    cfg, nodes, pods, quotas, rsv = synth.cluster5(600, 150, seed_config=96, rsv_frac=0.5, usage="u01")
    pods = {k: v.copy() for k, v in pods.items()}
    rng = np.random.default_rng(96)
    pods["rsv_class"] = np.where(rng.random(len(pods["rsv_class"])) < 0.7,
                                 rng.integers(0, synth.N_RSV_CLASSES, len(pods["rsv_class"])), -1).astype(np.int32)
    pods["flags"] &= ~np.uint32(abi.KG_POD_RSV_REQUIRED)
    kc = cfg.kg_config()
    ctx = engine.Context(0)
    snap = engine.Snapshot(ctx, kc, nodes)
    snap.upload_quotas(quotas)
    snap.upload_reservations(rsv)
    batch = engine.PodBatch(ctx, pods)
    keys0 = engine.eval_select(snap, batch, 1)
    state0, q0, r0 = snap.read_state(), snap.read_quotas(), snap.read_reservations(rsv)
    best = np.where(keys0[:, 0] != 0, abi.key_node(keys0[:, 0]), -1)
    done = []
    for j in range(abi.table_len(pods)):
        if best[j] >= 0:
            try:
                done.append((j, int(best[j]), engine.reserve(snap, batch, j, int(best[j]))))
            except engine.ReserveFailed:
                pass
    assert sum(1 for _, _, r in done if r.gpu_minors and r.rsv_rid >= 0) >= 2
    for j, node, rec in reversed(done):
        engine.unreserve(snap, batch, j, node, rec)
    oracle_lib.assert_state_restored(state0, snap.read_state())
    for a, b in zip(q0, snap.read_quotas()):
        assert np.array_equal(a, b)
    r1 = snap.read_reservations(rsv)
    for x in range(rsv.n_infos):
        assert list(r1.infos[x].allocated) == list(r0.infos[x].allocated), x
        assert r1.infos[x].allocated_pods == r0.infos[x].allocated_pods, x
    assert np.array_equal(engine.eval_select(snap, batch, 1), keys0)
    ctx.close()


@pytest.mark.gpu
def test_zone_pod_counts_saturate_at_255():
    """NUMANodeSharedStatus pod counts are kept in one byte and saturate at 255, on the device as in the oracle (and the
    host's zone_pods): a cpuset Reserve on NUMA nodes that already count 255 single-NUMA pods keeps 255 (the node stays
    busy), and its Unreserve then counts one less."""
    from koordinator_amd import engine
    cfg, t, p = _one_node([range(0, 2)], max_ref=1)
    t["numa_zone_pods"] = np.array([255 | (255 << 8)], np.uint64)
    t["numa_zone_status"] = np.array([1 | (1 << 2)], np.uint32)
    p["flags"] = ((p["flags"] & ~np.uint32(abi.KG_POD_NUMA_SKIP)) | abi.KG_POD_HAS_CPU).astype(np.uint32)
    kc = cfg.kg_config()
    st = oracle_lib.OracleState(kc, t)
    ok, orec = st.reserve(0, p, 0)
    assert ok and orec.flags & abi.KG_RECORD_CPUSET
    ctx = engine.Context(0)
    try:
        snap = engine.Snapshot(ctx, kc, t)
        batch = engine.PodBatch(ctx, p)
        drec = engine.reserve(snap, batch, 0, 0)
        assert list(drec.cpus) == list(orec.cpus)
        dev, want = snap.read_state(), st.table()
        assert int(want["numa_zone_pods"][0]) & 0xFFFF == 255 | (255 << 8)
        for c in ("numa_zone_pods", "numa_zone_status", "cpu_alloc"):
            assert np.array_equal(dev[c], want[c]), c
        engine.unreserve(snap, batch, 0, 0, drec)
        st.unreserve(0, p, 0, orec)
        dev, want = snap.read_state(), st.table()
        assert int(want["numa_zone_pods"][0]) & 0xFFFF != 255 | (255 << 8)  # one NUMA node counts 254 now
        for c in ("numa_zone_pods", "numa_zone_status", "cpu_alloc"):
            assert np.array_equal(dev[c], want[c]), c
    finally:
        ctx.close()
