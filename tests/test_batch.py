"""Whole-job placement: the FindOneNodePlugin slot driving the replay kernel and the
inline batch cycle (kg_snapshot_checkpoint / kg_snapshot_rollback / kg_batch_schedule, koordinator_amd.batch).

Reference: frameworkext/interface.go:115-145, framework_extender.go:356-407, batch/batch_scheduler.go:74-185,
batch/engine.go:92-294,348-371, batch/framework/types.go:275-341. The oracle restates the cycle in
oracle/kg_oracle.c kgo_batch_schedule; parity is bit-exact on result codes, status bits, NUMA zones, GPU
minors, the final node state and quota used.
"""
import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, batch, synth

STATE_COLS = ("req_cpu", "req_mem", "req_eph", "num_pods", "nz_cpu", "nz_mem", "sc_req0", "sc_req1",
              "zone_cpu_used0", "zone_cpu_used1", "zone_mem_used0", "zone_mem_used1",
              "la_fbase_np0", "la_fbase_np1", "la_fbase_prod0", "la_fbase_prod1")


def oracle_state_cols(st: oracle_lib.OracleState):
    t = st.table()
    return {k: t[k] for k in STATE_COLS}


def grouped(plan):
    """Batch order of kg_batch_schedule: groups in first-appearance order, each in batch order."""
    order, seen = [], {}
    for j, n in enumerate(plan):
        seen.setdefault(int(n), []).append(j)
    for js in seen.values():
        order.extend(js)
    return order


# ---------------------------------------------------------------------------------------------- CPU

def test_sort_pods_by_index():
    P = batch.JobPod
    pods = [P("ns", "b"), P("ns", "a"), P("ns", "z", annotations={batch.ANNOTATION_TOPOLOGY_INDEX: "2"}),
            P("ns", "y", annotations={batch.ANNOTATION_TOPOLOGY_INDEX: "1"}),
            P("ns", "c", annotations={batch.ANNOTATION_TOPOLOGY_INDEX: "x"})]
    order = batch.sort_pods_by_index(range(len(pods)), pods)
    assert [pods[i].name for i in order] == ["y", "z", "a", "b", "c"]


def test_filter_message_first_plugin():
    bits = abi.KG_ST_LA_CPU | abi.KG_ST_NRF_CPU | abi.KG_ST_NRF_MEM
    assert batch.filter_message(bits) == "Insufficient cpu, Insufficient memory"
    assert batch.filter_message(abi.KG_ST_LA_MEM) == "node(s) memory usage exceed threshold"


def test_oracle_batch_replayed_plan_commits():
    """A plan taken from the oracle's own replay passes the batch cycle pod by pod and ends in the replay's
    state: per node the pods arrive in the same order, and nodes do not interact."""
    cfg, nodes, pods = synth.small(300, 120, seed=41)
    kc = cfg.kg_config()
    a = oracle_lib.OracleState(kc, nodes)
    node, _ = a.replay(pods)
    ok = node >= 0
    assert ok.sum() > 60
    sub = abi.take(pods, np.flatnonzero(ok))
    plan = node[ok]
    b = oracle_lib.OracleState(kc, nodes)
    res, stat, zone, _m, _q, _n = b.batch_schedule(sub, plan)
    assert (res == abi.KG_BATCH_ASSUMED).all() and not stat.any()
    sa, sb = oracle_state_cols(a), oracle_state_cols(b)
    for k in STATE_COLS:
        assert np.array_equal(sa[k], sb[k]), k


def test_oracle_batch_failure_rolls_back():
    cfg, nodes, pods = synth.small(50, 400, seed=42)
    kc = cfg.kg_config()
    st = oracle_lib.OracleState(kc, nodes)
    before = oracle_state_cols(st)
    plan = np.zeros(abi.table_len(pods), np.int32)  # everything on node 0: it fills up
    plan[1::2] = 3
    res, stat, zone, _m, _q, _n = st.batch_schedule(pods, plan)
    assert (res == abi.KG_BATCH_FAILED).sum() == 2  # one per node
    assert (res == abi.KG_BATCH_SIBLING).any() and (res == abi.KG_BATCH_ROLLED_BACK).any()
    first = np.flatnonzero(res == abi.KG_BATCH_FAILED)
    for f in first:  # the failed pod's later group members carry its status
        later = [j for j in range(f + 1, len(plan)) if plan[j] == plan[f]]
        assert (res[later] == abi.KG_BATCH_SIBLING).all() and (stat[later] == stat[f]).all()
    after = oracle_state_cols(st)
    for k in STATE_COLS:
        assert np.array_equal(before[k], after[k]), k
    plan[5] = -1
    res, *_ = st.batch_schedule(pods, plan)
    assert (res == abi.KG_BATCH_NO_PLAN).all()


# ---------------------------------------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def ctx():
    from koordinator_amd import engine
    c = engine.Context(0)
    yield c
    c.close()


def gpu_state_cols(snap):
    t = snap.read_state()
    out = {}
    for k in STATE_COLS:
        out[k] = t[k]
    return out


@pytest.mark.gpu
def test_checkpoint_rollback(ctx):
    from koordinator_amd import engine
    cfg, nodes, pods = synth.small(700, 64, seed=43)
    snap = engine.Snapshot(ctx, cfg.kg_config(), nodes)
    pb = engine.PodBatch(ctx, pods)
    with pytest.raises(engine.EngineError):
        snap.rollback()  # no checkpoint yet
    before = gpu_state_cols(snap)
    keys0 = engine.eval_select(snap, pb, 2)
    g0 = snap.generation()
    snap.checkpoint()
    node, _ = engine.replay(snap, pb)
    assert (node >= 0).sum() > 32
    changed = gpu_state_cols(snap)
    assert any(not np.array_equal(before[k], changed[k]) for k in STATE_COLS)
    snap.rollback()
    assert snap.generation() > g0
    after = gpu_state_cols(snap)
    for k in STATE_COLS:
        assert np.array_equal(before[k], after[k]), k
    assert np.array_equal(engine.eval_select(snap, pb, 2), keys0)  # derived fast blocks restored too
    snap.rollback()  # a checkpoint can be rolled back to more than once
    snap.upload(nodes)
    with pytest.raises(engine.EngineError):
        snap.rollback()  # the re-upload invalidated it


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [44, 45])
def test_batch_schedule_planned_job(ctx, seed):
    """Planner (replay + rollback) then the inline batch cycle of its plan, against the oracle."""
    from koordinator_amd import engine
    cfg, nodes, pods = synth.small(900, 256, seed=seed)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    pb = engine.PodBatch(ctx, pods)
    before = gpu_state_cols(snap)
    snap.checkpoint()
    node, _tot, why = engine.replay(snap, pb, reasons=True)
    snap.rollback()
    ref_node, _rt, ref_why = oracle_lib.OracleState(kc, nodes).replay(pods, reasons=True)
    assert np.array_equal(node, ref_node) and np.array_equal(why, ref_why)
    after = gpu_state_cols(snap)
    for k in STATE_COLS:
        assert np.array_equal(before[k], after[k]), k
    ok = np.flatnonzero(node >= 0)
    sub = abi.take(pods, ok)
    plan = node[ok]
    order = grouped(plan)
    sub, plan = abi.take(sub, np.asarray(order)), plan[order]
    sb = engine.PodBatch(ctx, sub)
    res, stat, zone, minors = engine.batch_schedule(snap, sb, plan)
    ost = oracle_lib.OracleState(kc, nodes)
    rres, rstat, rzone, _m, _q, _n = ost.batch_schedule(sub, plan)
    assert (res == abi.KG_BATCH_ASSUMED).all()
    assert np.array_equal(res, rres) and np.array_equal(stat, rstat) and np.array_equal(zone, rzone)
    got, want = gpu_state_cols(snap), oracle_state_cols(ost)
    for k in STATE_COLS:
        assert np.array_equal(got[k], want[k]), k


@pytest.mark.gpu
def test_batch_schedule_failure_rolls_back(ctx):
    from koordinator_amd import engine
    cfg, nodes, pods = synth.small(60, 300, seed=46)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    before = gpu_state_cols(snap)
    plan = (np.arange(abi.table_len(pods)) % 3).astype(np.int32) * 7  # nodes 0, 7, 14 overfilled
    order = grouped(plan)
    pods, plan = abi.take(pods, np.asarray(order)), plan[order]
    pb = engine.PodBatch(ctx, pods)
    res, stat, zone, _minors = engine.batch_schedule(snap, pb, plan)
    rres, rstat, rzone, *_ = oracle_lib.OracleState(kc, nodes).batch_schedule(pods, plan)
    assert np.array_equal(res, rres) and np.array_equal(stat, rstat) and np.array_equal(zone, rzone)
    assert (res == abi.KG_BATCH_FAILED).sum() == 3 and (res == abi.KG_BATCH_ROLLED_BACK).any()
    after = gpu_state_cols(snap)
    for k in STATE_COLS:
        assert np.array_equal(before[k], after[k]), k
    plan[0] = -1
    res, *_ = engine.batch_schedule(snap, pb, plan)
    assert (res == abi.KG_BATCH_NO_PLAN).all()


@pytest.mark.gpu
@pytest.mark.parametrize("overfill", [False, True])
def test_batch_schedule_ext(ctx, overfill):
    """DeviceShare + ElasticQuota on top of the base plugins: GPU minors, quota gate and quota used."""
    from koordinator_amd import engine
    cfg, nodes, pods, quotas, _rsv = synth.cluster5(800, 200, seed_config=47, rsv_frac=0.0)
    kc = cfg.kg_config()
    kc.plugins = abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_LA | abi.KG_PLUGIN_NUMA | abi.KG_PLUGIN_DEV | abi.KG_PLUGIN_QUOTA
    snap = engine.Snapshot(ctx, kc, nodes)
    snap.upload_quotas(quotas)
    o = oracle_lib.OracleState(kc, nodes)
    ref_node, *_ = o.ext_replay(pods, quotas)
    ok = np.flatnonzero(ref_node >= 0)
    sub, plan = abi.take(pods, ok), ref_node[ok].astype(np.int32)
    if overfill:
        plan[len(plan) // 2:] = plan[0]
    order = grouped(plan)
    sub, plan = abi.take(sub, np.asarray(order)), plan[order]
    q_before = snap.read_quotas()[0].copy()
    pb = engine.PodBatch(ctx, sub)
    res, stat, zone, minors = engine.batch_schedule(snap, pb, plan)
    ost = oracle_lib.OracleState(kc, nodes)
    rres, rstat, rzone, rminors, qu, _qn = ost.batch_schedule(sub, plan, quotas)
    assert np.array_equal(res, rres) and np.array_equal(stat, rstat)
    assert np.array_equal(zone, rzone) and np.array_equal(minors, rminors)
    assert np.array_equal(snap.read_quotas()[0], qu)
    assert np.array_equal(snap.read_state()["dev_free"], ost.dev_free())
    if overfill:
        assert (res == abi.KG_BATCH_FAILED).sum() >= 1 and np.array_equal(snap.read_quotas()[0], q_before)
    else:
        assert (res == abi.KG_BATCH_ASSUMED).all() and (minors != 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("overfill", [False, True])
def test_batch_schedule_with_gpu_reservations(ctx, overfill):
    """Reservations that hold GPUs: the batch cycle follows each GPU pod's Reserve into the node's DeviceShare restore
    inputs and tables (kg_snapshot_upload_rsv_gpu); results, minors, quota used and the GPU tables equal the oracle's,
    and a failed job restores them (the select after it equals the oracle's on the untouched cluster)."""
    from koordinator_amd import engine
    cfg, nodes, pods, quotas, rsv = synth.cluster5(600, 160, seed_config=48, rsv_frac=0.5)
    assert any(int(i.dev) >= 0 for i in rsv.infos[:rsv.n_infos]) and rsv.n_gpu > 0
    pods = {k: v.copy() for k, v in pods.items()}
    rng = np.random.default_rng(48)
    pods["rsv_class"] = np.where(rng.random(len(pods["rsv_class"])) < 0.7,
                                 rng.integers(0, synth.N_RSV_CLASSES, len(pods["rsv_class"])), -1).astype(np.int32)
    pods["flags"] &= ~np.uint32(abi.KG_POD_RSV_REQUIRED)
    kc = cfg.kg_config()
    ref_node, *_ = oracle_lib.OracleState(kc, nodes).ext_replay(pods, quotas, rsv=rsv)
    ok = np.flatnonzero(ref_node >= 0)
    sub, plan = abi.take(pods, ok), ref_node[ok].astype(np.int32)
    if overfill:
        plan[len(plan) // 2:] = plan[0]
    order = grouped(plan)
    sub, plan = abi.take(sub, np.asarray(order)), plan[order]
    snap = engine.Snapshot(ctx, kc, nodes)
    snap.upload_quotas(quotas)
    snap.upload_reservations(rsv)
    pb = engine.PodBatch(ctx, sub)
    res, stat, zone, minors = engine.batch_schedule(snap, pb, plan)
    ost = oracle_lib.OracleState(kc, nodes)
    rres, rstat, rzone, rminors, qu, _qn = ost.batch_schedule(sub, plan, quotas, rsv)
    assert np.array_equal(res, rres) and np.array_equal(stat, rstat)
    assert np.array_equal(zone, rzone) and np.array_equal(minors, rminors)
    assert np.array_equal(snap.read_quotas()[0], qu)
    assert np.array_equal(snap.read_state()["dev_free"], ost.dev_free())
    if overfill:
        assert (res == abi.KG_BATCH_FAILED).sum() >= 1
        keys = engine.eval_select(snap, pb, 1)
        want = oracle_lib.ext_select(kc, nodes, sub, 1, quotas=quotas, rsv=rsv)
        assert np.array_equal(keys, want)
    else:
        assert (res == abi.KG_BATCH_ASSUMED).all() and (minors != 0).any()


def _rsv_batch_case(overfill):
    cfg, nodes, pods, quotas, rsv, _, _ = synth.cluster5(600, 160, seed_config=49, rsv_frac=0.5, rsv_gpu=False,
                                                         raw=True)
    pods = {k: v.copy() for k, v in pods.items()}
    rng = np.random.default_rng(49)
    pods["rsv_class"] = np.where(rng.random(len(pods["rsv_class"])) < 0.7,
                                 rng.integers(0, synth.N_RSV_CLASSES, len(pods["rsv_class"])), -1).astype(np.int32)
    pods["flags"] &= ~np.uint32(abi.KG_POD_RSV_REQUIRED)
    kc = cfg.kg_config()
    ref_node, *_ = oracle_lib.OracleState(kc, nodes).ext_replay(pods, quotas, rsv=rsv)
    ok = np.flatnonzero(ref_node >= 0)
    sub, plan = abi.take(pods, ok), ref_node[ok].astype(np.int32)
    if overfill:
        plan[len(plan) // 2:] = plan[0]
    order = grouped(plan)
    return kc, nodes, quotas, rsv, abi.take(sub, np.asarray(order)), plan[order]


def test_oracle_batch_with_reservation_views():
    """The oracle's batch cycle follows Reservation.Reserve: a planned job taken from the oracle replay with views
    (every pod on its replayed node, groups in replay order) commits whole."""
    kc, nodes, quotas, rsv, sub, plan = _rsv_batch_case(False)
    res, stat, *_ = oracle_lib.OracleState(kc, nodes).batch_schedule(sub, plan, quotas, rsv)
    assert (res == abi.KG_BATCH_ASSUMED).all(), stat[res != abi.KG_BATCH_ASSUMED]


@pytest.mark.gpu
@pytest.mark.parametrize("overfill", [False, True])
def test_batch_schedule_with_reservation_views(ctx, overfill):
    """kg_batch_schedule with reservation views (no GPU-holding reservation): each Reserve runs Reservation.Reserve
    on the node's views; results, GPU minors and quota used equal the oracle's, and a failed job restores the views
    (the select after it equals the oracle's on the untouched cluster)."""
    from koordinator_amd import engine
    kc, nodes, quotas, rsv, sub, plan = _rsv_batch_case(overfill)
    snap = engine.Snapshot(ctx, kc, nodes)
    snap.upload_quotas(quotas)
    snap.upload_reservations(rsv)
    pb = engine.PodBatch(ctx, sub)
    res, stat, zone, minors = engine.batch_schedule(snap, pb, plan)
    ost = oracle_lib.OracleState(kc, nodes)
    rres, rstat, rzone, rminors, qu, _qn = ost.batch_schedule(sub, plan, quotas, rsv)
    assert np.array_equal(res, rres) and np.array_equal(stat, rstat)
    assert np.array_equal(zone, rzone) and np.array_equal(minors, rminors)
    assert np.array_equal(snap.read_quotas()[0], qu)
    assert np.array_equal(snap.read_state()["dev_free"], ost.dev_free())
    if overfill:
        assert (res == abi.KG_BATCH_FAILED).sum() >= 1
        keys = engine.eval_select(snap, pb, 1)
        want = oracle_lib.ext_select(kc, nodes, sub, 1, quotas=quotas, rsv=rsv)
        assert np.array_equal(keys, want)
    else:
        assert (res == abi.KG_BATCH_ASSUMED).all()


@pytest.mark.gpu
def test_planner_and_batch_scheduler_end_to_end(ctx):
    """koordinator_amd.batch: FindOneNode plan -> BatchSchedule commit; an infeasible gang -> Unschedulable
    naming its first unplaced pod; a plan the cluster cannot hold -> the reference's example message."""
    from koordinator_amd import engine
    cfg, nodes, pods = synth.small(400, 96, seed=49)
    kc = cfg.kg_config()
    names = [f"node-{i:04d}" for i in range(abi.table_len(nodes))]
    snap = engine.Snapshot(ctx, kc, nodes)
    members = [batch.JobPod("team", f"worker-{j:03d}", uid=f"u{j}") for j in range(48)]
    job = abi.take(pods, np.arange(48))
    planner, sched = batch.ReplayPlanner(snap, names), batch.BatchScheduler(snap, names)
    plan, status, _why = planner.find_one_node(members, job)
    assert status.is_success() and len(plan.pod_to_node_name) == 48
    ref_node, _ = oracle_lib.OracleState(kc, nodes).replay(job)
    assert [plan.pod_to_node_name[m.key] for m in members] == [names[i] for i in ref_node]
    table_by_key = {m.key: (job, j) for j, m in enumerate(members)}
    out = sched.batch_schedule(plan, table_by_key)
    assert out.status.is_success() and len(out.assumed) == 48
    # the committed state equals the oracle's replay of the same job
    o = oracle_lib.OracleState(kc, nodes)
    o.replay(job)
    got, want = gpu_state_cols(snap), oracle_state_cols(o)
    for k in STATE_COLS:
        assert np.array_equal(got[k], want[k]), k
    # a gang with a pod that fits nowhere
    huge = abi.take(pods, np.arange(48, 52))
    huge["req_cpu"][2] = 10 ** 9
    gang = [batch.JobPod("team", f"big-{j}") for j in range(4)]
    plan2, st2, _ = planner.find_one_node(gang, huge)
    assert plan2 is None and st2.code == batch.UNSCHEDULABLE and "big-2" in st2.message
    assert "Insufficient cpu" in st2.message
    # a plan that overfills one node fails and leaves the state as it was
    job3 = abi.take(pods, np.arange(52, 96))
    m3 = [batch.JobPod("team", f"p-{j:02d}", uid=str(j)) for j in range(44)]
    bad = batch.BatchScheduleResult(m3, {m.key: names[5] for m in m3})
    out3 = sched.batch_schedule(bad, {m.key: (job3, j) for j, m in enumerate(m3)})
    assert out3.status.code == batch.UNSCHEDULABLE
    assert out3.status.message.startswith("job failed due to job batch schedule failed, assumed ")
    assert f"@{names[5]} failed due to filter pod team/" in out3.status.message
    # the failing pod's message is set on it and on every later pod of its node (engine.go:212-217)
    failing = [k for k, st in out3.pod_status.items() if "filter pod" in st.message]
    assert len(failing) >= 2 and len({out3.pod_status[k].message for k in failing}) == 1
    got2 = gpu_state_cols(snap)
    for k in STATE_COLS:
        assert np.array_equal(got2[k], got[k]), k
    missing = batch.BatchScheduleResult(m3[:2], {m3[0].key: names[1]})
    assert sched.batch_schedule(missing, {}).status.code == batch.ERROR


def _cpuset_batch_case(overfill, ext):
    """A planned job with cpuset-binding pods: the mixed cluster (cpusets under every NUMA policy), or config 5 with
    reservation views, quotas and cpusets; the plan is the oracle replay's placement (overfill: the second half of the
    job crowded onto one node so that its takes fail)."""
    if ext:
        cfg, nodes, pods, quotas, rsv = synth.cluster5(600, 160, seed_config=97, numa="mix", usage="u01", rsv_gpu=False,
                                                       rsv_frac=0.3)
        pods = {k: v.copy() for k, v in pods.items()}
        nodes, pods = synth.add_cpusets(nodes, pods, 97, bind_frac=0.25)
        kc = cfg.kg_config()
        ref_node, *_ = oracle_lib.OracleState(kc, nodes).ext_replay(pods, quotas, rsv=rsv)
    else:
        cfg, nodes, pods = synth.mixed(500, 200, seed=98)
        quotas = rsv = None
        kc = cfg.kg_config()
        ref_node, _ = oracle_lib.OracleState(kc, nodes).replay(pods)
    ok = np.flatnonzero(ref_node >= 0)
    sub, plan = abi.take(pods, ok), ref_node[ok].astype(np.int32)
    if overfill:
        bind = np.flatnonzero((sub["flags"] & abi.KG_POD_CPU_BIND) != 0)
        plan[bind] = plan[bind[0]]
        plan[len(plan) // 2:] = plan[bind[0]]
    order = grouped(plan)
    return kc, nodes, quotas, rsv, abi.take(sub, np.asarray(order)), plan[order]


@pytest.mark.parametrize("ext", [False, True])
def test_oracle_batch_with_cpuset_pods(ext):
    """The oracle's batch cycle of a replayed plan with cpuset pods commits whole (each take on its planned node)."""
    kc, nodes, quotas, rsv, sub, plan = _cpuset_batch_case(False, ext)
    assert ((sub["flags"] & abi.KG_POD_CPU_BIND) != 0).sum() >= 5
    res, stat, *_ = oracle_lib.OracleState(kc, nodes).batch_schedule(sub, plan, quotas, rsv)
    assert (res == abi.KG_BATCH_ASSUMED).all(), stat[res != abi.KG_BATCH_ASSUMED]


@pytest.mark.gpu
@pytest.mark.parametrize("ext,overfill", [(False, False), (False, True), (True, False), (True, True)])
def test_batch_schedule_with_cpuset_pods(ctx, ext, overfill):
    """kg_batch_schedule with cpuset-binding pods (the cooperative cycle: each pod's CPUs taken by the device
    accumulator on its planned node): results, zones, minors, quota used and the node state (CPU RefCounts, zone
    statuses and pod counts) equal the oracle's; a failed job restores everything."""
    from koordinator_amd import engine
    kc, nodes, quotas, rsv, sub, plan = _cpuset_batch_case(overfill, ext)
    snap = engine.Snapshot(ctx, kc, nodes)
    if ext:
        snap.upload_quotas(quotas)
        snap.upload_reservations(rsv)
    before = snap.read_state()
    pb = engine.PodBatch(ctx, sub)
    res, stat, zone, minors = engine.batch_schedule(snap, pb, plan)
    ost = oracle_lib.OracleState(kc, nodes)
    rres, rstat, rzone, rminors, qu, _qn = ost.batch_schedule(sub, plan, quotas, rsv)
    assert np.array_equal(res, rres) and np.array_equal(stat, rstat)
    assert np.array_equal(zone, rzone) and np.array_equal(minors, rminors)
    got, want = snap.read_state(), ost.table()
    for k in ("req_cpu", "cpuset_alloc_milli", "numa_zone_status", "numa_zone_pods", "cpu_alloc", "zone_cpu_used0",
              "zone_cpu_used1"):
        assert np.array_equal(got[k], want[k]), k
    if ext:
        assert np.array_equal(snap.read_quotas()[0], qu)
    if overfill:
        assert (res == abi.KG_BATCH_FAILED).sum() >= 1
        oracle_lib.assert_state_restored(before, got)
    else:
        assert (res == abi.KG_BATCH_ASSUMED).all()
