"""Config-5 parity of the HIP engine (through the C ABI) with the CPU oracle: DeviceShare GPU fit /
score / Reserve, Reservation restore / filter / nominate / score, ElasticQuota gate / Reserve, on top
of NodeResourcesFit + LoadAware + NodeNUMAResource.

Bar: bit-exact — filter status bits, int64 per-plugin raw scores, weighted totals after NormalizeScore,
selected hosts (deterministic tie-break), replay placements, GPU minors and final device / quota state.
"""
import re

import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, engine, synth

pytestmark = pytest.mark.gpu

FIELDS = ("status", "score_nrf", "score_la", "score_numa", "score_dev", "score_rsv", "total", "numa_zone")


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


def make(ctx, kc, nodes, pods, quotas, rsv):
    snap = engine.Snapshot(ctx, kc, nodes)
    if kc.plugins & abi.KG_PLUGIN_QUOTA:
        snap.upload_quotas(quotas)
    if kc.plugins & abi.KG_PLUGIN_RSV:
        snap.upload_reservations(rsv)
    return snap, engine.PodBatch(ctx, pods)


SUBSETS = {
    "all": abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_LA | abi.KG_PLUGIN_NUMA | abi.KG_PLUGIN_EXT,
    "dev": abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_DEV,
    "rsv": abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_LA | abi.KG_PLUGIN_RSV,
    "quota": abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_QUOTA,
    "dev_quota_numa": abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_LA | abi.KG_PLUGIN_NUMA | abi.KG_PLUGIN_DEV | abi.KG_PLUGIN_QUOTA,
}


@pytest.mark.parametrize("subset", list(SUBSETS))
@pytest.mark.parametrize("seed,n_nodes,n_pods,rsv_frac", [(11, 1200, 192, 0.05), (12, 600, 256, 0.4)])
def test_ext_verify(ctx, subset, seed, n_nodes, n_pods, rsv_frac):
    cfg, nodes, pods, quotas, rsv = synth.cluster5(n_nodes, n_pods, seed_config=seed, rsv_frac=rsv_frac)
    kc = cfg.kg_config()
    kc.plugins = SUBSETS[subset]
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_verify(snap, batch)
    ref = oracle_lib.ext_verify(kc, nodes, pods, quotas if kc.plugins & abi.KG_PLUGIN_QUOTA else None,
                                rsv if kc.plugins & abi.KG_PLUGIN_RSV else None)
    assert_equal(got, ref, subset)
    # the workload exercises every plugin's outcomes
    st = ref.status
    if kc.plugins & abi.KG_PLUGIN_DEV:
        assert (st & abi.KG_ST_DEV_INSUFFICIENT).any() and (ref.score_dev > 0).any()
    if kc.plugins & abi.KG_PLUGIN_RSV:
        assert (ref.score_rsv > 0).any() and (st & abi.KG_ST_RSV_AFFINITY).any()
    if kc.plugins & abi.KG_PLUGIN_QUOTA:
        assert (st & abi.KG_ST_QUOTA).any()
    assert (st == 0).any()


def test_gpu_pods_on_reservation_views(ctx):
    """GPU pods of a reservation class on nodes where reservations hold GPUs: the DeviceShare restore
    (tryAllocateFromReusable over the matched reservations, the base allocation outside them, the nominated
    reservation's table for the Score) on the device equals the oracle over every pair."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(500, 384, seed_config=13, rsv_frac=0.6)
    kc = cfg.kg_config()
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_verify(snap, batch)
    ref = oracle_lib.ext_verify(kc, nodes, pods, quotas, rsv)
    assert_equal(got, ref, "gpu+views")
    st = ref.status
    gpu_cls = (pods["dev_count"] > 0) & (pods["rsv_class"] >= 0)
    assert gpu_cls.sum() >= 10
    assert not (st & abi.KG_ST_UNSUPPORTED).any()
    assert (st[gpu_cls] & abi.KG_ST_DEV_RSV).any()  # required affinity, no matched reservation's GPUs fit
    view_nodes = np.zeros(len(nodes["req_cpu"]), bool)
    for v in rsv.view_list():
        if v.dev_base >= 0:
            view_nodes[v.node] = True
    ok = (st == 0) & gpu_cls[:, None] & view_nodes[None, :]
    assert ok.any() and (ref.score_dev[ok] > 0).any()
    keys = engine.eval_select(snap, batch, 2)
    assert np.array_equal(keys, oracle_lib.ext_select(kc, nodes, pods, 2, 0, quotas, rsv))


@pytest.mark.parametrize("k", [1, 3])
def test_ext_select(ctx, k):
    cfg, nodes, pods, quotas, rsv = synth.cluster5(2500, 300, seed_config=21, rsv_frac=0.2)
    kc = cfg.kg_config()
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_select(snap, batch, k)
    want = oracle_lib.ext_select(kc, nodes, pods, k, 0, quotas, rsv)
    assert np.array_equal(got, want)
    assert (want[:, 0] == 0).any() and (want[:, 0] != 0).any()


@pytest.mark.parametrize("k", [1, 3])
def test_ext_select_guess_rerun(ctx, capfd, monkeypatch, k):
    """One-pass fast-base select (kg_ext.hip k_ext_select / k_ext_fix_rows): each GPU pod's DeviceShare maximum
    over the fast-base records is first taken as its class's best fitting score. Here the nodes with the most
    free GPU (the LeastAllocated maxima) have no CPU left, so the guesses miss and the rows are re-run with the
    real maximum: keys still equal the oracle's."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(1500, 300, seed_config=23, rsv_frac=0.1)
    free = nodes["dev_free"][:, abi.KG_DEV_CORE, :].sum(1)
    top = np.argsort(-free, kind="stable")[:40]
    nodes["req_cpu"][top] = nodes["alloc_cpu"][top]
    nodes["nz_cpu"][top] = np.maximum(nodes["nz_cpu"][top], nodes["alloc_cpu"][top])
    kc = cfg.kg_config()
    monkeypatch.setenv("KG_TRACE_FIX", "1")
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_select(snap, batch, k)
    want = oracle_lib.ext_select(kc, nodes, pods, k, 0, quotas, rsv)
    assert np.array_equal(got, want)
    m = re.search(r"re-ran (\d+) of (\d+) rows", capfd.readouterr().err)
    assert m and int(m.group(1)) > 0, "no row re-run: the test no longer reaches k_ext_fix_rows"
    gpu = pods["dev_count"] > 0
    assert (want[gpu, 0] != 0).any()


def plain_pods(pods):
    """Pods without a GPU request, reservation class or reservation affinity: the select runs them
    through the fast k_select (kg_runtime.cpp ext_select_local split)."""
    cls = pods.get("rsv_class", np.full(len(pods["req_cpu"]), -1))
    return (pods["dev_count"] == 0) & (cls < 0) & ((pods["flags"] & abi.KG_POD_RSV_REQUIRED) == 0)


@pytest.mark.parametrize("subset", list(SUBSETS))
@pytest.mark.parametrize("k", [1, 4])
def test_ext_select_split(ctx, subset, k):
    """Select with the plain / config-5 pod split: both sub-batches scattered back in batch order,
    quota-rejected plain pods without a node, every plugin subset."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(1800, 400, seed_config=71, rsv_frac=0.2)
    kc = cfg.kg_config()
    kc.plugins = SUBSETS[subset]
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_select(snap, batch, k)
    want = oracle_lib.ext_select(kc, nodes, pods, k, 0, quotas if kc.plugins & abi.KG_PLUGIN_QUOTA else None,
                                 rsv if kc.plugins & abi.KG_PLUGIN_RSV else None)
    assert np.array_equal(got, want)
    plain = plain_pods(pods)
    assert plain.any() and (~plain).any()
    if kc.plugins & abi.KG_PLUGIN_QUOTA:
        assert (plain & (want[:, 0] == 0)).any()


def test_ext_select_split_big_values(ctx):
    """Plain pods on nodes outside the fast path's exact domain go through k_merge_big."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(900, 200, seed_config=72, rsv_frac=0.2)
    nodes = {k: v.copy() for k, v in nodes.items()}
    nodes["alloc_mem"][:40] = 1 << 50
    nodes["la_alloc1"][:40] = 1 << 50
    kc = cfg.kg_config()
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    for k in (1, 4):
        got = engine.eval_select(snap, batch, k)
        want = oracle_lib.ext_select(kc, nodes, pods, k, 0, quotas, rsv)
        assert np.array_equal(got, want)
    assert (abi.key_node(want[:, 0][want[:, 0] != 0]) < 40).any()


def test_ext_select_preferred_reservation_wins(ctx):
    """Reservation weight 5000 with the preferred (ordered) reservation node normalised to 100."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(800, 200, seed_config=31, rsv_frac=0.5)
    kc = cfg.kg_config()
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_select(snap, batch, 1)[:, 0]
    want = oracle_lib.ext_select(kc, nodes, pods, 1, 0, quotas, rsv)[:, 0]
    assert np.array_equal(got, want)
    tot = abi.key_total(want)
    assert (tot >= 5000 * 100).any()  # some pods land on their preferred reservation node


def test_ext_replay(ctx):
    cfg, nodes, pods, quotas, rsv = synth.cluster5(1500, 3000, seed_config=41)
    kc = cfg.kg_config()
    kc.plugins &= ~abi.KG_PLUGIN_RSV
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    node, total = engine.replay(snap, batch)
    minors = engine.replay_minors(batch)
    ost = oracle_lib.OracleState(kc, nodes)
    onode, ototal, ominors, oused, onp = ost.ext_replay(pods, quotas)
    assert np.array_equal(node, onode)
    assert np.array_equal(total, ototal)
    assert np.array_equal(minors, ominors)
    state = snap.read_state()
    assert np.array_equal(state["dev_free"], ost.dev_free())
    want = ost.table()
    for k in ("req_cpu", "req_mem", "num_pods", "nz_cpu", "nz_mem"):
        assert np.array_equal(state[k], want[k]), k
    used, _, npu, _ = snap.read_quotas()
    assert np.array_equal(used, oused) and np.array_equal(npu, onp)
    assert (node < 0).any() and (minors != 0).any()


def _without_gpu_inputs(rsv):
    """The same views and tables without the DeviceShare restore inputs of GPU-holding reservations."""
    r = abi.Reservations([], [])
    r.views, r.n_views, r.infos, r.n_infos, r.devs, r.n_devs = rsv.views, rsv.n_views, rsv.infos, rsv.n_infos, rsv.devs, \
        rsv.n_devs
    return r


def test_ext_replay_rejects_gpu_reservations_without_inputs(ctx):
    """Reservations that hold GPUs and no restore inputs: the replay cannot follow their DeviceShare tables
    (KG_UNSUPPORTED); with the inputs it runs (tests/test_rsv_replay.py checks it against the oracle)."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(300, 20, seed_config=42)
    assert rsv.n_gpu > 0
    snap, batch = make(ctx, cfg.kg_config(), nodes, pods, quotas, _without_gpu_inputs(rsv))
    with pytest.raises(engine.Unsupported):
        engine.replay(snap, batch)
    snap.upload_reservations(rsv)
    engine.replay(snap, batch)


def test_ext_assume_forget_roundtrip(ctx):
    cfg, nodes, pods, quotas, rsv = synth.cluster5(400, 64, seed_config=43)
    kc = cfg.kg_config()
    kc.plugins &= ~abi.KG_PLUGIN_RSV
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    before = snap.read_state()
    qb = snap.read_quotas()
    keys = engine.eval_select(snap, batch, 1)[:, 0]
    gpu = np.nonzero((pods["dev_count"] > 0) & (keys != 0))[0][:4]
    assert len(gpu) > 0
    done = []
    for j in gpu:
        i = int(abi.key_node(keys[j]))
        zone, minors = engine.assume_ext(snap, batch, int(j), i)
        assert bin(minors).count("1") == int(pods["dev_count"][j])
        done.append((int(j), i, zone, minors))
    mid = snap.read_state()
    assert not np.array_equal(mid["dev_free"], before["dev_free"])
    for j, i, zone, minors in reversed(done):
        engine.forget_ext(snap, batch, j, i, zone, minors)
    after = snap.read_state()
    for k in before:
        assert np.array_equal(before[k], after[k]), k
    qa = snap.read_quotas()
    for a, b in zip(qb, qa):
        assert np.array_equal(a, b)


def test_config5_full_size_sampled(ctx):
    """Config 5 at 100k nodes x 10k pods: select on the device, a pod sample re-checked on the oracle."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(100_000, 10_000)
    kc = cfg.kg_config()
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    keys = engine.eval_select(snap, batch, 1)[:, 0]
    idx = np.random.default_rng(5).choice(10_000, 24, replace=False)
    sample = abi.take(pods, idx)
    want = oracle_lib.ext_select(kc, nodes, sample, 1, 0, quotas, rsv)[:, 0]
    assert np.array_equal(keys[idx], want)
    assert (keys != 0).mean() > 0.5


def test_config5_full_size_verify_sampled(ctx):
    """Per-plugin parity at full size on the round-4 config-5 workload (synth.config5(): 100k nodes with 20 %
    SingleNUMANode, U(0, 1) GPU minor usage, reservations that hold GPUs): status bits, raw scores, totals and NUMA
    zones of a pod sample (GPU pods with and without a reservation class, class pods, plain pods) on every node."""
    cfg, nodes, pods, quotas, rsv = synth.config5()
    kc = cfg.kg_config()
    rng = np.random.default_rng(9)
    gpu, cls = pods["dev_count"] > 0, pods["rsv_class"] >= 0
    groups = [np.flatnonzero(gpu & cls), np.flatnonzero(gpu & ~cls), np.flatnonzero(~gpu & cls), np.flatnonzero(~gpu & ~cls)]
    idx = np.concatenate([rng.choice(g, 4, replace=False) for g in groups])
    sample = abi.take(pods, idx)
    snap, batch = make(ctx, kc, nodes, sample, quotas, rsv)
    got = engine.eval_verify(snap, batch)
    ref = oracle_lib.ext_verify(kc, nodes, sample, quotas, rsv)
    assert_equal(got, ref, "config5 full size")
    assert (ref.status == 0).any() and (ref.score_dev > 0).any() and (ref.score_rsv > 0).any()


@pytest.mark.parametrize("k", [1, 3])
def test_ext_shard_select_single_rank(ctx, k):
    """kg_shard_select's config-5 path (stats pass, RCCL all-reduce of the NormalizeScore inputs,
    select pass, all-gather of the per-shard top-k, merge) with one rank equals the global selection."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(1500, 256, seed_config=61, rsv_frac=0.3)
    kc = cfg.kg_config()
    sctx = engine.Context(0)
    try:
        sctx.shard_init(engine.shard_unique_id(), 0, 1)
        snap, batch = make(sctx, kc, nodes, pods, quotas, rsv)
        got = engine.shard_select(snap, batch, k)
        again = engine.result_keys(batch, k)
        status = engine.result_status(batch)
    finally:
        sctx.close()
    want = oracle_lib.ext_select(kc, nodes, pods, k, 0, quotas, rsv)
    assert np.array_equal(got, want)
    assert np.array_equal(again, want)
    ref = oracle_lib.ext_verify(kc, nodes, pods, quotas, rsv)
    assert np.array_equal(status, np.bitwise_or.reduce(ref.status & (abi.KG_ST_UNSUPPORTED | abi.KG_ST_QUOTA), axis=1))


@pytest.mark.parametrize("split", ["1", "0"])
def test_ext_result_status(ctx, monkeypatch, split):
    """kg_result_status on config 5 with cpuset-binding pods, some on SingleNUMANode nodes with a CPU topology (the
    cpuset inside the NUMA hints, on the device since ABI 9): quota-rejected pods are flagged KG_ST_QUOTA, no pod
    KG_ST_UNSUPPORTED — the OR of the oracle verify rows' bits (a cpuset-binding pod on a node without CPU topology
    fails its Filter; GPU pods on NUMA-policy nodes are on the device path too)."""
    monkeypatch.setenv("KG_EXT_SPLIT", split)
    cfg, nodes, pods, quotas, rsv = synth.cluster5(1200, 400, seed_config=73, rsv_frac=0.2)
    nodes = {k: v.copy() for k, v in nodes.items()}
    pods = {k: v.copy() for k, v in pods.items()}
    n = len(nodes["alloc_cpu"])
    nodes["numa_policy"][::50] = abi.KG_NUMA_SINGLE_NODE
    nodes["numa_zones"][::50] = np.maximum(nodes["numa_zones"][::50], 1)
    ti = np.full(n, -1, np.int32)
    ti[::25] = 0
    nodes["cpu_topo"] = ti
    nodes["cpu_topos"] = abi.cpu_topos_array([abi.cpu_topo_for_test(2, 1, 16, 2)])
    nodes["cpu_alloc"] = np.zeros((n, 2 * abi.KG_MAX_CPUS), np.uint8)
    nodes["cpu_max_ref"] = np.ones(n, np.uint8)
    pods["flags"][1::11] |= abi.KG_POD_CPU_BIND
    kc = cfg.kg_config()
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_select(snap, batch, 1)
    want = oracle_lib.ext_select(kc, nodes, pods, 1, 0, quotas, rsv)
    assert np.array_equal(got, want)
    ref = oracle_lib.ext_verify(kc, nodes, pods, quotas, rsv)
    vg = engine.eval_verify(snap, batch)
    badp = np.argwhere(vg.status != ref.status)
    assert not len(badp), [(int(j), int(i), hex(vg.status[j, i]), hex(ref.status[j, i])) for j, i in badp[:8]]
    engine.eval_select(snap, batch, 1)
    wstat = np.bitwise_or.reduce(ref.status & (abi.KG_ST_UNSUPPORTED | abi.KG_ST_QUOTA), axis=1)
    gstat = engine.result_status(batch)
    bad = np.flatnonzero(gstat != wstat)
    assert not len(bad), [(int(j), hex(gstat[j]), hex(wstat[j]), hex(pods["flags"][j]),
                           [(int(i), hex(ref.status[j, i])) for i in np.flatnonzero(ref.status[j] & abi.KG_ST_UNSUPPORTED)[:4]])
                          for j in bad[:6]]
    assert not (wstat & abi.KG_ST_UNSUPPORTED).any() and (wstat & abi.KG_ST_QUOTA).any() and (wstat == 0).any()
    # the cpuset-under-NUMA pairs were evaluated (some admitted with a zone)
    sel = ((pods["flags"] & abi.KG_POD_CPU_BIND) != 0)[:, None] & ((nodes["numa_policy"] != 0) & (ti >= 0))[None, :]
    assert (sel & (ref.status == 0)).any()


def _views_after_plain_pod(rsv, node, pods, j):
    """The restore of `node` after a pod that matches none of its reservations (and binds no GPU) lands there: the
    true NodeInfo and the default columns grow by the pod's requests, so every view of the node does too
    (transformer.go:740-811: view = default + the matched reservations' corrections). Returns (full, delta): the
    whole reservation set with those views shifted, and the node's views alone for kg_snapshot_update_views."""
    import ctypes as C
    def shifted(v):
        w = abi.KgRsvView()
        C.pointer(w)[0] = v
        for k, col in enumerate(("req_cpu", "req_mem", "req_eph", "sc_req0", "sc_req1")):
            w.req[k] += int(pods[col][j])
            w.pod_requested[k] += int(pods[col][j])
        w.nz_cpu += int(pods["nz_cpu"][j])
        w.nz_mem += int(pods["nz_mem"][j])
        w.num_pods += 1
        return w
    full = abi.Reservations([], [])
    full.views = (abi.KgRsvView * max(1, rsv.n_views))()
    mine = []
    for x in range(rsv.n_views):
        v = rsv.views[x]
        full.views[x] = shifted(v) if v.node == node else v
        if v.node == node:
            mine.append(full.views[x])
    full.n_views = rsv.n_views
    full.infos, full.n_infos, full.devs, full.n_devs = rsv.infos, rsv.n_infos, rsv.devs, rsv.n_devs
    delta = abi.Reservations([], [])
    delta.views = (abi.KgRsvView * max(1, len(mine)))(*mine)
    delta.n_views = len(mine)
    delta.infos, delta.n_infos, delta.devs, delta.n_devs = rsv.infos, rsv.n_infos, rsv.devs, rsv.n_devs
    return full, delta


def test_view_update_after_assume_on_view_node(ctx):
    """A Reserve on a node holding reservation views makes its views stale: selects refuse (KG_UNSUPPORTED) until
    kg_snapshot_update_views replaces that node's views with the recomputed restore; the next select then equals
    the oracle's on the updated state (the other nodes' views untouched)."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(600, 64, seed_config=74, rsv_frac=0.5)
    pods = {k: v.copy() for k, v in pods.items()}
    kc = cfg.kg_config()
    ref = oracle_lib.ext_verify(kc, nodes, pods, quotas, rsv)
    view_nodes = sorted({int(v.node) for v in rsv.view_list()})
    plain = [j for j in range(64) if pods["rsv_class"][j] < 0 and pods["dev_count"][j] == 0]
    pick = [(j, i) for j in plain for i in view_nodes if ref.status[j, i] == 0]
    assert pick
    j, i = pick[0]
    pods["quota"][j] = -1  # no ElasticQuota Reserve to follow in the oracle table
    ref = oracle_lib.ext_verify(kc, nodes, pods, quotas, rsv)
    assert ref.status[j, i] == 0
    # without the GPU restore inputs the Reserve cannot follow the node's GPU-holding reservations: its views go stale
    snap, batch = make(ctx, kc, nodes, pods, quotas, _without_gpu_inputs(rsv))
    engine.eval_select(snap, batch, 1)
    engine.assume_ext(snap, batch, j, i)
    with pytest.raises(engine.Unsupported):
        engine.eval_select(snap, batch, 1)
    full, delta = _views_after_plain_pod(rsv, i, pods, j)
    snap.update_views([i], delta)
    st = oracle_lib.OracleState(kc, nodes)
    st.assume(i, pods, j)
    after = dict(nodes)
    after.update(st.table())
    for k in (1, 3):
        got = engine.eval_select(snap, batch, k)
        assert np.array_equal(got, oracle_lib.ext_select(kc, after, pods, k, 0, quotas, full)), k
    # a listed node without views loses them; the rest of the snapshot keeps its own
    snap.update_views([i], abi.Reservations([], []))
    engine.eval_select(snap, batch, 1)


def test_pod_batch_without_config5_columns(ctx):
    """A pod batch uploaded without the config-5 columns (no GPU request, quota or reservation class) onto
    a batch object that held config-5 pods: kg_pods_upload sets their defaults on the device (memsets),
    so nothing of the previous upload survives."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(1500, 300, seed_config=23, rsv_frac=0.2)
    kc = cfg.kg_config()
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    engine.eval_select(snap, batch, 1)
    plain = {k: v for k, v in pods.items() if k not in ("dev_req", "dev_count", "dev_keys", "quota", "quota_keys",
                                                        "rsv_class")}
    batch.upload(plain)
    for k in (1, 3):
        got = engine.eval_select(snap, batch, k)
        assert np.array_equal(got, oracle_lib.ext_select(kc, nodes, plain, k, 0, quotas, rsv)), k
    assert not (engine.result_status(batch) & abi.KG_ST_QUOTA).any()


@pytest.mark.parametrize("numa", ["single", "mix"])
@pytest.mark.parametrize("mode", ["stored", "capped", "off"])
@pytest.mark.parametrize("k", [1, 3])
def test_ext_select_stored_pairs(ctx, monkeypatch, numa, mode, k):
    """The fast-base select's general records through its two kernels (k_ext_select_xs: the pairs the statistics pass
    stored; k_ext_select_sp: the special list's pairs of class pods, the lanes flagged because a pair was not stored,
    every pair without the store) equal the oracle's selection. "capped" stores 40 positions per lane (KG_XPAIRS_T), so
    class pods with more views are flagged; "off" stores nothing (KG_NO_XPAIRS); numa "mix" puts Restricted (F_BIG)
    records in the special list."""
    if mode == "capped":
        monkeypatch.setenv("KG_XPAIRS_T", "40")
    elif mode == "off":
        monkeypatch.setenv("KG_NO_XPAIRS", "1")
    cfg, nodes, pods, quotas, rsv = synth.cluster5(2000, 300, seed_config=67, rsv_frac=0.3, numa=numa, usage="u01")
    kc = cfg.kg_config()
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_select(snap, batch, k)
    want = oracle_lib.ext_select(kc, nodes, pods, k, 0, quotas, rsv)
    assert np.array_equal(got, want), np.argwhere(got != want)[:8].tolist()
    ref = oracle_lib.ext_verify(kc, nodes, pods, quotas, rsv)
    wstat = np.bitwise_or.reduce(ref.status & (abi.KG_ST_UNSUPPORTED | abi.KG_ST_QUOTA), axis=1)
    assert np.array_equal(engine.result_status(batch), wstat)


def test_ext_select_c1_beside_rerun(ctx, capfd, monkeypatch):
    """Top-1 with SingleNUMANode records: k_ext_select_c1 runs beside the one-pass select with the guessed maxima and
    re-runs on the rows k_ext_fix_rows lists (the first 256 over short chunks in one pod block, the rest in a second
    launch). The nodes with the most free GPU have no CPU left, so more than 256 rows are re-run; keys still equal the
    oracle's."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(1500, 2600, seed_config=29, rsv_frac=0.1, numa="single")
    free = nodes["dev_free"][:, abi.KG_DEV_CORE, :].sum(1)
    top = np.argsort(-free, kind="stable")[:60]
    nodes["req_cpu"][top] = nodes["alloc_cpu"][top]
    nodes["nz_cpu"][top] = np.maximum(nodes["nz_cpu"][top], nodes["alloc_cpu"][top])
    kc = cfg.kg_config()
    monkeypatch.setenv("KG_TRACE_FIX", "1")
    monkeypatch.setenv("KG_TRACE_SP", "1")
    snap, batch = make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_select(snap, batch, 1)
    want = oracle_lib.ext_select(kc, nodes, pods, 1, 0, quotas, rsv)
    assert np.array_equal(got, want), np.argwhere(got != want)[:8].tolist()
    err = capfd.readouterr().err
    m = re.search(r"re-ran (\d+) of (\d+) rows", err)
    c = re.search(r"class-1 (\d+)", err)
    assert m and int(m.group(1)) > 256, err[-400:]
    assert c and int(c.group(1)) > 0, "no class-1 list: the test no longer reaches the class-1 kernels"
