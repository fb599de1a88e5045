"""f3: DeviceShare as a NUMA hint provider (deviceshare/topology_hint.go:40-290) in the topology manager
(frameworkext/topologymanager/manager.go:65-154, policy*.go).

- The oracle's hint provider against the known answers of topology_hint_test.go (tests/golden/gpu_numa_kat.json).
- The device (through the C ABI) against the oracle, bit for bit, on config-5 clusters whose nodes carry every NUMA
  policy (synth.cluster5(numa="mix")): verify matrices (status bits, raw scores, totals, the Reserve's zone code),
  top-k selects, and the replay whose Reserve allocates GPU minors inside the stored NUMA affinity.
"""
import json
import os

import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, decode, synth
from koordinator_amd.config import config5_profile

HERE = os.path.dirname(os.path.abspath(__file__))


def _kat():
    with open(os.path.join(HERE, "golden", "gpu_numa_kat.json")) as f:
        return json.load(f)


def _node(K, assigned=()):
    """One node with the fakeDeviceCR GPUs and two NUMA zones (64 cores, 256Gi each), policy SingleNUMANode."""
    dv = K["device"]
    t = abi.empty_nodes(1)
    t["alloc_cpu"][:] = 128000
    t["alloc_mem"][:] = 512 << 30
    t["alloc_pods"][:] = 110
    t["numa_zones"][:] = 2
    t["numa_policy"][:] = abi.KG_NUMA_SINGLE_NODE
    for z in range(2):
        t[f"zone_cpu{z}"][:] = 64000
        t[f"zone_mem{z}"][:] = 256 << 30
    t["dev_minors"][0] = 8
    for m in range(8):
        t["dev_total"][0, :, m] = [dv["core"], dv["ratio"], dv["memory"]]
        t["dev_free"][0, :, m] = [dv["core"], dv["ratio"], dv["memory"]]
    for m, core, ratio in assigned:
        t["dev_free"][0, abi.KG_DEV_CORE, m] -= core
        t["dev_free"][0, abi.KG_DEV_RATIO, m] -= ratio
    infos = [{"minor": m, "topology": {"nodeID": q, "pcieID": pc}} for m, (q, pc) in enumerate(zip(dv["numa"], dv["pcie"]))]
    topo, tree = decode.gpu_topology(infos)
    t["dev_topo"] = np.array([topo], np.uint64)
    t["dev_part"] = np.array([abi.KG_GPU_TREE if tree else 0], np.uint32)
    t["dev_numa"] = np.array([decode.gpu_numa(infos)], np.uint32)
    return t


def _pod(req):
    p = abi.empty_pods(1)
    p["req_cpu"][:] = 4000
    p["req_mem"][:] = 8 << 30
    p["nz_cpu"][:] = 4000
    p["nz_mem"][:] = 8 << 30
    p["flags"][:] |= abi.KG_POD_HAS_CPU | abi.KG_POD_HAS_MEM
    vec, keys, cnt, shared = decode.gpu_requirements(req)
    p["dev_req"][0] = vec
    p["dev_keys"][0] = keys
    p["dev_count"][0] = cnt
    p["dev_flags"] = np.array([decode.gpu_pod_flags({"metadata": {"annotations": {}}}, shared)[0]], np.uint32)
    return p


def _cfg():
    kc = config5_profile().kg_config()
    kc.plugins = abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_NUMA | abi.KG_PLUGIN_DEV
    return kc


def _ids(mask):
    return [q for q in range(8) if (mask >> q) & 1]


K = _kat()


@pytest.mark.parametrize("c", K["hints"], ids=[f'{x["line"]}-{x["name"][:40]}' for x in K["hints"]])
def test_gpu_numa_hints_kat(c):
    """TestPlugin_GetPodTopologyHints (topology_hint_test.go:41-270), GPU lists."""
    nodes = _node(K, c["assigned"])
    pods = _pod({"koordinator.sh/gpu-core": c["gpu_core"], "koordinator.sh/gpu-memory-ratio": c["gpu_ratio"]})
    kind, got = oracle_lib.gpu_numa_hints(_cfg(), nodes, pods)
    if c["result"] == "fail":
        assert kind == "fail", got
        return
    assert kind == "hints"
    assert [[_ids(m), p, s] for m, p, s in got] == c["want"]


@pytest.mark.parametrize("c", K["allocate"], ids=[f'{x["line"]}-{x["name"][:40]}' for x in K["allocate"]])
def test_gpu_numa_allocate_kat(c):
    """TestPlugin_Allocate (topology_hint_test.go:272-419), GPU part: DeviceShare's Allocate under the affinity."""
    nodes = _node(K)
    pods = _pod({"koordinator.sh/gpu-core": c["gpu_core"], "koordinator.sh/gpu-memory": c["gpu_mem"]})
    numa = sum(1 << q for q in c["affinity"])
    code, minors = oracle_lib.gpu_alloc_numa(_cfg(), nodes, pods, numa)
    assert (code != 0) == c["error"]
    if not c["error"]:  # the minors lie inside the affinity's NUMA nodes
        assert minors and all(K["device"]["numa"][m] in c["affinity"] for m in _ids(minors))


def test_gpu_numa_merge_oracle():
    """The merge with DeviceShare's list on the KAT node: a 4-GPU pod with minor 0 taken fits only NUMA node 1, so
    SingleNUMANode admits it there (zone 1) and DeviceShare's Filter passes; a 5-GPU pod has no single-node hint
    (ErrNUMAHintCannotAligned); Restricted admits it over both nodes (zone 0x43); a 9-GPU pod fails in the
    provider ("Insufficient NUMA Scoped Devices")."""
    nodes = _node(K, [[0, 100, 100]])
    kc = _cfg()

    def run(n_gpus, policy):
        nodes["numa_policy"][:] = policy
        pods = _pod({"koordinator.sh/gpu-core": 100 * n_gpus, "koordinator.sh/gpu-memory-ratio": 100 * n_gpus})
        v = oracle_lib.ext_verify(kc, nodes, pods)
        return int(v.status[0, 0]), int(v.numa_zone[0, 0])

    assert run(4, abi.KG_NUMA_SINGLE_NODE) == (0, 1)
    st, _ = run(5, abi.KG_NUMA_SINGLE_NODE)
    assert st & abi.KG_ST_NUMA_ALIGN
    assert run(5, abi.KG_NUMA_RESTRICTED) == (0, 0x43)
    st, _ = run(9, abi.KG_NUMA_RESTRICTED)
    assert abi.dev_code(st) == abi.KG_DEV_CODE_NUMA_SCOPED


def test_cluster5_numa_mix_oracle():
    """The oracle over a mixed-policy config-5 cluster with reservations: no GPU pair leaves the device path (on
    reservation views too), GPU pods are admitted under NUMA affinities and fail on the provider's reasons."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(600, 160, seed_config=31, rsv_frac=0.3, numa="mix")
    kc = cfg.kg_config()
    v = oracle_lib.ext_verify(kc, nodes, pods, quotas, rsv)
    gpu = pods["dev_count"] > 0
    pol = nodes["numa_policy"] != abi.KG_NUMA_NONE
    st = v.status
    cpu_bind = (pods["flags"] & abi.KG_POD_CPU_BIND) != 0
    sel = gpu[:, None] & pol[None, :] & ~cpu_bind[:, None]
    assert sel.sum() > 1000
    assert not (st[sel] & abi.KG_ST_UNSUPPORTED).any()
    ok = sel & (st == 0)
    assert ok.any() and (v.numa_zone[ok] >= 0).any()
    codes = np.vectorize(abi.dev_code)(st[sel])
    assert (codes == abi.KG_DEV_CODE_NUMA_SCOPED).any()
    assert not (st & abi.KG_ST_UNSUPPORTED).any()


def test_config5_workload_stays_on_device():
    """BASELINE config 5 (synth.config5: 20% SingleNUMANode nodes, U(0, 1) GPU usage), a pod sample on the whole
    cluster: no pair needs the host path."""
    cfg, nodes, pods, quotas, rsv = synth.config5(20_000, 2_000)
    kc = cfg.kg_config()
    sub = abi.take(pods, np.arange(0, 2_000, 25))
    v = oracle_lib.ext_verify(kc, nodes, sub, quotas, rsv)
    assert not (v.status & abi.KG_ST_UNSUPPORTED).any()
    single = nodes["numa_policy"] == abi.KG_NUMA_SINGLE_NODE
    gpu = sub["dev_count"] > 0
    assert ((v.status == 0) & gpu[:, None] & single[None, :]).any()


def test_oracle_replay_matches_verify_numa_mix():
    """The oracle's mutable state keeps every static GPU column (dev_numa included): pod k of its replay lands on the
    argmax of the verify row computed on the state after pods < k."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(700, 600, seed_config=34, rsv_frac=0.0, numa="mix")
    kc = cfg.kg_config()
    kc.plugins &= ~(abi.KG_PLUGIN_RSV | abi.KG_PLUGIN_QUOTA)
    gpu_numa = np.flatnonzero(pods["dev_count"] > 0)[:6]
    for k in gpu_numa:
        st = oracle_lib.OracleState(kc, nodes)
        rnode, _, _, _, _ = st.ext_replay(abi.take(pods, np.arange(k + 1)), quotas)
        # state after pods < k: replay them again on a fresh state
        st2 = oracle_lib.OracleState(kc, nodes)
        if k:
            st2.ext_replay(abi.take(pods, np.arange(k)), quotas)
        t = dict(nodes)
        t.update(st2.table())
        t["dev_free"] = st2.dev_free()
        v = oracle_lib.ext_verify(kc, t, abi.take(pods, np.array([k])), quotas, None)
        tot = np.where(v.status[0] == 0, v.total[0], -1)
        want = int(np.argmax(tot)) if tot.max() >= 0 else -1
        if want >= 0 and 0x20 <= int(v.numa_zone[0, want]) < 0x40:
            want = -1  # the winner's Reserve fails
        assert rnode[k] == want, (k, rnode[k], want)


# ---- device parity ---------------------------------------------------------------------------------------------

FIELDS = ("status", "score_nrf", "score_la", "score_numa", "score_dev", "score_rsv", "total", "numa_zone")


@pytest.fixture(scope="module")
def ctx():
    from koordinator_amd import engine
    c = engine.Context(0)
    yield c
    c.close()


def _assert_equal(got, ref, what):
    for name in FIELDS:
        a, b = getattr(got, name), getattr(ref, name)
        if not np.array_equal(a, b):
            bad = np.argwhere(a != b)
            j, i = bad[0]
            raise AssertionError(f"{what}: {name} differs at {len(bad)} pairs, first pod {j} node {i}: "
                                 f"gpu={a[j, i]} oracle={b[j, i]}")


def _make(ctx, kc, nodes, pods, quotas, rsv):
    from koordinator_amd import engine
    snap = engine.Snapshot(ctx, kc, nodes)
    if kc.plugins & abi.KG_PLUGIN_QUOTA:
        snap.upload_quotas(quotas)
    if kc.plugins & abi.KG_PLUGIN_RSV:
        snap.upload_reservations(rsv)
    return snap, engine.PodBatch(ctx, pods)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,rsv_frac", [(31, 0.0), (32, 0.3)])
def test_gpu_numa_verify_device(ctx, seed, rsv_frac):
    from koordinator_amd import engine
    cfg, nodes, pods, quotas, rsv = synth.cluster5(900, 192, seed_config=seed, rsv_frac=rsv_frac, numa="mix")
    kc = cfg.kg_config()
    snap, batch = _make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_verify(snap, batch)
    ref = oracle_lib.ext_verify(kc, nodes, pods, quotas, rsv)
    _assert_equal(got, ref, f"numa mix seed {seed}")
    gpu = pods["dev_count"] > 0
    ok = gpu[:, None] & (nodes["numa_policy"] != abi.KG_NUMA_NONE)[None, :] & (ref.status == 0)
    assert ok.any()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 3])
def test_gpu_numa_select_device(ctx, k):
    from koordinator_amd import engine
    cfg, nodes, pods, quotas, rsv = synth.cluster5(2500, 256, seed_config=33, rsv_frac=0.1, numa="mix")
    kc = cfg.kg_config()
    snap, batch = _make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_select(snap, batch, k)
    assert np.array_equal(got, oracle_lib.ext_select(kc, nodes, pods, k, 0, quotas, rsv))


@pytest.mark.gpu
@pytest.mark.parametrize("k,gz", [(1, True), (3, True), (1, False)])
def test_gpu_numa_single_fast_base(ctx, monkeypatch, k, gz):
    """Config 5's shape (synth.config5: SingleNUMANode nodes, U(0, 1) GPU usage) on the fast-base select: the
    SingleNUMANode records take DeviceShare's hints from the per-class table (k_gpu_zone_sum + eval_c1), or with
    KG_NO_GZ the general path; both equal the oracle."""
    from koordinator_amd import engine
    if not gz:
        monkeypatch.setenv("KG_NO_GZ", "1")
    cfg, nodes, pods, quotas, rsv = synth.cluster5(3000, 512, seed_config=35, rsv_frac=0.1, numa="single", usage="u01")
    kc = cfg.kg_config()
    assert (nodes["numa_policy"] == abi.KG_NUMA_SINGLE_NODE).sum() > 300
    snap, batch = _make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_select(snap, batch, k)
    assert np.array_equal(got, oracle_lib.ext_select(kc, nodes, pods, k, 0, quotas, rsv))


@pytest.mark.gpu
def test_gpu_numa_replay_device(ctx):
    """One pod per cycle: the winner's Reserve allocates its GPUs inside the stored NUMA affinity (BestEffort nodes
    included, whose Reserve can fail on DeviceShare's hints); nodes, minors, reasons and quota state as the oracle."""
    from koordinator_amd import engine
    cfg, nodes, pods, quotas, rsv = synth.cluster5(700, 600, seed_config=34, rsv_frac=0.0, numa="mix")
    kc = cfg.kg_config()
    kc.plugins &= ~abi.KG_PLUGIN_RSV
    snap, batch = _make(ctx, kc, nodes, pods, quotas, rsv)
    node, total, reason = engine.replay(snap, batch, reasons=True)
    minors = engine.replay_minors(batch)
    st = oracle_lib.OracleState(kc, nodes)
    rnode, rtotal, rminors, qu, qnp, rreason = st.ext_replay(pods, quotas, reasons=True)
    assert np.array_equal(node, rnode)
    assert np.array_equal(total, rtotal)
    assert np.array_equal(minors, rminors)
    assert np.array_equal(reason, rreason)
    placed = node >= 0
    gpu_numa = placed & (pods["dev_count"] > 0) & (nodes["numa_policy"][np.maximum(node, 0)] != abi.KG_NUMA_NONE)
    assert gpu_numa.sum() >= 10
