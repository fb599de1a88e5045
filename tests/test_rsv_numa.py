"""Reservations holding NUMA / cpuset allocations (kg_node_columns.rsv_numa).

NodeNUMAResource's RestoreReservation (nodenumaresource/reservation.go:188-262) gives a matched reservation's reserved
CPUs and NUMA resources back to its owners and returns the unmatched reservations' double-counted owner usage; it is
read by the hints (resource_manager.go:131-160), tryAllocateFromReusable / tryAllocateFromNode (plugin.go:428-439,
807-851) and the Reserve. The engine does not restate it: on a node marked rsv_numa every pair where the plugin reads
it (the pod binds CPUs there, or the merged NUMA policy is not None) is KG_ST_UNSUPPORTED after the checks that precede
it (policy conflicts, filterAmplifiedCPUs, the CPU topology and bind-policy checks), and the sequential calls refuse.
Pairs the restore cannot affect (policy None, no CPU binding) are evaluated as before.

- CPU: the oracle's statuses on a marked cluster equal the unmarked ones except exactly the affected pairs; the host
  cache marks a node whose reservation carries a resource-status annotation and unmarks it on delete.
- GPU: the device verify matrix and select keys / outcome flags equal the oracle's on the marked cluster; kg_replay and
  kg_reserve refuse the affected pods, kg_reserve accepts the others."""
import copy
import json

import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, synth


def _marked(n_nodes=240, n_pods=160, seed=31):
    cfg, nodes, pods = synth.mixed(n_nodes, n_pods, seed=seed)
    rng = np.random.default_rng(seed)
    marked = dict(nodes)
    marked["rsv_numa"] = (rng.random(n_nodes) < 0.3).astype(np.uint8)
    return cfg, nodes, marked, pods


def _affected(nodes, pods):
    """(pod, node) pairs whose NodeNUMAResource reads the restore: marked node, the pod not skipped, and it binds CPUs
    there or the merged NUMA policy is not None (conflicting policies fail before)."""
    P, N = abi.table_len(pods), abi.table_len(nodes)
    f = pods["flags"][:, None]
    skip = (f & abi.KG_POD_NUMA_SKIP) != 0
    pod_pol = pods["numa_policy"][:, None]
    node_pol = nodes["numa_policy"][None, :]
    pol = np.where(pod_pol != abi.KG_NUMA_NONE, pod_pol, node_pol)
    has_topo = (nodes["cpu_topo"] >= 0)[None, :] if "cpu_topo" in nodes else np.zeros((1, N), bool)
    node_bind = (nodes["cpu_bind_policy"] != 0)[None, :] if "cpu_bind_policy" in nodes else np.zeros((1, N), bool)
    bind = ((f & abi.KG_POD_CPU_BIND) != 0) | (node_bind & (pods["req_cpu"][:, None] != 0))
    return (nodes["rsv_numa"][None, :] != 0) & ~skip & ((pol != abi.KG_NUMA_NONE) | (bind & has_topo))


def test_oracle_marks_exactly_the_affected_pairs():
    cfg, nodes, marked, pods = _marked()
    kc = cfg.kg_config()
    a = oracle_lib.eval_verify(kc, nodes, pods)
    b = oracle_lib.eval_verify(kc, marked, pods)
    unsup = (b.status & abi.KG_ST_UNSUPPORTED) != 0
    aff = _affected(marked, pods)
    # every unsupported pair is affected; an affected pair is unsupported unless a check before the restore decided it
    assert not (unsup & ~aff).any()
    decided = (a.status & (abi.KG_ST_NUMA_CONFLICT | abi.KG_ST_NUMA_AMP_CPU | abi.KG_ST_NUMA_CPU_TOPO |
                           abi.KG_ST_NUMA_CPU_BIND)) != 0
    assert (unsup | decided | ~aff).all()
    assert np.array_equal(a.status[~aff], b.status[~aff]) and np.array_equal(a.total[~aff], b.total[~aff])
    assert unsup.sum() > 50 and (~aff).sum() > 1000


def _annotated_reservation(node, cpus):
    return {"metadata": {"name": "r1", "uid": "u-r1", "annotations": {
                "scheduling.koordinator.sh/resource-status": json.dumps({"cpuset": cpus})}},
            "spec": {"owners": [{"object": {"name": "p"}}], "template": {"spec": {"containers": [
                {"resources": {"requests": {"cpu": "2"}}}]}}},
            "status": {"phase": "Available", "nodeName": node, "allocatable": {"cpu": "2"}}}


def test_host_cache_marks_nodes_with_numa_reservations():
    import test_cluster as tc
    w = tc.World(tc.world_cfg(), 6, 4)
    st = w.state
    assert int(st.table()["rsv_numa"].sum()) == 0
    r = _annotated_reservation("node-2", "0-1")
    st.on_reservation(copy.deepcopy(r))
    t = st.table()
    assert list(np.nonzero(t["rsv_numa"])[0]) == [2]
    plain = copy.deepcopy(r)
    plain["metadata"]["annotations"] = {}
    plain["metadata"]["uid"] = "u-r2"
    st.on_reservation(plain)  # a reservation without a resource status marks nothing
    assert list(np.nonzero(st.table()["rsv_numa"])[0]) == [2]
    st.on_reservation_delete(copy.deepcopy(r))
    assert int(st.table()["rsv_numa"].sum()) == 0


@pytest.mark.gpu
def test_device_marks_the_same_pairs_and_sequential_calls_refuse():
    from koordinator_amd import engine
    cfg, nodes, marked, pods = _marked()
    kc = cfg.kg_config()
    ctx = engine.Context(0)
    try:
        snap = engine.Snapshot(ctx, kc, marked)
        batch = engine.PodBatch(ctx, pods)
        got = engine.eval_verify(snap, batch)
        want = oracle_lib.eval_verify(kc, marked, pods)
        for name in ("status", "score_nrf", "score_la", "score_numa", "total", "numa_zone"):
            assert np.array_equal(getattr(got, name), getattr(want, name)), name
        keys = engine.eval_select(snap, batch, 1)
        assert np.array_equal(keys, oracle_lib.select(kc, marked, pods, 1))
        # a pod is flagged when an unsupported pair could change its selection: the select may skip a pair whose best
        # possible total (NodeResourcesFit and LoadAware scores + the NUMA weight x 100: the restore changes only the
        # NUMA part) cannot beat the pod's key (k_big_sel), so the unflagged pods' keys are exact
        flagged = (engine.result_status(batch) & abi.KG_ST_UNSUPPORTED) != 0
        unsup = (want.status & abi.KG_ST_UNSUPPORTED) != 0
        assert not (flagged & ~unsup.any(axis=1)).any()
        assert flagged.sum() >= 5
        bound = kc.weight_nrf * want.score_nrf + kc.weight_la * want.score_la + kc.weight_numa * 100
        for j in np.nonzero(unsup.any(axis=1) & ~flagged)[0]:
            for i in np.nonzero(unsup[j])[0]:
                assert int(abi.make_key(int(bound[j, i]), int(i))) < int(keys[j, 0]), (j, i)
        with pytest.raises(engine.Unsupported):
            engine.replay(snap, batch)
        aff = _affected(marked, pods)
        feas = want.status == 0
        j, i = np.argwhere(aff & ((want.status & abi.KG_ST_UNSUPPORTED) != 0))[0]
        with pytest.raises(engine.Unsupported):
            engine.reserve(snap, batch, int(j), int(i))
        j2, i2 = np.argwhere(~aff & feas)[0]
        engine.reserve(snap, batch, int(j2), int(i2))
    finally:
        ctx.close()
