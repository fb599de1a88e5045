"""Parity of the HIP engine (through the C ABI) with the CPU oracle and the reference's known answers.

Bar: bit-exact — filter status bits, int64 per-plugin scores, totals, NUMA zone choice, selected
hosts (deterministic tie-break) and replay placements / final node state.
"""
import os

import numpy as np
import pytest

import kat
import oracle_lib
from koordinator_amd import abi, engine, synth

pytestmark = pytest.mark.gpu

VERIFY_FIELDS = ("status", "score_nrf", "score_la", "score_numa", "total", "numa_zone")


@pytest.fixture(scope="module")
def ctx():
    c = engine.Context(0)
    yield c
    c.close()


def assert_verify_equal(got, ref, what=""):
    for name in VERIFY_FIELDS:
        a, b = getattr(got, name), getattr(ref, name)
        if not np.array_equal(a, b):
            bad = np.argwhere(a != b)
            j, i = bad[0]
            raise AssertionError(f"{what}: {name} differs at {len(bad)} pairs, first pod {j} node {i}: "
                                 f"gpu={a[j, i]} oracle={b[j, i]}")


LA = kat.load("loadaware_kat.json")


@pytest.mark.parametrize("case", LA["cases"], ids=[c["name"] for c in LA["cases"]])
def test_loadaware_kat_gpu(ctx, case):
    cfg, nodes, pods = kat.la_case(case, LA["node_default"])
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    got = engine.eval_verify(snap, batch)
    if case["kind"] == "filter":
        code, reason = kat.la_status(int(got.status[0, 0]) & abi.KG_ST_LA_MASK)
        assert code == case["want"]["code"], case["ref"]
        if "reason" in case["want"]:
            assert reason == case["want"]["reason"]
    else:
        assert got.score_la[0, 0] == case["want"]["score"], case["ref"]
    assert_verify_equal(got, oracle_lib.eval_verify(kc, nodes, pods), case["name"])


@pytest.mark.parametrize("seed,n_nodes,n_pods,numa,scale", [
    (1, 1000, 200, False, 1.0),   # config-1 shape (NodeResourcesFit + LoadAware)
    (2, 1500, 256, True, 1.0),    # + NodeNUMAResource (SingleNUMANode, amplification)
    (3, 700, 300, True, 12.0),    # large pods: NodeResourcesFit / NUMA alignment failures
    (4, 257, 65, True, 4.0),      # ragged sizes (not multiples of 64 / 256)
])
def test_verify_matrix_matches_oracle(ctx, seed, n_nodes, n_pods, numa, scale):
    cfg, nodes, pods = synth.small(n_nodes, n_pods, seed=seed, numa=numa, scale=scale)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    got = engine.eval_verify(snap, batch)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    assert_verify_equal(got, ref, f"seed {seed}")
    assert 0 < got.feasible.mean() < 1


@pytest.mark.parametrize("k", [1, 2, 4])
@pytest.mark.parametrize("seed,n_nodes,n_pods,scale", [(5, 2000, 333, 1.0), (6, 999, 1000, 8.0), (7, 64, 1, 1.0)])
def test_select_matches_oracle(ctx, k, seed, n_nodes, n_pods, scale):
    cfg, nodes, pods = synth.small(n_nodes, n_pods, seed=seed, scale=scale)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes, index_base=1000 * seed)
    batch = engine.PodBatch(ctx, pods)
    got = engine.eval_select(snap, batch, k)
    want = oracle_lib.select(kc, nodes, pods, k, index_base=1000 * seed)
    assert np.array_equal(got, want)


def test_select_ties_break_to_lowest_index(ctx):
    cfg, nodes, pods = synth.small(1, 8, seed=9)
    many = abi.take(nodes, np.zeros(500, np.int64))  # 500 identical nodes
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, many)
    batch = engine.PodBatch(ctx, pods)
    keys = engine.eval_select(snap, batch, 4)
    want = oracle_lib.select(kc, many, pods, 4)
    assert np.array_equal(keys, want)
    feas = keys[:, 0] != 0
    assert np.all(abi.key_node(keys[feas, 0]) == 0)
    assert np.all(abi.key_node(keys[feas, 1]) == 1)


def test_select_empty_and_unschedulable(ctx):
    cfg, nodes, pods = synth.small(50, 10, seed=10)
    kc = cfg.kg_config()
    huge = dict(pods)
    huge["req_cpu"] = np.full(10, 10 ** 9, np.int64)
    huge["flags"] = pods["flags"] | abi.KG_POD_HAS_CPU
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, huge)
    keys = engine.eval_select(snap, batch, 1)
    assert np.all(keys == 0)
    empty_nodes = abi.take(nodes, np.zeros(0, np.int64))
    snap0 = engine.Snapshot(ctx, kc, empty_nodes)
    keys0 = engine.eval_select(snap0, engine.PodBatch(ctx, pods), 1)
    assert np.all(keys0 == 0)


def test_large_values_take_exact_integer_path(ctx):
    cfg, nodes, pods = synth.small(300, 50, seed=11)
    big = {k: v.copy() for k, v in nodes.items()}
    big["alloc_mem"][:100] = 1 << 50  # beyond the exact-double range of the fast quotient
    big["la_alloc1"][:100] = 1 << 50
    big["req_mem"][100:200] = -(1 << 47)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, big)
    batch = engine.PodBatch(ctx, pods)
    assert_verify_equal(engine.eval_verify(snap, batch), oracle_lib.eval_verify(kc, big, pods), "big values")


@pytest.mark.parametrize("seed,n_nodes,n_pods,scale", [(12, 400, 900, 10.0), (13, 1000, 3000, 8.0)])
def test_replay_matches_oracle(ctx, seed, n_nodes, n_pods, scale):
    cfg, nodes, pods = synth.small(n_nodes, n_pods, seed=seed, scale=scale)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes, index_base=7)
    batch = engine.PodBatch(ctx, pods)
    node, total = engine.replay(snap, batch)
    st = oracle_lib.OracleState(kc, nodes)
    want_node, want_total = st.replay(pods, index_base=7)
    assert np.array_equal(node, want_node)
    assert np.array_equal(total, want_total)
    assert (node < 0).any() and (node >= 0).any()  # the cluster fills up
    got_state = snap.read_state()
    want_state = st.table()
    for k, v in got_state.items():
        assert np.array_equal(v, want_state[k]), k


def test_assume_forget_round_trip(ctx):
    cfg, nodes, pods = synth.small(200, 40, seed=14)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    before = snap.read_state()
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    st = oracle_lib.OracleState(kc, nodes)
    placed = []
    for j in range(40):
        feas = np.flatnonzero(ref.status[j] == 0)
        if len(feas) == 0:
            continue
        i = int(feas[j % len(feas)])
        engine.assume(snap, batch, j, i)
        st.assume(i, pods, j)
        placed.append((j, i, int(ref.numa_zone[j, i])))
    got = snap.read_state()
    want = st.table()
    for k, v in got.items():
        assert np.array_equal(v, want[k]), k
    # Unreserve with the zone each Reserve allocated from (read back from the oracle's view before it)
    st2 = oracle_lib.OracleState(kc, nodes)
    zones = []
    for j, i, _ in placed:
        view = st2.table()
        z = int(oracle_lib.eval_pair(kc, view, i, pods, j).zone)
        zones.append(z)
        st2.assume(i, pods, j)
    for (j, i, _), z in zip(reversed(placed), reversed(zones)):
        engine.forget(snap, batch, j, i, z)
    after = snap.read_state()
    for k, v in after.items():
        assert np.array_equal(v, before[k]), k


def test_update_rows(ctx):
    cfg, nodes, pods = synth.small(500, 64, seed=15)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    rows = np.array([3, 77, 499], np.uint32)
    _, other, _ = synth.small(3, 1, seed=16)
    snap.update_rows(rows, other)
    merged = {k: v.copy() for k, v in nodes.items()}
    for k in merged:
        merged[k][rows] = other[k]
    assert_verify_equal(engine.eval_verify(snap, batch), oracle_lib.eval_verify(kc, merged, pods), "update_rows")


def test_config2_full_size_properties(ctx):
    """10k nodes x 10k pods (config 2): sampled bit-exact selection + whole-matrix invariants."""
    cfg, nodes, pods = synth.cluster(2)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    keys = engine.eval_select(snap, batch, 4)
    # descending, distinct node indices, valid range
    assert np.all(keys[:, :-1] >= keys[:, 1:])
    nz = keys != 0
    idx = abi.key_node(keys)
    assert np.all((idx[nz] >= 0) & (idx[nz] < 10_000))
    rng = np.random.default_rng(0)
    sample = rng.choice(10_000, 96, replace=False)
    sub = abi.take(pods, sample)
    want = oracle_lib.select(kc, nodes, sub, 4)
    assert np.array_equal(keys[sample], want)
    # same batch evaluated again is bit-identical (deterministic reductions)
    again = engine.eval_select(snap, batch, 4)
    assert np.array_equal(keys, again)
