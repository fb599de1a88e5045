"""BASELINE configs 1 and 3 exercised whole on the device.

Config 1 (synth.cluster(1): 1k nodes x 500 pods, NodeResourcesFit + LoadAware): the full verify matrix
and the top-k selection equal the oracle's. Config 3 (synth.cluster(3): 50k pods placed one by one on
10k nodes): every placement and total equals the oracle's replay, committed as
tests/golden/config3_replay.npz (tests/golden/make_config3_golden.py)."""
import os
import sys

import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, synth

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_config3_golden  # noqa: E402

GOLDEN3 = os.path.join(HERE, "golden", "config3_replay.npz")


def golden3():
    g = np.load(GOLDEN3, allow_pickle=False)
    return g["node"], g["total"], str(g["digest"])


def test_config3_golden_matches_generator_and_oracle():
    """The committed vector belongs to today's generator, and its head is the oracle's sequential replay."""
    cfg, nodes, pods = synth.cluster(3)
    node, total, dig = golden3()
    assert dig == make_config3_golden.digest(nodes, pods)
    assert len(node) == abi.table_len(pods) == 50_000
    head = 1500
    want, wtot = oracle_lib.OracleState(cfg.kg_config(), nodes).replay(abi.take(pods, np.arange(head)))
    assert np.array_equal(want, node[:head]) and np.array_equal(wtot, total[:head])
    assert (node < 0).any() and (node >= 0).mean() > 0.9


@pytest.fixture(scope="module")
def ctx():
    from koordinator_amd import engine

    c = engine.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["window", "step"])
def test_config3_full_replay(ctx, monkeypatch, mode):
    from koordinator_amd import engine

    if mode == "step":
        monkeypatch.setenv("KG_REPLAY_STEP", "1")
    cfg, nodes, pods = synth.cluster(3)
    snap = engine.Snapshot(ctx, cfg.kg_config(), nodes)
    node, total = engine.replay(snap, engine.PodBatch(ctx, pods))
    want, wtot, _ = golden3()
    bad = np.flatnonzero(node != want)
    assert len(bad) == 0, f"{len(bad)} placements differ, first pod {bad[0]}: gpu {node[bad[0]]} oracle {want[bad[0]]}"
    assert np.array_equal(total, wtot)


@pytest.mark.gpu
def test_config3_full_replay_with_reasons(ctx):
    """The FitError diagnosis mode (per-pod OR of the filter bits) places exactly like the window replay;
    every unschedulable pod reports at least one NodeResourcesFit reason."""
    from koordinator_amd import engine

    cfg, nodes, pods = synth.cluster(3)
    snap = engine.Snapshot(ctx, cfg.kg_config(), nodes)
    node, total, why = engine.replay(snap, engine.PodBatch(ctx, pods), reasons=True)
    want, wtot, _ = golden3()
    assert np.array_equal(node, want) and np.array_equal(total, wtot)
    assert np.all(why[node < 0] & abi.KG_ST_NRF_MASK)


@pytest.mark.gpu
def test_config1_full_verify_and_select(ctx):
    from koordinator_amd import engine

    cfg, nodes, pods = synth.cluster(1)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    got = engine.eval_verify(snap, batch)
    ref = oracle_lib.eval_verify(kc, nodes, pods)
    for f in ("status", "score_nrf", "score_la", "score_numa", "total", "numa_zone"):
        a, b = getattr(got, f), getattr(ref, f)
        assert np.array_equal(a, b), f
    assert 0 < got.feasible.mean() < 1
    for k in (1, 3):
        assert np.array_equal(engine.eval_select(snap, batch, k), oracle_lib.select(kc, nodes, pods, k))
