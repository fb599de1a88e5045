"""Config-5 one-pod-per-cycle replay at the BASELINE size (synth.config5(): 100k nodes, every plugin, reservations
holding GPUs with their DeviceShare restore inputs, ElasticQuota), against the oracle's placements of the first
N_HEAD pods committed in tests/golden/replay5_head.npz (tests/golden/make_replay5_golden.py).

- CPU: the committed vector belongs to today's generator (digest) and its first pods re-check on the serial oracle.
- GPU: kg_replay of the first N_HEAD pods through the C ABI equals it bit for bit: nodes, totals, GPU minors, the
  FitError reasons and the final quota used."""
import os
import sys

import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_replay5_golden as G  # noqa: E402


@pytest.fixture(scope="module")
def work():
    return G.workload()


@pytest.fixture(scope="module")
def golden():
    z = np.load(G.PATH)
    return {k: z[k] for k in z.files}


def test_replay5_golden_matches_generator_and_oracle(work, golden):
    kc, nodes, pods, quotas, rsv = work
    assert str(golden["digest"]) == G._digest(nodes, pods, quotas, rsv), "generator changed: rerun make_replay5_golden.py"
    assert len(golden["node"]) == G.N_HEAD and (golden["node"] >= 0).sum() > 0.8 * G.N_HEAD
    n = 24
    node, total, minors, _, _ = oracle_lib.OracleState(kc, nodes).ext_replay(abi.take(pods, np.arange(n)), quotas, rsv=rsv)
    assert np.array_equal(node, golden["node"][:n]) and np.array_equal(total, golden["total"][:n])
    assert np.array_equal(minors, golden["minors"][:n])


@pytest.mark.gpu
@pytest.mark.parametrize("reasons", [False, True], ids=["fast_base", "with_reasons"])
def test_replay5_full_size_device(work, golden, reasons):
    """Without reasons the replay takes the fast-base step the bench times; with them every pair runs the general
    evaluation and reports its filter bits."""
    from koordinator_amd import engine
    kc, nodes, pods, quotas, rsv = work
    ctx = engine.Context(0)
    try:
        snap = engine.Snapshot(ctx, kc, nodes)
        snap.upload_quotas(quotas)
        snap.upload_reservations(rsv)
        batch = engine.PodBatch(ctx, abi.take(pods, np.arange(G.N_HEAD)))
        out = engine.replay(snap, batch, reasons=reasons)
        node, total = out[0], out[1]
        minors = engine.replay_minors(batch)
        used, _, npu, _ = snap.read_quotas()
    finally:
        ctx.close()
    bad = np.nonzero(node != golden["node"])[0]
    assert bad.size == 0, f"first differing pod {bad[:5]}"
    assert np.array_equal(total, golden["total"])
    assert np.array_equal(minors, golden["minors"])
    if reasons:
        assert np.array_equal(out[2], golden["reason"])
    assert np.array_equal(used, golden["quota_used"]) and np.array_equal(npu, golden["quota_np_used"])
