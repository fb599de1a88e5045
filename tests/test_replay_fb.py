"""Config-5 replay on the fast-base step kernel (k_ext_replay<false, true>): a batch whose pods are all in the fast domain
and whose GPU pods all have a request class replays without FitError reasons on the fast block (the fast-base select's
arithmetic), DeviceShare from the batch's DevSum table and the SingleNUMANode records' GPU hints from e.gz, both built at
the replay's start and refreshed on the winner after every Reserve that changes its minors. Placements, totals, minors,
quota used, the final node state and GPU tables equal the oracle replay's (oracle/kg_oracle.c kgo_ext_replay) at >= 10k
nodes, and equal the device replay with reasons (the general per-pair path) on the same inputs."""
import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, engine, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = engine.Context(0)
    yield c
    c.close()


def _cluster(n_nodes, n_pods, seed, numa):
    """cluster5 with GPU-holding reservations (their restore inputs) and 70% of the pods in a reservation class."""
    cfg, nodes, pods, quotas, rsv, _, _ = synth.cluster5(n_nodes, n_pods, seed_config=seed, rsv_frac=0.5, rsv_gpu=True,
                                                         raw=True, numa=numa)
    pods = {k: v.copy() for k, v in pods.items()}
    rng = np.random.default_rng(seed)
    pods["rsv_class"] = np.where(rng.random(n_pods) < 0.7, rng.integers(0, synth.N_RSV_CLASSES, n_pods),
                                 -1).astype(np.int32)
    pods["flags"] &= ~np.uint32(abi.KG_POD_RSV_REQUIRED)
    return cfg, nodes, pods, quotas, rsv


def _snap(ctx, kc, nodes, quotas, rsv):
    snap = engine.Snapshot(ctx, kc, nodes)
    snap.upload_quotas(quotas)
    snap.upload_reservations(rsv)
    return snap


@pytest.mark.parametrize("seed,numa", [(91, "single"), (92, "none")])
def test_fast_base_replay_matches_oracle(ctx, seed, numa):
    cfg, nodes, pods, quotas, rsv = _cluster(12_000, 400, seed, numa)
    assert rsv.n_gpu > 0 and (pods["dev_count"] > 0).sum() > 50
    kc = cfg.kg_config()
    snap = _snap(ctx, kc, nodes, quotas, rsv)
    batch = engine.PodBatch(ctx, pods)
    node, total = engine.replay(snap, batch)
    minors = engine.replay_minors(batch)
    st = oracle_lib.OracleState(kc, nodes)
    onode, ototal, ominors, qu, qn = st.ext_replay(pods, quotas, rsv=rsv)
    assert np.array_equal(node, onode)
    assert np.array_equal(total, ototal)
    assert np.array_equal(minors, ominors)
    used, _, npu, _ = snap.read_quotas()
    assert np.array_equal(used, qu) and np.array_equal(npu, qn)
    state = snap.read_state()
    assert np.array_equal(state["dev_free"], st.dev_free())
    want = st.table()
    for k in ("req_cpu", "req_mem", "num_pods", "nz_cpu", "nz_mem", "numa_zone_status"):
        assert np.array_equal(state[k], want[k]), k
    assert (node >= 0).sum() > 200 and (minors != 0).sum() > 20


def test_fast_base_replay_equals_the_general_path(ctx):
    """The same replay with reasons (every pair on eval_pair_ext) and without (fast-base pairs): same placements."""
    cfg, nodes, pods, quotas, rsv = _cluster(3000, 600, 93, "single")
    kc = cfg.kg_config()
    a = _snap(ctx, kc, nodes, quotas, rsv)
    node_a, total_a, _ = engine.replay(a, engine.PodBatch(ctx, pods), reasons=True)
    b = _snap(ctx, kc, nodes, quotas, rsv)
    batch = engine.PodBatch(ctx, pods)
    node_b, total_b = engine.replay(b, batch)
    assert np.array_equal(node_a, node_b)
    assert np.array_equal(total_a, total_b)
    assert np.array_equal(a.read_state()["dev_free"], b.read_state()["dev_free"])
