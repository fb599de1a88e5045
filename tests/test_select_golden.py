"""Whole-batch selectHost parity at the BASELINE sizes of the matrix-mode configurations.

The committed vectors tests/golden/select_config{2,4,5}.npz hold the oracle's top-3 keys of EVERY pod of
config 2 (10k x 10k), config 4 (100k nodes x 10k pods, one GPU), config 5 (100k x 10k with DeviceShare,
Reservation and ElasticQuota, 20% SingleNUMANode nodes) and the mixed bench config 6 (10k x 10k, Restricted /
BestEffort / CPU-bind-policy nodes, LSR pods: cpusets under NUMA policies too), made by tests/golden/make_select_golden.py. The CPU tests pin the vectors to
today's generator (cluster digest) and re-check a pod sample on the oracle; the GPU tests run the whole
batch through the C ABI (kg_eval_select, k = 1 and k = 3) and compare every key bit for bit."""
import os
import sys

import numpy as np
import pytest

import oracle_lib  # noqa: F401  (builds the oracle if needed)
from koordinator_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_select_golden as G  # noqa: E402

CONFIGS = [2, 4, 5, 6]


@pytest.mark.parametrize("config", CONFIGS)
def test_select_golden_matches_generator_and_oracle(config):
    keys, dig = G.load(config)
    kc, nodes, pods, quotas, rsv = G.workload(config)
    assert dig == G._digest(nodes, pods, quotas, rsv), "generator changed: rerun make_select_golden.py"
    n = abi.table_len(pods)
    assert keys.shape == (n, G.K)
    idx = np.concatenate([np.arange(8), np.random.default_rng(config).choice(n, 24, replace=False)])
    assert np.array_equal(keys[idx], G.oracle_keys(kc, nodes, pods, quotas, rsv, idx))
    # descending per pod, distinct nodes
    assert np.all(keys[:, :-1] >= keys[:, 1:])
    nz = keys[:, 1] != 0
    assert np.all(keys[nz, 0] != keys[nz, 1])


@pytest.fixture(scope="module")
def ctx():
    from koordinator_amd import engine

    c = engine.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("config", CONFIGS)
def test_select_whole_batch_bit_exact(ctx, config):
    from koordinator_amd import engine

    want, _ = G.load(config)
    kc, nodes, pods, quotas, rsv = G.workload(config)
    snap = engine.Snapshot(ctx, kc, nodes)
    if quotas is not None:
        snap.upload_quotas(quotas)
    if rsv is not None:
        snap.upload_reservations(rsv)
    batch = engine.PodBatch(ctx, pods)
    for k in (1, 3):
        got = engine.eval_select(snap, batch, k)
        st = engine.result_status(batch)
        assert not np.any(st & abi.KG_ST_UNSUPPORTED), "a pair left the device path"
        bad = np.flatnonzero(np.any(got != want[:, :k], axis=1))
        assert len(bad) == 0, (f"config {config} k={k}: {len(bad)} pods differ, first {bad[0]}: "
                               f"gpu {got[bad[0]]} oracle {want[bad[0], :k]}")
    batch.close()
    snap.close()
