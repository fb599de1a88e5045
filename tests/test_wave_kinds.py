"""The fast select's wave kinds (kg_eval.h fast_kind_match): kg_pods_upload groups a batch's pods so that
whole waves of prod pods (no scalar requests) or koord-batch pods (scalar requests only) run loops
specialised for them. Those loops must give exactly the general loop's keys, including on the nodes
where their shortcuts matter: "Too many pods" nodes (the batch loop reads the record flag instead of
comparing against the folded cpu headroom), nodes without scalar or cpu capacity (zero weights, zero
reciprocals), DaemonSet pods and skipped pods (general loop), and mixed waves at group boundaries."""
import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, synth

PROD, DS, SKIP, BIND = abi.KG_POD_PROD, abi.KG_POD_DAEMONSET, abi.KG_POD_NUMA_SKIP, abi.KG_POD_CPU_BIND


def wave_kind(pods, j):
    """Host restatement of the kind predicate (0 prod, 1 koord-batch, 2 general)."""
    f = int(pods["flags"][j])
    sc0, sc1 = int(pods["sc_req0"][j]), int(pods["sc_req1"][j])
    if (f & (PROD | DS | SKIP | BIND)) == PROD and f & (abi.KG_POD_HAS_CPU | abi.KG_POD_HAS_MEM) and sc0 == 0 and sc1 == 0:
        return 0
    if (f & (PROD | DS | SKIP | BIND | abi.KG_POD_HAS_CPU | abi.KG_POD_HAS_MEM)) == 0 and \
            pods["req_cpu"][j] == 0 and pods["req_mem"][j] == 0 and sc0 != 0 and sc1 != 0:
        return 1
    return 2


def edge_cluster(seed, n_nodes=1500, n_pods=900):
    cfg, nodes, pods = synth.small(n_nodes, n_pods, seed=seed, numa=True)
    nodes = {k: v.copy() for k, v in nodes.items()}
    pods = {k: v.copy() for k, v in pods.items()}
    r = np.random.default_rng(seed)
    full = r.random(n_nodes) < 0.08  # "Too many pods"
    nodes["num_pods"][full] = nodes["alloc_pods"][full]
    nodes["sc_alloc0"][r.random(n_nodes) < 0.1] = 0  # no batch-cpu capacity: weight 0, reciprocal 0
    nodes["sc_alloc1"][r.random(n_nodes) < 0.1] = 0
    zero_cpu = r.random(n_nodes) < 0.02
    nodes["alloc_cpu"][zero_cpu] = 0
    nodes["req_cpu"][zero_cpu] = 0
    nodes["nz_cpu"][zero_cpu] = 0
    one_zone = (nodes["numa_policy"] == abi.KG_NUMA_SINGLE_NODE) & (r.random(n_nodes) < 0.3)
    nodes["numa_zones"][one_zone] = 1  # node-level NUMA score on single-zone SingleNUMANode nodes
    # pods: DaemonSet prod pods, prod pods with one scalar request, batch pods with one scalar only
    ds = r.random(n_pods) < 0.05
    pods["flags"][ds] |= DS
    prod = (pods["flags"] & PROD) != 0
    one_sc = prod & (r.random(n_pods) < 0.05)
    pods["sc_req0"][one_sc] = 500
    batch = ~prod & (pods["sc_req0"] > 0)
    half = batch & (r.random(n_pods) < 0.05)
    pods["sc_req1"][half] = 0
    nohas = prod & (r.random(n_pods) < 0.03)  # prod pods without HAS_CPU / HAS_MEM: the general loop
    pods["flags"][nohas] &= ~np.uint32(abi.KG_POD_HAS_CPU | abi.KG_POD_HAS_MEM)
    return cfg, nodes, pods


def test_kinds_cover_every_loop():
    _, _, pods = edge_cluster(21)
    kinds = np.array([wave_kind(pods, j) for j in range(len(pods["flags"]))])
    for k in (0, 1, 2):
        assert (kinds == k).sum() >= 64, k


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [21, 22])
def test_wave_kinds_select_matches_oracle(seed):
    from koordinator_amd import engine
    cfg, nodes, pods = edge_cluster(seed)
    kc = cfg.kg_config()
    ctx = engine.Context(0)
    try:
        snap = engine.Snapshot(ctx, kc, nodes)
        batch = engine.PodBatch(ctx, pods)
        for k in (1, 3):
            got = engine.eval_select(snap, batch, k)
            want = oracle_lib.select(kc, nodes, pods, k)
            bad = np.flatnonzero((got != want).any(axis=1))
            assert not len(bad), (k, bad[:5], [wave_kind(pods, j) for j in bad[:5]])
        assert (want[:, 0] != 0).mean() > 0.3
    finally:
        ctx.close()
