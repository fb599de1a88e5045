"""The host decode at cluster scale: a 2000-node cluster built from Kubernetes-style objects (nodes with
amplification annotations, NUMA topologies, NodeMetrics, running pods with NUMA allocations) through the
event caches (cluster.ClusterState), and pending pods decoded from pod objects (decode.pods_table: containers,
init containers and restartable sidecars, overhead, limits, priority classes, QoS labels, batch resources,
LSR cpuset pods with resource-spec annotations). The CPU test checks the incremental rows against a rebuild
from the objects; the GPU test runs Filter + Score + selectHost and the verify matrix of the decoded inputs
on the device against the oracle."""
import json
import random

import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, decode
from test_cluster import World, tables_equal, world_cfg

N_NODES, N_EVENTS, N_PENDING = 2000, 6000, 600


def pending_objects(n, seed):
    r = random.Random(seed)
    pods = []
    for j in range(n):
        cpu = r.choice([100, 250, 500, 1000, 2000, 4000])
        mem = r.choice([128, 512, 1024, 4096])
        req = {"cpu": f"{cpu}m", "memory": f"{mem}Mi"}
        c = {"name": "main", "resources": {"requests": dict(req)}}
        if r.random() < 0.5:
            c["resources"]["limits"] = {"cpu": f"{2 * cpu}m", "memory": f"{2 * mem}Mi"}
        spec = {"containers": [c]}
        labels, ann = {}, {}
        k = r.random()
        if k < 0.15:  # init container larger than the app, plus a restartable sidecar
            spec["initContainers"] = [{"name": "init", "resources": {"requests": {"cpu": f"{cpu + 500}m"}}},
                                      {"name": "side", "restartPolicy": "Always",
                                       "resources": {"requests": {"cpu": "100m", "memory": "64Mi"}}}]
        elif k < 0.2:
            spec["overhead"] = {"cpu": "50m", "memory": "32Mi"}
        q = r.random()
        if q < 0.2:  # koord-batch pod: batch resources instead of cpu / memory
            labels["koordinator.sh/qosClass"] = "BE"
            spec["priority"] = 5500
            c["resources"] = {"requests": {"kubernetes.io/batch-cpu": str(cpu), "kubernetes.io/batch-memory": f"{mem}Mi"}}
        elif q < 0.3:  # LSR prod pod: binds cpusets (whole cores)
            labels["koordinator.sh/qosClass"] = "LSR"
            spec["priority"] = 9500
            c["resources"] = {"requests": {"cpu": str(max(1, cpu // 1000)), "memory": f"{mem}Mi"}}
            spec.pop("initContainers", None)
            spec.pop("overhead", None)
            if r.random() < 0.5:
                ann[decode.ANN_RESOURCE_SPEC] = json.dumps({"preferredCPUBindPolicy": r.choice(["SpreadByPCPUs", "FullPCPUs"])})
        elif q < 0.4:
            spec["priority"] = 7500  # koord-mid
        elif q < 0.45:
            spec["containers"] = [{"name": "empty", "resources": {}}]
        else:
            spec["priority"] = r.choice([9000, 9999])
        md = {"namespace": "default", "name": f"pending-{j}", "uid": f"pend-{j}", "labels": labels}
        if ann:
            md["annotations"] = ann
        pods.append({"metadata": md, "spec": spec, "status": {"phase": "Pending"}})
    return pods


@pytest.fixture(scope="module")
def world():
    cfg = world_cfg()
    cfg.plugins = abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_LA | abi.KG_PLUGIN_NUMA
    w = World(cfg, N_NODES, 77)
    for _ in range(N_EVENTS):
        w.step()
    return w


def test_decode_at_scale_matches_rebuild(world):
    tables_equal(world.state.table(), world.reference_table())
    pods = decode.pods_table(pending_objects(N_PENDING, 5), world.cfg)
    f = pods["flags"]
    assert (f & abi.KG_POD_CPU_BIND).any() and (f & abi.KG_POD_NUMA_SKIP).any()
    assert (pods["sc_req0"] > 0).any() and ((f & abi.KG_POD_PROD) != 0).any()
    t = world.state.table()
    assert (t["cpu_amp_ratio"] > 1).sum() > 100 and (t["numa_zones"] > 0).sum() > 20


@pytest.mark.gpu
def test_decoded_cluster_select_and_verify_on_gpu(world):
    from koordinator_amd import engine
    cfg = world.cfg
    kc = cfg.kg_config()
    nodes = world.state.table()
    pods = decode.pods_table(pending_objects(N_PENDING, 5), cfg)
    ctx = engine.Context(0)
    try:
        snap = engine.Snapshot(ctx, kc, nodes)
        batch = engine.PodBatch(ctx, pods)
        for k in (1, 3):
            assert np.array_equal(engine.eval_select(snap, batch, k), oracle_lib.select(kc, nodes, pods, k))
        got = engine.eval_verify(snap, batch)
        ref = oracle_lib.eval_verify(kc, nodes, pods)
        for name in ("status", "score_nrf", "score_la", "score_numa", "total", "numa_zone"):
            assert np.array_equal(getattr(got, name), getattr(ref, name)), name
        assert (ref.status == 0).mean() > 0.2
    finally:
        ctx.close()
