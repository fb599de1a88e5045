"""Host event-to-row-delta throughput of the f1 layer (koordinator_amd/cluster.py): ClusterState event handlers
(pod add / update / delete, NodeMetric) and SnapshotSync's row rebuild (rows_since + table), at 10k and 100k nodes.
The device upload of the delta (kg_snapshot_update_rows) is not included: this is the host half of a sync.

Usage: python tools/sync_rate.py [n_nodes ...] [--events E] [--out profiles/r3/sync_rate.json]
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from koordinator_amd import cluster, config  # noqa: E402


def nodes(n, r):
    return [{"metadata": {"name": f"node-{i}", "labels": {}, "annotations": {}},
             "status": {"allocatable": {"cpu": str(r.choice([32, 64, 96])), "memory": f"{r.choice([128, 256])}Gi",
                                        "pods": "110"}}} for i in range(n)]


def pod(seq, node, t, r):
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"uid": f"u{seq}", "namespace": "default", "name": f"p{seq}", "labels": {}, "annotations": {}},
            "spec": {"nodeName": node, "priority": r.choice([0, 9500]),
                     "containers": [{"name": "c", "resources": {"requests": {
                         "cpu": f"{r.choice([100, 250, 500, 1000])}m", "memory": f"{r.choice([128, 512, 1024])}Mi"}}}]},
            "status": {"phase": "Running",
                       "conditions": [{"type": "PodScheduled", "status": "True", "lastTransitionTime": t - 50}]}}


def metric(node, t, r):
    return {"metadata": {"name": node}, "spec": {"collectPolicy": {"reportIntervalSeconds": 60}},
            "status": {"updateTime": t - 1, "nodeMetric": {"nodeUsage": {"resources": {
                "cpu": f"{r.randrange(1000, 30000)}m", "memory": f"{r.randrange(1, 100)}Gi"}}}, "podsMetric": []}}


def measure(n_nodes, n_events, seed=0):
    r = random.Random(seed)
    cfg = config.bench_profile(numa=False)
    t_now = 1_000_000.0
    ns = nodes(n_nodes, r)
    t0 = time.perf_counter()
    st = cluster.ClusterState(cfg, ns, clock=lambda: t_now)
    build_s = time.perf_counter() - t0
    names = [x["metadata"]["name"] for x in ns]
    # prebuilt event objects (the informer hands over decoded objects; building them is not the layer's work)
    adds = [pod(i, r.choice(names), t_now, r) for i in range(n_events)]
    mets = [metric(r.choice(names), t_now, r) for _ in range(n_events // 4)]
    gen0 = st.generation
    t0 = time.perf_counter()
    for p in adds:
        st.on_pod_add(p)
    for m in mets:
        st.on_node_metric(m)
    ev_s = time.perf_counter() - t0
    st.tick()
    t0 = time.perf_counter()
    rows = st.rows_since(gen0)
    st.table(rows)
    rows_s = time.perf_counter() - t0
    return {"nodes": n_nodes, "events": len(adds) + len(mets), "pod_adds": len(adds), "node_metrics": len(mets),
            "state_build_s": round(build_s, 3), "events_per_s": (len(adds) + len(mets)) / ev_s,
            "rows_touched": int(len(rows)), "rows_rebuilt_per_s": len(rows) / rows_s if rows_s else None,
            "delta_rebuild_s": round(rows_s, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n_nodes", nargs="*", type=int, default=[10_000, 100_000])
    ap.add_argument("--events", type=int, default=20_000)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = [measure(n, a.events) for n in a.n_nodes]
    for x in res:
        print(json.dumps(x))
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"note": "host half of SnapshotSync (event handlers + row rebuild), one Python thread",
                       "cpu": os.cpu_count(), "results": res}, f, indent=1)


if __name__ == "__main__":
    main()
