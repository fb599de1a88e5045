"""Event-driven snapshot maintenance, host side.

1. LoadAware podAssignCache known answers transcribed from loadaware/pod_assign_cache_test.go
   (TestPodAssignCache_OnAdd :58-164, _OnUpdate :166-333, _OnUpdate_NodeNameChange :335-423,
   _OnDelete :425-571, TestShouldEstimatePodDeadline :573-653, TestNodeMetric :655-849), run on
   koordinator_amd.cluster.PodAssignCache.
2. Streams of random Pod / NodeMetric / NRT / Device events: after every batch the incrementally
   maintained rows equal rows rebuilt from scratch by decode.node_row over the same objects.
"""
import copy
import json
import random

import numpy as np
import pytest

from koordinator_amd import abi, cluster, decode
from koordinator_amd.config import LoadAwareArgs, SchedulerConfig

GI = 1 << 30
MI = 1 << 20
NOW = 1_000_000.0
MID_CPU, MID_MEM = "kubernetes.io/mid-cpu", "kubernetes.io/mid-memory"
PRIO_MID_DEFAULT = 7500  # extension.PriorityMidValueDefault (apis/extension/priority_utils.go:30)


def mk(uid="", ns="", name="", node="", phase=None, req=None, priority=None, conditions=None, annotations=None):
    """st.MakePod() with the builder calls the Go tests use."""
    md = {"namespace": ns, "name": name}
    if uid:
        md["uid"] = uid
    if annotations:
        md["annotations"] = dict(annotations)
    spec = {"containers": [{"name": "c", "resources": {"requests": dict(req)} if req else {}}]}
    if node:
        spec["nodeName"] = node
    if priority is not None:
        spec["priority"] = priority
    status = {}
    if phase:
        status["phase"] = phase
    if conditions:
        status["conditions"] = [dict(c) for c in conditions]
    return {"metadata": md, "spec": spec, "status": status}


def la_args(**kw):
    return LoadAwareArgs(**kw).defaulted()


def new_cache(factors=(100, 100), clock=NOW, **kw):
    la = la_args(estimated_scaling_factors={"cpu": factors[0], "memory": factors[1]}, **kw)
    return cluster.PodAssignCache(la, clock=lambda: clock)


def metric(name, **status):
    return {"metadata": {"name": name}, "status": status}


DEFAULT_EST = [250, 200 * MI]  # estimator.DefaultMilliCPURequest / DefaultMemoryRequest
TEST_KEY = ("default", "test")


# -- TestPodAssignCache_OnAdd (:58-164) ----------------------------------------------------------

@pytest.mark.parametrize("case", ["pending", "terminated", "no_resources", "prod", "non_prod", "reserve_pod"])
def test_on_add(case):
    node = "test-node"
    c = new_cache()
    c.add_or_update_node_metric(metric(node))
    pods = {
        "pending": mk(),
        "terminated": mk(node=node, phase="Failed"),
        "no_resources": mk("123456789", "default", "test", node, "Running"),
        "prod": mk("123456789", "default", "test", node, req={"cpu": "1", "memory": "4Gi"}),
        "non_prod": mk("123456789", "default", "test", node, priority=PRIO_MID_DEFAULT,
                       req={MID_CPU: "1k", MID_MEM: "4Gi"}),
        "reserve_pod": mk("reserve-uid-123", "default", "test-reservation", node, "Running",
                          annotations={"scheduling.koordinator.sh/reserve-pod": "true"}),
    }
    c.on_add(pods[case])
    n = c.get(node)
    if case in ("pending", "terminated", "reserve_pod"):
        assert len(n.pod_infos) == 0
        return
    if case == "no_resources":
        info = n.pod_infos["123456789"]
        assert info.timestamp == NOW and info.estimated == DEFAULT_EST and info.deadline is None
        assert n.node_delta == DEFAULT_EST and n.node_estimated == DEFAULT_EST
        assert n.node_delta_pods == {TEST_KEY} and n.node_estimated_pods == {TEST_KEY}
        return
    v = [1000, 4 * GI]
    assert n.node_delta == v and n.node_estimated == v
    assert n.node_delta_pods == {TEST_KEY} and n.node_estimated_pods == {TEST_KEY}
    if case == "prod":
        assert n.prod_delta == v and n.prod_delta_pods == {TEST_KEY}
    else:
        assert n.prod_delta == [0, 0] and n.prod_delta_pods == set()


# -- TestPodAssignCache_OnUpdate (:166-333) ------------------------------------------------------

def test_on_update():
    node = "test-node"
    sched = {"type": "PodScheduled", "status": "True", "lastTransitionTime": NOW + 1000e-9}
    init = {"type": "PodInitialized", "status": "True", "lastTransitionTime": NOW + 3000e-9}
    base = dict(uid="123456789", ns="default", name="test", node=node, phase="Running")
    cases = [
        ("pending", mk(), [], lambda n: len(n.pod_infos) == 0),
        ("terminated", mk(**{**base, "phase": "Failed"}), [mk(**base)], lambda n: len(n.pod_infos) == 0),
        ("no_resources", mk(**base), [],
         lambda n: (n.pod_infos["123456789"].timestamp == NOW and n.node_delta == DEFAULT_EST
                    and n.node_estimated == DEFAULT_EST and n.node_delta_pods == {TEST_KEY})),
        # metadata-only update: the cached pod (without the annotation) stays
        ("metadata_only", mk(**base, annotations={"foo": "bar"}), [mk(**base)],
         lambda n: "annotations" not in n.pod_infos["123456789"].pod["metadata"]),
        # conditions changed: renewed, timestamp from PodScheduled
        ("conditions", mk(**base, conditions=[sched, init]), [mk(**base, conditions=[sched])],
         lambda n: (n.pod_infos["123456789"].timestamp == sched["lastTransitionTime"]
                    and len(n.pod_infos["123456789"].pod["status"]["conditions"]) == 2
                    and n.node_delta == DEFAULT_EST and n.node_estimated == DEFAULT_EST)),
        # resources changed: renewed with the new estimate (no PodScheduled -> clock)
        ("resources", mk(**base, req={"cpu": "1", "memory": "4Gi"}), [mk(**base, conditions=[sched])],
         lambda n: (n.pod_infos["123456789"].timestamp == NOW
                    and n.pod_infos["123456789"].estimated == [1000, 4 * GI]
                    and n.node_delta == [1000, 4 * GI] and n.prod_delta == [1000, 4 * GI]
                    and n.node_estimated == [1000, 4 * GI] and n.prod_delta_pods == {TEST_KEY})),
    ]
    for name, pod, existing, want in cases:
        c = new_cache()
        c.add_or_update_node_metric(metric(node))
        for p in existing:
            c.on_add(p)
        c.on_update(None, pod)
        assert want(c.get(node)), name


# -- TestPodAssignCache_OnUpdate_NodeNameChange (:335-423) ----------------------------------------

@pytest.mark.parametrize("with_resources", [False, True])
def test_on_update_node_name_change(with_resources):
    req = {"cpu": "1", "memory": "4Gi"} if with_resources else None
    c = new_cache()
    c.add_or_update_node_metric(metric("node-a"))
    c.add_or_update_node_metric(metric("node-b"))
    old = mk("aaa", "default", "test-pod", "node-a", "Running", req=req)
    new = mk("aaa", "default", "test-pod", "node-b", "Running", req=req)
    c.on_add(old)
    c.on_update(old, new)
    src, dst = c.get("node-a"), c.get("node-b")
    assert len(src.pod_infos) == 0
    assert src.node_delta == [0, 0] and src.prod_delta == [0, 0] and src.node_estimated == [0, 0]
    assert src.node_delta_pods == set() and src.node_estimated_pods == set() and src.prod_delta_pods == set()
    v = [1000, 4 * GI] if with_resources else DEFAULT_EST
    key = {("default", "test-pod")}
    assert len(dst.pod_infos) == 1 and dst.node_delta == v and dst.node_estimated == v
    assert dst.node_delta_pods == key and dst.node_estimated_pods == key
    if with_resources:
        assert dst.prod_delta == v and dst.prod_delta_pods == key


# -- TestPodAssignCache_OnDelete (:425-571) ------------------------------------------------------

def test_on_delete():
    node = "test-node"

    def pm(name, prio, cpu, mem):
        return {"namespace": "default", "name": name, "priority": prio,
                "podUsage": {"resources": {"cpu": cpu, "memory": mem}}}

    m = metric(node, nodeMetric={"nodeUsage": {"resources": {"cpu": "70", "memory": "280Gi"}}},
               podsMetric=[pm("prod-0", "koord-prod", "50", "200Gi"), pm("prod-1", "koord-prod", "1", "6Gi"),
                           pm("prod-2", "koord-prod", "4", "2Gi"), pm("prod-3", "koord-mid", "3", "6Gi"),
                           pm("mid-1", "koord-mid", "1", "6Gi"), pm("mid-2", "koord-mid", "4", "2Gi"),
                           pm("mid-3", "koord-prod", "3", "6Gi")])
    c = new_cache(factors=(50, 50))
    c.add_or_update_node_metric(m)
    prod = {"cpu": "4", "memory": "8Gi"}
    mid = {MID_CPU: "4k", MID_MEM: "8Gi"}
    pods = [mk("1", "default", "prod-1", node, "Running", req=prod), mk("2", "default", "prod-2", node, "Running", req=prod),
            mk("3", "default", "prod-3", node, "Running", req=prod),
            mk("4", "default", "mid-1", node, "Running", req=mid, priority=PRIO_MID_DEFAULT),
            mk("5", "default", "mid-2", node, "Running", req=mid, priority=PRIO_MID_DEFAULT),
            mk("6", "default", "mid-3", node, "Running", req=mid, priority=PRIO_MID_DEFAULT)]
    for p in pods:
        c.on_add(p)
    n = c.get(node)
    assert n.prod_usage == [5000, 8 * GI]
    assert n.node_delta == [2000, 4 * GI]
    assert n.prod_delta == [3000, 6 * GI]
    assert n.node_estimated == [12000, 24 * GI]
    k = lambda *names: {("default", x) for x in names}  # noqa: E731
    assert n.node_delta_pods == k("prod-1", "prod-2", "mid-1", "mid-2")
    assert n.prod_delta_pods == k("prod-1", "prod-2", "prod-3")
    assert n.node_estimated_pods == k("prod-1", "prod-2", "prod-3", "mid-1", "mid-2", "mid-3")
    # deletes carry other specs (only the UID and node matter)
    c.on_delete(mk("1", "default", "prod-1", node, "Failed", req={"cpu": "2", "memory": "8Gi"}))
    for uid, name in [("2", "prod-2"), ("3", "prod-3"), ("4", "mid-1"), ("5", "mid-2"), ("6", "mid-3")]:
        c.on_delete(mk(uid, "default", name, node))
    n = c.get(node)
    assert len(n.pod_infos) == 0
    assert n.node_delta == [0, 0] and n.prod_delta == [0, 0] and n.node_estimated == [0, 0]
    assert n.node_delta_pods == set() and n.prod_delta_pods == set() and n.node_estimated_pods == set()


# -- TestShouldEstimatePodDeadline (:573-653) ----------------------------------------------------

def test_should_estimate_pod_deadline():
    now = NOW
    sched = {"type": "PodScheduled", "status": "True", "lastTransitionTime": now - 60}
    init_t = {"type": "PodInitialized", "status": "True", "lastTransitionTime": now - 30}
    init_m = {"type": "PodInitialized", "status": "True", "lastTransitionTime": now - 60}
    init_f = {"type": "PodInitialized", "status": "False", "lastTransitionTime": now - 60}
    A_S = "scheduling.koordinator.sh/load-estimated-seconds-after-pod-scheduled"
    A_I = "scheduling.koordinator.sh/load-estimated-seconds-after-initialized"
    cases = [
        ("disabled", {}, mk(), None),
        ("enabled for pod scheduled", dict(estimated_seconds_after_pod_scheduled=180),
         mk(ns="default", name="pod", conditions=[sched]), now + 120),
        ("disabled pod scheduled when pod initialized",
         dict(estimated_seconds_after_pod_scheduled=180, estimated_seconds_after_initialized=10),
         mk(ns="default", name="pod", conditions=[sched, init_t]), now - 20),
        ("enabled for pod initialized", dict(estimated_seconds_after_initialized=180),
         mk(ns="default", name="pod", conditions=[init_m]), now + 120),
        ("disabled for pod initialized when condition is not satisfied", dict(estimated_seconds_after_initialized=180),
         mk(ns="default", name="pod", conditions=[init_f]), None),
        ("after pod scheduled from metadata", dict(allow_customize_estimation=True),
         mk(ns="default", name="pod", conditions=[sched], annotations={A_S: "180"}), now + 120),
        ("after initialized from metadata", dict(allow_customize_estimation=True),
         mk(ns="default", name="pod", conditions=[init_m], annotations={A_I: "180"}), now + 120),
    ]
    for name, kw, pod, want in cases:
        la = la_args(**kw)
        assert decode.estimated_deadline(pod, now - 60, la) == want, name


# -- TestNodeMetric (:655-849) -------------------------------------------------------------------

def test_node_metric_disable_estimator():
    node = "test-node"
    m = metric(node, nodeMetric={"nodeUsage": {"resources": {"cpu": "72", "memory": "280Gi"}}},
               podsMetric=[None, {"name": "invalid"},
                           {"namespace": "default", "name": "prod-1", "priority": "koord-prod",
                            "podUsage": {"resources": {"cpu": "50", "memory": "200Gi"}}},
                           {"namespace": "default", "name": "mid-1", "priority": "koord-mid",
                            "podUsage": {"resources": {"cpu": "20", "memory": "75Gi"}}}])
    pods = [mk("1", "default", "prod-1", node, "Running", req={"cpu": "40", "memory": "160Gi"}),
            mk("2", "default", "mid-1", node, "Running", req={MID_CPU: "4k", MID_MEM: "8Gi"},
               priority=PRIO_MID_DEFAULT)]
    c = cluster.PodAssignCache(la_args(), clock=lambda: NOW)
    for p in pods:
        c.on_add(p)
    c.add_or_update_node_metric(m)
    assert c.get(node).prod_usage == [50000, 200 * GI]
    _delete_all(c, node, pods)


def test_node_metric_prod_usage_include_sys():
    node = "test-node"
    agg = [{"duration": "1m", "usage": {"avg": {"resources": {"cpu": "1", "memory": "2Gi"}},
                                        "p90": {"resources": {"cpu": "2", "memory": "4Gi"}}}},
           {"duration": "1h", "usage": {"avg": {"resources": {"cpu": "500m", "memory": "1Gi"}},
                                        "p90": {"resources": {"cpu": "1500m", "memory": "3Gi"}}}}]
    m = {"metadata": {"name": node}, "spec": {"collectPolicy": {"reportIntervalSeconds": 180}},
         "status": {"updateTime": NOW,
                    "nodeMetric": {"nodeUsage": {"resources": {"cpu": "2", "memory": "4Gi"}},
                                   "systemUsage": {"resources": {"cpu": "2", "memory": "4Gi"}},
                                   "aggregatedNodeUsages": agg}}}
    la = la_args(prod_usage_include_sys=True, estimated_scaling_factors={"cpu": 100, "memory": 100})
    c = cluster.PodAssignCache(la, clock=lambda: NOW)
    c.add_or_update_node_metric(m)
    n = c.get(node)
    assert n.update_time == NOW and n.report_interval == 180
    assert n.node_usage == [2000, 4 * GI] and n.prod_usage == [2000, 4 * GI]
    assert n.agg_usages == {("avg", 0.0): [500, 1 * GI], ("p90", 0.0): [1500, 3 * GI],
                            ("avg", 60.0): [1000, 2 * GI], ("p90", 60.0): [2000, 4 * GI],
                            ("avg", 3600.0): [500, 1 * GI], ("p90", 3600.0): [1500, 3 * GI]}
    _delete_all(c, node, [])


def _delete_all(c, node, pods):
    for p in pods:
        c.on_delete(p)
    c.delete_node_metric(node)
    assert c.get(node) is None  # tryCleanup removed the empty nodeInfo
    n = c.get(node)
    assert n is None  # GetNodeMetricAndEstimatedOfExisting -> NotFound


# ------------------------------------------------------------------------------------------------
# Streams of random events: incremental rows == rows rebuilt from scratch

GPU_RES = ("koordinator.sh/gpu-core", "koordinator.sh/gpu-memory-ratio", "koordinator.sh/gpu-memory")


class World:
    """Objects of a small cluster and a random event stream over them; `reference_table()` rebuilds every
    row from the current objects with decode.node_row (no incremental state)."""

    def __init__(self, cfg, n_nodes, seed):
        self.rng = random.Random(seed)
        self.cfg = cfg
        self.t = NOW
        self.nodes = []
        for i in range(n_nodes):
            ann = {}
            if i % 5 == 0:
                ann["node.koordinator.sh/resource-amplification-ratio"] = json.dumps({"cpu": 1.5})
            self.nodes.append({"metadata": {"name": f"node-{i}", "labels": {}, "annotations": ann},
                               "status": {"allocatable": {"cpu": str(self.rng.choice([32, 64, 96])),
                                                          "memory": f"{self.rng.choice([128, 256])}Gi",
                                                          "pods": "110"}}})
        self.names = [n["metadata"]["name"] for n in self.nodes]
        self.pods = {}      # uid -> pod (current object)
        self.metrics = {}   # node -> NodeMetric
        self.zones = {}     # node -> zones
        self.devices = {}   # node -> Device
        self.seq = 0
        self.state = cluster.ClusterState(cfg, self.nodes, clock=lambda: self.t)

    def _pod(self, node):
        self.seq += 1
        r = self.rng
        req = {"cpu": f"{r.choice([100, 250, 500, 1000, 2000])}m", "memory": f"{r.choice([128, 512, 1024, 4096])}Mi"}
        pod = mk(f"u{self.seq}", "default", f"p{self.seq}", node, "Running", req=req,
                 priority=r.choice([None, 9500, PRIO_MID_DEFAULT]),
                 conditions=[{"type": "PodScheduled", "status": "True",
                              "lastTransitionTime": self.t - r.choice([5, 50, 500])}])
        ann = {}
        if node in self.zones and r.random() < 0.4:
            z = r.randrange(len(self.zones[node]))
            ann[cluster.ANN_RESOURCE_STATUS] = json.dumps(
                {"numaNodeResources": [{"node": z, "resources": {"cpu": req["cpu"], "memory": req["memory"]}}]})
        if node in self.devices and r.random() < 0.5:
            m = r.randrange(4)
            ann[cluster.ANN_DEVICE_ALLOCATED] = json.dumps(
                {"gpu": [{"minor": m, "resources": {GPU_RES[0]: "25", GPU_RES[1]: "25", GPU_RES[2]: "4Gi"}}]})
        if ann:
            pod["metadata"]["annotations"] = ann
        return pod

    def _metric(self, node):
        r = self.rng
        pods = [p for p in self.pods.values() if p["spec"].get("nodeName") == node]
        pm = []
        for p in pods:
            if r.random() < 0.7:
                pm.append({"namespace": "default", "name": p["metadata"]["name"],
                           "priority": r.choice(["koord-prod", "koord-mid"]),
                           "podUsage": {"resources": {"cpu": f"{r.randrange(50, 2500)}m",
                                                      "memory": f"{r.randrange(64, 4096)}Mi"}}})
        return {"metadata": {"name": node},
                "spec": {"collectPolicy": {"reportIntervalSeconds": r.choice([60, 180])}},
                "status": {"updateTime": self.t - r.choice([1, 30, 100]),
                           "nodeMetric": {"nodeUsage": {"resources": {"cpu": f"{r.randrange(1000, 30000)}m",
                                                                      "memory": f"{r.randrange(1, 100)}Gi"}}},
                           "podsMetric": pm}}

    def _device(self, node):
        r = self.rng
        devs = [{"type": "gpu", "minor": m, "health": r.random() > 0.1,
                 "resources": {GPU_RES[0]: "100", GPU_RES[1]: "100", GPU_RES[2]: "80Gi"}} for m in range(4)]
        return {"metadata": {"name": node}, "spec": {"devices": devs}}

    def step(self):
        r = self.rng
        st = self.state
        self.t += r.choice([0.5, 2, 20])
        k = r.random()
        node = r.choice(self.names)
        if k < 0.35 or not self.pods:
            p = self._pod(node)
            self.pods[p["metadata"]["uid"]] = p
            st.on_pod_add(copy.deepcopy(p))
        elif k < 0.5:
            uid = r.choice(sorted(self.pods))
            st.on_pod_delete(copy.deepcopy(self.pods.pop(uid)))
        elif k < 0.62:
            uid = r.choice(sorted(self.pods))
            old = self.pods[uid]
            new = copy.deepcopy(old)
            # nodeName moves only for pods without allocations: the NUMA and DeviceShare handlers release
            # an allocation through the pod's new node (pod_eventhandler.go:95-141, eventhandler_pod.go
            # updatePod), so a moved allocation stays on the old node there as well
            if r.random() < 0.5 or old["metadata"].get("annotations"):
                new["spec"]["containers"][0]["resources"] = {"requests": {"cpu": f"{r.choice([300, 700])}m",
                                                                          "memory": "2Gi"}}
            else:
                new["spec"]["nodeName"] = node
            self.pods[uid] = new
            st.on_pod_update(copy.deepcopy(old), copy.deepcopy(new))
        elif k < 0.8:
            m = self._metric(node)
            self.metrics[node] = m
            st.on_node_metric(copy.deepcopy(m))
        elif k < 0.85 and node in self.metrics:
            del self.metrics[node]
            st.on_node_metric_delete(node)
        elif k < 0.92 and node not in self.zones:
            zones = [{"cpu": "16", "memory": "64Gi"}, {"cpu": "16", "memory": "64Gi"}]
            self.zones[node] = zones
            st.on_topology(node, zones, "")
        elif node not in self.devices:
            d = self._device(node)
            self.devices[node] = d
            st.on_device(copy.deepcopy(d))

    def reference_table(self):
        t = abi.empty_nodes(len(self.nodes))
        t["numa_zone_pods"] = np.zeros(len(self.nodes), np.uint64)  # no cpuset pods in this world
        t["rsv_numa"] = np.zeros(len(self.nodes), np.uint8)  # no reservation holds NUMA resources in this world
        for i, node in enumerate(self.nodes):
            name = self.names[i]
            pods = [p for p in self.pods.values() if p["spec"].get("nodeName") == name]
            zones = self.zones.get(name, [])
            used = [{} for _ in zones]
            for p in pods:
                a = cluster.pod_numa_allocation(p)
                if a is not None:
                    for z, res in a.numa:
                        decode._add(used[z], decode._rl(res))
            ni = decode.NodeInput(node=node, pods=pods, node_metric=self.metrics.get(name),
                                  assigned=[decode.AssignedPod(p, p["status"]["conditions"][0]["lastTransitionTime"])
                                            for p in pods],
                                  numa_zones=zones, numa_used=used)
            row = decode.node_row(ni, self.cfg, now=self.t)
            row["dev_minors"], row["dev_total"], row["dev_free"] = self._device_cols(name, pods)
            for k, v in row.items():
                t[k][i] = v
        return t

    def _device_cols(self, name, pods):
        tot = np.zeros((abi.KG_DEV_R, abi.KG_DEV_MINORS), np.int64)
        free = np.zeros_like(tot)
        d = self.devices.get(name)
        if d is None:
            return -1, tot, free
        for dev in d["spec"]["devices"]:
            if dev["health"]:
                for r, key in enumerate(GPU_RES):
                    tot[r, dev["minor"]] = decode.value(dev["resources"][key])
        free[:] = tot
        used = np.zeros_like(tot)
        for p in pods:
            for a in cluster.pod_device_allocations(p).get("gpu", []):
                for r, key in enumerate(GPU_RES):
                    used[r, a["minor"]] += decode.value(a["resources"][key])
        return 4, tot, np.maximum(tot - used, 0)


def world_cfg():
    return SchedulerConfig(plugins=abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_LA | abi.KG_PLUGIN_NUMA | abi.KG_PLUGIN_DEV,
                           loadaware=LoadAwareArgs(estimated_scaling_factors={"cpu": 80, "memory": 70}))


def tables_equal(a, b, rows=None):
    for k in a:
        x, y = a[k], b[k]
        if rows is not None:
            y = y[rows]
        assert np.array_equal(x, y), k


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_incremental_rows_match_rebuild(seed):
    w = World(world_cfg(), 12, seed)
    synced = 0
    for batch in range(30):
        for _ in range(w.rng.randrange(1, 12)):
            w.step()
        full = w.state.table()
        tables_equal(full, w.reference_table())
        rows = w.state.rows_since(synced)
        synced = w.state.generation
        assert len(rows) <= len(w.nodes)


def test_generations_mark_only_touched_rows():
    w = World(world_cfg(), 8, 5)
    st = w.state
    g0 = st.generation
    assert len(st.rows_since(g0)) == 0
    p = w._pod("node-3")
    st.on_pod_add(p)
    assert list(st.rows_since(g0)) == [3]
    g1 = st.generation
    moved = copy.deepcopy(p)
    moved["spec"]["nodeName"] = "node-5"
    st.on_pod_update(p, moved)
    assert sorted(st.rows_since(g1)) == [3, 5]
    g2 = st.generation
    st.on_node_metric(w._metric("node-1"))
    assert list(st.rows_since(g2)) == [1]


def test_assume_then_bind_counts_once():
    """AssumePod then the binding's Add event: NodeInfo keys pods by UID, podAssignCache renews."""
    w = World(world_cfg(), 4, 9)
    st = w.state
    pod = w._pod("")
    pod["spec"].pop("nodeName", None)
    assumed = st.assume(pod, "node-2")
    once = st.table([2])
    st.on_pod_add(assumed)
    tables_equal(st.table([2]), once)
    st.forget(assumed, "node-2")
    assert st.num_pods[2] == 0 and not st.req[2].any()


# ------------------------------------------------------------------------------------------------
# Device: a snapshot kept current by SnapshotSync selects exactly what the oracle selects on the rebuilt rows

@pytest.fixture(scope="module")
def gpu_ctx():
    from koordinator_amd import engine

    c = engine.Context(0)
    yield c
    c.close()


def _pending(cfg, n, seed, gpu):
    from koordinator_amd import synth

    rng = np.random.default_rng(seed)
    p = synth.pods(n, 1, rng=rng, la_factors=(80, 70))
    if gpu:
        for j in np.nonzero(rng.random(n) < 0.4)[0]:
            req = ({"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100} if rng.random() < 0.5
                   else {"koordinator.sh/gpu-core": 25, "koordinator.sh/gpu-memory-ratio": 25})
            vec, keys, cnt, _ = decode.gpu_requirements(req)
            p["dev_req"][j], p["dev_keys"][j], p["dev_count"][j] = vec, keys, cnt
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("gpu", [False, True], ids=["config2-plugins", "with-deviceshare"])
def test_event_stream_keeps_device_snapshot_exact(gpu_ctx, gpu):
    import oracle_lib
    from koordinator_amd import engine

    cfg = world_cfg()
    if not gpu:
        cfg.plugins = abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_LA | abi.KG_PLUGIN_NUMA
    kc = cfg.kg_config()
    w = World(cfg, 96, 11 if gpu else 7)
    for _ in range(150):  # a populated cluster before the snapshot is taken
        w.step()
    snap = engine.Snapshot(gpu_ctx, kc, w.state.table())
    sync = cluster.SnapshotSync(w.state, snap)
    pods = _pending(cfg, 200, 3, gpu)
    batch = engine.PodBatch(gpu_ctx, pods)
    sel = oracle_lib.ext_select if gpu else oracle_lib.select
    sent = 0
    for cycle in range(25):
        for _ in range(w.rng.randrange(1, 20)):
            w.step()
        if cycle % 5 == 4:  # NUMA policy change: the row changes storage class on the device
            name = w.rng.choice(w.names)
            w.zones[name] = [{"cpu": "32", "memory": "128Gi"}, {"cpu": "32", "memory": "128Gi"}]
            w.state.on_topology(name, w.zones[name], w.rng.choice(["", "SingleNUMANode"]))
        g0 = snap.generation()
        sent += sync.sync()
        assert snap.generation() == g0 + (1 if sync.last_rows else 0)
        full = w.state.table()
        state = snap.read_state()
        for k in state:
            if k == "dev_free" and not gpu:
                continue  # DeviceShare off: the snapshot keeps no GPU tables
            assert np.array_equal(state[k], full[k]), (cycle, k, np.nonzero(state[k] != full[k])[0][:5])
        got = engine.eval_select(snap, batch, 3)
        want = sel(kc, full, pods, 3)
        if not np.array_equal(got, want):
            fresh = engine.eval_select(engine.Snapshot(gpu_ctx, kc, full), batch, 3)
            bad = np.nonzero(np.any(got != want, axis=1))[0]
            raise AssertionError(f"cycle {cycle}: {len(bad)} pods differ (first {bad[:4]}); a fresh upload of the "
                                 f"same rows {'matches' if np.array_equal(fresh, want) else 'differs too'}; "
                                 f"got {got[bad[0]]} want {want[bad[0]]}")
    assert 0 < sent < 25 * len(w.nodes)  # deltas, not whole uploads


@pytest.mark.gpu
def test_assume_on_device_then_events_agree(gpu_ctx):
    """kg_assume applies a placement on the device; the host's assume + the binding's Add event then
    rebuild the same row, so the sync that follows leaves the device row unchanged."""
    from koordinator_amd import engine

    cfg = world_cfg()
    cfg.plugins = abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_LA | abi.KG_PLUGIN_NUMA
    kc = cfg.kg_config()
    w = World(cfg, 32, 21)
    for _ in range(80):
        w.step()
    w.state.tick()  # expiries up to now are in the rows the snapshot starts from
    snap = engine.Snapshot(gpu_ctx, kc, w.state.table())
    sync = cluster.SnapshotSync(w.state, snap)
    pod = w._pod("")
    pod["spec"].pop("nodeName", None)
    pod["metadata"].pop("annotations", None)
    ptab = decode.pods_table([pod], cfg)
    batch = engine.PodBatch(gpu_ctx, ptab)
    node = 5
    engine.assume(snap, batch, 0, node)
    on_device = snap.read_state()
    bound = w.state.assume(pod, w.names[node])
    w.state.on_pod_add(bound)
    assert sync.sync() == 1
    after = snap.read_state()
    for k in after:
        assert np.array_equal(after[k], on_device[k]), k


def test_metric_expiry_is_a_time_event():
    """isNodeMetricExpired depends on the clock: tick() marks the row once its deadline passes."""
    w = World(world_cfg(), 4, 13)
    st = w.state
    m = w._metric("node-2")
    st.on_node_metric(m)
    secs = st.la.node_metric_expiration_seconds
    ut = m["status"]["updateTime"]
    g = st.generation
    before = st.table([2])["la_flags"][0]
    assert not before & abi.KG_LA_EXPIRED
    w.t = ut + secs - 1
    st.tick()
    assert len(st.rows_since(g)) == 0
    w.t = ut + secs
    st.tick()
    assert list(st.rows_since(g)) == [2]
    assert st.table([2])["la_flags"][0] & abi.KG_LA_EXPIRED
