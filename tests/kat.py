"""Expansion of the transcribed known-answer fixtures (tests/golden/*.json) into objects and columns.

The expansion mirrors how the reference's test runners build their fixtures, e.g.
load_aware_test.go:1362-1473 (TestFilterUsage runner) and :2398-2489 (TestScore runner).
"""
from __future__ import annotations

import json
import os

from koordinator_amd import abi, decode, reasons
from koordinator_amd.config import AggregatedArgs, LoadAwareArgs, SchedulerConfig

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def make_pod(spec, node_name=""):
    """st.MakePod()-style compact pod -> Kubernetes-shaped dict."""
    if spec is None:
        return {"metadata": {}, "spec": {}}
    md = {"namespace": spec.get("namespace", ""), "name": spec.get("name", "")}
    if spec.get("labels"):
        md["labels"] = dict(spec["labels"])
    if spec.get("annotations"):
        md["annotations"] = dict(spec["annotations"])
    if spec.get("owner_kinds"):
        md["ownerReferences"] = [{"kind": k, "name": "owner"} for k in spec["owner_kinds"]]
    pspec = {"containers": [{"name": f"c{i}", "resources": {k: v for k, v in c.items() if k in ("requests", "limits")}}
                            for i, c in enumerate(spec.get("containers", []))]}
    if spec.get("init_containers"):
        pspec["initContainers"] = [
            {"name": f"i{i}", "resources": {k: v for k, v in c.items() if k in ("requests", "limits")},
             **({"restartPolicy": c["restartPolicy"]} if c.get("restartPolicy") else {})}
            for i, c in enumerate(spec["init_containers"])]
    if "priority" in spec:
        pspec["priority"] = spec["priority"]
    if spec.get("overhead"):
        pspec["overhead"] = spec["overhead"]
    if node_name:
        pspec["nodeName"] = node_name
    return {"metadata": md, "spec": pspec, "status": {}}


def make_node_metric(nm):
    if nm is None:
        return None
    status = {"updateTime": nm.get("update_time")}
    if "node_usage" in nm:
        info = {"nodeUsage": {"resources": nm["node_usage"]}}
        if nm.get("aggregated"):
            info["aggregatedNodeUsages"] = [
                {"duration": a["duration"], "usage": {t: {"resources": r} for t, r in a["usage"].items()}}
                for a in nm["aggregated"]]
        status["nodeMetric"] = info
    else:
        status["nodeMetric"] = None
    if nm.get("pods"):
        status["podsMetric"] = [{"namespace": p["namespace"], "name": p["name"], "priority": p.get("priority", ""),
                                 "podUsage": {"resources": p["usage"]}} for p in nm["pods"]]
    return {"spec": {"collectPolicy": {"reportIntervalSeconds": nm.get("report_interval", 60)}}, "status": status}


def la_args(a: dict) -> LoadAwareArgs:
    agg = None
    if a.get("aggregated"):
        g = a["aggregated"]
        agg = AggregatedArgs(usage_thresholds=g.get("usage_thresholds", {}),
                             usage_aggregation_type=g.get("usage_aggregation_type", ""),
                             usage_aggregated_duration=decode._duration(g.get("usage_aggregated_duration")),
                             score_aggregation_type=g.get("score_aggregation_type", ""),
                             score_aggregated_duration=decode._duration(g.get("score_aggregated_duration")))
    return LoadAwareArgs(
        filter_expired_node_metrics=a.get("filter_expired_node_metrics"),
        enable_schedule_when_node_metrics_expired=a.get("enable_schedule_when_node_metrics_expired"),
        usage_thresholds=a.get("usage_thresholds", {}),
        prod_usage_thresholds=a.get("prod_usage_thresholds", {}),
        dominant_resource_weight=a.get("dominant_resource_weight", 0),
        score_according_prod_usage=a.get("score_according_prod_usage", False),
        aggregated=agg)


def la_case(case, default_node):
    """(SchedulerConfig, nodes table, pods table) for one LoadAware known-answer case."""
    cfg = SchedulerConfig(plugins=abi.KG_PLUGIN_LA, loadaware=la_args(case.get("args", {})))
    node_spec = case.get("node", default_node)
    node = {"metadata": {"name": "test-node-1", "annotations": {}}, "status": {"allocatable": node_spec["allocatable"]}}
    if case.get("custom_thresholds"):
        node["metadata"]["annotations"][decode.ANN_CUSTOM_USAGE_THRESHOLDS] = json.dumps(case["custom_thresholds"])
    if case["kind"] == "filter":
        # TestFilterUsage pods carry a PodScheduled condition 10s in the past (load_aware_test.go:1399-1404)
        assigned = [decode.AssignedPod(make_pod(p, "test-node-1"), -10.0) for p in case.get("pods", [])]
    else:
        # TestScore pods have no PodScheduled condition: the cache stamps them at assign time, after
        # the NodeMetric's UpdateTime (pod_assign_cache.go:302-308)
        assigned = [decode.AssignedPod(make_pod(a["pod"], "test-node-1"), float(a.get("timestamp", 1)))
                    for a in case.get("assigned", [])]
    ni = decode.NodeInput(node=node, pods=[a.pod for a in assigned], node_metric=make_node_metric(case.get("node_metric")),
                          assigned=assigned)
    nodes = decode.nodes_table([ni], cfg)
    pods = decode.pods_table([make_pod(case.get("test_pod"))], cfg)
    return cfg, nodes, pods


def la_status(bits: int):
    """KG_ST_* bits of the LoadAware plugin -> (code, reason) of the Go Status."""
    return reasons.loadaware_status(bits)
