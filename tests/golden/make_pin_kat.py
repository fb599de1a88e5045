"""Writes tests/golden/pin_kat.json: known answers transcribed by hand from the reference's Go tests that
pin the NodeResourcesFit, amplified-CPU NodeNUMAResource, Reservation fit and DeviceShare fit / score
arithmetic. Values and expected results are copied from
the cited test tables; the builders in tests/pin_kat.py restate each test runner's fixture set-up (cited
there). No reference source is executed or embedded.

Units: cpu in cores unless a key ends in _m (milli-cores); memory / ephemeral storage in Gi unless a key
ends in _b (bytes); GPU core / memory-ratio in percent of a card, GPU memory in Gi.
"""
import json
import os

cases = {
    # frameworkext/job_nominated_pods_test.go:65-305 — upstream noderesources.Fits (FakeFitPlugin, :47-59)
    # on a node with 16 cpu / 110 pods; the nominated pods that are not removed count in the NodeInfo.
    "nrf_fits": [
        {"name": "insufficient resource cause nominated pod", "ref": "frameworkext/job_nominated_pods_test.go:75",
         "node": {"cpu": 16, "pods": 110}, "existing_cpu": [16], "pod_cpu": 16, "want": ["Insufficient cpu"]},
        {"name": "ignore nominated pod", "ref": "frameworkext/job_nominated_pods_test.go:130",
         "node": {"cpu": 16, "pods": 110}, "existing_cpu": [], "pod_cpu": 16, "want": []},
        {"name": "insufficient resource though ignore nominated pod",
         "ref": "frameworkext/job_nominated_pods_test.go:186",
         "node": {"cpu": 16, "pods": 110}, "existing_cpu": [16], "pod_cpu": 16, "want": ["Insufficient cpu"]},
    ],
    # reservation/plugin_test.go:6736-6853 TestFitsNodeWithIgnoredResources: fitsNode (the in-tree mirror
    # of upstream Fits) with ignored extended resources; scalar slot 0 = example.com/gpu, 1 = other.io/fpga.
    # fitsNode(podRequest, nodeAlloc, allPodsRequested, nil, nil, matched=0, allocatedPods=1, nil, ...).
    "fits_ignored": [
        {"name": "extended resource insufficient but ignored by name", "ref": "reservation/plugin_test.go:6747",
         "pod": {"cpu": 1, "sc0": 2}, "alloc": {"cpu": 8, "mem": 16, "pods": 100, "sc0": 1}, "requested": {"cpu": 4},
         "ignored": ["example.com/gpu"], "ignored_groups": [], "want": []},
        {"name": "extended resource insufficient but ignored by group", "ref": "reservation/plugin_test.go:6766",
         "pod": {"cpu": 1, "sc0": 2}, "alloc": {"cpu": 8, "mem": 16, "pods": 100, "sc0": 1}, "requested": {"cpu": 4},
         "ignored": [], "ignored_groups": ["example.com"], "want": []},
        {"name": "extended resource insufficient and not ignored", "ref": "reservation/plugin_test.go:6785",
         "pod": {"cpu": 1, "sc0": 2}, "alloc": {"cpu": 8, "mem": 16, "pods": 100, "sc0": 1}, "requested": {"cpu": 4},
         "ignored": [], "ignored_groups": [], "want": ["example.com/gpu"]},
        {"name": "only matching group is ignored, other extended resources still checked",
         "ref": "reservation/plugin_test.go:6804",
         "pod": {"cpu": 1, "sc0": 2, "sc1": 2}, "alloc": {"cpu": 8, "mem": 16, "pods": 100, "sc0": 1, "sc1": 1},
         "requested": {"cpu": 4}, "ignored": [], "ignored_groups": ["example.com"], "want": ["other.io/fpga"]},
        {"name": "native cpu unconditionally reported even when extended is ignored",
         "ref": "reservation/plugin_test.go:6825",
         "pod": {"cpu": 8, "sc0": 2}, "alloc": {"cpu": 4, "mem": 16, "pods": 100, "sc0": 1}, "requested": {"cpu": 0},
         "ignored": ["example.com/gpu"], "ignored_groups": [], "want": ["cpu"]},
    ],
    # noderesourcefitplus/node_resources_fit_plus_test.go:124-318 TestPlugin_Score: cpu / memory
    # LeastAllocated weight 1, nvidia.com/gpu MostAllocated weight 2 (:126-130); testNode1 holds a
    # 16 cpu / 32Gi / 4 gpu pod; the reference asserts scoreNode1 > scoreNode2 (:314-316). want_scores are
    # resourceScorer (node_resource_fit_plus_utils.go:58-86) evaluated by hand on these inputs.
    "nrfp_score": [
        {"name": "TestPlugin_Score", "ref": "noderesourcefitplus/node_resources_fit_plus_test.go:124-318",
         "nodes": [{"cpu": 96, "mem": 512, "gpu": 8, "eph": 100, "existing": {"cpu": 16, "mem": 32, "gpu": 4}},
                   {"cpu": 96, "mem": 512, "gpu": 8, "eph": 100, "existing": None}],
         "pod": {"cpu": 16, "mem": 32, "gpu": 2, "eph": 10},
         "resources": [["cpu", 1, "LeastAllocated"], ["memory", 1, "LeastAllocated"], ["nvidia.com/gpu", 2, "MostAllocated"]],
         "want": "node0 > node1", "want_scores": [75, 56]},
    ],
    # nodenumaresource/plugin_test.go:1139-1233 TestFilterWithAmplifiedCPUs: node-1 with cpu = NumCPUs of
    # buildCPUTopologyForTest(2, 1, 8, 2) = 32 cores and 40Gi, allocatable cpu amplified by the ratio
    # (makeNode, :142-148); cpuset pods are LSR prod pods whose CPUSet is 0..n-1 (makePodOnNode, :150-163);
    # the resource manager counts a node's cpuset allocation when the node has topology options (NRT).
    "numa_amp_filter": [
        {"name": "no resources requested always fits", "ref": "nodenumaresource/plugin_test.go:1150",
         "ratio": 2.0, "nrt": False, "existing": [{"cpu": 4, "cpuset": False}], "pod": None, "want": []},
        {"name": "no filtering without node cpu amplification", "ref": "nodenumaresource/plugin_test.go:1157",
         "ratio": 1.0, "nrt": False, "existing": [{"cpu": 32, "cpuset": False}], "pod": {"cpu": 32, "cpuset": False},
         "want": []},
        {"name": "cpu fits on no NRT node", "ref": "nodenumaresource/plugin_test.go:1164",
         "ratio": 2.0, "nrt": False, "existing": [{"cpu": 32, "cpuset": False}], "pod": {"cpu": 32, "cpuset": False},
         "want": []},
        {"name": "insufficient cpu", "ref": "nodenumaresource/plugin_test.go:1171",
         "ratio": 2.0, "nrt": False, "existing": [{"cpu": 64, "cpuset": False}], "pod": {"cpu": 32, "cpuset": False},
         "want": ["Insufficient amplified cpu"]},
        {"name": "insufficient cpu with cpuset pod on node", "ref": "nodenumaresource/plugin_test.go:1179",
         "ratio": 2.0, "nrt": True, "existing": [{"cpu": 32, "cpuset": True}], "pod": {"cpu": 32, "cpuset": False},
         "want": ["Insufficient amplified cpu"]},
        {"name": "insufficient cpu when scheduling cpuset pod", "ref": "nodenumaresource/plugin_test.go:1188",
         "ratio": 2.0, "nrt": True, "existing": [{"cpu": 32, "cpuset": False}], "pod": {"cpu": 32, "cpuset": True},
         "want": ["Insufficient amplified cpu"]},
        {"name": "insufficient cpu when scheduling cpuset pod with cpuset pod on node",
         "ref": "nodenumaresource/plugin_test.go:1197",
         "ratio": 2.0, "nrt": True, "existing": [{"cpu": 32, "cpuset": True}], "pod": {"cpu": 32, "cpuset": True},
         "want": ["Insufficient amplified cpu"]},
    ],
    # nodenumaresource/scoring_test.go:726-1008 TestScoreWithAmplifiedCPUs (default resources cpu 1,
    # memory 1); the nodes in nodeHasNRT carry the CPU topology buildCPUTopologyForTest(2, 1, 8, 2) (32 CPUs).
    # A cpuset-binding pod's request is amplified in its Score (getResourceOptions, plugin.go:772-778).
    "numa_amp_score": [
        {"name": "ScoringStrategy MostAllocated, non-cpuset pod", "ref": "nodenumaresource/scoring_test.go:739",
         "strategy": "MostAllocated", "nodes": [[32, 40, 1.0], [64, 60, 2.0], [32, 40, 2.0]], "nrt": [],
         "existing": [], "pod": {"cpu": 8, "mem": 16, "cpuset": False}, "want": [32, 16, 26]},
        {"name": "ScoringStrategy MostAllocated, cpuset pod", "ref": "nodenumaresource/scoring_test.go:756",
         "strategy": "MostAllocated", "nodes": [[32, 40, 1.0], [64, 60, 2.0], [32, 40, 2.0]],
         "nrt": ["node1", "node2", "node3"], "existing": [], "pod": {"cpu": 8, "mem": 16, "cpuset": True},
         "want": [32, 19, 32]},
        {"name": "ScoringStrategy MostAllocated, non-cpuset pods, and existing cpuset pod on node",
         "ref": "nodenumaresource/scoring_test.go:779",
         "strategy": "MostAllocated", "nodes": [[32, 40, 1.0], [64, 60, 2.0]], "nrt": ["node1", "node2"],
         "existing": [["node1", 20, 4, True], ["node2", 20, 4, True]], "pod": {"cpu": 8, "mem": 16, "cpuset": False},
         "want": [68, 35]},
        {"name": "ScoringStrategy MostAllocated, scheduling cpuset pod with existing non-cpuset pods",
         "ref": "nodenumaresource/scoring_test.go:804",
         "strategy": "MostAllocated", "nodes": [[32, 40, 1.0], [64, 60, 2.0]], "nrt": ["node1", "node2"],
         "existing": [["node1", 20, 4, False], ["node2", 20, 4, False]], "pod": {"cpu": 8, "mem": 16, "cpuset": True},
         "want": [68, 30]},
        {"name": "ScoringStrategy MostAllocated, cpuset pods on node, scheduling cpuset pod",
         "ref": "nodenumaresource/scoring_test.go:829",
         "strategy": "MostAllocated", "nodes": [[32, 40, 1.0], [64, 60, 2.0]], "nrt": ["node1", "node2"],
         "existing": [["node1", 20, 4, True], ["node2", 20, 4, True]], "pod": {"cpu": 8, "mem": 16, "cpuset": True},
         "want": [68, 38]},
        {"name": "ScoringStrategy LeastAllocated, no cpuset pod", "ref": "nodenumaresource/scoring_test.go:854",
         "strategy": "LeastAllocated", "nodes": [[32, 40, 1.0], [64, 60, 2.0]], "nrt": [],
         "existing": [["node1", 20, 4, False], ["node2", 20, 4, False]], "pod": {"cpu": 8, "mem": 16, "cpuset": False},
         "want": [31, 72]},
        {"name": "ScoringStrategy LeastAllocated, non-cpuset pod with existing cpuset pods",
         "ref": "nodenumaresource/scoring_test.go:874",
         "strategy": "LeastAllocated", "nodes": [[32, 40, 1.0], [64, 60, 2.0]], "nrt": ["node1", "node2"],
         "existing": [["node1", 20, 4, True], ["node2", 20, 4, True]], "pod": {"cpu": 8, "mem": 16, "cpuset": False},
         "want": [31, 64]},
        {"name": "ScoringStrategy LeastAllocated, scheduling cpuset pod with existing non-cpuset pods",
         "ref": "nodenumaresource/scoring_test.go:899",
         "strategy": "LeastAllocated", "nodes": [[32, 40, 1.0], [64, 60, 2.0]], "nrt": ["node1", "node2"],
         "existing": [["node1", 20, 4, False], ["node2", 20, 4, False]], "pod": {"cpu": 8, "mem": 16, "cpuset": True},
         "want": [31, 68]},
        {"name": "ScoringStrategy LeastAllocated, cpuset pods on node,scheduling cpuset pod",
         "ref": "nodenumaresource/scoring_test.go:924",
         "strategy": "LeastAllocated", "nodes": [[32, 40, 1.0], [64, 60, 2.0]], "nrt": ["node1", "node2"],
         "existing": [["node1", 20, 4, True], ["node2", 20, 4, True]], "pod": {"cpu": 8, "mem": 16, "cpuset": True},
         "want": [31, 61]},
    ],
    # reservation/plugin_test.go:1090-2546 Test_filterWithReservations: test-node allocatable cpu 32,
    # memory 32Gi, pods 100, batch-cpu 7500, batch-memory 10Gi (:1162-1174), no pods in the NodeInfo
    # (:2536-2537); one matched reservation per case. Reservation allocatable comes from its template
    # (ReservationRequests) or Status.Allocatable, Reserved from the node-reservation annotation, Allocated
    # from its assigned pods (frameworkext/reservation_info.go:92-132,490-500). The preemption cases
    # (preemptible / preemptibleInRRs) are not on the device path and are not transcribed.
    "rsv_filter": [
        {"name": "filter aligned reservation with nodeInfo", "ref": "reservation/plugin_test.go:1182",
         "affinity": True, "pod": {"cpu": 8, "mem": 8}, "pod_requested": {"cpu": 30, "mem": 24}, "r_allocated": {},
         "rsv": {"policy": "Aligned", "allocatable": {"cpu": 6}}, "want": []},
        {"name": "failed to filter aligned reservation with nodeInfo", "ref": "reservation/plugin_test.go:1229",
         "affinity": True, "pod": {"cpu": 8, "mem": 8}, "pod_requested": {"cpu": 32, "mem": 24}, "r_allocated": {},
         "rsv": {"policy": "Aligned", "allocatable": {"cpu": 6}}, "want": ["Insufficient cpu by node"]},
        {"name": "filter restricted reservation with nodeInfo", "ref": "reservation/plugin_test.go:1276",
         "affinity": False, "pod": {"cpu": 6, "mem": 8}, "pod_requested": {"cpu": 30, "mem": 24}, "r_allocated": {},
         "rsv": {"policy": "Restricted", "allocatable": {"cpu": 6}}, "want": []},
        {"name": "filter restricted reservation with affinity", "ref": "reservation/plugin_test.go:1322",
         "affinity": True, "pod": {"cpu": 6, "mem": 8}, "pod_requested": {"cpu": 30, "mem": 24}, "r_allocated": {},
         "rsv": {"policy": "Restricted", "allocatable": {"cpu": 6}}, "want": []},
        {"name": "filter restricted reservation with nodeInfo and matched requests are zero",
         "ref": "reservation/plugin_test.go:1369",
         "affinity": True, "pod": {"bcpu_m": 6000, "bmem": 8},
         "pod_requested": {"cpu": 30, "mem": 24, "bcpu_m": 1500, "bmem": 2}, "r_allocated": {"cpu_m": 6000},
         "rsv": {"policy": "Restricted", "allocatable": {"cpu": 6}}, "want": []},
        {"name": "failed to filter restricted reservation with nodeInfo", "ref": "reservation/plugin_test.go:1420",
         "affinity": True, "pod": {"cpu": 8, "mem": 8}, "pod_requested": {"cpu": 30, "mem": 24}, "r_allocated": {},
         "rsv": {"policy": "Restricted", "allocatable": {"cpu": 6}}, "want": ["Reservation(s) Insufficient cpu"]},
        {"name": "failed to filter restricted reservation since exceeding max pods",
         "ref": "reservation/plugin_test.go:1467 (testRInfo :1091-1160)",
         "affinity": True, "pod": {"cpu": 3}, "pod_requested": {"cpu": 30, "mem": 24}, "r_allocated": {"cpu_m": 2000},
         "rsv": {"policy": "Restricted", "allocatable": {"cpu": 7, "pods": 2}, "reserved": {"cpu": 1},
                 "assigned_cpu": [1, 1]},
         "want": ["Reservation(s) Too many pods"]},
        {"name": "failed to filter restricted reservation since unmatched resources are insufficient",
         "ref": "reservation/plugin_test.go:1493",
         "affinity": True, "pod": {"bcpu_m": 8000, "bmem": 8},
         "pod_requested": {"cpu": 30, "mem": 24, "bcpu_m": 1500, "bmem": 2}, "r_allocated": {"cpu_m": 2000},
         "rsv": {"policy": "Restricted", "allocatable": {"cpu": 6}},
         "want": ["Insufficient kubernetes.io/batch-cpu by node"]},
        {"name": "filter restricted reservation and ignore matched requests are zero without affinity",
         "ref": "reservation/plugin_test.go:1545",
         "affinity": False, "pod": {"bcpu_m": 8000, "bmem": 8},
         "pod_requested": {"cpu": 30, "mem": 24, "bcpu_m": 1500, "bmem": 2}, "r_allocated": {"cpu_m": 6000},
         "rsv": {"policy": "Restricted", "allocatable": {"cpu": 6}},
         "want": ["Insufficient kubernetes.io/batch-cpu by node"]},
        {"name": "failed to filter restricted reservation due to reserved", "ref": "reservation/plugin_test.go:1597",
         "affinity": True, "pod": {"cpu": 6, "mem": 8}, "pod_requested": {"cpu": 30, "mem": 24}, "r_allocated": {},
         "rsv": {"policy": "Restricted", "allocatable": {"cpu": 6}, "reserved": {"cpu": 2}},
         "want": ["Reservation(s) Insufficient cpu"]},
    ],
    # deviceshare/plugin_test.go:1138-3221 Test_Plugin_Filter, the GPU-only cases (FPGA / RDMA / NPU
    # resources, designated allocation and hami cases are not on the device path); test-node's Device has
    # the listed healthy GPU minors.
    "dev_filter": [
        {"name": "insufficient device resource 1", "ref": "deviceshare/plugin_test.go:1208",
         "minors": [], "pod": {"gpu-core": 100, "gpu-memory-ratio": 100}, "want": "KG_ST_DEV_NO_DEVICE"},
        {"name": "insufficient device resource 2", "ref": "deviceshare/plugin_test.go:1227",
         "minors": [{"total": [100, 100, 16], "free": [75, 75, 12]}], "pod": {"gpu-core": 100, "gpu-memory-ratio": 100},
         "want": "KG_ST_DEV_INSUFFICIENT"},
        {"name": "sufficient device resource 3", "ref": "deviceshare/plugin_test.go:1738",
         "minors": [{"total": [100, 100, 16], "free": [100, 100, 16]}], "pod": {"gpu-core": 100, "gpu-memory-ratio": 100},
         "want": 0},
        {"name": "sufficient device resource 4", "ref": "deviceshare/plugin_test.go:1815",
         "minors": [{"total": [100, 100, 16], "free": [25, 25, 4]}, {"total": [100, 100, 16], "free": [100, 100, 16]}],
         "pod": {"gpu-core": 100, "gpu-memory-ratio": 100}, "want": 0},
        {"name": "sufficient device resource 5", "ref": "deviceshare/plugin_test.go:1900",
         "minors": [{"total": [100, 100, 16], "free": [25, 25, 4]}, {"total": [100, 100, 16], "free": [100, 100, 16]}],
         "pod": {"gpu-memory-ratio": 100}, "want": 0},
    ],
    # deviceshare/scoring_test.go:1255-1335 Test_resourceAllocationScorer_scoreDevice (default weights
    # gpu-memory-ratio 1, gpu-memory 1): one minor with only gpu-memory-ratio; the device scores the node
    # as the sum over its minors, which for one minor is scoreDevice. A fully used minor fails the device
    # Filter first (its score is never taken; the reference's 0 is the verify row's 0).
    "dev_score_device": [
        {"name": "completely idle", "ref": "deviceshare/scoring_test.go:1265",
         "req": 50, "total": 100, "free": 100, "strategy": "LeastAllocated", "want": 50},
        {"name": "completely used", "ref": "deviceshare/scoring_test.go:1278",
         "req": 50, "total": 100, "free": 0, "strategy": "LeastAllocated", "want": 0, "infeasible": True},
        {"name": "remaining resources", "ref": "deviceshare/scoring_test.go:1291",
         "req": 30, "total": 100, "free": 50, "strategy": "LeastAllocated", "want": 20},
        {"name": "remaining resources with MostAllocated", "ref": "deviceshare/scoring_test.go:1304",
         "req": 30, "total": 100, "free": 50, "strategy": "MostAllocated", "want": 80},
    ],
    # deviceshare/scoring_test.go:275-366 TestScore with the MostAllocated strategy (same node as
    # "remaining device resources 1 / 2": one 100 / 100 / 16Gi minor with 75 / 75 / 12Gi free).
    "dev_score_most": [
        {"name": "remaining device resources with MostAllocated strategy 1", "ref": "deviceshare/scoring_test.go:275",
         "minors": [{"total": [100, 100, 16], "free": [75, 75, 12]}], "pod": {"gpu-core": 50, "gpu-memory-ratio": 50},
         "want": 50},
        {"name": "remaining device resources with MostAllocated strategy 2", "ref": "deviceshare/scoring_test.go:321",
         "minors": [{"total": [100, 100, 16], "free": [75, 75, 12]}], "pod": {"gpu-core": 50, "gpu-memory": 8},
         "want": 50},
    ],
    # deviceshare/scoring_test.go:602-667 TestScoreExtension (DefaultNormalizeScore over the feasible
    # nodes): the raw node score comes from one minor with only gpu-memory-ratio (scoreDevice as above,
    # requested = total - free + request), so raw 10 = total 100, free 30, request 20 and raw 0 = free 20,
    # request 20. The two-node case with a raw 200 (above MaxNodeScore) has no device-path input.
    "dev_normalize": [
        {"name": "node score 0", "ref": "deviceshare/scoring_test.go:609", "raw": [[20, 20]], "want": [0]},
        {"name": "only one node has score", "ref": "deviceshare/scoring_test.go:624", "raw": [[30, 20]],
         "want": [100]},
    ],
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pin_kat.json")
    with open(out, "w") as f:
        json.dump(cases, f, indent=1)
    print(out, sum(len(v) for v in cases.values()), "cases")
