"""Writes tests/golden/ext_kat.json: known-answer cases for the config-5 plugins, transcribed by hand
from the reference's own Go tests (values and expected results copied from the cited test tables;
no reference source is executed or embedded). Units: cpu in milli-cores, memory in bytes."""
import json
import os

GI = 1 << 30
MINOR_16G = [100, 100, 16 * GI]  # gpuResources, deviceshare/scoring_test.go:48-52

cases = {
    # deviceshare/scoring_test.go:41-600 TestScore (LeastAllocated default strategy: gpu-memory-ratio 1,
    # gpu-memory 1); pod requests are the raw GPU requests (calcDesiredRequestsAndCountForGPU path)
    "deviceshare_score": [
        {"name": "no device resources", "ref": "deviceshare/scoring_test.go:97-115",
         "minors": [], "pod": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100},
         "want": {"status": "KG_ST_DEV_NO_DEVICE"}},
        {"name": "completely idle node", "ref": "deviceshare/scoring_test.go:116-143",
         "minors": [{"total": MINOR_16G, "free": MINOR_16G}],
         "pod": {"koordinator.sh/gpu-core": 100, "koordinator.sh/gpu-memory-ratio": 100},
         "want": {"score": 50}},
        {"name": "multiple GPU devices and completely idle", "ref": "deviceshare/scoring_test.go:144-180",
         "minors": [{"total": MINOR_16G, "free": MINOR_16G}, {"total": MINOR_16G, "free": MINOR_16G}],
         "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50},
         "want": {"score": 87}},
        {"name": "remaining device resources 1", "ref": "deviceshare/scoring_test.go:181-227",
         "minors": [{"total": MINOR_16G, "free": [75, 75, 12 * GI]}],
         "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50},
         "want": {"score": 50}},
        {"name": "remaining device resources 2", "ref": "deviceshare/scoring_test.go:228-274",
         "minors": [{"total": MINOR_16G, "free": [75, 75, 12 * GI]}],
         "pod": {"koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory": 8 * GI},
         "want": {"score": 50}},
    ],
    # reservation/scoring_test.go:42-289 TestScore: node 16 cpu / 128Gi, no pods; Score after PreScore
    # (nominated reservation -> ScoreReservation, MostAllocated over the reservation's allocatable)
    "reservation_score": [
        {"name": "no reservation matched on the node", "ref": "reservation/scoring_test.go:137-141",
         "node": [16000, 128 * GI], "reservations": [], "pod": [2000, 4 * GI], "want": [0]},
        {"name": "reservation matched but zero-request pod", "ref": "reservation/scoring_test.go:142-150",
         "node": [16000, 128 * GI], "reservations": [{"allocatable": [2000, 4 * GI]}], "pod": None, "want": [0]},
        {"name": "reservation matched and pod has part empty resource requests",
         "ref": "reservation/scoring_test.go:151-174",
         "node": [16000, 128 * GI], "reservations": [{"allocatable": [4000, 8 * GI]}], "pod": [2000, 4 * GI],
         "want": [50]},
        {"name": "allocated reservation matched and pod has part empty resource requests",
         "ref": "reservation/scoring_test.go:175-204",
         "node": [16000, 128 * GI], "reservations": [{"allocatable": [2000, 4 * GI], "allocated": [2000, 3 * GI]}],
         "pod": [2000, 4 * GI], "want": [0]},
        {"name": "multi reservations matched and pod has part empty resource requests",
         "ref": "reservation/scoring_test.go:205-230",
         "node": [16000, 128 * GI],
         "reservations": [{"allocatable": [4000, 8 * GI]}, {"allocatable": [2000, 4 * GI]}],
         "pod": [2000, 4 * GI], "want": [100]},
    ],
    # reservation/scoring_test.go:291-474 TestScoreWithOrder: 4 nodes without allocatable, one 4C8G
    # reservation each, the 4th labelled with an order: raw Score and NormalizeScore'd values
    "reservation_order": [
        {"name": "preferred node by reservation order", "ref": "reservation/scoring_test.go:291-474",
         "nodes": 4, "allocatable": [4000, 8 * GI], "orders": [0, 0, 0, 123456], "pod": [4000, 8 * GI],
         "want_score": [100, 100, 100, 1000], "want_normalized": [10, 10, 10, 100]},
    ],
    # elasticquota/plugin_test.go:712-806 TestPlugin_PreFilter (pod requests masked to cpu + memory;
    # used empty; usedLimit = runtime, or the default quota's max when runtime quota is disabled)
    "elasticquota_prefilter": [
        {"name": "default", "ref": "elasticquota/plugin_test.go:721-735",
         "limit": [0, 20], "pod": [1, 2], "want_pass": False},
        {"name": "used dimension larger than runtime, but value is enough", "ref": "elasticquota/plugin_test.go:736-747",
         "limit": [10, 20], "pod": [1, 2], "want_pass": True},
        {"name": "value not enough", "ref": "elasticquota/plugin_test.go:748-764",
         "limit": [1, 2], "pod": [1, 3], "want_pass": False},
        {"name": "runtime not enough, but disable runtime", "ref": "elasticquota/plugin_test.go:777-789",
         "limit": [1 << 40, 1 << 40], "pod": [1, 3], "want_pass": True},
    ],
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ext_kat.json")
    with open(out, "w") as f:
        json.dump(cases, f, indent=1)
    print("wrote", out)
