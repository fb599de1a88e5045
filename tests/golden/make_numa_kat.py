"""Writes tests/golden/numa_kat.json: NodeNUMAResource known answers transcribed by hand from the
reference's Go tests (NUMA policies SingleNUMANode / Restricted, hint and score strategies). Nodes have
`zones` equal NUMA zones (allocatable / zones each); `used[z]` lists the (cpu cores, memory Gi) of the
pods allocated on zone z; pods without a pod-level NUMA policy."""
import json
import os

cases = {
    # nodenumaresource/plugin_test.go:2614-2835 TestFilterWithNUMANodeScoring: the affinity stored by
    # Filter (NUMAScoringStrategy = hint scoring)
    "affinity": [
        {"name": "single numa nodes and select most allocated", "ref": "nodenumaresource/plugin_test.go:2651-2671",
         "node": [104, 256], "policy": "SINGLE_NODE", "zones": 2, "used": {"0": [[4, 8]], "1": [[40, 8]]},
         "pod": [4, 40], "hint": "MostAllocated", "want_zone": 1},
        {"name": "single numa nodes and select least allocated", "ref": "nodenumaresource/plugin_test.go:2673-2693",
         "node": [104, 256], "policy": "SINGLE_NODE", "zones": 2, "used": {"0": [[4, 8]], "1": [[40, 8]]},
         "pod": [4, 40], "hint": "LeastAllocated", "want_zone": 0},
        {"name": "single numa nodes and only one node can be used", "ref": "nodenumaresource/plugin_test.go:2695-2715",
         "node": [104, 256], "policy": "SINGLE_NODE", "zones": 2, "used": {"0": [[4, 8]], "1": [[52, 8]]},
         "pod": [4, 40], "hint": "LeastAllocated", "want_zone": 0},
        {"name": "restricted numa nodes and select most allocated and preferred",
         "ref": "nodenumaresource/plugin_test.go:2717-2743",
         "node": [104, 256], "policy": "RESTRICTED", "zones": 4,
         "used": {"0": [[24, 8]], "1": [[23, 8]], "2": [[4, 8]], "3": [[8, 8]]},
         "pod": [4, 40], "hint": "MostAllocated", "want_zone": 3},
        {"name": "restricted numa nodes and select least allocated and preferred",
         "ref": "nodenumaresource/plugin_test.go:2745-2771",
         "node": [104, 256], "policy": "RESTRICTED", "zones": 4,
         "used": {"0": [[24, 8]], "1": [[23, 8]], "2": [[4, 8]], "3": [[8, 8]]},
         "pod": [4, 40], "hint": "LeastAllocated", "want_zone": 2},
    ],
    # nodenumaresource/scoring_test.go:54-337 TestNUMANodeScore (ScoringStrategy MostAllocated, default
    # LeastAllocated hint scoring); existing pods count on the node and on NUMA zone 0
    "score": [
        {"name": "single numa nodes score", "ref": "nodenumaresource/scoring_test.go:64-104",
         "nodes": [{"node": [104, 256], "zones": 2}, {"node": [64, 128], "zones": 1}], "policy": "SINGLE_NODE",
         "existing": [[], []], "pod": [21, 40], "want": [35, 31]},
        {"name": "restricted numa nodes score", "ref": "nodenumaresource/scoring_test.go:105-145",
         "nodes": [{"node": [104, 256], "zones": 2}, {"node": [64, 128], "zones": 1}], "policy": "RESTRICTED",
         "existing": [[], []], "pod": [50, 40], "want": [63, 54]},
        {"name": "single numa nodes score with same capacity but different requested",
         "ref": "nodenumaresource/scoring_test.go:146-200",
         "nodes": [{"node": [104, 256], "zones": 2}] * 3, "policy": "SINGLE_NODE",
         "existing": [[[4, 8]], [[8, 32]], [[32, 40]]], "pod": [4, 40], "want": [19, 19, 19]},
    ],
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "numa_kat.json")
    with open(out, "w") as f:
        json.dump(cases, f, indent=1)
    print("wrote", out)
