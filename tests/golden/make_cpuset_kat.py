"""Writes tests/golden/cpuset_kat.json: the reference's own known-answer tests of the cpuset accumulator,
transcribed from pkg/scheduler/plugins/nodenumaresource/cpu_accumulator_test.go (values only: topology
shape, allocated CPUs, request, policies, expected cpuset).

  TestTakeFullPCPUs                          :59-173   (FullPCPUs, NUMAMostAllocated)
  TestTakeFullPCPUsWithNUMALeastAllocated    :175-289
  TestTakeSpreadByPCPUs                      :301-361
  TestTakeSpreadByPCPUsWithNUMALeastAllocated :373-433
  TestTakeCPUsWithExclusivePolicy            :435-558
  TestTakeCPUsWithMaxRefCount                :560-599  (sequence: addCPUs between takes, maxRefCount 2)
  TestTakeCPUsSortByRefCount                 :601-651  (sequence)
  TestTakePreferredCPUs                      :758-777

buildCPUTopologyForTest(sockets, nodesPerSocket, coresPerNode, cpusPerCore) (:30-57) numbers CPUs, cores and
nodes consecutively; the KAT keeps the four numbers and the test side rebuilds the topology.
"""
import json
import os


def cs(s):
    """cpuset.MustParse syntax -> sorted list"""
    out = []
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(out)


FULL, SPREAD = "FullPCPUs", "SpreadByPCPUs"
MOST, LEAST = "MostAllocated", "LeastAllocated"
PCPU, NUMA, NONE = "PCPULevel", "NUMANodeLevel", "None"


def take(name, src, topo, allocated, needed, want, bind, strategy, excl=NONE, alloc_excl=None, error=False):
    return {"name": name, "source": src, "topo": topo, "max_ref": 1, "allocated": cs(allocated),
            "alloc_excl": alloc_excl, "needed": needed, "bind": bind, "excl": excl, "strategy": strategy,
            "want": cs(want), "error": error}


cases = []
F = "cpu_accumulator_test.go:59 TestTakeFullPCPUs"
cases += [
    take("allocate on non-NUMA node", F, [1, 1, 4, 2], "", 2, "0,1", FULL, MOST),
    take("with allocated cpus", F, [1, 1, 4, 2], "0,1", 2, "2,3", FULL, MOST),
    take("allocate whole socket", F, [2, 1, 4, 2], "", 8, "0-7", FULL, MOST),
    take("allocate across socket", F, [2, 1, 4, 2], "", 12, "0-11", FULL, MOST),
    take("allocate whole socket with partially-allocated socket", F, [2, 1, 4, 2], "0,1", 8, "8-15", FULL, MOST),
    take("allocate in the smallest idle socket", F, [2, 2, 4, 2], "0-5,16-23", 6, "24-29", FULL, MOST),
    take("allocate the most of CPUs on the same socket", F, [2, 2, 4, 2], "0-5,16-23", 12, "6-15,24-25", FULL, MOST),
    take("allocate from first socket", F, [2, 2, 4, 2], "0-3,8-11", 4, "4-7", FULL, MOST),
    take("allocate with less spread cpus", F, [2, 2, 2, 2], "0,2,4,8,12", 4, "10,11,14,15", FULL, MOST),
    take("allocate with the most spread cpus", F, [2, 2, 2, 2], "0,2,4,8,10,12", 6, "5,6,7,13,14,15", FULL, MOST),
    take("allocate with the most spread cpus on the smallest idle cpus socket", F, [2, 2, 2, 2],
         "0,2,4,8,9,10,12", 6, "6,7,11,13,14,15", FULL, MOST),
]
F = "cpu_accumulator_test.go:175 TestTakeFullPCPUsWithNUMALeastAllocated"
cases += [
    take("allocate on non-NUMA node", F, [1, 1, 4, 2], "", 2, "0,1", FULL, LEAST),
    take("with allocated cpus", F, [1, 1, 4, 2], "0,1", 2, "2,3", FULL, LEAST),
    take("allocate whole socket", F, [2, 1, 4, 2], "", 8, "0-7", FULL, LEAST),
    take("allocate across socket", F, [2, 1, 4, 2], "", 12, "0-11", FULL, LEAST),
    take("allocate whole socket with partially-allocated socket", F, [2, 1, 4, 2], "0,1", 8, "8-15", FULL, LEAST),
    take("allocate in the most idle socket", F, [2, 2, 4, 2], "0-5,16-23", 6, "8-13", FULL, LEAST),
    take("allocate the most of CPUs on the same socket", F, [2, 2, 4, 2], "0-5,16-23", 12, "6-15,24-25", FULL, LEAST),
    take("allocate from second socket", F, [2, 2, 4, 2], "0-3,8-11", 4, "16-19", FULL, LEAST),
    take("allocate with less spread cpus", F, [2, 2, 2, 2], "0,2,4,8,12", 4, "10,11,14,15", FULL, LEAST),
    take("allocate with the less spread cpus 2", F, [2, 2, 2, 2], "0,2,4,8,10,12", 6, "6,7,14,15,1,3", FULL, LEAST),
    take("allocate with the most spread cpus on the most idle cpus socket 3", F, [2, 2, 4, 2],
         "0,2,4,8,9,10,12", 6, "16-21", FULL, LEAST),
]
F = "cpu_accumulator_test.go:301 TestTakeSpreadByPCPUs"
cases += [
    take("allocate on non-NUMA node", F, [1, 1, 4, 2], "", 4, "0,2,4,6", SPREAD, MOST),
    take("allocate satisfied the partially-allocated socket", F, [2, 1, 4, 2], "0,2", 4, "1,3,4,6", SPREAD, MOST),
    take("allocate cpus on full-free socket", F, [2, 1, 4, 2], "0,1,2,3", 4, "8,10,12,14", SPREAD, MOST),
    take("allocate most of CPUs in the same socket and overlapped-cores", F, [2, 1, 4, 2], "0,2", 6, "1,3-7",
         SPREAD, MOST),
]
F = "cpu_accumulator_test.go:373 TestTakeSpreadByPCPUsWithNUMALeastAllocated"
cases += [
    take("allocate on non-NUMA node", F, [1, 1, 4, 2], "", 4, "0,2,4,6", SPREAD, LEAST),
    take("allocate satisfied the partially-allocated socket", F, [2, 1, 4, 2], "0,2", 4, "8,10,12,14", SPREAD, LEAST),
    take("allocate cpus on full-free socket", F, [2, 1, 4, 2], "0,1,2,3", 4, "8,10,12,14", SPREAD, LEAST),
    take("allocate most of CPUs in the same socket and overlapped-cores", F, [2, 1, 4, 2], "0,2", 6,
         "8,10,12,14,9,11", SPREAD, LEAST),
]
# TestTakeCPUsWithExclusivePolicy: allocated CPUs carry allocatedExclusivePolicy (default PCPULevel); the
# request's exclusive policy defaults to PCPULevel and its bind policy to SpreadByPCPUs (:541-550)
F = "cpu_accumulator_test.go:435 TestTakeCPUsWithExclusivePolicy"
cases += [
    take("allocate cpus on full-free socket with PCPULevel", F, [2, 1, 4, 2], "0,2", 4, "8,10,12,14", SPREAD, MOST,
         excl=PCPU, alloc_excl=PCPU),
    take("allocate overlapped cpus with PCPULevel", F, [2, 1, 4, 2], "", 10, "0,1,2,3,4,6,8,10,12,14", SPREAD, MOST,
         excl=PCPU, alloc_excl=PCPU),
    take("allocate cpus on large-size partially-allocated socket with PCPULevel", F, [2, 1, 8, 2], "0,2", 4,
         "4,6,8,10", SPREAD, MOST, excl=PCPU, alloc_excl=PCPU),
    take("allocate cpus with none exclusive policy", F, [2, 1, 8, 2], "0,2", 4, "1,3,4,6", SPREAD, MOST, excl=NONE,
         alloc_excl=PCPU),
    take("allocate cpus on full-free socket with NUMANodeLevel", F, [2, 1, 4, 2], "0,2", 4, "8,10,12,14", SPREAD,
         MOST, excl=NUMA, alloc_excl=NUMA),
    take("allocate cpus on partially-allocated socket without NUMANodeLevel", F, [2, 1, 4, 2], "0,2", 4, "1,3,4,6",
         SPREAD, MOST, excl=NONE, alloc_excl=NUMA),
    take("allocate cpus on full-free socket with NUMANodeLevel with PCPUs", F, [2, 1, 4, 2], "0,2", 4, "8,9,10,11",
         FULL, MOST, excl=NUMA, alloc_excl=NUMA),
    take("allocate cpus on partially-allocated socket without NUMANodeLevel with PCPUs", F, [2, 1, 4, 2], "0,2", 4,
         "4,5,6,7", FULL, MOST, excl=NONE, alloc_excl=NUMA),
]

# sequences: takeCPUs on getAvailableCPUs(maxRefCount 2), then addCPUs(result, PCPULevel) (node_allocation.go
# :103-130: RefCount++, ExclusivePolicy = the pod's)
sequences = [
    {"name": "TestTakeCPUsWithMaxRefCount", "source": "cpu_accumulator_test.go:560", "topo": [1, 1, 4, 2],
     "max_ref": 2, "strategy": MOST, "excl": NONE, "add_excl": PCPU,
     "steps": [{"needed": 4, "bind": FULL, "want": cs("0-3")},
               {"needed": 5, "bind": FULL, "want": cs("0,4-7")},
               {"needed": 4, "bind": FULL, "want": cs("2-5")}]},
    {"name": "TestTakeCPUsSortByRefCount", "source": "cpu_accumulator_test.go:601", "topo": [1, 1, 16, 2],
     "max_ref": 2, "strategy": MOST, "excl": NONE, "add_excl": PCPU,
     "steps": [{"needed": 16, "bind": SPREAD, "want": cs("0,2,4,6,8,10,12,14,16,18,20,22,24,26,28,30")},
               {"needed": 16, "bind": FULL, "want": cs("0-15")},
               {"needed": 16, "bind": SPREAD, "want": cs("1,3,5,7,9,11,13,15,17,19,21,23,25,27,29,31")},
               {"needed": 16, "bind": FULL, "want": cs("16-31")}],
     "final_available": []},
]

preferred = {"name": "TestTakePreferredCPUs", "source": "cpu_accumulator_test.go:758", "topo": [2, 1, 16, 2],
             "calls": [
                 {"avail": "all", "preferred": None, "needed": 2, "want": [0, 2]},
                 {"avail": "all", "preferred": [0, 2], "needed": 2, "want": [0, 2]},
                 {"avail": "all-minus-0,2", "preferred": [], "needed": 2, "want": [1, 3]},
                 {"avail": "all", "preferred": [11, 13, 15, 17], "needed": 2, "want": [11, 13]},
             ], "bind": SPREAD, "strategy": MOST}

here = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(here, "cpuset_kat.json"), "w") as f:
    json.dump({"takes": cases, "sequences": sequences, "preferred": preferred}, f, indent=1)
print(len(cases), "take cases,", len(sequences), "sequences, 1 preferred set")
