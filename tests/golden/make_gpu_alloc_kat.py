"""Known answers of the DeviceShare GPU allocator (partitions, topology scopes, shared bin-packing),
transcribed from /root/reference/pkg/scheduler/plugins/deviceshare/allocator_gpu_test.go. Writes
gpu_alloc_kat.json next to this file.

Only the GPU half of each case is kept: the reference tests also allocate RDMA VFs jointly; the GPU minors
they expect are what the GPU allocator returns (the joint allocation of those cases allocates the GPUs
first and puts the VFs next to them). A case expecting an error records it as "error" with the allocator
code the restatement derives (the reference asserts only wantErr).

Device CRs (GPU minors, NUMA node, PCIe id; every GPU 100 core / 100 ratio / 83201216Ki memory):
  fakeH800DeviceCR (allocator_gpu_test.go:42-49): minors 0-3 on NUMA 0 with PCIe 0,2,3,4, minors 4-7 on NUMA 1
                    with PCIe 5,6,7,8;
  fakeDeviceCR (device_allocator_test.go:65-72): NUMA 0 PCIe 0 {0,1}, PCIe 1 {2,3}; NUMA 1 PCIe 2 {4,5},
                    PCIe 3 {6,7}.
Assigned allocations: gpuResourceList (full GPU) and gpuSharedResourceList (50 core / 50 ratio / 42599022592
bytes) of device_allocator_test.go:45-55."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

H800 = [(0, "0"), (0, "2"), (0, "3"), (0, "4"), (1, "5"), (1, "6"), (1, "7"), (1, "8")]
FAKE = [(0, "0"), (0, "0"), (0, "1"), (0, "1"), (1, "2"), (1, "2"), (1, "3"), (1, "3")]


def case(name, line, device, want, *, model="", honor=True, assigned=(), shared=(), n=1, gpu_shared=False,
         scope="", error=None, scorer=None):
    return dict(name=name, line=line, device=device, model=model, honor=honor, assigned=list(assigned),
                assigned_shared=list(shared), n=n, gpu_shared=gpu_shared, scope=scope, want=list(want), error=error,
                scorer=scorer)


# TestAllocateByPartition (allocator_gpu_test.go:56-971): node labelled gpu-model = modelSeries and
# gpu-partition-policy = Honor unless the case sets another policy (:851-861); Hopper designated table.
PARTITION = [
    case("allocate 1 GPU and 1 VF", 93, "h800", [0], model="H800", n=1),
    case("allocate 2 GPU and 2 VF", 123, "h800", [0, 1], model="H800", n=2),
    case("allocate 3 GPU", 171, "h800", [], model="H800", n=3, error="PART_COUNT"),
    case("allocate 4 GPU and 4 VF", 178, "h800", [0, 1, 2, 3], model="H800", n=4),
    case("allocate 6 GPU and 3 VF", 262, "h800", [], model="H800", n=6, error="PART_COUNT"),
    case("allocate 8 GPU and 8 VF", 269, "h800", list(range(8)), model="H800", n=8),
    case("allocate 2 GPU and 2 VF with assigned devices", 425, "h800", [0, 1], model="H800", n=2, assigned=[2, 3]),
    case("allocate 2 GPU and 2 VF with assigned devices; BinPack", 516, "h800", [6, 7], model="H800", n=2,
         assigned=[4]),
    case("allocate 1 GPU and 1 VF with assigned devices; BinPack", 589, "h800", [5], model="H800", n=1,
         assigned=[4]),
    case("allocate 2 GPU and 2 VF with assigned devices; H100", 644, "h800", [0, 1], model="H100", n=2,
         assigned=[2, 3]),
    case("allocate 2 GPU and 2 VF with assigned devices; H100; gpuPartitionPolicyPrefer", 735, "h800", [4, 5, 6],
         model="H100", honor=False, n=3, assigned=[2, 3]),
]

# TestAllocateByTopology (:973-1419): fakeDeviceCR, no model label (no partition table), no scorer.
TOPOLOGY = [
    case("allocate 1 GPU and 1 VF with assigned devices; topology scope BinPack", 986, "fake", [4], n=1,
         assigned=[5], honor=False),
    case("allocate 2 GPU and 1 VF with assigned devices; topology scope BinPack", 1040, "fake", [6, 7], n=2,
         assigned=[5], honor=False),
    case("allocate 1 GPU and 1 VF with assigned devices; requiredTopologyScope PCIE and BinPack", 1098, "fake",
         [6, 7], n=2, assigned=[5], scope="PCIe", honor=False),
    case("allocate 1 GPU and 1 VF with assigned devices; requiredTopologyScope NUMANode", 1157, "fake",
         [0, 1, 2, 3], n=4, assigned=[5], scope="NUMANode", honor=False),
    case("allocate 1 GPU and 1 VF with assigned devices; requiredTopologyScope NUMANode, insufficient devices",
         1238, "fake", [], n=4, assigned=[5, 0], scope="NUMANode", honor=False, error="TOPO_SCOPED"),
]

# TestAllocateSharedGPU (:1421-1691): gpu.shared 1 + ratio 50 + core 50; MostAllocated scorer over
# gpu-memory-ratio (weight 1, :1659-1669).
MOST_RATIO = {"most": True, "weights": [0, 1, 0]}
SHARED = [
    case("allocate 1 GPU and 1 VF with assigned devices; topology scope BinPack", 1434, "fake", [4], n=1,
         gpu_shared=True, assigned=[5], honor=False, scorer=MOST_RATIO),
    case("two scope, both not empty, shared binpack take Precedence", 1488, "fake", [7], n=1, gpu_shared=True,
         assigned=[5], shared=[7], honor=False, scorer=MOST_RATIO),
]


def main():
    out = {"devices": {"h800": H800, "fake": FAKE},
           "gpu": {"core": 100, "ratio": 100, "memory": 83201216 * 1024},
           "shared_alloc": {"core": 50, "ratio": 50, "memory": 42599022592},
           "cases": PARTITION + TOPOLOGY + SHARED}
    with open(os.path.join(HERE, "gpu_alloc_kat.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
