"""Known answers of DeviceShare as a NUMA hint provider, transcribed from
/root/reference/pkg/scheduler/plugins/deviceshare/topology_hint_test.go. Writes gpu_numa_kat.json next to this file.

Node: fakeDeviceCR (device_allocator_test.go:65-72): GPU minors 0-3 on NUMA node 0 (PCIe 0: {0, 1}, PCIe 1: {2, 3}),
minors 4-7 on NUMA node 1 (PCIe 2: {4, 5}, PCIe 3: {6, 7}); every GPU 100 gpu-core, 100 gpu-memory-ratio,
83201216Ki gpu-memory. No partition table, no GPU model label.

Only the GPU device type is modelled: the RDMA / FPGA halves of the reference cases are dropped. In
"generate gpu&rdma hints" (:69-86) the GPU list does not depend on the RDMA request (no joint allocation, every mask
also fits the RDMA VFs), so its GPU list is the GPU-only answer. Cases of other device types only (fpga, rdma VF
hints) and Test_generateDesignatedHints (:421, designated allocations are not on the device path)
are not transcribed.

Hints: (NUMA node ids of the affinity, Preferred, Score); defaultNUMAScore = 500 (topology_hint.go:36)."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = [
    # TestPlugin_GetPodTopologyHints (topology_hint_test.go:41-270)
    dict(name="generate gpu&rdma hints (GPU list)", line=69, gpu_core=100, gpu_ratio=100, assigned=[],
         result="hints", want=[[[0], True, 500], [[1], True, 0], [[0, 1], False, 500]]),
    dict(name="generate gpu&rdma hints but large gpu requests", line=88, gpu_core=1700, gpu_ratio=1700, assigned=[],
         result="fail", want=None),
    # gpuRequests (core 100, ratio 100) assigned on minor 0 (:103-112, the pod requests 4 GPUs)
    dict(name="generate gpu hints with assigned devices", line=97, gpu_core=400, gpu_ratio=400,
         assigned=[[0, 100, 100]], result="hints", want=[[[1], True, 500], [[0, 1], False, 500]]),
    # the joint GPU & RDMA allocation (:186-211): on fakeDeviceCR every GPU mask also holds RDMA VFs under the same
    # PCIe switches, so the GPU list the test asserts is the GPU-only answer of :69 (the RDMA half is not modelled)
    dict(name="generate joint-allocate gpu&rdma hints (GPU list)", line=186, gpu_core=100, gpu_ratio=100, assigned=[],
         result="hints", want=[[[0], True, 500], [[1], True, 0], [[0, 1], False, 500]]),
]

# TestPlugin_Allocate (topology_hint_test.go:272-419): gpuRequests there = gpu-core 100 + gpu-memory 8Gi
ALLOCATE = [
    dict(name="allocate gpu&rdma by affinity (GPU part)", line=295, gpu_core=100, gpu_mem=8 << 30, affinity=[0],
         error=False),
    # :362 "generate joint-allocate gpu&rdma hints" (Allocate under NUMA node 0): its GPU part; the other cases of
    # TestPlugin_Allocate (:305-361) request FPGA / RDMA only
    dict(name="allocate joint gpu&rdma under NUMA node 0 (GPU part)", line=362, gpu_core=100, gpu_mem=8 << 30,
         affinity=[0], error=False),
]

DEVICE = {"numa": [0, 0, 0, 0, 1, 1, 1, 1], "pcie": ["0", "0", "1", "1", "2", "2", "3", "3"],
          "core": 100, "ratio": 100, "memory": 83201216 * 1024}

if __name__ == "__main__":
    with open(os.path.join(HERE, "gpu_numa_kat.json"), "w") as f:
        json.dump({"device": DEVICE, "hints": CASES, "allocate": ALLOCATE}, f, indent=1)
