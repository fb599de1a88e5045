"""Builders for the GPU allocator known answers of tests/golden/gpu_alloc_kat.json (make_gpu_alloc_kat.py)."""
import json
import os

import numpy as np

from koordinator_amd import abi, decode
from koordinator_amd.config import config5_profile

HERE = os.path.dirname(os.path.abspath(__file__))
CODES = {"PART_COUNT": abi.KG_DEV_CODE_PART_COUNT, "TOPO_SCOPED": abi.KG_DEV_CODE_TOPO_SCOPED,
         "PARTITIONED": abi.KG_DEV_CODE_PARTITIONED, "GPU_DEVICES": abi.KG_DEV_CODE_GPU_DEVICES}


def load():
    with open(os.path.join(HERE, "golden", "gpu_alloc_kat.json")) as f:
        return json.load(f)


def build(K, c):
    """(kg_config, node table of one node, pod table of one pod) of a case, through the host decode."""
    kc = config5_profile().kg_config()
    kc.plugins = abi.KG_PLUGIN_DEV
    if c["scorer"]:
        kc.dev_most_allocated = 1 if c["scorer"]["most"] else 0
        for r, w in enumerate(c["scorer"]["weights"]):
            kc.dev_w[r] = w
    nodes = abi.empty_nodes(1)
    nodes["alloc_cpu"][:] = 64000
    nodes["alloc_mem"][:] = 256 << 30
    nodes["alloc_pods"][:] = 110
    g, sh = K["gpu"], K["shared_alloc"]
    nodes["dev_minors"][0] = 8
    for m in range(8):
        nodes["dev_total"][0, :, m] = [g["core"], g["ratio"], g["memory"]]
        nodes["dev_free"][0, :, m] = [g["core"], g["ratio"], g["memory"]]
    for m in c["assigned"]:
        nodes["dev_free"][0, :, m] = 0
    for m in c["assigned_shared"]:
        nodes["dev_free"][0, :, m] -= [sh["core"], sh["ratio"], sh["memory"]]
    infos = [{"minor": m, "topology": {"nodeID": q, "pcieID": pcie}} for m, (q, pcie) in enumerate(K["devices"][c["device"]])]
    topo, tree = decode.gpu_topology(infos)
    node = {"metadata": {"labels": {decode.LABEL_GPU_MODEL: c["model"]} if c["model"] else {}}}
    if c["honor"]:
        node["metadata"]["labels"][decode.LABEL_GPU_PARTITION_POLICY] = "Honor"
    table, honor = decode.gpu_partition_table(None, node)
    tabs = decode.GpuPartitionTables()
    part = tabs.add(table) | (abi.KG_GPU_HONOR if honor else 0) | (abi.KG_GPU_TREE if tree else 0)
    nodes["dev_topo"] = np.array([topo], np.uint64)
    nodes["dev_part"] = np.array([part], np.uint32)
    nodes["gpu_parts"] = tabs.array()
    pods = abi.empty_pods(1)
    req = {"koordinator.sh/gpu-core": 100 * c["n"], "koordinator.sh/gpu-memory-ratio": 100 * c["n"]}
    if c["gpu_shared"]:  # gpu.shared n + ratio 50 + core 50 (allocator_gpu_test.go:1612-1616)
        req = {"koordinator.sh/gpu.shared": c["n"], "koordinator.sh/gpu-core": 50, "koordinator.sh/gpu-memory-ratio": 50}
    vec, keys, cnt, shared = decode.gpu_requirements(req)
    pods["dev_req"][0] = vec
    pods["dev_keys"][0] = keys
    pods["dev_count"][0] = cnt
    pod = {"metadata": {"annotations": {}}}
    if c["scope"]:
        pod["metadata"]["annotations"][decode.ANN_DEVICE_ALLOCATE_HINT] = json.dumps(
            {"gpu": {"requiredTopologyScope": c["scope"]}})
    flags, bw = decode.gpu_pod_flags(pod, shared)
    pods["dev_flags"] = np.array([flags], np.uint32)
    pods["dev_ring_bw"] = np.array([bw], np.int64)
    return kc, nodes, pods


def minors_of(mask: int):
    return [m for m in range(abi.KG_DEV_MINORS) if (mask >> m) & 1]
