"""ctypes mirror of include/koordgpu.h plus numpy column tables.

The node and pod tables are plain dicts of numpy arrays keyed by the column names below; the
helpers turn them into the C structs of the boundary (pointers into the numpy buffers, which the
caller keeps alive for the duration of the call).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict

import numpy as np

KG_ABI_VERSION = 12
KG_LA_R = 2
KG_NSCALAR = 2
KG_MAX_ZONES = 4
KG_DEV_MINORS = 8
KG_DEV_R = 3
KG_DEV_CORE, KG_DEV_RATIO, KG_DEV_MEM = 0, 1, 2
KG_QUOTA_R = 4
KG_RSV_R = 5

KG_OK, KG_INVALID_ARG, KG_DEVICE_ERROR, KG_OOM, KG_UNSUPPORTED, KG_NO_DEVICE, KG_RESERVE_FAILED = range(7)

KG_PLUGIN_NRF = 0x1
KG_PLUGIN_LA = 0x2
KG_PLUGIN_NUMA = 0x4
KG_PLUGIN_DEV = 0x8
KG_PLUGIN_RSV = 0x10
KG_PLUGIN_QUOTA = 0x20
KG_PLUGIN_EXT = KG_PLUGIN_DEV | KG_PLUGIN_RSV | KG_PLUGIN_QUOTA

KG_LA_HAS_METRIC = 0x1
KG_LA_NM_NIL = 0x2
KG_LA_EXPIRED = 0x4
KG_LA_PROD_THR = 0x8
KG_LA_AGG_THR = 0x10

KG_NUMA_NONE = 0
KG_NUMA_BEST_EFFORT = 1
KG_NUMA_RESTRICTED = 2
KG_NUMA_SINGLE_NODE = 3

KG_POD_DAEMONSET = 0x1
KG_POD_PROD = 0x2
KG_POD_NUMA_SKIP = 0x4
KG_POD_HAS_CPU = 0x8
KG_POD_HAS_MEM = 0x10
KG_POD_CPU_BIND = 0x20
KG_POD_CPU_POLICY_SHIFT = 8
KG_POD_CPU_REQUIRED = 0x400
KG_POD_CPU_EXCL_SHIFT = 11
KG_NODE_CPU_BIND_NONE, KG_NODE_CPU_BIND_FULL_PCPUS_ONLY, KG_NODE_CPU_BIND_SPREAD_BY_PCPUS = 0, 1, 2
KG_POD_NON_PREEMPTIBLE = 0x40
KG_POD_RSV_REQUIRED = 0x80

KG_RSV_DEFAULT, KG_RSV_ALIGNED, KG_RSV_RESTRICTED = 0, 1, 2

KG_ST_NRF_PODS = 0x1
KG_ST_NRF_CPU = 0x2
KG_ST_NRF_MEM = 0x4
KG_ST_NRF_EPH = 0x8
KG_ST_NRF_SC0 = 0x10
KG_ST_NRF_SC1 = 0x20
KG_ST_NRF_MASK = 0x3F
KG_ST_LA_EXPIRED = 0x100
KG_ST_LA_CPU = 0x200
KG_ST_LA_MEM = 0x400
KG_ST_LA_AGG = 0x800
KG_ST_LA_MASK = 0x0F00
KG_ST_NUMA_INSUF_CPU = 0x1000   # BestEffort Reserve: "Insufficient NUMA cpu"
KG_ST_NUMA_INSUF_MEM = 0x2000   # "Insufficient NUMA memory"
KG_ST_NUMA_INSUF_NODE = 0x4000  # "node(s) Insufficient NUMA Node resources"
KG_ST_NUMA_RESERVE = KG_ST_NUMA_INSUF_CPU | KG_ST_NUMA_INSUF_MEM | KG_ST_NUMA_INSUF_NODE
ZONE_RESERVE_FAIL = 0x20        # numa_zone code | (KG_ST_NUMA_INSUF_* >> 12): the pair's Reserve fails
KG_ST_NUMA_AMP_CPU = 0x10000
KG_ST_NUMA_CONFLICT = 0x20000
KG_ST_NUMA_NO_RES = 0x40000
KG_ST_NUMA_ALIGN = 0x80000
KG_ST_NUMA_UNSATISFIED = 0x100000
KG_ST_NUMA_CPU_TOPO = 0x200000
KG_ST_NUMA_CPU_BIND = 0x400000
KG_ST_NUMA_CPUS = 0x800000
KG_ST_NUMA_MASK = 0xFF7000
KG_ST_DEV_INSUFFICIENT = 0x01000000
KG_ST_DEV_NO_DEVICE = 0x02000000
KG_ST_DEV_MASK = 0x030000C0  # 4-bit reason code: bits 24-25 low half, bits 6-7 high half
KG_DEV_CODE_INSUFFICIENT, KG_DEV_CODE_NO_DEVICE, KG_DEV_CODE_GPU_DEVICES, KG_DEV_CODE_TOPO_SCOPED = 1, 2, 3, 4
KG_DEV_CODE_PARTITIONED, KG_DEV_CODE_NO_PARTITION, KG_DEV_CODE_PART_COUNT, KG_DEV_CODE_NO_TREE = 5, 6, 7, 8
KG_DEV_CODE_MULTI_SHARED = 9
KG_DEV_CODE_NUMA_SCOPED = 10  # ErrInsufficientNUMAScopedDevices (deviceshare/topology_hint.go:34)
KG_DEV_CODE_NO_TEMPLATE = 11  # ErrNoMatchedGPUSharedResourceTemplate (deviceshare/allocator_gpu.go:40)


def dev_code(st: int) -> int:
    """KG_ST_DEV_CODE: the DeviceShare reason code of a status word."""
    return ((st >> 24) & 3) | (((st >> 6) & 3) << 2)


def dev_status(code: int) -> int:
    """KG_ST_DEV_MAKE"""
    return ((code & 3) << 24) | (((code >> 2) & 3) << 6)


# GPU topology / partitions (kg_node_columns.dev_topo / dev_part / gpu_parts, kg_pod_columns.dev_flags)
KG_GPU_NO_SCOPE = 0xFF
# kg_node_columns.dev_numa: a nibble per minor, the GPU's NUMA node id (deviceshare/numa_topology.go:43-100)
KG_GPU_NUMA_ANY = 0xE   # Topology.NodeID == -1
KG_GPU_NUMA_NONE = 0xF  # no Topology
KG_GPU_HONOR = 0x100
KG_GPU_TREE = 0x200
KG_GPU_TMPL_SHIFT = 12  # dev_part bits 12-15: the node's shared-resource template key
KG_GPU_TMPL_NONE = 15
KG_ZONE_RECORD_SHIFT = 8  # numa_zone_status bit 8 + z: zone z holds an allocatedResources record
KG_GPU_MAX_TABLES = 16
KG_GPU_POD_SHARED = 0x1
KG_GPU_POD_HONOR = 0x2
KG_GPU_POD_RESTRICTED = 0x4
KG_GPU_POD_RING_BW = 0x8
KG_GPU_POD_SCOPE_SHIFT = 4
KG_GPU_POD_TEMPLATE = 0x100
# DeviceTopologyScopeLevel (apis/extension/device_share.go:185-190); 5 = a scope name without a level
GPU_SCOPE_LEVEL = {"": 0, "Node": 1, "NUMANode": 2, "PCIe": 3, "Device": 4}
GPU_PARTITION_DTYPE = np.dtype([("table", np.uint8), ("n_gpus", np.uint8), ("minors", np.uint8), ("pad_", np.uint8),
                                ("alloc_score", np.int32), ("ring_bw", np.int64)])
KG_ST_RSV_AFFINITY = 0x04000000
KG_ST_RSV_NODE = 0x08000000
KG_ST_RSV_RESERVATION = 0x10000000
KG_ST_RSV_MASK = 0x1C000000
KG_ST_QUOTA = 0x20000000
KG_ST_DEV_RSV = 0x40000000  # "Reservation(s) Insufficient gpu devices"
KG_ST_UNSUPPORTED = 0x80000000
# kg_batch_schedule per-pod result codes
KG_BATCH_ASSUMED, KG_BATCH_FAILED, KG_BATCH_SIBLING, KG_BATCH_ROLLED_BACK, KG_BATCH_NO_PLAN = range(5)

_p64 = C.POINTER(C.c_int64)
_pu32 = C.POINTER(C.c_uint32)
_pf64 = C.POINTER(C.c_double)
_pi32 = C.POINTER(C.c_int32)


class KgConfig(C.Structure):
    _fields_ = [
        ("plugins", C.c_uint32),
        ("weight_nrf", C.c_int64),
        ("weight_la", C.c_int64),
        ("weight_numa", C.c_int64),
        ("nrf_w_cpu", C.c_int64),
        ("nrf_w_mem", C.c_int64),
        ("nrf_w_sc", C.c_int64 * KG_NSCALAR),
        ("la_score_enabled", C.c_uint32),
        ("la_filter_expired", C.c_uint32),
        ("la_schedule_expired", C.c_uint32),
        ("la_score_prod", C.c_uint32),
        ("la_w", C.c_int64 * KG_LA_R),
        ("la_dominant_w", C.c_int64),
        ("numa_w_cpu", C.c_int64),
        ("numa_w_mem", C.c_int64),
        ("numa_hint_w_cpu", C.c_int64),
        ("numa_hint_w_mem", C.c_int64),
        ("weight_dev", C.c_int64),
        ("weight_rsv", C.c_int64),
        ("dev_w", C.c_int64 * KG_DEV_R),
        ("numa_most_allocated", C.c_uint32),
        ("numa_hint_most_allocated", C.c_uint32),
        ("dev_most_allocated", C.c_uint32),
        ("nrf_most_allocated", C.c_uint32),
        ("nrf_ignored_scalars", C.c_uint32),
        ("rsv_ignored_scalars", C.c_uint32),
    ]


class KgNodeColumns(C.Structure):
    _fields_ = [
        ("alloc_cpu", _p64), ("alloc_mem", _p64), ("alloc_eph", _p64), ("alloc_pods", _p64),
        ("req_cpu", _p64), ("req_mem", _p64), ("req_eph", _p64), ("num_pods", _p64),
        ("nz_cpu", _p64), ("nz_mem", _p64),
        ("sc_alloc", _p64 * KG_NSCALAR), ("sc_req", _p64 * KG_NSCALAR),
        ("la_flags", _pu32),
        ("la_alloc", _p64 * KG_LA_R),
        ("la_thr_usage", _p64 * KG_LA_R),
        ("la_thr_prod", _p64 * KG_LA_R),
        ("la_thr_agg", _p64 * KG_LA_R),
        ("la_fbase_np", _p64 * KG_LA_R),
        ("la_fbase_prod", _p64 * KG_LA_R),
        ("la_sbase_np", _p64 * KG_LA_R),
        ("la_sbase_prod", _p64 * KG_LA_R),
        ("numa_policy", _pu32),
        ("numa_zones", _pu32),
        ("cpu_amp_ratio", _pf64),
        ("cpuset_alloc_milli", _p64),
        ("zone_cpu", _p64 * KG_MAX_ZONES),
        ("zone_mem", _p64 * KG_MAX_ZONES),
        ("zone_cpu_used", _p64 * KG_MAX_ZONES),
        ("zone_mem_used", _p64 * KG_MAX_ZONES),
        ("dev_minors", _pi32), ("dev_total", _p64), ("dev_free", _p64),
        ("numa_zone_status", _pu32),
        # cpuset binding: cpu_topo (int32 per node), cpu_topos (kg_cpu_topo[]), cpu_alloc (kg_cpu_alloc per node)
        ("cpu_topo", _pi32), ("cpu_topos", C.c_void_p), ("n_cpu_topos", C.c_uint32), ("cpu_alloc", C.c_void_p),
        ("cpu_max_ref", C.POINTER(C.c_uint8)), ("cpu_bind_policy", C.POINTER(C.c_uint8)),
        ("cpu_strategy", C.POINTER(C.c_uint8)),
        # GPU topology tree / partition tables
        ("dev_topo", C.POINTER(C.c_uint64)), ("dev_part", _pu32), ("gpu_parts", C.c_void_p), ("n_gpu_parts", C.c_uint32),
        # GPU NUMA node ids (DeviceShare as a NUMA hint provider)
        ("dev_numa", _pu32),
        # cpuset pods per NUMA node in singleNUMANode (byte z) / sharedNode (byte KG_MAX_ZONES + z)
        ("numa_zone_pods", C.POINTER(C.c_uint64)),
        # a reservation on the node holds a NUMA / cpuset allocation (the device does not follow its restore)
        ("rsv_numa", C.POINTER(C.c_uint8)),
    ]


class KgNodeState(C.Structure):
    _fields_ = [
        ("req_cpu", _p64), ("req_mem", _p64), ("req_eph", _p64), ("num_pods", _p64),
        ("nz_cpu", _p64), ("nz_mem", _p64),
        ("sc_req", _p64 * KG_NSCALAR),
        ("la_fbase_np", _p64 * KG_LA_R), ("la_fbase_prod", _p64 * KG_LA_R),
        ("la_sbase_np", _p64 * KG_LA_R), ("la_sbase_prod", _p64 * KG_LA_R),
        ("zone_cpu_used", _p64 * KG_MAX_ZONES), ("zone_mem_used", _p64 * KG_MAX_ZONES),
        ("dev_free", _p64),
        ("cpuset_alloc_milli", _p64), ("cpu_alloc", C.c_void_p),
        ("numa_zone_status", C.POINTER(C.c_uint32)),
        ("numa_zone_pods", C.POINTER(C.c_uint64)),
    ]


KG_RECORD_CPUSET = 0x1
KG_RECORD_QUOTA = 0x2


class KgReserveRecord(C.Structure):
    """kg_reserve_record: what one kg_reserve took, for its kg_unreserve."""
    _fields_ = [("numa_zone", C.c_int32), ("gpu_minors", C.c_uint32), ("rsv_rid", C.c_int32), ("flags", C.c_uint32),
                ("zone_amounts", C.c_int64 * (2 * KG_MAX_ZONES)), ("cpus", C.c_uint64 * 4)]  # KG_MAX_CPUS / 64


class KgPodColumns(C.Structure):
    _fields_ = [
        ("req_cpu", _p64), ("req_mem", _p64), ("req_eph", _p64),
        ("sc_req", _p64 * KG_NSCALAR),
        ("nz_cpu", _p64), ("nz_mem", _p64),
        ("la_est", _p64 * KG_LA_R),
        ("flags", _pu32),
        ("numa_policy", _pu32),
        ("dev_req", _p64), ("dev_count", _pu32), ("dev_keys", _pu32),
        ("quota", _pi32), ("quota_keys", _pu32),
        ("rsv_class", _pi32),
        ("dev_flags", _pu32), ("dev_ring_bw", _p64), ("dev_tmpl", _pu32),
    ]


class KgVerifyOut(C.Structure):
    _fields_ = [
        ("status", _pu32),
        ("score_nrf", _p64),
        ("score_la", _p64),
        ("score_numa", _p64),
        ("total", _p64),
        ("numa_zone", C.POINTER(C.c_int8)),
        ("score_dev", _p64),
        ("score_rsv", _p64),
    ]


class KgQuotaColumns(C.Structure):
    _fields_ = [("used", _p64), ("used_limit", _p64), ("min", _p64), ("np_used", _p64),
                ("used_keys", _pu32), ("limit_keys", _pu32), ("min_keys", _pu32), ("np_used_keys", _pu32)]


class KgRsvView(C.Structure):
    _fields_ = [("node", C.c_uint32), ("cls", C.c_uint32), ("first", C.c_uint32), ("count", C.c_uint32),
                ("req", C.c_int64 * KG_RSV_R), ("nz_cpu", C.c_int64), ("nz_mem", C.c_int64), ("num_pods", C.c_int64),
                ("pod_requested", C.c_int64 * KG_RSV_R), ("r_allocated", C.c_int64 * KG_RSV_R),
                ("dev_base", C.c_int32), ("pad_", C.c_uint32)]


class KgRsvInfo(C.Structure):
    _fields_ = [("policy", C.c_uint32), ("names", C.c_uint32), ("allocate_once", C.c_uint32), ("dev", C.c_int32),
                ("order", C.c_int64), ("allocatable", C.c_int64 * KG_RSV_R), ("allocated", C.c_int64 * KG_RSV_R),
                ("reserved", C.c_int64 * KG_RSV_R), ("max_pods", C.c_int64), ("allocated_pods", C.c_int64),
                ("rid", C.c_uint32), ("allocated_keys", C.c_uint32), ("dev_minors", C.c_uint32), ("pad_", C.c_uint32)]


class KgRsvDev(C.Structure):
    _fields_ = [("total", (C.c_int64 * KG_DEV_MINORS) * KG_DEV_R), ("free", (C.c_int64 * KG_DEV_MINORS) * KG_DEV_R)]


KG_MAX_CPUS = 256
KG_CPU_BIND = {"": 0, "None": 0, "FullPCPUs": 1, "SpreadByPCPUs": 2}
KG_CPU_EXCL = {"": 0, "None": 0, "PCPULevel": 1, "NUMANodeLevel": 2}
KG_NUMA_STRATEGY = {"MostAllocated": 0, "LeastAllocated": 1}


class KgCpuTopo(C.Structure):
    _fields_ = [("n_cpus", C.c_uint16), ("n_cores", C.c_uint16), ("n_nodes", C.c_uint16), ("n_sockets", C.c_uint16),
                ("core", C.c_uint8 * KG_MAX_CPUS), ("numa", C.c_uint8 * KG_MAX_CPUS),
                ("socket", C.c_uint8 * KG_MAX_CPUS)]


class KgCpuAlloc(C.Structure):
    _fields_ = [("ref", C.c_uint8 * KG_MAX_CPUS), ("excl", C.c_uint8 * KG_MAX_CPUS)]


class KgCpusetRequest(C.Structure):
    _fields_ = [("topo", C.c_uint32), ("alloc", C.c_int32), ("avail", C.c_uint64 * 4), ("preferred", C.c_uint64 * 4),
                ("needed", C.c_int32), ("max_ref", C.c_int32), ("bind", C.c_int32), ("excl", C.c_int32),
                ("strategy", C.c_int32), ("has_preferred", C.c_int32)]


def cpu_topos_array(topos) -> np.ndarray:
    """list of KgCpuTopo -> uint8 [T, sizeof(kg_cpu_topo)] (the node table's cpu_topos column)."""
    out = np.zeros((len(topos), C.sizeof(KgCpuTopo)), np.uint8)
    for k, t in enumerate(topos):
        out[k] = np.frombuffer(bytes(t), np.uint8)
    return out


def cpu_topo(core, numa, socket) -> KgCpuTopo:
    """kg_cpu_topo from per-CPU ids (any integers): dense ranks in id order (the accumulator's tie-breaks)."""
    t = KgCpuTopo()
    n = len(core)
    if n > KG_MAX_CPUS:
        raise ValueError(f"{n} CPUs > {KG_MAX_CPUS}")
    for name, ids in (("core", core), ("numa", numa), ("socket", socket)):
        rank = {v: r for r, v in enumerate(sorted(set(ids)))}
        arr = getattr(t, name)
        for i, v in enumerate(ids):
            arr[i] = rank[v]
        setattr(t, {"core": "n_cores", "numa": "n_nodes", "socket": "n_sockets"}[name], len(rank))
    t.n_cpus = n
    return t


def cpu_topo_for_test(sockets, nodes_per_socket, cores_per_node, cpus_per_core) -> KgCpuTopo:
    """nodenumaresource/cpu_accumulator_test.go:30-57 buildCPUTopologyForTest."""
    core, numa, socket = [], [], []
    nid = cid = 0
    for s in range(sockets):
        for _ in range(nodes_per_socket):
            for _ in range(cores_per_node):
                for _ in range(cpus_per_core):
                    core.append(cid)
                    numa.append(nid)
                    socket.append(s)
                cid += 1
            nid += 1
    return cpu_topo(core, numa, socket)


def cpu_mask(cpus) -> np.ndarray:
    m = np.zeros(4, np.uint64)
    for c in cpus:
        m[c >> 6] |= np.uint64(1) << np.uint64(c & 63)
    return m


def mask_cpus(m) -> list:
    return [w * 64 + b for w in range(4) for b in range(64) if (int(m[w]) >> b) & 1]


# ----------------------------------------------------------------------------------------------
# column tables

def _indexed(name, n):
    return [f"{name}{i}" for i in range(n)]


NODE_I64 = (
    ["alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "req_cpu", "req_mem", "req_eph", "num_pods",
     "nz_cpu", "nz_mem"]
    + _indexed("sc_alloc", KG_NSCALAR) + _indexed("sc_req", KG_NSCALAR)
    + _indexed("la_alloc", KG_LA_R) + _indexed("la_thr_usage", KG_LA_R) + _indexed("la_thr_prod", KG_LA_R)
    + _indexed("la_thr_agg", KG_LA_R) + _indexed("la_fbase_np", KG_LA_R) + _indexed("la_fbase_prod", KG_LA_R)
    + _indexed("la_sbase_np", KG_LA_R) + _indexed("la_sbase_prod", KG_LA_R)
    + ["cpuset_alloc_milli"]
    + _indexed("zone_cpu", KG_MAX_ZONES) + _indexed("zone_mem", KG_MAX_ZONES)
    + _indexed("zone_cpu_used", KG_MAX_ZONES) + _indexed("zone_mem_used", KG_MAX_ZONES)
)
NODE_U32 = ["la_flags", "numa_policy", "numa_zones", "numa_zone_status"]
NODE_F64 = ["cpu_amp_ratio"]
NODE_DEV = ["dev_total", "dev_free"]  # int64 [n][KG_DEV_R][KG_DEV_MINORS]

NODE_STATE = (
    ["req_cpu", "req_mem", "req_eph", "num_pods", "nz_cpu", "nz_mem"] + _indexed("sc_req", KG_NSCALAR)
    + _indexed("la_fbase_np", KG_LA_R) + _indexed("la_fbase_prod", KG_LA_R)
    + _indexed("la_sbase_np", KG_LA_R) + _indexed("la_sbase_prod", KG_LA_R)
    + _indexed("zone_cpu_used", KG_MAX_ZONES) + _indexed("zone_mem_used", KG_MAX_ZONES)
)

POD_I64 = (["req_cpu", "req_mem", "req_eph"] + _indexed("sc_req", KG_NSCALAR) + ["nz_cpu", "nz_mem"]
           + _indexed("la_est", KG_LA_R))
POD_U32 = ["flags", "numa_policy", "dev_count", "dev_keys", "quota_keys"]
# optional GPURequirements columns (absent: no partition / topology requirement / template): dev_flags uint32,
# dev_ring_bw int64, dev_tmpl uint32 (2 bits per template key: candidate templates 0 / 1 / several)
POD_I32 = ["quota", "rsv_class"]

Table = Dict[str, np.ndarray]


def empty_nodes(n: int) -> Table:
    t: Table = {k: np.zeros(n, np.int64) for k in NODE_I64}
    t.update({k: np.zeros(n, np.uint32) for k in NODE_U32})
    t["cpu_amp_ratio"] = np.zeros(n, np.float64)
    t["dev_minors"] = np.full(n, -1, np.int32)  # no Device object
    for k in NODE_DEV:
        t[k] = np.zeros((n, KG_DEV_R, KG_DEV_MINORS), np.int64)
    return t


def empty_pods(n: int) -> Table:
    t: Table = {k: np.zeros(n, np.int64) for k in POD_I64}
    t.update({k: np.zeros(n, np.uint32) for k in POD_U32})
    t.update({k: np.full(n, -1, np.int32) for k in POD_I32})
    t["dev_req"] = np.zeros((n, KG_DEV_R), np.int64)
    return t


def table_len(t: Table) -> int:
    return int(len(next(iter(t.values()))))


def concat(tables) -> Table:
    keys = tables[0].keys()
    return {k: (tables[0][k] if k in TABLE_KEYS else np.concatenate([t[k] for t in tables])) for k in keys}


# table-level arrays of a node table (not one entry per node): shared by every row subset
TABLE_KEYS = ("cpu_topos", "gpu_parts")


def take(t: Table, idx) -> Table:
    return {k: (v if k in TABLE_KEYS else np.ascontiguousarray(v[idx])) for k, v in t.items()}


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def _check(t: Table, names, dtype):
    for k in names:
        a = t[k]
        if a.dtype != dtype or not a.flags["C_CONTIGUOUS"]:
            t[k] = np.ascontiguousarray(a, dtype=dtype)


def node_columns(t: Table) -> KgNodeColumns:
    if "numa_zone_status" not in t:
        t["numa_zone_status"] = np.zeros(table_len(t), np.uint32)
    _check(t, NODE_I64, np.int64)
    _check(t, NODE_U32, np.uint32)
    _check(t, NODE_F64, np.float64)
    s = KgNodeColumns()
    for k in ["alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "req_cpu", "req_mem", "req_eph",
              "num_pods", "nz_cpu", "nz_mem", "cpuset_alloc_milli"]:
        setattr(s, k, _ptr(t[k], C.c_int64))
    for k in range(KG_NSCALAR):
        s.sc_alloc[k] = _ptr(t[f"sc_alloc{k}"], C.c_int64)
        s.sc_req[k] = _ptr(t[f"sc_req{k}"], C.c_int64)
    for name in ["la_alloc", "la_thr_usage", "la_thr_prod", "la_thr_agg", "la_fbase_np", "la_fbase_prod",
                 "la_sbase_np", "la_sbase_prod"]:
        arr = getattr(s, name)
        for r in range(KG_LA_R):
            arr[r] = _ptr(t[f"{name}{r}"], C.c_int64)
    for name in ["zone_cpu", "zone_mem", "zone_cpu_used", "zone_mem_used"]:
        arr = getattr(s, name)
        for z in range(KG_MAX_ZONES):
            arr[z] = _ptr(t[f"{name}{z}"], C.c_int64)
    s.la_flags = _ptr(t["la_flags"], C.c_uint32)
    s.numa_policy = _ptr(t["numa_policy"], C.c_uint32)
    s.numa_zones = _ptr(t["numa_zones"], C.c_uint32)
    if "numa_zone_status" in t:
        s.numa_zone_status = _ptr(t["numa_zone_status"], C.c_uint32)
    s.cpu_amp_ratio = _ptr(t["cpu_amp_ratio"], C.c_double)
    if "dev_minors" in t:
        t["dev_minors"] = np.ascontiguousarray(t["dev_minors"], np.int32)
        for k in NODE_DEV:
            t[k] = np.ascontiguousarray(t[k], np.int64)
        s.dev_minors = _ptr(t["dev_minors"], C.c_int32)
        s.dev_total = _ptr(t["dev_total"], C.c_int64)
        s.dev_free = _ptr(t["dev_free"], C.c_int64)
    if "cpu_topo" in t:
        # cpuset tables: cpu_topos uint8 [T, sizeof kg_cpu_topo]; cpu_alloc uint8 [n, 512]
        t["cpu_topo"] = np.ascontiguousarray(t["cpu_topo"], np.int32)
        t["cpu_topos"] = np.ascontiguousarray(t["cpu_topos"], np.uint8)
        s.cpu_topo = _ptr(t["cpu_topo"], C.c_int32)
        s.cpu_topos = t["cpu_topos"].ctypes.data
        s.n_cpu_topos = len(t["cpu_topos"])
        if "cpu_alloc" in t:
            t["cpu_alloc"] = np.ascontiguousarray(t["cpu_alloc"], np.uint8)
            s.cpu_alloc = t["cpu_alloc"].ctypes.data
        for k in ("cpu_max_ref", "cpu_bind_policy", "cpu_strategy"):
            if k in t:
                t[k] = np.ascontiguousarray(t[k], np.uint8)
                setattr(s, k, t[k].ctypes.data_as(C.POINTER(C.c_uint8)))
    if "dev_topo" in t:
        t["dev_topo"] = np.ascontiguousarray(t["dev_topo"], np.uint64)
        s.dev_topo = t["dev_topo"].ctypes.data_as(C.POINTER(C.c_uint64))
    if "dev_part" in t:
        t["dev_part"] = np.ascontiguousarray(t["dev_part"], np.uint32)
        s.dev_part = _ptr(t["dev_part"], C.c_uint32)
    if "dev_numa" in t:
        t["dev_numa"] = np.ascontiguousarray(t["dev_numa"], np.uint32)
        s.dev_numa = _ptr(t["dev_numa"], C.c_uint32)
    if "numa_zone_pods" in t:
        t["numa_zone_pods"] = np.ascontiguousarray(t["numa_zone_pods"], np.uint64)
        s.numa_zone_pods = t["numa_zone_pods"].ctypes.data_as(C.POINTER(C.c_uint64))
    if "rsv_numa" in t:  # a reservation on the node holds a NUMA / cpuset allocation
        t["rsv_numa"] = np.ascontiguousarray(t["rsv_numa"], np.uint8)
        s.rsv_numa = t["rsv_numa"].ctypes.data_as(C.POINTER(C.c_uint8))
    if "gpu_parts" in t and len(t["gpu_parts"]):
        t["gpu_parts"] = np.ascontiguousarray(t["gpu_parts"], GPU_PARTITION_DTYPE)
        s.gpu_parts = t["gpu_parts"].ctypes.data
        s.n_gpu_parts = len(t["gpu_parts"])
    s._keep = t  # keep the buffers alive with the struct
    return s


def node_state_struct(t: Table) -> KgNodeState:
    s = KgNodeState()
    for k in ["req_cpu", "req_mem", "req_eph", "num_pods", "nz_cpu", "nz_mem"]:
        setattr(s, k, _ptr(t[k], C.c_int64))
    for k in range(KG_NSCALAR):
        s.sc_req[k] = _ptr(t[f"sc_req{k}"], C.c_int64)
    for name in ["la_fbase_np", "la_fbase_prod", "la_sbase_np", "la_sbase_prod"]:
        arr = getattr(s, name)
        for r in range(KG_LA_R):
            arr[r] = _ptr(t[f"{name}{r}"], C.c_int64)
    for name in ["zone_cpu_used", "zone_mem_used"]:
        arr = getattr(s, name)
        for z in range(KG_MAX_ZONES):
            arr[z] = _ptr(t[f"{name}{z}"], C.c_int64)
    if "dev_free" in t:
        s.dev_free = _ptr(t["dev_free"], C.c_int64)
    if "cpuset_alloc_milli" in t:
        s.cpuset_alloc_milli = _ptr(t["cpuset_alloc_milli"], C.c_int64)
    if "cpu_alloc" in t:
        s.cpu_alloc = t["cpu_alloc"].ctypes.data
    if "numa_zone_status" in t:
        s.numa_zone_status = _ptr(t["numa_zone_status"], C.c_uint32)
    if "numa_zone_pods" in t:
        s.numa_zone_pods = t["numa_zone_pods"].ctypes.data_as(C.POINTER(C.c_uint64))
    s._keep = t
    return s


def empty_node_state(n: int) -> Table:
    t = {k: np.zeros(n, np.int64) for k in NODE_STATE}
    t["dev_free"] = np.zeros((n, KG_DEV_R, KG_DEV_MINORS), np.int64)
    t["cpuset_alloc_milli"] = np.zeros(n, np.int64)
    t["cpu_alloc"] = np.zeros((n, 2 * KG_MAX_CPUS), np.uint8)
    t["numa_zone_status"] = np.zeros(n, np.uint32)
    t["numa_zone_pods"] = np.zeros(n, np.uint64)
    return t


def pod_columns(t: Table) -> KgPodColumns:
    _check(t, POD_I64, np.int64)
    _check(t, ["flags", "numa_policy"], np.uint32)
    s = KgPodColumns()
    for k in ["req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem"]:
        setattr(s, k, _ptr(t[k], C.c_int64))
    for k in range(KG_NSCALAR):
        s.sc_req[k] = _ptr(t[f"sc_req{k}"], C.c_int64)
    for r in range(KG_LA_R):
        s.la_est[r] = _ptr(t[f"la_est{r}"], C.c_int64)
    s.flags = _ptr(t["flags"], C.c_uint32)
    s.numa_policy = _ptr(t["numa_policy"], C.c_uint32)
    # config-5 columns are optional, each on its own (absent: no GPU request / quota / reservation class)
    _check(t, [k for k in POD_U32 + ["dev_flags", "dev_tmpl"] if k in t], np.uint32)
    _check(t, [k for k in POD_I32 if k in t], np.int32)
    if "dev_req" in t:
        t["dev_req"] = np.ascontiguousarray(t["dev_req"], np.int64)
        s.dev_req = _ptr(t["dev_req"], C.c_int64)
    for k, ct in (("dev_count", C.c_uint32), ("dev_keys", C.c_uint32), ("quota", C.c_int32),
                  ("quota_keys", C.c_uint32), ("rsv_class", C.c_int32), ("dev_flags", C.c_uint32),
                  ("dev_tmpl", C.c_uint32)):
        if k in t:
            setattr(s, k, _ptr(t[k], ct))
    if "dev_ring_bw" in t:
        t["dev_ring_bw"] = np.ascontiguousarray(t["dev_ring_bw"], np.int64)
        s.dev_ring_bw = _ptr(t["dev_ring_bw"], C.c_int64)
    s._keep = t
    return s


QUOTA_I64 = ["used", "used_limit", "min", "np_used"]     # [q][KG_QUOTA_R]
QUOTA_U32 = ["used_keys", "limit_keys", "min_keys", "np_used_keys"]


def empty_quotas(q: int) -> Table:
    t: Table = {k: np.zeros((q, KG_QUOTA_R), np.int64) for k in QUOTA_I64}
    t.update({k: np.zeros(q, np.uint32) for k in QUOTA_U32})
    return t


def quota_columns(t: Table) -> KgQuotaColumns:
    for k in QUOTA_I64:
        t[k] = np.ascontiguousarray(t[k], np.int64)
    for k in QUOTA_U32:
        t[k] = np.ascontiguousarray(t[k], np.uint32)
    s = KgQuotaColumns()
    for k in QUOTA_I64:
        setattr(s, k, _ptr(t[k], C.c_int64))
    for k in QUOTA_U32:
        setattr(s, k, _ptr(t[k], C.c_uint32))
    s._keep = t
    return s


class KgRsvGpu(C.Structure):
    """kg_rsv_gpu: DeviceShare restore inputs of a GPU-holding reservation (or, rid -1, of its node)."""
    _fields_ = [("node", C.c_uint32), ("rid", C.c_int32), ("policy", C.c_uint32), ("allocated_pods", C.c_uint32),
                ("a", (C.c_int64 * KG_DEV_MINORS) * KG_DEV_R), ("b", (C.c_int64 * KG_DEV_MINORS) * KG_DEV_R)]


class Reservations:
    """Reservation restore views and matched reservations (kg_rsv_view / kg_rsv_info arrays), their GPU restore tables
    and (gpu) the DeviceShare restore inputs of the GPU-holding reservations (kg_rsv_gpu dicts: node, rid, policy,
    allocated_pods, a, b)."""

    def __init__(self, views, infos, devs=(), gpu=()):
        self.views = (KgRsvView * max(1, len(views)))()
        self.infos = (KgRsvInfo * max(1, len(infos)))()
        self.devs = (KgRsvDev * max(1, len(devs)))()
        self.n_views, self.n_infos, self.n_devs = len(views), len(infos), len(devs)
        self.gpu = (KgRsvGpu * max(1, len(gpu)))()
        self.n_gpu = len(gpu)
        for x, g in enumerate(gpu):
            e = self.gpu[x]
            e.node, e.rid = int(g["node"]), int(g["rid"])
            e.policy, e.allocated_pods = int(g.get("policy", 0)), int(g.get("allocated_pods", 0))
            for key in ("a", "b"):
                t = np.asarray(g.get(key, np.zeros((KG_DEV_R, KG_DEV_MINORS))), np.int64).reshape(KG_DEV_R, KG_DEV_MINORS)
                arr = getattr(e, key)
                for r in range(KG_DEV_R):
                    for m in range(KG_DEV_MINORS):
                        arr[r][m] = int(t[r, m])
        for x in range(len(views)):
            self.views[x].dev_base = -1
        for x in range(len(infos)):
            self.infos[x].dev = -1
        for x, (tot, fr) in enumerate(devs):
            t = np.asarray(tot, np.int64).reshape(KG_DEV_R, KG_DEV_MINORS)
            f = np.asarray(fr, np.int64).reshape(KG_DEV_R, KG_DEV_MINORS)
            for r in range(KG_DEV_R):
                for m in range(KG_DEV_MINORS):
                    self.devs[x].total[r][m] = int(t[r, m])
                    self.devs[x].free[r][m] = int(f[r, m])
        for a, rows in ((self.views, views), (self.infos, infos)):
            for x, row in enumerate(rows):
                for k, v in row.items():
                    f = getattr(a[x], k)
                    if isinstance(f, int):
                        setattr(a[x], k, int(v))
                    else:
                        for q, y in enumerate(v):
                            f[q] = int(y)

    def view_list(self):
        return [self.views[x] for x in range(self.n_views)]

    def shard(self, lo: int, hi: int) -> "Reservations":
        """Views of nodes [lo, hi) re-indexed to the shard (matched reservations are shared)."""
        r = Reservations([], [])
        keep = [self.views[x] for x in range(self.n_views) if lo <= self.views[x].node < hi]
        r.views = (KgRsvView * max(1, len(keep)))()
        for x, v in enumerate(keep):
            C.pointer(r.views[x])[0] = v
            r.views[x].node = v.node - lo
        r.n_views = len(keep)
        r.infos, r.n_infos = self.infos, self.n_infos
        r.devs, r.n_devs = self.devs, self.n_devs
        keep_g = [self.gpu[x] for x in range(self.n_gpu) if lo <= self.gpu[x].node < hi]
        r.gpu = (KgRsvGpu * max(1, len(keep_g)))()
        for x, g in enumerate(keep_g):
            C.pointer(r.gpu[x])[0] = g
            r.gpu[x].node = g.node - lo
        r.n_gpu = len(keep_g)
        return r


class VerifyResult:
    """Host buffers of a verify-mode evaluation, [n_pods][n_nodes]."""

    def __init__(self, n_pods: int, n_nodes: int):
        shape = (n_pods, n_nodes)
        self.status = np.zeros(shape, np.uint32)
        self.score_nrf = np.zeros(shape, np.int64)
        self.score_la = np.zeros(shape, np.int64)
        self.score_numa = np.zeros(shape, np.int64)
        self.total = np.zeros(shape, np.int64)
        self.numa_zone = np.zeros(shape, np.int8)
        self.score_dev = np.zeros(shape, np.int64)
        self.score_rsv = np.zeros(shape, np.int64)

    def struct(self) -> KgVerifyOut:
        s = KgVerifyOut()
        s.status = _ptr(self.status, C.c_uint32)
        s.score_nrf = _ptr(self.score_nrf, C.c_int64)
        s.score_la = _ptr(self.score_la, C.c_int64)
        s.score_numa = _ptr(self.score_numa, C.c_int64)
        s.total = _ptr(self.total, C.c_int64)
        s.numa_zone = _ptr(self.numa_zone, C.c_int8)
        s.score_dev = _ptr(self.score_dev, C.c_int64)
        s.score_rsv = _ptr(self.score_rsv, C.c_int64)
        return s

    @property
    def feasible(self) -> np.ndarray:
        return self.status == 0


def make_key(total: int, node: int) -> int:
    return ((int(total) & 0xFFFFFFFF) << 32) | (0xFFFFFFFF - int(node))


def key_node(key) -> np.ndarray:
    key = np.asarray(key, np.uint64)
    out = (np.uint64(0xFFFFFFFF) - (key & np.uint64(0xFFFFFFFF))).astype(np.int64)
    return np.where(key == 0, -1, out)


def key_total(key) -> np.ndarray:
    key = np.asarray(key, np.uint64)
    return np.where(key == 0, -1, (key >> np.uint64(32)).astype(np.int64))
