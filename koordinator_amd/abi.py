"""ctypes mirror of include/koordgpu.h plus numpy column tables.

The node and pod tables are plain dicts of numpy arrays keyed by the column names below; the
helpers turn them into the C structs of the boundary (pointers into the numpy buffers, which the
caller keeps alive for the duration of the call).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict

import numpy as np

KG_ABI_VERSION = 1
KG_LA_R = 2
KG_NSCALAR = 2
KG_MAX_ZONES = 4

KG_OK, KG_INVALID_ARG, KG_DEVICE_ERROR, KG_OOM, KG_UNSUPPORTED, KG_NO_DEVICE = range(6)

KG_PLUGIN_NRF = 0x1
KG_PLUGIN_LA = 0x2
KG_PLUGIN_NUMA = 0x4

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

KG_ST_NRF_PODS = 0x1
KG_ST_NRF_CPU = 0x2
KG_ST_NRF_MEM = 0x4
KG_ST_NRF_EPH = 0x8
KG_ST_NRF_SC0 = 0x10
KG_ST_NRF_SC1 = 0x20
KG_ST_NRF_MASK = 0xFF
KG_ST_LA_EXPIRED = 0x100
KG_ST_LA_CPU = 0x200
KG_ST_LA_MEM = 0x400
KG_ST_LA_AGG = 0x800
KG_ST_LA_MASK = 0xFF00
KG_ST_NUMA_AMP_CPU = 0x10000
KG_ST_NUMA_CONFLICT = 0x20000
KG_ST_NUMA_NO_RES = 0x40000
KG_ST_NUMA_ALIGN = 0x80000
KG_ST_NUMA_MASK = 0xFF0000
KG_ST_UNSUPPORTED = 0x80000000

_p64 = C.POINTER(C.c_int64)
_pu32 = C.POINTER(C.c_uint32)
_pf64 = C.POINTER(C.c_double)


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
    ]


class KgNodeState(C.Structure):
    _fields_ = [
        ("req_cpu", _p64), ("req_mem", _p64), ("req_eph", _p64), ("num_pods", _p64),
        ("nz_cpu", _p64), ("nz_mem", _p64),
        ("sc_req", _p64 * KG_NSCALAR),
        ("la_fbase_np", _p64 * KG_LA_R), ("la_fbase_prod", _p64 * KG_LA_R),
        ("la_sbase_np", _p64 * KG_LA_R), ("la_sbase_prod", _p64 * KG_LA_R),
        ("zone_cpu_used", _p64 * KG_MAX_ZONES), ("zone_mem_used", _p64 * KG_MAX_ZONES),
    ]


class KgPodColumns(C.Structure):
    _fields_ = [
        ("req_cpu", _p64), ("req_mem", _p64), ("req_eph", _p64),
        ("sc_req", _p64 * KG_NSCALAR),
        ("nz_cpu", _p64), ("nz_mem", _p64),
        ("la_est", _p64 * KG_LA_R),
        ("flags", _pu32),
        ("numa_policy", _pu32),
    ]


class KgVerifyOut(C.Structure):
    _fields_ = [
        ("status", _pu32),
        ("score_nrf", _p64),
        ("score_la", _p64),
        ("score_numa", _p64),
        ("total", _p64),
        ("numa_zone", C.POINTER(C.c_int8)),
    ]


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
NODE_U32 = ["la_flags", "numa_policy", "numa_zones"]
NODE_F64 = ["cpu_amp_ratio"]

NODE_STATE = (
    ["req_cpu", "req_mem", "req_eph", "num_pods", "nz_cpu", "nz_mem"] + _indexed("sc_req", KG_NSCALAR)
    + _indexed("la_fbase_np", KG_LA_R) + _indexed("la_fbase_prod", KG_LA_R)
    + _indexed("la_sbase_np", KG_LA_R) + _indexed("la_sbase_prod", KG_LA_R)
    + _indexed("zone_cpu_used", KG_MAX_ZONES) + _indexed("zone_mem_used", KG_MAX_ZONES)
)

POD_I64 = (["req_cpu", "req_mem", "req_eph"] + _indexed("sc_req", KG_NSCALAR) + ["nz_cpu", "nz_mem"]
           + _indexed("la_est", KG_LA_R))
POD_U32 = ["flags", "numa_policy"]

Table = Dict[str, np.ndarray]


def empty_nodes(n: int) -> Table:
    t: Table = {k: np.zeros(n, np.int64) for k in NODE_I64}
    t.update({k: np.zeros(n, np.uint32) for k in NODE_U32})
    t["cpu_amp_ratio"] = np.zeros(n, np.float64)
    return t


def empty_pods(n: int) -> Table:
    t: Table = {k: np.zeros(n, np.int64) for k in POD_I64}
    t.update({k: np.zeros(n, np.uint32) for k in POD_U32})
    return t


def table_len(t: Table) -> int:
    return int(len(next(iter(t.values()))))


def concat(tables) -> Table:
    keys = tables[0].keys()
    return {k: np.concatenate([t[k] for t in tables]) for k in keys}


def take(t: Table, idx) -> Table:
    return {k: np.ascontiguousarray(v[idx]) for k, v in t.items()}


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def _check(t: Table, names, dtype):
    for k in names:
        a = t[k]
        if a.dtype != dtype or not a.flags["C_CONTIGUOUS"]:
            t[k] = np.ascontiguousarray(a, dtype=dtype)


def node_columns(t: Table) -> KgNodeColumns:
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
    s.cpu_amp_ratio = _ptr(t["cpu_amp_ratio"], C.c_double)
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
    s._keep = t
    return s


def empty_node_state(n: int) -> Table:
    return {k: np.zeros(n, np.int64) for k in NODE_STATE}


def pod_columns(t: Table) -> KgPodColumns:
    _check(t, POD_I64, np.int64)
    _check(t, POD_U32, np.uint32)
    s = KgPodColumns()
    for k in ["req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem"]:
        setattr(s, k, _ptr(t[k], C.c_int64))
    for k in range(KG_NSCALAR):
        s.sc_req[k] = _ptr(t[f"sc_req{k}"], C.c_int64)
    for r in range(KG_LA_R):
        s.la_est[r] = _ptr(t[f"la_est{r}"], C.c_int64)
    s.flags = _ptr(t["flags"], C.c_uint32)
    s.numa_policy = _ptr(t["numa_policy"], C.c_uint32)
    s._keep = t
    return s


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

    def struct(self) -> KgVerifyOut:
        s = KgVerifyOut()
        s.status = _ptr(self.status, C.c_uint32)
        s.score_nrf = _ptr(self.score_nrf, C.c_int64)
        s.score_la = _ptr(self.score_la, C.c_int64)
        s.score_numa = _ptr(self.score_numa, C.c_int64)
        s.total = _ptr(self.total, C.c_int64)
        s.numa_zone = _ptr(self.numa_zone, C.c_int8)
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
