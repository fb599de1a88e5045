"""ctypes binding of the CPU parity oracle (oracle/liboracle_kg.so). Test infrastructure only."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from koordinator_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle_kg.so")

_lib = None


class KgoPair(C.Structure):
    _fields_ = [("status", C.c_uint32), ("s_nrf", C.c_int64), ("s_la", C.c_int64), ("s_numa", C.c_int64),
                ("total", C.c_int64), ("zone", C.c_int32)]


class KgoExt(C.Structure):
    _fields_ = [("quotas", C.POINTER(abi.KgQuotaColumns)), ("n_quotas", C.c_uint32),
                ("views", C.POINTER(abi.KgRsvView)), ("n_views", C.c_uint32),
                ("infos", C.POINTER(abi.KgRsvInfo)), ("n_infos", C.c_uint32),
                ("devs", C.POINTER(abi.KgRsvDev)), ("n_devs", C.c_uint32),
                ("gpu", C.POINTER(abi.KgRsvGpu)), ("n_gpu", C.c_uint32)]


def make_ext(quotas=None, rsv=None) -> KgoExt:
    e = KgoExt()
    keep = []
    if quotas is not None:
        qc = abi.quota_columns(quotas)
        keep.append(qc)
        e.quotas = C.pointer(qc)
        e.n_quotas = len(quotas["used"])
    if rsv is not None:
        e.views = C.cast(rsv.views, C.POINTER(abi.KgRsvView))
        e.n_views = rsv.n_views
        e.infos = C.cast(rsv.infos, C.POINTER(abi.KgRsvInfo))
        e.n_infos = rsv.n_infos
        e.devs = C.cast(rsv.devs, C.POINTER(abi.KgRsvDev))
        e.n_devs = rsv.n_devs
        if getattr(rsv, "n_gpu", 0):
            e.gpu = C.cast(rsv.gpu, C.POINTER(abi.KgRsvGpu))
            e.n_gpu = rsv.n_gpu
        keep.append(rsv)
    e._keep = keep
    return e


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = C.CDLL(ORACLE_SO)
        P = C.POINTER
        L.kgo_eval_pair.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, P(abi.KgPodColumns), C.c_uint32,
                                    P(KgoPair)]
        L.kgo_eval_verify.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, P(abi.KgPodColumns),
                                      C.c_uint32, P(abi.KgVerifyOut)]
        L.kgo_select.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, C.c_uint32, P(abi.KgPodColumns),
                                 C.c_uint32, C.c_uint32, P(C.c_uint64)]
        L.kgo_select_parallel.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, C.c_uint32,
                                          P(abi.KgPodColumns), C.c_uint32, C.c_int, P(C.c_uint64)]
        L.kgo_select_parallel.restype = C.c_int
        L.kgo_state_new.argtypes = [P(abi.KgNodeColumns), C.c_uint32]
        L.kgo_state_new.restype = C.c_void_p
        L.kgo_state_free.argtypes = [C.c_void_p]
        L.kgo_state_view.argtypes = [C.c_void_p, P(abi.KgNodeColumns)]
        L.kgo_assume.argtypes = [P(abi.KgConfig), C.c_void_p, C.c_uint32, P(abi.KgPodColumns), C.c_uint32]
        L.kgo_assume.restype = C.c_int
        L.kgo_forget.argtypes = [P(abi.KgConfig), C.c_void_p, C.c_uint32, P(abi.KgPodColumns), C.c_uint32, C.c_int32]
        L.kgo_replay.argtypes = [P(abi.KgConfig), C.c_void_p, C.c_uint32, P(abi.KgPodColumns), C.c_uint32,
                                 P(C.c_int32), P(C.c_int64), P(C.c_uint32)]
        L.kgo_replay_parallel.argtypes = [P(abi.KgConfig), C.c_void_p, C.c_uint32, P(abi.KgPodColumns), C.c_uint32,
                                          C.c_int, P(C.c_int32), P(C.c_int64)]
        L.kgo_replay_parallel.restype = C.c_int
        L.kgo_ext_verify.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, P(abi.KgPodColumns),
                                     C.c_uint32, P(KgoExt), P(abi.KgVerifyOut)]
        L.kgo_ext_verify.restype = C.c_int
        L.kgo_ext_select.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, C.c_uint32,
                                     P(abi.KgPodColumns), C.c_uint32, P(KgoExt), C.c_uint32, P(C.c_uint64)]
        L.kgo_ext_select.restype = C.c_int
        L.kgo_ext_replay.argtypes = [P(abi.KgConfig), C.c_void_p, C.c_uint32, P(abi.KgPodColumns), C.c_uint32,
                                     P(KgoExt), P(C.c_int32), P(C.c_int64), P(C.c_uint32), P(C.c_int64),
                                     P(C.c_int64), P(C.c_uint32)]
        L.kgo_ext_replay.restype = C.c_int
        L.kgo_ext_replay_parallel.argtypes = L.kgo_ext_replay.argtypes + [C.c_int]
        L.kgo_ext_replay_parallel.restype = C.c_int
        L.kgo_ext_pair_nominated.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, C.c_uint32,
                                             P(abi.KgPodColumns), C.c_uint32, P(KgoExt)]
        L.kgo_ext_pair_nominated.restype = C.c_int64
        L.kgo_batch_schedule.argtypes = [P(abi.KgConfig), C.c_void_p, P(abi.KgPodColumns), C.c_uint32, P(KgoExt),
                                         P(C.c_int32), P(C.c_uint32), P(C.c_uint32), P(C.c_int32), P(C.c_uint32),
                                         P(C.c_int64), P(C.c_int64)]
        L.kgo_batch_schedule.restype = C.c_int
        L.kgo_take_cpus.argtypes = [P(abi.KgCpuTopo), C.c_int, P(C.c_uint64), P(abi.KgCpuAlloc), C.c_int, C.c_int,
                                    C.c_int, C.c_int, P(C.c_uint64)]
        L.kgo_take_cpus.restype = C.c_int
        L.kgo_take_preferred_cpus.argtypes = [P(abi.KgCpuTopo), C.c_int, P(C.c_uint64), P(C.c_uint64),
                                              P(abi.KgCpuAlloc), C.c_int, C.c_int, C.c_int, C.c_int, P(C.c_uint64)]
        L.kgo_take_preferred_cpus.restype = C.c_int
        L.kgo_ext_shard_stats.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, C.c_uint32,
                                          P(abi.KgPodColumns), C.c_uint32, P(KgoExt), P(C.c_uint32), P(C.c_uint32),
                                          P(C.c_uint64)]
        L.kgo_ext_shard_stats.restype = C.c_int
        L.kgo_ext_shard_select.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, C.c_uint32,
                                           P(abi.KgPodColumns), C.c_uint32, P(KgoExt), P(C.c_uint32), P(C.c_uint32),
                                           P(C.c_uint64), C.c_uint32, P(C.c_uint64)]
        L.kgo_ext_shard_select.restype = C.c_int
        L.kgo_gpu_numa_hints.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, P(abi.KgPodColumns),
                                         C.c_uint32, P(C.c_int), P(C.c_uint32), P(C.c_int), P(C.c_int64), P(C.c_uint32)]
        L.kgo_gpu_numa_hints.restype = C.c_int
        L.kgo_gpu_alloc_numa.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, P(abi.KgPodColumns),
                                         C.c_uint32, C.c_uint32, P(C.c_uint32)]
        L.kgo_gpu_alloc_numa.restype = C.c_uint32
        L.kgo_numa_allocate.argtypes = [P(abi.KgNodeColumns), C.c_uint32, P(abi.KgPodColumns), C.c_uint32, C.c_uint32,
                                        P(C.c_uint64), P(C.c_int64)]
        L.kgo_numa_allocate.restype = C.c_int
        L.kgo_numa_hints.argtypes = [P(abi.KgConfig), P(abi.KgNodeColumns), C.c_uint32, P(abi.KgPodColumns), C.c_uint32,
                                     C.c_uint32, P(C.c_uint32), P(C.c_int32)]
        L.kgo_numa_hints.restype = C.c_int
        L.kgo_reserve.argtypes = [P(abi.KgConfig), C.c_void_p, C.c_uint32, P(abi.KgPodColumns), C.c_uint32,
                                  P(abi.KgReserveRecord)]
        L.kgo_reserve.restype = C.c_int
        L.kgo_unreserve.argtypes = [P(abi.KgConfig), C.c_void_p, C.c_uint32, P(abi.KgPodColumns), C.c_uint32,
                                    P(abi.KgReserveRecord)]
        L.kgo_ext_session_new.argtypes = [P(abi.KgConfig), C.c_void_p, P(KgoExt)]
        L.kgo_ext_session_new.restype = C.c_void_p
        L.kgo_ext_session_free.argtypes = [C.c_void_p]
        L.kgo_ext_session_filter.argtypes = [C.c_void_p, C.c_uint32, P(abi.KgPodColumns), C.c_uint32]
        L.kgo_ext_session_filter.restype = C.c_uint32
        L.kgo_ext_reserve.argtypes = [C.c_void_p, C.c_uint32, P(abi.KgPodColumns), C.c_uint32, P(abi.KgReserveRecord)]
        L.kgo_ext_reserve.restype = C.c_int
        L.kgo_ext_unreserve.argtypes = [C.c_void_p, C.c_uint32, P(abi.KgPodColumns), C.c_uint32, P(abi.KgReserveRecord)]
        L.kgo_ext_unreserve.restype = C.c_int
        L.kgo_ext_session_read.argtypes = [C.c_void_p, P(abi.KgRsvView), P(abi.KgRsvInfo), P(abi.KgRsvDev), P(C.c_int64),
                                           P(C.c_int64)]
        L.kgo_mem_bytes_to_ratio.argtypes = [C.c_int64, C.c_int64]
        L.kgo_mem_bytes_to_ratio.restype = C.c_int64
        L.kgo_amplify.argtypes = [C.c_int64, C.c_double]
        L.kgo_amplify.restype = C.c_int64
        L.kgo_la_usage_percent.argtypes = [C.c_int64, C.c_int64]
        L.kgo_la_usage_percent.restype = C.c_int64
        _lib = L
    return _lib


def take_cpus(topo, max_ref, avail, alloc, needed, bind, excl, strategy, preferred=None):
    """kgo_take_cpus / kgo_take_preferred_cpus: (rc, cpus)."""
    out = np.zeros(4, np.uint64)
    av = np.ascontiguousarray(avail, np.uint64)
    P = C.POINTER
    if preferred is None:
        rc = lib().kgo_take_cpus(C.byref(topo), max_ref, av.ctypes.data_as(P(C.c_uint64)),
                                 C.byref(alloc) if alloc is not None else None, needed, bind, excl, strategy,
                                 out.ctypes.data_as(P(C.c_uint64)))
    else:
        pf = np.ascontiguousarray(preferred, np.uint64)
        rc = lib().kgo_take_preferred_cpus(C.byref(topo), max_ref, av.ctypes.data_as(P(C.c_uint64)),
                                           pf.ctypes.data_as(P(C.c_uint64)),
                                           C.byref(alloc) if alloc is not None else None, needed, bind, excl, strategy,
                                           out.ctypes.data_as(P(C.c_uint64)))
    return rc, abi.mask_cpus(out)


def eval_pair(cfg, nodes: abi.Table, i: int, pods: abi.Table, j: int) -> KgoPair:
    out = KgoPair()
    nc, pc = abi.node_columns(nodes), abi.pod_columns(pods)
    lib().kgo_eval_pair(C.byref(cfg), C.byref(nc), i, C.byref(pc), j, C.byref(out))
    return out


def eval_verify(cfg, nodes: abi.Table, pods: abi.Table) -> abi.VerifyResult:
    nn, np_ = abi.table_len(nodes), abi.table_len(pods)
    res = abi.VerifyResult(np_, nn)
    nc, pc, vo = abi.node_columns(nodes), abi.pod_columns(pods), res.struct()
    lib().kgo_eval_verify(C.byref(cfg), C.byref(nc), nn, C.byref(pc), np_, C.byref(vo))
    return res


def select(cfg, nodes: abi.Table, pods: abi.Table, k: int = 1, index_base: int = 0) -> np.ndarray:
    nn, np_ = abi.table_len(nodes), abi.table_len(pods)
    keys = np.zeros((np_, k), np.uint64)
    nc, pc = abi.node_columns(nodes), abi.pod_columns(pods)
    lib().kgo_select(C.byref(cfg), C.byref(nc), nn, index_base, C.byref(pc), np_, k,
                     keys.ctypes.data_as(C.POINTER(C.c_uint64)))
    return keys


def select_parallel(cfg, nodes: abi.Table, pods: abi.Table, workers: int = 16, index_base: int = 0) -> np.ndarray:
    nn, np_ = abi.table_len(nodes), abi.table_len(pods)
    keys = np.zeros(np_, np.uint64)
    nc, pc = abi.node_columns(nodes), abi.pod_columns(pods)
    rc = lib().kgo_select_parallel(C.byref(cfg), C.byref(nc), nn, index_base, C.byref(pc), np_, workers,
                                   keys.ctypes.data_as(C.POINTER(C.c_uint64)))
    assert rc == 0
    return keys


def ext_verify(cfg, nodes: abi.Table, pods: abi.Table, quotas=None, rsv=None) -> abi.VerifyResult:
    nn, np_ = abi.table_len(nodes), abi.table_len(pods)
    res = abi.VerifyResult(np_, nn)
    nc, pc, vo, e = abi.node_columns(nodes), abi.pod_columns(pods), res.struct(), make_ext(quotas, rsv)
    assert lib().kgo_ext_verify(C.byref(cfg), C.byref(nc), nn, C.byref(pc), np_, C.byref(e), C.byref(vo)) == 0
    return res


def gpu_numa_hints(cfg, nodes: abi.Table, pods: abi.Table, node: int = 0, pod: int = 0):
    """DeviceShare's NUMA hint provider (kgo_gpu_numa_hints): ("hints", [(mask, preferred, score)]),
    ("nopref", None) or ("fail", KG_DEV_CODE_*)."""
    nc, pc = abi.node_columns(nodes), abi.pod_columns(pods)
    n = C.c_int(0)
    code = C.c_uint32(0)
    masks, pref, scores = np.zeros(15, np.uint32), np.zeros(15, np.int32), np.zeros(15, np.int64)
    P = C.POINTER
    r = lib().kgo_gpu_numa_hints(C.byref(cfg), C.byref(nc), node, C.byref(pc), pod, C.byref(n),
                                 masks.ctypes.data_as(P(C.c_uint32)), pref.ctypes.data_as(P(C.c_int)),
                                 scores.ctypes.data_as(P(C.c_int64)), C.byref(code))
    if r == 2:
        return "fail", int(code.value)
    if r == 1:
        return "nopref", None
    return "hints", [(int(masks[t]), bool(pref[t]), int(scores[t])) for t in range(n.value)]


def gpu_alloc_numa(cfg, nodes: abi.Table, pods: abi.Table, numa: int, node: int = 0, pod: int = 0):
    """DeviceShare's Allocate under a NUMA affinity: (KG_DEV_CODE_* or 0, minors mask)."""
    nc, pc = abi.node_columns(nodes), abi.pod_columns(pods)
    minors = C.c_uint32(0)
    code = lib().kgo_gpu_alloc_numa(C.byref(cfg), C.byref(nc), node, C.byref(pc), pod, numa, C.byref(minors))
    return int(code), int(minors.value)


def numa_hints(cfg, nodes: abi.Table, pods: abi.Table, policy: int, node: int = 0, pod: int = 0):
    """NodeNUMAResource's hint lists of the requested resources (cpu, then memory): [[(mask, preferred)]]; an empty
    list for a resource without hints."""
    nc, pc = abi.node_columns(nodes), abi.pod_columns(pods)
    out = np.zeros(32, np.uint32)
    ln = np.zeros(2, np.int32)
    n = lib().kgo_numa_hints(C.byref(cfg), C.byref(nc), node, C.byref(pc), pod, policy,
                             out.ctypes.data_as(C.POINTER(C.c_uint32)), ln.ctypes.data_as(C.POINTER(C.c_int32)))
    lists = []
    for li in range(max(n, 0)):
        hs = [int(v) for v in out[16 * li:16 * li + ln[li]]]
        lists.append([] if len(hs) == 1 and hs[0] & 0x200 else [(h & 0xFF, bool(h & 0x100)) for h in hs])
    return lists


def numa_allocate(nodes: abi.Table, pods: abi.Table, mask: int, node: int = 0, pod: int = 0):
    """resourceManager.Allocate under a NUMA affinity: (ok, CPUs of a cpuset-binding pod, split [resource][zone])."""
    nc, pc = abi.node_columns(nodes), abi.pod_columns(pods)
    cpus = np.zeros(4, np.uint64)
    al = np.zeros(2 * abi.KG_MAX_ZONES, np.int64)
    rc = lib().kgo_numa_allocate(C.byref(nc), node, C.byref(pc), pod, mask, cpus.ctypes.data_as(C.POINTER(C.c_uint64)),
                                 al.ctypes.data_as(C.POINTER(C.c_int64)))
    return rc == 0, abi.mask_cpus(cpus), al.reshape(2, abi.KG_MAX_ZONES)


def ext_select(cfg, nodes: abi.Table, pods: abi.Table, k: int = 1, index_base: int = 0, quotas=None,
               rsv=None) -> np.ndarray:
    nn, np_ = abi.table_len(nodes), abi.table_len(pods)
    keys = np.zeros((np_, k), np.uint64)
    nc, pc, e = abi.node_columns(nodes), abi.pod_columns(pods), make_ext(quotas, rsv)
    assert lib().kgo_ext_select(C.byref(cfg), C.byref(nc), nn, index_base, C.byref(pc), np_, C.byref(e), k,
                                keys.ctypes.data_as(C.POINTER(C.c_uint64))) == 0
    return keys


def ext_shard_stats(cfg, nodes: abi.Table, pods: abi.Table, index_base: int, quotas=None, rsv=None):
    nn, np_ = abi.table_len(nodes), abi.table_len(pods)
    dm, rm, pf = np.zeros(np_, np.uint32), np.zeros(np_, np.uint32), np.zeros(np_, np.uint64)
    nc, pc, e = abi.node_columns(nodes), abi.pod_columns(pods), make_ext(quotas, rsv)
    P = C.POINTER
    assert lib().kgo_ext_shard_stats(C.byref(cfg), C.byref(nc), nn, index_base, C.byref(pc), np_, C.byref(e),
                                     dm.ctypes.data_as(P(C.c_uint32)), rm.ctypes.data_as(P(C.c_uint32)),
                                     pf.ctypes.data_as(P(C.c_uint64))) == 0
    return dm, rm, pf


def ext_shard_select(cfg, nodes: abi.Table, pods: abi.Table, index_base: int, dm, rm, pf, k: int = 1, quotas=None,
                     rsv=None) -> np.ndarray:
    nn, np_ = abi.table_len(nodes), abi.table_len(pods)
    keys = np.zeros((np_, k), np.uint64)
    nc, pc, e = abi.node_columns(nodes), abi.pod_columns(pods), make_ext(quotas, rsv)
    P = C.POINTER
    dm, rm, pf = (np.ascontiguousarray(x) for x in (dm, rm, pf))
    assert lib().kgo_ext_shard_select(C.byref(cfg), C.byref(nc), nn, index_base, C.byref(pc), np_, C.byref(e),
                                      dm.ctypes.data_as(P(C.c_uint32)), rm.ctypes.data_as(P(C.c_uint32)),
                                      pf.ctypes.data_as(P(C.c_uint64)), k, keys.ctypes.data_as(P(C.c_uint64))) == 0
    return keys


class OracleState:
    """Mutable oracle snapshot for Assume / replay."""

    def __init__(self, cfg, nodes: abi.Table):
        self.cfg = cfg
        self.n = abi.table_len(nodes)
        nc = abi.node_columns(nodes)
        self.h = lib().kgo_state_new(C.byref(nc), self.n)

    def __del__(self):
        if getattr(self, "h", None):
            lib().kgo_state_free(self.h)
            self.h = None

    def assume(self, node: int, pods: abi.Table, pod: int) -> bool:
        """Reserve; False when the NodeNUMAResource Reserve fails (nothing applied)."""
        pc = abi.pod_columns(pods)
        return lib().kgo_assume(C.byref(self.cfg), self.h, node, C.byref(pc), pod) == 0

    def forget(self, node: int, pods: abi.Table, pod: int, zone: int):
        pc = abi.pod_columns(pods)
        lib().kgo_forget(C.byref(self.cfg), self.h, node, C.byref(pc), pod, zone)

    def reserve(self, node: int, pods: abi.Table, pod: int):
        """kgo_reserve: (ok, record)."""
        pc = abi.pod_columns(pods)
        rec = abi.KgReserveRecord()
        rc = lib().kgo_reserve(C.byref(self.cfg), self.h, node, C.byref(pc), pod, C.byref(rec))
        assert rc >= 0
        return rc == 0, rec

    def unreserve(self, node: int, pods: abi.Table, pod: int, rec):
        pc = abi.pod_columns(pods)
        lib().kgo_unreserve(C.byref(self.cfg), self.h, node, C.byref(pc), pod, C.byref(rec))

    def replay(self, pods: abi.Table, index_base: int = 0, reasons: bool = False):
        np_ = abi.table_len(pods)
        out_node = np.zeros(np_, np.int32)
        out_total = np.zeros(np_, np.int64)
        out_reason = np.zeros(np_, np.uint32)
        pc = abi.pod_columns(pods)
        lib().kgo_replay(C.byref(self.cfg), self.h, index_base, C.byref(pc), np_,
                         out_node.ctypes.data_as(C.POINTER(C.c_int32)), out_total.ctypes.data_as(C.POINTER(C.c_int64)),
                         out_reason.ctypes.data_as(C.POINTER(C.c_uint32)))
        return (out_node, out_total, out_reason) if reasons else (out_node, out_total)

    def replay_parallel(self, pods: abi.Table, workers: int = 16, index_base: int = 0):
        """The replay CPU baseline: each cycle's Filter / Score on the 16-worker parallelizer."""
        np_ = abi.table_len(pods)
        out_node = np.zeros(np_, np.int32)
        out_total = np.zeros(np_, np.int64)
        pc = abi.pod_columns(pods)
        rc = lib().kgo_replay_parallel(C.byref(self.cfg), self.h, index_base, C.byref(pc), np_, workers,
                                       out_node.ctypes.data_as(C.POINTER(C.c_int32)),
                                       out_total.ctypes.data_as(C.POINTER(C.c_int64)))
        assert rc == 0
        return out_node, out_total

    def ext_replay(self, pods: abi.Table, quotas=None, index_base: int = 0, reasons: bool = False, rsv=None,
                   workers: int = 1):
        """kgo_ext_replay (workers > 1: kgo_ext_replay_parallel, each cycle's nodes on worker threads)."""
        np_ = abi.table_len(pods)
        out_node = np.zeros(np_, np.int32)
        out_total = np.zeros(np_, np.int64)
        out_minors = np.zeros(np_, np.uint32)
        out_reason = np.zeros(np_, np.uint32)
        nq = len(quotas["used"]) if quotas is not None else 0
        qu = np.zeros((max(nq, 1), abi.KG_QUOTA_R), np.int64)
        qn = np.zeros((max(nq, 1), abi.KG_QUOTA_R), np.int64)
        pc, e = abi.pod_columns(pods), make_ext(quotas, rsv)
        P = C.POINTER
        args = (C.byref(self.cfg), self.h, index_base, C.byref(pc), np_, C.byref(e),
                out_node.ctypes.data_as(P(C.c_int32)), out_total.ctypes.data_as(P(C.c_int64)),
                out_minors.ctypes.data_as(P(C.c_uint32)), qu.ctypes.data_as(P(C.c_int64)),
                qn.ctypes.data_as(P(C.c_int64)), out_reason.ctypes.data_as(P(C.c_uint32)))
        rc = lib().kgo_ext_replay_parallel(*args, int(workers)) if workers > 1 else lib().kgo_ext_replay(*args)
        assert rc == 0
        if reasons:
            return out_node, out_total, out_minors, qu[:nq], qn[:nq], out_reason
        return out_node, out_total, out_minors, qu[:nq], qn[:nq]

    def batch_schedule(self, pods: abi.Table, plan_node, quotas=None, rsv=None):
        """kgo_batch_schedule: (result codes, status bits, zone, minors, quota used, quota np_used)."""
        np_ = abi.table_len(pods)
        plan = np.ascontiguousarray(plan_node, np.int32)
        res = np.zeros(np_, np.uint32)
        stat = np.zeros(np_, np.uint32)
        zone = np.zeros(np_, np.int32)
        minors = np.zeros(np_, np.uint32)
        nq = len(quotas["used"]) if quotas is not None else 0
        qu = np.zeros((max(nq, 1), abi.KG_QUOTA_R), np.int64)
        qn = np.zeros((max(nq, 1), abi.KG_QUOTA_R), np.int64)
        pc, e = abi.pod_columns(pods), make_ext(quotas, rsv)
        P = C.POINTER
        rc = lib().kgo_batch_schedule(C.byref(self.cfg), self.h, C.byref(pc), np_, C.byref(e),
                                      plan.ctypes.data_as(P(C.c_int32)), res.ctypes.data_as(P(C.c_uint32)),
                                      stat.ctypes.data_as(P(C.c_uint32)), zone.ctypes.data_as(P(C.c_int32)),
                                      minors.ctypes.data_as(P(C.c_uint32)), qu.ctypes.data_as(P(C.c_int64)),
                                      qn.ctypes.data_as(P(C.c_int64)))
        assert rc == 0
        return res, stat, zone, minors, qu[:nq], qn[:nq]

    def dev_free(self) -> np.ndarray:
        v = abi.KgNodeColumns()
        lib().kgo_state_view(self.h, C.byref(v))
        if not v.dev_free:
            return None
        return np.ctypeslib.as_array(v.dev_free, shape=(self.n, abi.KG_DEV_R, abi.KG_DEV_MINORS)).copy()

    def table(self) -> abi.Table:
        """Copy of the current node columns."""
        v = abi.KgNodeColumns()
        lib().kgo_state_view(self.h, C.byref(v))
        n = self.n
        t = {}

        def grab(ptr, dtype):
            return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)

        for k in ["alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "req_cpu", "req_mem", "req_eph", "num_pods",
                  "nz_cpu", "nz_mem", "cpuset_alloc_milli"]:
            t[k] = grab(getattr(v, k), np.int64)
        for k in range(abi.KG_NSCALAR):
            t[f"sc_alloc{k}"] = grab(v.sc_alloc[k], np.int64)
            t[f"sc_req{k}"] = grab(v.sc_req[k], np.int64)
        for name in ["la_alloc", "la_thr_usage", "la_thr_prod", "la_thr_agg", "la_fbase_np", "la_fbase_prod",
                     "la_sbase_np", "la_sbase_prod"]:
            for r in range(abi.KG_LA_R):
                t[f"{name}{r}"] = grab(getattr(v, name)[r], np.int64)
        for name in ["zone_cpu", "zone_mem", "zone_cpu_used", "zone_mem_used"]:
            for z in range(abi.KG_MAX_ZONES):
                t[f"{name}{z}"] = grab(getattr(v, name)[z], np.int64)
        t["la_flags"] = grab(v.la_flags, np.uint32)
        t["numa_policy"] = grab(v.numa_policy, np.uint32)
        t["numa_zones"] = grab(v.numa_zones, np.uint32)
        t["numa_zone_status"] = grab(v.numa_zone_status, np.uint32)
        t["numa_zone_pods"] = grab(v.numa_zone_pods, np.uint64)
        t["cpu_amp_ratio"] = grab(v.cpu_amp_ratio, np.float64)
        df = self.dev_free()
        t["dev_free"] = df if df is not None else np.zeros((n, abi.KG_DEV_R, abi.KG_DEV_MINORS), np.int64)
        if v.cpu_alloc:
            raw = C.string_at(v.cpu_alloc, n * 2 * abi.KG_MAX_CPUS)
            t["cpu_alloc"] = np.frombuffer(raw, np.uint8).reshape(n, 2 * abi.KG_MAX_CPUS).copy()
        return t


class ExtSession:
    """kgo_ext_session: Reserve / Unreserve with every config-5 plugin (NodeInfo, LoadAware, NUMA incl. cpusets,
    DeviceShare with the GPU restore, ElasticQuota, Reservation) over an OracleState, the oracle side of
    kg_reserve / kg_unreserve."""

    def __init__(self, state: OracleState, quotas=None, rsv=None):
        self.state = state
        self.rsv = rsv
        self.nq = len(quotas["used"]) if quotas is not None else 0
        self.e = make_ext(quotas, rsv)
        self.h = lib().kgo_ext_session_new(C.byref(state.cfg), state.h, C.byref(self.e))
        assert self.h, "GPU-holding reservations without their restore inputs"

    def __del__(self):
        if getattr(self, "h", None):
            lib().kgo_ext_session_free(self.h)
            self.h = None

    def filter(self, node: int, pods: abi.Table, pod: int) -> int:
        """The pair's Filter status bits on the current state (0 = feasible; a failing Reserve's NUMA bits too)."""
        pc = abi.pod_columns(pods)
        return int(lib().kgo_ext_session_filter(self.h, node, C.byref(pc), pod))

    def reserve(self, node: int, pods: abi.Table, pod: int):
        """(ok, record); ok False when the NodeNUMAResource Reserve fails (nothing applied)."""
        pc = abi.pod_columns(pods)
        rec = abi.KgReserveRecord()
        rc = lib().kgo_ext_reserve(self.h, node, C.byref(pc), pod, C.byref(rec))
        return rc == 0, rec

    def unreserve(self, node: int, pods: abi.Table, pod: int, rec) -> bool:
        """False (nothing applied) for a record already given back."""
        pc = abi.pod_columns(pods)
        return lib().kgo_ext_unreserve(self.h, node, C.byref(pc), pod, C.byref(rec)) == 0

    def read_reservations(self) -> abi.Reservations:
        """The views / infos / GPU restore tables as the session holds them, in the layout of the uploaded rsv."""
        r = self.rsv
        out = abi.Reservations([], [])
        out.views = (abi.KgRsvView * max(1, r.n_views))()
        out.infos = (abi.KgRsvInfo * max(1, r.n_infos))()
        out.devs = (abi.KgRsvDev * max(1, r.n_devs))()
        out.n_views, out.n_infos, out.n_devs = r.n_views, r.n_infos, r.n_devs
        lib().kgo_ext_session_read(self.h, out.views, out.infos, out.devs, None, None)
        return out

    def read_quotas(self):
        used = np.zeros((max(self.nq, 1), abi.KG_QUOTA_R), np.int64)
        npu = np.zeros((max(self.nq, 1), abi.KG_QUOTA_R), np.int64)
        P = C.POINTER
        lib().kgo_ext_session_read(self.h, None, None, None, used.ctypes.data_as(P(C.c_int64)),
                                   npu.ctypes.data_as(P(C.c_int64)))
        return used[:self.nq], npu[:self.nq]


def assert_state_restored(before, after):
    """Every column of `after` equals `before`, except the allocation records of numa_zone_status (bits
    KG_ZONE_RECORD_SHIFT + z), which Unreserve leaves in place (resource_manager.go:478-483 Release keeps the zone's
    allocatedResources entry): those may only have been added."""
    from koordinator_amd import abi
    low = np.uint32((1 << abi.KG_ZONE_RECORD_SHIFT) - 1)
    for k in before:
        if k == "numa_zone_status":
            assert np.array_equal(before[k] & low, after[k] & low), k
            assert not (before[k] & ~after[k]).any(), k
        else:
            assert np.array_equal(before[k], after[k]), k


def ext_pair_nominated(kc, nodes, i, pods, j, quotas=None, rsv=None) -> int:
    """kgo_ext_pair_nominated: the reservation (index into rsv's infos) pod j is nominated to on node i, -1 = none."""
    nc, pc, e = abi.node_columns(nodes), abi.pod_columns(pods), make_ext(quotas, rsv)
    return int(lib().kgo_ext_pair_nominated(C.byref(kc), C.byref(nc), abi.table_len(nodes), i, C.byref(pc), j,
                                            C.byref(e)))
