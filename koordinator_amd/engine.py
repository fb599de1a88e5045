"""Python binding of libkoordgpu.so (the C ABI of include/koordgpu.h) over ctypes.

This is the product path: every evaluation runs the HIP kernels through the library. There is no
CPU fallback — if the library is missing or no device is present the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref
from typing import Optional

import numpy as np

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
# KG_LIB_PATH: A/B measurements of alternative builds (tools/); the product loads the in-tree library
LIB_PATH = os.environ.get("KG_LIB_PATH") or os.path.join(HERE, "libkoordgpu.so")

_lib = None


class EngineError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"koordgpu: {msg} (status {status})")
        self.status = status


class Unsupported(EngineError):
    pass


class ReserveFailed(EngineError):
    """kg_assume / kg_assume_ext: the NodeNUMAResource Reserve fails on that node (BestEffort allocation)."""


def lib():
    """Load libkoordgpu.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    P, u32, i32, i64, u64, vp = C.POINTER, C.c_uint32, C.c_int32, C.c_int64, C.c_uint64, C.c_void_p
    st = C.c_int
    L.kg_abi_version.restype = C.c_int
    L.kg_status_string.argtypes = [st]
    L.kg_status_string.restype = C.c_char_p
    L.kg_device_count.restype = C.c_int
    L.kg_open.argtypes = [C.c_int, P(vp)]
    L.kg_open.restype = st
    L.kg_close.argtypes = [vp]
    L.kg_close.restype = st
    L.kg_last_error.argtypes = [vp]
    L.kg_last_error.restype = C.c_char_p
    L.kg_sync.argtypes = [vp]
    L.kg_sync.restype = st
    L.kg_snapshot_create.argtypes = [vp, P(abi.KgConfig), u32, u32, P(vp)]
    L.kg_snapshot_create.restype = st
    L.kg_snapshot_upload.argtypes = [vp, P(abi.KgNodeColumns)]
    L.kg_snapshot_upload.restype = st
    L.kg_snapshot_update_rows.argtypes = [vp, P(u32), u32, P(abi.KgNodeColumns)]
    L.kg_snapshot_update_rows.restype = st
    L.kg_snapshot_generation.argtypes = [vp, P(C.c_uint64)]
    L.kg_snapshot_generation.restype = st
    L.kg_snapshot_read_state.argtypes = [vp, P(abi.KgNodeState)]
    L.kg_snapshot_read_state.restype = st
    L.kg_snapshot_destroy.argtypes = [vp]
    L.kg_snapshot_destroy.restype = st
    L.kg_pods_create.argtypes = [vp, u32, P(vp)]
    L.kg_pods_create.restype = st
    L.kg_pods_upload.argtypes = [vp, P(abi.KgPodColumns), u32]
    L.kg_pods_upload.restype = st
    L.kg_pods_destroy.argtypes = [vp]
    L.kg_pods_destroy.restype = st
    L.kg_eval_verify.argtypes = [vp, vp, P(abi.KgVerifyOut)]
    L.kg_eval_verify.restype = st
    L.kg_eval_select.argtypes = [vp, vp, u32]
    L.kg_eval_select.restype = st
    L.kg_result_keys.argtypes = [vp, P(u64)]
    L.kg_result_keys.restype = st
    L.kg_result_status.argtypes = [vp, P(u32)]
    L.kg_result_status.restype = st
    L.kg_replay.argtypes = [vp, vp, P(i32), P(i64), P(u32)]
    L.kg_replay.restype = st
    L.kg_assume.argtypes = [vp, vp, u32, u32]
    L.kg_assume.restype = st
    L.kg_forget.argtypes = [vp, vp, u32, u32, i32]
    L.kg_forget.restype = st
    L.kg_assume_numa.argtypes = [vp, vp, u32, u32, P(i32), P(C.c_int64)]
    L.kg_assume_numa.restype = st
    L.kg_forget_numa.argtypes = [vp, vp, u32, u32, i32, P(C.c_int64)]
    L.kg_forget_numa.restype = st
    L.kg_profile_enable.argtypes = [vp, C.c_int]
    L.kg_profile_enable.restype = st
    L.kg_profile_read.argtypes = [vp, P(C.c_double), P(u64), C.c_int]
    L.kg_profile_read.restype = st
    L.kg_shard_unique_id.argtypes = [P(C.c_uint8)]
    L.kg_shard_unique_id.restype = st
    L.kg_shard_init.argtypes = [vp, P(C.c_uint8), C.c_int, C.c_int]
    L.kg_shard_init.restype = st
    L.kg_shard_select.argtypes = [vp, vp, u32, P(u64)]
    L.kg_shard_select.restype = st
    L.kg_make_key.argtypes = [i64, u32]
    L.kg_make_key.restype = u64
    L.kg_key_node.argtypes = [u64]
    L.kg_key_node.restype = i32
    L.kg_key_total.argtypes = [u64]
    L.kg_key_total.restype = i64
    L.kg_merge_keys.argtypes = [P(u64), u32, u32, u32, P(u64)]
    L.kg_merge_keys.restype = st
    L.kg_snapshot_upload_quotas.argtypes = [vp, P(abi.KgQuotaColumns), u32]
    L.kg_snapshot_upload_quotas.restype = st
    L.kg_snapshot_read_quotas.argtypes = [vp, P(i64), P(u32), P(i64), P(u32)]
    L.kg_snapshot_read_quotas.restype = st
    L.kg_snapshot_upload_reservations.argtypes = [vp, P(abi.KgRsvView), u32, P(abi.KgRsvInfo), u32, P(abi.KgRsvDev), u32]
    L.kg_snapshot_upload_reservations.restype = st
    L.kg_snapshot_update_views.argtypes = [vp, P(u32), u32, P(abi.KgRsvView), u32, P(abi.KgRsvInfo), u32,
                                           P(abi.KgRsvDev), u32]
    L.kg_snapshot_update_views.restype = st
    L.kg_assume_ext.argtypes = [vp, vp, u32, u32, P(i32), P(u32)]
    L.kg_assume_ext.restype = st
    L.kg_forget_ext.argtypes = [vp, vp, u32, u32, i32, u32]
    L.kg_forget_ext.restype = st
    L.kg_replay_minors.argtypes = [vp, P(u32)]
    L.kg_replay_minors.restype = st
    L.kg_snapshot_checkpoint.argtypes = [vp]
    L.kg_snapshot_checkpoint.restype = st
    L.kg_snapshot_rollback.argtypes = [vp]
    L.kg_snapshot_rollback.restype = st
    L.kg_batch_schedule.argtypes = [vp, vp, P(i32), P(u32), P(u32), P(i32), P(u32)]
    L.kg_batch_schedule.restype = st
    L.kg_cpuset_take.argtypes = [vp, P(abi.KgCpuTopo), u32, P(abi.KgCpuAlloc), u32, P(abi.KgCpusetRequest), u32,
                                 P(u64), P(i32)]
    L.kg_cpuset_take.restype = st
    L.kg_reserve.argtypes = [vp, vp, u32, u32, P(abi.KgReserveRecord)]
    L.kg_reserve.restype = st
    L.kg_unreserve.argtypes = [vp, vp, u32, u32, P(abi.KgReserveRecord)]
    L.kg_unreserve.restype = st
    L.kg_snapshot_read_reservations.argtypes = [vp, P(abi.KgRsvView), u32, P(abi.KgRsvInfo), u32]
    L.kg_snapshot_read_reservations.restype = st
    L.kg_snapshot_read_rsv_devs.argtypes = [vp, P(abi.KgRsvDev), u32]
    L.kg_snapshot_read_rsv_devs.restype = st
    L.kg_snapshot_upload_rsv_gpu.argtypes = [vp, P(abi.KgRsvGpu), u32]
    L.kg_snapshot_upload_rsv_gpu.restype = st
    if L.kg_abi_version() != abi.KG_ABI_VERSION:
        raise ImportError(f"libkoordgpu ABI {L.kg_abi_version()} != {abi.KG_ABI_VERSION}")
    _lib = L
    return L


def device_count() -> int:
    return lib().kg_device_count()


def _u64p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint64))


class Context:
    """kg_ctx: one HIP device + stream (+ RCCL communicator when sharded)."""

    def __init__(self, device: int = 0):
        self.L = lib()
        h = C.c_void_p()
        s = self.L.kg_open(device, C.byref(h))
        if s != abi.KG_OK:
            raise EngineError(s, f"kg_open(device={device}) failed: {self.L.kg_status_string(s).decode()}")
        self.h = h
        self.device = device
        self._children = weakref.WeakSet()  # snapshots / pod batches, closed before the context

    def check(self, s: int, what: str):
        if s == abi.KG_OK:
            return
        msg = self.L.kg_last_error(self.h).decode() or self.L.kg_status_string(s).decode()
        cls = Unsupported if s == abi.KG_UNSUPPORTED else ReserveFailed if s == abi.KG_RESERVE_FAILED else EngineError
        raise cls(s, f"{what}: {msg}")

    def sync(self):
        self.check(self.L.kg_sync(self.h), "kg_sync")

    def profile(self, enable: bool = True):
        self.check(self.L.kg_profile_enable(self.h, int(enable)), "kg_profile_enable")

    def profile_read(self, reset: bool = False):
        ms, n = C.c_double(), C.c_uint64()
        self.check(self.L.kg_profile_read(self.h, C.byref(ms), C.byref(n), int(reset)), "kg_profile_read")
        return ms.value, n.value

    def shard_init(self, uid: bytes, rank: int, world: int):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self.check(self.L.kg_shard_init(self.h, buf, rank, world), "kg_shard_init")

    def close(self):
        if getattr(self, "h", None):
            for child in list(self._children):
                child.close()
            self.L.kg_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    s = lib().kg_shard_unique_id(buf)
    if s != abi.KG_OK:
        raise EngineError(s, "kg_shard_unique_id failed")
    return bytes(buf)


class Snapshot:
    """kg_snap: device-resident node snapshot (one shard)."""

    def __init__(self, ctx: Context, cfg: abi.KgConfig, nodes: abi.Table, index_base: int = 0):
        self.ctx = ctx
        self.cfg = cfg
        self.n = abi.table_len(nodes)
        self.index_base = index_base
        h = C.c_void_p()
        ctx.check(ctx.L.kg_snapshot_create(ctx.h, C.byref(cfg), self.n, index_base, C.byref(h)), "kg_snapshot_create")
        self.h = h
        ctx._children.add(self)
        self.upload(nodes)

    def upload(self, nodes: abi.Table):
        cols = abi.node_columns(nodes)
        self.ctx.check(self.ctx.L.kg_snapshot_upload(self.h, C.byref(cols)), "kg_snapshot_upload")
        self.has_cpu = "cpu_topo" in nodes

    def update_rows(self, rows, nodes: abi.Table):
        rows = np.ascontiguousarray(rows, np.uint32)
        cols = abi.node_columns(nodes)
        self.ctx.check(self.ctx.L.kg_snapshot_update_rows(self.h, rows.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                          len(rows), C.byref(cols)), "kg_snapshot_update_rows")

    def generation(self) -> int:
        g = C.c_uint64()
        self.ctx.check(self.ctx.L.kg_snapshot_generation(self.h, C.byref(g)), "kg_snapshot_generation")
        return int(g.value)

    def read_state(self) -> abi.Table:
        t = abi.empty_node_state(self.n)
        s = abi.node_state_struct(t)
        self.ctx.check(self.ctx.L.kg_snapshot_read_state(self.h, C.byref(s)), "kg_snapshot_read_state")
        if not getattr(self, "has_cpu", False):
            t.pop("cpu_alloc")  # no CPU topologies in this snapshot
        return t

    def checkpoint(self):
        """Save the Reserve state (records, zones, GPU minors, quota used) for rollback()."""
        self.ctx.check(self.ctx.L.kg_snapshot_checkpoint(self.h), "kg_snapshot_checkpoint")

    def rollback(self):
        self.ctx.check(self.ctx.L.kg_snapshot_rollback(self.h), "kg_snapshot_rollback")

    def upload_quotas(self, quotas: abi.Table):
        self.n_quotas = len(quotas["used"])
        qc = abi.quota_columns(quotas)
        self.ctx.check(self.ctx.L.kg_snapshot_upload_quotas(self.h, C.byref(qc), self.n_quotas),
                       "kg_snapshot_upload_quotas")

    def read_quotas(self):
        nq = getattr(self, "n_quotas", 0)
        used = np.zeros((max(nq, 1), abi.KG_QUOTA_R), np.int64)
        npu = np.zeros((max(nq, 1), abi.KG_QUOTA_R), np.int64)
        uk = np.zeros(max(nq, 1), np.uint32)
        nk = np.zeros(max(nq, 1), np.uint32)
        P = C.POINTER
        self.ctx.check(self.ctx.L.kg_snapshot_read_quotas(self.h, used.ctypes.data_as(P(C.c_int64)),
                                                          uk.ctypes.data_as(P(C.c_uint32)),
                                                          npu.ctypes.data_as(P(C.c_int64)),
                                                          nk.ctypes.data_as(P(C.c_uint32))), "kg_snapshot_read_quotas")
        return used[:nq], uk[:nq], npu[:nq], nk[:nq]

    def upload_reservations(self, rsv: abi.Reservations):
        self.ctx.check(self.ctx.L.kg_snapshot_upload_reservations(
            self.h, C.cast(rsv.views, C.POINTER(abi.KgRsvView)), rsv.n_views,
            C.cast(rsv.infos, C.POINTER(abi.KgRsvInfo)), rsv.n_infos,
            C.cast(rsv.devs, C.POINTER(abi.KgRsvDev)), rsv.n_devs), "kg_snapshot_upload_reservations")
        if getattr(rsv, "n_gpu", 0):  # the DeviceShare restore inputs of GPU-holding reservations
            self.ctx.check(self.ctx.L.kg_snapshot_upload_rsv_gpu(self.h, C.cast(rsv.gpu, C.POINTER(abi.KgRsvGpu)),
                                                                 rsv.n_gpu), "kg_snapshot_upload_rsv_gpu")

    def read_reservations(self, rsv: abi.Reservations) -> abi.Reservations:
        """The views, infos and GPU restore tables as the device holds them now (Reservation.Reserve / Unreserve ran
        there), in the layout of the uploaded `rsv` (same counts)."""
        out = abi.Reservations([], [])
        out.views = (abi.KgRsvView * max(1, rsv.n_views))()
        out.infos = (abi.KgRsvInfo * max(1, rsv.n_infos))()
        out.n_views, out.n_infos = rsv.n_views, rsv.n_infos
        out.devs, out.n_devs = rsv.devs, rsv.n_devs
        self.ctx.check(self.ctx.L.kg_snapshot_read_reservations(
            self.h, C.cast(out.views, C.POINTER(abi.KgRsvView)), rsv.n_views,
            C.cast(out.infos, C.POINTER(abi.KgRsvInfo)), rsv.n_infos), "kg_snapshot_read_reservations")
        if rsv.n_devs:  # the GPU restore tables as the device rebuilt them
            out.devs = (abi.KgRsvDev * rsv.n_devs)()
            self.ctx.check(self.ctx.L.kg_snapshot_read_rsv_devs(self.h, C.cast(out.devs, C.POINTER(abi.KgRsvDev)),
                                                                rsv.n_devs), "kg_snapshot_read_rsv_devs")
        return out

    def update_views(self, nodes, rsv: abi.Reservations):
        """kg_snapshot_update_views: the views of `nodes` replaced by rsv's (which name only those nodes)."""
        nd = np.ascontiguousarray(np.asarray(nodes, np.uint32))
        self.ctx.check(self.ctx.L.kg_snapshot_update_views(
            self.h, nd.ctypes.data_as(C.POINTER(C.c_uint32)), len(nd),
            C.cast(rsv.views, C.POINTER(abi.KgRsvView)), rsv.n_views,
            C.cast(rsv.infos, C.POINTER(abi.KgRsvInfo)), rsv.n_infos,
            C.cast(rsv.devs, C.POINTER(abi.KgRsvDev)), rsv.n_devs), "kg_snapshot_update_views")

    def close(self):
        if getattr(self, "h", None) and getattr(self.ctx, "h", None):
            self.ctx.L.kg_snapshot_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PodBatch:
    """kg_pods: device-resident pending pods + result buffers."""

    def __init__(self, ctx: Context, pods: abi.Table, capacity: Optional[int] = None):
        self.ctx = ctx
        n = abi.table_len(pods)
        cap = max(1, capacity or n)
        h = C.c_void_p()
        ctx.check(ctx.L.kg_pods_create(ctx.h, cap, C.byref(h)), "kg_pods_create")
        self.h = h
        ctx._children.add(self)
        self.capacity = cap
        self.upload(pods)

    def upload(self, pods: abi.Table):
        self.n = abi.table_len(pods)
        # the column struct of the same table (same dict, same arrays, possibly new contents) is reused: building it
        # costs ~125 us of Python per upload, a cgo caller's struct of pointers costs nothing
        key = getattr(self, "_cols_key", None)
        if key is not None and key[0] is pods and len(key[1]) == len(pods) and all(
                a is b for a, b in zip(key[1], pods.values())):
            cols = self._cols
        else:
            cols = abi.pod_columns(pods)
            self._cols, self._cols_key = cols, (pods, tuple(pods.values()))
        self.ctx.check(self.ctx.L.kg_pods_upload(self.h, C.byref(cols), self.n), "kg_pods_upload")

    def close(self):
        if getattr(self, "h", None) and getattr(self.ctx, "h", None):
            self.ctx.L.kg_pods_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def eval_verify(snap: Snapshot, pods: PodBatch) -> abi.VerifyResult:
    res = abi.VerifyResult(pods.n, snap.n)
    s = res.struct()
    snap.ctx.check(snap.ctx.L.kg_eval_verify(snap.h, pods.h, C.byref(s)), "kg_eval_verify")
    return res


def eval_select_async(snap: Snapshot, pods: PodBatch, k: int = 1):
    snap.ctx.check(snap.ctx.L.kg_eval_select(snap.h, pods.h, k), "kg_eval_select")


def result_keys(pods: PodBatch, k: int) -> np.ndarray:
    out = np.zeros((pods.n, k), np.uint64)
    pods.ctx.check(pods.ctx.L.kg_result_keys(pods.h, _u64p(out)), "kg_result_keys")
    return out


def result_status(pods: PodBatch) -> np.ndarray:
    """Per-pod outcome flags of the last select: KG_ST_UNSUPPORTED (some pair needs the reference plugin on
    the host), KG_ST_QUOTA (ElasticQuota PreFilter rejected the pod), or 0."""
    out = np.zeros(pods.n, np.uint32)
    pods.ctx.check(pods.ctx.L.kg_result_status(pods.h, out.ctypes.data_as(C.POINTER(C.c_uint32))), "kg_result_status")
    return out


def eval_select(snap: Snapshot, pods: PodBatch, k: int = 1) -> np.ndarray:
    eval_select_async(snap, pods, k)
    return result_keys(pods, k)


def replay(snap: Snapshot, pods: PodBatch, reasons: bool = False):
    """One pod per cycle with device-resident Assume: (node, total) or, with reasons=True, (node, total,
    reason) where reason[j] is the OR of the KG_ST_* filter bits over the nodes in pod j's cycle."""
    node = np.zeros(pods.n, np.int32)
    total = np.zeros(pods.n, np.int64)
    reason = np.zeros(pods.n, np.uint32) if reasons else None
    snap.ctx.check(snap.ctx.L.kg_replay(snap.h, pods.h, node.ctypes.data_as(C.POINTER(C.c_int32)),
                                        total.ctypes.data_as(C.POINTER(C.c_int64)),
                                        reason.ctypes.data_as(C.POINTER(C.c_uint32)) if reasons else None),
                   "kg_replay")
    return (node, total, reason) if reasons else (node, total)


def assume(snap: Snapshot, pods: PodBatch, pod: int, node: int):
    snap.ctx.check(snap.ctx.L.kg_assume(snap.h, pods.h, pod, node), "kg_assume")


def forget(snap: Snapshot, pods: PodBatch, pod: int, node: int, zone: int):
    snap.ctx.check(snap.ctx.L.kg_forget(snap.h, pods.h, pod, node, zone), "kg_forget")


def assume_numa(snap: Snapshot, pods: PodBatch, pod: int, node: int):
    """kg_assume_numa: (zone code, [2, KG_MAX_ZONES] cpu / memory taken per zone)."""
    zone = C.c_int32()
    amounts = np.zeros(2 * abi.KG_MAX_ZONES, np.int64)
    snap.ctx.check(snap.ctx.L.kg_assume_numa(snap.h, pods.h, pod, node, C.byref(zone),
                                             amounts.ctypes.data_as(C.POINTER(C.c_int64))), "kg_assume_numa")
    return zone.value, amounts.reshape(2, abi.KG_MAX_ZONES)


def forget_numa(snap: Snapshot, pods: PodBatch, pod: int, node: int, zone: int, amounts: np.ndarray):
    a = np.ascontiguousarray(amounts, np.int64).reshape(-1)
    assert a.size == 2 * abi.KG_MAX_ZONES
    snap.ctx.check(snap.ctx.L.kg_forget_numa(snap.h, pods.h, pod, node, zone, a.ctypes.data_as(C.POINTER(C.c_int64))),
                   "kg_forget_numa")


def replay_minors(pods: PodBatch) -> np.ndarray:
    out = np.zeros(pods.n, np.uint32)
    pods.ctx.check(pods.ctx.L.kg_replay_minors(pods.h, out.ctypes.data_as(C.POINTER(C.c_uint32))), "kg_replay_minors")
    return out


def assume_ext(snap: Snapshot, pods: PodBatch, pod: int, node: int):
    zone, minors = C.c_int32(), C.c_uint32()
    snap.ctx.check(snap.ctx.L.kg_assume_ext(snap.h, pods.h, pod, node, C.byref(zone), C.byref(minors)), "kg_assume_ext")
    return zone.value, minors.value


def forget_ext(snap: Snapshot, pods: PodBatch, pod: int, node: int, zone: int, minors: int):
    snap.ctx.check(snap.ctx.L.kg_forget_ext(snap.h, pods.h, pod, node, zone, minors), "kg_forget_ext")


def reserve(snap: Snapshot, pods: PodBatch, pod: int, node: int) -> abi.KgReserveRecord:
    """kg_reserve: every enabled plugin's Reserve; the record its kg_unreserve gives back."""
    rec = abi.KgReserveRecord()
    snap.ctx.check(snap.ctx.L.kg_reserve(snap.h, pods.h, pod, node, C.byref(rec)), "kg_reserve")
    return rec


def unreserve(snap: Snapshot, pods: PodBatch, pod: int, node: int, rec: abi.KgReserveRecord):
    snap.ctx.check(snap.ctx.L.kg_unreserve(snap.h, pods.h, pod, node, C.byref(rec)), "kg_unreserve")


def batch_schedule(snap: Snapshot, pods: PodBatch, plan_node):
    """Inline batch cycle of a planned job (kg_batch_schedule): per pod (result code KG_BATCH_*, filter
    status bits, NUMA zone, GPU minors). Raises Unsupported when a pod needs the host path (state rolled back)."""
    plan = np.ascontiguousarray(plan_node, np.int32)
    if len(plan) != pods.n:
        raise ValueError(f"plan has {len(plan)} entries for {pods.n} pods")
    res = np.zeros(pods.n, np.uint32)
    stat = np.zeros(pods.n, np.uint32)
    zone = np.zeros(pods.n, np.int32)
    minors = np.zeros(pods.n, np.uint32)
    P = C.POINTER
    snap.ctx.check(snap.ctx.L.kg_batch_schedule(snap.h, pods.h, plan.ctypes.data_as(P(C.c_int32)),
                                                res.ctypes.data_as(P(C.c_uint32)), stat.ctypes.data_as(P(C.c_uint32)),
                                                zone.ctypes.data_as(P(C.c_int32)), minors.ctypes.data_as(P(C.c_uint32))),
                   "kg_batch_schedule")
    return res, stat, zone, minors


def cpuset_take(ctx: Context, topos, allocs, reqs):
    """kg_cpuset_take: device cpuset accumulator over a list of KgCpusetRequest -> (masks [n, 4], rc [n])."""
    n = len(reqs)
    T = (abi.KgCpuTopo * max(len(topos), 1))(*topos)
    A = (abi.KgCpuAlloc * max(len(allocs), 1))(*allocs) if allocs else None
    R = (abi.KgCpusetRequest * max(n, 1))(*reqs)
    out = np.zeros((max(n, 1), 4), np.uint64)
    rc = np.zeros(max(n, 1), np.int32)
    ctx.check(ctx.L.kg_cpuset_take(ctx.h, T, len(topos), A, len(allocs) if allocs else 0, R, n, _u64p(out),
                                   rc.ctypes.data_as(C.POINTER(C.c_int32))), "kg_cpuset_take")
    return out[:n], rc[:n]


def shard_select(snap: Snapshot, pods: PodBatch, k: int = 1, download: bool = True) -> Optional[np.ndarray]:
    """Node-sharded select over RCCL: per-pod global top-k keys [pods, k] (identical on every rank)."""
    out = np.zeros((pods.n, k), np.uint64) if download else None
    snap.ctx.check(snap.ctx.L.kg_shard_select(snap.h, pods.h, k, _u64p(out) if download else None), "kg_shard_select")
    return out


def merge_keys(keys: np.ndarray) -> np.ndarray:
    """Host selectHost over gathered shard keys, keys[shard][pod][k] -> [pod][k] (no device needed)."""
    keys = np.ascontiguousarray(keys, np.uint64)
    n_shards, n_pods, k = keys.shape
    out = np.zeros((n_pods, k), np.uint64)
    s = lib().kg_merge_keys(_u64p(keys), n_shards, n_pods, k, _u64p(out))
    if s != abi.KG_OK:
        raise EngineError(s, "kg_merge_keys failed")
    return out
