"""Event-driven snapshot maintenance: the scheduler-side caches that turn informer
events into snapshot row deltas, and the sync that ships those deltas to a device snapshot.

The reference keeps one cache per plugin, each fed by its own informer handlers:
  * framework NodeInfo (k8s scheduler cache): Requested / NonZeroRequested / pod count of assigned pods,
    AssumePod / ForgetPod for the scheduler's own placements;
  * LoadAware podAssignCache (loadaware/pod_assign_cache.go:89-707): OnAdd / OnUpdate / OnDelete (:365-413),
    AddOrUpdateNodeMetric / DeleteNodeMetric (:498-616), assign / unAssign from Reserve / Unreserve
    (load_aware.go:226-233);
  * NodeNUMAResource resourceManager (nodenumaresource/pod_eventhandler.go:53-149, node_allocation.go):
    per-node pod allocations (cpuset, NUMA zone resources) from the resource-status annotation;
  * DeviceShare nodeDeviceCache (deviceshare/device_cache.go:518-548 updateNodeDevice,
    eventhandler_pod.go updatePod / deletePod): per-minor total, used and free.
ClusterState mirrors all four over one set of nodes, bumps a generation counter per event and stamps each
node it touched with it (the NodeInfo.Generation scheme of the k8s cache's UpdateSnapshot); SnapshotSync
then sends every row newer than the snapshot's last sync in ONE batched kg_snapshot_update_rows call.

Times are seconds on the cache clock (`clock()`), None being Go's zero time. The node set is fixed for a
snapshot's life: adding or removing a node is a new snapshot (kg_snapshot_create + upload)."""
from __future__ import annotations

import heapq
import json
from fractions import Fraction
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Set, Tuple

import numpy as np

from . import abi
from .config import CPU, DEV_RESOURCES, MEMORY, SchedulerConfig
from .decode import (ANN_AMPLIFICATION, LoadAwareNodeCache, NODEINFO_KEYS, Unsupported, _is_terminated, _rl, amplify,
                     assign_info, is_reserve_pod, la_cols, milli_value, node_static_cols, nodeinfo_cols,
                     pod_request_vec, pod_requests, value, zone_used_cols)

ANN_RESOURCE_STATUS = "scheduling.koordinator.sh/resource-status"
ANN_DEVICE_ALLOCATED = "scheduling.koordinator.sh/device-allocated"


def _md(obj) -> dict:
    return obj.get("metadata") or {}


def _uid(pod) -> str:
    md = _md(pod)
    return md.get("uid") or f"{md.get('namespace', '')}/{md.get('name', '')}"


def _node_name(pod) -> str:
    return (pod.get("spec") or {}).get("nodeName") or ""


def _nn(pod) -> Tuple[str, str]:
    md = _md(pod)
    return md.get("namespace", ""), md.get("name", "")


# ------------------------------------------------------------------------------------------------
# LoadAware podAssignCache

class PodAssignCache:
    """podAssignCache (loadaware/pod_assign_cache.go:89-707): nodeInfo entries by node name, created on the
    first object for a node and removed when both its metric and its pods are gone (tryCleanup, :281-288).
    Single-threaded here: the reference's lock protocol (:42-88) orders concurrent handlers, and the event
    stream this cache sees is already serialised. `on_change(node)` is called for every node an event
    touches."""

    def __init__(self, la, clock: Callable[[], float] = lambda: 0.0,
                 on_change: Callable[[str], None] = lambda name: None):
        self.la = la
        self.clock = clock
        self.items: Dict[str, LoadAwareNodeCache] = {}
        self.on_change = on_change

    def get(self, name: str) -> Optional[LoadAwareNodeCache]:
        return self.items.get(name)

    def _get_or_create(self, name: str) -> LoadAwareNodeCache:
        n = self.items.get(name)
        if n is None:
            n = LoadAwareNodeCache(la=self.la)
            self.items[name] = n
        return n

    def _try_cleanup(self, name: str, n: LoadAwareNodeCache):
        if n.empty():
            self.items.pop(name, None)

    def pod_info(self, name: str, pod):
        """getPodAssignInfo (:215-226)."""
        if not name:
            return None
        n = self.items.get(name)
        return None if n is None else n.pod_infos.get(_uid(pod))

    def assign(self, name: str, pod):
        """assign (:291-327): terminated and reserve pods are not cached."""
        if not name or _is_terminated(pod) or is_reserve_pod(pod):
            return
        info = assign_info(pod, self.la, now=self.clock())
        self._get_or_create(name).add_or_update_pod(_uid(pod), info)
        self.on_change(name)

    def unassign(self, name: str, pod):
        """unAssign (:356-363) -> nodeInfo.DeletePod (:449-466)."""
        if not name:
            return
        n = self.items.get(name)
        if n is not None:
            n.delete_pod(_uid(pod))
            self._try_cleanup(name, n)
            self.on_change(name)

    def on_add(self, pod):
        """OnAdd (:365-371)."""
        self.assign(_node_name(pod), pod)

    def on_update(self, old, pod):
        """OnUpdate (:373-396): a pod moved off a node is removed there first; an uncached pod is assigned,
        a terminated one removed, and a cached one renewed only when its spec or conditions changed."""
        if pod is None:
            return
        if old is not None and _node_name(old) and _node_name(old) != _node_name(pod):
            self.unassign(_node_name(old), pod)
        cached = self.pod_info(_node_name(pod), pod)
        if cached is None:
            self.assign(_node_name(pod), pod)
        elif _is_terminated(pod):
            self.unassign(_node_name(pod), pod)
        elif (pod.get("spec") != cached.pod.get("spec")
              or (pod.get("status") or {}).get("conditions") != (cached.pod.get("status") or {}).get("conditions")):
            self.assign(_node_name(pod), pod)

    def on_delete(self, pod):
        """OnDelete (:398-413)."""
        self.unassign(_node_name(pod), pod)

    def add_or_update_node_metric(self, metric: dict):
        """AddOrUpdateNodeMetric (:498-509, nodeInfo side :520-603)."""
        name = _md(metric).get("name", "")
        self._get_or_create(name).set_metric(metric)
        self.on_change(name)

    def delete_node_metric(self, name: str):
        """DeleteNodeMetric (:511-516, :605-616)."""
        n = self.items.get(name)
        if n is not None:
            n.clear_metric()
            self._try_cleanup(name, n)
            self.on_change(name)


# ------------------------------------------------------------------------------------------------
# NodeNUMAResource resourceManager allocations

def parse_cpuset(s: str) -> Set[int]:
    """cpuset.Parse: Linux CPU list format ("0-3,8,10-11")."""
    out: Set[int] = set()
    s = (s or "").strip()
    if not s:
        return out
    for part in s.split(","):
        part = part.strip()
        if "-" in part:
            a, b = part.split("-", 1)
            lo, hi = int(a), int(b)
            if hi < lo:
                raise ValueError(f"invalid cpuset range {part!r}")
            out.update(range(lo, hi + 1))
        else:
            out.add(int(part))
    return out


@dataclass
class _PodAllocation:
    cpus: Set[int]
    numa: List[Tuple[int, Dict[str, object]]]  # (zone, ResourceList)


@dataclass
class NodeAllocation:
    """NodeAllocation (nodenumaresource/node_allocation.go:33-243) restricted to what the snapshot reads:
    allocated cpus with reference counts, allocated resources per zone and the per-zone shared status."""
    pods: Dict[str, _PodAllocation] = field(default_factory=dict)
    cpu_refs: Dict[int, int] = field(default_factory=dict)
    zone_res: Dict[int, Dict[str, object]] = field(default_factory=dict)
    single: Dict[int, Set[str]] = field(default_factory=dict)
    shared: Dict[int, Set[str]] = field(default_factory=dict)

    def add(self, uid: str, a: _PodAllocation, cpu_zone: Dict[int, int]):
        """addPodAllocation (:111-156); an existing allocation of the uid is kept."""
        if uid in self.pods:
            return
        self.pods[uid] = a
        used = set()
        for c in a.cpus:
            self.cpu_refs[c] = self.cpu_refs.get(c, 0) + 1
            used.add(cpu_zone.get(c, 0))
        if len(used) > 1:
            for z in used:
                self.shared.setdefault(z, set()).add(uid)
        elif len(used) == 1:
            self.single.setdefault(next(iter(used)), set()).add(uid)
        for z, res in a.numa:
            cur = self.zone_res.setdefault(z, {})
            for k, q in _rl(res).items():
                cur[k] = cur.get(k, 0) + q

    def release(self, uid: str, cpu_zone: Dict[int, int]):
        """release (:158-190)."""
        a = self.pods.pop(uid, None)
        if a is None:
            return
        used = set()
        for c in a.cpus:
            if c not in self.cpu_refs:
                continue
            self.cpu_refs[c] -= 1
            if self.cpu_refs[c] == 0:
                del self.cpu_refs[c]
            used.add(cpu_zone.get(c, 0))
        for z in used:
            self.shared.get(z, set()).discard(uid)
            self.single.get(z, set()).discard(uid)
        for z, res in a.numa:
            cur = self.zone_res.get(z)
            if cur is not None:  # quotav1.SubtractWithNonNegativeResult
                for k, q in _rl(res).items():
                    cur[k] = max(cur.get(k, 0) - q, 0)

    def zone_status(self, n_zones: int) -> int:
        """NUMANodeSharedStatus per zone (:52-68), 2 bits each."""
        st = 0
        for z in range(n_zones):
            s = 0
            if self.single.get(z) and not self.shared.get(z):
                s = 1
            elif self.single.get(z) or self.shared.get(z):
                s = 2
            st |= s << (2 * z)
        return st


def pod_numa_allocation(pod) -> Optional[_PodAllocation]:
    """podEventHandler.updatePod (pod_eventhandler.go:108-139): the resource-status annotation's cpuset and
    NUMA zone resources; None when it carries neither (or does not parse)."""
    ann = _md(pod).get("annotations") or {}
    raw = ann.get(ANN_RESOURCE_STATUS)
    if not raw:
        return None
    try:
        st = json.loads(raw)
        cpus = parse_cpuset(st.get("cpuset", ""))
    except (ValueError, TypeError):
        return None
    numa = [(int(r.get("node", 0)), r.get("resources") or {}) for r in st.get("numaNodeResources") or []]
    if not numa and not cpus:
        return None
    return _PodAllocation(cpus, numa)


# ------------------------------------------------------------------------------------------------
# DeviceShare nodeDeviceCache (GPU minors)

GPU = "gpu"


@dataclass
class NodeDevice:
    """nodeDevice (deviceshare/device_cache.go:44-130): deviceTotal / deviceUsed per type and minor, and the
    allocateSet that keeps one pod's allocation from being counted twice (isValid, :209-228)."""
    total: Dict[str, Dict[int, Dict[str, int]]] = field(default_factory=dict)
    used: Dict[str, Dict[int, Dict[str, int]]] = field(default_factory=dict)
    allocate_set: Dict[str, Dict[Tuple[str, str], list]] = field(default_factory=dict)
    has_device: bool = False

    def reset_total(self, resources: Dict[str, Dict[int, Dict[str, int]]]):
        """resetDeviceTotal (:119-130): a type absent from the new Device keeps an empty table."""
        for t in self.total:
            resources.setdefault(t, {})
        self.total = resources

    def free(self, t: str) -> Dict[int, Dict[str, int]]:
        """resetDeviceFree (:101-117): total minus used, clamped at zero, per minor."""
        out = {m: dict(r) for m, r in self.total.get(t, {}).items()}
        for m, u in self.used.get(t, {}).items():
            tot = self.total.get(t, {}).get(m, {})
            out[m] = {k: max(tot.get(k, 0) - u.get(k, 0), 0) for k in set(tot) | set(u)}
            out[m] = {k: v for k, v in out[m].items() if k in tot or v != 0}
        return out

    def update_cache_used(self, allocations: Dict[str, list], pod, add: bool):
        """updateCacheUsed (:132-143) with updateDeviceUsed (:184-210) and updateAllocateSet."""
        key = _nn(pod)
        for t, allocs in allocations.items():
            aset = self.allocate_set.setdefault(t, {})
            if add and key in aset:
                continue  # already counted (e.g. after Reserve)
            if not add and key not in aset:
                continue
            used = self.used.setdefault(t, {})
            for a in allocs:
                m = int(a.get("minor", 0))
                res = {k: value(q) for k, q in (a.get("resources") or {}).items()}
                cur = used.setdefault(m, {})
                if add:
                    for k, v in res.items():
                        cur[k] = cur.get(k, 0) + v
                else:
                    for k, v in res.items():
                        cur[k] = max(cur.get(k, 0) - v, 0)
                    if all(v == 0 for v in cur.values()):
                        del used[m]
            if not add and not used:
                del self.used[t]
            if add:
                aset[key] = allocs
            else:
                del aset[key]


def device_resources(device: dict) -> Dict[str, Dict[int, Dict[str, int]]]:
    """buildDeviceResources (device_cache.go:550-568): an unhealthy device reports no resources."""
    out: Dict[str, Dict[int, Dict[str, int]]] = {}
    for d in (device.get("spec") or {}).get("devices") or []:
        t = d.get("type", "")
        res = {} if not d.get("health", False) else {k: value(q) for k, q in (d.get("resources") or {}).items()}
        out.setdefault(t, {})[int(d.get("minor", 0))] = res
    return out


def pod_device_allocations(pod) -> Dict[str, list]:
    """apiext.GetDeviceAllocations: the device-allocated annotation ({} when absent or unparsable)."""
    raw = (_md(pod).get("annotations") or {}).get(ANN_DEVICE_ALLOCATED)
    if not raw:
        return {}
    try:
        d = json.loads(raw)
    except ValueError:
        return {}
    return {t: list(v or []) for t, v in d.items()} if isinstance(d, dict) else {}


class NodeDeviceCache:
    """nodeDeviceCache (device_cache.go:455-548) with the pod handlers of eventhandler_pod.go."""

    def __init__(self, on_change: Callable[[str], None] = lambda name: None):
        self.infos: Dict[str, NodeDevice] = {}
        self.on_change = on_change

    def update_node_device(self, device: dict):
        """updateNodeDevice (:518-548), GPU partition / topology-scope state aside (row f4)."""
        name = _md(device).get("name", "")
        if not name:
            return
        info = self.infos.setdefault(name, NodeDevice())
        info.reset_total(device_resources(device))
        info.has_device = True
        self.on_change(name)

    def remove_node_device(self, name: str):
        """removeNodeDevice (:486-494)."""
        if self.infos.pop(name, None) is not None:
            self.on_change(name)

    def update_pod(self, old, pod):
        """updatePod (eventhandler_pod.go): note that an old allocation is released through the NEW node's
        entry, as the reference does."""
        if not _node_name(pod):
            if old is not None and _node_name(old):
                self.delete_pod(old)
            return
        if _is_terminated(pod):
            self.delete_pod(pod)
            return
        allocs = pod_device_allocations(pod)
        old_allocs = pod_device_allocations(old) if old is not None else {}
        if not allocs and not old_allocs:
            return
        name = _node_name(pod)
        info = self.infos.setdefault(name, NodeDevice())
        if old is not None and _node_name(old) and old_allocs:
            info.update_cache_used(old_allocs, old, False)
        if allocs:
            info.update_cache_used(allocs, pod, True)
        self.on_change(name)

    def delete_pod(self, pod):
        """deletePod (eventhandler_pod.go)."""
        name = _node_name(pod)
        if not name:
            return
        allocs = pod_device_allocations(pod)
        if not allocs:
            return
        info = self.infos.get(name)
        if info is None:
            return
        info.update_cache_used(allocs, pod, False)
        self.on_change(name)

    def columns(self, name: str):
        """(dev_minors, dev_total[R][M], dev_free[R][M]) of the node's GPU minors (kg_node_columns)."""
        tot = np.zeros((abi.KG_DEV_R, abi.KG_DEV_MINORS), np.int64)
        free = np.zeros_like(tot)
        info = self.infos.get(name)
        if info is None or not info.has_device:
            return -1, tot, free
        t = info.total.get(GPU, {})
        f = info.free(GPU)
        minors = sorted(set(t) | set(f))
        if minors != list(range(len(minors))) or len(minors) > abi.KG_DEV_MINORS:
            raise Unsupported(f"GPU minors {minors} of node {name} are not 0..{abi.KG_DEV_MINORS - 1}")
        for m in minors:
            for r, key in enumerate(DEV_RESOURCES):
                tot[r, m] = t.get(m, {}).get(key, 0)
                free[r, m] = f.get(m, {}).get(key, 0)
        return len(minors), tot, free


# ------------------------------------------------------------------------------------------------
# The cluster state and its sync to a device snapshot

@dataclass
class _NodeTopology:
    zones: List[Dict[str, str]] = field(default_factory=list)
    kubelet_policy: str = ""
    cpu_zone: Dict[int, int] = field(default_factory=dict)  # cpu id -> NUMA node (CPUTopology); {} = none


class ClusterState:
    """Every cache the device path's plugins read, kept per node from informer events, with generations.

    Event entry points (each the fan-out of one informer event to the caches that register for it):
      on_pod_add / on_pod_update / on_pod_delete   Pod events (NodeInfo, podAssignCache, NUMA, DeviceShare)
      on_node_update                               Node events (allocatable, labels, annotations)
      on_node_metric / on_node_metric_delete       NodeMetric events (podAssignCache)
      on_topology                                  NodeResourceTopology events (zones, kubelet policy, cpus)
      on_device / on_device_delete                 Device events (nodeDeviceCache)
      assume / forget                              the scheduler's own Reserve / Unreserve of a placement
    """

    def __init__(self, cfg: SchedulerConfig, nodes: Sequence[dict], clock: Callable[[], float] = lambda: 0.0):
        self.cfg = cfg
        self.la = cfg.la()
        self.clock = clock
        self.nodes = [dict(n) for n in nodes]
        self.names = [_md(n).get("name", "") for n in self.nodes]
        self.index = {name: i for i, name in enumerate(self.names)}
        if len(self.index) != len(self.names):
            raise ValueError("node names must be unique")
        n = len(self.nodes)
        width = len(NODEINFO_KEYS) + abi.KG_NSCALAR
        self.req = np.zeros((n, width), np.int64)
        self.num_pods = np.zeros(n, np.int64)
        self.node_pods: Dict[str, Tuple[int, List[int]]] = {}  # uid -> (node row, request vector)
        self.topo = [_NodeTopology() for _ in range(n)]
        self.numa = [NodeAllocation() for _ in range(n)]
        self.generation = 0
        self.row_gen = np.zeros(n, np.uint64)
        self.assign_cache = PodAssignCache(self.la, clock, self._touch_name)
        self.devices = NodeDeviceCache(self._touch_name)
        # reservation restore inputs (views) and ElasticQuota tables: their own generations, so a sync re-uploads
        # the views of the nodes whose reservations changed and the quota table only when it changed
        self.rsv_gen = np.zeros(n, np.uint64)
        self.reservations = ReservationCache(cfg, self._touch_rsv)
        self.quotas = QuotaCache(cfg)
        # NodeMetric expiry is a function of time (isNodeMetricExpired, loadaware/helper.go:35-40): a timer per
        # metric marks the row when its deadline passes (tick), as an event would
        self._expiry: List[Tuple[float, int, int]] = []  # (deadline, row, metric token)
        self._metric_token = [0] * n

    # -- generations -----------------------------------------------------------------------------
    def _touch(self, i: int):
        self.generation += 1
        self.row_gen[i] = self.generation

    def _touch_name(self, name: str):
        i = self.index.get(name)
        if i is not None:
            self._touch(i)

    def _touch_rsv(self, name: str):
        i = self.index.get(name)
        if i is not None:
            self.generation += 1
            self.rsv_gen[i] = self.generation

    def rsv_rows_since(self, generation: int) -> np.ndarray:
        """Nodes whose reservations changed after `generation` (their restore views need rebuilding)."""
        return np.nonzero(self.rsv_gen > np.uint64(generation))[0].astype(np.uint32)

    def tick(self):
        """Mark the rows whose NodeMetric expired since the last tick (the clock's time events)."""
        now = self.clock()
        while self._expiry and self._expiry[0][0] <= now:
            _, i, token = heapq.heappop(self._expiry)
            if token == self._metric_token[i]:
                self._touch(i)

    def rows_since(self, generation: int) -> np.ndarray:
        """Snapshot rows changed after `generation` (UpdateSnapshot's NodeInfo.Generation test)."""
        return np.nonzero(self.row_gen > np.uint64(generation))[0].astype(np.uint32)

    # -- NodeInfo (k8s scheduler cache) ---------------------------------------------------------
    def _nodeinfo_remove(self, uid: str):
        ent = self.node_pods.pop(uid, None)
        if ent is None:
            return
        i, vec = ent
        self.req[i] -= vec
        self.num_pods[i] -= 1
        self._touch(i)

    def _nodeinfo_add(self, pod):
        i = self.index.get(_node_name(pod))
        if i is None:
            return
        vec = pod_request_vec(pod, self.cfg)
        self.node_pods[_uid(pod)] = (i, vec)
        self.req[i] += vec
        self.num_pods[i] += 1
        self._touch(i)

    def _nodeinfo_update(self, pod):
        """addPod / updatePod / removePod of the scheduler cache: assigned, non-terminated pods only, keyed
        by UID (so a binding that confirms an assumed pod replaces it rather than adding it twice)."""
        self._nodeinfo_remove(_uid(pod))
        if _node_name(pod) and not _is_terminated(pod):
            self._nodeinfo_add(pod)

    # -- NUMA resourceManager --------------------------------------------------------------------
    def _numa_release(self, name: str, uid: str):
        i = self.index.get(name)
        if i is None:
            return
        if uid in self.numa[i].pods:
            self.numa[i].release(uid, self.topo[i].cpu_zone)
            self._touch(i)

    def _numa_update(self, old, pod):
        """podEventHandler.updatePod / deletePod (pod_eventhandler.go:95-149); Update = release + add."""
        if not _node_name(pod):
            if old is not None and _node_name(old):
                self._numa_release(_node_name(old), _uid(old))
            return
        if _is_terminated(pod):
            self._numa_release(_node_name(pod), _uid(pod))
            return
        a = pod_numa_allocation(pod)
        if a is None:
            return
        i = self.index.get(_node_name(pod))
        if i is None:
            return
        self.numa[i].release(_uid(pod), self.topo[i].cpu_zone)
        self.numa[i].add(_uid(pod), a, self.topo[i].cpu_zone)
        self._touch(i)

    # -- events ----------------------------------------------------------------------------------
    def on_pod_add(self, pod):
        self._nodeinfo_update(pod)
        self.assign_cache.on_add(pod)
        self._numa_update(None, pod)
        self.devices.update_pod(None, pod)
        self.reservations.add_pod(pod)
        self.quotas.on_pod(None, pod)

    def on_pod_update(self, old, pod):
        self._nodeinfo_update(pod)
        self.assign_cache.on_update(old, pod)
        self._numa_update(old, pod)
        self.devices.update_pod(old, pod)
        self.reservations.update_pod(old, pod)
        self.quotas.on_pod(old, pod)

    def on_pod_delete(self, pod):
        self._nodeinfo_remove(_uid(pod))
        self.assign_cache.on_delete(pod)
        self._numa_release(_node_name(pod), _uid(pod))
        self.devices.delete_pod(pod)
        self.reservations.delete_pod(pod)
        self.quotas.on_pod_delete(pod)

    # reservation / quota informers (reservation/eventhandler_reservation.go, elasticquota/quota_handler.go)
    @staticmethod
    def _reserve_pod(r: dict) -> dict:
        """reservationutil.NewReservePod: the fake pod an Available reservation holds in NodeInfo, requesting its
        allocatable."""
        md, status = _md(r), r.get("status") or {}
        alloc = {k: v for k, v in (status.get("allocatable") or {}).items() if k != "pods"}
        return {"metadata": {"uid": "reserve-pod/" + md.get("uid", ""), "name": md.get("name", "")},
                "spec": {"nodeName": status.get("nodeName", ""), "containers": [{"resources": {"requests": alloc}}]}}

    def on_reservation(self, r: dict):
        """Reservation add / update: the reservation cache (updateReservation) and its reserve pod in NodeInfo
        while it is Available on a node."""
        self.reservations.update_reservation(r)
        rp = self._reserve_pod(r)
        if (r.get("status") or {}).get("phase") == "Available" and _node_name(rp):
            self._nodeinfo_update(rp)
        else:
            self._nodeinfo_remove(_uid(rp))

    def on_reservation_delete(self, r: dict):
        self.reservations.delete_reservation(r)
        self._nodeinfo_remove(_uid(self._reserve_pod(r)))

    def reservation_restore(self, pods: Sequence[dict], rows: Optional[abi.Table] = None):
        """The Reservation transformer's restore for a pending batch: owner-match classes of the pods over the
        matchable reservations (rsvmatch.match_classes), then decode.reservation_restore over the current rows.
        Returns (rsv_class per pod, restored node table, abi.Reservations)."""
        from . import decode, rsvmatch
        infos = [ri for ri in self.reservations.infos.values() if ri.matchable() and ri.node in self.index]
        infos.sort(key=lambda ri: (self.index[ri.node], ri.uid))
        nodes_by_name = {n: self.nodes[i] for n, i in self.index.items()}
        cls, rsv_cls, _ = rsvmatch.match_classes(list(pods), [pod_requests(p) for p in pods], [ri.obj for ri in infos],
                                                 nodes_by_name)
        by_uid = {ri.uid: c for ri, c in zip(infos, rsv_cls)}
        resv = self.reservations.restore_inputs(self.index, lambda ri: by_uid.get(ri.uid, []))
        table = self.table() if rows is None else rows
        t, views, vinfos, devs = decode.reservation_restore(table, resv)
        return np.array(cls, np.int32), t, abi.Reservations(views, vinfos, devs)

    def on_quota(self, q: dict):
        self.quotas.on_quota(q)

    def on_quota_delete(self, name: str):
        self.quotas.on_quota_delete(name)

    def assume(self, pod, node_name: str):
        """The scheduler's Reserve of a placement: cache AssumePod (NodeInfo) and LoadAware Reserve
        (podAssignCache.assign, load_aware.go:226-229)."""
        p = dict(pod)
        p["spec"] = dict(pod.get("spec") or {}, nodeName=node_name)
        self._nodeinfo_update(p)
        self.assign_cache.assign(node_name, p)
        return p

    def forget(self, pod, node_name: str):
        """Unreserve: ForgetPod and podAssignCache.unAssign (load_aware.go:231-233)."""
        self._nodeinfo_remove(_uid(pod))
        self.assign_cache.unassign(node_name, pod)

    def on_node_update(self, node: dict):
        i = self.index[_md(node).get("name", "")]
        self.nodes[i] = dict(node)
        self._touch(i)

    def on_node_metric(self, metric: dict):
        self.assign_cache.add_or_update_node_metric(metric)
        i = self.index.get(_md(metric).get("name", ""))
        if i is not None:
            self._metric_token[i] += 1
            secs = self.la.node_metric_expiration_seconds
            ut = (metric.get("status") or {}).get("updateTime")
            if secs is not None and secs > 0 and ut is not None:
                heapq.heappush(self._expiry, (float(ut) + secs, i, self._metric_token[i]))

    def on_node_metric_delete(self, name: str):
        self.assign_cache.delete_node_metric(name)
        i = self.index.get(name)
        if i is not None:
            self._metric_token[i] += 1

    def on_topology(self, name: str, zones: List[Dict[str, str]], kubelet_policy: str = "",
                    cpu_zone: Optional[Dict[int, int]] = None):
        i = self.index[name]
        t = self.topo[i]
        t.zones = list(zones)
        t.kubelet_policy = kubelet_policy
        if cpu_zone is not None and cpu_zone != t.cpu_zone:
            t.cpu_zone = dict(cpu_zone)
            old = self.numa[i]
            self.numa[i] = NodeAllocation()
            for uid, a in old.pods.items():  # re-place the allocations on the new topology
                self.numa[i].add(uid, a, t.cpu_zone)
        self._touch(i)

    def on_device(self, device: dict):
        self.devices.update_node_device(device)

    def on_device_delete(self, name: str):
        self.devices.remove_node_device(name)

    # -- rows ------------------------------------------------------------------------------------
    def _zone_used(self, i: int) -> Tuple[List[Dict[str, object]], int]:
        """getAvailableNUMANodeResources' totalAllocated (node_allocation.go:221-243, no reusable
        reservations) and the node's allocated cpuset size (plugin.go:485-490)."""
        t = self.topo[i]
        alloc = self.numa[i]
        ratio = float(json.loads((_md(self.nodes[i]).get("annotations") or {}).get(ANN_AMPLIFICATION) or "{}")
                      .get(CPU, 1.0))
        used: List[Dict[str, object]] = []
        for z in range(len(t.zones)):
            res = dict(alloc.zone_res.get(z, {}))
            if z in alloc.zone_res and ratio > 1 and t.cpu_zone:
                cs = sum(1 for c in alloc.cpu_refs if t.cpu_zone.get(c, 0) == z) * 1000
                cpu = milli_value(res.get(CPU, 0))
                res[CPU] = Fraction(cpu - cs + amplify(cs, ratio), 1000)
            used.append(res)
        cpuset_milli = len(alloc.cpu_refs) * 1000 if t.cpu_zone else 0
        return used, cpuset_milli

    def row(self, i: int) -> Dict[str, object]:
        """Snapshot row of node i from the incrementally maintained caches."""
        name = self.names[i]
        t = self.topo[i]
        row = node_static_cols(self.nodes[i], self.cfg, t.zones, t.kubelet_policy)
        row.update(nodeinfo_cols(self.req[i], int(self.num_pods[i])))
        cache = self.assign_cache.get(name) or LoadAwareNodeCache(la=self.la)
        row.update(la_cols(self.nodes[i], cache.metric, cache, self.la, self.clock()))
        used, cpuset_milli = self._zone_used(i)
        row.update(zone_used_cols(used, cpuset_milli))
        row["numa_zone_status"] = self.numa[i].zone_status(len(t.zones)) if t.cpu_zone else 0
        row["dev_minors"], row["dev_total"], row["dev_free"] = self.devices.columns(name)
        return row

    def table(self, rows: Optional[Iterable[int]] = None) -> abi.Table:
        rows = range(len(self.nodes)) if rows is None else list(rows)
        t = abi.empty_nodes(len(rows))
        for k, i in enumerate(rows):
            for key, v in self.row(int(i)).items():
                t[key][k] = v
        return t


class SnapshotSync:
    """Keeps device snapshots of a ClusterState current: each sync() sends the rows whose generation is
    newer than the last sync, as one batched kg_snapshot_update_rows per shard (a shard owns the global
    rows [index_base, index_base + n)). Rows are rebuilt from the caches, so a row the device changed by
    kg_assume is overwritten with the host's view of the same placement once its events arrive."""

    def __init__(self, state: ClusterState, snaps):
        self.state = state
        self.snaps = list(snaps) if isinstance(snaps, (list, tuple)) else [snaps]
        self.synced = state.generation
        self.last_rows = 0

    def sync(self) -> int:
        self.state.tick()
        rows = self.state.rows_since(self.synced)
        self.synced = self.state.generation
        self.last_rows = len(rows)
        if len(rows) == 0:
            return 0
        table = self.state.table(rows)
        for s in self.snaps:
            lo, hi = s.index_base, s.index_base + s.n
            sel = np.nonzero((rows >= lo) & (rows < hi))[0]
            if len(sel):
                s.update_rows(rows[sel] - lo, abi.take(table, sel))
        return len(rows)


# ---- Reservation cache (reservation/cache.go:761-1104, frameworkext/reservation_info.go) --------------------

ANN_RESERVATION_ALLOCATED = "scheduling.koordinator.sh/reservation-allocated"
LABEL_RESERVATION_ORDER = "scheduling.koordinator.sh/reservation-order"
RSV_VEC = (CPU, MEMORY, "ephemeral-storage")  # KG_RSV_R order: cpu, memory, ephemeral-storage, scalar0, scalar1


ANN_RESERVATION_RESTRICTED_OPTIONS = "scheduling.koordinator.sh/reservation-restricted-options"


def restricted_resources(names: List[str], annotations: Dict[str, str]) -> List[str]:
    """NewReservationInfo's ResourceNames of a Restricted reservation (frameworkext/reservation_info.go:92-107):
    the allocatable names intersected with the restricted-options annotation's resources
    (GetReservationRestrictedResources, util/reservation/reservation.go:677-694), all names when the
    intersection is empty; an annotation that does not parse (apis/extension/reservation.go:199-207) leaves the
    names as they are."""
    raw = annotations.get(ANN_RESERVATION_RESTRICTED_OPTIONS, "")
    if not raw:
        return names
    try:
        opts = json.loads(raw)
    except ValueError:
        return names
    if not isinstance(opts, dict):
        return names
    want = opts.get("resources") or []
    if not isinstance(want, list):
        return names
    out = [n for n in names if n in want]
    return out or names


class ReservationInfo:
    """frameworkext.ReservationInfo of a Reservation object: Allocatable (status), ResourceNames (its keys),
    Allocated = Σ Mask(requests, ResourceNames) of the assigned pods, the owners / policy / order the restore and
    the matching read."""

    def __init__(self, r: dict, cfg: SchedulerConfig):
        self.cfg = cfg
        self.assigned: Dict[str, List[int]] = {}  # pod uid -> masked request vector
        self.update(r)

    def update(self, r: dict):
        self.obj = r
        md, spec, status = _md(r), r.get("spec") or {}, r.get("status") or {}
        self.uid = md.get("uid", "")
        self.name = md.get("name", "")
        self.node = status.get("nodeName", "")
        self.phase = status.get("phase", "")
        alloc = status.get("allocatable") or {}
        self.allocatable = self._vec(alloc)
        self.max_pods = value(alloc["pods"]) if "pods" in alloc else -1
        self.policy = {"Aligned": abi.KG_RSV_ALIGNED, "Restricted": abi.KG_RSV_RESTRICTED}.get(
            spec.get("allocatePolicy", ""), abi.KG_RSV_DEFAULT)
        self.names = sorted(alloc)
        if self.policy == abi.KG_RSV_RESTRICTED:
            self.names = restricted_resources(self.names, md.get("annotations") or {})
        self.allocate_once = spec.get("allocateOnce", True) is not False
        self.terminating = md.get("deletionTimestamp") is not None
        try:
            self.order = int((md.get("labels") or {}).get(LABEL_RESERVATION_ORDER, "0"))
        except ValueError:
            self.order = 0

    def _vec(self, rl: dict) -> List[int]:
        names = [self.cfg.scalar_resources[k] if k < len(self.cfg.scalar_resources) else "" for k in range(abi.KG_NSCALAR)]
        out = []
        for k, key in enumerate(list(RSV_VEC) + names):
            q = rl.get(key)
            out.append(0 if q is None else (milli_value(q) if key == CPU else value(q)))
        return out

    def mask(self, req: Dict[str, object]) -> List[int]:
        """quotav1.Mask(requests, ResourceNames) as a KG_RSV_R vector."""
        return self._vec({k: v for k, v in req.items() if k in self.names})

    @property
    def allocated(self) -> List[int]:
        tot = [0] * abi.KG_RSV_R
        for v in self.assigned.values():
            tot = [a + b for a, b in zip(tot, v)]
        return tot

    def matchable(self) -> bool:
        """IsMatchable (reservation_info.go:546-569): Available, and not an allocate-once reservation with pods."""
        if self.phase != "Available":
            return False
        return not (self.allocate_once and len(self.assigned) > 0)


class ReservationCache:
    """reservationCache: reservation infos by uid, the reservations of each node, and the assigned-pod
    bookkeeping of addPod / updatePod / deletePod (keyed by the pod's reservation-allocated annotation)."""

    def __init__(self, cfg: SchedulerConfig, on_change: Callable[[str], None] = lambda node: None):
        self.cfg = cfg
        self.infos: Dict[str, ReservationInfo] = {}
        self.on_node: Dict[str, Set[str]] = {}
        self.on_change = on_change

    def update_reservation(self, r: dict):
        """updateReservation / assumeReservation (cache.go:785-844)."""
        uid = _md(r).get("uid", "")
        ri = self.infos.get(uid)
        old_node = ri.node if ri else ""
        if ri is None:
            ri = self.infos[uid] = ReservationInfo(r, self.cfg)
        else:
            ri.update(r)
        if old_node and old_node != ri.node:
            self.on_node.get(old_node, set()).discard(uid)
            self.on_change(old_node)
        if ri.node:
            self.on_node.setdefault(ri.node, set()).add(uid)
            self.on_change(ri.node)

    def delete_reservation(self, r: dict):
        """DeleteReservation / forgetReservation (cache.go:789-791,893-918)."""
        uid = _md(r).get("uid", "")
        ri = self.infos.pop(uid, None)
        node = (r.get("status") or {}).get("nodeName", "") or (ri.node if ri else "")
        if node:
            self.on_node.get(node, set()).discard(uid)
            self.on_change(node)

    @staticmethod
    def reservation_of(pod) -> str:
        raw = (_md(pod).get("annotations") or {}).get(ANN_RESERVATION_ALLOCATED)
        return (json.loads(raw) or {}).get("uid", "") if raw else ""

    def _add(self, ruid: str, pod) -> bool:
        ri = self.infos.get(ruid)
        if ri is None or ri.terminating or _uid(pod) in ri.assigned:
            return False  # addPods: unknown / terminating reservation; AddAssignedPod skips repeats
        ri.assigned[_uid(pod)] = ri.mask(pod_requests(pod))
        self.on_change(ri.node)
        return True

    def _remove(self, ruid: str, pod):
        ri = self.infos.get(ruid)
        if ri is not None and ri.assigned.pop(_uid(pod), None) is not None:
            self.on_change(ri.node)

    def add_pod(self, pod):
        ruid = self.reservation_of(pod)
        if ruid:
            self._add(ruid, pod)

    def update_pod(self, old, pod):
        """updatePod (cache.go:1047-1079): the old reservation forgets the pod, the new one adds it."""
        o, n = self.reservation_of(old) if old else "", self.reservation_of(pod)
        if o:
            self._remove(o, old)
        if n and not _is_terminated(pod):
            self._add(n, pod)

    def delete_pod(self, pod):
        ruid = self.reservation_of(pod)
        if ruid:
            self._remove(ruid, pod)

    def assume_pod(self, ruid: str, pod):
        """assumePod (cache.go:1004-1006): the scheduler's Reserve into a reservation."""
        return self._add(ruid, pod)

    def forget_pod(self, ruid: str, pod):
        self._remove(ruid, pod)

    def restore_inputs(self, node_index: Dict[str, int], classes_of=None) -> List[dict]:
        """The matchable reservations of every node as decode.reservation_restore reads them
        (ForEachMatchableReservationOnNode, cache.go:1162-1180); classes_of(info) -> owner-match classes."""
        out = []
        for name in sorted(self.on_node, key=lambda nm: node_index.get(nm, -1)):
            i = node_index.get(name)
            if i is None:
                continue
            for uid in sorted(self.on_node[name]):
                ri = self.infos[uid]
                if not ri.matchable():
                    continue
                names = 0
                for k, key in enumerate(list(RSV_VEC) + list(self.cfg.scalar_resources[:abi.KG_NSCALAR])):
                    if key in ri.names:
                        names |= 1 << k
                out.append(dict(node=i, cls=classes_of(ri) if classes_of else [], uid=uid,
                                allocatable=ri.allocatable, allocated=ri.allocated if ri.assigned else None,
                                reserved=None, allocated_pods=len(ri.assigned), policy=ri.policy, order=ri.order,
                                allocate_once=ri.allocate_once, max_pods=ri.max_pods, names=names))
        return out


# ---- ElasticQuota cache (elasticquota/quota_handler.go, core/group_quota_manager.go) ------------------------

LABEL_QUOTA_NAME = "quota.scheduling.koordinator.sh/name"
QUOTA_VEC = (CPU, MEMORY)  # KG_QUOTA_R order: cpu, memory, scalar0, scalar1


class QuotaCache:
    """Flat ElasticQuotas (EnableCheckParentQuota false, EnableRuntimeQuota false: usedLimit = max) kept from
    quota and pod events: OnQuotaAdd / OnQuotaUpdate / OnQuotaDelete set max / min, OnPodAdd / OnPodUpdate /
    OnPodDelete move the pod's request (Mask(requests, max names)) in and out of its quota's used, and of the
    non-preemptible used for non-preemptible pods. Rows are quota indices (stable: a deleted quota's row is
    cleared, not reused)."""

    def __init__(self, cfg: SchedulerConfig):
        self.cfg = cfg
        self.index: Dict[str, int] = {}
        self.max: List[Optional[Dict[str, object]]] = []
        self.min: List[Dict[str, object]] = []
        self.pods: Dict[str, Tuple[int, List[int], bool]] = {}  # uid -> (quota row, masked request, non-preemptible)
        self.generation = 0

    def _keys(self) -> List[str]:
        return list(QUOTA_VEC) + list(self.cfg.scalar_resources[:abi.KG_NSCALAR])

    def _vec(self, rl: Dict[str, object]) -> Tuple[List[int], int]:
        v, keys = [], 0
        for k, key in enumerate(self._keys()):
            q = rl.get(key)
            if q is not None:
                keys |= 1 << k
            v.append(0 if q is None else (milli_value(q) if key == CPU else value(q)))
        return v, keys

    def on_quota(self, q: dict):
        name = _md(q).get("name", "")
        spec = q.get("spec") or {}
        if name not in self.index:
            self.index[name] = len(self.max)
            self.max.append(None)
            self.min.append({})
        i = self.index[name]
        self.max[i] = dict(spec.get("max") or {})
        self.min[i] = dict(spec.get("min") or {})
        self.generation += 1

    def on_quota_delete(self, name: str):
        """OnQuotaDelete (quota_handler.go:102-133): the quota info goes with its used; its pods migrate to the
        default quota group, which this flat cache does not hold, so they leave the cache. A quota re-created
        under the same name starts from zero used, as the reference's new QuotaInfo does; its pods count again
        from their next OnPodAdd / OnPodUpdate (masked by the names current then, group_quota_manager.go:752)."""
        i = self.index.get(name)
        if i is not None:
            self.max[i] = None
            for uid in [u for u, ent in self.pods.items() if ent[0] == i]:
                del self.pods[uid]
            self.generation += 1

    def _quota_of(self, pod) -> Optional[int]:
        name = (_md(pod).get("labels") or {}).get(LABEL_QUOTA_NAME)
        i = self.index.get(name) if name else None
        return i if i is not None and self.max[i] is not None else None

    def on_pod(self, old, pod):
        """OnPodAdd / OnPodUpdate: an assigned, non-terminated pod counts in its quota's used."""
        uid = _uid(pod)
        ent = self.pods.pop(uid, None)
        if ent is not None:
            self.generation += 1
        i = self._quota_of(pod)
        if i is None or not _node_name(pod) or _is_terminated(pod):
            return
        mx = self.max[i]
        req = {k: v for k, v in pod_requests(pod).items() if k in mx}
        vec, _ = self._vec(req)
        np_ = (_md(pod).get("labels") or {}).get("quota.scheduling.koordinator.sh/preemptible") == "false"
        self.pods[uid] = (i, vec, np_)
        self.generation += 1

    def on_pod_delete(self, pod):
        if self.pods.pop(_uid(pod), None) is not None:
            self.generation += 1

    def columns(self) -> abi.Table:
        n = len(self.max)
        t = abi.empty_quotas(n)
        for i in range(n):
            if self.max[i] is None:
                continue
            t["used_limit"][i], t["limit_keys"][i] = self._vec(self.max[i])
            t["min"][i], t["min_keys"][i] = self._vec(self.min[i])
        for i, vec, np_ in self.pods.values():
            t["used"][i] += vec
            t["used_keys"][i] |= t["limit_keys"][i]
            if np_:
                t["np_used"][i] += vec
                t["np_used_keys"][i] |= t["limit_keys"][i]
        return t
