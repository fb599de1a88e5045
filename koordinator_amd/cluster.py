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
                     pod_request_vec, pod_requests, value, zone_used_cols, ResourceList)

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

    def zone_pods(self, n_zones: int) -> int:
        """The pods behind the statuses (kg_node_columns.numa_zone_pods): byte z = singleNUMANode[z], byte 4 + z =
        sharedNode[z] (saturating at 255), so that a device Release leaves the statuses the reference leaves."""
        w = 0
        for z in range(min(n_zones, abi.KG_MAX_ZONES)):
            w |= min(len(self.single.get(z, ())), 255) << (8 * z)
            w |= min(len(self.shared.get(z, ())), 255) << (8 * (abi.KG_MAX_ZONES + z))
        return w

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
        # the reservation's annotations travel with it (its resource status: the cpuset / NUMA resources it holds)
        return {"metadata": {"uid": "reserve-pod/" + md.get("uid", ""), "name": md.get("name", ""),
                             "annotations": dict(md.get("annotations") or {})},
                "spec": {"nodeName": status.get("nodeName", ""), "containers": [{"resources": {"requests": alloc}}]}}

    def on_reservation(self, r: dict):
        """Reservation add / update: the reservation cache (updateReservation) and its reserve pod in NodeInfo
        while it is Available on a node; the NUMA resource manager takes the reserve pod's resource status like a
        pod's (NewReservationToPodEventHandler, nodenumaresource/pod_eventhandler.go:47-49)."""
        self.reservations.update_reservation(r)
        rp = self._reserve_pod(r)
        if (r.get("status") or {}).get("phase") == "Available" and _node_name(rp):
            self._nodeinfo_update(rp)
            self._numa_update(None, rp)
        else:
            self._nodeinfo_remove(_uid(rp))
            if _node_name(rp):
                self._numa_release(_node_name(rp), _uid(rp))

    def on_reservation_delete(self, r: dict):
        self.reservations.delete_reservation(r)
        rp = self._reserve_pod(r)
        self._nodeinfo_remove(_uid(rp))
        if _node_name(rp):
            self._numa_release(_node_name(rp), _uid(rp))

    def reservation_restore(self, pods: Sequence[dict], rows: Optional[abi.Table] = None):
        """The Reservation transformer's restore for a pending batch: owner-match classes of the pods over the
        matchable reservations (rsvmatch.match_classes), then decode.reservation_restore over the current rows.
        Returns (rsv_class per pod, restored node table, abi.Reservations)."""
        from . import decode, rsvmatch
        infos = list({ri.uid: ri for _, ri in self.reservations.matchable_infos(self.index)}.values())
        nodes_by_name = {n: self.nodes[i] for n, i in self.index.items()}
        cls, rsv_cls, _ = rsvmatch.match_classes(list(pods), [pod_requests(p) for p in pods], [ri.obj for ri in infos],
                                                 nodes_by_name)
        by_uid = {ri.uid: c for ri, c in zip(infos, rsv_cls)}
        resv = self.reservations.restore_inputs(self.index, lambda ri: by_uid.get(ri.uid, []))
        table = self.table() if rows is None else rows
        t, views, vinfos, devs = decode.reservation_restore(table, resv)
        return np.array(cls, np.int32), t, abi.Reservations(views, vinfos, devs)

    def on_quota(self, q: dict, add: bool = False):
        self.quotas.on_quota(q, add)

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
        row = node_static_cols(self.nodes[i], self.cfg, t.zones, t.kubelet_policy, self.la)
        row.update(nodeinfo_cols(self.req[i], int(self.num_pods[i])))
        cache = self.assign_cache.get(name) or LoadAwareNodeCache(la=self.la)
        row.update(la_cols(self.nodes[i], cache.metric, cache, self.la, self.clock()))
        used, cpuset_milli = self._zone_used(i)
        row.update(zone_used_cols(used, cpuset_milli))
        row["numa_zone_status"] = self.numa[i].zone_status(len(t.zones)) if t.cpu_zone else 0
        row["numa_zone_pods"] = self.numa[i].zone_pods(len(t.zones)) if t.cpu_zone else 0
        # a reservation's reserve pod holds a NUMA / cpuset allocation here (kg_node_columns.rsv_numa)
        row["rsv_numa"] = int(any(uid.startswith("reserve-pod/") for uid in self.numa[i].pods))
        row["dev_minors"], row["dev_total"], row["dev_free"] = self.devices.columns(name)
        return row

    def table(self, rows: Optional[Iterable[int]] = None) -> abi.Table:
        rows = range(len(self.nodes)) if rows is None else list(rows)
        t = abi.empty_nodes(len(rows))
        t["numa_zone_pods"] = np.zeros(len(rows), np.uint64)
        t["rsv_numa"] = np.zeros(len(rows), np.uint8)
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
    names as they are (and is the info's ParseError, restricted_options_ok)."""
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


def restricted_options_ok(annotations: Dict[str, str]) -> bool:
    """GetReservationRestrictedOptions (apis/extension/reservation.go:199-207) parses the annotation without error."""
    raw = annotations.get(ANN_RESERVATION_RESTRICTED_OPTIONS, "")
    if not raw:
        return True
    try:
        opts = json.loads(raw)
    except ValueError:
        return False
    return isinstance(opts, dict) and isinstance(opts.get("resources") or [], list)


# quotav1 (k8s.io/apiserver/pkg/quota/v1) over ResourceList (name -> exact Fraction)
def quota_add(a: Optional[ResourceList], b: ResourceList) -> ResourceList:
    """quotav1.Add: every key of a and b, summed."""
    out = dict(a or {})
    for k, v in b.items():
        out[k] = out.get(k, Fraction(0)) + v
    return out


def quota_sub_nonneg(a: Optional[ResourceList], b: ResourceList) -> ResourceList:
    """quotav1.SubtractWithNonNegativeResult: a - b per key of a (floored at 0), keys only in b at 0."""
    out = {}
    for k, v in (a or {}).items():
        d = v - b.get(k, Fraction(0))
        out[k] = d if d > 0 else Fraction(0)
    for k in b:
        out.setdefault(k, Fraction(0))
    return out


def quota_mask(a: Optional[ResourceList], names: Iterable[str]) -> ResourceList:
    """quotav1.Mask: the keys of a among names."""
    names = set(names)
    return {k: v for k, v in (a or {}).items() if k in names}


def reservation_requests(r: dict) -> ResourceList:
    """reservationutil.ReservationRequests (util/reservation/reservation.go:393-404): status.allocatable of an
    Available reservation on a node, else the PodRequests of its template."""
    status, spec = r.get("status") or {}, r.get("spec") or {}
    if status.get("phase") == "Available" and status.get("nodeName"):
        return _rl(status.get("allocatable"))
    tmpl = spec.get("template")
    if tmpl is not None:
        return pod_requests({"spec": (tmpl or {}).get("spec") or {}})
    return {}


class ReservationInfo:
    """frameworkext.ReservationInfo of a Reservation object (reservation_info.go:92-132,400-442,490-569):
    Allocatable (ReservationRequests), ResourceNames (its keys, sorted; restricted for a Restricted policy),
    Allocated (quotav1.Add of each assigned pod's Mask(requests, ResourceNames) at its add, nil until the first
    pod; masked again when ResourceNames change; SubtractWithNonNegativeResult at a pod's removal), AssignedPods,
    and the owners / policy / order the restore and the matching read."""

    def __init__(self, r: dict, cfg: SchedulerConfig):
        self.cfg = cfg
        self.assigned: Dict[str, ResourceList] = {}  # AssignedPods: pod uid -> PodRequirement.Requests
        self.allocated_rl: Optional[ResourceList] = None
        self._set(r)

    def _set(self, r: dict):
        self.obj = r
        md, spec, status = _md(r), r.get("spec") or {}, r.get("status") or {}
        self.uid = md.get("uid", "")
        self.name = md.get("name", "")
        self.node = status.get("nodeName", "")
        self.phase = status.get("phase", "")
        self.allocatable_rl = reservation_requests(r)
        alloc = status.get("allocatable") or {}
        self.max_pods = value(alloc["pods"]) if "pods" in alloc else -1
        self.policy = {"Aligned": abi.KG_RSV_ALIGNED, "Restricted": abi.KG_RSV_RESTRICTED}.get(
            spec.get("allocatePolicy", ""), abi.KG_RSV_DEFAULT)
        names = sorted(self.allocatable_rl)
        ann = md.get("annotations") or {}
        self.parse_error = False
        if self.policy == abi.KG_RSV_RESTRICTED:
            names = restricted_resources(names, ann)
            self.parse_error = not restricted_options_ok(ann)
        self.names = names
        self.allocate_once = spec.get("allocateOnce", True) is not False
        self.terminating = md.get("deletionTimestamp") is not None
        try:
            self.order = int((md.get("labels") or {}).get(LABEL_RESERVATION_ORDER, "0"))
        except ValueError:
            self.order = 0

    def update(self, r: dict):
        """UpdateReservation (reservation_info.go:400-442): Allocated masked by the new ResourceNames."""
        self._set(r)
        if self.allocated_rl is not None:
            self.allocated_rl = quota_mask(self.allocated_rl, self.names)

    def add_assigned_pod(self, uid: str, requests: ResourceList) -> bool:
        """AddAssignedPod (:490-500): a repeated pod is skipped."""
        if uid in self.assigned:
            return False
        self.allocated_rl = quota_add(self.allocated_rl, quota_mask(requests, self.names))
        self.assigned[uid] = dict(requests)
        return True

    def remove_assigned_pod(self, uid: str) -> bool:
        """RemoveAssignedPod (:502-514)."""
        req = self.assigned.pop(uid, None)
        if req is None:
            return False
        if req:
            self.allocated_rl = quota_sub_nonneg(self.allocated_rl, quota_mask(req, self.names))
        return True

    @property
    def allocated_pods(self) -> int:
        return len(self.assigned)

    def _vec(self, rl: Optional[ResourceList]) -> List[int]:
        names = [self.cfg.scalar_resources[k] if k < len(self.cfg.scalar_resources) else "" for k in range(abi.KG_NSCALAR)]
        out = []
        for key in list(RSV_VEC) + names:
            q = (rl or {}).get(key)
            out.append(0 if q is None else (milli_value(q) if key == CPU else value(q)))
        return out

    @property
    def allocatable(self) -> List[int]:
        return self._vec(self.allocatable_rl)

    @property
    def allocated(self) -> List[int]:
        """Allocated as a KG_RSV_R vector (zeros while nil)."""
        return self._vec(self.allocated_rl)

    def allocated_keys(self) -> int:
        """The cpu / memory keys present in Allocated (bit 0 / 1): GetNonZeroRequestForResource reads the value of a
        present key and the default of a missing one (reservation_info.go:516-529,581-605)."""
        a = self.allocated_rl or {}
        return (1 if CPU in a else 0) | (2 if MEMORY in a else 0)

    def is_matchable(self) -> bool:
        """IsMatchable (reservation_info.go:546-569): Available on a node, no parse error, not an allocate-once
        reservation with pods."""
        if self.phase != "Available" or not self.node or self.parse_error:
            return False
        return not (self.allocate_once and self.allocated_pods > 0)

    matchable = is_matchable


class ReservationCache:
    """reservationCache (reservation/cache.go:761-1205): reservation infos by uid, reservationsOnNode,
    matchableOnNode and allocatedOnNode (refreshed the way the reference refreshes them: matchable on reservation
    updates only, allocated on pod adds / removals too), and the assigned-pod bookkeeping of addPod / updatePod /
    deletePod (keyed by the pod's reservation-allocated annotation)."""

    def __init__(self, cfg: SchedulerConfig, on_change: Callable[[str], None] = lambda node: None):
        self.cfg = cfg
        self.infos: Dict[str, ReservationInfo] = {}
        self.on_node: Dict[str, Set[str]] = {}
        self.matchable_on_node: Dict[str, Set[str]] = {}
        self.allocated_on_node: Dict[str, Set[str]] = {}
        self.on_change = on_change

    @staticmethod
    def _drop(m: Dict[str, Set[str]], node: str, uid: str):
        s = m.get(node)
        if s is not None:
            s.discard(uid)
            if not s:
                del m[node]

    def _refresh(self, ri: ReservationInfo, node: str):
        """The matchable / allocated refresh of updateReservation / updateReservationIfExists (:813-843)."""
        if ri.is_matchable():
            self.matchable_on_node.setdefault(node, set()).add(ri.uid)
            if ri.allocated_pods > 0:
                self.allocated_on_node.setdefault(node, set()).add(ri.uid)
            elif node in self.allocated_on_node:
                self.allocated_on_node[node].discard(ri.uid)
        else:
            self._drop(self.matchable_on_node, node, ri.uid)
            self._drop(self.allocated_on_node, node, ri.uid)

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
            self.on_change(old_node)
        if ri.node:
            self.on_node.setdefault(ri.node, set()).add(uid)
            self._refresh(ri, ri.node)
            self.on_change(ri.node)

    def update_reservation_if_exists(self, r: dict):
        """updateReservationIfExists (cache.go:846-891): an unknown reservation is not created."""
        uid = _md(r).get("uid", "")
        ri = self.infos.get(uid)
        if ri is None:
            return
        ri.update(r)
        if ri.node:
            self._refresh(ri, ri.node)
            self.on_change(ri.node)

    def delete_reservation(self, r: dict):
        """DeleteReservation / forgetReservation (cache.go:789-791,893-918): the sets of the object's node."""
        uid = _md(r).get("uid", "")
        ri = self.infos.pop(uid, None)
        node = (r.get("status") or {}).get("nodeName", "")
        # the reference clears the object's node only; a tombstone without nodeName would leave the uid in the sets of
        # the node the cache knew, where for_each_matchable skips it (infos no longer hold it)
        for m in (self.on_node, self.matchable_on_node, self.allocated_on_node):
            self._drop(m, node, uid)
        for n in {node, ri.node if ri else ""} - {""}:
            self.on_change(n)
        return ri

    def get(self, uid: str) -> Optional[ReservationInfo]:
        """getReservationInfoByUID (cache.go:1115-1123)."""
        return self.infos.get(uid)

    def list_all_nodes(self, matchable: bool) -> List[str]:
        """ListAllNodes (cache.go:1138-1160): nodes with matchable reservations, or (matchable False) with allocated
        ones; nothing when no node has a matchable reservation."""
        if not self.matchable_on_node:
            return []
        return sorted(self.matchable_on_node if matchable else self.allocated_on_node)

    def for_each_matchable(self, node: str, fn) -> None:
        """ForEachMatchableReservationOnNode (cache.go:1162-1180): fn(info) -> continue?"""
        for uid in sorted(self.matchable_on_node.get(node, ())):
            ri = self.infos.get(uid)
            if ri is None:  # a delete whose object named another node left the uid here
                continue
            if not fn(ri):
                return

    def list_available(self, node: str, list_all: bool) -> List[ReservationInfo]:
        """ListAvailableReservationInfosOnNode (cache.go:1182-1205)."""
        if not list_all:
            out: List[ReservationInfo] = []
            self.for_each_matchable(node, lambda ri: out.append(ri) or True)
            return out
        return [self.infos[u] for u in sorted(self.on_node.get(node, ())) if u in self.infos]

    @staticmethod
    def reservation_of(pod) -> str:
        raw = (_md(pod).get("annotations") or {}).get(ANN_RESERVATION_ALLOCATED)
        return (json.loads(raw) or {}).get("uid", "") if raw else ""

    def _add(self, ruid: str, pod) -> bool:
        """addPods (cache.go:1020-1045): unknown / terminating reservations refuse."""
        ri = self.infos.get(ruid)
        if ri is None or ri.terminating:
            return False
        added = ri.add_assigned_pod(_uid(pod), pod_requests(pod))
        if ri.is_matchable() and ri.allocated_pods > 0 and ri.node:
            self.allocated_on_node.setdefault(ri.node, set()).add(ruid)
        self.on_change(ri.node)
        return added

    def _remove(self, ruid: str, pod):
        """deletePods (cache.go:1085-1105)."""
        ri = self.infos.get(ruid)
        if ri is None:
            return
        ri.remove_assigned_pod(_uid(pod))
        if ri.allocated_pods == 0 and ri.node:
            self._drop(self.allocated_on_node, ri.node, ruid)
        self.on_change(ri.node)

    def add_pod(self, pod):
        ruid = self.reservation_of(pod)
        if ruid:
            self._add(ruid, pod)

    def update_pod_in(self, old_ruid: str, new_ruid: str, old, pod):
        """updatePod (cache.go:1047-1079): the old reservation forgets the pod, the new one adds it."""
        ri = self.infos.get(old_ruid)
        if ri is not None and old is not None:
            self._remove(old_ruid, old)
        ri = self.infos.get(new_ruid)
        if ri is not None and pod is not None:
            ri.add_assigned_pod(_uid(pod), pod_requests(pod))
            if ri.is_matchable() and ri.allocated_pods > 0 and ri.node:
                self.allocated_on_node.setdefault(ri.node, set()).add(new_ruid)
            self.on_change(ri.node)

    def update_pod(self, old, pod):
        """The pod event handler's update: reservations named by the old and new reservation-allocated
        annotations (a terminated pod leaves its reservation)."""
        o, n = self.reservation_of(old) if old else "", self.reservation_of(pod)
        self.update_pod_in(o, n if not _is_terminated(pod) else "", old, pod)

    def delete_pod(self, pod):
        ruid = self.reservation_of(pod)
        if ruid:
            self._remove(ruid, pod)

    def assume_pod(self, ruid: str, pod):
        """assumePod (cache.go:1004-1006): the scheduler's Reserve into a reservation."""
        return self._add(ruid, pod)

    def forget_pod(self, ruid: str, pod):
        self._remove(ruid, pod)

    def matchable_infos(self, node_index: Dict[str, int]) -> List[Tuple[str, ReservationInfo]]:
        """The (node, reservation) pairs ForEachMatchableReservationOnNode visits on the indexed nodes, in node order,
        keyed by the node walked: a reservation whose nodeName changed stays in its old node's sets (updateReservation
        adds it to the new node's and removes nothing, cache.go:793-844), so the old node's walk visits it as well."""
        out: List[Tuple[str, ReservationInfo]] = []
        for name in sorted(self.matchable_on_node, key=lambda nm: node_index.get(nm, -1)):
            if name in node_index:
                self.for_each_matchable(name, lambda ri, nm=name: out.append((nm, ri)) or True)
        return out

    def restore_inputs(self, node_index: Dict[str, int], classes_of=None) -> List[dict]:
        """The matchable reservations of every node as decode.reservation_restore reads them
        (ForEachMatchableReservationOnNode, cache.go:1162-1180), one entry per (node walked, reservation);
        classes_of(info) -> owner-match classes."""
        out = []
        for name, ri in self.matchable_infos(node_index):
            names = 0
            for k, key in enumerate(list(RSV_VEC) + list(self.cfg.scalar_resources[:abi.KG_NSCALAR])):
                if key in ri.names:
                    names |= 1 << k
            out.append(dict(node=node_index[name], cls=classes_of(ri) if classes_of else [], uid=ri.uid,
                            allocatable=ri.allocatable,
                            allocated=ri.allocated if ri.allocated_rl is not None else None,
                            allocated_keys=ri.allocated_keys(), reserved=None, allocated_pods=ri.allocated_pods,
                            policy=ri.policy, order=ri.order, allocate_once=ri.allocate_once, max_pods=ri.max_pods,
                            names=names))
        return out


# ---- ElasticQuota cache (elasticquota/quota_handler.go, core/group_quota_manager.go) ------------------------

LABEL_QUOTA_NAME = "quota.scheduling.koordinator.sh/name"
DEFAULT_QUOTA_NAME = "koordinator-default-quota"  # apis/extension/elastic_quota.go DefaultQuotaName
SYSTEM_QUOTA_NAME = "koordinator-system-quota"  # SystemQuotaName
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

    def on_quota(self, q: dict, add: bool = False):
        """OnQuotaAdd (add=True) / OnQuotaUpdate (quota_handler.go:35-100): a quota being deleted is ignored; an Add
        of a quota already held does not overwrite it."""
        md = _md(q)
        name = md.get("name", "")
        spec = q.get("spec") or {}
        if md.get("deletionTimestamp") is not None:
            return
        # OnQuotaAdd (quota_handler.go:55-58) keeps a quota it already holds, except the default and system quotas
        if add and name in self.index and self.max[self.index[name]] is not None and \
                name not in (DEFAULT_QUOTA_NAME, SYSTEM_QUOTA_NAME):
            return
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
