"""Host-side decode of Kubernetes-shaped objects into the engine's node and pod columns.

This is the work the Go side of the boundary does before calling the C ABI (SURVEY.md §8b,
"Host-side pre-computation"): resource.Quantity arithmetic, PodRequests, priority / QoS
classification, the LoadAware estimator and podAssignCache aggregates at a frozen snapshot time,
EstimateNode, custom threshold annotations and the NUMA topology options.

Objects are plain dicts in the shape of the Kubernetes JSON (``metadata``, ``spec``, ``status``).
Times are float seconds relative to the frozen snapshot time ``now`` (None = unset).
"""
from __future__ import annotations

import functools
import json
import math
import re
from dataclasses import dataclass, field
from fractions import Fraction
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .config import (BATCH_CPU, BATCH_MEMORY, CPU, EPHEMERAL, LA_RESOURCES, MEMORY, MID_CPU, MID_MEMORY, PODS,
                     LoadAwareArgs, SchedulerConfig)


class Unsupported(Exception):
    """The object needs a feature that is not on the device path (caller keeps the Go plugin)."""


# ---------------------------------------------------------------------------------------------
# resource.Quantity (k8s.io/apimachinery v0.35.6)

_SUFFIX = {
    "Ki": Fraction(2 ** 10), "Mi": Fraction(2 ** 20), "Gi": Fraction(2 ** 30), "Ti": Fraction(2 ** 40),
    "Pi": Fraction(2 ** 50), "Ei": Fraction(2 ** 60),
    "n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": Fraction(1),
    "k": Fraction(10 ** 3), "M": Fraction(10 ** 6), "G": Fraction(10 ** 9), "T": Fraction(10 ** 12),
    "P": Fraction(10 ** 15), "E": Fraction(10 ** 18),
}
_QRE = re.compile(r"^([+-]?[0-9.]+)([eE][+-]?[0-9]+|[a-zA-Z]*)$")


def parse_quantity(q) -> Fraction:
    """Exact value of a Quantity string (or number)."""
    if isinstance(q, Fraction):
        return q
    if isinstance(q, int):
        return Fraction(q)
    if isinstance(q, float):
        return Fraction(q)
    if isinstance(q, str):
        return _parse_quantity_str(q)
    return _parse_quantity_str(str(q))


@functools.lru_cache(maxsize=65536)
def _parse_quantity_str(q: str) -> Fraction:
    """parse_quantity of a string, memoised: an event stream repeats a few hundred distinct quantities, and a
    Fraction is immutable (the host event layer spent a third of its time here)."""
    m = _QRE.match(q.strip())
    if not m:
        raise ValueError(f"invalid quantity {q!r}")
    num, suf = m.groups()
    v = Fraction(num)
    if suf and suf[0] in "eE" and len(suf) > 1 and (suf[1:].lstrip("+-").isdigit()):
        return v * Fraction(10) ** int(suf[1:])
    if suf not in _SUFFIX:
        raise ValueError(f"invalid quantity suffix {q!r}")
    return v * _SUFFIX[suf]


def value(q) -> int:
    """Quantity.Value(): rounded up to the nearest integer."""
    return math.ceil(parse_quantity(q))


def milli_value(q) -> int:
    """Quantity.MilliValue(): value*1000 rounded up."""
    return math.ceil(parse_quantity(q) * 1000)


def vec_value(name: str, q) -> int:
    """getResourceValue (loadaware/helper.go:124-129): cpu in milli, others as Value()."""
    return milli_value(q) if name == CPU else value(q)


def go_round(x: float) -> float:
    """math.Round: nearest integer, halves away from zero."""
    t = math.trunc(x)
    if abs(x - t) >= 0.5:
        t += math.copysign(1.0, x)
    return t


ResourceList = Dict[str, Fraction]


def _rl(d) -> ResourceList:
    return {k: parse_quantity(v) for k, v in (d or {}).items()}


def _add(dst: ResourceList, src: ResourceList):
    for k, v in src.items():
        dst[k] = dst[k] + v if k in dst else v


def _max(dst: ResourceList, src: ResourceList):
    for k, v in src.items():
        if k not in dst or v > dst[k]:
            dst[k] = v


# ---------------------------------------------------------------------------------------------
# Pods

def _containers(pod):
    return (pod.get("spec") or {}).get("containers") or []


def _init_containers(pod):
    return (pod.get("spec") or {}).get("initContainers") or []


def _restartable(c) -> bool:
    return c.get("restartPolicy") == "Always"


def pod_requests(pod, non_missing: Optional[ResourceList] = None) -> ResourceList:
    """k8s.io/component-helpers resource.PodRequests (KEP-753 sidecar rules, overhead added)."""
    def creqs(c):
        r = _rl((c.get("resources") or {}).get("requests"))
        if non_missing:
            for k, v in non_missing.items():
                if k not in r:
                    r[k] = v
        return r

    containers, inits = _containers(pod), _init_containers(pod)
    if len(containers) == 1 and not inits and not (pod.get("spec") or {}).get("overhead"):
        return creqs(containers[0])  # the common pod: one container, its requests as they are
    reqs: ResourceList = {}
    for c in containers:
        _add(reqs, creqs(c))
    restartable: ResourceList = {}
    init_reqs: ResourceList = {}
    for c in inits:
        cr = creqs(c)
        if _restartable(c):
            _add(reqs, cr)
            _add(restartable, cr)
            cr = dict(restartable)
        else:
            tmp: ResourceList = {}
            _add(tmp, cr)
            _add(tmp, restartable)
            cr = tmp
        _max(init_reqs, cr)
    _max(reqs, init_reqs)
    overhead = (pod.get("spec") or {}).get("overhead")
    if overhead:
        _add(reqs, _rl(overhead))
    return reqs


def pod_limits(pod) -> ResourceList:
    """resource.PodLimits: container limits aggregated like requests; overhead added to present limits."""
    lim: ResourceList = {}
    for c in _containers(pod):
        _add(lim, _rl((c.get("resources") or {}).get("limits")))
    restartable: ResourceList = {}
    init_lim: ResourceList = {}
    for c in _init_containers(pod):
        cl = _rl((c.get("resources") or {}).get("limits"))
        if _restartable(c):
            _add(lim, cl)
            _add(restartable, cl)
            cl = dict(restartable)
        else:
            tmp: ResourceList = {}
            _add(tmp, cl)
            _add(tmp, restartable)
            cl = tmp
        _max(init_lim, cl)
    _max(lim, init_lim)
    overhead = (pod.get("spec") or {}).get("overhead")
    if overhead:
        for k, v in _rl(overhead).items():
            if k in lim:
                lim[k] += v
    return lim


# upstream schedutil.DefaultMilliCPURequest / DefaultMemoryRequest (100m / 200Mi)
NON_MISSING = {CPU: Fraction(1, 10), MEMORY: Fraction(200 * 1024 * 1024)}

LABEL_PRIORITY_CLASS = "koordinator.sh/priority-class"
LABEL_QOS = "koordinator.sh/qosClass"
PRIORITY_RANGES = [("koord-prod", 9000, 9999), ("koord-mid", 7000, 7999), ("koord-batch", 5000, 5999),
                   ("koord-free", 3000, 3999)]
PROD, MID, BATCH, FREE, NONE = "koord-prod", "koord-mid", "koord-batch", "koord-free", ""


def kube_qos(pod) -> str:
    """qos.GetPodQOS (k8s.io/kubernetes pkg/apis/core/v1/helper/qos): cpu/memory only."""
    st = (pod.get("status") or {}).get("qosClass")
    if st:
        return st
    requests: ResourceList = {}
    limits: ResourceList = {}
    guaranteed = True
    for c in list(_containers(pod)) + list(_init_containers(pod)):
        res = c.get("resources") or {}
        for name, q in _rl(res.get("requests")).items():
            if name in (CPU, MEMORY) and q > 0:
                requests[name] = requests.get(name, Fraction(0)) + q
        found = set()
        for name, q in _rl(res.get("limits")).items():
            if name in (CPU, MEMORY) and q > 0:
                found.add(name)
                limits[name] = limits.get(name, Fraction(0)) + q
        if not {CPU, MEMORY} <= found:
            guaranteed = False
    if not requests and not limits:
        return "BestEffort"
    if guaranteed:
        for name, req in requests.items():
            if name not in limits or limits[name] != req:
                guaranteed = False
                break
    if guaranteed and len(requests) == len(limits):
        return "Guaranteed"
    return "Burstable"


def koord_qos_raw(pod) -> str:
    labels = (pod.get("metadata") or {}).get("labels") or {}
    q = labels.get(LABEL_QOS)
    return q if q in ("LSE", "LSR", "LS", "BE", "SYSTEM") else ""


def priority_class(pod) -> str:
    """extension.GetPodPriorityClassWithDefault (apis/extension/priority_utils.go:37-57)."""
    labels = (pod.get("metadata") or {}).get("labels") or {}
    raw = NONE
    if LABEL_PRIORITY_CLASS in labels:
        v = labels[LABEL_PRIORITY_CLASS]
        raw = v if v in (PROD, MID, BATCH, FREE) else NONE
    else:
        p = (pod.get("spec") or {}).get("priority")
        if p is not None:
            for name, lo, hi in PRIORITY_RANGES:
                if lo <= p <= hi:
                    raw = name
                    break
    if raw != NONE:
        return raw
    qos = koord_qos_raw(pod)
    if not qos:
        qos = {"Guaranteed": "LSR", "Burstable": "LS", "BestEffort": "BE"}[kube_qos(pod)]
    if qos in ("SYSTEM", "LSE", "LSR", "LS"):
        return PROD
    if qos == "BE":
        return BATCH
    return NONE


def translate_resource(pclass: str, name: str) -> str:
    """TranslateResourceNameByPriorityClass (apis/extension/resource.go:64-70)."""
    if pclass in (PROD, NONE):
        return name
    table = {BATCH: {CPU: BATCH_CPU, MEMORY: BATCH_MEMORY}, MID: {CPU: MID_CPU, MEMORY: MID_MEMORY}}
    return table.get(pclass, {}).get(name, "")


DEFAULT_EST_MILLI_CPU = 250
DEFAULT_EST_MEMORY = 200 * 1024 * 1024


def _estimated_used_by_resource(requests: ResourceList, limits: ResourceList, name: str, factor: int) -> int:
    """estimatedUsedByResource (loadaware/estimator/default_estimator.go:87-120)."""
    lq = limits.get(name, Fraction(0))
    rq = requests.get(name, Fraction(0))
    q = lq if lq > rq else rq
    if q == 0:
        if name in (CPU, BATCH_CPU):
            return DEFAULT_EST_MILLI_CPU
        if name in (MEMORY, BATCH_MEMORY):
            return DEFAULT_EST_MEMORY
        return 0
    if name == CPU:
        est = int(go_round(float(milli_value(q)) * float(factor) / 100))
        lim = milli_value(lq)
    else:
        est = int(go_round(float(value(q)) * float(factor) / 100))
        lim = value(lq)
    if lim > 0 and est > lim:
        est = lim
    return est


ANN_CUSTOM_ESTIMATED_SCALING_FACTORS = "scheduling.koordinator.sh/load-estimated-scaling-factors"


def estimate_pod(pod, la: LoadAwareArgs) -> List[int]:
    """DefaultEstimator.EstimatePod -> vectorizer.ToFactorVec (default_estimator.go:57-85)."""
    factors = dict(la.estimated_scaling_factors or {})
    if la.allow_customize_estimation:
        ann = ((pod.get("metadata") or {}).get("annotations") or {}).get(ANN_CUSTOM_ESTIMATED_SCALING_FACTORS)
        if ann:
            try:
                custom = {k: int(v) for k, v in json.loads(ann).items()}
            except Exception:
                custom = {}
            if custom:
                for k, v in factors.items():
                    custom.setdefault(k, v)
                factors = custom
    requests, limits = pod_requests(pod), pod_limits(pod)
    pc = priority_class(pod)
    est = {}
    for name, f in factors.items():
        est[name] = _estimated_used_by_resource(requests, limits, translate_resource(pc, name), f)
    return [est.get(r, 0) for r in LA_RESOURCES]


def is_daemonset_pod(pod) -> bool:
    return any(o.get("kind") == "DaemonSet" for o in ((pod.get("metadata") or {}).get("ownerReferences") or []))


ANN_NUMA_TOPOLOGY_SPEC = "scheduling.koordinator.sh/numa-topology-spec"
ANN_RESOURCE_SPEC = "scheduling.koordinator.sh/resource-spec"
DEFAULT_CPU_BIND_POLICY = "FullPCPUs"  # NodeNUMAResourceArgs default (v1/defaults.go:50)


def cpu_bind_flags(pod, req_cpu_milli: int, default_policy: str = DEFAULT_CPU_BIND_POLICY) -> int:
    """KG_POD_CPU_* bits of an AllowUseCPUSet pod (nodenumaresource/plugin.go:331-349,
    apis/extension/numa_aware.go:63-71,231-244). A Full/Spread policy with a fractional cpu request is
    ErrInvalidRequestedCPUs at PreFilter: Unsupported here (the pod never reaches Filter)."""
    ann = (pod.get("metadata") or {}).get("annotations") or {}
    spec = json.loads(ann[ANN_RESOURCE_SPEC]) if ann.get(ANN_RESOURCE_SPEC) else {}
    preferred = spec.get("preferredCPUBindPolicy") or ""
    if preferred in ("", "Default"):
        preferred = default_policy or DEFAULT_CPU_BIND_POLICY
    required = spec.get("requiredCPUBindPolicy") or ""
    if required == "Default":
        required = default_policy or DEFAULT_CPU_BIND_POLICY
    policy = required or preferred
    if policy not in ("FullPCPUs", "SpreadByPCPUs"):
        return 0
    if req_cpu_milli % 1000 != 0:
        raise Unsupported("cpuset-binding pod with a fractional cpu request (ErrInvalidRequestedCPUs at PreFilter)")
    if req_cpu_milli <= 0:
        return 0
    flags = abi.KG_POD_CPU_BIND | (abi.KG_CPU_BIND[policy] << abi.KG_POD_CPU_POLICY_SHIFT)
    if required:
        flags |= abi.KG_POD_CPU_REQUIRED
    flags |= abi.KG_CPU_EXCL.get(spec.get("preferredCPUExclusivePolicy") or "", 0) << abi.KG_POD_CPU_EXCL_SHIFT
    return flags


def pod_row(pod, cfg: SchedulerConfig) -> Dict[str, int]:
    """Pod columns (kg_pod_columns) for one pending pod."""
    la = cfg.la()
    req = pod_requests(pod)
    nz = pod_requests(pod, NON_MISSING)
    row = {
        "req_cpu": milli_value(req.get(CPU, 0)),
        "req_mem": value(req.get(MEMORY, 0)),
        "req_eph": value(req.get(EPHEMERAL, 0)),
        "nz_cpu": milli_value(nz.get(CPU, 0)),
        "nz_mem": value(nz.get(MEMORY, 0)),
    }
    for k, name in enumerate(cfg.scalar_resources):
        row[f"sc_req{k}"] = value(req.get(name, 0))
    if cfg.plugins & abi.KG_PLUGIN_NRF:
        # fitsRequest checks every requested scalar; only the snapshot's scalar slots are on device
        for name, q in req.items():
            if name in (CPU, MEMORY, EPHEMERAL, PODS) or name in cfg.scalar_resources:
                continue
            if q != 0:
                raise Unsupported(f"scalar resource {name} is not a snapshot column")
    for r, v in enumerate(estimate_pod(pod, la)):
        row[f"la_est{r}"] = v
    flags = 0
    if is_daemonset_pod(pod):
        flags |= abi.KG_POD_DAEMONSET
    pc = priority_class(pod)
    if pc == PROD:
        flags |= abi.KG_POD_PROD
    if all(v == 0 for v in req.values()):
        flags |= abi.KG_POD_NUMA_SKIP
    if CPU in req:
        flags |= abi.KG_POD_HAS_CPU
    if MEMORY in req:
        flags |= abi.KG_POD_HAS_MEM
    # AllowUseCPUSet (nodenumaresource/util.go:49-56) and the PreFilter's bind request (plugin.go:319-349):
    # LSE/LSR prod pods bind cpusets with the resource-spec annotation's policies, DefaultCPUBindPolicy
    # (FullPCPUs, v1/defaults.go:50) filling in "" / "Default"; a required policy wins
    if koord_qos_raw(pod) in ("LSE", "LSR") and pc == PROD and (cfg.plugins & abi.KG_PLUGIN_NUMA):
        flags |= cpu_bind_flags(pod, row["req_cpu"], cfg.default_cpu_bind_policy)
    ann = (pod.get("metadata") or {}).get("annotations") or {}
    if ann.get(ANN_NUMA_TOPOLOGY_SPEC):
        raise Unsupported("pod NUMA topology spec (exclusive-policy admission) is not on the device path")
    row["flags"] = flags
    row["numa_policy"] = abi.KG_NUMA_NONE
    return row


def pods_table(pods: Sequence[dict], cfg: SchedulerConfig) -> abi.Table:
    t = abi.empty_pods(len(pods))
    for j, p in enumerate(pods):
        for k, v in pod_row(p, cfg).items():
            t[k][j] = v
    return t


# ---------------------------------------------------------------------------------------------
# Nodes

ANN_CUSTOM_USAGE_THRESHOLDS = "scheduling.koordinator.sh/usage-thresholds"
ANN_RAW_ALLOCATABLE = "node.koordinator.sh/raw-allocatable"
ANN_AMPLIFICATION = "node.koordinator.sh/resource-amplification-ratio"
LABEL_NUMA_POLICY = "node.koordinator.sh/numa-topology-policy"
NUMA_POLICIES = {"": abi.KG_NUMA_NONE, "BestEffort": abi.KG_NUMA_BEST_EFFORT,
                 "Restricted": abi.KG_NUMA_RESTRICTED, "SingleNUMANode": abi.KG_NUMA_SINGLE_NODE}


def amplify(origin: int, ratio: float) -> int:
    """extension.Amplify (apis/extension/node_resource_amplification.go:170-175)."""
    if ratio <= 1:
        return origin
    return int(math.ceil(float(origin) * float(ratio)))


def _pod_key(pod) -> Tuple[str, str]:
    md = pod.get("metadata") or {}
    return (md.get("namespace", ""), md.get("name", ""))


def _is_terminated(pod) -> bool:
    return ((pod.get("status") or {}).get("phase") in ("Succeeded", "Failed"))


@dataclass
class _Profile:
    usage: List[int]
    prod: List[int]
    agg: Optional[Tuple[List[int], str, float]]


def _factor_vec(m: Dict[str, int]) -> List[int]:
    return [int(m.get(r, 0)) for r in LA_RESOURCES]


def filter_profile(node, la: LoadAwareArgs) -> _Profile:
    """NewUsageThresholdsFilterProfile + generateUsageThresholdsFilterProfile (loadaware/helper.go:59-121)."""
    base_agg = None
    a = la.aggregated
    if a is not None and len(a.usage_thresholds) > 0 and a.usage_aggregation_type != "":
        base_agg = (_factor_vec(a.usage_thresholds), a.usage_aggregation_type, a.usage_aggregated_duration)
    prof = _Profile(usage=_factor_vec(la.usage_thresholds) if la.usage_thresholds else [0] * abi.KG_LA_R,
                    prod=_factor_vec(la.prod_usage_thresholds) if la.prod_usage_thresholds else [0] * abi.KG_LA_R,
                    agg=base_agg)
    ann = ((node.get("metadata") or {}).get("annotations") or {}).get(ANN_CUSTOM_USAGE_THRESHOLDS)
    if ann is None:
        return prof
    try:
        c = json.loads(ann)
    except Exception:
        return prof
    cu = c.get("usageThresholds") or {}
    cp = c.get("prodUsageThresholds") or {}
    ca = c.get("aggregatedUsage")
    if ca is not None and not (len(ca.get("usageThresholds") or {}) > 0 and ca.get("usageAggregationType", "") != ""):
        ca = None
    if len(cu) == 0 and len(cp) == 0 and ca is None:
        return prof
    out = _Profile(usage=prof.usage if len(cu) == 0 else _factor_vec(cu),
                   prod=prof.prod if len(cp) == 0 else _factor_vec(cp), agg=prof.agg)
    if ca is not None:
        out.agg = (_factor_vec(ca["usageThresholds"]), ca["usageAggregationType"],
                   _duration(ca.get("usageAggregatedDuration")))
    return out


def _duration(d) -> float:
    """metav1.Duration from a Go duration string ("5m", "300s", "1h30m") or seconds."""
    if d is None:
        return 0.0
    if isinstance(d, (int, float)):
        return float(d)
    total = 0.0
    for num, unit in re.findall(r"([0-9.]+)(ns|us|ms|s|m|h)", d):
        total += float(num) * {"ns": 1e-9, "us": 1e-6, "ms": 1e-3, "s": 1, "m": 60, "h": 3600}[unit]
    return total


def estimate_node_allocatable(node) -> Dict[str, Fraction]:
    """DefaultEstimator.EstimateNode (default_estimator.go:122-141)."""
    alloc = _rl((node.get("status") or {}).get("allocatable"))
    ann = ((node.get("metadata") or {}).get("annotations") or {}).get(ANN_RAW_ALLOCATABLE)
    if ann:
        try:
            raw = _rl(json.loads(ann))
        except Exception:
            raw = {}
        for k, v in raw.items():
            alloc[k] = v
    return alloc


@dataclass
class AssignedPod:
    pod: dict
    timestamp: float  # podAssignInfo.timestamp, seconds relative to now


ANN_CUSTOM_EST_SECONDS_AFTER_SCHEDULED = "scheduling.koordinator.sh/load-estimated-seconds-after-pod-scheduled"
ANN_CUSTOM_EST_SECONDS_AFTER_INITIALIZED = "scheduling.koordinator.sh/load-estimated-seconds-after-initialized"
ANN_RESERVE_POD = "scheduling.koordinator.sh/reserve-pod"
DEFAULT_NODE_METRIC_REPORT_INTERVAL = 60.0  # loadaware DefaultNodeMetricReportInterval


def pod_condition(pod, ctype: str) -> Optional[dict]:
    """podutil.GetPodCondition: the condition of that type, or None. lastTransitionTime is seconds (None = zero)."""
    for c in (pod.get("status") or {}).get("conditions") or []:
        if c.get("type") == ctype:
            return c
    return None


def is_reserve_pod(pod) -> bool:
    """reservationutil.IsReservePod (pkg/util/reservation/reservation.go:197-199)."""
    return ((pod.get("metadata") or {}).get("annotations") or {}).get(ANN_RESERVE_POD) == "true"


def _custom_seconds(pod, key: str) -> int:
    """extension.GetCustomEstimatedSecondsAfter* (apis/extension/load_aware.go:84-100): -1 when absent."""
    s = ((pod.get("metadata") or {}).get("annotations") or {}).get(key, "")
    if s:
        try:
            return int(s, 10)
        except ValueError:
            pass
    return -1


def estimated_deadline(pod, timestamp: float, la: LoadAwareArgs) -> Optional[float]:
    """podAssignCache.shouldEstimatePodDeadline (pod_assign_cache.go:329-354); None is the zero time."""
    after_sched = after_init = -1
    if la.allow_customize_estimation:
        after_sched = _custom_seconds(pod, ANN_CUSTOM_EST_SECONDS_AFTER_SCHEDULED)
        after_init = _custom_seconds(pod, ANN_CUSTOM_EST_SECONDS_AFTER_INITIALIZED)
    if la.estimated_seconds_after_pod_scheduled is not None and after_sched < 0:
        after_sched = la.estimated_seconds_after_pod_scheduled
    if la.estimated_seconds_after_initialized is not None and after_init < 0:
        after_init = la.estimated_seconds_after_initialized
    if after_init > 0:
        c = pod_condition(pod, "PodInitialized")
        if c is not None and c.get("status") == "True" and c.get("lastTransitionTime") is not None:
            return float(c["lastTransitionTime"]) + after_init
    if after_sched > 0 and timestamp is not None:
        return timestamp + after_sched
    return None


@dataclass
class PodAssignInfo:
    """podAssignInfo (pod_assign_cache.go:127-132)."""
    pod: dict
    timestamp: float
    estimated: Optional[List[int]]   # None: the estimator returned nothing (assign(): empty vector)
    deadline: Optional[float] = None  # estimatedDeadline, None = zero time


def assign_info(pod, la: LoadAwareArgs, now: float = 0.0, timestamp: Optional[float] = None) -> PodAssignInfo:
    """The podAssignInfo podAssignCache.assign builds (pod_assign_cache.go:291-315): the PodScheduled
    condition's transition time when True, else the cache clock (or an explicit `timestamp`)."""
    e = estimate_pod(pod, la)
    est = None if all(x == 0 for x in e) else e
    if timestamp is None:
        c = pod_condition(pod, "PodScheduled")
        if c is not None and c.get("status") == "True" and c.get("lastTransitionTime") is not None:
            timestamp = float(c["lastTransitionTime"])
        else:
            timestamp = now
    return PodAssignInfo(pod, timestamp, est, estimated_deadline(pod, timestamp, la))


def _vadd(v, x):
    for i, a in enumerate(x):
        v[i] += a


def _vsub(v, x):
    for i, a in enumerate(x):
        v[i] -= a


def _add_delta(v, x, y) -> bool:
    """ResourceVector.AddDelta (loadaware/helper.go:231-242): v += max(0, x - y) per entry (in place)."""
    changed = False
    for i, val in enumerate(x):
        if y is not None:
            val -= y[i]
        if val > 0:
            v[i] += val
            changed = True
    return changed


def _sub_delta(v, x, y) -> bool:
    """ResourceVector.SubDelta (loadaware/helper.go:251-262)."""
    changed = False
    for i, val in enumerate(x):
        if y is not None:
            val -= y[i]
        if val > 0:
            v[i] -= val
            changed = True
    return changed


class LoadAwareNodeCache:
    """nodeInfo of loadaware/pod_assign_cache.go:101-125 for one node, maintained incrementally:
    AddOrUpdateNodeMetric (:520-603), DeleteNodeMetric (:605-616), AddOrUpdatePod (:418-447) and
    DeletePod (:449-466) with addPod / deletePod (:618-707). Times are seconds on the cache clock;
    None is Go's zero time.

    LoadAwareNodeCache(metric, assigned, la) builds the node at a frozen time from a NodeMetric and the
    pods assigned to it, which is what the incremental path reaches by any order of the same events."""

    def __init__(self, metric: Optional[dict] = None, assigned: Iterable[AssignedPod] = (),
                 la: Optional[LoadAwareArgs] = None):
        self.la = la
        self.pod_infos: Dict[str, PodAssignInfo] = {}
        self.update_time: Optional[float] = None  # kept across metric updates that carry none (:586-588)
        self._clear_metric_state()
        self.metric = None
        if metric is not None:
            self.set_metric(metric)
        for i, ap in enumerate(assigned):
            uid = (ap.pod.get("metadata") or {}).get("uid") or f"#{i}"
            self.add_or_update_pod(uid, assign_info(ap.pod, la, timestamp=ap.timestamp))

    def _clear_metric_state(self):
        zero = [0] * abi.KG_LA_R
        self.report_interval = DEFAULT_NODE_METRIC_REPORT_INTERVAL
        self.node_usage: Optional[List[int]] = None
        self.prod_usage = list(zero)
        self.agg_usages: Dict[Tuple[str, float], List[int]] = {}
        self.pod_usages: Dict[Tuple[str, str], List[int]] = {}
        self.prod_pods = set()
        self.node_delta, self.prod_delta, self.node_estimated = list(zero), list(zero), list(zero)
        self.node_delta_pods, self.prod_delta_pods, self.node_estimated_pods = set(), set(), set()

    @staticmethod
    def _vec(resources) -> List[int]:
        res = resources or {}
        return [vec_value(r, res[r]) if r in res else 0 for r in LA_RESOURCES]

    def empty(self) -> bool:
        return self.metric is None and not self.pod_infos

    # -- NodeMetric events -------------------------------------------------------------------------
    def set_metric(self, metric: dict):
        """nodeInfo.AddOrUpdateNodeMetric (pod_assign_cache.go:520-603): every derived vector is rebuilt
        and every cached pod re-added."""
        self._clear_metric_state()
        st = metric.get("status") or {}
        spec = metric.get("spec") or {}
        info = st.get("nodeMetric")
        if info is not None:
            self.node_usage = self._vec((info.get("nodeUsage") or {}).get("resources"))
            max_d: Dict[str, float] = {}
            for agg in info.get("aggregatedNodeUsages") or []:
                d = _duration(agg.get("duration"))
                for t, u in (agg.get("usage") or {}).items():
                    res = (u or {}).get("resources") or {}
                    if len(res) == 0:
                        continue
                    self.agg_usages[(t, d)] = self._vec(res)
                    if d > max_d.get(t, 0.0):
                        max_d[t] = d
            for t, d in max_d.items():
                self.agg_usages[(t, 0.0)] = self.agg_usages[(t, d)]
            if self.la.prod_usage_include_sys:
                _vadd(self.prod_usage, self._vec((info.get("systemUsage") or {}).get("resources")))
        for pm in st.get("podsMetric") or []:
            if pm is None:
                continue
            res = (pm.get("podUsage") or {}).get("resources") or {}
            if len(res) == 0:
                continue
            key = (pm.get("namespace", ""), pm.get("name", ""))
            self.pod_usages[key] = self._vec(res)
            if pm.get("priority") == PROD:
                self.prod_pods.add(key)
        self.metric = metric
        ri = (spec.get("collectPolicy") or {}).get("reportIntervalSeconds")
        if ri is not None:
            self.report_interval = float(ri)
        ut = st.get("updateTime")
        if ut is not None:
            self.update_time = float(ut)
        for info_ in self.pod_infos.values():
            self._add_pod(info_)

    def clear_metric(self):
        """nodeInfo.DeleteNodeMetric (pod_assign_cache.go:605-616): only the metric pointer is dropped."""
        self.metric = None

    # -- pod events ------------------------------------------------------------------------------
    def add_or_update_pod(self, uid: str, info: PodAssignInfo):
        """nodeInfo.AddOrUpdatePod (pod_assign_cache.go:418-447)."""
        old = self.pod_infos.get(uid)
        self.pod_infos[uid] = info
        if self.metric is not None:
            if old is not None:
                self._delete_pod(old)
            self._add_pod(info)

    def delete_pod(self, uid: str):
        """nodeInfo.DeletePod (pod_assign_cache.go:449-466)."""
        old = self.pod_infos.pop(uid, None)
        if self.metric is not None and old is not None:
            self._delete_pod(old)

    def _should(self, info: PodAssignInfo, u) -> bool:
        # u == nil || updateTime - reportInterval < timestamp || (deadline set && deadline > updateTime)
        if u is None:
            return True
        if self.update_time is None or self.update_time - self.report_interval < info.timestamp:
            return True
        return info.deadline is not None and info.deadline > self.update_time

    def _add_pod(self, info: PodAssignInfo):
        """nodeInfo.addPod (pod_assign_cache.go:618-662)."""
        key = _pod_key(info.pod)
        u = self.pod_usages.get(key)
        prod = priority_class(info.pod) == PROD
        active_prod = prod and key in self.prod_pods
        if active_prod:
            _vadd(self.prod_usage, u)
        e = info.estimated
        if e is None:
            return
        should = self._should(info, u)
        if should and _add_delta(self.node_delta, e, u):
            self.node_delta_pods.add(key)
        _vadd(self.node_estimated, e)
        self.node_estimated_pods.add(key)
        if not prod:
            return
        if not active_prod and u is not None:
            u, should = None, True
        if should and _add_delta(self.prod_delta, e, u):
            self.prod_delta_pods.add(key)

    def _delete_pod(self, info: PodAssignInfo):
        """nodeInfo.deletePod (pod_assign_cache.go:669-707), the reverse of addPod."""
        key = _pod_key(info.pod)
        u = self.pod_usages.get(key)
        prod = priority_class(info.pod) == PROD
        active_prod = prod and key in self.prod_pods
        if active_prod:
            _vsub(self.prod_usage, u)
        e = info.estimated
        if e is None:
            return
        should = self._should(info, u)
        if should and _sub_delta(self.node_delta, e, u):
            self.node_delta_pods.discard(key)
        _vsub(self.node_estimated, e)
        self.node_estimated_pods.discard(key)
        if not prod:
            return
        if not active_prod and u is not None:
            u, should = None, True
        if should and _sub_delta(self.prod_delta, e, u):
            self.prod_delta_pods.discard(key)

    def estimated_of_existing(self, prod_pod: bool, agg_type: str = "", agg_duration: float = 0.0):
        """GetNodeMetricAndEstimatedOfExisting (pod_assign_cache.go:163-201); None = NotFound."""
        if self.metric is None:
            return None
        if prod_pod:
            return [a + b for a, b in zip(self.prod_usage, self.prod_delta)]
        if agg_type:
            usage = self.agg_usages.get((agg_type, agg_duration))
            if usage is None and agg_duration == 0:
                usage = self.node_usage
        else:
            usage = self.node_usage
        if usage is not None:
            return [a + b for a, b in zip(usage, self.node_delta)]
        return list(self.node_estimated)


@dataclass
class NodeInput:
    """Everything the snapshot needs about one node."""

    node: dict
    pods: List[dict] = field(default_factory=list)           # pods bound/assumed on the node (NodeInfo)
    node_metric: Optional[dict] = None                      # slo NodeMetric
    assigned: Optional[List[AssignedPod]] = None            # podAssignCache entries (default: pods)
    numa_zones: Optional[List[Dict[str, str]]] = None       # NodeResourceTopology zone resources
    numa_used: Optional[List[Dict[str, str]]] = None        # resourceManager allocated per zone
    kubelet_numa_policy: str = ""                           # NRT topology policy
    cpuset_allocated_milli: int = 0


NODEINFO_KEYS = ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem")


def pod_request_vec(pod, cfg: SchedulerConfig) -> List[int]:
    """What framework.NodeInfo.AddPod adds for one pod: Requested (cpu, memory, ephemeral-storage, the
    snapshot's scalar slots) and NonZeroRequested (cpu, memory), in NODEINFO_KEYS + sc_req order."""
    r = pod_requests(pod)
    nz = pod_requests(pod, NON_MISSING)
    v = [milli_value(r.get(CPU, 0)), value(r.get(MEMORY, 0)), value(r.get(EPHEMERAL, 0)),
         milli_value(nz.get(CPU, 0)), value(nz.get(MEMORY, 0))]
    v += [value(r.get(name, 0)) for name in cfg.scalar_resources]
    v += [0] * (abi.KG_NSCALAR - len(cfg.scalar_resources))
    return v


def nodeinfo_cols(requested: Sequence[int], num_pods: int) -> Dict[str, object]:
    """Requested / NonZeroRequested / pod count columns from the sum of pod_request_vec over the node's pods."""
    row: Dict[str, object] = {k: int(requested[i]) for i, k in enumerate(NODEINFO_KEYS)}
    for k in range(abi.KG_NSCALAR):
        row[f"sc_req{k}"] = int(requested[len(NODEINFO_KEYS) + k])
    row["num_pods"] = num_pods
    return row


def node_static_cols(node: dict, cfg: SchedulerConfig, zones: Optional[List[Dict[str, str]]] = None,
                     kubelet_numa_policy: str = "", la=None) -> Dict[str, object]:
    """Columns that follow the Node object (allocatable, LoadAware thresholds, NUMA policy and amplification)
    and the NodeResourceTopology zones. la: cfg.la() when the caller holds it (defaulting deep-copies the args)."""
    if la is None:
        la = cfg.la()
    alloc = _rl((node.get("status") or {}).get("allocatable"))
    row: Dict[str, object] = {
        "alloc_cpu": milli_value(alloc.get(CPU, 0)),
        "alloc_mem": value(alloc.get(MEMORY, 0)),
        "alloc_eph": value(alloc.get(EPHEMERAL, 0)),
        "alloc_pods": value(alloc.get(PODS, 0)),
    }
    for k in range(abi.KG_NSCALAR):
        row[f"sc_alloc{k}"] = value(alloc.get(cfg.scalar_resources[k], 0)) if k < len(cfg.scalar_resources) else 0
    est_alloc = estimate_node_allocatable(node)
    for r, name in enumerate(LA_RESOURCES):
        row[f"la_alloc{r}"] = vec_value(name, est_alloc[name]) if name in est_alloc else 0
    prof = filter_profile(node, la)
    for r in range(abi.KG_LA_R):
        row[f"la_thr_usage{r}"] = prof.usage[r]
        row[f"la_thr_prod{r}"] = prof.prod[r]
        row[f"la_thr_agg{r}"] = prof.agg[0][r] if prof.agg else 0
    md = node.get("metadata") or {}
    labels = md.get("labels") or {}
    policy_name = labels.get(LABEL_NUMA_POLICY, "") or kubelet_numa_policy
    if policy_name not in NUMA_POLICIES:
        raise Unsupported(f"NUMA topology policy {policy_name!r}")
    row["numa_policy"] = NUMA_POLICIES[policy_name]
    ratio = 1.0
    ann = (md.get("annotations") or {}).get(ANN_AMPLIFICATION)
    if ann:
        ratio = float(json.loads(ann).get(CPU, 1.0))
    row["cpu_amp_ratio"] = ratio
    zones = zones or []
    if len(zones) > abi.KG_MAX_ZONES:
        raise Unsupported(f"{len(zones)} NUMA zones > {abi.KG_MAX_ZONES}")
    row["numa_zones"] = len(zones)
    for z in range(abi.KG_MAX_ZONES):
        if z < len(zones):
            zr = _rl(zones[z])
            # amplifyNUMANodeResources (nodenumaresource/util.go:101-124)
            row[f"zone_cpu{z}"] = amplify(milli_value(zr.get(CPU, 0)), ratio)
            row[f"zone_mem{z}"] = value(zr.get(MEMORY, 0))
        else:
            row[f"zone_cpu{z}"] = row[f"zone_mem{z}"] = 0
    return row


def la_cols(node: dict, metric: Optional[dict], cache: LoadAwareNodeCache, la: LoadAwareArgs,
            now: float = 0.0) -> Dict[str, object]:
    """LoadAware flags and the Filter / Score bases GetNodeMetricAndEstimatedOfExisting returns for the node
    (load_aware.go:150-376 reads them per pod; they depend only on the node and the pod's prod-ness)."""
    prof = filter_profile(node, la)
    flags = 0
    if any(x != 0 for x in prof.prod):
        flags |= abi.KG_LA_PROD_THR
    if prof.agg is not None:
        flags |= abi.KG_LA_AGG_THR
    zero = [0] * abi.KG_LA_R
    fb_np = fb_prod = sb_np = sb_prod = zero
    if metric is not None:
        flags |= abi.KG_LA_HAS_METRIC
        st = metric.get("status") or {}
        if st.get("nodeMetric") is None:
            flags |= abi.KG_LA_NM_NIL
        secs = la.node_metric_expiration_seconds
        if secs is not None:
            ut = st.get("updateTime")
            if ut is None or (secs > 0 and (now - float(ut)) >= secs):
                flags |= abi.KG_LA_EXPIRED
        if prof.agg is not None:
            fb_np = cache.estimated_of_existing(False, prof.agg[1], prof.agg[2])
        else:
            fb_np = cache.estimated_of_existing(False)
        fb_prod = cache.estimated_of_existing(True)
        a = la.aggregated
        if a is not None and a.score_aggregation_type != "":
            sb_np = cache.estimated_of_existing(False, a.score_aggregation_type, a.score_aggregated_duration)
        else:
            sb_np = cache.estimated_of_existing(False)
        sb_prod = cache.estimated_of_existing(True)
    row: Dict[str, object] = {"la_flags": flags}
    for r in range(abi.KG_LA_R):
        row[f"la_fbase_np{r}"] = fb_np[r]
        row[f"la_fbase_prod{r}"] = fb_prod[r]
        row[f"la_sbase_np{r}"] = sb_np[r]
        row[f"la_sbase_prod{r}"] = sb_prod[r]
    return row


def zone_used_cols(used: Optional[List[Dict[str, str]]], cpuset_allocated_milli: int = 0) -> Dict[str, object]:
    """resourceManager allocations per NUMA zone (node_allocation.go:221-243) and the node's cpuset total."""
    used = used or []
    row: Dict[str, object] = {"cpuset_alloc_milli": int(cpuset_allocated_milli)}
    for z in range(abi.KG_MAX_ZONES):
        ur = _rl(used[z]) if z < len(used) else {}
        row[f"zone_cpu_used{z}"] = milli_value(ur.get(CPU, 0))
        row[f"zone_mem_used{z}"] = value(ur.get(MEMORY, 0))
    return row


def node_row(ni: NodeInput, cfg: SchedulerConfig, now: float = 0.0) -> Dict[str, object]:
    """Snapshot row of one node built from scratch (the incremental path is cluster.ClusterState)."""
    la = cfg.la()
    row = node_static_cols(ni.node, cfg, ni.numa_zones, ni.kubelet_numa_policy, la)
    req = [0] * (len(NODEINFO_KEYS) + abi.KG_NSCALAR)
    for p in ni.pods:  # NodeInfo.AddPod for every pod on the node
        for i, x in enumerate(pod_request_vec(p, cfg)):
            req[i] += x
    row.update(nodeinfo_cols(req, len(ni.pods)))
    assigned = ni.assigned
    if assigned is None:
        assigned = [AssignedPod(p, 0.0) for p in ni.pods]
    assigned = [a for a in assigned if not _is_terminated(a.pod) and not is_reserve_pod(a.pod)]  # assign(): :292
    row.update(la_cols(ni.node, ni.node_metric, LoadAwareNodeCache(ni.node_metric, assigned, la), la, now))
    row.update(zone_used_cols(ni.numa_used, ni.cpuset_allocated_milli))
    return row


def nodes_table(nodes: Sequence[NodeInput], cfg: SchedulerConfig) -> abi.Table:
    t = abi.empty_nodes(len(nodes))
    for i, ni in enumerate(nodes):
        for k, v in node_row(ni, cfg).items():
            t[k][i] = v
    return t


# ------------------------------------------------------------------------------------------------
# DeviceShare / Reservation / ElasticQuota host decode (config 5)

def gpu_requirements(requests: Dict[str, int]) -> Tuple[List[int], int, int, bool]:
    """calcDesiredRequestsAndCountForGPU (deviceshare/devicehandler_gpu.go:53-96) on the koordinator
    GPU resources of a pod (after the nvidia.com/gpu conversion): per-instance request vector
    [gpu-core, gpu-memory-ratio, gpu-memory], the key mask of requestsPerGPU, numberOfGPUs and whether
    the request is shared. Go integer division (all values non-negative)."""
    from .config import GPU_CORE, GPU_MEMORY, GPU_MEMORY_RATIO
    gpu_shared = requests.get("koordinator.sh/gpu.shared")
    desired = 1
    ratio = requests.get(GPU_MEMORY_RATIO)
    if gpu_shared is not None and gpu_shared > 0:
        desired = gpu_shared
    elif ratio is not None and ratio > 100 and ratio % 100 == 0:
        desired = ratio // 100
    req = [0, 0, 0]
    keys = 0
    shared = False
    if GPU_CORE in requests:
        req[abi.KG_DEV_CORE] = requests[GPU_CORE] // desired
        keys |= 1 << abi.KG_DEV_CORE
    if ratio is not None:
        per = ratio // desired
        shared = per < 100
        req[abi.KG_DEV_RATIO] = per
        keys |= 1 << abi.KG_DEV_RATIO
    elif GPU_MEMORY in requests:
        shared = True
        req[abi.KG_DEV_MEM] = requests[GPU_MEMORY] // desired
        keys |= 1 << abi.KG_DEV_MEM
    return req, keys, desired, shared


RSV_DIMS = ("cpu", "memory", "ephemeral-storage", "scalar0", "scalar1")  # KG_RSV_R order


# ---- DeviceShare reservation restore (GPU minors) ----------------------------------------------------
# A device table here is int64 [KG_DEV_R][KG_DEV_MINORS] (gpu-core, gpu-memory-ratio, gpu-memory per minor)
# with a presence mask over minors (a deviceResources map holds a minor or not).

def _dz():
    return np.zeros((abi.KG_DEV_R, abi.KG_DEV_MINORS), np.int64)


def _dtab(v):
    return _dz() if v is None else np.asarray(v, np.int64).reshape(abi.KG_DEV_R, abi.KG_DEV_MINORS).copy()


def _dmask(a) -> np.ndarray:
    return np.any(a != 0, axis=0)


def dev_effective(total, used, free, pre, pre_mask, req=None, req_mask=None):
    """The (total, free) an allocation sees (nodeDevice.calcFreeWithPreemptible, device_cache.go:322-364, and
    nodeDevice.filter, :366-410): a minor holding preemptible resources frees them from its used (never below
    zero), and if any such minor then has something left, the other minors keep their free; allocating
    from a reservation's required resources keeps only those minors, each capped by them
    (util.MinResourceList). Minors outside the result have total and free 0."""
    total, used, free = _dtab(total), _dtab(used), _dtab(free)
    F = free.copy()
    merged = {}
    for m in range(abi.KG_DEV_MINORS):
        if pre_mask[m]:
            u = np.maximum(used[:, m] - pre[:, m], 0)
            rem = np.maximum(total[:, m] - u, 0)
            if np.any(rem != 0):
                merged[m] = rem
    for m, rem in merged.items():
        F[:, m] = rem
    T = total.copy()
    if req_mask is not None:
        for m in range(abi.KG_DEV_MINORS):
            if req_mask[m]:
                F[:, m] = np.minimum(F[:, m], req[:, m])
            else:
                F[:, m] = 0
                T[:, m] = 0
    return T, F


def dev_reusable(total, used, free, unmatched_used, matched_allocated, matched_allocatable, matched):
    """Effective device tables of one node for one pod's restore state (deviceshare/reservation.go):
      matched[i] = (policy, allocatable, remained) of the i-th matched reservation holding GPUs, each a
      (table, mask) pair; unmatched_used / matched_allocated / matched_allocatable are the merged tables
      (mergeReservationAllocations, :94-117).
    Returns (per_matched, base): per_matched[i] = (total, free) that tryAllocateFromReusable (:344-410)
    allocates from for reservation i (preemptible = unmatched used + matched allocated + its remained; the
    Restricted policy only its minors, capped by calcRequiredDeviceResources :436-455), and base = (total,
    free) of the allocation outside the reservations (plugin.go:417-419: unmatched used + matched
    allocatable)."""
    uu, uum = unmatched_used
    ma, mam = matched_allocated
    mal, malm = matched_allocatable
    out = []
    for policy, (alloc, alloc_mask), (rem, rem_mask) in matched:
        pre = uu + ma + rem
        pm = uum | mam | rem_mask
        if policy == abi.KG_RSV_RESTRICTED:
            req_mask = rem_mask.copy() if rem_mask.any() else alloc_mask.copy()
            req = np.where(rem_mask[None, :], rem, 0)
            out.append(dev_effective(total, used, free, pre, pm, req, req_mask & alloc_mask))
        else:
            out.append(dev_effective(total, used, free, pre, pm))
    base = dev_effective(total, used, free, uu + mal, uum | malm)
    return out, base


def dev_reservation_parts(r: dict):
    """(allocatable, allocated, remained, used-when-unmatched) of one reservation's GPUs (RestoreReservation's
    filterFn, reservation.go:163-186): `dev_alloc` is the reserve pod's allocation (nodeDevice.getUsed),
    `dev_allocated` its assigned pods' allocations on those minors (appendAllocatedByHints). Each part is
    a (table, mask) pair; None when the reservation holds no GPU."""
    alloc = _dtab(r.get("dev_alloc"))
    amask = _dmask(alloc)
    if not amask.any():
        return None
    allocated = np.where(amask[None, :], _dtab(r.get("dev_allocated")), 0)
    almask = _dmask(allocated)
    rem = alloc - allocated  # subtractAllocated(.., false): negative kept, zero minors dropped
    rmask = _dmask(rem)
    used = np.where(_dmask(np.maximum(allocated, 0))[None, :], np.maximum(allocated, 0), 0)
    return (alloc, amask), (allocated, almask), (rem, rmask), (used, _dmask(used))



def reservation_restore(nodes: abi.Table, reservations: Sequence[dict]):
    """Host restatement of the Reservation transformer (reservation/transformer.go:147-350,740-935).

    `nodes` is the true NodeInfo view (reserve pods and the pods allocated to reservations both
    counted, as NodeInfo accounts them). Each reservation is a dict: node, cls (owner-match class, or the
    list of classes that match it as rsvmatch.match_classes returns them),
    allocatable / allocated / reserved (KG_RSV_R vectors, allocated None while Allocated is nil; allocated_keys:
    bit 0 / 1 when Allocated holds a cpu / memory key, default both),
    allocated_pods, policy, order, allocate_once, max_pods.

    Returns (nodes_default, views, infos, devs): the snapshot columns as seen by pods matching nothing on
    the node (every reservation with assigned pods corrected by updateNodeInfoRequestedForUnmatched),
    and per (class, node) the restored view with its matched reservations (kg_rsv_view / kg_rsv_info
    dicts for abi.Reservations). Reserve pods request their Allocatable; the non-zero request of a
    present cpu / memory key is the value itself (GetNonZeroRequestForResource,
    frameworkext/reservation_info.go:581-605).

    DeviceShare (nodes with dev_minors >= 0): a reservation may carry `dev_alloc` (its reserve pod's GPU
    allocation, [KG_DEV_R][KG_DEV_MINORS]) and `dev_allocated` (its pods' allocations on those minors);
    `nodes["dev_used"]` (optional, default total - free) is the node's used per minor. The default
    columns' dev_free then give back what pods use inside unmatched reservations, and `devs` holds the
    (total, free) tables views (dev_base) and matched reservations (dev) allocate from (dev_reusable)."""
    out = {k: np.array(v, copy=True) for k, v in nodes.items()}
    # a reservation whose reserve pod holds a NUMA / cpuset allocation (`numa_held`): NodeNUMAResource's own restore
    # (nodenumaresource/reservation.go:188-262) is not restated; the node is marked for the engine (rsv_numa)
    held = sorted({int(r["node"]) for r in reservations if r.get("numa_held")})
    if held or "rsv_numa" in out:
        n_rows = len(next(iter(nodes.values())))
        rn = np.array(out["rsv_numa"], np.uint8, copy=True) if "rsv_numa" in out else np.zeros(n_rows, np.uint8)
        rn[held] = 1
        out["rsv_numa"] = rn
    req_cols = ["req_cpu", "req_mem", "req_eph", "sc_req0", "sc_req1"]
    by_node: Dict[int, List[int]] = {}
    for x, r in enumerate(reservations):
        by_node.setdefault(int(r["node"]), []).append(x)

    def vec(r, key):
        v = r.get(key)
        return [0] * abi.KG_RSV_R if v is None else [int(a) for a in v]

    def nz(v, r):
        # GetNonZeroRequestForResource per key of Allocated: the value of a present key, else the default
        keys = r.get("allocated_keys", 3) if r.get("allocated") is not None else 0
        cpu = v[0] if keys & 1 else 100                  # DefaultMilliCPURequest
        mem = v[1] if keys & 2 else 200 * 1024 * 1024    # DefaultMemoryRequest
        return cpu, mem

    for i, xs in by_node.items():
        for x in xs:  # default view: every reservation with assigned pods is unmatched
            r = reservations[x]
            if int(r.get("allocated_pods", 0)) > 0:
                a = vec(r, "allocated")
                for k, c in enumerate(req_cols):
                    out[c][i] -= a[k]
                ncpu, nmem = nz(a, r)
                out["nz_cpu"][i] -= ncpu
                out["nz_mem"][i] -= nmem
    views, infos, devs = [], [], []
    dev_on = "dev_minors" in nodes and "dev_total" in nodes
    parts = [dev_reservation_parts(r) for r in reservations]

    def node_dev(i):
        tot = np.asarray(nodes["dev_total"][i], np.int64)
        fr = np.asarray(nodes["dev_free"][i], np.int64)
        used = np.asarray(nodes["dev_used"][i], np.int64) if "dev_used" in nodes else tot - fr
        return tot, used, fr

    def merged(xs, part):
        t, m = _dz(), np.zeros(abi.KG_DEV_MINORS, bool)
        for x in xs:
            if parts[x] is not None:
                t += parts[x][part][0]
                m |= parts[x][part][1]
        return t, m

    for i, xs in by_node.items():  # default view: unmatched = the reservations with assigned pods
        if dev_on and int(nodes["dev_minors"][i]) >= 0:
            gx = [x for x in xs if parts[x] is not None and int(reservations[x].get("allocated_pods", 0)) > 0]
            if gx:
                tot, used, fr = node_dev(i)
                uu = merged(gx, 3)
                out["dev_free"][i] = dev_effective(tot, used, fr, uu[0], uu[1])[1]
    def classes_of(r):  # one owner-match class, or the list of classes that match it (rsvmatch.match_classes)
        c = r["cls"]
        return {int(c)} if np.isscalar(c) else {int(v) for v in c}

    for i in sorted(by_node):
        classes = sorted({c for x in by_node[i] for c in classes_of(reservations[x])})
        for c in classes:
            matched = [x for x in by_node[i] if c in classes_of(reservations[x])]
            req = [int(out[col][i]) for col in req_cols]
            nzc, nzm = int(out["nz_cpu"][i]), int(out["nz_mem"][i])
            pod_requested = list(req)
            r_alloc = [0] * abi.KG_RSV_R
            for x in matched:
                r = reservations[x]
                a = vec(r, "allocated")
                if int(r.get("allocated_pods", 0)) > 0:  # its unmatched correction is undone
                    for k in range(abi.KG_RSV_R):
                        req[k] += a[k]
                        pod_requested[k] += a[k]
                    ncpu, nmem = nz(a, r)
                    nzc += ncpu
                    nzm += nmem
                rp = vec(r, "allocatable")  # restoreMatchedReservation: RemovePod(reserve pod)
                for k in range(abi.KG_RSV_R):
                    req[k] -= rp[k]
                    r_alloc[k] += a[k]
                ncpu, nmem = nz(rp, {"allocated": rp})
                nzc -= ncpu
                nzm -= nmem
            dev_base, dev_idx = -1, {}
            if dev_on and int(nodes["dev_minors"][i]) >= 0 and any(parts[x] is not None for x in by_node[i]):
                # RestoreReservation (deviceshare/reservation.go:149-200): matched = the class's reservations
                # holding GPUs, unmatched = the node's others that hold GPUs and have assigned pods
                tot, used, fr = node_dev(i)
                gm = [x for x in matched if parts[x] is not None]
                gu = [x for x in by_node[i] if x not in matched and parts[x] is not None
                      and int(reservations[x].get("allocated_pods", 0)) > 0]
                per, base = dev_reusable(tot, used, fr, merged(gu, 3), merged(gm, 1), merged(gm, 0),
                                         [(int(reservations[x].get("policy", abi.KG_RSV_DEFAULT)), parts[x][0],
                                           parts[x][2]) for x in gm])
                dev_base = len(devs)
                devs.append(base)
                for x, tf in zip(gm, per):
                    dev_idx[x] = len(devs)
                    devs.append(tf)
            first = len(infos)
            for x in matched:
                r = reservations[x]
                alloc = vec(r, "allocatable")
                names = 0
                for k in range(abi.KG_RSV_R):
                    if alloc[k] != 0 or (r.get("names") is not None and (int(r["names"]) >> k) & 1):
                        names |= 1 << k
                infos.append(dict(policy=int(r.get("policy", abi.KG_RSV_DEFAULT)), names=names,
                                  allocate_once=int(bool(r.get("allocate_once", True))), order=int(r.get("order", 0)),
                                  allocatable=alloc, allocated=vec(r, "allocated"), reserved=vec(r, "reserved"),
                                  max_pods=int(r.get("max_pods", -1)), allocated_pods=int(r.get("allocated_pods", 0)),
                                  dev=dev_idx.get(x, -1), rid=x,
                                  allocated_keys=(int(r.get("allocated_keys", 3)) if r.get("allocated") is not None
                                                  else 0),
                                  # the reserved minors a pod allocating from the reservation takes first
                                  # (tryAllocateFromReusable's preferred set, deviceshare/reservation.go:308)
                                  dev_minors=(int(sum(1 << int(m) for m in np.nonzero(parts[x][0][1])[0]))
                                              if dev_on and parts[x] is not None and x in dev_idx else 0)))
            views.append(dict(node=i, cls=c, first=first, count=len(matched), req=req, nz_cpu=nzc, nz_mem=nzm,
                              num_pods=int(out["num_pods"][i]) - len(matched), pod_requested=pod_requested,
                              r_allocated=r_alloc, dev_base=dev_base))
    return out, views, infos, devs


def reservation_gpu_raw(nodes: abi.Table, reservations: Sequence[dict]) -> List[dict]:
    """The DeviceShare restore inputs of the GPU-holding reservations (kg_rsv_gpu entries for abi.Reservations(gpu=)):
    per node holding one, its raw used (nodeDevice.deviceUsed: `dev_used`, else total - free) as the rid -1 entry, and
    per such reservation (rid = its index, as reservation_restore numbers them) its reserve pod's allocation, its
    assigned pods' allocations on those minors, policy and assigned pod count (RestoreReservation's inputs,
    deviceshare/reservation.go:149-186). A device Reserve into such a node follows them (kg_snapshot_upload_rsv_gpu)."""
    if "dev_minors" not in nodes or "dev_total" not in nodes:
        return []
    out, seen = [], set()
    for x, r in enumerate(reservations):
        parts = dev_reservation_parts(r)
        i = int(r["node"])
        if parts is None or int(nodes["dev_minors"][i]) < 0:
            continue
        if i not in seen:
            seen.add(i)
            tot = np.asarray(nodes["dev_total"][i], np.int64)
            used = np.asarray(nodes["dev_used"][i], np.int64) if "dev_used" in nodes else tot - np.asarray(nodes["dev_free"][i], np.int64)
            out.append(dict(node=i, rid=-1, a=used))
        out.append(dict(node=i, rid=x, policy=int(r.get("policy", abi.KG_RSV_DEFAULT)),
                        allocated_pods=int(r.get("allocated_pods", 0)), a=parts[0][0], b=parts[1][0]))
    return out


def quota_keys(pods: abi.Table, max_keys: np.ndarray) -> np.ndarray:
    """Keys of quotav1.Mask(PodRequests, Max names) over KG_QUOTA_R = {cpu, memory, scalar0, scalar1}
    (elasticquota/plugin.go:279-280): a key is present when the pod requests it."""
    f = pods["flags"]
    have = (np.where(f & abi.KG_POD_HAS_CPU, 1, 0) | np.where(f & abi.KG_POD_HAS_MEM, 2, 0)
            | np.where(pods["sc_req0"] != 0, 4, 0) | np.where(pods["sc_req1"] != 0, 8, 0))
    q = pods["quota"]
    mk = np.where(q >= 0, max_keys[np.maximum(q, 0)], 0)
    return (have & mk).astype(np.uint32)


# ---- DeviceShare GPU topology tree and partition tables (deviceshare/allocator_gpu.go, allocator_gpu_helper.go)

ANN_GPU_PARTITIONS = "scheduling.koordinator.sh/gpu-partitions"          # Device: GPUPartitionTable JSON
ANN_GPU_PARTITION_SPEC = "scheduling.koordinator.sh/gpu-partition-spec"  # Pod: GPUPartitionSpec JSON
ANN_DEVICE_ALLOCATE_HINT = "scheduling.koordinator.sh/device-allocate-hint"
LABEL_GPU_PARTITION_POLICY = "node.koordinator.sh/gpu-partition-policy"
LABEL_GPU_VENDOR = "node.koordinator.sh/gpu-vendor"
LABEL_GPU_MODEL = "node.koordinator.sh/gpu-model"


def _hopper_table() -> Dict[int, List[dict]]:
    """GPUPartitionIndexOfNVIDIAHopper (allocator_gpu_helper.go:28-147): NVLink pairs / quads / all eight, every
    partition and group of AllocationScore 1."""
    return {1: [{"minors": [m], "allocationScore": 1} for m in range(8)],
            2: [{"minors": [2 * k, 2 * k + 1], "allocationScore": 1} for k in range(4)],
            4: [{"minors": [0, 1, 2, 3], "allocationScore": 1}, {"minors": [4, 5, 6, 7], "allocationScore": 1}],
            8: [{"minors": list(range(8)), "allocationScore": 1}]}


def gpu_partition_table(device: Optional[dict], node: dict) -> Tuple[Optional[Dict[int, List[dict]]], bool]:
    """(GPUPartitionTable, honor) of a node: the Device annotation's table with the Device's GPUPartitionPolicy
    label (device_cache.go:536-545, apiext.GetGPUPartitionTable / GetGPUPartitionPolicy), else the designated
    table of the node's GPU model with the Node's label (GetDesignatedGPUPartitionIndexer,
    allocator_gpu_helper.go:149-162; an empty vendor counts as nvidia)."""
    meta = (device or {}).get("metadata", {})
    raw = (meta.get("annotations") or {}).get(ANN_GPU_PARTITIONS)
    if raw:
        table = {int(k): v for k, v in json.loads(raw).items()}
        honor = (meta.get("labels") or {}).get(LABEL_GPU_PARTITION_POLICY) == "Honor"
        return table, honor
    labels = node.get("metadata", {}).get("labels") or {}
    honor = labels.get(LABEL_GPU_PARTITION_POLICY) == "Honor"
    if labels.get(LABEL_GPU_VENDOR, "") in ("", "nvidia") and labels.get(LABEL_GPU_MODEL) in ("H100", "H800", "H20"):
        return _hopper_table(), honor
    return None, honor


def gpu_partition_entries(table: Dict[int, List[dict]], index: int) -> List[tuple]:
    """kg_gpu_partition rows of one table in GetGPUPartitionIndexer order (allocator_gpu_helper.go:165-199):
    per GPU count, AllocationScore groups ascending, each group in the table's order. RingBusBandwidth in
    bytes (-1 = none)."""
    rows = []
    for n in sorted(table):
        parts = table[n]
        for score in sorted({int(p.get("allocationScore", 0)) for p in parts}):
            for p in parts:
                if int(p.get("allocationScore", 0)) != score:
                    continue
                mask = 0
                for m in p["minors"]:
                    mask |= 1 << int(m)
                bw = p.get("ringBusBandwidth")
                rows.append((index, int(n), mask, 0, score, -1 if bw is None else value(bw)))
    return rows


class GpuPartitionTables:
    """Distinct partition tables of a snapshot (kg_node_columns.gpu_parts) and the dev_part of each node."""

    def __init__(self):
        self._index: Dict[str, int] = {}
        self._rows: List[tuple] = []

    def add(self, table: Optional[Dict[int, List[dict]]]) -> int:
        """1 + the table's index (0 for None)."""
        if table is None:
            return 0
        key = json.dumps({str(k): v for k, v in sorted(table.items())}, sort_keys=True)
        if key not in self._index:
            if len(self._index) >= abi.KG_GPU_MAX_TABLES:
                raise Unsupported(f"more than {abi.KG_GPU_MAX_TABLES} distinct GPU partition tables")
            self._index[key] = len(self._index)
            self._rows += gpu_partition_entries(table, self._index[key])
        return 1 + self._index[key]

    def array(self) -> np.ndarray:
        return np.array(self._rows, dtype=abi.GPU_PARTITION_DTYPE)


def gpu_topology(gpu_infos: Sequence[dict]) -> Tuple[int, bool]:
    """dev_topo of a node from its GPU DeviceInfos (minor, topology {nodeID, pcieID}) and whether the node has a
    topology tree: GetGPUTopologyScope (allocator_gpu_helper.go:201-262) returns nil without infos or when one
    lacks a Topology. Byte m = (rank of the NUMA node id) << 4 | rank of (NUMA node id, PCIe id), PCIe ids in
    string order within a NUMA node (the scopes' sort order)."""
    if not gpu_infos or any(d.get("topology") is None for d in gpu_infos):
        return (1 << 64) - 1, False
    numa_ids = sorted({int(d["topology"].get("nodeID", 0)) for d in gpu_infos})
    pairs = sorted({(int(d["topology"].get("nodeID", 0)), str(d["topology"].get("pcieID", ""))) for d in gpu_infos})
    # the device decodes each rank with 3 bits into DEV_MINORS-entry tables (kg_ext.h gpu_scope)
    if len(numa_ids) > abi.KG_DEV_MINORS or len(pairs) > abi.KG_DEV_MINORS:
        raise Unsupported(f"GPU topology with more than {abi.KG_DEV_MINORS} NUMA nodes or PCIe switches")
    topo = (1 << 64) - 1
    for d in gpu_infos:
        m = int(d.get("minor", 0))
        if m >= abi.KG_DEV_MINORS:
            raise Unsupported(f"GPU minor {m} >= {abi.KG_DEV_MINORS}")
        t = d["topology"]
        q = numa_ids.index(int(t.get("nodeID", 0)))
        r = pairs.index((int(t.get("nodeID", 0)), str(t.get("pcieID", ""))))
        topo &= ~(0xFF << (8 * m))
        topo |= ((q << 4) | r) << (8 * m)
    return topo, True


def gpu_numa(gpu_infos: Sequence[dict]) -> int:
    """dev_numa of a node from its GPU DeviceInfos: nibble m = the NUMA node id of GPU minor m
    (NUMATopology.deviceToNodeID, deviceshare/numa_topology.go:43-100), KG_GPU_NUMA_ANY for Topology.NodeID -1,
    KG_GPU_NUMA_NONE without a Topology (or no such minor). Ids are NUMA zone ids below KG_MAX_ZONES."""
    v = (1 << 32) - 1
    ids = set()
    for d in gpu_infos or ():
        m = int(d.get("minor", 0))
        if m >= abi.KG_DEV_MINORS:
            raise Unsupported(f"GPU minor {m} >= {abi.KG_DEV_MINORS}")
        t = d.get("topology")
        if t is None:
            q = abi.KG_GPU_NUMA_NONE
        else:
            q = int(t.get("nodeID", 0))
            if q == -1:
                q = abi.KG_GPU_NUMA_ANY
            elif not 0 <= q < abi.KG_MAX_ZONES:
                raise Unsupported(f"GPU NUMA node id {q} outside the device's {abi.KG_MAX_ZONES} zones")
            else:
                ids.add(q)
        v &= ~(0xF << (4 * m))
        v |= q << (4 * m)
    if len(ids) > abi.KG_MAX_ZONES:
        raise Unsupported(f"GPUs on more than {abi.KG_MAX_ZONES} NUMA nodes")
    return v


def gpu_pod_flags(pod: dict, shared: bool) -> Tuple[int, int]:
    """(dev_flags, dev_ring_bw) of a GPU pod: parseGPURequirements (deviceshare/utils.go:516-545) beyond the
    request: GPUPartitionSpec (apiext.GetGPUPartitionSpec: present -> honor, AllocatePolicy Restricted,
    RingBusBandwidth) and the gpu DeviceHint's RequiredTopologyScope."""
    ann = pod.get("metadata", {}).get("annotations") or {}
    flags = abi.KG_GPU_POD_SHARED if shared else 0
    bw = 0
    raw = ann.get(ANN_GPU_PARTITION_SPEC)
    if raw is not None:
        spec = json.loads(raw)
        flags |= abi.KG_GPU_POD_HONOR
        if spec.get("allocatePolicy", "BestEffort") == "Restricted":
            flags |= abi.KG_GPU_POD_RESTRICTED
        if spec.get("ringBusBandwidth") is not None:
            flags |= abi.KG_GPU_POD_RING_BW
            bw = value(spec["ringBusBandwidth"])
    raw = ann.get(ANN_DEVICE_ALLOCATE_HINT)
    if raw is not None:
        hint = (json.loads(raw) or {}).get("gpu") or {}
        scope = hint.get("requiredTopologyScope", "")
        if scope:
            level = abi.GPU_SCOPE_LEVEL.get(scope, 5)
            flags |= level << abi.KG_GPU_POD_SCOPE_SHIFT
    return flags, bw


# ---- GPU shared-resource templates (deviceshare/gpu_shared_resource_templates_cache.go) ----------------------

class NoMatchedTemplate(Exception):
    """parseGPURequirements' PreFilter error ErrNoMatchedGPUSharedResourceTemplate (deviceshare/utils.go:544-546):
    a pod enforcing a template matched none of any key; the pod fails PreFilter, no node is evaluated."""


def gpu_template_key(node: dict) -> str:
    """buildGPUSharedResourceTemplatesKey(vendor, model) of a node's labels (allocator_gpu.go:140,
    gpu_shared_resource_templates_cache.go:80-82)."""
    labels = node.get("metadata", {}).get("labels") or {}
    return f"{labels.get(LABEL_GPU_VENDOR, '')}-{labels.get(LABEL_GPU_MODEL, '')}"


class GpuSharedResourceTemplates:
    """gpuSharedResourceTemplatesCache (gpu_shared_resource_templates_cache.go:30-78) with the plugin's
    GPUSharedResourceTemplatesConfig.MatchedResources, and its device encoding: the configured keys in sorted
    order are the template keys of dev_part bits 12-15 (at most KG_GPU_TMPL_NONE of them), a pod's
    candidateGPUSharedResourceTemplates become 2 bits per key in kg_pod_columns.dev_tmpl."""

    def __init__(self, infos: Optional[Dict[str, Dict[str, Dict[str, object]]]] = None,
                 matched_resources: Sequence[str] = ()):
        self.infos = {key: {name: {r: parse_quantity(q) for r, q in (tmpl or {}).items()}
                            for name, tmpl in (templates or {}).items()}
                      for key, templates in (infos or {}).items()}
        self.matched_resources = set(matched_resources)
        self.keys = sorted(self.infos)
        if len(self.keys) > abi.KG_GPU_TMPL_NONE:
            raise Unsupported(f"more than {abi.KG_GPU_TMPL_NONE} GPU shared-resource template keys")

    @classmethod
    def from_configmap(cls, cm: dict, matched_resources: Sequence[str] = ()) -> "GpuSharedResourceTemplates":
        """setTemplatesInfosFromConfigMap (:71-78): the YAML map under data.yaml; a malformed one raises
        ValueError (the cache keeps its previous infos in the reference's event handler)."""
        import yaml
        try:
            infos = yaml.safe_load((cm.get("data") or {}).get("data.yaml", ""))
        except yaml.YAMLError as e:
            raise ValueError(f"invalid GPU shared-resource templates: {e}") from e
        if infos is not None and not isinstance(infos, dict):
            raise ValueError("invalid GPU shared-resource templates: not a map")
        return cls(infos, matched_resources)

    def find_matched(self, resources: Dict[str, object], strict: bool) -> Dict[str, Dict[str, Dict[str, Fraction]]]:
        """findMatchedTemplates (:41-62): per key, the templates equal to `resources` (quotav1.Equals: the same
        names with equal quantities); not strict, each template is first masked to the resource names."""
        want = {r: parse_quantity(q) for r, q in resources.items()}
        out = {}
        for key, templates in self.infos.items():
            matched = {}
            for name, tmpl in templates.items():
                t = tmpl if strict else {r: q for r, q in tmpl.items() if r in want}
                if t == want:
                    matched[name] = dict(tmpl)
            if matched:
                out[key] = matched
        return out

    def node_key(self, node: dict) -> int:
        """The node's template key index for dev_part bits 12-15 (KG_GPU_TMPL_NONE: no templates for its key)."""
        key = gpu_template_key(node)
        return self.keys.index(key) if key in self.infos else abi.KG_GPU_TMPL_NONE

    def requests_per_gpu(self, req: Sequence[int], keys: int) -> Dict[str, int]:
        from .config import DEV_RESOURCES
        return {DEV_RESOURCES[r]: int(req[r]) for r in range(abi.KG_DEV_R) if (keys >> r) & 1}

    def pod_template(self, rpg: Dict[str, object], shared: bool) -> Tuple[int, int, Dict[str, Dict]]:
        """(KG_GPU_POD_TEMPLATE or 0, dev_tmpl, candidate templates) of a GPU pod from its requestsPerGPU (resource
        name -> quantity; requests_per_gpu() of gpu_requirements' vector): a shared request naming one of the
        matched resources enforces a template (utils.go:540-547) and takes the strictly matched templates as
        candidates; none at all raises NoMatchedTemplate."""
        if not shared or not (set(rpg) & self.matched_resources):
            return 0, 0, {}
        cands = self.find_matched(rpg, True)
        if not cands:
            raise NoMatchedTemplate("no matched GPU shared resource template")
        tmpl = 0
        for key, matched in cands.items():
            tmpl |= min(len(matched), 2) << (2 * self.keys.index(key))
        return abi.KG_GPU_POD_TEMPLATE, tmpl, cands

    @staticmethod
    def allocation_template(cands: Dict[str, Dict], node: dict) -> Optional[str]:
        """appendTemplateInfoToAllocations' name (allocator_gpu.go:144-153): the node key's only candidate, else
        None (several candidates fall through to the plain allocator without a name)."""
        matched = cands.get(gpu_template_key(node)) or {}
        return next(iter(matched)) if len(matched) == 1 else None
