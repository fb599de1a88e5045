"""Whole-job placement on the device: the FindOneNodePlugin slot driving the replay kernel.

Reference behaviour mirrored here (names, argument meaning, status codes and messages):

  FindOneNodePlugin.FindOneNode, BatchScheduleResult   frameworkext/interface.go:115-145
  how the framework consumes a plan                    frameworkext/framework_extender.go:356-407
  a planner over the whole gang                        coscheduling/core/network_topology_workflow.go:70-160
  BatchScheduler.BatchSchedule                         batch/batch_scheduler.go:74-185
  Engine.RunSchedulingCycle, ValidateAndGroupByRequest batch/engine.go:92-294,348-371
  JobResult.ExampleMessage                             batch/framework/types.go:275-341

`ReplayPlanner.find_one_node` places every pending member of the job with the sequential replay kernel
(one pod per cycle, Reserve applied on the device between pods) on the live snapshot and rolls the snapshot
back afterwards (kg_snapshot_checkpoint / kg_snapshot_rollback), so a plan costs no copy of the cluster.
`BatchScheduler.batch_schedule` then runs the inline batch cycle of the plan on the device
(kg_batch_schedule): per planned node, in pod-name order, PreFilter + Filter on that node and Reserve; on any
failure every assumed pod is undone (CleanupAssumedPods) and the job status carries the reference's
example message. Go is not in this image, so this Python layer stands where the Go plugin would; the
numbers all come from the HIP kernels behind include/koordgpu.h (no CPU fallback).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi, engine, reasons

# fwktype.Code values the path returns
SUCCESS = "Success"
ERROR = "Error"
UNSCHEDULABLE = "Unschedulable"
UNSCHEDULABLE_AND_UNRESOLVABLE = "UnschedulableAndUnresolvable"
SKIP = "Skip"

# batch/engine.go:55-68, batch_scheduler.go:96-101, network_topology_workflow.go:37-38
ERR_PRE_FILTER_FAILED = "pre-filter failed for pod {ns}/{name}/{uid}, {msg}"
ERR_FILTER_POD_FAILED = "filter pod {ns}/{name}/{uid} on node {node} failed, err: {msg}"
ERR_RESERVE_POD_FAILED = "reserve pod {ns}/{name}/{uid} on node {node} failed, err: {msg}"
ERR_PLAN_MISSING_NODE = "batch schedule plan missing node for pod {key}"
ERR_NO_PENDING_PODS = "no pending pods"
JOB_SCHEDULE_FAILED = "job batch schedule failed"
# network_topology.go:35 AnnotationGangPodNetworkTopologyIndex
ANNOTATION_TOPOLOGY_INDEX = "gang.scheduling.koordinator.sh/network-topology-index"

# Filter plugin order of the shipped profile: the first failing plugin's reasons make the Status message
_FILTER_ORDER = ("NodeResourcesFit", "LoadAwareScheduling", "NodeNUMAResource", "DeviceShare", "Reservation",
                 "(host path)")


@dataclass
class Status:
    code: str = SUCCESS
    message: str = ""

    def is_success(self) -> bool:
        return self.code == SUCCESS


@dataclass
class JobPod:
    """A member pod as the planner sees it: its key parts and its row of the pod columns (abi.Table)."""
    namespace: str
    name: str
    uid: str = ""
    annotations: Dict[str, str] = field(default_factory=dict)

    @property
    def key(self) -> str:  # batch/framework/types.go:343-345 GetPodKey
        return f"{self.namespace}/{self.name}"


@dataclass
class BatchScheduleResult:
    """frameworkext.BatchScheduleResult: every member pod and its planned node."""
    pods: List[JobPod]
    pod_to_node_name: Dict[str, str]


def topology_index(p: JobPod) -> int:
    """apis/extension/network_topology.go:72-85 GetPodNetworkTopologyIndex (-1 when absent or malformed)."""
    s = p.annotations.get(ANNOTATION_TOPOLOGY_INDEX)
    if s is None:
        return -1
    try:
        return int(s)
    except ValueError:
        return -1


def sort_pods_by_index(idx: Sequence[int], pods: Sequence[JobPod]) -> List[int]:
    """apis/extension/network_topology.go:89-103 SortPodsByIndex: indexed pods first, by index, then by name."""
    def key(i):
        t = topology_index(pods[i])
        return (0, t, pods[i].name) if t >= 0 else (1, 0, pods[i].name)
    return sorted(idx, key=key)


def filter_message(bits: int, scalar_names=reasons.DEFAULT_SCALARS) -> str:
    """The Status message of the first failing Filter plugin (the framework stops at the first failure)."""
    by = reasons.plugin_reasons(bits, scalar_names)
    for plugin in _FILTER_ORDER:
        if plugin in by:
            return ", ".join(by[plugin])
    return ""


class ReplayPlanner:
    """FindOneNodePlugin backed by kg_replay: the whole job is placed on the device in one call."""

    name = "KoordGPUReplayPlanner"

    def __init__(self, snap: engine.Snapshot, node_names: Sequence[str]):
        self.snap = snap
        self.node_names = list(node_names)

    def find_one_node(self, members: Sequence[JobPod], table: abi.Table
                      ) -> Tuple[Optional[BatchScheduleResult], Status, Optional[np.ndarray]]:
        """Plan for all pending members (rows of `table` in `members` order). Returns (plan, status, reason
        bits per member in plan order); Skip when there is no job, Unschedulable when some member finds no
        node (the whole gang must fit: the status names the first such pod and its plugin reasons)."""
        if len(members) == 0:
            return None, Status(SKIP), None
        order = sort_pods_by_index(range(len(members)), members)
        sub = abi.take(table, np.asarray(order, np.int64))
        pods = engine.PodBatch(self.snap.ctx, sub)
        try:
            self.snap.checkpoint()
            try:
                node, _total, why = engine.replay(self.snap, pods, reasons=True)
            finally:
                self.snap.rollback()
        finally:
            pods.close()
        ordered = [members[i] for i in order]
        for t, p in enumerate(ordered):
            if node[t] < 0:
                msg = filter_message(int(why[t])) or "no feasible node"
                return None, Status(UNSCHEDULABLE, f"pod {p.key}: {msg}"), why
        plan = BatchScheduleResult(ordered, {p.key: self.node_names[node[t] - self.snap.index_base]
                                             for t, p in enumerate(ordered)})
        return plan, Status(SUCCESS), why


@dataclass
class JobOutcome:
    status: Status
    pod_status: Dict[str, Status]
    assumed: Dict[str, Tuple[str, int, int]]  # key -> (node, NUMA zone, GPU minors) of the committed pods


class BatchScheduler:
    """batch.BatchScheduler over kg_batch_schedule (the scheduling cycle runs on the device)."""

    def __init__(self, snap: engine.Snapshot, node_names: Sequence[str]):
        self.snap = snap
        self.node_index = {n: i for i, n in enumerate(node_names)}

    def batch_schedule(self, plan: BatchScheduleResult, table_by_key: Dict[str, Tuple[abi.Table, int]]) -> JobOutcome:
        """table_by_key[key] = (pod table, row). Success commits every member's Reserve on the snapshot."""
        for p in plan.pods:
            if not plan.pod_to_node_name.get(p.key):
                return JobOutcome(Status(ERROR, ERR_PLAN_MISSING_NODE.format(key=p.key)), {}, {})
        # buildJobRequest + ValidateAndGroupByRequest: per node, pods by name; nodes in first-appearance order
        groups: Dict[str, List[JobPod]] = {}
        for p in plan.pods:
            groups.setdefault(plan.pod_to_node_name[p.key], []).append(p)
        if not groups:
            return JobOutcome(Status(ERROR, "no pods to schedule"), {}, {})
        batch: List[Tuple[str, JobPod]] = []
        for node_name, ps in groups.items():
            for p in sorted(ps, key=lambda q: q.name):
                batch.append((node_name, p))
        rows = [abi.take(table_by_key[p.key][0], np.asarray([table_by_key[p.key][1]], np.int64)) for _, p in batch]
        sub = abi.concat(rows)
        plan_node = np.asarray([self.node_index[n] - self.snap.index_base for n, _ in batch], np.int32)
        pods = engine.PodBatch(self.snap.ctx, sub)
        try:
            res, stat, zone, minors = engine.batch_schedule(self.snap, pods, plan_node)
        finally:
            pods.close()
        pod_status: Dict[str, Status] = {}
        assumed: Dict[str, Tuple[str, int, int]] = {}
        n_assumed, failed = 0, []
        node_msg: Dict[str, Tuple[int, str]] = {}  # the failing pod's status, set on it and every later pod of its node
        for t, (node_name, p) in enumerate(batch):
            r = int(res[t])
            if r in (abi.KG_BATCH_ASSUMED, abi.KG_BATCH_ROLLED_BACK):
                n_assumed += 1
                pod_status[p.key] = Status(SUCCESS)
                if r == abi.KG_BATCH_ASSUMED:
                    assumed[p.key] = (node_name, int(zone[t]), int(minors[t]))
            elif r in (abi.KG_BATCH_FAILED, abi.KG_BATCH_SIBLING):
                bits = int(stat[t])
                code = UNSCHEDULABLE
                if r == abi.KG_BATCH_SIBLING and node_name in node_msg:
                    # engine.go:188-219: errMsg is formatted once, from the pod that failed, and set on
                    # every pod k >= j of the node group
                    code, msg = node_msg[node_name]
                elif bits & abi.KG_ST_NUMA_RESERVE:
                    code = ERROR  # fwktype.Error (engine.go:278-280)  # Filter passed, the NodeNUMAResource Reserve failed (engine.go:275-283)
                    msg = ERR_RESERVE_POD_FAILED.format(ns=p.namespace, name=p.name, uid=p.uid, node=node_name,
                                                       msg=", ".join(reasons.plugin_reasons(bits & abi.KG_ST_NUMA_RESERVE)
                                                                     ["NodeNUMAResource"]))
                elif bits & abi.KG_ST_QUOTA:  # the ElasticQuota gate runs in PreFilter
                    msg = ERR_PRE_FILTER_FAILED.format(ns=p.namespace, name=p.name, uid=p.uid,
                                                      msg=reasons.plugin_reasons(bits)["ElasticQuota"][0])
                else:
                    msg = ERR_FILTER_POD_FAILED.format(ns=p.namespace, name=p.name, uid=p.uid, node=node_name,
                                                      msg=filter_message(bits))
                if r == abi.KG_BATCH_FAILED:
                    node_msg[node_name] = (code, msg)
                pod_status[p.key] = Status(code, msg)
                failed.append((p.key, node_name))
        if not failed:
            return JobOutcome(Status(SUCCESS), pod_status, assumed)
        # JobResult.ExampleMessage, taken before the cleanup rewrites the assumed pods' statuses
        first_key, first_node = min(failed)
        msg = (f"job failed due to {JOB_SCHEDULE_FAILED}, assumed {n_assumed} pods, failed {len(failed)} pods, "
               f"first failed pod {first_key}@{first_node} failed due to {pod_status[first_key].message}")
        on_node = sorted(p.key for n, p in batch if n == first_node and
                         int(res[[q.key for _, q in batch].index(p.key)]) == abi.KG_BATCH_ROLLED_BACK)
        if on_node:
            msg += f", assumed pods on node {first_node}: " + ", ".join(on_node)
        for key in pod_status:
            if pod_status[key].is_success():
                pod_status[key] = Status(UNSCHEDULABLE, JOB_SCHEDULE_FAILED)
        return JobOutcome(Status(UNSCHEDULABLE, msg), pod_status, {})
