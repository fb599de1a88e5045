"""KG_ST_* status bits -> the reference plugins' Filter failure reasons (the FitError diagnosis).

The device reports one status word per (pod, node) pair (kg_eval_verify) or, for a replayed pod, the OR
of those words over every node in its cycle (kg_replay out_reason). This module turns the bits back into
the reason strings the Go plugins put into their fwktype.Status, so the caller can build the
unschedulable pod's FitError exactly as the framework would:

  NodeResourcesFit   upstream noderesources.Fits reasons ("Too many pods", "Insufficient <resource>")
  LoadAwareScheduling  pkg/scheduler/plugins/loadaware/load_aware.go:48-51
  NodeNUMAResource   pkg/scheduler/plugins/nodenumaresource/plugin.go:54-63,
                     nodenumaresource/topology_hint.go:37, frameworkext/topologymanager/manager.go:32-33
  DeviceShare        deviceshare/device_allocator.go:434, devicehandler_gpu.go:43 ("Insufficient gpu devices")
  Reservation        reservation/plugin.go:60,68,495
  ElasticQuota       elasticquota/plugin.go:281 ("Insufficient quotas, ...")

Bits that stand for a formatted message carry its fixed prefix; the variable part (which resource, the
quota's numbers) is not encoded in a bit and is left as a placeholder in angle brackets.
"""
from __future__ import annotations

from . import abi

DEFAULT_SCALARS = ("kubernetes.io/batch-cpu", "kubernetes.io/batch-memory")


def plugin_reasons(bits: int, scalar_names=DEFAULT_SCALARS) -> dict:
    """{plugin name: [reason, ...]} of one status word (or an OR of several)."""
    bits = int(bits)
    out: dict = {}

    def add(plugin, msg):
        out.setdefault(plugin, []).append(msg)

    nrf = (
        (abi.KG_ST_NRF_PODS, "Too many pods"),
        (abi.KG_ST_NRF_CPU, "Insufficient cpu"),
        (abi.KG_ST_NRF_MEM, "Insufficient memory"),
        (abi.KG_ST_NRF_EPH, "Insufficient ephemeral-storage"),
        (abi.KG_ST_NRF_SC0, f"Insufficient {scalar_names[0]}"),
        (abi.KG_ST_NRF_SC1, f"Insufficient {scalar_names[1]}"),
    )
    for bit, msg in nrf:
        if bits & bit:
            add("NodeResourcesFit", msg)
    if bits & abi.KG_ST_LA_EXPIRED:
        add("LoadAwareScheduling", "node(s) nodeMetric expired")
    for bit, res in ((abi.KG_ST_LA_CPU, "cpu"), (abi.KG_ST_LA_MEM, "memory")):
        if bits & bit:
            if bits & abi.KG_ST_LA_AGG:
                add("LoadAwareScheduling", f"node(s) {res} aggregated usage exceed threshold")
            else:
                add("LoadAwareScheduling", f"node(s) {res} usage exceed threshold")
    numa = (
        (abi.KG_ST_NUMA_AMP_CPU, "Insufficient amplified cpu"),
        (abi.KG_ST_NUMA_CONFLICT, "node(s) NUMA Topology policy not match"),
        (abi.KG_ST_NUMA_NO_RES, "node(s) missing NUMA resources"),
        (abi.KG_ST_NUMA_ALIGN, "Unaligned NUMA Hint cause <hints>"),
        (abi.KG_ST_NUMA_UNSATISFIED, "Unsatisfied NUMA <resource>"),
        (abi.KG_ST_NUMA_CPU_TOPO, "node(s) invalid CPU Topology"),
        (abi.KG_ST_NUMA_CPU_BIND, "node(s) cpu bind policy conflicts / SMT alignment / invalid requested cpus"),
        (abi.KG_ST_NUMA_CPUS, "not enough cpus available to satisfy request"),
        # Reserve of a BestEffort node (plugin.go:612-623, resource_manager.go:135,300-309)
        (abi.KG_ST_NUMA_INSUF_CPU, "Insufficient NUMA cpu"),
        (abi.KG_ST_NUMA_INSUF_MEM, "Insufficient NUMA memory"),
        (abi.KG_ST_NUMA_INSUF_NODE, "node(s) Insufficient NUMA Node resources"),
    )
    for bit, msg in numa:
        if bits & bit:
            add("NodeNUMAResource", msg)
    code = abi.dev_code(bits)
    if code:  # GPU allocator reasons (deviceshare/allocator_gpu.go:31-41, device_allocator.go:432)
        add("DeviceShare", DEV_CODE_REASONS.get(code, "Insufficient gpu devices"))
    if bits & abi.KG_ST_DEV_RSV:  # makeReasonsByReservation (deviceshare/plugin.go)
        add("DeviceShare", "Reservation(s) Insufficient gpu devices")
    if bits & abi.KG_ST_RSV_AFFINITY:
        add("Reservation", "node(s) no reservations match reservation affinity")
    if bits & abi.KG_ST_RSV_NODE:
        add("Reservation", "Insufficient <resource> by node")
    if bits & abi.KG_ST_RSV_RESERVATION:
        add("Reservation", "node(s) no reservation(s) to meet the requirements")
    if bits & abi.KG_ST_QUOTA:
        add("ElasticQuota", "Insufficient quotas, <quota state>")
    if bits & abi.KG_ST_UNSUPPORTED:
        add("(host path)", "pair evaluated by the reference plugin on the host")
    return out


DEV_CODE_REASONS = {
    abi.KG_DEV_CODE_INSUFFICIENT: "Insufficient gpu devices",
    abi.KG_DEV_CODE_NO_DEVICE: "Insufficient gpu devices",
    abi.KG_DEV_CODE_GPU_DEVICES: "Insufficient GPU Devices",
    abi.KG_DEV_CODE_TOPO_SCOPED: "Insufficient Topology Scoped GPU Devices",
    abi.KG_DEV_CODE_PARTITIONED: "Insufficient Partitioned GPU Devices",
    abi.KG_DEV_CODE_NO_PARTITION: "node(s) missing GPU Partition Table",
    abi.KG_DEV_CODE_PART_COUNT: "node(s) Unsupported number of GPU requests",
    abi.KG_DEV_CODE_NO_TREE: "node(s) missing GPU Device Topology Tree",
    abi.KG_DEV_CODE_MULTI_SHARED: "node(s) Unsupported Multi-Shared GPU",
    abi.KG_DEV_CODE_NUMA_SCOPED: "Insufficient NUMA Scoped Devices",
    abi.KG_DEV_CODE_NO_TEMPLATE: "no matched GPU shared resource template",
}


def reasons(bits: int, scalar_names=DEFAULT_SCALARS) -> list:
    """Flat list of the reasons in plugin filter order."""
    return [m for msgs in plugin_reasons(bits, scalar_names).values() for m in msgs]


def loadaware_status(bits: int):
    """LoadAware bits of one pair -> (code, reason) of the Go Status (load_aware.go:150-220)."""
    msgs = plugin_reasons(int(bits) & abi.KG_ST_LA_MASK).get("LoadAwareScheduling")
    return ("Unschedulable", msgs[0]) if msgs else ("Success", None)
