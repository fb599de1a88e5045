"""Plugin arguments of the Filter/Score path, defaulted like the reference.

Mirrors pkg/scheduler/apis/config/types.go:31-101 (LoadAwareSchedulingArgs) and the v1 defaulting
in pkg/scheduler/apis/config/v1/defaults.go:32-48,100-163; NodeResourcesFit args follow the shipped
profile config/manager/scheduler-config.yaml:17-31 (upstream LeastAllocated cpu=1, memory=1 when
unset).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from . import abi

CPU = "cpu"
MEMORY = "memory"
EPHEMERAL = "ephemeral-storage"
PODS = "pods"
BATCH_CPU = "kubernetes.io/batch-cpu"
BATCH_MEMORY = "kubernetes.io/batch-memory"
MID_CPU = "kubernetes.io/mid-cpu"
MID_MEMORY = "kubernetes.io/mid-memory"
GPU_CORE = "koordinator.sh/gpu-core"
GPU_MEMORY_RATIO = "koordinator.sh/gpu-memory-ratio"
GPU_MEMORY = "koordinator.sh/gpu-memory"
DEV_RESOURCES = (GPU_CORE, GPU_MEMORY_RATIO, GPU_MEMORY)  # KG_DEV_CORE, KG_DEV_RATIO, KG_DEV_MEM

# LoadAware vectorizer (loadaware/helper.go:162-173): cpu and memory, sorted by name.
LA_RESOURCES = (CPU, MEMORY)

DEFAULT_NODE_METRIC_EXPIRATION_SECONDS = 180
DEFAULT_RESOURCE_WEIGHTS = {CPU: 1, MEMORY: 1}
DEFAULT_USAGE_THRESHOLDS = {CPU: 65, MEMORY: 95}
DEFAULT_ESTIMATED_SCALING_FACTORS = {CPU: 85, MEMORY: 70}


@dataclass
class AggregatedArgs:
    usage_thresholds: Dict[str, int] = field(default_factory=dict)
    usage_aggregation_type: str = ""
    usage_aggregated_duration: float = 0.0  # seconds
    score_aggregation_type: str = ""
    score_aggregated_duration: float = 0.0


@dataclass
class LoadAwareArgs:
    filter_expired_node_metrics: Optional[bool] = None
    node_metric_expiration_seconds: Optional[int] = None
    enable_schedule_when_node_metrics_expired: Optional[bool] = None
    resource_weights: Dict[str, int] = field(default_factory=dict)
    dominant_resource_weight: int = 0
    usage_thresholds: Dict[str, int] = field(default_factory=dict)
    prod_usage_thresholds: Dict[str, int] = field(default_factory=dict)
    prod_usage_include_sys: bool = False
    score_according_prod_usage: bool = False
    estimated_scaling_factors: Optional[Dict[str, int]] = None
    estimated_seconds_after_pod_scheduled: Optional[int] = None
    estimated_seconds_after_initialized: Optional[int] = None
    allow_customize_estimation: bool = False
    aggregated: Optional[AggregatedArgs] = None

    def defaulted(self) -> "LoadAwareArgs":
        """SetDefaults_LoadAwareSchedulingArgs (v1/defaults.go:100-125)."""
        a = copy.deepcopy(self)
        if a.filter_expired_node_metrics is None:
            a.filter_expired_node_metrics = True
        if a.enable_schedule_when_node_metrics_expired is None:
            a.enable_schedule_when_node_metrics_expired = False
        if a.node_metric_expiration_seconds is None:
            a.node_metric_expiration_seconds = DEFAULT_NODE_METRIC_EXPIRATION_SECONDS
        if len(a.resource_weights) == 0 and a.dominant_resource_weight == 0:
            a.resource_weights = dict(DEFAULT_RESOURCE_WEIGHTS)
        if len(a.usage_thresholds) == 0:
            a.usage_thresholds = dict(DEFAULT_USAGE_THRESHOLDS)
        if a.estimated_scaling_factors is None:
            a.estimated_scaling_factors = dict(DEFAULT_ESTIMATED_SCALING_FACTORS)
        else:
            for k, v in DEFAULT_ESTIMATED_SCALING_FACTORS.items():
                a.estimated_scaling_factors.setdefault(k, v)
        return a


@dataclass
class SchedulerConfig:
    """One koord-scheduler profile restricted to the device path's plugins."""

    plugins: int = abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_LA | abi.KG_PLUGIN_NUMA
    weight_nrf: int = 1
    weight_la: int = 1
    weight_numa: int = 1
    # NodeResourcesFit LeastAllocated strategy (shipped profile: cpu, memory, batch-cpu, batch-memory).
    nrf_resources: List[Tuple[str, int]] = field(
        default_factory=lambda: [(CPU, 1), (MEMORY, 1), (BATCH_CPU, 1), (BATCH_MEMORY, 1)])
    # Scalar resources carried in the snapshot's two scalar slots.
    scalar_resources: Tuple[str, str] = (BATCH_CPU, BATCH_MEMORY)
    loadaware: LoadAwareArgs = field(default_factory=LoadAwareArgs)
    # NodeNUMAResource ScoringStrategy / NUMAScoringStrategy (v1/defaults.go:128-162).
    numa_scoring: List[Tuple[str, int]] = field(default_factory=lambda: [(CPU, 1), (MEMORY, 1)])
    numa_hint_scoring: List[Tuple[str, int]] = field(default_factory=lambda: [(CPU, 1), (MEMORY, 1)])
    # DeviceShare (score weight 1) and Reservation (score weight 5000) of the shipped profile
    # (config/manager/scheduler-config.yaml:91-96); DeviceShare LeastAllocated resources
    # (v1/defaults.go:254-277: gpu-memory-ratio 1, gpu-memory 1; rdma / fpga are not GPU minors).
    weight_dev: int = 1
    weight_rsv: int = 5000
    dev_scoring: List[Tuple[str, int]] = field(
        default_factory=lambda: [(GPU_MEMORY_RATIO, 1), (GPU_MEMORY, 1)])
    # ScoringStrategy types ("LeastAllocated" default / "MostAllocated")
    numa_strategy: str = "LeastAllocated"
    numa_hint_strategy: str = "LeastAllocated"
    dev_strategy: str = "LeastAllocated"
    # NodeResourcesFit per-resource MostAllocated (upstream MostAllocated strategy = every resource;
    # NodeResourcesFitPlus allows a mix)
    nrf_most: Tuple[str, ...] = ()
    # IgnoredResources / IgnoredResourceGroups of NodeResourcesFit and of the Reservation plugin (extended
    # resources only; a group is the name's prefix before "/")
    nrf_ignored: Tuple[str, ...] = ()
    nrf_ignored_groups: Tuple[str, ...] = ()
    rsv_ignored: Tuple[str, ...] = ()
    rsv_ignored_groups: Tuple[str, ...] = ()
    # NodeNUMAResourceArgs.DefaultCPUBindPolicy (v1/defaults.go:50, plugin.go:327-334): fills in a pod's
    # "" / "Default" bind policy
    default_cpu_bind_policy: str = "FullPCPUs"

    def _ignore_mask(self, names, groups) -> int:
        m = 0
        for k, name in enumerate(self.scalar_resources):
            if name in names or (name.split("/", 1)[0] in groups and "/" in name):
                m |= 1 << k
        return m

    def la(self) -> LoadAwareArgs:
        return self.loadaware.defaulted()

    def kg_config(self) -> abi.KgConfig:
        la = self.la()
        c = abi.KgConfig()
        c.plugins = self.plugins
        c.weight_nrf = self.weight_nrf
        c.weight_la = self.weight_la
        c.weight_numa = self.weight_numa
        w = dict(self.nrf_resources)
        for name in w:
            if name not in (CPU, MEMORY) and name not in self.scalar_resources:
                raise ValueError(f"NodeResourcesFit scoring resource {name!r} is not a snapshot column")
        c.nrf_w_cpu = w.get(CPU, 0)
        c.nrf_w_mem = w.get(MEMORY, 0)
        for k, name in enumerate(self.scalar_resources):
            c.nrf_w_sc[k] = w.get(name, 0)
        # scoreWeights = vectorizer.ToFactorVec(ResourceWeights); nil if DominantResourceWeight == 0
        # and all weights zero (load_aware.go:112-116)
        la_w = [la.resource_weights.get(r, 0) for r in LA_RESOURCES]
        c.la_score_enabled = int(not (la.dominant_resource_weight == 0 and all(x == 0 for x in la_w)))
        for r in range(abi.KG_LA_R):
            c.la_w[r] = la_w[r]
        c.la_dominant_w = la.dominant_resource_weight
        c.la_filter_expired = int(bool(la.filter_expired_node_metrics) and la.node_metric_expiration_seconds is not None)
        c.la_schedule_expired = int(bool(la.enable_schedule_when_node_metrics_expired))
        c.la_score_prod = int(bool(la.score_according_prod_usage))
        ns = dict(self.numa_scoring)
        c.numa_w_cpu, c.numa_w_mem = ns.get(CPU, 0), ns.get(MEMORY, 0)
        nh = dict(self.numa_hint_scoring)
        c.numa_hint_w_cpu, c.numa_hint_w_mem = nh.get(CPU, 0), nh.get(MEMORY, 0)
        c.weight_dev = self.weight_dev
        c.weight_rsv = self.weight_rsv
        c.numa_most_allocated = int(self.numa_strategy == "MostAllocated")
        c.numa_hint_most_allocated = int(self.numa_hint_strategy == "MostAllocated")
        c.dev_most_allocated = int(self.dev_strategy == "MostAllocated")
        names = (CPU, MEMORY) + tuple(self.scalar_resources)
        c.nrf_most_allocated = sum(1 << r for r, name in enumerate(names) if name in self.nrf_most)
        c.nrf_ignored_scalars = self._ignore_mask(self.nrf_ignored, self.nrf_ignored_groups)
        c.rsv_ignored_scalars = self._ignore_mask(self.rsv_ignored, self.rsv_ignored_groups)
        ds = dict(self.dev_scoring)
        for r, name in enumerate(DEV_RESOURCES):
            c.dev_w[r] = ds.get(name, 0)
        return c


def shipped_profile() -> SchedulerConfig:
    """config/manager/scheduler-config.yaml:15-47 restricted to NodeResourcesFit, LoadAware, NUMA."""
    return SchedulerConfig(
        loadaware=LoadAwareArgs(filter_expired_node_metrics=False, node_metric_expiration_seconds=300,
                                resource_weights={CPU: 1, MEMORY: 1}, usage_thresholds={CPU: 0, MEMORY: 0},
                                estimated_scaling_factors={CPU: 85, MEMORY: 70}))


def config5_profile() -> SchedulerConfig:
    """Config 5 of BASELINE.md: configs 1-2's plugins plus DeviceShare, Reservation and ElasticQuota."""
    plugins = (abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_LA | abi.KG_PLUGIN_NUMA | abi.KG_PLUGIN_DEV | abi.KG_PLUGIN_RSV
               | abi.KG_PLUGIN_QUOTA)
    return SchedulerConfig(plugins=plugins, loadaware=LoadAwareArgs())


def bench_profile(numa: bool = True) -> SchedulerConfig:
    """Configs 1-2 of BASELINE.md: LoadAware defaults (thresholds cpu 65 / mem 95)."""
    plugins = abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_LA | (abi.KG_PLUGIN_NUMA if numa else 0)
    return SchedulerConfig(plugins=plugins, loadaware=LoadAwareArgs())
