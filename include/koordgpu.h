/*
 * koordgpu.h — C ABI of the MI355X Filter/Score evaluation engine for koord-scheduler.
 *
 * This is the drop-in boundary. The reference scheduler (Go, k8s.io/kubernetes v1.35.6 framework
 * wrapped by koordinator's frameworkext) evaluates one pod against every node per scheduling cycle
 * through the plugin interfaces below; a batch-aware plugin (see INTEGRATION.md for the cgo stub)
 * replaces those per-node calls with calls into this library:
 *
 *   fwktype.PreFilterPlugin.PreFilter   pkg/scheduler/plugins/loadaware/load_aware.go:139
 *       -> kg_pods_upload + kg_eval_verify / kg_eval_select (whole-cycle results, one call per batch)
 *   fwktype.FilterPlugin.Filter         pkg/scheduler/plugins/loadaware/load_aware.go:150
 *                                       pkg/scheduler/plugins/nodenumaresource/plugin.go:363
 *                                       upstream noderesources.Fits (restated, reservation/plugin.go:915-965)
 *       -> bit lookup in kg_verify_out.status (per pod, per node)
 *   fwktype.ScorePlugin.Score           pkg/scheduler/plugins/loadaware/load_aware.go:235
 *                                       pkg/scheduler/plugins/nodenumaresource/scoring.go:67
 *       -> lookup in kg_verify_out.score_* (int64, same values the Go plugins return)
 *   selectHost (upstream schedulePod)   -> kg_eval_select (deterministic tie-break)
 *   fwktype.ReservePlugin.Reserve       pkg/scheduler/plugins/loadaware/load_aware.go:226
 *                                       pkg/scheduler/plugins/nodenumaresource/plugin.go:585
 *       -> kg_assume;  Unreserve (load_aware.go:231) -> kg_forget
 *   one-pod-per-cycle replay            -> kg_replay (device-resident Assume between pods)
 *   node informer / NodeMetric / NRT event handlers
 *       (loadaware/pod_assign_cache.go:365-413,498-603) -> kg_snapshot_update_rows
 *
 * Conventions: plain C types only; every input buffer is caller-owned and read synchronously
 * (nothing is retained after a call returns); every output buffer is caller-allocated host memory.
 * Functions return kg_status and never abort; kg_last_error() gives the message of the last failure
 * on a context. Integer semantics are Go's: int64 two's complement, truncating division.
 */
#ifndef KOORDGPU_H
#define KOORDGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KG_ABI_VERSION 12

/* LoadAware resource vector width: the default vectorizer is {cpu, memory}
 * (pkg/scheduler/plugins/loadaware/helper.go:162-173, sorted by name). */
#define KG_LA_R 2
/* Scalar (extended) resources on the NodeResourcesFit path, e.g. kubernetes.io/batch-cpu,
 * kubernetes.io/batch-memory (config/manager/scheduler-config.yaml:21-31). */
#define KG_NSCALAR 2
/* NUMA zones per node supported on device (nodenumaresource/node_allocation.go:221-243). */
#define KG_MAX_ZONES 4
/* DeviceShare: GPU minors per node and per-minor resources {gpu-core, gpu-memory-ratio, gpu-memory}
 * (deviceshare/device_cache.go nodeDevice.deviceTotal / deviceFree, apis/extension/device_share.go). */
#define KG_DEV_MINORS 8
#define KG_DEV_R 3
#define KG_DEV_CORE 0
#define KG_DEV_RATIO 1
#define KG_DEV_MEM 2
/* ElasticQuota resource dimensions {cpu, memory, scalar0, scalar1}: the pod request columns
 * req_cpu, req_mem, sc_req[0], sc_req[1] (elasticquota/plugin.go:279-281). */
#define KG_QUOTA_R 4
/* Reservation resource dimensions {cpu, memory, ephemeral-storage, scalar0, scalar1}
 * (framework.Resource fields used by reservation/plugin.go:915-965). */
#define KG_RSV_R 5

typedef enum kg_status {
    KG_OK = 0,
    KG_INVALID_ARG = 1,
    KG_DEVICE_ERROR = 2,
    KG_OOM = 3,
    KG_UNSUPPORTED = 4, /* feature not on the device path: caller runs the reference plugin */
    KG_NO_DEVICE = 5,
    KG_RESERVE_FAILED = 6, /* kg_assume / kg_assume_ext: the pod's Reserve failed (a BestEffort NUMA allocation,
                            * nodenumaresource/plugin.go:612-623): nothing was applied, the pod stays unscheduled */
} kg_status;

/* Enabled plugins (kg_config.plugins). */
#define KG_PLUGIN_NRF 0x1u  /* upstream NodeResourcesFit: Fits + LeastAllocated score          */
#define KG_PLUGIN_LA 0x2u   /* LoadAwareScheduling (loadaware/load_aware.go)                     */
#define KG_PLUGIN_NUMA 0x4u /* NodeNUMAResource (nodenumaresource/plugin.go, scoring.go)         */
#define KG_PLUGIN_DEV 0x8u  /* DeviceShare GPU fit + score (deviceshare/plugin.go, scoring.go)      */
#define KG_PLUGIN_RSV 0x10u /* Reservation restore / filter / score (reservation/plugin.go, scoring.go) */
#define KG_PLUGIN_QUOTA 0x20u /* ElasticQuota PreFilter gate + Reserve (elasticquota/plugin.go)     */
#define KG_PLUGIN_EXT (KG_PLUGIN_DEV | KG_PLUGIN_RSV | KG_PLUGIN_QUOTA)

/* Node LoadAware flags (kg_node_columns.la_flags). Computed by the host at a frozen snapshot time. */
#define KG_LA_HAS_METRIC 0x1u /* podAssignCache holds a NodeMetric for the node (pod_assign_cache.go:169-172) */
#define KG_LA_NM_NIL 0x2u     /* NodeMetric.Status.NodeMetric == nil (load_aware.go:207-210)               */
#define KG_LA_EXPIRED 0x4u    /* isNodeMetricExpired (helper.go:35-40); set only when NodeMetricExpirationSeconds != nil */
#define KG_LA_PROD_THR 0x8u   /* node filter profile has non-empty ProdUsageThresholds (load_aware.go:162)  */
#define KG_LA_AGG_THR 0x10u   /* node filter profile has an AggregatedUsage profile (load_aware.go:167)     */

/* NUMA topology policies (apis/extension/numa_aware.go:168-171). */
#define KG_NUMA_NONE 0u
#define KG_NUMA_BEST_EFFORT 1u
#define KG_NUMA_RESTRICTED 2u
#define KG_NUMA_SINGLE_NODE 3u

/* Pod flags (kg_pod_columns.flags). */
#define KG_POD_DAEMONSET 0x1u /* owned by a DaemonSet (loadaware/helper.go:141-149)                    */
#define KG_POD_PROD 0x2u      /* GetPodPriorityClassWithDefault == prod (apis/extension/priority_utils.go:37-57) */
#define KG_POD_NUMA_SKIP 0x4u /* PodRequests all zero -> NodeNUMAResource Skip (nodenumaresource/plugin.go:277-283) */
#define KG_POD_HAS_CPU 0x8u   /* "cpu" key present in PodRequests                                       */
#define KG_POD_HAS_MEM 0x10u  /* "memory" key present in PodRequests                                    */
#define KG_POD_CPU_BIND 0x20u /* state.requestCPUBind: LSE/LSR pod with a Full/Spread cpuset bind policy */
#define KG_POD_NON_PREEMPTIBLE 0x40u /* extension.IsPodNonPreemptible (elasticquota/plugin.go:288)     */
/* cpuset binding request of a KG_POD_CPU_BIND pod (plugin.go:319-349: requestCPUBind, the resolved
 * preferred/required CPUBindPolicy, the preferred CPUExclusivePolicy); numCPUsNeeded = req_cpu / 1000. */
#define KG_POD_CPU_POLICY_SHIFT 8    /* 2 bits KG_CPU_BIND_*: cpuBindPolicy (required one if set)        */
#define KG_POD_CPU_REQUIRED 0x400u   /* the policy is RequiredCPUBindPolicy                              */
#define KG_POD_CPU_EXCL_SHIFT 11     /* 2 bits KG_CPU_EXCL_*                                             */
#define KG_POD_RSV_REQUIRED 0x80u    /* pod has a reservation affinity (reservation/transformer.go:148,
                                      * stateData.hasAffinity): must allocate from a reservation      */

/* GPURequirements flags (kg_pod_columns.dev_flags). */
#define KG_GPU_POD_SHARED 0x1u      /* gpuShared: per-GPU gpu-core / memory ratio below 100 (devicehandler_gpu.go:53-96) */
#define KG_GPU_POD_HONOR 0x2u       /* GPUPartitionSpec annotation present: honorGPUPartition                    */
#define KG_GPU_POD_RESTRICTED 0x4u  /* GPUPartitionSpec AllocatePolicy Restricted                                */
#define KG_GPU_POD_RING_BW 0x8u     /* GPUPartitionSpec RingBusBandwidth set (kg_pod_columns.dev_ring_bw)          */
#define KG_GPU_POD_SCOPE_SHIFT 4    /* 3 bits: DeviceTopologyScopeLevel of the required scope (0 none, 2 NUMANode,
                                     * 3 PCIe, 4 Device; apis/extension/device_share.go:185-190)               */
#define KG_GPU_POD_TEMPLATE 0x100u  /* enforceGPUSharedResourceTemplate (deviceshare/utils.go:540-547): the
                                     * allocator starts at allocateByTemplate (allocator_gpu.go:135-159), per
                                     * node key kg_pod_columns.dev_tmpl                                        */

/* Reservation allocate policies (apis/scheduling/v1alpha1 ReservationAllocatePolicy). */
#define KG_RSV_DEFAULT 0u
#define KG_RSV_ALIGNED 1u
#define KG_RSV_RESTRICTED 2u

/* Per-(pod,node) filter status bits (kg_verify_out.status). Plugin order follows the framework's
 * filter order: NodeResourcesFit, LoadAwareScheduling, NodeNUMAResource. */
#define KG_ST_NRF_PODS 0x1u   /* "Too many pods"                          */
#define KG_ST_NRF_CPU 0x2u    /* "Insufficient cpu"                       */
#define KG_ST_NRF_MEM 0x4u    /* "Insufficient memory"                    */
#define KG_ST_NRF_EPH 0x8u    /* "Insufficient ephemeral-storage"         */
#define KG_ST_NRF_SC0 0x10u   /* "Insufficient <scalar 0>"                */
#define KG_ST_NRF_SC1 0x20u   /* "Insufficient <scalar 1>"                */
#define KG_ST_NRF_MASK 0x3Fu
#define KG_ST_LA_EXPIRED 0x100u /* ErrReasonNodeMetricExpired                        */
#define KG_ST_LA_CPU 0x200u     /* ErrReasonUsageExceedThreshold, cpu                */
#define KG_ST_LA_MEM 0x400u     /* ErrReasonUsageExceedThreshold, memory             */
#define KG_ST_LA_AGG 0x800u     /* set with LA_CPU/LA_MEM: "aggregated usage" reason */
#define KG_ST_LA_MASK 0x0F00u
/* NodeNUMAResource Reserve failures of a BestEffort node (the Filter does not admit there, plugin.go:446-455;
 * Reserve runs the topology manager, plugin.go:612-623, and the allocation of its best hint,
 * resource_manager.go:300-309). Reported by kg_replay's out_reason and kg_batch_schedule's status. */
#define KG_ST_NUMA_INSUF_CPU 0x1000u  /* "Insufficient NUMA cpu"                              */
#define KG_ST_NUMA_INSUF_MEM 0x2000u  /* "Insufficient NUMA memory"                           */
#define KG_ST_NUMA_INSUF_NODE 0x4000u /* "node(s) Insufficient NUMA Node resources" (no zones)  */
#define KG_ST_NUMA_AMP_CPU 0x10000u  /* ErrInsufficientAmplifiedCPU                          */
#define KG_ST_NUMA_CONFLICT 0x20000u /* ErrNotMatchNUMATopology (UnschedulableAndUnresolvable) */
#define KG_ST_NUMA_NO_RES 0x40000u   /* "node(s) missing NUMA resources"                      */
#define KG_ST_NUMA_ALIGN 0x80000u    /* ErrNUMAHintCannotAligned                              */
#define KG_ST_NUMA_UNSATISFIED 0x100000u /* ErrUnsatisfiedNUMAResource: a requested resource has no NUMA hint
                                            (frameworkext/topologymanager/policy.go:166-173)     */
#define KG_ST_NUMA_CPU_TOPO 0x200000u /* ErrInvalidCPUTopology (UnschedulableAndUnresolvable)              */
#define KG_ST_NUMA_CPU_BIND 0x400000u /* ErrCPUBindPolicyConflict / ErrSMTAlignmentError / ErrInvalidRequestedCPUs
                                       * (UnschedulableAndUnresolvable, plugin.go:388-418, util.go:131-135) */
#define KG_ST_NUMA_CPUS 0x800000u     /* ErrNotEnoughCPUs: the required bind policy's CPUs do not cover the pod */
#define KG_ST_NUMA_MASK 0xFF7000u
#define KG_ST_DEV_INSUFFICIENT 0x01000000u /* "Insufficient gpu devices" (Unschedulable, device_allocator.go:432) */
#define KG_ST_DEV_NO_DEVICE 0x02000000u    /* no GPU minors on the node's Device (UnschedulableAndUnresolvable,
                                              devicehandler_gpu.go:41-44)                              */
/* DeviceShare reasons are a 4-bit code: bits 24-25 are its low half, bits 6-7 its high half
 * (KG_ST_DEV_CODE). Codes 3.. come from the GPU allocator (deviceshare/allocator_gpu.go:31-41). */
#define KG_ST_DEV_MASK 0x030000C0u
#define KG_ST_DEV_CODE(st) ((((st) >> 24) & 3u) | ((((st) >> 6) & 3u) << 2))
#define KG_ST_DEV_MAKE(code) (((((uint32_t)(code)) & 3u) << 24) | (((((uint32_t)(code)) >> 2) & 3u) << 6))
#define KG_DEV_CODE_INSUFFICIENT 1u      /* "Insufficient gpu devices" (defaultAllocateDevices)                 */
#define KG_DEV_CODE_NO_DEVICE 2u         /* no GPU minors on the node's Device                                  */
#define KG_DEV_CODE_GPU_DEVICES 3u       /* ErrInsufficientGPUDevices: the topology-tree allocation failed       */
#define KG_DEV_CODE_TOPO_SCOPED 4u       /* ErrInsufficientTopologyScopedGPUDevices (required topology scope)    */
#define KG_DEV_CODE_PARTITIONED 5u       /* ErrInsufficientPartitionedDevice (partitions honored)                */
#define KG_DEV_CODE_NO_PARTITION 6u      /* ErrNodeMissingGPUPartitionTable (partitions honored)                 */
#define KG_DEV_CODE_PART_COUNT 7u        /* ErrUnsupportedGPURequests: no partition of that GPU count (honored)  */
#define KG_DEV_CODE_NO_TREE 8u           /* ErrNodeMissingGPUDeviceTopologyTree (required topology scope)        */
#define KG_DEV_CODE_MULTI_SHARED 9u      /* ErrUnsupportedMultiSharedGPU (required topology scope)               */
#define KG_DEV_CODE_NUMA_SCOPED 10u      /* ErrInsufficientNUMAScopedDevices (topology_hint.go:34): the NUMA hint
                                            provider found fewer GPUs in a NUMA mask than requested             */
#define KG_DEV_CODE_NO_TEMPLATE 11u      /* ErrNoMatchedGPUSharedResourceTemplate (allocator_gpu.go:40,142-143)  */
#define KG_ST_RSV_AFFINITY 0x04000000u     /* ErrReasonReservationAffinity (reservation/plugin.go:366-368)  */
#define KG_ST_RSV_NODE 0x08000000u         /* "Insufficient <r> by node" (reservation/plugin.go:498-525)    */
#define KG_ST_RSV_RESERVATION 0x10000000u  /* reservation-level reasons / no reservation meets the pod      */
#define KG_ST_RSV_MASK 0x1C000000u
#define KG_ST_QUOTA 0x20000000u            /* ElasticQuota PreFilter: "Insufficient quotas" / non-preemptible
                                              (pod-level, reported on every node)                       */
#define KG_ST_DEV_RSV 0x40000000u          /* "Reservation(s) Insufficient gpu devices": the pod must allocate from a
                                            * matched reservation and none fits (deviceshare/reservation.go:404-406) */
#define KG_ST_UNSUPPORTED 0x80000000u /* pair needs the host path (e.g. cpuset binding)        */

typedef struct kg_ctx kg_ctx;   /* one per device per scheduler profile */
typedef struct kg_snap kg_snap; /* device-resident node snapshot (one shard) */
typedef struct kg_pods kg_pods; /* device-resident pending-pod batch + result buffers */

/* Plugin arguments that shape the arithmetic (pkg/scheduler/apis/config/types.go:31-435 after
 * v1 defaulting, pkg/scheduler/apis/config/v1/defaults.go:100-163). */
typedef struct kg_config {
    uint32_t plugins;      /* KG_PLUGIN_* */
    int64_t weight_nrf;    /* score plugin weights (config/manager/scheduler-config.yaml:87-98) */
    int64_t weight_la;
    int64_t weight_numa;
    /* NodeResourcesFit LeastAllocated scoringStrategy weights, resources {cpu, memory, scalar0, scalar1};
     * 0 = resource not listed. */
    int64_t nrf_w_cpu, nrf_w_mem, nrf_w_sc[KG_NSCALAR];
    /* LoadAwareScheduling */
    uint32_t la_score_enabled;      /* scoreWeights != nil (load_aware.go:113-116)              */
    uint32_t la_filter_expired;     /* FilterExpiredNodeMetrics (load_aware.go:199)             */
    uint32_t la_schedule_expired;   /* EnableScheduleWhenNodeMetricsExpired (load_aware.go:201) */
    uint32_t la_score_prod;         /* ScoreAccordingProdUsage (load_aware.go:256)              */
    int64_t la_w[KG_LA_R];          /* ResourceWeights by vectorizer index {cpu, memory}        */
    int64_t la_dominant_w;          /* DominantResourceWeight                                   */
    /* NodeNUMAResource LeastAllocated ScoringStrategy (node score) and NUMAScoringStrategy (hints). */
    int64_t numa_w_cpu, numa_w_mem;
    int64_t numa_hint_w_cpu, numa_hint_w_mem;
    /* DeviceShare / Reservation score plugin weights (config/manager/scheduler-config.yaml:91-96) and
     * DeviceShare LeastAllocated weights over {gpu-core, gpu-memory-ratio, gpu-memory}, 0 = resource
     * not listed (defaults ratio 1, memory 1: pkg/scheduler/apis/config/v1/defaults.go:254-277). */
    int64_t weight_dev;
    int64_t weight_rsv;
    int64_t dev_w[KG_DEV_R];
    /* ScoringStrategy type MostAllocated instead of LeastAllocated (nodenumaresource/most_allocated.go,
     * deviceshare/scoring.go:283-308): NodeNUMAResource node score, its NUMA hint score, DeviceShare. */
    uint32_t numa_most_allocated;
    uint32_t numa_hint_most_allocated;
    uint32_t dev_most_allocated;
    /* NodeResourcesFit scoringStrategy per resource: bit r set = MostAllocated for resource r of {cpu,
     * memory, scalar0, scalar1} (all bits: upstream's MostAllocated strategy; a mix: the per-resource
     * types of NodeResourcesFitPlus, noderesourcefitplus/node_resource_fit_plus_utils.go:58-86). */
    uint32_t nrf_most_allocated;
    /* Scalar resources left out of the fit checks (bit k: scalar k), from NodeResourcesFitArgs
     * IgnoredResources / IgnoredResourceGroups and the Reservation plugin's ignored resources
     * (reservation/plugin.go:897-909: extended resources only, never the native ones). */
    uint32_t nrf_ignored_scalars;
    uint32_t rsv_ignored_scalars;
} kg_config;

/* Node snapshot, struct-of-arrays host columns, n_nodes entries each (caller-owned, copied). */
/* ---- cpuset binding (NodeNUMAResource with LSE/LSR pods) ----------------------- */
#define KG_MAX_CPUS 256
/* CPU bind policies (apis/scheduling/config CPUBindPolicy) and exclusive policies (CPUExclusivePolicy). */
#define KG_CPU_BIND_NONE 0u
#define KG_CPU_BIND_FULL_PCPUS 1u
#define KG_CPU_BIND_SPREAD_BY_PCPUS 2u
#define KG_CPU_EXCL_NONE 0u
#define KG_CPU_EXCL_PCPU_LEVEL 1u
#define KG_CPU_EXCL_NUMA_NODE_LEVEL 2u
/* Node CPU bind policy (apis/extension NodeCPUBindPolicy via GetNodeCPUBindPolicy). */
#define KG_NODE_CPU_BIND_NONE 0u
#define KG_NODE_CPU_BIND_FULL_PCPUS_ONLY 1u
#define KG_NODE_CPU_BIND_SPREAD_BY_PCPUS 2u
/* NUMA allocate strategy of the accumulator (NUMAMostAllocated / NUMALeastAllocated). */
#define KG_NUMA_MOST_ALLOCATED 0u
#define KG_NUMA_LEAST_ALLOCATED 1u
/* CPU topology of one node (nodenumaresource/cpu_topology.go CPUTopology). CPU ids are 0..n_cpus-1; core,
 * NUMA node and socket ids are dense ranks of the reference's ids (order preserved: the accumulator breaks
 * ties by id). n_sockets == 0 (or any count 0): no valid topology (CPUTopology.IsValid). */
typedef struct kg_cpu_topo {
    uint16_t n_cpus, n_cores, n_nodes, n_sockets;
    uint8_t core[KG_MAX_CPUS];
    uint8_t numa[KG_MAX_CPUS];
    uint8_t socket[KG_MAX_CPUS];
} kg_cpu_topo;
/* CPUs already allocated on a node (NodeAllocation.allocatedCPUs): per CPU its RefCount (0 = free) and the
 * CPUExclusivePolicy of the allocation that holds it. */
typedef struct kg_cpu_alloc {
    uint8_t ref[KG_MAX_CPUS];
    uint8_t excl[KG_MAX_CPUS];
} kg_cpu_alloc;

/* One takeCPUs / takePreferredCPUs request (nodenumaresource/cpu_accumulator.go:30-246). */
typedef struct kg_cpuset_request {
    uint32_t topo;          /* index into the topologies of the call                                   */
    int32_t alloc;          /* index into the allocations of the call, -1 = nothing allocated          */
    uint64_t avail[4];      /* allocatable CPUs (NodeAllocation.getAvailableCPUs)                       */
    uint64_t preferred[4];  /* preferred CPUs (takePreferredCPUs); used when has_preferred               */
    int32_t needed;         /* numCPUsNeeded                                                            */
    int32_t max_ref;        /* TopologyOptions.MaxRefCount (>= 1)                                       */
    int32_t bind;           /* KG_CPU_BIND_*                                                            */
    int32_t excl;           /* the pod's KG_CPU_EXCL_*                                                  */
    int32_t strategy;       /* KG_NUMA_MOST_ALLOCATED / KG_NUMA_LEAST_ALLOCATED                         */
    int32_t has_preferred;
} kg_cpuset_request;

/* One GPU partition (apis/extension/device_share.go:221-227 GPUPartition). */
#define KG_GPU_NO_SCOPE 0xFFu
#define KG_GPU_HONOR 0x100u
#define KG_GPU_TREE 0x200u
#define KG_GPU_TMPL_SHIFT 12 /* dev_part bits 12-15: the node's shared-resource template key (KG_GPU_TMPL_NONE = none) */
#define KG_GPU_TMPL_NONE 15u
#define KG_ZONE_RECORD_SHIFT 8 /* numa_zone_status: zone z has an allocation record (node_allocation.go:145-154) */
#define KG_GPU_MAX_TABLES 16
#define KG_GPU_MAX_PARTS 1024
typedef struct kg_gpu_partition {
    uint8_t table;           /* partition table index (dev_part - 1)                                   */
    uint8_t n_gpus;          /* the table key: number of GPUs (1..8)                                   */
    uint8_t minors;          /* MinorsHash: bit m = minor m                                            */
    uint8_t pad_;
    int32_t alloc_score;     /* AllocationScore                                                        */
    int64_t ring_bw;         /* RingBusBandwidth in bytes, -1 = none                                   */
} kg_gpu_partition;

typedef struct kg_node_columns {
    /* upstream NodeInfo (k8s v1.35.6): Allocatable / Requested / NonZeroRequested / len(Pods) */
    const int64_t *alloc_cpu, *alloc_mem, *alloc_eph, *alloc_pods;
    const int64_t *req_cpu, *req_mem, *req_eph, *num_pods;
    const int64_t *nz_cpu, *nz_mem;
    const int64_t *sc_alloc[KG_NSCALAR], *sc_req[KG_NSCALAR];
    /* LoadAwareScheduling: EstimateNode allocatable, thresholds of the node's filter profile after
     * its custom-threshold annotation (helper.go:83-121), and the estimated usage of existing pods
     * returned by GetNodeMetricAndEstimatedOfExisting (pod_assign_cache.go:163-201) for the filter
     * (non-prod / prod pod) and the score (non-prod / prod pod). */
    const uint32_t* la_flags;
    const int64_t* la_alloc[KG_LA_R];
    const int64_t* la_thr_usage[KG_LA_R];
    const int64_t* la_thr_prod[KG_LA_R];
    const int64_t* la_thr_agg[KG_LA_R];
    const int64_t* la_fbase_np[KG_LA_R];
    const int64_t* la_fbase_prod[KG_LA_R];
    const int64_t* la_sbase_np[KG_LA_R];
    const int64_t* la_sbase_prod[KG_LA_R];
    /* NodeNUMAResource */
    const uint32_t* numa_policy;        /* KG_NUMA_* after merging node label and kubelet policy     */
    const uint32_t* numa_zones;         /* number of NUMA zones with resources (0..KG_MAX_ZONES)     */
    const double* cpu_amp_ratio;        /* cpu amplification ratio (<= 1: none)                      */
    const int64_t* cpuset_alloc_milli;  /* milli-cpu allocated as cpusets                            */
    const int64_t* zone_cpu[KG_MAX_ZONES];      /* zone totals (amplified, util.go:101-124)          */
    const int64_t* zone_mem[KG_MAX_ZONES];
    const int64_t* zone_cpu_used[KG_MAX_ZONES]; /* zone allocated                                     */
    const int64_t* zone_mem_used[KG_MAX_ZONES];
    /* DeviceShare: the node's GPU minors (nodeDevice of deviceshare/device_cache.go). dev_minors < 0:
     * the node has no Device object (Filter passes, Score 0: deviceshare/plugin.go:398-401,
     * scoring.go:58-61); otherwise minors 0..dev_minors-1. dev_total / dev_free are row-major
     * [node][KG_DEV_R][KG_DEV_MINORS] with 0 <= free <= total (NULL = no DeviceShare data). */
    const int32_t* dev_minors;
    const int64_t* dev_total;
    const int64_t* dev_free;
    /* NUMA node shared status per zone, 2 bits each (0 idle, 1 single, 2 shared; NUMANodeSharedStatus,
     * nodenumaresource/node_allocation.go:52-68) for the Required exclusive policy of pods with a
     * pod-level NUMA policy (NULL = all idle). */
    const uint32_t* numa_zone_status;  /* 2 bits per zone NUMANodeSharedStatus; bit KG_ZONE_RECORD_SHIFT + z: the
                                        * NodeAllocation holds an allocatedResources record for zone z */
    /* cpuset binding (NodeNUMAResource, LSE/LSR pods; all may be NULL = no CPU topology anywhere):
     * cpu_topo[i] indexes cpu_topos (-1 = the node has no CPU topology: ErrInvalidCPUTopology for a
     * cpuset-binding pod); cpu_alloc[i] = the node's allocated CPUs (NULL = none). cpuset_alloc_milli must
     * then equal 1000 x the CPUs with RefCount > 0. cpu_max_ref (NULL = 1), cpu_bind_policy
     * (KG_NODE_CPU_BIND_*, GetNodeCPUBindPolicy) and cpu_strategy (KG_NUMA_MOST/LEAST_ALLOCATED,
     * GetNUMAAllocateStrategy) are per node. */
    const int32_t* cpu_topo;
    const kg_cpu_topo* cpu_topos;
    uint32_t n_cpu_topos;
    const kg_cpu_alloc* cpu_alloc;
    const uint8_t* cpu_max_ref;
    const uint8_t* cpu_bind_policy;
    const uint8_t* cpu_strategy;
    /* DeviceShare GPU topology and partitions (deviceshare/allocator_gpu.go:72-451, allocator_gpu_helper.go
     * :150-275; all may be NULL = no tree, no partition table, Prefer policy):
     * dev_topo[i]: byte m = GPU minor m's place in the topology tree (GetGPUTopologyScope): high nibble the
     *   rank of its NUMA node id (numeric order), low nibble the rank of its (NUMA node, PCIe id) pair
     *   (PCIe ids in string order within a NUMA node); each rank < 8 (the device reads 3 bits of each nibble;
     *   more than 8 NUMA nodes or pairs is unsupported); KG_GPU_NO_SCOPE = the minor is in no NUMA / PCIe scope;
     * dev_part[i]: bits 0-7 = 1 + the node's partition table in gpu_parts (0 = none: GetGPUPartitionIndexer of
     *   the Device annotation, else the designated table of the node's GPU model), KG_GPU_HONOR = the
     *   GPUPartitionPolicy label is Honor, KG_GPU_TREE = the node has a topology tree (every GPU DeviceInfo
     *   carries a Topology), bits 12-15 (KG_GPU_TMPL_SHIFT) = the index of the node's GPU shared-resource
     *   template key buildGPUSharedResourceTemplatesKey(vendor, model) among the configured keys, or
     *   KG_GPU_TMPL_NONE when the configuration holds no templates for that key;
     * gpu_parts: every partition of every table (kg_gpu_partition), grouped by table, then GPU count, then
     *   AllocationScore ascending; within a group in the table's order (GetGPUPartitionIndexer). */
    const uint64_t* dev_topo;
    const uint32_t* dev_part;
    const struct kg_gpu_partition* gpu_parts;
    uint32_t n_gpu_parts;
    /* DeviceShare NUMA topology (deviceshare/numa_topology.go:43-100, NUMATopology.deviceToNodeID; NULL = every
     * minor without a topology): nibble m of dev_numa[i] = GPU minor m's NUMA node id (0..KG_MAX_ZONES-1, the NRT zone of
     * that id; the upload rejects larger ids), KG_GPU_NUMA_ANY = its Topology.NodeID is -1 (in every NUMA mask, in no NUMA scope), KG_GPU_NUMA_NONE =
     * no Topology (left out whenever a NUMA affinity restricts the allocation, device_allocator.go:155-159).
     * GPU pods on nodes whose NUMA policy is not None join the topology manager's hint merge with these
     * (deviceshare/topology_hint.go:40-290). */
    const uint32_t* dev_numa;
    /* The cpuset pods behind numa_zone_status (NodeAllocation.singleNUMANode / sharedNode, node_allocation.go:111-143):
     * byte z (z < KG_MAX_ZONES) = pods whose CPUs lie in NUMA node z only, byte KG_MAX_ZONES + z = pods whose CPUs span z
     * and another node (saturating at 255). A cpuset Release (kg_unreserve) takes its pod out again, so the statuses it
     * leaves follow from these counts. NULL: one pod per non-idle status (single -> 1 / 0, shared -> 0 / 1); when given,
     * the 2-bit statuses of numa_zone_status are derived from them. */
    const uint64_t* numa_zone_pods;
    /* 1: a reservation on the node (matched by the pod or not) holds a NUMA or cpuset allocation (its reserve pod's
     * resource status). NodeNUMAResource's RestoreReservation (nodenumaresource/reservation.go:188-262) gives such
     * allocations back to the owners of a matched reservation and the double-counted owner usage of unmatched ones,
     * in the hints (resource_manager.go:131-160), tryAllocateFromReusable / tryAllocateFromNode (plugin.go:428-439,
     * 807-851) and the Reserve; the device does not follow that restore, so every pair on such a node where the
     * plugin reads it (the pod binds CPUs there, or the merged NUMA policy is not None) is KG_ST_UNSUPPORTED and the
     * sequential calls (kg_replay, kg_batch_schedule, kg_reserve, kg_assume*) refuse those pods (KG_UNSUPPORTED).
     * NULL = none (ABI 12). */
    const uint8_t* rsv_numa;
} kg_node_columns;
#define KG_GPU_NUMA_ANY 0xEu
#define KG_GPU_NUMA_NONE 0xFu

/* Mutable node state that Assume/Forget change; used to read a snapshot back after kg_replay. */
typedef struct kg_node_state {
    int64_t *req_cpu, *req_mem, *req_eph, *num_pods, *nz_cpu, *nz_mem;
    int64_t* sc_req[KG_NSCALAR];
    int64_t *la_fbase_np[KG_LA_R], *la_fbase_prod[KG_LA_R];
    int64_t *la_sbase_np[KG_LA_R], *la_sbase_prod[KG_LA_R];
    int64_t *zone_cpu_used[KG_MAX_ZONES], *zone_mem_used[KG_MAX_ZONES];
    int64_t* dev_free; /* [node][KG_DEV_R][KG_DEV_MINORS] */
    int64_t* cpuset_alloc_milli;
    kg_cpu_alloc* cpu_alloc; /* [node] (nodes without a CPU topology: zeros) */
    uint32_t* numa_zone_status; /* NUMANodeSharedStatus, 2 bits per zone (a cpuset Reserve changes it) */
    uint64_t* numa_zone_pods;   /* kg_node_columns.numa_zone_pods */
} kg_node_state;

/* Pending pods, struct-of-arrays host columns (caller-owned, copied). */
typedef struct kg_pod_columns {
    const int64_t *req_cpu, *req_mem, *req_eph; /* PodRequests: milli-cpu, bytes, bytes            */
    const int64_t* sc_req[KG_NSCALAR];
    const int64_t *nz_cpu, *nz_mem;             /* non-zero requests (100m / 200Mi defaults)        */
    const int64_t* la_est[KG_LA_R];             /* DefaultEstimator.EstimatePod (estimator/default_estimator.go:57-120) */
    const uint32_t* flags;                      /* KG_POD_*                                         */
    const uint32_t* numa_policy;                /* pod NUMA topology policy annotation, KG_NUMA_*   */
    /* DeviceShare GPURequirements (deviceshare/utils.go:516-545, devicehandler_gpu.go:53-96):
     * per-instance request [pod][KG_DEV_R], number of GPUs (0 = no GPU request: PreFilter Skip) and
     * the keys present in requestsPerGPU (bit KG_DEV_*). */
    const int64_t* dev_req;
    const uint32_t* dev_count;
    const uint32_t* dev_keys;
    /* ElasticQuota: quota index (-1 = none: PreFilter Skip) and the keys of PodRequests masked by the
     * quota's Max names (bit r of KG_QUOTA_R), elasticquota/plugin.go:279-281. */
    const int32_t* quota;
    const uint32_t* quota_keys;
    /* Reservation owner-match class (-1 = the pod matches no reservation): pods of one class match
     * the same reservations (reservation/transformer.go:233-240, checkReservationMatchedOrIgnored). */
    const int32_t* rsv_class;
    /* GPURequirements beyond the request (deviceshare/utils.go:516-545; NULL = none): KG_GPU_POD_* flags and
     * the GPUPartitionSpec RingBusBandwidth in bytes (read when KG_GPU_POD_RING_BW is set). */
    const uint32_t* dev_flags;
    const int64_t* dev_ring_bw;
    /* candidateGPUSharedResourceTemplates of a KG_GPU_POD_TEMPLATE pod (deviceshare/utils.go:540-547,
     * gpu_shared_resource_templates_cache.go:41-62): 2 bits per template key k < KG_GPU_TMPL_NONE (the node's
     * key in dev_part bits 12-15) = how many templates of key k the pod's requestsPerGPU matched: 0 none, 1 one,
     * 2 several. NULL = no template pods. */
    const uint32_t* dev_tmpl;
} kg_pod_columns;

/* Verify-mode outputs, [n_pods][n_nodes] row-major, caller-allocated host buffers (NULL = skip). */
typedef struct kg_verify_out {
    uint32_t* status;     /* KG_ST_* bits per plugin; 0 = feasible                         */
    int64_t* score_nrf;   /* NodeResourcesFit score (0 when infeasible or plugin disabled)  */
    int64_t* score_la;    /* LoadAwareScheduling score                                      */
    int64_t* score_numa;  /* NodeNUMAResource score                                         */
    int64_t* total;       /* Σ weight·score, -1 when infeasible                             */
    int8_t* numa_zone;    /* NUMA allocation the Reserve would make: -1 none, 0..3 one zone,
                             0x40 | zone mask for a split over several zones, 0x20 | bits when
                             the Reserve fails (BestEffort: bits = KG_ST_NUMA_INSUF_* >> 12,
                             0x08 the cpuset take), 0x30 | KG_DEV_CODE_* when the GPU allocation
                             under the Reserve's NUMA affinity fails (a GPU pod on a BestEffort node).
                             A GPU pod's Reserve allocates its minors inside the NUMA nodes of this
                             affinity (deviceshare/plugin.go:585-600) */
    int64_t* score_dev;   /* DeviceShare Score before NormalizeScore (0 when infeasible)    */
    int64_t* score_rsv;   /* Reservation Score before NormalizeScore (1000 on the preferred
                             node, reservation/scoring.go:40,191-198; 0 when infeasible)     */
} kg_verify_out;

/* ElasticQuota table, [quota][KG_QUOTA_R] values with per-quota key masks (bit r = key present).
 * used / used_limit: the PreFilter's state.used / state.usedLimit (runtime when EnableRuntimeQuota,
 * else max; elasticquota/plugin.go:274-284); min / np_used: CalculateInfo.Min and the non-preemptible
 * used (:286-293). Quotas are flat (no parent check: EnableCheckParentQuota=false). */
typedef struct kg_quota_columns {
    const int64_t *used, *used_limit, *min, *np_used;
    const uint32_t *used_keys, *limit_keys, *min_keys, *np_used_keys;
} kg_quota_columns;

/* Restored NodeInfo of one node as pods of one owner class see it, after the Reservation transformer
 * (reservation/transformer.go:740-811): the unmatched reservations' double-counted Allocated returned
 * (updateNodeInfoRequestedForUnmatched :918-935) and the matched reserve pods removed
 * (restoreMatchedReservation :855-878). The snapshot columns hold the view of pods that match nothing
 * on the node (every reservation unmatched). */
typedef struct kg_rsv_view {
    uint32_t node;                       /* local node index                                         */
    uint32_t cls;                        /* owner-match class (kg_pod_columns.rsv_class)             */
    uint32_t first, count;               /* matched reservations: kg_rsv_info[first, first + count)  */
    int64_t req[KG_RSV_R];               /* restored Requested                                       */
    int64_t nz_cpu, nz_mem, num_pods;    /* restored NonZeroRequested and len(Pods)                  */
    int64_t pod_requested[KG_RSV_R];     /* nodeRState.podRequested (after the unmatched correction) */
    int64_t r_allocated[KG_RSV_R];       /* nodeRState.rAllocated: Σ Allocated of matched reservations */
    /* DeviceShare: kg_rsv_dev index of the GPU minors a pod of this class allocates from outside its
     * reservations (unmatched reservations' used and matched reservations' allocatable given back:
     * deviceshare/plugin.go:397-419, reservation.go:94-117); -1 = the node's own minors. */
    int32_t dev_base;
    uint32_t pad_;
} kg_rsv_view;

/* One matched reservation (frameworkext.ReservationInfo). */
typedef struct kg_rsv_info {
    uint32_t policy;                     /* KG_RSV_*                                                 */
    uint32_t names;                      /* bit r: resource r in ResourceNames (keys of Allocatable) */
    uint32_t allocate_once;              /* IsAllocateOnce (apis/extension/reservation.go:167)       */
    int32_t dev;                         /* kg_rsv_dev index of the GPU minors a pod allocates from this
                                          * reservation (tryAllocateFromReusable, deviceshare/reservation.go
                                          * :344-410); -1 = it reserves no GPU                         */
    int64_t order;                       /* LabelReservationOrder, 0 = none; |order| < 2^31          */
    int64_t allocatable[KG_RSV_R], allocated[KG_RSV_R], reserved[KG_RSV_R];
    int64_t max_pods;                    /* "pods" in Allocatable, -1 = absent                       */
    int64_t allocated_pods;              /* len(AssignedPods)                                        */
    uint32_t rid;                        /* the reservation's id on its node: the copies of one reservation
                                          * in the views of several classes share it (a Reserve into it
                                          * updates all of them)                                       */
    uint32_t allocated_keys;             /* bit 0 / 1: Allocated holds a cpu / memory key (0 while nil):
                                          * GetNonZeroRequestForResource of the unmatched correction   */
    uint32_t dev_minors;                 /* the GPU minors the reservation reserves (bit m; ABI 12): a pod allocating
                                          * from it takes them first (tryAllocateFromReusable's preferred set,
                                          * deviceshare/reservation.go:308; defaultAllocateDevices ->
                                          * sortDeviceResourcesByMinor, device_resources.go:187-209)      */
    uint32_t pad_;
} kg_rsv_info;

/* GPU minors as one restore sees them (nodeDevice.calcFreeWithPreemptible / filter, deviceshare/
 * device_cache.go:322-410): total and free per resource (KG_DEV_CORE / _RATIO / _MEM) and minor; a minor
 * outside the allocation's reach has total 0 and free 0. */
typedef struct kg_rsv_dev {
    int64_t total[KG_DEV_R][KG_DEV_MINORS];
    int64_t free[KG_DEV_R][KG_DEV_MINORS];
} kg_rsv_dev;

/* ------------------------------------------------------------------------------------------------ */
int kg_abi_version(void);
const char* kg_status_string(kg_status s);
/* Number of visible HIP devices (0 without a GPU; never fails). */
int kg_device_count(void);

kg_status kg_open(int device, kg_ctx** out);
kg_status kg_close(kg_ctx* ctx);
/* Message of the last failed call on ctx (empty string if none). Valid until the next call. */
const char* kg_last_error(const kg_ctx* ctx);
/* Wait for all work queued on the context's stream. */
kg_status kg_sync(kg_ctx* ctx);

/* Snapshot of n_nodes nodes whose global snapshot indices are [index_base, index_base + n_nodes). */
kg_status kg_snapshot_create(kg_ctx* ctx, const kg_config* cfg, uint32_t n_nodes, uint32_t index_base,
                             kg_snap** out);
kg_status kg_snapshot_upload(kg_snap* snap, const kg_node_columns* cols);
/* Replace rows[i] (local index) with entry i of cols (each column has n entries): the informer-event
 * deltas of one scheduling cycle in one call (one staged copy + one scatter launch on the device). */
kg_status kg_snapshot_update_rows(kg_snap* snap, const uint32_t* rows, uint32_t n, const kg_node_columns* cols);
/* Generation of the snapshot: bumped by every call that changes its contents (upload, update_rows,
 * kg_assume / kg_forget and their _ext forms, kg_replay, quota and reservation uploads). A caller that
 * stamps its host cache with it can tell whether the device has seen every delta (k8s UpdateSnapshot's
 * NodeInfo.Generation scheme; the host side is koordinator_amd.cluster). */
kg_status kg_snapshot_generation(kg_snap* snap, uint64_t* out);
kg_status kg_snapshot_read_state(kg_snap* snap, kg_node_state* out);
/* ElasticQuota table (KG_PLUGIN_QUOTA): n_quotas entries, copied; Reserve updates used / np_used. */
kg_status kg_snapshot_upload_quotas(kg_snap* snap, const kg_quota_columns* cols, uint32_t n_quotas);
/* Read back used / np_used (and their key masks) after kg_replay / kg_assume_ext. */
kg_status kg_snapshot_read_quotas(kg_snap* snap, int64_t* used, uint32_t* used_keys, int64_t* np_used,
                                  uint32_t* np_used_keys);
/* Reservation views of this snapshot (KG_PLUGIN_RSV), replacing any earlier upload. Views of one
 * class must name distinct nodes; at most 64 classes and 8 reservations per view. */
kg_status kg_snapshot_upload_reservations(kg_snap* snap, const kg_rsv_view* views, uint32_t n_views,
                                          const kg_rsv_info* infos, uint32_t n_infos, const kg_rsv_dev* devs,
                                          uint32_t n_devs);
/* DeviceShare restore inputs of the reservations that hold GPUs (deviceshare/reservation.go:139-198 RestoreReservation
 * reads them from nodeDevice every cycle): per such node one entry with rid -1 whose `a` is the node's deviceUsed, and
 * one entry per GPU-holding reservation on it (kg_rsv_info.rid): `a` = its reserve pod's allocation (allocatable),
 * `b` = its assigned pods' allocations on those minors (allocated), its policy and assigned pod count. With them
 * kg_replay, kg_batch_schedule and kg_reserve / kg_unreserve follow a Reserve into such a node on the device (the
 * node's used, the reservation the pod joins, and the restore tables of the record, the views and the reservations,
 * rebuilt as transformer.go:740-935 + reservation.go:139-198,278-380 would); without them those calls refuse
 * (KG_UNSUPPORTED) or mark the node's views stale. kg_snapshot_upload_reservations / kg_snapshot_update_views drop
 * the inputs (upload them again after). */
typedef struct kg_rsv_gpu {
    uint32_t node;           /* local node index                                                        */
    int32_t rid;             /* kg_rsv_info.rid, -1 = the node's entry                                  */
    uint32_t policy;         /* KG_RSV_* (reservation entries)                                          */
    uint32_t allocated_pods; /* len(AssignedPods) (reservation entries)                                 */
    int64_t a[KG_DEV_R][KG_DEV_MINORS];
    int64_t b[KG_DEV_R][KG_DEV_MINORS];
} kg_rsv_gpu;
kg_status kg_snapshot_upload_rsv_gpu(kg_snap* snap, const kg_rsv_gpu* entries, uint32_t n);
/* Replace the views (with their reservations and GPU restore tables) of the nodes in nodes[0, n_nodes) by views[0, n_views)
 * (each naming one of those nodes; a listed node without views loses its views); every other node keeps its views.
 * The incremental form of kg_snapshot_upload_reservations for the nodes a Reserve / Unreserve or an event changed
 * (the Reservation transformer's per-node restore, reservation/transformer.go:740-935): it clears their staleness. */
kg_status kg_snapshot_update_views(kg_snap* snap, const uint32_t* nodes, uint32_t n_nodes, const kg_rsv_view* views,
                                   uint32_t n_views, const kg_rsv_info* infos, uint32_t n_infos, const kg_rsv_dev* devs,
                                   uint32_t n_devs);
kg_status kg_snapshot_destroy(kg_snap* snap);

kg_status kg_pods_create(kg_ctx* ctx, uint32_t capacity, kg_pods** out);
kg_status kg_pods_upload(kg_pods* pods, const kg_pod_columns* cols, uint32_t n_pods);
kg_status kg_pods_destroy(kg_pods* pods);

/* Full per-plugin Filter/Score matrix for every (pod, node) pair (the FilterPlugin/ScorePlugin
 * results the Go plugins would return). */
kg_status kg_eval_verify(kg_snap* snap, kg_pods* pods, kg_verify_out* out);
/* Filter + Score + selectHost for every pending pod against the snapshot as it is (matrix mode):
 * per pod the k best packed keys (kg_make_key), descending, 0 = no feasible node. The launch is
 * asynchronous; results stay on the device until kg_result_keys. */
kg_status kg_eval_select(kg_snap* snap, kg_pods* pods, uint32_t k);
kg_status kg_result_keys(kg_pods* pods, uint64_t* out_keys /* n_pods * k */);
/* Per-pod outcome flags of the last kg_eval_select / kg_shard_select (n_pods entries):
 *   KG_ST_UNSUPPORTED  some (pod, node) pair needs the host path (cpuset binding, a failing BestEffort
 *                      NUMA Reserve, DeviceShare with device NUMA hints, ...): the pod's keys cover only
 *                      the pairs the device decided, so the caller runs the reference plugins for it;
 *   KG_ST_QUOTA        the ElasticQuota PreFilter rejected the pod (no node evaluated, keys 0);
 *   0                  the keys are the complete Filter/Score/selectHost result. */
kg_status kg_result_status(kg_pods* pods, uint32_t* out_status);
/* Sequential scheduling of pods[0..n) one at a time with Assume applied on the device between pods
 * (the reference's one-pod-per-cycle semantics). out_node[i] = global node index or -1 (no feasible node,
 * or the selected node's Reserve failed: KG_ST_NUMA_INSUF_* in out_reason).
 * out_reason (may be NULL): per pod, the OR of the KG_ST_* filter status bits over every node of the
 * snapshot as it stood in that pod's cycle (0 when every node passed) — the per-plugin reasons the
 * caller turns into the FitError diagnosis of an unschedulable pod (load_aware.go:48-51,
 * nodenumaresource/plugin.go:54-63).
 * With reservation views (KG_PLUGIN_RSV) each placement runs Reservation.Reserve on the device
 * (reservation/plugin.go:1295-1408): the pod joins its nominated reservation (Allocated += Mask(requests,
 * ResourceNames), one more assigned pod, every copy of it sharing kg_rsv_info.rid) and the node's views change as the
 * next cycle's restore would give them (transformer.go:740-935); the Reservation score (nominated reservation's
 * score, reservation order) is normalised per pod like in kg_eval_select. KG_UNSUPPORTED while a reservation holds
 * GPUs (its DeviceShare restore tables follow the reserve pods' allocations). */
kg_status kg_replay(kg_snap* snap, kg_pods* pods, int32_t* out_node, int64_t* out_total, uint32_t* out_reason);
/* Reserve/Unreserve of pod `pod` (batch index) on local node `node`. KG_RESERVE_FAILED: the NodeNUMAResource
 * Reserve fails on that node (BestEffort allocation), nothing applied. */
kg_status kg_assume(kg_snap* snap, kg_pods* pods, uint32_t pod, uint32_t node);
kg_status kg_forget(kg_snap* snap, kg_pods* pods, uint32_t pod, uint32_t node, int32_t numa_zone);
/* kg_assume that also returns the NodeNUMAResource allocation it made: *out_zone as kg_verify_out.numa_zone,
 * out_zone_amounts[2 * KG_MAX_ZONES] = cpu (milli) per zone, then memory (bytes) per zone (zeros when no zone was
 * allocated). The reference keeps that allocation for the Unreserve (nodenumaresource/plugin.go:585-635 Reserve,
 * :700 Unreserve -> resource_manager.go:478-483 Release); kg_forget_numa takes it back, including a split over
 * several zones (zone code 0x40 | mask), which kg_forget refuses. */
kg_status kg_assume_numa(kg_snap* snap, kg_pods* pods, uint32_t pod, uint32_t node, int32_t* out_zone,
                         int64_t* out_zone_amounts);
kg_status kg_forget_numa(kg_snap* snap, kg_pods* pods, uint32_t pod, uint32_t node, int32_t numa_zone,
                         const int64_t* zone_amounts);
/* Reserve with every enabled plugin's state (NodeInfo, LoadAware, NUMA zone, DeviceShare minors via
 * defaultAllocateDevices order, ElasticQuota used); returns the NUMA zone and the GPU minor bitmask
 * the Unreserve needs (deviceshare/plugin.go:507-569, elasticquota/plugin.go:622-636). With reservation views
 * and no GPU-holding reservation it also runs Reservation.Reserve on the node's views (as kg_replay does); the
 * host copies are read back before the next kg_snapshot_update_views. kg_forget_ext cannot name the reservation:
 * the node's views turn stale until the caller re-uploads them (kg_snapshot_update_views). */
kg_status kg_assume_ext(kg_snap* snap, kg_pods* pods, uint32_t pod, uint32_t node, int32_t* out_zone,
                        uint32_t* out_minors);
kg_status kg_forget_ext(kg_snap* snap, kg_pods* pods, uint32_t pod, uint32_t node, int32_t numa_zone,
                        uint32_t minors);
/* GPU minors chosen for each pod by the last kg_replay (bitmask; 0 = none), n_pods entries. */
kg_status kg_replay_minors(kg_pods* pods, uint32_t* out);

/* What one Reserve took, as the reference keeps it for the Unreserve (CycleState and the plugins' caches): the NUMA
 * zone code and per-zone amounts (nodenumaresource/plugin.go:585-635 -> resource_manager.go Update), the cpuset CPUs
 * (NodeAllocation.addPodAllocation), the GPU minors (deviceshare/plugin.go:507-569) and the reservation the pod joined
 * (reservation/plugin.go:1295-1408 assumePods; rsv_rid = kg_rsv_info.rid on the node, -1 = none). */
typedef struct kg_reserve_record {
    int32_t numa_zone;                        /* the pair's kg_verify_out.numa_zone (-1 = none)              */
    uint32_t gpu_minors;                      /* DeviceShare minors taken (bit m = minor m)                  */
    int32_t rsv_rid;                          /* nominated reservation's rid, -1 = none                      */
    uint32_t flags;                           /* KG_RECORD_*                                                 */
    int64_t zone_amounts[2 * KG_MAX_ZONES];   /* cpu milli per zone, then memory bytes per zone              */
    uint64_t cpus[KG_MAX_CPUS / 64];          /* cpuset CPUs taken                                           */
} kg_reserve_record;
#define KG_RECORD_CPUSET 0x1u  /* the Reserve took cpuset CPUs (cpus) */
#define KG_RECORD_QUOTA 0x2u   /* the Reserve added the pod to its ElasticQuota's used */
#define KG_RECORD_RELEASED 0x4u /* kg_unreserve gave the record back: a second Unreserve of it is refused */

/* Reserve of pod `pod` on local node `node` with every enabled plugin (kg_assume / kg_assume_ext: NodeInfo,
 * LoadAware, NodeNUMAResource incl. cpusets, DeviceShare, ElasticQuota, Reservation.Reserve on the node's views),
 * filling *out with what the Unreserve needs. KG_RESERVE_FAILED: nothing applied. */
kg_status kg_reserve(kg_snap* snap, kg_pods* pods, uint32_t pod, uint32_t node, kg_reserve_record* out);
/* Unreserve of a kg_reserve: every plugin gives back what the record says it took (load_aware.go:231-233,
 * nodenumaresource/plugin.go:700-720 -> resource_manager.go:478-483 Release incl. the cpuset CPUs and the NUMA
 * single / shared sets, deviceshare/plugin.go Unreserve, elasticquota/plugin.go:638-652, reservation/plugin.go:1409-1460
 * forgetPods: the reservation's Allocated and assigned pods, and the node's views as the next restore builds them).
 * The record is marked KG_RECORD_RELEASED on success; a record so marked is refused (KG_INVALID_ARG, nothing applied):
 * the reference's NodeAllocation.release and forgetPods do nothing for a pod they no longer hold (ABI 12). */
kg_status kg_unreserve(kg_snap* snap, kg_pods* pods, uint32_t pod, uint32_t node, kg_reserve_record* rec);
/* Copy of the snapshot's reservation views and infos as the device holds them (after Reservation.Reserve /
 * Unreserve on the device): n_views / n_infos entries as uploaded, in upload order. */
kg_status kg_snapshot_read_reservations(kg_snap* snap, kg_rsv_view* views, uint32_t n_views, kg_rsv_info* infos,
                                        uint32_t n_infos);
/* Copy of the GPU restore tables (kg_rsv_dev, n_devs as uploaded) as the device holds them: a Reserve / Unreserve into a
 * node with GPU-holding reservations rebuilds that node's tables (ABI 12). */
kg_status kg_snapshot_read_rsv_devs(kg_snap* snap, kg_rsv_dev* devs, uint32_t n_devs);

/* Device cpuset accumulator, one request per workgroup: out[4 * i] = the CPUs chosen for request i,
 * rc[i] = 0, -1 (ErrNotEnoughCPUs: fewer allocatable CPUs than needed) or -2 ("failed to allocate cpus").
 * Topologies need <= 8 NUMA nodes, <= 8 sockets and <= 8 CPUs per core (KG_UNSUPPORTED otherwise). */
kg_status kg_cpuset_take(kg_ctx* ctx, const kg_cpu_topo* topos, uint32_t n_topos, const kg_cpu_alloc* allocs,
                         uint32_t n_allocs, const kg_cpuset_request* reqs, uint32_t n, uint64_t* out, int32_t* rc);

/* ---- whole-job placement (FindOneNodePlugin slot, frameworkext/interface.go:118-127) ----------------
 * Checkpoint / rollback of everything Reserve changes (node records, NUMA zones, GPU minors, quota used):
 * a planner replays the job on the live snapshot and rolls back, so the plan costs no copy of the cluster
 * (the reference clones NodeInfos per plan, coscheduling/core/network_topology_workflow.go:98-118). One
 * checkpoint per snapshot; a new checkpoint replaces the old. Rollback fails if the snapshot was re-uploaded
 * or had rows updated since the checkpoint (its records may have moved). Both bump the generation. */
kg_status kg_snapshot_checkpoint(kg_snap* snap);
kg_status kg_snapshot_rollback(kg_snap* snap);

/* kg_batch_schedule result codes, per pod */
#define KG_BATCH_ASSUMED 0u     /* PreFilter + Filter passed on the planned node; Reserve applied          */
#define KG_BATCH_FAILED 1u      /* PreFilter / Filter failed on the planned node: status holds the bits    */
#define KG_BATCH_SIBLING 2u     /* after a failed pod of the same node (engine.go:188-192): its status     */
#define KG_BATCH_ROLLED_BACK 3u /* was assumed, undone because the job failed (CleanupAssumedPods)         */
#define KG_BATCH_NO_PLAN 4u     /* plan_node < 0: the job fails before any pod is assumed (batch_scheduler.go:96-101) */
/* Inline batch scheduling cycle for a planned job (batch/batch_scheduler.go:74-185 BatchSchedule,
 * batch/engine.go:92-294 RunSchedulingCycle): plan_node[j] = local node of pod j. Pods are grouped by
 * planned node; each group runs in batch order (the caller orders a node's pods by name, engine.go
 * :357-359): PreFilter (ElasticQuota gate on the current used) + Filter on that node, then Reserve. If every
 * pod is assumed the state stays committed and the call returns KG_OK; otherwise every assumed pod is
 * undone (result KG_BATCH_ROLLED_BACK, CleanupAssumedPods) and the call still returns KG_OK, the per-pod
 * codes telling which pod failed and why. out_zone / out_minors (may be NULL): NUMA zone and GPU minors
 * of each assumed pod. KG_UNSUPPORTED when some pair needs the host path (the state is rolled back) or
 * when reservation views are uploaded (a Reserve into a view changes its restore). */
kg_status kg_batch_schedule(kg_snap* snap, kg_pods* pods, const int32_t* plan_node, uint32_t* out_result,
                            uint32_t* out_status, int32_t* out_zone, uint32_t* out_minors);

/* Timing of the dominant kernel with HIP events on the launch stream. */
kg_status kg_profile_enable(kg_ctx* ctx, int enable);
kg_status kg_profile_read(kg_ctx* ctx, double* total_ms, uint64_t* launches, int reset);

/* Multi-GPU node sharding over RCCL (one process per GPU). */
kg_status kg_shard_unique_id(uint8_t out[128]);
kg_status kg_shard_init(kg_ctx* ctx, const uint8_t id[128], int rank, int world);
/* Local select of the per-pod top k (1 <= k <= 4; k = 3 mirrors upstream
 * numberOfHighestScoredNodesToReport) + RCCL all-gather of the P x k per-shard keys + the same global
 * selectHost on every rank. out_keys (host, n_pods * k entries, descending per pod) may be NULL to leave
 * the result on the device (kg_result_keys reads it). */
kg_status kg_shard_select(kg_snap* snap, kg_pods* pods, uint32_t k, uint64_t* out_keys);

/* Host-only helpers (no device needed). */
/* Packed selection key: (total << 32) | (0xFFFFFFFF - node); max key = highest total, lowest index. */
uint64_t kg_make_key(int64_t total, uint32_t node);
int32_t kg_key_node(uint64_t key);    /* -1 for key 0 */
int64_t kg_key_total(uint64_t key);   /* -1 for key 0 */
/* Global selectHost over gathered per-shard keys: keys[shard][pod][k] -> out[pod][k]. */
kg_status kg_merge_keys(const uint64_t* keys, uint32_t n_shards, uint32_t n_pods, uint32_t k, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* KOORDGPU_H */
