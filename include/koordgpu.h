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

#define KG_ABI_VERSION 1

/* LoadAware resource vector width: the default vectorizer is {cpu, memory}
 * (pkg/scheduler/plugins/loadaware/helper.go:162-173, sorted by name). */
#define KG_LA_R 2
/* Scalar (extended) resources on the NodeResourcesFit path, e.g. kubernetes.io/batch-cpu,
 * kubernetes.io/batch-memory (config/manager/scheduler-config.yaml:21-31). */
#define KG_NSCALAR 2
/* NUMA zones per node supported on device (nodenumaresource/node_allocation.go:221-243). */
#define KG_MAX_ZONES 4

typedef enum kg_status {
    KG_OK = 0,
    KG_INVALID_ARG = 1,
    KG_DEVICE_ERROR = 2,
    KG_OOM = 3,
    KG_UNSUPPORTED = 4, /* feature not on the device path: caller runs the reference plugin */
    KG_NO_DEVICE = 5,
} kg_status;

/* Enabled plugins (kg_config.plugins). */
#define KG_PLUGIN_NRF 0x1u  /* upstream NodeResourcesFit: Fits + LeastAllocated score          */
#define KG_PLUGIN_LA 0x2u   /* LoadAwareScheduling (loadaware/load_aware.go)                     */
#define KG_PLUGIN_NUMA 0x4u /* NodeNUMAResource (nodenumaresource/plugin.go, scoring.go)         */

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
#define KG_POD_CPU_BIND 0x20u /* LSE/LSR prod pod requesting cpuset binding: not on the device path      */

/* Per-(pod,node) filter status bits (kg_verify_out.status). Plugin order follows the framework's
 * filter order: NodeResourcesFit, LoadAwareScheduling, NodeNUMAResource. */
#define KG_ST_NRF_PODS 0x1u   /* "Too many pods"                          */
#define KG_ST_NRF_CPU 0x2u    /* "Insufficient cpu"                       */
#define KG_ST_NRF_MEM 0x4u    /* "Insufficient memory"                    */
#define KG_ST_NRF_EPH 0x8u    /* "Insufficient ephemeral-storage"         */
#define KG_ST_NRF_SC0 0x10u   /* "Insufficient <scalar 0>"                */
#define KG_ST_NRF_SC1 0x20u   /* "Insufficient <scalar 1>"                */
#define KG_ST_NRF_MASK 0xFFu
#define KG_ST_LA_EXPIRED 0x100u /* ErrReasonNodeMetricExpired                        */
#define KG_ST_LA_CPU 0x200u     /* ErrReasonUsageExceedThreshold, cpu                */
#define KG_ST_LA_MEM 0x400u     /* ErrReasonUsageExceedThreshold, memory             */
#define KG_ST_LA_AGG 0x800u     /* set with LA_CPU/LA_MEM: "aggregated usage" reason */
#define KG_ST_LA_MASK 0xFF00u
#define KG_ST_NUMA_AMP_CPU 0x10000u  /* ErrInsufficientAmplifiedCPU                          */
#define KG_ST_NUMA_CONFLICT 0x20000u /* ErrNotMatchNUMATopology (UnschedulableAndUnresolvable) */
#define KG_ST_NUMA_NO_RES 0x40000u   /* "node(s) missing NUMA resources"                      */
#define KG_ST_NUMA_ALIGN 0x80000u    /* ErrNUMAHintCannotAligned                              */
#define KG_ST_NUMA_MASK 0xFF0000u
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
} kg_config;

/* Node snapshot, struct-of-arrays host columns, n_nodes entries each (caller-owned, copied). */
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
} kg_node_columns;

/* Mutable node state that Assume/Forget change; used to read a snapshot back after kg_replay. */
typedef struct kg_node_state {
    int64_t *req_cpu, *req_mem, *req_eph, *num_pods, *nz_cpu, *nz_mem;
    int64_t* sc_req[KG_NSCALAR];
    int64_t *la_fbase_np[KG_LA_R], *la_fbase_prod[KG_LA_R];
    int64_t *la_sbase_np[KG_LA_R], *la_sbase_prod[KG_LA_R];
    int64_t *zone_cpu_used[KG_MAX_ZONES], *zone_mem_used[KG_MAX_ZONES];
} kg_node_state;

/* Pending pods, struct-of-arrays host columns (caller-owned, copied). */
typedef struct kg_pod_columns {
    const int64_t *req_cpu, *req_mem, *req_eph; /* PodRequests: milli-cpu, bytes, bytes            */
    const int64_t* sc_req[KG_NSCALAR];
    const int64_t *nz_cpu, *nz_mem;             /* non-zero requests (100m / 200Mi defaults)        */
    const int64_t* la_est[KG_LA_R];             /* DefaultEstimator.EstimatePod (estimator/default_estimator.go:57-120) */
    const uint32_t* flags;                      /* KG_POD_*                                         */
    const uint32_t* numa_policy;                /* pod NUMA topology policy annotation, KG_NUMA_*   */
} kg_pod_columns;

/* Verify-mode outputs, [n_pods][n_nodes] row-major, caller-allocated host buffers (NULL = skip). */
typedef struct kg_verify_out {
    uint32_t* status;     /* KG_ST_* bits per plugin; 0 = feasible                         */
    int64_t* score_nrf;   /* NodeResourcesFit score (0 when infeasible or plugin disabled)  */
    int64_t* score_la;    /* LoadAwareScheduling score                                      */
    int64_t* score_numa;  /* NodeNUMAResource score                                         */
    int64_t* total;       /* Σ weight·score, -1 when infeasible                             */
    int8_t* numa_zone;    /* zone the NUMA Reserve would allocate from, -1 = none           */
} kg_verify_out;

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
/* Replace rows[i] (local index) with entry i of cols (each column has n entries). */
kg_status kg_snapshot_update_rows(kg_snap* snap, const uint32_t* rows, uint32_t n, const kg_node_columns* cols);
kg_status kg_snapshot_read_state(kg_snap* snap, kg_node_state* out);
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
/* Sequential scheduling of pods[0..n) one at a time with Assume applied on the device between pods
 * (the reference's one-pod-per-cycle semantics). out_node[i] = global node index or -1. */
kg_status kg_replay(kg_snap* snap, kg_pods* pods, int32_t* out_node, int64_t* out_total);
/* Reserve/Unreserve of pod `pod` (batch index) on local node `node`. */
kg_status kg_assume(kg_snap* snap, kg_pods* pods, uint32_t pod, uint32_t node);
kg_status kg_forget(kg_snap* snap, kg_pods* pods, uint32_t pod, uint32_t node, int32_t numa_zone);

/* Timing of the dominant kernel with HIP events on the launch stream. */
kg_status kg_profile_enable(kg_ctx* ctx, int enable);
kg_status kg_profile_read(kg_ctx* ctx, double* total_ms, uint64_t* launches, int reset);

/* Multi-GPU node sharding over RCCL (one process per GPU). */
kg_status kg_shard_unique_id(uint8_t out[128]);
kg_status kg_shard_init(kg_ctx* ctx, const uint8_t id[128], int rank, int world);
/* Local select (k=1) + RCCL all-gather of per-shard best keys + global selectHost.
 * out_keys (host, n_pods entries) may be NULL to leave the result on the device. */
kg_status kg_shard_select(kg_snap* snap, kg_pods* pods, uint64_t* out_keys);

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
