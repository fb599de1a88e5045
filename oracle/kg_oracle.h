/*
 * kg_oracle.h — CPU restatement of koord-scheduler's Filter/Score/selectHost/Assume arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY. This is the parity oracle for the MI355X engine: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the checker or
 * as the timed CPU baseline. The product path (koordinator_amd/, libkoordgpu.so) never links or
 * calls it.
 *
 * Parity pinning: the reference is Go (no Go toolchain in this image), so no
 * oracle/_ref build exists. The restatement is pinned by the reference's own known-answer tests,
 * transcribed as fixtures under tests/golden/ (see tests/test_oracle_golden.py).
 */
#ifndef KG_ORACLE_H
#define KG_ORACLE_H

#include "../include/koordgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kgo_pair {
    uint32_t status;   /* KG_ST_* bits, 0 = feasible */
    int64_t s_nrf, s_la, s_numa;
    int64_t total;     /* -1 when infeasible */
    int32_t zone;      /* NUMA zone Reserve would allocate from, -1 = none */
} kgo_pair;

/* One (pod, node) evaluation of every enabled plugin. */
void kgo_eval_pair(const kg_config* cfg, const kg_node_columns* nodes, uint32_t node,
                   const kg_pod_columns* pods, uint32_t pod, kgo_pair* out);

/* Verify matrix, [n_pods][n_nodes]. */
void kgo_eval_verify(const kg_config* cfg, const kg_node_columns* nodes, uint32_t n_nodes,
                     const kg_pod_columns* pods, uint32_t n_pods, kg_verify_out* out);

/* selectHost with the build-defined deterministic tie-break: top-k packed keys per pod. */
void kgo_select(const kg_config* cfg, const kg_node_columns* nodes, uint32_t n_nodes, uint32_t index_base,
                const kg_pod_columns* pods, uint32_t n_pods, uint32_t k, uint64_t* keys);

/* Upstream-shaped CPU baseline: per pod, Filter over all nodes on n_workers threads with the
 * chunked parallelizer of pkg/util/parallelize/parallelism.go:29-49, then Score over the feasible
 * nodes the same way, then selectHost. keys: one key per pod. */
int kgo_select_parallel(const kg_config* cfg, const kg_node_columns* nodes, uint32_t n_nodes,
                        uint32_t index_base, const kg_pod_columns* pods, uint32_t n_pods,
                        int n_workers, uint64_t* keys);

/* Mutable copy of a snapshot for Assume/replay. */
typedef struct kgo_state kgo_state;
kgo_state* kgo_state_new(const kg_node_columns* cols, uint32_t n_nodes);
void kgo_state_free(kgo_state* st);
/* Column view of the state (pointers stay valid until kgo_state_free). */
void kgo_state_view(kgo_state* st, kg_node_columns* view);
/* Reserve of pod on node (a16: NodeInfo.AddPod, podAssignCache.assign, NUMA Reserve). */
/* Reserve: 0, or 1 when the NodeNUMAResource Reserve fails (BestEffort allocation; nothing applied). */
int kgo_assume(const kg_config* cfg, kgo_state* st, uint32_t node, const kg_pod_columns* pods, uint32_t pod);
/* Unreserve (reverse of kgo_assume with the zone chosen at Reserve). */
void kgo_forget(const kg_config* cfg, kgo_state* st, uint32_t node, const kg_pod_columns* pods, uint32_t pod,
                int32_t zone);
/* Reserve with the record its Unreserve gives back (kg_reserve_record; plugins of the state: NodeInfo, LoadAware,
 * NodeNUMAResource incl. cpusets, DeviceShare minors): 0, or 1 when the NodeNUMAResource Reserve fails. */
int kgo_reserve(const kg_config* cfg, kgo_state* st, uint32_t node, const kg_pod_columns* pods, uint32_t pod,
                kg_reserve_record* rec);
/* Unreserve of a kgo_reserve (NUMA amounts and cpuset CPUs of the record released, GPU minors given back). */
void kgo_unreserve(const kg_config* cfg, kgo_state* st, uint32_t node, const kg_pod_columns* pods, uint32_t pod,
                   const kg_reserve_record* rec);
/* One-pod-per-cycle scheduling with Assume between pods. out_reason (may be NULL): per pod, the OR of
 * the filter status bits over every node in that pod's cycle (the FitError diagnosis). */
void kgo_replay(const kg_config* cfg, kgo_state* st, uint32_t index_base, const kg_pod_columns* pods,
                uint32_t n_pods, int32_t* out_node, int64_t* out_total, uint32_t* out_reason);

/* Replay CPU baseline: each pod's cycle on the parallelizer (kgo_select_parallel), then its Reserve. */
int kgo_replay_parallel(const kg_config* cfg, kgo_state* st, uint32_t index_base, const kg_pod_columns* pods,
                        uint32_t n_pods, int n_workers, int32_t* out_node, int64_t* out_total);

/* Config-5 plugins (DeviceShare, Reservation, ElasticQuota): the tables the plugins read besides the
 * node columns. quotas: state at the start of the batch; views / infos: Reservation restore views. */
typedef struct kgo_ext {
    const kg_quota_columns* quotas;
    uint32_t n_quotas;
    const kg_rsv_view* views;
    uint32_t n_views;
    const kg_rsv_info* infos;
    uint32_t n_infos;
    const kg_rsv_dev* devs; /* GPU restore tables named by kg_rsv_view.dev_base / kg_rsv_info.dev */
    uint32_t n_devs;
    const kg_rsv_gpu* gpu;  /* DeviceShare restore inputs of GPU-holding reservations (replay / batch follow them) */
    uint32_t n_gpu;
} kgo_ext;

/* Verify matrix with every enabled plugin incl. KG_PLUGIN_DEV / RSV / QUOTA: raw Score values, totals
 * after NormalizeScore (DeviceShare, Reservation) and the weights. */
int kgo_ext_verify(const kg_config* cfg, const kg_node_columns* nodes, uint32_t n_nodes, const kg_pod_columns* pods,
                   uint32_t n_pods, const kgo_ext* ext, kg_verify_out* out);
int kgo_ext_select(const kg_config* cfg, const kg_node_columns* nodes, uint32_t n_nodes, uint32_t index_base,
                   const kg_pod_columns* pods, uint32_t n_pods, const kgo_ext* ext, uint32_t k, uint64_t* keys);
/* Replay with DeviceShare / ElasticQuota Reserve between pods; out_minors: GPU minors chosen per pod;
 * quota_*_out: final used / non-preemptible used [quota][KG_QUOTA_R]. -1 with KG_PLUGIN_RSV. */
int kgo_ext_replay(const kg_config* cfg, kgo_state* st, uint32_t index_base, const kg_pod_columns* pods,
                   uint32_t n_pods, const kgo_ext* ext, int32_t* out_node, int64_t* out_total, uint32_t* out_minors,
                   int64_t* quota_used_out, int64_t* quota_np_used_out, uint32_t* out_reason);
/* kgo_ext_replay with each cycle's nodes evaluated on `workers` threads (the CPU baseline of the config-5 replay). */
int kgo_ext_replay_parallel(const kg_config* c, kgo_state* st, uint32_t base, const kg_pod_columns* p, uint32_t np,
                            const kgo_ext* e, int32_t* out_node, int64_t* out_total, uint32_t* out_minors,
                            int64_t* quota_used_out, int64_t* quota_np_used_out, uint32_t* out_reason, int workers);
int64_t kgo_mem_bytes_to_ratio(int64_t bytes, int64_t total);
int64_t kgo_ext_pair_nominated(const kg_config* c, const kg_node_columns* n, uint32_t nn, uint32_t i,
                               const kg_pod_columns* p, uint32_t j, const kgo_ext* e);
/* Inline batch cycle of a planned job (batch/engine.go:92-294): per-pod KG_BATCH_* codes, status bits, NUMA
 * zone and GPU minors; a failed job leaves the state as it was. -1 with KG_PLUGIN_RSV. */
int kgo_batch_schedule(const kg_config* cfg, kgo_state* st, const kg_pod_columns* pods, uint32_t n_pods,
                       const kgo_ext* ext, const int32_t* plan_node, uint32_t* out_result, uint32_t* out_status,
                       int32_t* out_zone, uint32_t* out_minors, int64_t* quota_used_out, int64_t* quota_np_used_out);
/* Reserve / Unreserve with every config-5 plugin over one kgo_state (borrowed; it must outlive the session): the
 * session holds mutable copies of the reservation views / infos / GPU restore tables and inputs and the quota used,
 * which kgo_ext_reserve / kgo_ext_unreserve follow as kg_reserve / kg_unreserve do on the device. NULL when the
 * reservations hold GPUs without their restore inputs. */
typedef struct kgo_ext_session kgo_ext_session;
kgo_ext_session* kgo_ext_session_new(const kg_config* cfg, kgo_state* st, const kgo_ext* ext);
void kgo_ext_session_free(kgo_ext_session* x);
uint32_t kgo_ext_session_filter(kgo_ext_session* x, uint32_t node, const kg_pod_columns* pods, uint32_t pod);
int kgo_ext_reserve(kgo_ext_session* x, uint32_t node, const kg_pod_columns* pods, uint32_t pod, kg_reserve_record* rec);
int kgo_ext_unreserve(kgo_ext_session* x, uint32_t node, const kg_pod_columns* pods, uint32_t pod, kg_reserve_record* rec);
void kgo_ext_session_read(const kgo_ext_session* x, kg_rsv_view* views, kg_rsv_info* infos, kg_rsv_dev* devs,
                          int64_t* quota_used, int64_t* quota_np_used);
/* Node-sharded two-pass selection: per-shard NormalizeScore inputs (to be max / min all-reduced over
 * the shards), then the shard's top-k with the global inputs. */
int kgo_ext_shard_stats(const kg_config* cfg, const kg_node_columns* nodes, uint32_t n_nodes, uint32_t index_base,
                        const kg_pod_columns* pods, uint32_t n_pods, const kgo_ext* ext, uint32_t* dev_max,
                        uint32_t* rsv_max, uint64_t* pref);
int kgo_ext_shard_select(const kg_config* cfg, const kg_node_columns* nodes, uint32_t n_nodes, uint32_t index_base,
                         const kg_pod_columns* pods, uint32_t n_pods, const kgo_ext* ext, const uint32_t* dev_max,
                         const uint32_t* rsv_max, const uint64_t* pref, uint32_t k, uint64_t* keys);

/* cpuset accumulator (nodenumaresource/cpu_accumulator.go takeCPUs / takePreferredCPUs, kg_cpuset.c):
 * 0 = ok (out = the chosen CPUs), -1 = ErrNotEnoughCPUs, -2 = "failed to allocate cpus". */
/* Test hook: resourceManager.Allocate of pod j on node i under the NUMA affinity `mask` (0 = none): 0 with the CPUs of a
 * cpuset-binding pod and the NUMA split [resource][zone] (cpu milli, memory bytes), or 1 (resource_manager.go:197-262). */
/* Test hook: the NodeNUMAResource hint lists of pod j on node i (resourceManager.GetTopologyHints + filterProvidersHints)
 * for the requested resources, cpu then memory: per hint mask | 0x100 Preferred | 0x200 the unsatisfied nil hint of an
 * empty list. Returns the number of lists, -1 without NUMA nodes. */
int kgo_numa_hints(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j,
                   uint32_t policy, uint32_t out[2 * 16], int32_t len[2]);
int kgo_numa_allocate(const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j, uint32_t mask,
                      uint64_t cpus[4], int64_t al[2 * KG_MAX_ZONES]);
int kgo_take_cpus(const kg_cpu_topo* t, int max_ref, const uint64_t avail[4], const kg_cpu_alloc* allocated,
                  int needed, int bind_policy, int excl_policy, int strategy, uint64_t out[4]);
int kgo_take_preferred_cpus(const kg_cpu_topo* t, int max_ref, const uint64_t avail[4], const uint64_t preferred[4],
                            const kg_cpu_alloc* allocated, int needed, int bind_policy, int excl_policy, int strategy,
                            uint64_t out[4]);

/* DeviceShare as a NUMA hint provider (deviceshare/topology_hint.go:40-290) for pod j on node i: 0 = a hint
 * list (n_out entries of NUMA masks, Preferred, Score), 1 = no preference, 2 = the provider fails (*code =
 * KG_DEV_CODE_*). masks / pref / scores hold up to 15 entries. */
int kgo_gpu_numa_hints(const kg_config* cfg, const kg_node_columns* nodes, uint32_t node, const kg_pod_columns* pods,
                       uint32_t pod, int* n_out, uint32_t* masks, int* pref, int64_t* scores, uint32_t* code);
/* DeviceShare's Allocate under a NUMA affinity (bit per NUMA node id, 0 = nil): 0 + minors, or KG_DEV_CODE_*. */
uint32_t kgo_gpu_alloc_numa(const kg_config* cfg, const kg_node_columns* nodes, uint32_t node, const kg_pod_columns* pods,
                            uint32_t pod, uint32_t numa, uint32_t* minors);

/* Helpers shared with tests. */
int64_t kgo_amplify(int64_t origin, double ratio);
int64_t kgo_la_usage_percent(int64_t estimated, int64_t total);

#ifdef __cplusplus
}
#endif
#endif
