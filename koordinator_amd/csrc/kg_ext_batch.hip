// kg_ext_batch.hip — CDNA4 (gfx950) inline batch scheduling cycle of a whole-job plan (k_batch, and k_batch_coop
// with cpuset-binding pods). Split from kg_ext.hip so the translation units compile in parallel.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kg_cpuset_reserve.h"
#include "kg_ext.h"
#include "kg_ext_wave.h"
#include "kg_kernels.h"

namespace kg {

// Inline batch scheduling cycle of a whole-job plan (batch/engine.go:92-294 RunSchedulingCycle): the
// plan's pods are grouped by planned node; per group, in the caller's order, PreFilter (the ElasticQuota
// gate against the current used) + Filter on that node, then Reserve (NodeInfo, LoadAware, NUMA zone,
// GPU minors, quota used). The first failure in a group stops it: the later pods of the group get the
// same status (engine.go:188-192 "for k := j"), the earlier ones stay assumed until the host decides on
// cleanup. Groups hold disjoint nodes, so one lane per group runs them in parallel like the engine's
// parallelizer.Until over podRequestsByNode; with ElasticQuota on (a state every group shares) lane 0
// runs the groups in order instead, which keeps the quota verdicts deterministic.
template <bool EXACT, bool EXT>
__global__ __launch_bounds__(64) void k_batch(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones,
                                              DevRec* __restrict__ devs, ExtDev e, PodsDev pods,
                                              const uint32_t* __restrict__ grp_begin, const uint32_t* __restrict__ grp_pods,
                                              const uint32_t* __restrict__ grp_rec, uint32_t n_groups, bool serial,
                                              KCfg cfg, uint32_t* __restrict__ result, uint32_t* __restrict__ status,
                                              int32_t* __restrict__ zone_out, uint32_t* __restrict__ minors_out) {
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t g0 = serial ? 0u : lane, g1 = serial ? (lane == 0 ? n_groups : 0u) : min(lane + 1u, n_groups);
    for (uint32_t g = g0; g < g1; g++) {
        const uint32_t rec = grp_rec[g];
        int64_t* n = nodes[rec].v;
        uint32_t failed = 0;
        for (uint32_t t = grp_begin[g]; t < grp_begin[g + 1]; t++) {
            const uint32_t j = grp_pods[t];
            zone_out[j] = -1;
            minors_out[j] = 0;
            if (failed) {
                result[j] = KG_BATCH_SIBLING;
                status[j] = failed;
                continue;
            }
            const PodV q = load_pod(pods, j);
            uint32_t st;
            int32_t zone;
            uint32_t mask = 0;
            int32_t nom = -1;
            PodX qx{};
            if constexpr (EXT) {
                qx = load_podx(pods, j);
                uint32_t qst = 0;
                if ((cfg.plugins & KG_PLUGIN_QUOTA) && qx.quota >= 0 && (uint32_t)qx.quota < e.n_quotas)
                    qst = quota_gate(e.qlim[qx.quota], e.qstate[qx.quota], q, qx);
                const PairX r = eval_pair_ext<EXACT>(cfg, e, n, zones + rec, devs ? devs + rec : nullptr, rec, q, qx, qst);
                st = r.status;
                zone = r.zone;
                nom = r.nom;
                if (!st && !zone_reserve_fails(zone) && (cfg.plugins & KG_PLUGIN_DEV) && devs)
                    mask = dev_choose_site(cfg, e, n, zones + rec, devs + rec, pod_view(cfg, e, n, rec, qx), nom, qx, zone);
            } else {
                const PairOut r = eval_pair<EXACT>(cfg, n, zones + rec, q);
                st = r.status;
                zone = r.zone;
            }
            if (!st && zone_reserve_fails(zone)) st = zone_fail_status(zone);  // Reserve fails (engine.go:270-280)
            if (st) {
                failed = st;
                result[j] = KG_BATCH_FAILED;
                status[j] = st;
                continue;
            }
            apply_assume(cfg, n, zones + rec, q, zone, 1);
            if constexpr (EXT) {
                if ((cfg.plugins & KG_PLUGIN_QUOTA) && qx.quota >= 0 && (uint32_t)qx.quota < e.n_quotas) {
                    quota_add(e.qstate[qx.quota], q, qx, 1);
                    quota_add(e.qstate[e.n_quotas + qx.quota], q, qx, 1);
                }
                // Reservation.Reserve on the node's views (a group's node is its lane's alone), then DeviceShare's
                const bool rsv_on = (cfg.plugins & KG_PLUGIN_RSV) && n[N_RSV_CLASSES] != 0 && e.views;
                if (rsv_on) rsv_reserve_dev(e, n, zones + rec, rec, q, nom);
                dev_reserve_apply(cfg, e, n, rec, devs ? devs + rec : nullptr, mask, qx,
                                  (rsv_on && nom >= 0) ? (int32_t)e.infos[nom].rid : -1, 1);
            }
            result[j] = KG_BATCH_ASSUMED;
            status[j] = 0;
            zone_out[j] = zone;
            minors_out[j] = mask;
        }
    }
}

// The batch cycle with cpuset-binding pods (NodeNUMAResource Reserve -> resourceManager.Allocate: a take by the device
// accumulator, a whole wave in LDS): one workgroup of one wave runs the groups in order, every lane evaluates each pod
// (uniform work), the wave takes the CPUs, lane 0 applies the other Reserves. Same results as k_batch plus the cpusets
// (a failed take fails the pod and its group's later pods: ErrNotEnoughCPUs, zone code ZONE_CPUSET_FAIL).
template <bool EXACT>
__global__ __launch_bounds__(64) void k_batch_coop(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones,
                                                   DevRec* __restrict__ devs, ExtDev e, PodsDev pods,
                                                   const uint32_t* __restrict__ grp_begin,
                                                   const uint32_t* __restrict__ grp_pods,
                                                   const uint32_t* __restrict__ grp_rec, uint32_t n_groups, KCfg cfg,
                                                   kg_cpu_alloc* __restrict__ allocs, const kg_cpu_topo* __restrict__ topos,
                                                   uint32_t* __restrict__ result, uint32_t* __restrict__ status,
                                                   int32_t* __restrict__ zone_out, uint32_t* __restrict__ minors_out) {
    __shared__ CpusetLds L;
    const bool lead = threadIdx.x == 0;
    for (uint32_t g = 0; g < n_groups; g++) {
        const uint32_t rec = grp_rec[g];
        int64_t* n = nodes[rec].v;
        uint32_t failed = 0;
        for (uint32_t t = grp_begin[g]; t < grp_begin[g + 1]; t++) {
            const uint32_t j = grp_pods[t];
            if (failed) {
                if (lead) {
                    result[j] = KG_BATCH_SIBLING;
                    status[j] = failed;
                    zone_out[j] = -1;
                    minors_out[j] = 0;
                }
                continue;
            }
            const PodV q = load_pod(pods, j);
            const PodX qx = load_podx(pods, j);
            uint32_t qst = 0;
            if ((cfg.plugins & KG_PLUGIN_QUOTA) && qx.quota >= 0 && (uint32_t)qx.quota < e.n_quotas)
                qst = quota_gate(e.qlim[qx.quota], e.qstate[qx.quota], q, qx);
            const PairX r = eval_pair_ext<EXACT>(cfg, e, n, zones + rec, devs ? devs + rec : nullptr, rec, q, qx, qst);
            uint32_t st = r.status;
            const int32_t zone = r.zone;
            uint32_t mask = 0;
            if (!st && !zone_reserve_fails(zone) && (cfg.plugins & KG_PLUGIN_DEV) && devs)
                mask = dev_choose_site(cfg, e, n, zones + rec, devs + rec, pod_view(cfg, e, n, rec, qx), r.nom, qx, zone);
            if (!st && zone_reserve_fails(zone)) st = zone_fail_status(zone);  // Reserve fails (engine.go:270-280)
            __syncthreads();  // every lane has read the state the pod was evaluated on
            if (!st && (cfg.plugins & KG_PLUGIN_NUMA) && cpuset_bound_dev(zones[rec], q.flags, q.req_cpu) &&
                cpuset_reserve_wave(nodes, zones, allocs, topos, pods, j, rec, zone, L, nullptr) != 0)
                st = zone_fail_status(ZONE_CPUSET_FAIL);
            if (st) {
                failed = st;
                if (lead) {
                    result[j] = KG_BATCH_FAILED;
                    status[j] = st;
                    zone_out[j] = -1;
                    minors_out[j] = 0;
                }
                __syncthreads();
                continue;
            }
            if (lead) {
                apply_assume(cfg, n, zones + rec, q, zone, 1);
                if ((cfg.plugins & KG_PLUGIN_QUOTA) && qx.quota >= 0 && (uint32_t)qx.quota < e.n_quotas) {
                    quota_add(e.qstate[qx.quota], q, qx, 1);
                    quota_add(e.qstate[e.n_quotas + qx.quota], q, qx, 1);
                }
                const bool rsv_on = (cfg.plugins & KG_PLUGIN_RSV) && n[N_RSV_CLASSES] != 0 && e.views;
                if (rsv_on) rsv_reserve_dev(e, n, zones + rec, rec, q, r.nom);
                dev_reserve_apply(cfg, e, n, rec, devs ? devs + rec : nullptr, mask, qx,
                                  (rsv_on && r.nom >= 0) ? (int32_t)e.infos[r.nom].rid : -1, 1);
                result[j] = KG_BATCH_ASSUMED;
                status[j] = 0;
                zone_out[j] = zone;
                minors_out[j] = mask;
            }
            __syncthreads();  // lane 0's Reserve before the next pod's evaluation
        }
    }
}

// launcher

hipError_t launch_batch(NodeRec* nodes, ZoneRec* zones, DevRec* devs, const ExtDev& e, const PodsDev& pods,
                        const uint32_t* grp_begin, const uint32_t* grp_pods, const uint32_t* grp_rec, uint32_t n_groups,
                        bool ext, const KCfg& cfg, bool exact, uint32_t* result, uint32_t* status, int32_t* zone,
                        uint32_t* minors, hipStream_t s, kg_cpu_alloc* allocs, const kg_cpu_topo* topos) {
    if (n_groups == 0) return hipSuccess;
    if (allocs && topos) {  // cpuset-binding pods: the cooperative cycle
        if (exact)
            k_batch_coop<true><<<1, 64, 0, s>>>(nodes, zones, devs, e, pods, grp_begin, grp_pods, grp_rec, n_groups, cfg,
                                                allocs, topos, result, status, zone, minors);
        else
            k_batch_coop<false><<<1, 64, 0, s>>>(nodes, zones, devs, e, pods, grp_begin, grp_pods, grp_rec, n_groups, cfg,
                                                 allocs, topos, result, status, zone, minors);
        return hipGetLastError();
    }
    const bool serial = ext && (cfg.plugins & KG_PLUGIN_QUOTA);
    const dim3 grid(serial ? 1u : (n_groups + 63) / 64), block(64);
#define KG_BATCH(EX, XT)                                                                                              \
    k_batch<EX, XT><<<grid, block, 0, s>>>(nodes, zones, devs, e, pods, grp_begin, grp_pods, grp_rec, n_groups, serial, \
                                           cfg, result, status, zone, minors)
    if (exact && ext) KG_BATCH(true, true);
    else if (exact) KG_BATCH(true, false);
    else if (ext) KG_BATCH(false, true);
    else KG_BATCH(false, false);
#undef KG_BATCH
    return hipGetLastError();
}

}  // namespace kg
