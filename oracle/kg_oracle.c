/*
 * kg_oracle.c — CPU restatement of the koord-scheduler Filter/Score hot path (parity oracle).
 *
 * TEST INFRASTRUCTURE ONLY (see kg_oracle.h). Every function follows the Go source it names with
 * Go's integer semantics (int64, truncating division) and IEEE float64 exactly where Go uses it.
 * Upstream k8s.io/kubernetes v1.35.6 pieces (not vendored in the reference, go.mod:70,295) are
 * restated from their published semantics as summarised in SURVEY.md §8(c-1).
 */
#define _GNU_SOURCE
#include "kg_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define MAX_NODE_SCORE 100 /* k8s.io/kube-scheduler framework.MaxNodeScore */

/* ---------------------------------------------------------------------------------------------- */
/* shared arithmetic                                                                              */

/* leastRequestedScore: nodenumaresource/least_allocated.go:50-58,
 * noderesourcefitplus/node_resource_fit_plus_utils.go:47-56 (same as upstream least_allocated.go). */
static int64_t least_requested_score(int64_t requested, int64_t capacity) {
    if (capacity == 0) return 0;
    if (requested > capacity) return 0;
    return ((capacity - requested) * MAX_NODE_SCORE) / capacity;
}

/* extension.Amplify: apis/extension/node_resource_amplification.go:170-175. */
int64_t kgo_amplify(int64_t origin, double ratio) {
    if (ratio <= 1) return origin;
    return (int64_t)ceil((double)origin * ratio);
}

/* filterNodeUsage usage: int64(math.Round(float64(estimated) / float64(total) * 100))
 * loadaware/load_aware.go:326. C round() is half away from zero like math.Round. */
int64_t kgo_la_usage_percent(int64_t estimated, int64_t total) {
    double q = (double)estimated / (double)total;
    double p = q * 100.0;
    return (int64_t)round(p);
}

/* Node quantities a Reservation restore changes for the pods of one owner class (kg_rsv_view):
 * NodeResourcesFit and NodeNUMAResource read the restored NodeInfo, LoadAware and DeviceShare do not. */
typedef struct kgo_over {
    int64_t req[KG_RSV_R]; /* cpu, memory, ephemeral-storage, scalar0, scalar1 */
    int64_t nz_cpu, nz_mem, num_pods;
} kgo_over;

#define N_REQ_CPU(n, i, ov) ((ov) ? (ov)->req[0] : (n)->req_cpu[i])
#define N_REQ_MEM(n, i, ov) ((ov) ? (ov)->req[1] : (n)->req_mem[i])
#define N_REQ_EPH(n, i, ov) ((ov) ? (ov)->req[2] : (n)->req_eph[i])
#define N_REQ_SC(n, k, i, ov) ((ov) ? (ov)->req[3 + (k)] : (n)->sc_req[k][i])
#define N_NZ_CPU(n, i, ov) ((ov) ? (ov)->nz_cpu : (n)->nz_cpu[i])
#define N_NZ_MEM(n, i, ov) ((ov) ? (ov)->nz_mem : (n)->nz_mem[i])
#define N_NUM_PODS(n, i, ov) ((ov) ? (ov)->num_pods : (n)->num_pods[i])

/* ---------------------------------------------------------------------------------------------- */
/* NodeResourcesFit (upstream v1.35.6)                                              */

static uint32_t nrf_filter(const kg_config* c, const kg_node_columns* n, uint32_t i, const kgo_over* ov,
                           const kg_pod_columns* p, uint32_t j) {
    uint32_t st = 0;
    /* fitsRequest: len(nodeInfo.Pods)+1 > allowedPodNumber */
    if (N_NUM_PODS(n, i, ov) + 1 > n->alloc_pods[i]) st |= KG_ST_NRF_PODS;
    /* (the all-zero early return yields the same verdict as the guarded checks below) */
    if (p->req_cpu[j] > 0 && p->req_cpu[j] > n->alloc_cpu[i] - N_REQ_CPU(n, i, ov)) st |= KG_ST_NRF_CPU;
    if (p->req_mem[j] > 0 && p->req_mem[j] > n->alloc_mem[i] - N_REQ_MEM(n, i, ov)) st |= KG_ST_NRF_MEM;
    if (p->req_eph[j] > 0 && p->req_eph[j] > n->alloc_eph[i] - N_REQ_EPH(n, i, ov)) st |= KG_ST_NRF_EPH;
    for (int k = 0; k < KG_NSCALAR; k++) {
        int64_t q = p->sc_req[k][j];
        if (q == 0) continue; /* "Skip in case request quantity is zero" */
        if ((c->nrf_ignored_scalars >> k) & 1u) continue; /* NodeResourcesFitArgs IgnoredResources(Groups) */
        if (q > n->sc_alloc[k][i] - N_REQ_SC(n, k, i, ov)) st |= (k == 0 ? KG_ST_NRF_SC0 : KG_ST_NRF_SC1);
    }
    return st;
}

/* resourceAllocationScorer.score + leastResourceScorer with NonZeroRequested for cpu/memory and
 * Requested for scalars; scalars the pod does not request are bypassed (0, 0); resources with
 * allocatable 0 are skipped (mirrors noderesourcefitplus/node_resource_fit_plus_utils.go:114-139). */
static int64_t most_requested_score(int64_t requested, int64_t capacity);

static int64_t nrf_score(const kg_config* c, const kg_node_columns* n, uint32_t i, const kgo_over* ov,
                         const kg_pod_columns* p, uint32_t j) {
    int64_t alloc[2 + KG_NSCALAR], req[2 + KG_NSCALAR], w[2 + KG_NSCALAR];
    alloc[0] = n->alloc_cpu[i];
    req[0] = N_NZ_CPU(n, i, ov) + p->nz_cpu[j];
    w[0] = c->nrf_w_cpu;
    alloc[1] = n->alloc_mem[i];
    req[1] = N_NZ_MEM(n, i, ov) + p->nz_mem[j];
    w[1] = c->nrf_w_mem;
    for (int k = 0; k < KG_NSCALAR; k++) {
        int64_t q = p->sc_req[k][j];
        if (q == 0) {
            alloc[2 + k] = 0;
            req[2 + k] = 0;
        } else {
            alloc[2 + k] = n->sc_alloc[k][i];
            req[2 + k] = N_REQ_SC(n, k, i, ov) + q;
        }
        w[2 + k] = c->nrf_w_sc[k];
    }
    int64_t score = 0, wsum = 0;
    for (int r = 0; r < 2 + KG_NSCALAR; r++) {
        if (w[r] == 0) continue; /* resource not in the scoring strategy */
        if (alloc[r] == 0) continue;
        /* per-resource strategy: LeastAllocated, or MostAllocated (mostRequestedScore,
         * noderesourcefitplus/node_resource_fit_plus_utils.go:36-45) */
        const int most = (c->nrf_most_allocated >> r) & 1u;
        score += (most ? most_requested_score(req[r], alloc[r]) : least_requested_score(req[r], alloc[r])) * w[r];
        wsum += w[r];
    }
    if (wsum == 0) return 0;
    return score / wsum;
}

/* ---------------------------------------------------------------------------------------------- */
/* LoadAwareScheduling                                                                             */

/* Plugin.Filter: loadaware/load_aware.go:150-220 + filterNodeUsage :316-345. */
static uint32_t la_filter(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                          uint32_t j) {
    if (p->flags[j] & KG_POD_DAEMONSET) return 0; /* :159-161 */
    uint32_t f = n->la_flags[i];
    int prod_pod = (f & KG_LA_PROD_THR) && (p->flags[j] & KG_POD_PROD); /* :164 */
    int is_agg = 0;
    const int64_t* const* thr;
    if (prod_pod) {
        thr = n->la_thr_prod;
    } else if (f & KG_LA_AGG_THR) {
        thr = n->la_thr_agg;
        is_agg = 1;
    } else {
        thr = n->la_thr_usage;
    }
    int empty = 1;
    for (int r = 0; r < KG_LA_R; r++)
        if (thr[r][i] != 0) empty = 0;
    if (empty) return 0; /* :175-177 */
    if (!(f & KG_LA_HAS_METRIC)) return 0; /* NotFound -> skip the node, :191-197 */
    if (c->la_filter_expired && (f & KG_LA_EXPIRED)) { /* :199-205 */
        if (!c->la_schedule_expired) return KG_ST_LA_EXPIRED;
        return 0;
    }
    if (f & KG_LA_NM_NIL) return 0; /* :207-210 */
    const int64_t* const* base = prod_pod ? n->la_fbase_prod : n->la_fbase_np;
    for (int r = 0; r < KG_LA_R; r++) {
        int64_t value = thr[r][i];
        if (value == 0) continue;
        int64_t total = n->la_alloc[r][i];
        if (total == 0) continue;
        int64_t estimated = base[r][i] + p->la_est[r][j];
        int64_t usage = kgo_la_usage_percent(estimated, total);
        if (usage <= value) continue;
        return (r == 0 ? KG_ST_LA_CPU : KG_ST_LA_MEM) | (is_agg ? KG_ST_LA_AGG : 0);
    }
    return 0;
}

/* loadAwareSchedulingScorer: load_aware.go:347-365; leastUsedScore :367-376. */
static int64_t la_scorer(int64_t dominant_w, const int64_t* w, const int64_t* used, const int64_t* alloc) {
    int64_t node_score = 0, dominant_score = 0, weight_sum = 0;
    if (dominant_w != 0) {
        dominant_score = MAX_NODE_SCORE;
        weight_sum = dominant_w;
    }
    for (int r = 0; r < KG_LA_R; r++) {
        int64_t s = least_requested_score(used[r], alloc[r]);
        node_score += s * w[r];
        weight_sum += w[r];
        if (dominant_score > s) dominant_score = s;
    }
    node_score += dominant_score * dominant_w;
    if (weight_sum <= 0) return 0;
    return node_score / weight_sum;
}

/* Plugin.Score: load_aware.go:235-292. */
static int64_t la_score(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                        uint32_t j) {
    if (!c->la_score_enabled) return 0;
    uint32_t f = n->la_flags[i];
    int prod_pod = c->la_score_prod && (p->flags[j] & KG_POD_PROD); /* :256 */
    if (!(f & KG_LA_HAS_METRIC)) return 0;                        /* :265-272 */
    if (f & KG_LA_EXPIRED) return 0;                              /* :273-275 */
    if (f & KG_LA_NM_NIL) return 0;                               /* :276-279 */
    const int64_t* const* base = prod_pod ? n->la_sbase_prod : n->la_sbase_np;
    int64_t used[KG_LA_R], alloc[KG_LA_R];
    for (int r = 0; r < KG_LA_R; r++) {
        used[r] = base[r][i] + p->la_est[r][j];
        alloc[r] = n->la_alloc[r][i];
    }
    return la_scorer(c->la_dominant_w, c->la_w, used, alloc);
}

/* ---------------------------------------------------------------------------------------------- */
/* NodeNUMAResource                                                                                */

/* leastResourceScorer / mostResourceScorer over {cpu, memory} with resources of allocatable 0 dropped
 * (nodenumaresource/scoring.go:222-238, least_allocated.go:30-58, most_allocated.go:30-62). */
static int64_t most_requested_score(int64_t requested, int64_t capacity) {
    if (capacity == 0) return 0;
    if (requested > capacity) requested = capacity;
    return (requested * MAX_NODE_SCORE) / capacity;
}

static int64_t numa_scorer(int most, int64_t w_cpu, int64_t w_mem, int64_t alloc_cpu, int64_t req_cpu, int64_t alloc_mem,
                           int64_t req_mem) {
    int64_t score = 0, wsum = 0;
    if (alloc_cpu != 0 && w_cpu != 0) {
        score += (most ? most_requested_score(req_cpu, alloc_cpu) : least_requested_score(req_cpu, alloc_cpu)) * w_cpu;
        wsum += w_cpu;
    }
    if (alloc_mem != 0 && w_mem != 0) {
        score += (most ? most_requested_score(req_mem, alloc_mem) : least_requested_score(req_mem, alloc_mem)) * w_mem;
        wsum += w_mem;
    }
    if (wsum == 0) return 0;
    return score / wsum;
}

/* the plugin's node score (ScoringStrategy) and its NUMA hint score (NUMAScoringStrategy) */
static int64_t numa_node_score(const kg_config* c, int64_t ac, int64_t rc, int64_t am, int64_t rm) {
    return numa_scorer(c->numa_most_allocated != 0, c->numa_w_cpu, c->numa_w_mem, ac, rc, am, rm);
}

static int64_t numa_hint_score(const kg_config* c, int64_t ac, int64_t rc, int64_t am, int64_t rm) {
    return numa_scorer(c->numa_hint_most_allocated != 0, c->numa_hint_w_cpu, c->numa_hint_w_mem, ac, rc, am, rm);
}

static int64_t sub_nonneg(int64_t a, int64_t b) { return a - b < 0 ? 0 : a - b; }

static uint32_t numa_merge_policy(uint32_t node_policy, uint32_t pod_policy, int* conflict) {
    /* mergeTopologyPolicy: nodenumaresource/util.go:58-66 */
    *conflict = 0;
    if (node_policy != KG_NUMA_NONE && pod_policy != KG_NUMA_NONE && pod_policy != node_policy) {
        *conflict = 1;
        return 0;
    }
    if (pod_policy != KG_NUMA_NONE) node_policy = pod_policy;
    return node_policy;
}

/* ---- NUMA topology manager: hints (resource_manager.go:529-657) and policy merge
 *      (frameworkext/topologymanager/policy*.go) for non-cpuset pods ---------------------------------- */

/* bitmask.IterateBitMasks order (pkg/util/bitmask/bitmask.go:206-221): by size, then lexicographic */
static const uint8_t NUMA_MASKS[KG_MAX_ZONES][15] = {
    {1},
    {1, 2, 3},
    {1, 2, 4, 3, 5, 6, 7},
    {1, 2, 4, 8, 3, 5, 9, 6, 10, 12, 7, 11, 13, 14, 15},
};
static const uint32_t NUMA_NMASKS[KG_MAX_ZONES] = {1, 3, 7, 15};

static int popcount32(uint32_t x) { return __builtin_popcount(x); }

typedef struct numa_zones {
    uint32_t Z, status;
    int64_t tot[2][KG_MAX_ZONES], used[2][KG_MAX_ZONES], avail[2][KG_MAX_ZONES];
} numa_zones;

static const kg_cpu_topo* cpu_topology(const kg_node_columns* n, uint32_t i);

/* CPUs of NUMA node z with an allocation (RefCount > 0): allocatedCPUs.CPUsInNUMANodes(z) */
static void cpus_allocated_by_zone(const kg_node_columns* n, uint32_t i, const kg_cpu_topo* t, int64_t cs[KG_MAX_ZONES]) {
    for (int z = 0; z < KG_MAX_ZONES; z++) cs[z] = 0;
    for (int c = 0; t && n->cpu_alloc && c < t->n_cpus; c++)
        if (n->cpu_alloc[i].ref[c] > 0 && t->numa[c] < KG_MAX_ZONES) cs[t->numa[c]]++;
}

/* NodeAllocation.getAvailableNUMANodeResources (node_allocation.go:221-243): a zone's allocated resources (its
 * allocatedResources record, numa_zone_status bit KG_ZONE_RECORD_SHIFT + z) on an amplified node count the zone's
 * cpuset CPUs amplified (allocated - cs * 1000 + Amplify(cs * 1000)); available = total - allocated, not below 0 */
static void numa_zones_load(const kg_node_columns* n, uint32_t i, numa_zones* x) {
    memset(x, 0, sizeof(*x));
    x->Z = n->numa_zones[i];
    x->status = n->numa_zone_status ? n->numa_zone_status[i] : 0;
    const double ratio = n->cpu_amp_ratio ? n->cpu_amp_ratio[i] : 1.0;
    const kg_cpu_topo* t = ratio > 1 ? cpu_topology(n, i) : NULL;
    int64_t cs[KG_MAX_ZONES];
    cpus_allocated_by_zone(n, i, t, cs);
    for (uint32_t z = 0; z < x->Z && z < KG_MAX_ZONES; z++) {
        x->tot[0][z] = n->zone_cpu[z][i];
        x->tot[1][z] = n->zone_mem[z][i];
        x->used[0][z] = n->zone_cpu_used[z][i];
        x->used[1][z] = n->zone_mem_used[z][i];
        if (t && ((x->status >> (KG_ZONE_RECORD_SHIFT + z)) & 1u))
            x->used[0][z] += kgo_amplify(cs[z] * 1000, ratio) - cs[z] * 1000;
        for (int r = 0; r < 2; r++) x->avail[r][z] = sub_nonneg(x->tot[r][z], x->used[r][z]); /* node_allocation.go:240 */
    }
}

/* tryBestToDistributeEvenly (resource_manager.go:264-318) of the pod's cpu / memory requests over the
 * zones of `mask`. The per-resource zone order comes from sort.Slice whose less(i, j) reads
 * totalAvailable by the positions i, j rather than by the zone ids being sorted (:276-279); sort.Slice
 * runs insertion sort for n <= 12, so the swaps depend only on the availability of zones 0..n-1. */
/* A cpuset-binding pod under a NUMA policy (ResourceOptions with requestCPUBind): what tryAllocateFromNode checks
 * of its CPUs under a hint (resource_manager.go:168-194 trimNUMANodeResources, :320-334 splitQuantity, :357-463
 * allocateCPUSet). cnt[z]: the available CPUs (RefCount < maxRefCount) of NUMA node z after
 * filterCPUsByRequiredCPUBindPolicy when the policy is required. */
typedef struct numa_bind {
    int required, full, cpc, needed;
    int64_t cnt[KG_MAX_ZONES];
} numa_bind;

static int numa_split(const numa_zones* x, uint32_t mask, const int64_t* req, const int* has,
                      int64_t alloc[2][KG_MAX_ZONES], const numa_bind* b) {
    int nodes[KG_MAX_ZONES], n = 0;
    for (uint32_t z = 0; z < x->Z; z++)
        if ((mask >> z) & 1u) nodes[n++] = (int)z;
    memset(alloc, 0, sizeof(int64_t) * 2 * KG_MAX_ZONES);
    for (int r = 0; r < 2; r++) {
        if (!has[r]) continue;
        int s[KG_MAX_ZONES];
        memcpy(s, nodes, sizeof(nodes));
        for (int a = 1; a < n; a++)
            for (int b = a; b > 0 && x->avail[r][b] < x->avail[r][b - 1]; b--) {
                int t = s[b];
                s[b] = s[b - 1];
                s[b - 1] = t;
            }
        int64_t q = req[r];
        for (int t = 0; t < n; t++) {
            int64_t split = q / (n - t); /* splitQuantity :320-334 (milli-cpu / bytes) */
            if (r == 0 && b) {           /* requestCPUBind: whole CPUs of quantity.Value() (rounded up) */
                const int64_t v = (q + 999) / 1000;
                split = b->required && b->full ? (v / b->cpc) / (n - t) * b->cpc * 1000 : v / (n - t) * 1000;
            }
            int64_t av = x->avail[r][s[t]];
            int64_t got = av > split ? split : av; /* allocateRes :336-355 */
            if (got != 0) {
                alloc[r][s[t]] = got;
                q -= got;
            }
        }
        if (q != 0) return 0; /* "Insufficient NUMA <resource>" */
    }
    return 1;
}

/* allocateCPUSet over the allocated NUMA nodes (resource_manager.go:391-429): on each, min(its available CPUs,
 * allocated cpu / 1000) CPUs (takePreferredCPUs takes exactly that many when they are available); together they must
 * number numCPUsNeeded (ErrNotEnoughCPUs), and a required FullPCPUs policy needs whole cores on each
 * (satisfiedRequiredCPUBindPolicy :452-460; the filtered CPUs hold whole free cores, so a take of a multiple of
 * CPUsPerCore is whole cores). 0, KG_ST_NUMA_CPUS or KG_ST_NUMA_CPU_BIND. */
static uint32_t numa_bind_check(const numa_bind* b, const int64_t al[2][KG_MAX_ZONES], uint32_t Z) {
    int64_t sum = 0;
    int partial = 0;
    for (uint32_t z = 0; z < Z && z < KG_MAX_ZONES; z++) {
        if (al[0][z] == 0 && al[1][z] == 0) continue; /* not an allocated NUMA node */
        int64_t k = al[0][z] / 1000;
        if (b->cnt[z] < k) k = b->cnt[z];
        sum += k;
        partial |= b->required && b->full && (k % b->cpc) != 0;
    }
    if (sum != b->needed) return KG_ST_NUMA_CPUS;
    return partial ? KG_ST_NUMA_CPU_BIND : 0u;
}

typedef struct numa_hint {
    uint32_t mask; /* 0 = nil affinity */
    int pref, unsat;
    int64_t score;
} numa_hint;

typedef struct numa_lists {
    int n_lists;
    int len[2];
    numa_hint h[2][15];
    int reasons;
} numa_lists;

/* generateResourceHints + filterProvidersHints: per requested resource (cpu, then memory) the hints of
 * the masks whose allocation succeeds and that avoid zones lacking the resource; Preferred = narrowest
 * size, or every hint under Restricted. A requested resource without hints contributes one unsatisfied
 * nil hint and a reason (policy.go:166-173). */
static void numa_hints(const kg_config* c, const numa_zones* x, const int64_t* req, const int* has, uint32_t policy,
                       numa_lists* L, const numa_bind* b, int64_t score_cpu) {
    const uint32_t Z = x->Z;
    uint32_t lack[2] = {0, 0};
    for (uint32_t z = 0; z < Z; z++)
        for (int r = 0; r < 2; r++)
            if (x->avail[r][z] == 0) lack[r] |= 1u << z;
    int minsize[2] = {(int)Z, (int)Z};
    uint32_t okm[2] = {0, 0};
    int64_t score[15];
    const uint8_t* masks = NUMA_MASKS[Z - 1];
    for (uint32_t k = 0; k < NUMA_NMASKS[Z - 1]; k++) {
        uint32_t m = masks[k];
        int64_t T[2] = {0, 0}, A[2] = {0, 0};
        for (uint32_t z = 0; z < Z; z++)
            if ((m >> z) & 1u)
                for (int r = 0; r < 2; r++) {
                    T[r] += x->tot[r][z];
                    A[r] += x->avail[r][z];
                }
        /* numaScorer over requested = SubtractWithNonNegativeResult(total, available) */
        /* (the pod's requests as the options hold them: a cpuset-binding pod's cpu amplified, score_cpu) */
        score[k] = numa_hint_score(c, T[0], sub_nonneg(T[0], A[0]) + score_cpu, T[1], sub_nonneg(T[1], A[1]) + req[1]);
        int64_t al[2][KG_MAX_ZONES];
        if (!numa_split(x, m, req, has, al, b)) continue;
        if (b && numa_bind_check(b, al, Z)) continue;
        for (int r = 0; r < 2; r++) {
            if (!has[r] || (m & lack[r])) continue;
            if (popcount32(m) < minsize[r]) minsize[r] = popcount32(m);
            okm[r] |= 1u << k;
        }
    }
    L->n_lists = 0;
    L->reasons = 0;
    for (int r = 0; r < 2; r++) {
        if (!has[r]) continue;
        int li = L->n_lists++;
        int len = 0;
        for (uint32_t k = 0; k < NUMA_NMASKS[Z - 1]; k++) {
            if (!((okm[r] >> k) & 1u)) continue;
            numa_hint* h = &L->h[li][len++];
            h->mask = masks[k];
            h->pref = popcount32(masks[k]) == minsize[r] || policy == KG_NUMA_RESTRICTED;
            h->unsat = 0;
            h->score = score[k];
        }
        if (len == 0) {
            L->reasons++;
            numa_hint* h = &L->h[li][len++];
            h->mask = 0;
            h->pref = 0;
            h->unsat = 1;
            h->score = 0;
        }
        L->len[li] = len;
    }
}

/* checkExclusivePolicy with NumaTopologyExclusiveRequired (policy.go:73-93) */
static int numa_excl_ok(uint32_t mask, uint32_t status) {
    if (popcount32(mask) > 1) {
        for (uint32_t z = 0; z < KG_MAX_ZONES; z++)
            if (((mask >> z) & 1u) && ((status >> (2 * z)) & 3u) == 1u) return 0;
        return 1;
    }
    uint32_t z = (uint32_t)__builtin_ctz(mask);
    return ((status >> (2 * z)) & 3u) != 2u;
}

/* mergePermutation + the bestHint update of mergeFilteredHints (policy.go:98-137,198-260) */
static void numa_merge_one(uint32_t all, int excl, uint32_t status, const numa_hint* perm, int np, numa_hint* best) {
    uint32_t merged = all, first = 0;
    int pref = 1, unsat = 0, naff = 0, maxc = 0;
    for (int t = 0; t < np; t++) {
        const numa_hint* v = &perm[t];
        if (v->mask) {
            if (naff == 0) first = v->mask;
            else if (v->mask != first) pref = 0;
            naff++;
            merged &= v->mask;
            if (popcount32(v->mask) > maxc) maxc = popcount32(v->mask);
        }
        if (!v->pref) pref = 0;
        if (v->unsat) unsat = 1;
    }
    int satisfied = (naff == 0 || maxc == popcount32(merged)) && !unsat;
    if (popcount32(merged) == 0) return;
    if (excl && !numa_excl_ok(merged, status)) pref = 0;
    int64_t score = 0;
    for (int t = 0; t < np; t++)
        if (perm[t].mask && perm[t].mask == merged) score += perm[t].score;
    numa_hint m = {merged, pref, !satisfied, score};
    if (m.pref && !best->pref) {
        *best = m;
        return;
    }
    if (!m.pref && best->pref) return;
    int cm = popcount32(m.mask), cb = popcount32(best->mask);
    int narrower = cm == cb ? m.mask < best->mask : cm < cb;
    if (!narrower) {
        if (cm == cb && m.score > best->score) *best = m;
        return;
    }
    *best = m;
}

/* The DeviceShare hint provider's answer for one (GPU pod, node) pair (deviceshare/topology_hint.go:40-290):
 * fail = the provider's status is not a success (code: its KG_ST_* bits, a DeviceShare reason); nopref = no
 * preference (no Device object, no GPU with a NUMA node: a single preferred nil hint); else the "gpu" hint list
 * in IterateBitMasks order over the GPUs' NUMA node ids. */
typedef struct gpu_hints {
    int fail, nopref, n;
    uint32_t code;
    uint32_t mask[15];
    int pref[15];
    int64_t score[15];
} gpu_hints;

/* Policy Merge (policy_single_numa_node.go:69-90, policy_restricted.go:50-62, policy_best_effort.go:48-60).
 * Returns 0 admitted (affinity mask in *mask_out, 0 = none), else a KG_ST_NUMA_* reason. Permutations
 * run cpu-major, then memory, then the DeviceShare provider's "gpu" list (providers in plugin order,
 * NodeNUMAResource before DeviceShare); the reference iterates Go map order over a provider's resources,
 * which matters only when two merged hints tie on preference, width and score (parity unpinned there).
 * gh (nullable): the DeviceShare provider's list of a GPU pod (not failed). */
static uint32_t numa_admit(const kg_config* c, const numa_zones* x, const int64_t* req, const int* has, uint32_t policy,
                           int excl, uint32_t* mask_out, const gpu_hints* gh, const numa_bind* b, int64_t score_cpu) {
    numa_lists L;
    numa_hints(c, x, req, has, policy, &L, b, score_cpu);
    const uint32_t all = (1u << x->Z) - 1u;
    *mask_out = 0;
    if (L.reasons && policy != KG_NUMA_BEST_EFFORT) return KG_ST_NUMA_UNSATISFIED;
    /* the third list: the provider's hints, or its "no preference" hint (filterProvidersHints, policy.go:145-152) */
    numa_hint G[15];
    int ng = 0;
    if (gh) {
        if (gh->nopref) {
            G[ng].mask = 0;
            G[ng].pref = 1;
            G[ng].unsat = 0;
            G[ng++].score = 0;
        } else {
            for (int t = 0; t < gh->n; t++) {
                G[ng].mask = gh->mask[t];
                G[ng].pref = gh->pref[t];
                G[ng].unsat = 0;
                G[ng++].score = gh->score[t];
            }
        }
    }
    if (policy == KG_NUMA_SINGLE_NODE && gh) { /* filterSingleNumaHints on the gpu list too */
        int w = 0;
        for (int t = 0; t < ng; t++)
            if (G[t].pref && (G[t].mask == 0 || popcount32(G[t].mask) == 1)) G[w++] = G[t];
        ng = w;
    }
    if (policy == KG_NUMA_SINGLE_NODE) { /* filterSingleNumaHints */
        for (int li = 0; li < L.n_lists; li++) {
            int w = 0;
            for (int t = 0; t < L.len[li]; t++) {
                numa_hint h = L.h[li][t];
                if (h.pref && (h.mask == 0 || popcount32(h.mask) == 1)) L.h[li][w++] = h;
            }
            L.len[li] = w;
        }
    }
    numa_hint best = {all, 0, 0, 0};
    /* iterateAllProviderTopologyHints (policy.go:262-299) over the lists [cpu,] [memory,] [gpu] */
    const numa_hint* lists[3];
    int lens[3], nl = 0;
    for (int li = 0; li < L.n_lists; li++) {
        lists[nl] = L.h[li];
        lens[nl++] = L.len[li];
    }
    if (gh) {
        lists[nl] = G;
        lens[nl++] = ng;
    }
    if (nl == 0) {
        /* no NUMA resource requested: the providers' "no preference" hints */
        numa_merge_one(all, excl, x->status, NULL, 0, &best);
    } else {
        int idx[3] = {0, 0, 0};
        int empty = 0;
        for (int t = 0; t < nl; t++) empty |= lens[t] == 0;
        while (!empty) {
            numa_hint perm[3];
            for (int t = 0; t < nl; t++) perm[t] = lists[t][idx[t]];
            numa_merge_one(all, excl, x->status, perm, nl, &best);
            int t = nl - 1;
            while (t >= 0 && ++idx[t] == lens[t]) idx[t--] = 0;
            if (t < 0) break;
        }
    }
    if (policy == KG_NUMA_BEST_EFFORT) {
        *mask_out = best.unsat ? all : best.mask;
        return 0;
    }
    if (!best.pref) return KG_ST_NUMA_ALIGN;
    *mask_out = (policy == KG_NUMA_SINGLE_NODE && best.mask == all) ? 0 : best.mask;
    return 0;
}

/* zone code of an allocation: -1 none, the zone for one zone, 0x40 | mask for several; a BestEffort Reserve
 * that fails: KGO_ZONE_RESERVE_FAIL | KG_ST_NUMA_INSUF_* >> 12 (the ABI's numa_zone codes) */
#define KGO_ZONE_RESERVE_FAIL 0x20
static int zone_fails(int32_t z) { return z >= 0x20 && z < 0x40; }
static uint32_t zone_fail_bits(int32_t z) {
    if (z & 0x10) /* DeviceShare in the Reserve's topology manager: its code, 0xF = Reservation(s) Insufficient gpu devices */
        return ((z & 0xF) == 0xF) ? KG_ST_DEV_RSV : KG_ST_DEV_MAKE((uint32_t)z & 0xFu);
    return (((uint32_t)z & 7u) << 12) | ((z & 8) ? KG_ST_NUMA_CPUS : 0u);
}
/* the cpuset accumulator finds no CPUs at Reserve (resource_manager.go:385,427 ErrNotEnoughCPUs) */
#define KGO_ZONE_CPUSET_FAIL (KGO_ZONE_RESERVE_FAIL | 8)
static int32_t numa_code(uint32_t mask) {
    if (!mask) return -1;
    return popcount32(mask) == 1 ? (int32_t)__builtin_ctz(mask) : (int32_t)(0x40u | mask);
}

static uint32_t numa_code_mask(int32_t code) {
    if (code < 0) return 0;
    return code >= 0x40 ? (uint32_t)code & 0xFu : 1u << code;
}

/* ---- cpuset binding (plugin.go:396-440, resource_manager.go:357-499,659-722) ---------------------- */

static const kg_cpu_topo* cpu_topology(const kg_node_columns* n, uint32_t i) {
    if (!n->cpu_topo || !n->cpu_topos || n->cpu_topo[i] < 0 || (uint32_t)n->cpu_topo[i] >= n->n_cpu_topos) return NULL;
    const kg_cpu_topo* t = &n->cpu_topos[n->cpu_topo[i]];
    /* CPUTopology.IsValid (cpu_topology.go:79-81) */
    return (t->n_sockets && t->n_nodes && t->n_cores && t->n_cpus) ? t : NULL;
}

static int cpu_max_ref(const kg_node_columns* n, uint32_t i) {
    const int m = n->cpu_max_ref ? n->cpu_max_ref[i] : 1;
    return m < 1 ? 1 : m;
}

/* NodeAllocation.getAvailableCPUs (node_allocation.go:192-220), no reserved / preferred CPUs */
static void cpu_available(const kg_node_columns* n, uint32_t i, const kg_cpu_topo* t, uint64_t m[4]) {
    memset(m, 0, 4 * sizeof(uint64_t));
    const int mr = cpu_max_ref(n, i);
    for (int c = 0; c < t->n_cpus; c++) {
        const int ref = n->cpu_alloc ? n->cpu_alloc[i].ref[c] : 0;
        if (ref < mr) m[c >> 6] |= 1ull << (c & 63);
    }
}

static int mask_count(const uint64_t m[4]) {
    return __builtin_popcountll(m[0]) + __builtin_popcountll(m[1]) + __builtin_popcountll(m[2]) + __builtin_popcountll(m[3]);
}

/* filterCPUsByRequiredCPUBindPolicy (resource_manager.go:659-699): FullPCPUs keeps the cores whose every CPU
 * is available, SpreadByPCPUs the smallest available CPU of each core */
static void cpu_filter_required(const kg_cpu_topo* t, uint32_t policy, uint64_t m[4]) {
    const int cpc = t->n_cpus / t->n_cores;
    int cnt[KG_MAX_CPUS] = {0}, first[KG_MAX_CPUS];
    for (int k = 0; k < KG_MAX_CPUS; k++) first[k] = -1;
    for (int c = 0; c < t->n_cpus; c++)
        if ((m[c >> 6] >> (c & 63)) & 1ull) {
            cnt[t->core[c]]++;
            if (first[t->core[c]] < 0) first[t->core[c]] = c;
        }
    uint64_t o[4] = {0, 0, 0, 0};
    for (int c = 0; c < t->n_cpus; c++) {
        if (!((m[c >> 6] >> (c & 63)) & 1ull)) continue;
        const int keep = policy == KG_CPU_BIND_FULL_PCPUS ? cnt[t->core[c]] == cpc : first[t->core[c]] == c;
        if (keep) o[c >> 6] |= 1ull << (c & 63);
    }
    memcpy(m, o, sizeof(o));
}

/* the pod's resolved bind policy on node i (getCPUBindPolicy, util.go:101-119): required or preferred, the
 * node policy overriding both; *required tells whether it is required */
static uint32_t cpu_bind_policy(const kg_pod_columns* p, uint32_t j, uint32_t node_bind, int* required) {
    const uint32_t pol = (p->flags[j] >> KG_POD_CPU_POLICY_SHIFT) & 3u;
    const int pod_req = (p->flags[j] & KG_POD_CPU_REQUIRED) != 0;
    *required = pod_req;
    if (pod_req) return pol;
    if (node_bind == KG_NODE_CPU_BIND_SPREAD_BY_PCPUS) {
        *required = 1;
        return KG_CPU_BIND_SPREAD_BY_PCPUS;
    }
    if (node_bind == KG_NODE_CPU_BIND_FULL_PCPUS_ONLY) {
        *required = 1;
        return KG_CPU_BIND_FULL_PCPUS;
    }
    return pol;
}

/* resourceManager.allocateCPUSet on NUMA policy None (no hint): 0 and the CPUs, or -1 */
static int cpuset_allocate(const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j, uint32_t node_bind,
                           uint64_t out[4]) {
    const kg_cpu_topo* t = cpu_topology(n, i);
    if (!t) return -1;
    int required;
    const uint32_t bind = cpu_bind_policy(p, j, node_bind, &required);
    uint64_t avail[4];
    cpu_available(n, i, t, avail);
    if (required) cpu_filter_required(t, bind, avail);
    const int needed = (int)(p->req_cpu[j] / 1000);
    if (mask_count(avail) < needed) return -1; /* ErrNotEnoughCPUs */
    const uint32_t excl = (p->flags[j] >> KG_POD_CPU_EXCL_SHIFT) & 3u;
    const uint32_t strategy = n->cpu_strategy ? n->cpu_strategy[i] : KG_NUMA_MOST_ALLOCATED;
    if (kgo_take_cpus(t, cpu_max_ref(n, i), avail, n->cpu_alloc ? &n->cpu_alloc[i] : NULL, needed, (int)bind, (int)excl,
                      (int)strategy, out))
        return -1;
    if (required) { /* satisfiedRequiredCPUBindPolicy (resource_manager.go:701-722) */
        int cores = 0;
        uint8_t seen[KG_MAX_CPUS] = {0};
        for (int c = 0; c < t->n_cpus; c++)
            if (((out[c >> 6] >> (c & 63)) & 1ull) && !seen[t->core[c]]) {
                seen[t->core[c]] = 1;
                cores++;
            }
        const int size = mask_count(out), cpc = t->n_cpus / t->n_cores;
        if (bind == KG_CPU_BIND_FULL_PCPUS ? cores * cpc != size : cores != size) return -1;
    }
    return 0;
}

/* the cpuset part of Filter for a pod that binds CPUs on node i (plugin.go:396-440). Under a NUMA policy the CPUs
 * are part of every allocation the topology manager tries (numa_bind); under None a required policy allocates in
 * Filter (tryAllocateFromNode), a preferred one only at Reserve: *zone_out = KGO_ZONE_CPUSET_FAIL when that fails */
static uint32_t cpuset_filter(const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j, uint32_t policy,
                              uint32_t node_bind, int32_t* zone_out) {
    const kg_cpu_topo* t = cpu_topology(n, i);
    if (!t) return KG_ST_NUMA_CPU_TOPO; /* ErrInvalidCPUTopology */
    const uint32_t pod_pol = (p->flags[j] >> KG_POD_CPU_POLICY_SHIFT) & 3u;
    const int pod_req = (p->flags[j] & KG_POD_CPU_REQUIRED) != 0;
    uint32_t required = pod_req ? pod_pol : KG_CPU_BIND_NONE;
    if (node_bind == KG_NODE_CPU_BIND_FULL_PCPUS_ONLY) required = KG_CPU_BIND_FULL_PCPUS;
    else if (node_bind == KG_NODE_CPU_BIND_SPREAD_BY_PCPUS) required = KG_CPU_BIND_SPREAD_BY_PCPUS;
    if (pod_req && pod_pol != required) return KG_ST_NUMA_CPU_BIND; /* ErrCPUBindPolicyConflict */
    const int64_t needed = p->req_cpu[j] / 1000;
    if (required == KG_CPU_BIND_FULL_PCPUS && needed % (t->n_cpus / t->n_cores) != 0)
        return KG_ST_NUMA_CPU_BIND; /* ErrSMTAlignmentError */
    /* the allocation from here on reads the restore of NUMA / cpuset-holding reservations (plugin.go:428-439,
     * reservation.go:188-262): not restated (kg_node_columns.rsv_numa) */
    if (n->rsv_numa && n->rsv_numa[i]) return KG_ST_UNSUPPORTED;
    if (policy != KG_NUMA_NONE) return 0;
    uint64_t out[4];
    if (required != KG_CPU_BIND_NONE) {
        if (cpuset_allocate(n, i, p, j, node_bind, out)) return KG_ST_NUMA_CPUS; /* tryAllocateFromNode */
        return 0;
    }
    /* no allocation in Filter; the Reserve's allocateCPUSet fails (ErrNotEnoughCPUs) when the node has too few CPUs */
    if (cpuset_allocate(n, i, p, j, node_bind, out)) *zone_out = KGO_ZONE_CPUSET_FAIL;
    return 0;
}

/* numa_bind of a cpuset-binding pod on node i (getCPUBindPolicy, util.go:101-119; getAvailableCPUs and
 * filterCPUsByRequiredCPUBindPolicy per NUMA node) */
static void numa_bind_load(const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j, uint32_t node_bind,
                           numa_bind* b) {
    const kg_cpu_topo* t = cpu_topology(n, i);
    const uint32_t bind = cpu_bind_policy(p, j, node_bind, &b->required);
    b->full = bind == KG_CPU_BIND_FULL_PCPUS;
    b->cpc = t->n_cores ? t->n_cpus / t->n_cores : 1;
    b->needed = (int)(p->req_cpu[j] / 1000);
    uint64_t avail[4];
    cpu_available(n, i, t, avail);
    if (b->required) cpu_filter_required(t, bind, avail);
    for (int z = 0; z < KG_MAX_ZONES; z++) b->cnt[z] = 0;
    for (int c = 0; c < t->n_cpus; c++)
        if (((avail[c >> 6] >> (c & 63)) & 1ull) && t->numa[c] < KG_MAX_ZONES) b->cnt[t->numa[c]]++;
}

/* DeviceShare as a NUMA hint provider for a GPU pod (defined with the GPU allocator below). The site: the pair's
 * reservation view (v, its tables in e) or none. */
typedef struct numa_gpu_out {
    const struct kgo_ext* e;
    const kg_rsv_view* v;
    int done;      /* the topology manager admitted the pod with DeviceShare's Allocate: its Filter passes */
    uint32_t mask; /* the stored affinity (0 = nil) DeviceShare's Score and Reserve then use */
} numa_gpu_out;
static void gpu_numa_hints(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j,
                           const numa_gpu_out* gx, gpu_hints* h);
static uint32_t gpu_alloc_site(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                               uint32_t j, const numa_gpu_out* gx, uint32_t numa, uint32_t* minors);
#define KGO_ZONE_GPU_FAIL 0x30
/* the zone code of a DeviceShare failure in the Reserve's topology manager: its code, 0xF for "Reservation(s)
 * Insufficient gpu devices" */
static int32_t zone_gpu_fail(uint32_t st) {
    return KGO_ZONE_GPU_FAIL | (int32_t)((st & KG_ST_DEV_RSV) ? 0xFu : KG_ST_DEV_CODE(st));
}

/* Filter (plugin.go:363-459) + Score (scoring.go:67-151,153-199) of one pair. gx (nullable): a GPU pod on a
 * node with a Device object (DeviceShare joins the topology manager: topology_hint.go:40-290, manager.go:65-154). */
static uint32_t numa_eval(const kg_config* c, const kg_node_columns* n, uint32_t i, const kgo_over* ov,
                          const kg_pod_columns* p, uint32_t j, int64_t* score_out, int32_t* zone_out, numa_gpu_out* gx) {
    *score_out = 0;
    *zone_out = -1;
    if (gx) {
        gx->done = 0;
        gx->mask = 0;
    }
    if (p->flags[j] & KG_POD_NUMA_SKIP) return 0; /* PreFilter Skip: no Filter, no Score */
    int conflict;
    uint32_t policy = numa_merge_policy(n->numa_policy[i], p->numa_policy[j], &conflict);
    if (conflict) return KG_ST_NUMA_CONFLICT; /* plugin.go:377-381 */
    int cpu_bind = (p->flags[j] & KG_POD_CPU_BIND) != 0;
    double ratio = n->cpu_amp_ratio[i];
    int64_t pod_cpu = p->req_cpu[j];
    /* requestCPUBind (util.go:121-138): a node CPU bind policy binds every pod with a cpu request */
    const uint32_t node_bind = n->cpu_bind_policy ? n->cpu_bind_policy[i] : KG_NODE_CPU_BIND_NONE;
    if (!cpu_bind && pod_cpu != 0 && node_bind != KG_NODE_CPU_BIND_NONE) {
        if (pod_cpu % 1000 != 0) return KG_ST_NUMA_CPU_BIND; /* ErrInvalidRequestedCPUs */
        cpu_bind = 1;
    }
    /* filterAmplifiedCPUs: plugin.go:461-498; a cpuset-binding pod's request is amplified too (:477-479) */
    if (pod_cpu != 0 && ratio > 1) {
        int64_t allocated = n->cpuset_alloc_milli[i];
        int64_t requested = N_REQ_CPU(n, i, ov);
        if (requested >= allocated && allocated > 0) {
            requested = requested - allocated;
            requested += kgo_amplify(allocated, ratio);
        }
        const int64_t need = cpu_bind ? kgo_amplify(pod_cpu, ratio) : pod_cpu;
        if (need > n->alloc_cpu[i] - requested) return KG_ST_NUMA_AMP_CPU;
    }
    if (cpu_bind) {
        const uint32_t st = cpuset_filter(n, i, p, j, policy, node_bind, zone_out);
        if (st) return st;
    }
    /* a NUMA policy on a node whose reservations hold NUMA / cpuset allocations: the hints and allocations read their
     * restore (resource_manager.go:131-160), not restated */
    if (policy != KG_NUMA_NONE && n->rsv_numa && n->rsv_numa[i]) return KG_ST_UNSUPPORTED;
    if (policy == KG_NUMA_NONE) {
        /* scoreWithAmplifiedCPUs, scoring.go:132-151 */
        int64_t req_cpu = N_REQ_CPU(n, i, ov);
        if (!(pod_cpu == 0 || ratio <= 1)) {
            int64_t allocated = n->cpuset_alloc_milli[i];
            req_cpu = req_cpu - allocated + kgo_amplify(allocated, ratio);
        }
        /* getResourceOptions (plugin.go:772-778): a cpuset-binding pod's request is amplified */
        const int64_t own = cpu_bind && ratio > 1 ? kgo_amplify(pod_cpu, ratio) : pod_cpu;
        *score_out = numa_node_score(c, n->alloc_cpu[i], req_cpu + own, n->alloc_mem[i],
                                     N_REQ_MEM(n, i, ov) + p->req_mem[j]);
        return 0;
    }
    /* FilterByNUMANode (topology_hint.go:31-41): SingleNUMANode / Restricted admit in Filter; BestEffort
     * admits at Reserve only (plugin.go:446-455,612-623), its Score sees no affinity */
    numa_zones x;
    numa_zones_load(n, i, &x);
    const int64_t req[2] = {p->req_cpu[j], p->req_mem[j]};
    const int has[2] = {(p->flags[j] & KG_POD_HAS_CPU) != 0, (p->flags[j] & KG_POD_HAS_MEM) != 0};
    /* podNUMAExclusive defaults to Required when the pod carries its own NUMA policy (plugin.go:449-454) */
    const int excl = p->numa_policy[j] != KG_NUMA_NONE;
    uint32_t mask = 0;
    /* a cpuset-binding pod: the CPUs of every allocation under a hint (numa_bind), the cpu available to a required
     * policy trimmed to its filtered CPUs (trimNUMANodeResources, resource_manager.go:159-194), its cpu request
     * amplified where the options' requests count (hint scores, scores; getResourceOptions, plugin.go:774-778), and
     * the Score's requested cpu = the node's cpuset CPUs amplified (calculateAllocatableAndRequested, scoring.go:190-197) */
    numa_bind nb;
    const numa_bind* bp = NULL;
    int64_t score_cpu = pod_cpu;
    if (cpu_bind) {
        numa_bind_load(n, i, p, j, node_bind, &nb);
        bp = &nb;
        if (nb.required)
            for (uint32_t z = 0; z < x.Z && z < KG_MAX_ZONES; z++)
                if (x.avail[0][z] > nb.cnt[z] * 1000) x.avail[0][z] = nb.cnt[z] * 1000;
        score_cpu = kgo_amplify(pod_cpu, ratio);
    }
    const int64_t bind_cpu = kgo_amplify(n->cpuset_alloc_milli[i], ratio);
    if (policy == KG_NUMA_BEST_EFFORT) {
        /* Filter: nothing more; Score: node allocatable / requested without an allocation (scoring.go:184-189).
         * The zone is what the Reserve would do: FilterByNUMANode under BestEffort (always admits) and the
         * allocation of its best hint; a failure is reported as the zone code ZONE_RESERVE_FAIL | bits:
         * GetTopologyHints without NUMA resources -> "node(s) Insufficient NUMA Node resources"
         * (resource_manager.go:133-136), tryBestToDistributeEvenly -> "Insufficient NUMA <r>" (:300-309) */
        *score_out = numa_node_score(c, n->alloc_cpu[i], N_REQ_CPU(n, i, ov) + pod_cpu, n->alloc_mem[i],
                                     N_REQ_MEM(n, i, ov) + p->req_mem[j]);
        if (cpu_bind) { /* Score's tryAllocateFromNode without an affinity: the node's CPUs, else score 0 */
            uint64_t out[4];
            *score_out = cpuset_allocate(n, i, p, j, node_bind, out)
                             ? 0
                             : numa_node_score(c, n->alloc_cpu[i], bind_cpu + score_cpu, n->alloc_mem[i],
                                               N_REQ_MEM(n, i, ov) + p->req_mem[j]);
        }
        if (x.Z == 0) {
            *zone_out = KGO_ZONE_RESERVE_FAIL | (int32_t)(KG_ST_NUMA_INSUF_NODE >> 12);
            return 0;
        }
        /* a GPU pod: the DeviceShare provider's hints join the merge; a provider failure fails the Reserve
         * (accumulateProvidersHints -> Admit, manager.go:80-87), so does DeviceShare's Allocate under the best hint
         * (allocateResources, after the NUMA allocation) */
        gpu_hints gh;
        if (gx) {
            gpu_numa_hints(c, n, i, p, j, gx, &gh);
            if (gh.fail) {
                *zone_out = zone_gpu_fail(gh.code);
                return 0;
            }
        }
        numa_admit(c, &x, req, has, policy, excl, &mask, gx ? &gh : NULL, bp, score_cpu);
        int64_t al[2][KG_MAX_ZONES];
        int32_t fail = 0;
        for (int r = 0; r < 2 && mask; r++) {
            const int one[2] = {r == 0 && has[0], r == 1 && has[1]};
            if (one[r] && !numa_split(&x, mask, req, one, al, bp)) fail |= 1 << r;
        }
        *zone_out = fail ? KGO_ZONE_RESERVE_FAIL | fail : numa_code(mask);
        if (!fail && bp) { /* allocateCPUSet over the allocated NUMA nodes (the whole node without an affinity) */
            uint64_t out[4];
            if (mask) {
                numa_split(&x, mask, req, has, al, bp);
                if (numa_bind_check(bp, al, x.Z)) fail = *zone_out = KGO_ZONE_CPUSET_FAIL;
            } else if (cpuset_allocate(n, i, p, j, node_bind, out)) {
                fail = *zone_out = KGO_ZONE_CPUSET_FAIL;
            }
        }
        if (!fail && gx) {
            uint32_t minors;
            const uint32_t st = gpu_alloc_site(c, n, i, p, j, gx, mask, &minors);
            if (st) *zone_out = zone_gpu_fail(st);
        }
        return 0;
    }
    if (x.Z == 0) return KG_ST_NUMA_NO_RES;
    gpu_hints gh;
    if (gx) {
        gpu_numa_hints(c, n, i, p, j, gx, &gh);
        if (gh.fail) return gh.code; /* the provider's status (manager.go:80-87) */
    }
    uint32_t st = numa_admit(c, &x, req, has, policy, excl, &mask, gx ? &gh : NULL, bp, score_cpu);
    if (st) return st;
    int64_t al[2][KG_MAX_ZONES];
    /* allocateResources under the best hint: not reached with a mask (a preferred best hint is one of the providers'
     * feasible masks); without one a cpuset-binding pod takes CPUs from the whole node */
    if (mask && !numa_split(&x, mask, req, has, al, bp)) return KG_ST_UNSUPPORTED;
    if (mask && bp && numa_bind_check(bp, al, x.Z)) return KG_ST_UNSUPPORTED;
    if (!mask && bp) {
        uint64_t out[4];
        if (cpuset_allocate(n, i, p, j, node_bind, out)) return KG_ST_NUMA_CPUS;
    }
    if (gx) { /* allocateResources: DeviceShare's Allocate under the best hint (topology_hint.go:100-157) */
        uint32_t minors;
        const uint32_t st2 = gpu_alloc_site(c, n, i, p, j, gx, mask, &minors);
        if (st2) return st2;
        gx->done = 1;
        gx->mask = mask;
    }
    *zone_out = numa_code(mask);
    if (!mask || !(p->req_cpu[j] | p->req_mem[j])) {
        /* calculateAllocatableAndRequested without NUMANodeResources (no affinity, or no cpu / memory request):
         * node allocatable / requested (scoring.go:168-189) */
        *score_out = numa_node_score(c, n->alloc_cpu[i], (bp ? bind_cpu : N_REQ_CPU(n, i, ov)) + score_cpu,
                                     n->alloc_mem[i], N_REQ_MEM(n, i, ov) + p->req_mem[j]);
        return 0;
    }
    /* the zones that received an allocation: their totals and their allocated */
    int64_t T[2] = {0, 0}, U[2] = {0, 0};
    for (uint32_t z = 0; z < x.Z; z++) {
        if (al[0][z] == 0 && al[1][z] == 0) continue;
        for (int r = 0; r < 2; r++) {
            T[r] += x.tot[r][z];
            U[r] += x.used[r][z];
        }
    }
    *score_out = numa_node_score(c, T[0], (bp ? bind_cpu : U[0]) + score_cpu, T[1], U[1] + p->req_mem[j]);
    return 0;
}

/* ---------------------------------------------------------------------------------------------- */

void kgo_eval_pair(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j,
                   kgo_pair* out) {
    uint32_t st = 0;
    int64_t s_numa = 0;
    int32_t zone = -1;
    if (c->plugins & KG_PLUGIN_NRF) st |= nrf_filter(c, n, i, NULL, p, j);
    if (c->plugins & KG_PLUGIN_LA) st |= la_filter(c, n, i, p, j);
    if (c->plugins & KG_PLUGIN_NUMA) st |= numa_eval(c, n, i, NULL, p, j, &s_numa, &zone, NULL);
    out->status = st;
    /* Score functions are defined for every node (the Go ScorePlugin.Score can be called on any
     * node); the NUMA score exists only where its Filter admitted the pod (it needs the hint). */
    out->s_nrf = (c->plugins & KG_PLUGIN_NRF) ? nrf_score(c, n, i, NULL, p, j) : 0;
    out->s_la = (c->plugins & KG_PLUGIN_LA) ? la_score(c, n, i, p, j) : 0;
    out->s_numa = (c->plugins & KG_PLUGIN_NUMA) && !(st & (KG_ST_NUMA_MASK | KG_ST_UNSUPPORTED)) ? s_numa : 0;
    if (st) {
        out->total = -1;
        out->zone = -1;
        return;
    }
    out->zone = zone;
    /* RunScorePlugins: Σ weight · score (no ScoreExtensions on these plugins) */
    out->total = c->weight_nrf * out->s_nrf + c->weight_la * out->s_la + c->weight_numa * out->s_numa;
}

void kgo_eval_verify(const kg_config* c, const kg_node_columns* n, uint32_t nn, const kg_pod_columns* p,
                     uint32_t np, kg_verify_out* o) {
    for (uint32_t j = 0; j < np; j++) {
        for (uint32_t i = 0; i < nn; i++) {
            kgo_pair r;
            kgo_eval_pair(c, n, i, p, j, &r);
            size_t x = (size_t)j * nn + i;
            if (o->status) o->status[x] = r.status;
            if (o->score_nrf) o->score_nrf[x] = r.s_nrf;
            if (o->score_la) o->score_la[x] = r.s_la;
            if (o->score_numa) o->score_numa[x] = r.s_numa;
            if (o->total) o->total[x] = r.total;
            if (o->numa_zone) o->numa_zone[x] = (int8_t)r.zone;
        }
    }
}

static uint64_t make_key(int64_t total, uint32_t node) {
    return ((uint64_t)total << 32) | (uint64_t)(0xFFFFFFFFu - node);
}

static void topk_insert(uint64_t* top, uint32_t k, uint64_t key) {
    if (key <= top[k - 1]) return;
    uint32_t pos = k - 1;
    while (pos > 0 && top[pos - 1] < key) {
        top[pos] = top[pos - 1];
        pos--;
    }
    top[pos] = key;
}

void kgo_select(const kg_config* c, const kg_node_columns* n, uint32_t nn, uint32_t base, const kg_pod_columns* p,
                uint32_t np, uint32_t k, uint64_t* keys) {
    for (uint32_t j = 0; j < np; j++) {
        uint64_t* top = keys + (size_t)j * k;
        memset(top, 0, sizeof(uint64_t) * k);
        for (uint32_t i = 0; i < nn; i++) {
            kgo_pair r;
            kgo_eval_pair(c, n, i, p, j, &r);
            if (r.status) continue;
            topk_insert(top, k, make_key(r.total, base + i));
        }
    }
}

/* ---------------------------------------------------------------------------------------------- */
/* Upstream-shaped parallel CPU baseline. parallelizer.Until(ctx, n, f): workers = min(16, ...),     */
/* chunkSize = max(1, min(sqrt(n), n/workers+1)) (pkg/util/parallelize/parallelism.go:35-49).        */

typedef struct par_job {
    const kg_config* c;
    const kg_node_columns* n;
    const kg_pod_columns* p;
    uint32_t nn, pod, base;
    int phase; /* 0 filter, 1 score */
    uint8_t* feasible;
    int64_t* total;
    int32_t* zone; /* NUMA zone the pair's Reserve would allocate from (filter phase) */
    volatile int next_chunk;
    int chunk, n_items;
    const uint32_t* items; /* phase 1: feasible node list */
} par_job;

typedef struct par_pool {
    pthread_t* th;
    int n, workers;
    pthread_barrier_t start, done;
    par_job* job;
    int quit;
    par_job jb;
    uint32_t* items;
} par_pool;

static void par_run(par_job* jb) {
    for (;;) {
        int c0 = __atomic_fetch_add(&jb->next_chunk, 1, __ATOMIC_RELAXED);
        int lo = c0 * jb->chunk;
        if (lo >= jb->n_items) break;
        int hi = lo + jb->chunk;
        if (hi > jb->n_items) hi = jb->n_items;
        for (int x = lo; x < hi; x++) {
            if (jb->phase == 0) {
                uint32_t st = 0;
                uint32_t i = (uint32_t)x;
                if (jb->c->plugins & KG_PLUGIN_NRF) st |= nrf_filter(jb->c, jb->n, i, NULL, jb->p, jb->pod);
                if (jb->c->plugins & KG_PLUGIN_LA) st |= la_filter(jb->c, jb->n, i, jb->p, jb->pod);
                int64_t s = 0;
                int32_t z = -1;
                if (jb->c->plugins & KG_PLUGIN_NUMA) {
                    st |= numa_eval(jb->c, jb->n, i, NULL, jb->p, jb->pod, &s, &z, NULL);
                    jb->total[i] = s; /* NUMA score is produced by the same resource-manager walk */
                }
                jb->zone[i] = st ? -1 : z;
                jb->feasible[i] = st == 0;
            } else {
                uint32_t i = jb->items[x];
                int64_t t = 0;
                const kg_config* c = jb->c;
                if (c->plugins & KG_PLUGIN_NRF) t += c->weight_nrf * nrf_score(c, jb->n, i, NULL, jb->p, jb->pod);
                if (c->plugins & KG_PLUGIN_LA) t += c->weight_la * la_score(c, jb->n, i, jb->p, jb->pod);
                if (c->plugins & KG_PLUGIN_NUMA) t += c->weight_numa * jb->total[i];
                jb->total[i] = t;
            }
        }
    }
}

static void* par_worker(void* arg) {
    par_pool* pool = (par_pool*)arg;
    for (;;) {
        pthread_barrier_wait(&pool->start);
        if (pool->quit) break;
        par_run(pool->job);
        pthread_barrier_wait(&pool->done);
    }
    return NULL;
}

static int chunk_size(int n, int workers) {
    int s = (int)sqrt((double)n);
    int t = n / workers + 1;
    int c = s < t ? s : t;
    return c < 1 ? 1 : c;
}

static int par_open(par_pool* pool, int workers, uint32_t nn) {
    if (workers < 1) workers = 1;
    memset(pool, 0, sizeof(*pool));
    pool->workers = workers;
    pool->n = workers - 1; /* the calling thread is worker 0 */
    pool->th = (pthread_t*)calloc((size_t)(pool->n > 0 ? pool->n : 1), sizeof(pthread_t));
    pool->jb.feasible = (uint8_t*)malloc(nn ? nn : 1);
    pool->jb.total = (int64_t*)malloc(sizeof(int64_t) * (nn ? nn : 1));
    pool->jb.zone = (int32_t*)malloc(sizeof(int32_t) * (nn ? nn : 1));
    pool->items = (uint32_t*)malloc(sizeof(uint32_t) * (nn ? nn : 1));
    if (!pool->th || !pool->jb.feasible || !pool->jb.total || !pool->jb.zone || !pool->items) return -1;
    pool->job = &pool->jb;
    pthread_barrier_init(&pool->start, NULL, (unsigned)workers);
    pthread_barrier_init(&pool->done, NULL, (unsigned)workers);
    for (int t = 0; t < pool->n; t++) pthread_create(&pool->th[t], NULL, par_worker, pool);
    return 0;
}

static void par_close(par_pool* pool) {
    pool->quit = 1;
    pthread_barrier_wait(&pool->start);
    for (int t = 0; t < pool->n; t++) pthread_join(pool->th[t], NULL);
    pthread_barrier_destroy(&pool->start);
    pthread_barrier_destroy(&pool->done);
    free(pool->th);
    free(pool->jb.feasible);
    free(pool->jb.total);
    free(pool->jb.zone);
    free(pool->items);
}

/* One scheduling cycle of pod j on the pool: findNodesThatPassFilters (parallel Filter), then, with more
 * than one feasible node, prioritizeNodes (parallel Score) and selectHost. Returns the best key and the
 * NUMA zone of the chosen pair. */
static uint64_t par_cycle(par_pool* pool, const kg_config* c, const kg_node_columns* n, uint32_t nn, uint32_t base,
                          const kg_pod_columns* p, uint32_t j, int32_t* zone_out) {
    par_job* jb = &pool->jb;
    uint32_t* items = pool->items;
    jb->c = c;
    jb->n = n;
    jb->p = p;
    jb->nn = nn;
    jb->pod = j;
    jb->base = base;
    jb->phase = 0;
    jb->n_items = (int)nn;
    jb->chunk = chunk_size((int)nn, pool->workers);
    jb->next_chunk = 0;
    pthread_barrier_wait(&pool->start);
    par_run(jb);
    pthread_barrier_wait(&pool->done);
    uint32_t nf = 0;
    for (uint32_t i = 0; i < nn; i++)
        if (jb->feasible[i]) items[nf++] = i;
    uint64_t best = 0;
    int32_t zone = -1;
    if (nf > 1) {
        /* prioritizeNodes */
        jb->phase = 1;
        jb->items = items;
        jb->n_items = (int)nf;
        jb->chunk = chunk_size((int)nf, pool->workers);
        jb->next_chunk = 0;
        pthread_barrier_wait(&pool->start);
        par_run(jb);
        pthread_barrier_wait(&pool->done);
        /* selectHost (deterministic tie-break) */
        for (uint32_t x = 0; x < nf; x++) {
            uint64_t key = make_key(jb->total[items[x]], base + items[x]);
            if (key > best) {
                best = key;
                zone = jb->zone[items[x]];
            }
        }
    } else if (nf == 1) {
        /* exactly one feasible node: chosen without scoring; key still carries its total */
        kgo_pair r;
        kgo_eval_pair(c, n, items[0], p, j, &r);
        best = make_key(r.total, base + items[0]);
        zone = jb->zone[items[0]];
    }
    if (zone_out) *zone_out = zone;
    return best;
}

int kgo_select_parallel(const kg_config* c, const kg_node_columns* n, uint32_t nn, uint32_t base,
                        const kg_pod_columns* p, uint32_t np, int workers, uint64_t* keys) {
    par_pool pool;
    if (par_open(&pool, workers, nn)) return -1;
    for (uint32_t j = 0; j < np; j++) keys[j] = par_cycle(&pool, c, n, nn, base, p, j, NULL);
    par_close(&pool);
    return 0;
}

/* ---------------------------------------------------------------------------------------------- */
/* Mutable state, Assume, replay                                                                   */

enum {
    C_ALLOC_CPU, C_ALLOC_MEM, C_ALLOC_EPH, C_ALLOC_PODS, C_REQ_CPU, C_REQ_MEM, C_REQ_EPH, C_NUM_PODS, C_NZ_CPU,
    C_NZ_MEM, C_SC_ALLOC, C_SC_REQ = C_SC_ALLOC + KG_NSCALAR, C_LA_ALLOC = C_SC_REQ + KG_NSCALAR,
    C_LA_THR_USAGE = C_LA_ALLOC + KG_LA_R, C_LA_THR_PROD = C_LA_THR_USAGE + KG_LA_R,
    C_LA_THR_AGG = C_LA_THR_PROD + KG_LA_R, C_LA_FB_NP = C_LA_THR_AGG + KG_LA_R,
    C_LA_FB_PROD = C_LA_FB_NP + KG_LA_R, C_LA_SB_NP = C_LA_FB_PROD + KG_LA_R,
    C_LA_SB_PROD = C_LA_SB_NP + KG_LA_R, C_CPUSET = C_LA_SB_PROD + KG_LA_R, C_ZONE_CPU,
    C_ZONE_MEM = C_ZONE_CPU + KG_MAX_ZONES, C_ZONE_CPU_USED = C_ZONE_MEM + KG_MAX_ZONES,
    C_ZONE_MEM_USED = C_ZONE_CPU_USED + KG_MAX_ZONES, C_NCOLS = C_ZONE_MEM_USED + KG_MAX_ZONES
};

struct kgo_state {
    uint32_t n;
    int64_t* col[C_NCOLS];
    uint32_t *la_flags, *numa_policy, *numa_zones, *zone_status;
    uint64_t* zone_pods; /* cpuset pods per NUMA node: byte z singleNUMANode, byte KG_MAX_ZONES + z sharedNode */
    double* amp;
    int32_t* dev_minors;          /* DeviceShare (NULL when the snapshot has no device tables) */
    int64_t *dev_total, *dev_free; /* [node][KG_DEV_R][KG_DEV_MINORS] */
    uint64_t* dev_topo;            /* GPU topology / partition tables / GPU NUMA nodes (static) */
    uint32_t* dev_part;
    uint32_t* dev_numa;
    kg_gpu_partition* gpu_parts;
    uint32_t n_gpu_parts;
    /* cpuset binding (NULL when no node has a CPU topology) */
    int32_t* cpu_topo;
    kg_cpu_topo* cpu_topos;
    uint32_t n_cpu_topos;
    kg_cpu_alloc* cpu_alloc;
    uint8_t *cpu_max_ref, *cpu_bind, *cpu_strategy;
    uint8_t* rsv_numa; /* a reservation on the node holds a NUMA / cpuset allocation (static; NULL = none) */
};

static int64_t* dup64(const int64_t* s, uint32_t n) {
    int64_t* d = (int64_t*)calloc(n ? n : 1, sizeof(int64_t));
    if (s) memcpy(d, s, sizeof(int64_t) * n);
    return d;
}

/* NUMANodeSharedStatus (node_allocation.go:60-68) of node i from its single / shared cpuset pod counts; the allocation
 * record bits stay */
static void zone_pods_status(kgo_state* st, uint32_t i) {
    uint32_t x = st->zone_status[i] & ~0xFFu;
    for (int z = 0; z < KG_MAX_ZONES; z++) {
        const uint32_t single = (uint32_t)(st->zone_pods[i] >> (8 * z)) & 0xFFu;
        const uint32_t shared = (uint32_t)(st->zone_pods[i] >> (8 * (KG_MAX_ZONES + z))) & 0xFFu;
        x |= (shared ? 2u : single ? 1u : 0u) << (2 * z);
    }
    st->zone_status[i] = x;
}

/* addPodAllocation / release (node_allocation.go:111-143,164-200): the pod's uid joins (sign 1) or leaves (-1)
 * singleNUMANode of its one NUMA node, or sharedNode of each of several (used: NUMA nodes of its CPUs) */
static void zone_pods_add(kgo_state* st, uint32_t i, uint32_t used, int sign) {
    const int multi = (used & (used - 1)) != 0;
    for (int z = 0; z < KG_MAX_ZONES; z++) {
        if (!((used >> z) & 1u)) continue;
        const int sh = 8 * (multi ? KG_MAX_ZONES + z : z);
        int c = (int)((st->zone_pods[i] >> sh) & 0xFFu) + sign;
        c = c < 0 ? 0 : c > 255 ? 255 : c;
        st->zone_pods[i] = (st->zone_pods[i] & ~(0xFFull << sh)) | ((uint64_t)c << sh);
    }
    zone_pods_status(st, i);
}

kgo_state* kgo_state_new(const kg_node_columns* s, uint32_t n) {
    kgo_state* st = (kgo_state*)calloc(1, sizeof(kgo_state));
    st->n = n;
    st->col[C_ALLOC_CPU] = dup64(s->alloc_cpu, n);
    st->col[C_ALLOC_MEM] = dup64(s->alloc_mem, n);
    st->col[C_ALLOC_EPH] = dup64(s->alloc_eph, n);
    st->col[C_ALLOC_PODS] = dup64(s->alloc_pods, n);
    st->col[C_REQ_CPU] = dup64(s->req_cpu, n);
    st->col[C_REQ_MEM] = dup64(s->req_mem, n);
    st->col[C_REQ_EPH] = dup64(s->req_eph, n);
    st->col[C_NUM_PODS] = dup64(s->num_pods, n);
    st->col[C_NZ_CPU] = dup64(s->nz_cpu, n);
    st->col[C_NZ_MEM] = dup64(s->nz_mem, n);
    for (int k = 0; k < KG_NSCALAR; k++) {
        st->col[C_SC_ALLOC + k] = dup64(s->sc_alloc[k], n);
        st->col[C_SC_REQ + k] = dup64(s->sc_req[k], n);
    }
    for (int r = 0; r < KG_LA_R; r++) {
        st->col[C_LA_ALLOC + r] = dup64(s->la_alloc[r], n);
        st->col[C_LA_THR_USAGE + r] = dup64(s->la_thr_usage[r], n);
        st->col[C_LA_THR_PROD + r] = dup64(s->la_thr_prod[r], n);
        st->col[C_LA_THR_AGG + r] = dup64(s->la_thr_agg[r], n);
        st->col[C_LA_FB_NP + r] = dup64(s->la_fbase_np[r], n);
        st->col[C_LA_FB_PROD + r] = dup64(s->la_fbase_prod[r], n);
        st->col[C_LA_SB_NP + r] = dup64(s->la_sbase_np[r], n);
        st->col[C_LA_SB_PROD + r] = dup64(s->la_sbase_prod[r], n);
    }
    st->col[C_CPUSET] = dup64(s->cpuset_alloc_milli, n);
    for (int z = 0; z < KG_MAX_ZONES; z++) {
        st->col[C_ZONE_CPU + z] = dup64(s->zone_cpu[z], n);
        st->col[C_ZONE_MEM + z] = dup64(s->zone_mem[z], n);
        st->col[C_ZONE_CPU_USED + z] = dup64(s->zone_cpu_used[z], n);
        st->col[C_ZONE_MEM_USED + z] = dup64(s->zone_mem_used[z], n);
    }
    st->la_flags = (uint32_t*)calloc(n ? n : 1, 4);
    st->numa_policy = (uint32_t*)calloc(n ? n : 1, 4);
    st->numa_zones = (uint32_t*)calloc(n ? n : 1, 4);
    st->amp = (double*)calloc(n ? n : 1, 8);
    st->zone_status = (uint32_t*)calloc(n ? n : 1, 4);
    if (s->numa_zone_status) memcpy(st->zone_status, s->numa_zone_status, 4 * (size_t)n);
    st->zone_pods = (uint64_t*)calloc(n ? n : 1, 8);
    if (s->rsv_numa) {
        st->rsv_numa = (uint8_t*)calloc(n ? n : 1, 1);
        memcpy(st->rsv_numa, s->rsv_numa, n);
    }
    for (uint32_t i = 0; i < n; i++) {
        if (s->numa_zone_pods) {
            st->zone_pods[i] = s->numa_zone_pods[i];
            zone_pods_status(st, i);
        } else { /* one pod per non-idle status */
            for (int z = 0; z < KG_MAX_ZONES; z++) {
                const uint32_t x = (st->zone_status[i] >> (2 * z)) & 3u;
                if (x == 1u) st->zone_pods[i] |= 1ull << (8 * z);
                if (x >= 2u) st->zone_pods[i] |= 1ull << (8 * (KG_MAX_ZONES + z));
            }
        }
    }
    if (s->la_flags) memcpy(st->la_flags, s->la_flags, 4 * (size_t)n);
    if (s->numa_policy) memcpy(st->numa_policy, s->numa_policy, 4 * (size_t)n);
    if (s->numa_zones) memcpy(st->numa_zones, s->numa_zones, 4 * (size_t)n);
    if (s->cpu_amp_ratio) memcpy(st->amp, s->cpu_amp_ratio, 8 * (size_t)n);
    if (s->dev_minors && s->dev_total && s->dev_free) {
        size_t m = (size_t)(n ? n : 1) * KG_DEV_R * KG_DEV_MINORS;
        st->dev_minors = (int32_t*)calloc(n ? n : 1, 4);
        st->dev_total = (int64_t*)calloc(m, 8);
        st->dev_free = (int64_t*)calloc(m, 8);
        memcpy(st->dev_minors, s->dev_minors, 4 * (size_t)n);
        memcpy(st->dev_total, s->dev_total, 8 * (size_t)n * KG_DEV_R * KG_DEV_MINORS);
        memcpy(st->dev_free, s->dev_free, 8 * (size_t)n * KG_DEV_R * KG_DEV_MINORS);
        if (s->dev_topo) {
            st->dev_topo = (uint64_t*)calloc(n ? n : 1, 8);
            memcpy(st->dev_topo, s->dev_topo, 8 * (size_t)n);
        }
        if (s->dev_numa) {
            st->dev_numa = (uint32_t*)calloc(n ? n : 1, 4);
            memcpy(st->dev_numa, s->dev_numa, 4 * (size_t)n);
        }
        if (s->dev_part) {
            st->dev_part = (uint32_t*)calloc(n ? n : 1, 4);
            memcpy(st->dev_part, s->dev_part, 4 * (size_t)n);
        }
        if (s->gpu_parts && s->n_gpu_parts) {
            st->n_gpu_parts = s->n_gpu_parts;
            st->gpu_parts = (kg_gpu_partition*)calloc(s->n_gpu_parts, sizeof(kg_gpu_partition));
            memcpy(st->gpu_parts, s->gpu_parts, sizeof(kg_gpu_partition) * s->n_gpu_parts);
        }
    }
    if (s->cpu_topo && s->cpu_topos) {
        const size_t m = n ? n : 1;
        st->cpu_topo = (int32_t*)calloc(m, 4);
        memcpy(st->cpu_topo, s->cpu_topo, 4 * (size_t)n);
        st->n_cpu_topos = s->n_cpu_topos;
        st->cpu_topos = (kg_cpu_topo*)calloc(s->n_cpu_topos ? s->n_cpu_topos : 1, sizeof(kg_cpu_topo));
        memcpy(st->cpu_topos, s->cpu_topos, sizeof(kg_cpu_topo) * s->n_cpu_topos);
        st->cpu_alloc = (kg_cpu_alloc*)calloc(m, sizeof(kg_cpu_alloc));
        if (s->cpu_alloc) memcpy(st->cpu_alloc, s->cpu_alloc, sizeof(kg_cpu_alloc) * (size_t)n);
        st->cpu_max_ref = (uint8_t*)calloc(m, 1);
        st->cpu_bind = (uint8_t*)calloc(m, 1);
        st->cpu_strategy = (uint8_t*)calloc(m, 1);
        for (uint32_t i = 0; i < n; i++) st->cpu_max_ref[i] = 1;
        if (s->cpu_max_ref) memcpy(st->cpu_max_ref, s->cpu_max_ref, n);
        if (s->cpu_bind_policy) memcpy(st->cpu_bind, s->cpu_bind_policy, n);
        if (s->cpu_strategy) memcpy(st->cpu_strategy, s->cpu_strategy, n);
    }
    return st;
}

void kgo_state_free(kgo_state* st) {
    if (!st) return;
    for (int c = 0; c < C_NCOLS; c++) free(st->col[c]);
    free(st->la_flags);
    free(st->numa_policy);
    free(st->numa_zones);
    free(st->amp);
    free(st->zone_status);
    free(st->zone_pods);
    free(st->dev_minors);
    free(st->dev_topo);
    free(st->dev_part);
    free(st->dev_numa);
    free(st->rsv_numa);
    free(st->gpu_parts);
    free(st->dev_total);
    free(st->dev_free);
    free(st->cpu_topo);
    free(st->cpu_topos);
    free(st->cpu_alloc);
    free(st->cpu_max_ref);
    free(st->cpu_bind);
    free(st->cpu_strategy);
    free(st);
}

void kgo_state_view(kgo_state* st, kg_node_columns* v) {
    memset(v, 0, sizeof(*v));
    v->alloc_cpu = st->col[C_ALLOC_CPU];
    v->alloc_mem = st->col[C_ALLOC_MEM];
    v->alloc_eph = st->col[C_ALLOC_EPH];
    v->alloc_pods = st->col[C_ALLOC_PODS];
    v->req_cpu = st->col[C_REQ_CPU];
    v->req_mem = st->col[C_REQ_MEM];
    v->req_eph = st->col[C_REQ_EPH];
    v->num_pods = st->col[C_NUM_PODS];
    v->nz_cpu = st->col[C_NZ_CPU];
    v->nz_mem = st->col[C_NZ_MEM];
    for (int k = 0; k < KG_NSCALAR; k++) {
        v->sc_alloc[k] = st->col[C_SC_ALLOC + k];
        v->sc_req[k] = st->col[C_SC_REQ + k];
    }
    v->la_flags = st->la_flags;
    for (int r = 0; r < KG_LA_R; r++) {
        v->la_alloc[r] = st->col[C_LA_ALLOC + r];
        v->la_thr_usage[r] = st->col[C_LA_THR_USAGE + r];
        v->la_thr_prod[r] = st->col[C_LA_THR_PROD + r];
        v->la_thr_agg[r] = st->col[C_LA_THR_AGG + r];
        v->la_fbase_np[r] = st->col[C_LA_FB_NP + r];
        v->la_fbase_prod[r] = st->col[C_LA_FB_PROD + r];
        v->la_sbase_np[r] = st->col[C_LA_SB_NP + r];
        v->la_sbase_prod[r] = st->col[C_LA_SB_PROD + r];
    }
    v->numa_policy = st->numa_policy;
    v->numa_zones = st->numa_zones;
    v->cpu_amp_ratio = st->amp;
    v->cpuset_alloc_milli = st->col[C_CPUSET];
    for (int z = 0; z < KG_MAX_ZONES; z++) {
        v->zone_cpu[z] = st->col[C_ZONE_CPU + z];
        v->zone_mem[z] = st->col[C_ZONE_MEM + z];
        v->zone_cpu_used[z] = st->col[C_ZONE_CPU_USED + z];
        v->zone_mem_used[z] = st->col[C_ZONE_MEM_USED + z];
    }
    v->numa_zone_status = st->zone_status;
    v->numa_zone_pods = st->zone_pods;
    v->dev_minors = st->dev_minors;
    v->dev_total = st->dev_total;
    v->dev_free = st->dev_free;
    v->dev_topo = st->dev_topo;
    v->dev_part = st->dev_part;
    v->dev_numa = st->dev_numa;
    v->rsv_numa = st->rsv_numa;
    v->gpu_parts = st->gpu_parts;
    v->n_gpu_parts = st->n_gpu_parts;
    v->cpu_topo = st->cpu_topo;
    v->cpu_topos = st->cpu_topos;
    v->n_cpu_topos = st->n_cpu_topos;
    v->cpu_alloc = st->cpu_alloc;
    v->cpu_max_ref = st->cpu_max_ref;
    v->cpu_bind_policy = st->cpu_bind;
    v->cpu_strategy = st->cpu_strategy;
}

/* NodeNUMAResource Reserve of a cpuset-binding pod on a NUMA-policy-None node: the accumulator's CPUs
 * enter NodeAllocation.allocatedCPUs (addPodAllocation, node_allocation.go:111-130: RefCount++, the pod's
 * exclusive policy), and cpuset_alloc_milli follows the allocated CPU count */
/* resourceManager.Allocate of a cpuset-binding pod on node i (resource_manager.go:197-262,357-463): under the NUMA
 * affinity `mask` the split of its requests over those NUMA nodes (*al, *have_al = 1) and one take per allocated node,
 * without one a take over the node; the CPUs in out. Returns 1 when it fails. */
static int numa_bind_take(const kg_node_columns* v, uint32_t i, const kg_pod_columns* p, uint32_t j, uint32_t node_bind,
                          uint32_t mask, uint64_t out[4], int64_t al[2][KG_MAX_ZONES], int* have_al) {
    *have_al = 0;
    for (int w = 0; w < 4; w++) out[w] = 0;
    if (!mask) return cpuset_allocate(v, i, p, j, node_bind, out) ? 1 : 0;
    const kg_cpu_topo* t = cpu_topology(v, i);
    if (!t) return 1;
    numa_zones x;
    numa_zones_load(v, i, &x);
    numa_bind nb;
    numa_bind_load(v, i, p, j, node_bind, &nb);
    if (nb.required)
        for (uint32_t z = 0; z < x.Z && z < KG_MAX_ZONES; z++)
            if (x.avail[0][z] > nb.cnt[z] * 1000) x.avail[0][z] = nb.cnt[z] * 1000;
    const int64_t req[2] = {p->req_cpu[j], p->req_mem[j]};
    const int has[2] = {(p->flags[j] & KG_POD_HAS_CPU) != 0, (p->flags[j] & KG_POD_HAS_MEM) != 0};
    if (!numa_split(&x, mask, req, has, al, &nb) || numa_bind_check(&nb, al, x.Z)) return 1;
    *have_al = 1;
    int required;
    const uint32_t pol = cpu_bind_policy(p, j, node_bind, &required);
    const uint32_t excl = (p->flags[j] >> KG_POD_CPU_EXCL_SHIFT) & 3u;
    uint64_t avail[4];
    cpu_available(v, i, t, avail);
    if (required) cpu_filter_required(t, pol, avail);
    const uint32_t strategy = v->cpu_strategy ? v->cpu_strategy[i] : KG_NUMA_MOST_ALLOCATED;
    const kg_cpu_alloc* alloc = v->cpu_alloc ? &v->cpu_alloc[i] : NULL;
    for (uint32_t z = 0; z < x.Z && z < KG_MAX_ZONES; z++) {
        if (al[0][z] == 0 && al[1][z] == 0) continue;
        int64_t k = al[0][z] / 1000;
        if (nb.cnt[z] < k) k = nb.cnt[z];
        if (k == 0) continue;
        uint64_t in_z[4] = {0, 0, 0, 0}, got[4];
        for (int cc = 0; cc < t->n_cpus; cc++)
            if (t->numa[cc] == z && ((avail[cc >> 6] >> (cc & 63)) & 1ull)) in_z[cc >> 6] |= 1ull << (cc & 63);
        if (kgo_take_cpus(t, cpu_max_ref(v, i), in_z, alloc, (int)k, (int)pol, (int)excl, (int)strategy, got)) return 1;
        for (int w = 0; w < 4; w++) out[w] |= got[w];
    }
    return 0;
}

int kgo_numa_hints(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j,
                   uint32_t policy, uint32_t out[2 * 16], int32_t len[2]) {
    numa_zones x;
    numa_zones_load(n, i, &x);
    if (x.Z == 0) return -1;
    const uint32_t node_bind = n->cpu_bind_policy ? n->cpu_bind_policy[i] : KG_NODE_CPU_BIND_NONE;
    const int bind = (p->flags[j] & KG_POD_CPU_BIND) || (node_bind != KG_NODE_CPU_BIND_NONE && p->req_cpu[j] != 0);
    numa_bind nb;
    int64_t score_cpu = p->req_cpu[j];
    if (bind) {
        numa_bind_load(n, i, p, j, node_bind, &nb);
        if (nb.required)
            for (uint32_t z = 0; z < x.Z && z < KG_MAX_ZONES; z++)
                if (x.avail[0][z] > nb.cnt[z] * 1000) x.avail[0][z] = nb.cnt[z] * 1000;
        score_cpu = kgo_amplify(p->req_cpu[j], n->cpu_amp_ratio[i]);
    }
    const int64_t req[2] = {p->req_cpu[j], p->req_mem[j]};
    const int has[2] = {(p->flags[j] & KG_POD_HAS_CPU) != 0, (p->flags[j] & KG_POD_HAS_MEM) != 0};
    numa_lists L;
    numa_hints(c, &x, req, has, policy, &L, bind ? &nb : NULL, score_cpu);
    for (int li = 0; li < L.n_lists; li++) {
        len[li] = L.len[li];
        for (int t = 0; t < L.len[li]; t++)
            out[16 * li + t] = L.h[li][t].mask | (L.h[li][t].pref ? 0x100u : 0u) | (L.h[li][t].unsat ? 0x200u : 0u);
    }
    return L.n_lists;
}

int kgo_numa_allocate(const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j, uint32_t mask,
                      uint64_t cpus[4], int64_t al_out[2 * KG_MAX_ZONES]) {
    const uint32_t node_bind = n->cpu_bind_policy ? n->cpu_bind_policy[i] : KG_NODE_CPU_BIND_NONE;
    const int bind = (p->flags[j] & KG_POD_CPU_BIND) || (node_bind != KG_NODE_CPU_BIND_NONE && p->req_cpu[j] != 0);
    int64_t al[2][KG_MAX_ZONES];
    memset(al, 0, sizeof(al));
    for (int w = 0; w < 4; w++) cpus[w] = 0;
    if (bind) {
        int have;
        if (numa_bind_take(n, i, p, j, node_bind, mask, cpus, al, &have)) return 1;
    } else if (mask) {
        numa_zones x;
        numa_zones_load(n, i, &x);
        const int64_t req[2] = {p->req_cpu[j], p->req_mem[j]};
        const int has[2] = {(p->flags[j] & KG_POD_HAS_CPU) != 0, (p->flags[j] & KG_POD_HAS_MEM) != 0};
        if (!numa_split(&x, mask, req, has, al, NULL)) return 1;
    }
    memcpy(al_out, al, sizeof(al));
    return 0;
}

/* NodeNUMAResource Reserve of a cpuset-binding pod (plugin.go:585-635 -> resourceManager.Allocate / Update): the CPUs
 * of numa_bind_take under the affinity of the pair's zone code enter the node's allocation (*al: the NUMA split the
 * Reserve records). Returns 1 when Allocate fails (nothing of the pod is applied). */
static int cpuset_reserve(const kg_config* c, kgo_state* st, uint32_t i, const kg_pod_columns* p, uint32_t j, int32_t zone,
                          int64_t al[2][KG_MAX_ZONES], int* have_al, uint64_t* taken) {
    *have_al = 0;
    if (!(c->plugins & KG_PLUGIN_NUMA) || !st->cpu_topo || (p->flags[j] & KG_POD_NUMA_SKIP)) return 0;
    const uint32_t node_bind = st->cpu_bind[i];
    const int bind = (p->flags[j] & KG_POD_CPU_BIND) || (node_bind != KG_NODE_CPU_BIND_NONE && p->req_cpu[j] != 0);
    if (!bind) return 0;
    int conflict;
    const uint32_t policy = numa_merge_policy(st->numa_policy[i], p->numa_policy[j], &conflict);
    kg_node_columns v;
    kgo_state_view(st, &v);
    uint64_t out[4];
    const uint32_t excl = (p->flags[j] >> KG_POD_CPU_EXCL_SHIFT) & 3u;
    const kg_cpu_topo* t = cpu_topology(&v, i);
    const uint32_t mask = (policy != KG_NUMA_NONE && zone >= 0 && !zone_fails(zone)) ? numa_code_mask(zone) : 0u;
    if (numa_bind_take(&v, i, p, j, node_bind, mask, out, al, have_al)) return 1;
    int allocated = 0;
    uint32_t used = 0; /* usedNUMA: NUMA nodes of the CPUs taken */
    for (int cc = 0; cc < t->n_cpus; cc++) {
        if ((out[cc >> 6] >> (cc & 63)) & 1ull) {
            st->cpu_alloc[i].ref[cc]++;
            st->cpu_alloc[i].excl[cc] = (uint8_t)excl;
            used |= 1u << t->numa[cc];
        }
        allocated += st->cpu_alloc[i].ref[cc] > 0;
    }
    st->col[C_CPUSET][i] = 1000 * (int64_t)allocated;
    /* addPodAllocation (node_allocation.go:111-143): the uid joins singleNUMANode of its one NUMA node or
     * sharedNode of each of several; NUMANodeSharedStatus (:60-68) follows (2 bits per zone < 4) */
    zone_pods_add(st, i, used, 1);
    if (taken)
        for (int w = 0; w < 4; w++) taken[w] = out[w];
    return 0;
}

/* NodeAllocation.release of a cpuset pod's CPUs (node_allocation.go:164-200): RefCount-- (a CPU at 0 leaves
 * allocatedCPUs), the uid leaves the NUMA nodes' single / shared sets, cpuset_alloc_milli follows */
static void cpuset_release(kgo_state* st, uint32_t i, const uint64_t* cpus) {
    if (!st->cpu_topo || st->cpu_topo[i] < 0) return;
    kg_node_columns v;
    kgo_state_view(st, &v);
    const kg_cpu_topo* t = cpu_topology(&v, i);
    if (!t) return;
    uint32_t used = 0;
    int allocated = 0;
    for (int cc = 0; cc < t->n_cpus; cc++) {
        if (((cpus[cc >> 6] >> (cc & 63)) & 1ull) && st->cpu_alloc[i].ref[cc] > 0) {
            if (--st->cpu_alloc[i].ref[cc] == 0) st->cpu_alloc[i].excl[cc] = 0;
            used |= 1u << t->numa[cc];
        }
        allocated += st->cpu_alloc[i].ref[cc] > 0;
    }
    st->col[C_CPUSET][i] = 1000 * (int64_t)allocated;
    zone_pods_add(st, i, used, -1);
}

/* Reserve (sign 1) / Unreserve (-1) of pod j on node i; a Reserve returns KGO_ZONE_CPUSET_FAIL when the
 * cpuset accumulator fails (nothing applied), else 0 */
/* amounts (nullable): the NUMA allocation per zone (cpu, then memory), written by a Reserve and given back by an
 * Unreserve; cpus (nullable): the cpuset CPUs a Reserve took / an Unreserve releases */
static int apply(const kg_config* c, kgo_state* st, uint32_t i, const kg_pod_columns* p, uint32_t j, int32_t zone,
                 int64_t sign, int64_t* amounts, uint64_t* cpus) {
    int64_t bal[2][KG_MAX_ZONES];
    int have_bal = 0;
    if (sign > 0 && cpuset_reserve(c, st, i, p, j, zone, bal, &have_bal, cpus)) return KGO_ZONE_CPUSET_FAIL;
    if (sign < 0 && cpus) cpuset_release(st, i, cpus);
    /* upstream NodeInfo.AddPod / RemovePod: Requested, NonZeroRequested, len(Pods) */
    st->col[C_REQ_CPU][i] += sign * p->req_cpu[j];
    st->col[C_REQ_MEM][i] += sign * p->req_mem[j];
    st->col[C_REQ_EPH][i] += sign * p->req_eph[j];
    for (int k = 0; k < KG_NSCALAR; k++) st->col[C_SC_REQ + k][i] += sign * p->sc_req[k][j];
    st->col[C_NZ_CPU][i] += sign * p->nz_cpu[j];
    st->col[C_NZ_MEM][i] += sign * p->nz_mem[j];
    st->col[C_NUM_PODS][i] += sign;
    /* podAssignCache.assign -> nodeInfo.addPod (pod_assign_cache.go:291-327,618-662): with no pod
     * usage reported yet (u == nil) the whole estimate enters nodeDelta / nodeEstimated, and prodDelta
     * for prod pods; only when the cache holds the node's NodeMetric (AddOrUpdatePod :441-447). */
    if ((c->plugins & KG_PLUGIN_LA) && (st->la_flags[i] & KG_LA_HAS_METRIC)) {
        for (int r = 0; r < KG_LA_R; r++) {
            int64_t e = p->la_est[r][j];
            int64_t d = e > 0 ? e : 0; /* AddDelta(e, nil) adds max(0, e) */
            st->col[C_LA_FB_NP + r][i] += sign * d;
            st->col[C_LA_SB_NP + r][i] += sign * d;
            if (p->flags[j] & KG_POD_PROD) {
                st->col[C_LA_FB_PROD + r][i] += sign * d;
                st->col[C_LA_SB_PROD + r][i] += sign * d;
            }
        }
    }
    /* NodeNUMAResource Reserve -> resourceManager.Update (plugin.go:585-635): the allocation split of
     * the affinity, recomputed from the zone state the pair was evaluated on (Reserve runs right after) */
    if ((c->plugins & KG_PLUGIN_NUMA) && zone >= 0) {
        uint32_t mask = numa_code_mask(zone);
        int64_t al[2][KG_MAX_ZONES];
        memset(al, 0, sizeof(al));
        if (sign < 0 && amounts) {
            for (int z = 0; z < KG_MAX_ZONES; z++) {
                al[0][z] = amounts[z];
                al[1][z] = amounts[KG_MAX_ZONES + z];
            }
        } else if (have_bal) {
            memcpy(al, bal, sizeof(al));
        } else if (popcount32(mask) == 1) {
            int z = __builtin_ctz(mask);
            al[0][z] = p->req_cpu[j];
            al[1][z] = p->req_mem[j];
        } else {
            kg_node_columns v;
            kgo_state_view(st, &v);
            numa_zones x;
            numa_zones_load(&v, i, &x);
            const int64_t req[2] = {p->req_cpu[j], p->req_mem[j]};
            const int has[2] = {(p->flags[j] & KG_POD_HAS_CPU) != 0, (p->flags[j] & KG_POD_HAS_MEM) != 0};
            /* a multi-zone split is only reproducible before the Reserve: Unreserve of one is not restated */
            if (sign > 0) numa_split(&x, mask, req, has, al, NULL);
        }
        for (uint32_t z = 0; z < KG_MAX_ZONES; z++) {
            st->col[C_ZONE_CPU_USED + z][i] += sign * al[0][z];
            st->col[C_ZONE_MEM_USED + z][i] += sign * al[1][z];
            /* addPodAllocation creates the zone's allocatedResources record; release never removes it */
            if (sign > 0 && (al[0][z] != 0 || al[1][z] != 0)) st->zone_status[i] |= 1u << (KG_ZONE_RECORD_SHIFT + z);
            if (sign > 0 && amounts) {
                amounts[z] = al[0][z];
                amounts[KG_MAX_ZONES + z] = al[1][z];
            }
        }
    }
    return 0;
}

/* Reserve of pod j on node i: 0, or 1 when the NodeNUMAResource Reserve fails (nothing applied) */
int kgo_assume(const kg_config* c, kgo_state* st, uint32_t i, const kg_pod_columns* p, uint32_t j) {
    kg_node_columns v;
    kgo_state_view(st, &v);
    kgo_pair r;
    kgo_eval_pair(c, &v, i, p, j, &r);
    int32_t zone = r.status ? -1 : r.zone;
    if (zone_fails(zone)) return 1;
    return apply(c, st, i, p, j, zone, 1, NULL, NULL) != 0;
}

void kgo_forget(const kg_config* c, kgo_state* st, uint32_t i, const kg_pod_columns* p, uint32_t j, int32_t zone) {
    (void)apply(c, st, i, p, j, zone, -1, NULL, NULL);
}

void kgo_replay(const kg_config* c, kgo_state* st, uint32_t base, const kg_pod_columns* p, uint32_t np,
                int32_t* out_node, int64_t* out_total, uint32_t* out_reason) {
    kg_node_columns v;
    kgo_state_view(st, &v);
    for (uint32_t j = 0; j < np; j++) {
        uint64_t best = 0;
        int32_t best_zone = -1;
        uint32_t why = 0;
        for (uint32_t i = 0; i < st->n; i++) {
            kgo_pair r;
            kgo_eval_pair(c, &v, i, p, j, &r);
            why |= r.status;
            if (r.status) continue;
            uint64_t key = make_key(r.total, base + i);
            if (key > best) {
                best = key;
                best_zone = r.zone;
            }
        }
        if (out_reason) out_reason[j] = why;
        if (!best || zone_fails(best_zone)) { /* no feasible node, or the selected node's Reserve fails */
            if (best && out_reason) out_reason[j] |= zone_fail_bits(best_zone);
            out_node[j] = -1;
            if (out_total) out_total[j] = -1;
            continue;
        }
        uint32_t g = 0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu);
        const int32_t f = apply(c, st, g - base, p, j, best_zone, 1, NULL, NULL);
        if (f) { /* the cpuset Reserve fails: the pod stays unscheduled */
            if (out_reason) out_reason[j] |= zone_fail_bits(f);
            out_node[j] = -1;
            if (out_total) out_total[j] = -1;
            continue;
        }
        out_node[j] = (int32_t)g;
        if (out_total) out_total[j] = (int64_t)(best >> 32);
    }
}

/* The CPU baseline of replay: every pod's cycle on the upstream-shaped parallelizer (kgo_select_parallel's
 * filter / score phases over n_workers threads), then its Reserve, sequentially across pods. */
int kgo_replay_parallel(const kg_config* c, kgo_state* st, uint32_t base, const kg_pod_columns* p, uint32_t np,
                        int workers, int32_t* out_node, int64_t* out_total) {
    kg_node_columns v;
    kgo_state_view(st, &v);
    par_pool pool;
    if (par_open(&pool, workers, st->n)) return -1;
    for (uint32_t j = 0; j < np; j++) {
        int32_t zone = -1;
        const uint64_t best = par_cycle(&pool, c, &v, st->n, base, p, j, &zone);
        if (!best || zone_fails(zone)) {
            out_node[j] = -1;
            if (out_total) out_total[j] = -1;
            continue;
        }
        const uint32_t g = 0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu);
        if (apply(c, st, g - base, p, j, zone, 1, NULL, NULL)) {
            out_node[j] = -1;
            if (out_total) out_total[j] = -1;
            continue;
        }
        out_node[j] = (int32_t)g;
        if (out_total) out_total[j] = (int64_t)(best >> 32);
    }
    par_close(&pool);
    return 0;
}

/* ============================================================================================== */
/* Config-5 plugins: DeviceShare (a12-a13), Reservation (a10-a11), ElasticQuota (a14)              */

#define DEVX(tab, i, r, m) ((tab)[((size_t)(i) * KG_DEV_R + (size_t)(r)) * KG_DEV_MINORS + (size_t)(m)])

/* resourceAllocationScorer.scoreNode / scoreDevice + leastResourceScorer (deviceshare/scoring.go:197-281):
 * resources with a zero total are skipped; requested = total >= free ? total - free + podRequest : total. */
static int64_t dev_least(const kg_config* c, const int64_t* total, const int64_t* free_, const int64_t* preq) {
    const int64_t* w = c->dev_w;
    int64_t score = 0, wsum = 0;
    for (int r = 0; r < KG_DEV_R; r++) {
        if (w[r] == 0 || total[r] == 0) continue;
        int64_t req = total[r] >= free_[r] ? total[r] - free_[r] + preq[r] : total[r];
        /* ScoringStrategy LeastAllocated / MostAllocated (deviceshare/scoring.go:164-181,263-323) */
        score += (c->dev_most_allocated ? most_requested_score(req, total[r]) : least_requested_score(req, total[r])) * w[r];
        wsum += w[r];
    }
    return wsum == 0 ? 0 : score / wsum;
}

static void dev_pod_req(const kg_pod_columns* p, uint32_t j, int64_t* preq, uint32_t* keys) {
    *keys = p->dev_keys ? p->dev_keys[j] : 0;
    for (int r = 0; r < KG_DEV_R; r++)
        preq[r] = ((*keys >> r) & 1u) && p->dev_req ? p->dev_req[(size_t)j * KG_DEV_R + r] : 0;
}

/* defaultAllocateDevices predicate (device_allocator.go:391-402): skip minors whose free resources are
 * all zero; quotav1.LessThanOrEqual(requestPerInstance, free) over the request's keys. */
static int dev_minor_fits(const int64_t* fr, const int64_t* preq, uint32_t keys) {
    if (fr[0] == 0 && fr[1] == 0 && fr[2] == 0) return 0;
    for (int r = 0; r < KG_DEV_R; r++)
        if (((keys >> r) & 1u) && preq[r] > fr[r]) return 0;
    return 1;
}

/* ---- GPUAllocator.Allocate (deviceshare/allocator_gpu.go:72-133) ------------------------------------
 * A device table is a pair of [KG_DEV_R][KG_DEV_MINORS] blocks (total, free) over minors 0..D-1. */

typedef struct gpu_req {
    int64_t preq[KG_DEV_R];
    uint32_t keys, n, flags;
    int64_t ring_bw;
    uint32_t tmpl; /* candidate template counts per key (kg_pod_columns.dev_tmpl) */
} gpu_req;

static void gpu_req_of(const kg_pod_columns* p, uint32_t j, gpu_req* g) {
    dev_pod_req(p, j, g->preq, &g->keys);
    g->n = p->dev_count ? p->dev_count[j] : 0;
    g->flags = p->dev_flags ? p->dev_flags[j] : 0;
    g->ring_bw = (g->flags & KG_GPU_POD_RING_BW) && p->dev_ring_bw ? p->dev_ring_bw[j] : 0;
    g->tmpl = (g->flags & KG_GPU_POD_TEMPLATE) && p->dev_tmpl ? p->dev_tmpl[j] : 0;
}

#define TAB(t, r, m) ((t)[(size_t)(r) * KG_DEV_MINORS + (size_t)(m)])

/* hashDevices(getRealUsed(original used, refined total, refined used)) (:59-70,239-254): the minors the table
 * has something used on (free != total, i.e. a deviceUsed entry), plus `outside` (minors used on the node that
 * a filtered table does not hold). */
static uint32_t used_minors_hash(const int64_t* T, const int64_t* F, int32_t D, uint32_t outside) {
    uint32_t h = outside;
    for (int32_t m = 0; m < D; m++)
        for (int r = 0; r < KG_DEV_R; r++)
            if (TAB(F, r, m) != TAB(T, r, m)) h |= 1u << m;
    return h;
}

/* hashDevices(removeZeroDevice(deviceTotal)) (:87,112-120) */
static uint32_t total_minors_hash(const int64_t* T, int32_t D) {
    uint32_t h = 0;
    for (int32_t m = 0; m < D; m++)
        for (int r = 0; r < KG_DEV_R; r++)
            if (TAB(T, r, m) != 0) h |= 1u << m;
    return h;
}

/* the partitions of table `tbl` for `ngpu` GPUs (GPUPartitionIndexer[ngpu]): entries [*b, *e) of gpu_parts */
static int part_range(const kg_node_columns* n, uint32_t tbl, uint32_t ngpu, uint32_t* b, uint32_t* e) {
    *b = *e = 0;
    int found = 0;
    for (uint32_t t = 0; n->gpu_parts && t < n->n_gpu_parts; t++) {
        const kg_gpu_partition* q = &n->gpu_parts[t];
        if (q->table != tbl || q->n_gpus != ngpu) continue;
        if (!found) *b = t;
        *e = t + 1;
        found = 1;
    }
    return found;
}

static int partition_feasible(const kg_gpu_partition* q, uint32_t used, uint32_t total, const gpu_req* g) {
    if (q->minors & used) return 0;
    if ((total & q->minors) != q->minors) return 0;
    if (g->flags & KG_GPU_POD_RING_BW) {
        if (q->ring_bw < 0) return 0;
        if (g->ring_bw > q->ring_bw) return 0;
    }
    return 1;
}

/* allocateByPartition (:177-237) + selectPartitionByBinPack (:261-296); returns 0 and the minors, or an
 * allocator code. The caller applies the honor rule of the deferred status reset. */
static uint32_t allocate_by_partition(const kg_node_columns* n, uint32_t tbl1, const gpu_req* g, uint32_t used,
                                      uint32_t total, uint32_t* mask) {
    *mask = 0;
    if (tbl1 == 0) return KG_DEV_CODE_NO_PARTITION;
    const uint32_t tbl = tbl1 - 1;
    uint32_t b, e;
    if (!part_range(n, tbl, g->n, &b, &e)) return KG_DEV_CODE_PART_COUNT;
    /* feasiblePartitions over the AllocationScore groups in ascending order, stopping after the first group
     * that adds any (or after the first group under the Restricted policy) */
    uint32_t feas[KG_GPU_MAX_PARTS];
    uint32_t nf = 0;
    uint32_t t = b;
    while (t < e) {
        uint32_t ge = t;
        while (ge < e && n->gpu_parts[ge].alloc_score == n->gpu_parts[t].alloc_score) ge++;
        for (uint32_t u = t; u < ge; u++)
            if (partition_feasible(&n->gpu_parts[u], used, total, g)) feas[nf++] = u;
        if (nf > 0 || (g->flags & KG_GPU_POD_RESTRICTED)) break;
        t = ge;
    }
    if (nf == 0) return KG_DEV_CODE_PARTITIONED;
    if (nf == 1) {
        *mask = n->gpu_parts[feas[0]].minors;
        return 0;
    }
    static const uint32_t sizes[3] = {8, 4, 2};
    static const int64_t score_of[3] = {10000, 100, 1};
    int64_t sc[KG_GPU_MAX_PARTS];
    for (uint32_t k = 0; k < nf; k++) {
        int64_t score = 0;
        const uint32_t allocated = used | n->gpu_parts[feas[k]].minors;
        for (int z = 0; z < 3; z++) {
            if (sizes[z] < g->n) continue;
            uint32_t b2, e2;
            if (!part_range(n, tbl, sizes[z], &b2, &e2)) continue;
            /* indexerOfGPUNumber[0]: the lowest AllocationScore group */
            for (uint32_t u = b2; u < e2 && n->gpu_parts[u].alloc_score == n->gpu_parts[b2].alloc_score; u++) {
                if (n->gpu_parts[u].minors & allocated) continue;
                score += score_of[z] * (int64_t)n->gpu_parts[u].alloc_score;
            }
        }
        sc[k] = score;
    }
    /* sort.Slice by BinPackScore desc: an insertion sort for <= 12 elements (stable), first maximum wins */
    uint32_t best = 0;
    for (uint32_t k = 1; k < nf; k++)
        if (sc[k] > sc[best]) best = k;
    *mask = n->gpu_parts[feas[best]].minors;
    return 0;
}

/* GPUTopologyScope (allocator_gpu_helper.go:201-262): node -> NUMA nodes (by id) -> PCIe (by id) */
typedef struct gpu_scope {
    int level;                 /* DeviceTopologyScopeLevel: node 1, NUMA node 2, PCIe 3 */
    uint32_t minors;           /* bit set; scope.minors is this set in ascending order */
    int n_children;
    struct gpu_scope* children;
} gpu_scope;

typedef struct scope_result {
    uint32_t mask;             /* allocations (0 = nil) */
    int cne, depth;
    int64_t score;
} scope_result;

typedef struct scope_ctx {
    const kg_config* c;
    const int64_t *T, *F;
    const gpu_req* g;
    int shared, level;
    uint32_t used, total;
} scope_ctx;

/* DeviceLevelContext (:404-414): satisfied = LessThanOrEqual(requestsPerGPU, free) && minor in the refined
 * total; the shared score is scoreDevice(requestsPerGPU, freeResources, totalResources) with the call site's
 * argument order (free in the total slot, total in the free slot). */
static int minor_satisfied(const scope_ctx* x, int m) {
    if (!((x->total >> m) & 1u)) return 0;
    for (int r = 0; r < KG_DEV_R; r++)
        if (((x->g->keys >> r) & 1u) && x->g->preq[r] > TAB(x->F, r, m)) return 0;
    return 1;
}

static int64_t minor_shared_score(const scope_ctx* x, int m) {
    int64_t t[KG_DEV_R], f[KG_DEV_R];
    for (int r = 0; r < KG_DEV_R; r++) {
        t[r] = TAB(x->T, r, m);
        f[r] = TAB(x->F, r, m);
    }
    return dev_least(x->c, f, t, x->g->preq);
}

static scope_result allocate_from_scope(const scope_ctx* x, const gpu_scope* sc, int cne, int depth) {
    scope_result none = {0, 0, 0, -1};
    if ((uint32_t)__builtin_popcount(sc->minors) < x->g->n) return none;
    depth++;
    if (sc->minors & x->used) cne++;
    scope_result best = none;
    int have = 0;
    for (int k = 0; k < sc->n_children; k++) {
        const gpu_scope* ch = &sc->children[k];
        if ((uint32_t)__builtin_popcount(ch->minors) < x->g->n) continue;
        scope_result r = allocate_from_scope(x, ch, cne, depth);
        if (r.mask) {
            if (!have) {
                best = r;
                have = 1;
                continue;
            }
            if (best.depth < r.depth || (best.depth == r.depth && best.cne < r.cne)) best = r;
            if (x->shared && best.depth == r.depth && best.cne == r.cne && best.score < r.score) best = r;
        }
    }
    if (have) return best;
    if (x->level > sc->level) return none;
    uint32_t cand = 0, count = 0;
    int best_minor = -1, satisfied = 0;
    int64_t best_score = -1;
    for (int m = 0; m < KG_DEV_MINORS; m++) {
        if (!((sc->minors >> m) & 1u)) continue;
        if (!minor_satisfied(x, m)) continue;
        if (!x->shared) {
            cand |= 1u << m;
            if (++count == x->g->n) {
                satisfied = 1;
                break;
            }
            continue;
        }
        satisfied = 1;
        const int64_t s = minor_shared_score(x, m);
        if (s > best_score) {
            best_minor = m;
            best_score = s;
        }
    }
    if (!satisfied) return none;
    scope_result r = {x->shared ? (best_minor >= 0 ? 1u << best_minor : 0u) : cand, cne, depth, best_score};
    return r;
}

/* build the tree of one node from dev_topo (NUMA rank in the high nibble, PCIe rank in the low one) */
static void build_scope(uint64_t topo, int32_t D, gpu_scope* root, gpu_scope* numa, gpu_scope* pcie) {
    root->level = 1;
    root->minors = D >= 32 ? ~0u : (1u << D) - 1u;
    root->n_children = 0;
    root->children = numa;
    int np = 0;
    for (uint32_t q = 0; q < 15; q++) {
        uint32_t qm = 0;
        for (int32_t m = 0; m < D; m++) {
            const uint32_t b = (uint32_t)(topo >> (8 * m)) & 0xFFu;
            if (b != KG_GPU_NO_SCOPE && (b >> 4) == q) qm |= 1u << m;
        }
        if (!qm) continue;
        gpu_scope* ns = &numa[root->n_children++];
        ns->level = 2;
        ns->minors = qm;
        ns->n_children = 0;
        ns->children = &pcie[np];
        for (uint32_t r = 0; r < 16; r++) {
            uint32_t rm = 0;
            for (int32_t m = 0; m < D; m++) {
                const uint32_t b = (uint32_t)(topo >> (8 * m)) & 0xFFu;
                if (b != KG_GPU_NO_SCOPE && (b >> 4) == q && (b & 15u) == r) rm |= 1u << m;
            }
            if (!rm) continue;
            gpu_scope* ps = &pcie[np++];
            ps->level = 3;
            ps->minors = rm;
            ps->n_children = 0;
            ps->children = NULL;
            ns->n_children++;
        }
    }
}

/* defaultAllocateDevices (device_allocator.go:355-437): scoreDevices + sortDeviceResourcesByMinor (the preferred
 * minors first, then score desc, minor asc, device_resources.go:171-209), the first numberOfGPUs minors that fit.
 * pref: requestCtx.preferred, the reserved minors of the reservation the pod allocates from (reservation.go:308). */
static uint32_t default_allocate(const kg_config* c, const int64_t* T, const int64_t* F, int32_t D, const gpu_req* g,
                                 uint32_t pref, uint32_t* mask) {
    int64_t sc[KG_DEV_MINORS];
    int order[KG_DEV_MINORS];
    for (int32_t m = 0; m < D; m++) {
        int64_t t[KG_DEV_R], f[KG_DEV_R];
        for (int r = 0; r < KG_DEV_R; r++) {
            t[r] = TAB(T, r, m);
            f[r] = TAB(F, r, m);
        }
        sc[m] = dev_least(c, t, f, g->preq);
        order[m] = m;
    }
    for (int32_t a = 1; a < D; a++) { /* stable insertion sort: preferred first, score desc (minor asc on ties) */
        int v = order[a];
        int32_t b = a;
        const int pv = (pref >> v) & 1u;
        while (b > 0 && (((pref >> order[b - 1]) & 1u) < (uint32_t)pv ||
                         (((pref >> order[b - 1]) & 1u) == (uint32_t)pv && sc[order[b - 1]] < sc[v]))) {
            order[b] = order[b - 1];
            b--;
        }
        order[b] = v;
    }
    uint32_t got = 0;
    *mask = 0;
    for (int32_t t = 0; t < D && got < g->n; t++) {
        int m = order[t];
        int64_t fr[KG_DEV_R];
        for (int r = 0; r < KG_DEV_R; r++) fr[r] = TAB(F, r, m);
        if (!dev_minor_fits(fr, g->preq, g->keys)) continue;
        *mask |= 1u << m;
        got++;
    }
    if (got < g->n) {
        *mask = 0;
        return KG_DEV_CODE_INSUFFICIENT;
    }
    return 0;
}

/* GPUAllocator.Allocate: allocateByTemplate, then allocateByPartition, then generalAllocate =
 * allocateByDeviceTopology, then defaultAllocateDevices. Returns 0 with the minors, or a KG_DEV_CODE_*. */
static uint32_t gpu_allocate(const kg_config* c, const kg_node_columns* n, uint32_t i, const int64_t* T,
                             const int64_t* F, int32_t D, uint32_t outside, const gpu_req* g, uint32_t pref,
                             uint32_t* mask) {
    *mask = 0;
    const uint32_t part = n->dev_part ? n->dev_part[i] : 0u;
    const uint64_t topo = n->dev_topo ? n->dev_topo[i] : ~0ull;
    const int shared = (g->flags & KG_GPU_POD_SHARED) != 0;
    const uint32_t sf = (g->flags >> KG_GPU_POD_SCOPE_SHIFT) & 7u;
    const int required = sf != 0; /* requiredTopologyScope != "" */
    const int level = sf > 4 ? 0 : (int)sf;
    const int honor = (g->flags & KG_GPU_POD_HONOR) || (part & KG_GPU_HONOR);
    const uint32_t used = used_minors_hash(T, F, D, outside);
    const uint32_t total = total_minors_hash(T, D);
    /* allocateByTemplate (:135-159): the pod's candidate templates under the node's vendor-model key; none
     * fails, exactly one goes straight to generalAllocate (the template name only annotates the allocation),
     * several fall through (the volcano-style choice is a TODO in the reference) */
    int by_template = 0;
    if (g->flags & KG_GPU_POD_TEMPLATE) {
        const uint32_t key = (part >> KG_GPU_TMPL_SHIFT) & 15u;
        const uint32_t cand = key == KG_GPU_TMPL_NONE ? 0u : (g->tmpl >> (2 * key)) & 3u;
        if (cand == 0) return KG_DEV_CODE_NO_TEMPLATE;
        by_template = cand == 1;
    }
    /* allocateByPartition: shared GPUs skip it; a failure stands only when partitions are honored */
    if (!shared && !by_template) {
        uint32_t code = allocate_by_partition(n, part & 0xFFu, g, used, total, mask);
        if (code == 0) return 0;
        if (honor) return code;
    }
    /* allocateByDeviceTopology (:312-337): UnschedulableAndUnresolvable statuses vanish when no scope is
     * required; an Unschedulable one (the tree found nothing) stands */
    if (!(part & KG_GPU_TREE)) {
        if (required) return KG_DEV_CODE_NO_TREE;
    } else if (shared && g->n > 1) {
        if (required) return KG_DEV_CODE_MULTI_SHARED;
    } else {
        gpu_scope root, numa[16], pcie[16 * 16];
        build_scope(topo, D, &root, numa, pcie);
        scope_ctx x = {c, T, F, g, shared, level, used, total};
        scope_result r = allocate_from_scope(&x, &root, 0, 0);
        if (r.mask) {
            *mask = r.mask;
            return 0;
        }
        return required ? KG_DEV_CODE_TOPO_SCOPED : KG_DEV_CODE_GPU_DEVICES;
    }
    return default_allocate(c, T, F, D, g, pref, mask);
}

static uint32_t dev_code_status(uint32_t code) { return code ? KG_ST_DEV_MAKE(code) : 0u; }

/* DeviceShare Filter (deviceshare/plugin.go:345-421 -> AutopilotAllocator.Allocate -> GPUAllocator.Allocate)
 * and the node Score (scoring.go:45-104 -> AutopilotAllocator.score -> scoreNode over the minor sums). */
static uint32_t dev_eval(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                         uint32_t j, int64_t* raw) {
    *raw = 0;
    gpu_req g;
    gpu_req_of(p, j, &g);
    if (g.n == 0) return 0;                                 /* PreFilter Skip */
    int32_t D = n->dev_minors ? n->dev_minors[i] : -1;
    if (D < 0) return 0;                                    /* no Device object: pass, Score 0 */
    if (D == 0) return KG_ST_DEV_NO_DEVICE;                 /* devicehandler_gpu.go:41-44 */
    const int64_t* T = &DEVX(n->dev_total, i, 0, 0);
    const int64_t* F = &DEVX(n->dev_free, i, 0, 0);
    uint32_t mask;
    const uint32_t code = gpu_allocate(c, n, i, T, F, D, 0u, &g, 0u, &mask);
    if (code) return dev_code_status(code);
    int64_t Ts[KG_DEV_R] = {0, 0, 0}, Fs[KG_DEV_R] = {0, 0, 0};
    for (int32_t m = 0; m < D; m++)
        for (int r = 0; r < KG_DEV_R; r++) {
            Ts[r] += TAB(T, r, m);
            Fs[r] += TAB(F, r, m);
        }
    *raw = dev_least(c, Ts, Fs, g.preq);
    return 0;
}

/* ---- DeviceShare under a NUMA affinity (topology_hint.go:40-290; AutopilotAllocator.filterNodeDevice,
 *      device_allocator.go:143-176; nodeDevice.filter, device_cache.go:367-415) ----------------------------- */

static uint32_t gpu_numa_nib(const kg_node_columns* n, uint32_t i, int m) {
    return n->dev_numa ? (n->dev_numa[i] >> (4 * m)) & 0xFu : KG_GPU_NUMA_NONE;
}

/* the minors filterNodeDevice keeps under a NUMA affinity (bit per NUMA node id): a Topology whose NodeID is -1
 * or in the affinity (device_allocator.go:155-159) */
static uint32_t gpu_numa_allowed(const kg_node_columns* n, uint32_t i, int32_t D, uint32_t numa) {
    uint32_t a = 0;
    for (int32_t m = 0; m < D && m < KG_DEV_MINORS; m++) {
        const uint32_t q = gpu_numa_nib(n, i, m);
        if (q == KG_GPU_NUMA_ANY || (q < KG_GPU_NUMA_ANY && ((numa >> q) & 1u))) a |= 1u << m;
    }
    return a;
}

/* The allocator on one table under NUMA affinity `numa` (0 = nil): the node's own devices (t == NULL; unfiltered
 * when numa is 0) or a reservation restore table (kg_rsv_dev, already a filtered nodeDevice). The filtered nodeDevice
 * keeps the table's minors the affinity allows; getRealUsed (allocator_gpu.go:59-70) counts the node's used minors it
 * leaves out. Returns 0 with the minors, or a KG_DEV_CODE_*. */
static uint32_t gpu_alloc_tab_numa_pref(const kg_config* c, const kg_node_columns* n, uint32_t i,
                                        const kg_pod_columns* p, uint32_t j, const kg_rsv_dev* t, uint32_t numa,
                                        uint32_t pref, uint32_t* minors) {
    gpu_req g;
    gpu_req_of(p, j, &g);
    const int32_t D = n->dev_minors[i];
    const int64_t* NT = &DEVX(n->dev_total, i, 0, 0);
    const int64_t* NF = &DEVX(n->dev_free, i, 0, 0);
    *minors = 0;
    if (D == 0) return KG_DEV_CODE_NO_DEVICE; /* Prepare: no GPU on the Device (devicehandler_gpu.go:41-44) */
    if (!t && !numa) return gpu_allocate(c, n, i, NT, NF, D, 0u, &g, pref, minors);
    const int64_t* T = t ? &t->total[0][0] : NT;
    const int64_t* F = t ? &t->free[0][0] : NF;
    const uint32_t allowed = numa ? gpu_numa_allowed(n, i, D, numa) : (D >= 32 ? ~0u : (1u << D) - 1u);
    int64_t T2[KG_DEV_R * KG_DEV_MINORS], F2[KG_DEV_R * KG_DEV_MINORS];
    uint32_t outside = 0;
    for (int m = 0; m < KG_DEV_MINORS; m++) {
        int in_tab = !t, node_used = 0;
        for (int r = 0; r < KG_DEV_R; r++) {
            if (t) in_tab |= TAB(T, r, m) != 0;
            if (m < D) node_used |= TAB(NF, r, m) != TAB(NT, r, m);
        }
        const int in = m < D && ((allowed >> m) & 1u) && in_tab;
        for (int r = 0; r < KG_DEV_R; r++) {
            TAB(T2, r, m) = in ? TAB(T, r, m) : 0;
            TAB(F2, r, m) = in ? TAB(F, r, m) : 0;
        }
        if (node_used && !in) outside |= 1u << m;
    }
    return gpu_allocate(c, n, i, T2, F2, D, outside, &g, pref, minors);
}

static uint32_t gpu_alloc_tab_numa(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                                   uint32_t j, const kg_rsv_dev* t, uint32_t numa, uint32_t* minors) {
    return gpu_alloc_tab_numa_pref(c, n, i, p, j, t, numa, 0u, minors);
}

/* DeviceShare's allocation for the pair under NUMA affinity `numa`: off views the node's devices; on a view
 * tryAllocateFromReusable over the matched reservations reserving GPUs in view order (deviceshare/reservation.go
 * :344-410), then, unless the pod requires a reservation ("Reservation(s) Insufficient gpu devices"), the allocation
 * outside them (the view's base table). 0 with the minors, or the status bits. */
static uint32_t gpu_alloc_site(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                               uint32_t j, const numa_gpu_out* gx, uint32_t numa, uint32_t* minors) {
    const kg_rsv_view* v = gx ? gx->v : NULL;
    uint32_t code;
    if (!v) {
        code = gpu_alloc_tab_numa(c, n, i, p, j, NULL, numa, minors);
        return code ? KG_ST_DEV_MAKE(code) : 0u;
    }
    if (n->dev_minors[i] == 0) return KG_ST_DEV_NO_DEVICE;
    int any = 0;
    for (uint32_t t = 0; t < v->count; t++) {
        const int32_t di = gx->e->infos[v->first + t].dev;
        if (di < 0) continue;
        any = 1;
        if (!gpu_alloc_tab_numa(c, n, i, p, j, &gx->e->devs[di], numa, minors)) return 0;
    }
    if (any && (p->flags[j] & KG_POD_RSV_REQUIRED)) return KG_ST_DEV_RSV;
    code = gpu_alloc_tab_numa(c, n, i, p, j, v->dev_base >= 0 ? &gx->e->devs[v->dev_base] : NULL, numa, minors);
    return code ? KG_ST_DEV_MAKE(code) : 0u;
}

/* AutopilotAllocator.score (device_allocator.go:486-508) on a table under NUMA affinity `numa`: scoreNode over the
 * filtered devices' sums; 0 when the filter drops the GPU type (no free left in the table; the node's unfiltered
 * devices without an affinity skip that check). t == NULL: the node's devices. */
static int64_t gpu_score_tab_numa(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                                  uint32_t j, const kg_rsv_dev* t, uint32_t numa) {
    gpu_req g;
    gpu_req_of(p, j, &g);
    const int32_t D = n->dev_minors[i];
    const int64_t* T = t ? &t->total[0][0] : &DEVX(n->dev_total, i, 0, 0);
    const int64_t* F = t ? &t->free[0][0] : &DEVX(n->dev_free, i, 0, 0);
    const int Dt = t ? KG_DEV_MINORS : D;
    const uint32_t allowed = numa ? gpu_numa_allowed(n, i, D, numa) : ~0u;
    int64_t Ts[KG_DEV_R] = {0, 0, 0}, Fs[KG_DEV_R] = {0, 0, 0};
    int any = 0;
    for (int m = 0; m < Dt; m++)
        for (int r = 0; r < KG_DEV_R; r++) {
            any |= TAB(F, r, m) != 0;
            if (!((allowed >> m) & 1u)) continue;
            Ts[r] += TAB(T, r, m);
            Fs[r] += TAB(F, r, m);
        }
    if ((t || numa) && !any) return 0;
    return dev_least(c, Ts, Fs, g.preq);
}

/* DeviceShare's Score of a feasible pair (scoring.go:45-104): on a view the nominated reservation's table (0 when it
 * reserves no GPU, scoreWithNominatedReservation) or the base table, off views the node's devices; under the stored
 * NUMA affinity. */
static int64_t gpu_score_site(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                              uint32_t j, const kgo_ext* e, const kg_rsv_view* v, uint32_t numa, int nom) {
    if (!v) return gpu_score_tab_numa(c, n, i, p, j, NULL, numa);
    if (nom >= 0) {
        const int32_t di = e->infos[v->first + (uint32_t)nom].dev;
        return di >= 0 ? gpu_score_tab_numa(c, n, i, p, j, &e->devs[di], numa) : 0;
    }
    return gpu_score_tab_numa(c, n, i, p, j, v->dev_base >= 0 ? &e->devs[v->dev_base] : NULL, numa);
}

/* AutopilotAllocator.Allocate of the pod's GPUs on the node's own devices under NUMA affinity `numa` (Reserve). */
static uint32_t gpu_alloc_numa(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                               uint32_t j, uint32_t numa, uint32_t* minors) {
    return gpu_alloc_tab_numa(c, n, i, p, j, NULL, numa, minors);
}

/* GetPodTopologyHints -> generateTopologyHints (topology_hint.go:40-66,159-280): per NUMA mask over the GPUs' NUMA
 * node ids (IterateBitMasks order), the GPUs inside must number the request ("Insufficient NUMA Scoped Devices") and
 * DeviceShare's allocation at the pair's site must succeed under the mask; Preferred = the narrowest feasible width,
 * Score 500 when the allocation equals the full mask's (hashAllocateResult). The full mask's failure is the provider's
 * status even when narrower masks fit (:191-196,271-279). */
static void gpu_numa_hints(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j,
                           const numa_gpu_out* gx, gpu_hints* h) {
    memset(h, 0, sizeof(*h));
    gpu_req g;
    gpu_req_of(p, j, &g);
    const int32_t D = n->dev_minors ? n->dev_minors[i] : -1;
    if (D < 0) { /* no nodeDevice: nil hints */
        h->nopref = 1;
        return;
    }
    uint32_t idset = 0;
    for (int32_t m = 0; m < D && m < KG_DEV_MINORS; m++) {
        const uint32_t q = gpu_numa_nib(n, i, m);
        if (q < KG_GPU_NUMA_ANY) idset |= 1u << q;
    }
    if (!idset) { /* numaTopology.nodes is empty: no mask is iterated, the hints map stays empty */
        h->nopref = 1;
        return;
    }
    int ids[8], gn = 0;
    for (int q = 0; q < 8; q++)
        if ((idset >> q) & 1u) ids[gn++] = q;
    const uint8_t* km = NUMA_MASKS[gn - 1];
    uint32_t best_alloc = 0, full_st = 0, feas[15], allocs[15];
    int minsize = gn, nf = 0;
    for (uint32_t k = 0; k < NUMA_NMASKS[gn - 1]; k++) {
        uint32_t m = 0;
        for (int b = 0; b < gn; b++)
            if ((km[k] >> b) & 1u) m |= 1u << ids[b];
        const int full = popcount32(km[k]) == gn;
        uint32_t cnt = 0;
        for (int32_t mi = 0; mi < D && mi < KG_DEV_MINORS; mi++) {
            const uint32_t q = gpu_numa_nib(n, i, mi);
            if (q < KG_GPU_NUMA_ANY && ((m >> q) & 1u)) cnt++;
        }
        if (cnt < g.n) { /* calcTotalDevicesByNUMA */
            if (full) full_st = KG_ST_DEV_MAKE(KG_DEV_CODE_NUMA_SCOPED);
            continue;
        }
        uint32_t alloc;
        const uint32_t st = gpu_alloc_site(c, n, i, p, j, gx, m, &alloc);
        if (st) {
            if (full) full_st = st;
            continue;
        }
        if (full) best_alloc = alloc;
        if (popcount32(m) < minsize) minsize = popcount32(m);
        feas[nf] = m;
        allocs[nf++] = alloc;
    }
    if (full_st || nf == 0) {
        h->fail = 1;
        h->code = full_st ? full_st : KG_ST_DEV_MAKE(KG_DEV_CODE_NUMA_SCOPED);
        return;
    }
    h->n = nf;
    for (int t = 0; t < nf; t++) {
        h->mask[t] = feas[t];
        h->pref[t] = popcount32(feas[t]) == minsize;
        h->score[t] = allocs[t] == best_alloc ? 500 : 0; /* defaultNUMAScore */
    }
}

/* kgo_gpu_numa_hints (tests): the provider's answer off reservation views as 0 = hints (n, masks, pref, scores),
 * 1 = no preference, 2 = failure (*code = the KG_DEV_CODE_* of its status). */
int kgo_gpu_numa_hints(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j,
                       int* n_out, uint32_t* masks, int* pref, int64_t* scores, uint32_t* code) {
    gpu_hints h;
    gpu_numa_hints(c, n, i, p, j, NULL, &h);
    *n_out = h.n;
    *code = KG_ST_DEV_CODE(h.code);
    for (int t = 0; t < h.n; t++) {
        masks[t] = h.mask[t];
        pref[t] = h.pref[t];
        scores[t] = h.score[t];
    }
    return h.fail ? 2 : h.nopref ? 1 : 0;
}

/* kgo_gpu_alloc_numa (tests): DeviceShare's Allocate under a NUMA affinity (topology_hint.go:100-157). */
uint32_t kgo_gpu_alloc_numa(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j,
                            uint32_t numa, uint32_t* minors) {
    return gpu_alloc_numa(c, n, i, p, j, numa, minors);
}

/* minors used on node i (free != total) that a restore table leaves out (total 0 everywhere) */
static uint32_t outside_used(const kg_node_columns* n, uint32_t i, const kg_rsv_dev* t, int32_t D) {
    uint32_t o = 0;
    for (int32_t m = 0; m < D; m++) {
        int used = 0, in_tab = 0;
        for (int r = 0; r < KG_DEV_R; r++) {
            used |= DEVX(n->dev_free, i, r, m) != DEVX(n->dev_total, i, r, m);
            in_tab |= t->total[r][m] != 0;
        }
        if (used && !in_tab) o |= 1u << m;
    }
    return o;
}

/* The same Filter and Score on one GPU restore table (kg_rsv_dev: the free / total a reservation restore
 * hands the allocator, device_cache.go:322-410). Score: AutopilotAllocator.score (device_allocator.go
 * :486-508) leaves the GPU type out when every free value is zero (nodeDevice.filter), giving 0. */
static uint32_t dev_eval_tab(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_rsv_dev* t, int32_t D,
                             const kg_pod_columns* p, uint32_t j, int64_t* raw) {
    *raw = 0;
    gpu_req g;
    gpu_req_of(p, j, &g);
    int64_t T[KG_DEV_R] = {0, 0, 0}, F[KG_DEV_R] = {0, 0, 0};
    int any = 0;
    for (int m = 0; m < KG_DEV_MINORS; m++)
        for (int r = 0; r < KG_DEV_R; r++) {
            T[r] += t->total[r][m];
            F[r] += t->free[r][m];
            any |= t->free[r][m] != 0;
        }
    *raw = any ? dev_least(c, T, F, g.preq) : 0;
    uint32_t mask;
    return dev_code_status(gpu_allocate(c, n, i, &t->total[0][0], &t->free[0][0], D, outside_used(n, i, t, D), &g, 0u, &mask));
}

/* DeviceShare Filter of a GPU pod on a reservation view (deviceshare/plugin.go:397-419):
 * tryAllocateFromReusable (reservation.go:344-410) over the matched reservations reserving GPUs in view
 * order, the first that fits wins; none fitting fails a pod with a reservation affinity ("Reservation(s)
 * Insufficient gpu devices") and sends any other pod to the allocation outside the reservations. */
static uint32_t dev_filter_view(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                                uint32_t j, const kgo_ext* e, const kg_rsv_view* v) {
    int32_t D = n->dev_minors ? n->dev_minors[i] : -1;
    if (D < 0) return 0;
    if (D == 0) return KG_ST_DEV_NO_DEVICE;
    int any = 0;
    int64_t raw;
    for (uint32_t t = 0; t < v->count; t++) {
        int32_t di = e->infos[v->first + t].dev;
        if (di < 0) continue;
        any = 1;
        if (dev_eval_tab(c, n, i, &e->devs[di], D, p, j, &raw) == 0) return 0;
    }
    if (any && (p->flags[j] & KG_POD_RSV_REQUIRED)) return KG_ST_DEV_RSV;
    if (v->dev_base >= 0) return dev_eval_tab(c, n, i, &e->devs[v->dev_base], D, p, j, &raw);
    return dev_eval(c, n, i, p, j, &raw);
}

/* Reserve-time minors: the allocation GPUAllocator.Allocate makes on node i (0 when it fails), inside the NUMA
 * affinity the topology manager stored for the pair (DeviceShare Reserve, plugin.go:585-600): the zone code of
 * the NodeNUMAResource allocation (-1 = nil affinity). */
static uint32_t dev_choose(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                           uint32_t j, int32_t zone) {
    gpu_req g;
    gpu_req_of(p, j, &g);
    int32_t D = n->dev_minors ? n->dev_minors[i] : -1;
    if (g.n == 0 || D <= 0) return 0;
    uint32_t mask;
    const uint32_t numa = (zone >= 0 && !zone_fails(zone)) ? numa_code_mask(zone) : 0u;
    const uint32_t code = gpu_alloc_numa(c, n, i, p, j, numa, &mask);
    return code ? 0u : mask;
}

/* Per-minor allocation after fillGPUTotalMem (devicehandler_gpu.go:98-135): gpu-memory from the ratio
 * (ratio * total / 100) or the ratio from gpu-memory (int64(float64(mem)/float64(total)*100)). */
int64_t kgo_mem_bytes_to_ratio(int64_t bytes, int64_t total) {
    volatile double q = (double)bytes / (double)total;
    volatile double r = q * 100.0;
    return (int64_t)r;
}

static void dev_alloc_of(const int64_t* preq, uint32_t keys, int64_t total_mem, int64_t* alloc) {
    alloc[KG_DEV_CORE] = (keys & (1u << KG_DEV_CORE)) ? preq[KG_DEV_CORE] : 0;
    int has_r = (keys & (1u << KG_DEV_RATIO)) != 0, has_m = (keys & (1u << KG_DEV_MEM)) != 0;
    if (has_r && has_m) {
        alloc[KG_DEV_RATIO] = preq[KG_DEV_RATIO];
        alloc[KG_DEV_MEM] = preq[KG_DEV_MEM];
    } else if (has_m) {
        alloc[KG_DEV_MEM] = preq[KG_DEV_MEM];
        alloc[KG_DEV_RATIO] = kgo_mem_bytes_to_ratio(preq[KG_DEV_MEM], total_mem);
    } else {
        int64_t ratio = has_r ? preq[KG_DEV_RATIO] : 0;
        alloc[KG_DEV_RATIO] = ratio;
        alloc[KG_DEV_MEM] = ratio * total_mem / 100;
    }
}

static void dev_apply(const int64_t* total_tab, int64_t* free_tab, uint32_t i, uint32_t mask, const int64_t* preq,
                      uint32_t keys, int64_t sign) {
    for (int m = 0; m < KG_DEV_MINORS; m++) {
        if (!((mask >> m) & 1u)) continue;
        int64_t a[KG_DEV_R];
        dev_alloc_of(preq, keys, DEVX(total_tab, i, KG_DEV_MEM, m), a);
        for (int r = 0; r < KG_DEV_R; r++) DEVX(free_tab, i, r, m) -= sign * a[r];
    }
}

/* ---- ElasticQuota ----------------------------------------------------------------------------- */

typedef struct kgo_quota_state {
    uint32_t n;
    const kg_quota_columns* lim;
    int64_t *used, *np_used;
    uint32_t *used_keys, *np_keys;
} kgo_quota_state;

static void quota_pod_req(const kg_pod_columns* p, uint32_t j, int64_t* req, uint32_t* keys) {
    *keys = p->quota_keys ? p->quota_keys[j] : 0;
    const int64_t v[KG_QUOTA_R] = {p->req_cpu[j], p->req_mem[j], p->sc_req[0][j], p->sc_req[1][j]};
    for (int r = 0; r < KG_QUOTA_R; r++) req[r] = ((*keys >> r) & 1u) ? v[r] : 0;
}

/* quotav1.LessThanOrEqual(a, b): every key of b that a also has must satisfy a <= b. */
static int quota_le(const int64_t* a, uint32_t akeys, const int64_t* b, uint32_t bkeys) {
    for (int r = 0; r < KG_QUOTA_R; r++)
        if (((bkeys & akeys) >> r) & 1u)
            if (a[r] > b[r]) return 0;
    return 1;
}

/* ElasticQuota PreFilter (elasticquota/plugin.go:257-309), flat quotas. */
static uint32_t quota_gate(const kgo_quota_state* q, const kg_pod_columns* p, uint32_t j) {
    int32_t qi = p->quota ? p->quota[j] : -1;
    if (qi < 0 || !q || (uint32_t)qi >= q->n) return 0;
    int64_t req[KG_QUOTA_R], a[KG_QUOTA_R];
    uint32_t rk;
    quota_pod_req(p, j, req, &rk);
    const size_t o = (size_t)qi * KG_QUOTA_R;
    for (int r = 0; r < KG_QUOTA_R; r++) a[r] = req[r] + q->used[o + r];
    if (!quota_le(a, rk | q->used_keys[qi], q->lim->used_limit + o, q->lim->limit_keys[qi])) return KG_ST_QUOTA;
    if (p->flags[j] & KG_POD_NON_PREEMPTIBLE) {
        for (int r = 0; r < KG_QUOTA_R; r++) a[r] = req[r] + q->np_used[o + r];
        if (!quota_le(a, rk | q->np_keys[qi], q->lim->min + o, q->lim->min_keys[qi])) return KG_ST_QUOTA;
    }
    return 0;
}

/* Reserve / Unreserve: GroupQuotaManager.updatePodUsedNoLock adds Mask(PodRequests, Max names) to used
 * (and non-preemptible used), never below zero (core/group_quota_manager.go:765-805,1008-1046). */
static void quota_apply(kgo_quota_state* q, const kg_pod_columns* p, uint32_t j, int64_t sign) {
    int32_t qi = p->quota ? p->quota[j] : -1;
    if (qi < 0 || !q || (uint32_t)qi >= q->n) return;
    int64_t req[KG_QUOTA_R];
    uint32_t rk;
    quota_pod_req(p, j, req, &rk);
    const size_t o = (size_t)qi * KG_QUOTA_R;
    int np = (p->flags[j] & KG_POD_NON_PREEMPTIBLE) != 0;
    for (int r = 0; r < KG_QUOTA_R; r++) {
        if (!((rk >> r) & 1u)) continue;
        int64_t u = q->used[o + r] + sign * req[r];
        q->used[o + r] = u < 0 ? 0 : u;
        if (np) {
            int64_t v = q->np_used[o + r] + sign * req[r];
            q->np_used[o + r] = v < 0 ? 0 : v;
        }
    }
    q->used_keys[qi] |= rk;
    if (np) q->np_keys[qi] |= rk;
}

static kgo_quota_state* quota_state_new(const kg_quota_columns* cols, uint32_t n) {
    if (!cols || n == 0) return NULL;
    kgo_quota_state* q = (kgo_quota_state*)calloc(1, sizeof(*q));
    q->n = n;
    q->lim = cols;
    q->used = (int64_t*)calloc((size_t)n * KG_QUOTA_R, 8);
    q->np_used = (int64_t*)calloc((size_t)n * KG_QUOTA_R, 8);
    q->used_keys = (uint32_t*)calloc(n, 4);
    q->np_keys = (uint32_t*)calloc(n, 4);
    memcpy(q->used, cols->used, (size_t)n * KG_QUOTA_R * 8);
    memcpy(q->np_used, cols->np_used, (size_t)n * KG_QUOTA_R * 8);
    memcpy(q->used_keys, cols->used_keys, (size_t)n * 4);
    memcpy(q->np_keys, cols->np_used_keys, (size_t)n * 4);
    return q;
}

static void quota_state_free(kgo_quota_state* q) {
    if (!q) return;
    free(q->used);
    free(q->np_used);
    free(q->used_keys);
    free(q->np_keys);
    free(q);
}

/* ---- Reservation ------------------------------------------------------------------------------ */

/* quotav1.ResourceNames(PodRequests) over the KG_RSV_R dimensions (keys present; scalar / ephemeral
 * requests are present when non-zero). */
static uint32_t rsv_pod_names(const kg_pod_columns* p, uint32_t j) {
    uint32_t m = 0;
    if (p->flags[j] & KG_POD_HAS_CPU) m |= 1u;
    if (p->flags[j] & KG_POD_HAS_MEM) m |= 2u;
    if (p->req_eph[j] != 0) m |= 4u;
    if (p->sc_req[0][j] != 0) m |= 8u;
    if (p->sc_req[1][j] != 0) m |= 16u;
    return m;
}

static void rsv_pod_req(const kg_pod_columns* p, uint32_t j, int64_t* r) {
    r[0] = p->req_cpu[j];
    r[1] = p->req_mem[j];
    r[2] = p->req_eph[j];
    r[3] = p->sc_req[0][j];
    r[4] = p->sc_req[1][j];
}

/* ReservationInfo.GetAvailable: max(0, Allocatable - Allocated - Reserved), reservation_info.go:516-519. */
static void rsv_remained(const kg_rsv_info* r, int64_t* out) {
    for (int k = 0; k < KG_RSV_R; k++) {
        int64_t v = r->allocatable[k] - r->allocated[k] - r->reserved[k];
        out[k] = v < 0 ? 0 : v;
    }
}

/* fitsNode (reservation/plugin.go:915-965); returns a bitmask of insufficient resources (bit 5 = pods). */
static uint32_t rsv_fits_node(const int64_t* preq, uint32_t pnames, const int64_t* alloc, int64_t allowed,
                              const int64_t* requested, const int64_t* r_alloc, const int64_t* rem, int64_t matched,
                              int64_t pods, uint32_t ign) {
    uint32_t bad = 0;
    if (pods - matched + 1 > allowed) bad |= 1u << 5;
    if (preq[0] == 0 && preq[1] == 0 && preq[2] == 0 && !(pnames & 0x18u)) return bad;
    for (int k = 0; k < KG_RSV_R; k++) {
        if (k >= 3 && !((pnames >> k) & 1u)) continue; /* scalar resources the pod requests */
        if (k >= 3 && ((ign >> (k - 3)) & 1u)) continue; /* isResourceIgnored (plugin.go:897-909,951-953) */
        if (preq[k] > alloc[k] - (requested[k] - rem[k] - r_alloc[k])) bad |= 1u << k;
    }
    return bad;
}

/* fitsReservation (reservation/plugin.go:973-1057). */
static uint32_t rsv_fits_reservation(const int64_t* preq, uint32_t pnames, const kg_rsv_info* r, uint32_t ign) {
    uint32_t bad = 0;
    if (r->max_pods >= 0 && r->allocated_pods + 1 > r->max_pods) bad |= 1u << 5;
    for (int k = 0; k < KG_RSV_R; k++) {
        if (!((r->names >> k) & 1u)) continue;
        if (k >= 3 && ((ign >> (k - 3)) & 1u)) continue; /* isResourceIgnored (:1014-1016) */
        if (!((pnames >> k) & 1u) || preq[k] == 0) continue;
        int64_t used = r->allocated[k] < 0 ? 0 : r->allocated[k];
        int64_t cap = r->allocatable[k] - r->reserved[k];
        if (preq[k] <= cap - used) continue;
        bad |= 1u << k;
    }
    return bad;
}

typedef struct rsv_ctx {
    const kg_node_columns* n;
    uint32_t i;
    const kg_rsv_view* v;
    const kg_rsv_info* infos;
    int64_t preq[KG_RSV_R], alloc[KG_RSV_R];
    uint32_t pnames;
    int required;
    uint32_t ign; /* ReservationArgs ignored scalar resources (bit k: scalar k) */
} rsv_ctx;

static void rsv_ctx_init(rsv_ctx* x, const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_rsv_view* v,
                         const kg_rsv_info* infos, const kg_pod_columns* p, uint32_t j) {
    x->ign = c->rsv_ignored_scalars;
    x->n = n;
    x->i = i;
    x->v = v;
    x->infos = infos;
    rsv_pod_req(p, j, x->preq);
    x->pnames = rsv_pod_names(p, j);
    x->required = (p->flags[j] & KG_POD_RSV_REQUIRED) != 0;
    x->alloc[0] = n->alloc_cpu[i];
    x->alloc[1] = n->alloc_mem[i];
    x->alloc[2] = n->alloc_eph[i];
    x->alloc[3] = n->sc_alloc[0][i];
    x->alloc[4] = n->sc_alloc[1][i];
}

/* fitsNodeAndReservation (reservation/plugin.go:858-895) for matched reservation r: 0 = fits. */
static int rsv_fits_one(const rsv_ctx* x, const kg_rsv_info* r, uint32_t* bn, uint32_t* br) {
    int64_t rem[KG_RSV_R];
    rsv_remained(r, rem);
    *bn = rsv_fits_node(x->preq, x->pnames, x->alloc, x->n->alloc_pods[x->i], x->v->pod_requested,
                        x->v->r_allocated, rem, (int64_t)x->v->count, x->v->num_pods, x->ign);
    *br = 0;
    if (r->policy == KG_RSV_RESTRICTED) {
        *br = rsv_fits_reservation(x->preq, x->pnames, r, x->ign);
        return (*bn == 0 && *br == 0) ? 0 : 1;
    }
    return *bn == 0 ? 0 : 1;
}

/* Reservation Filter for a normal pod (reservation/plugin.go:319-409) -> filterWithReservations
 * (:411-527); RunReservationFilterPlugins passes for cpu/memory reservations. */
static uint32_t rsv_filter(const rsv_ctx* x) {
    if (!x->v) return x->required ? KG_ST_RSV_AFFINITY : 0;
    uint32_t any_node = 0, any_resv = 0;
    for (uint32_t t = 0; t < x->v->count; t++) {
        const kg_rsv_info* r = &x->infos[x->v->first + t];
        if (!x->required && !(r->names & x->pnames)) continue;
        uint32_t bn, br;
        if (rsv_fits_one(x, r, &bn, &br) == 0) return 0;
        any_node |= bn;
        any_resv |= br;
    }
    if (x->required) return KG_ST_RSV_RESERVATION * (any_resv != 0 || any_node == 0) | (any_node ? KG_ST_RSV_NODE : 0);
    if (any_node) return KG_ST_RSV_NODE;
    int64_t zero[KG_RSV_R] = {0, 0, 0, 0, 0};
    uint32_t bn = rsv_fits_node(x->preq, x->pnames, x->alloc, x->n->alloc_pods[x->i], x->v->pod_requested,
                                x->v->r_allocated, zero, (int64_t)x->v->count, x->v->num_pods, x->ign);
    return bn ? KG_ST_RSV_NODE : 0;
}

/* findMostPreferredReservationByOrder (reservation/scoring.go:295-314): index of the smallest non-zero
 * order among infos[first, first+count) passing `ok` (NULL = all), -1 if none. */
static int rsv_most_preferred(const kg_rsv_info* infos, uint32_t first, uint32_t count, const int* ok) {
    int best = -1;
    int64_t sel = INT64_MAX;
    for (uint32_t t = 0; t < count; t++) {
        if (ok && !ok[t]) continue;
        int64_t o = infos[first + t].order;
        if (o != 0 && sel > o) {
            sel = o;
            best = (int)t;
        }
    }
    return best;
}

/* ScoreReservation (reservation/scoring.go:262-289): MostAllocated over RemoveZeros(Allocatable),
 * requested = PodRequests + Allocated, MilliValue arithmetic (cpu is milli already). */
static int64_t rsv_score_reservation(const rsv_ctx* x, const kg_rsv_info* r) {
    int64_t w = 0, s = 0;
    for (int k = 0; k < KG_RSV_R; k++) {
        int64_t cap = r->allocatable[k];
        if (cap == 0) continue;
        w++;
        int64_t req = x->preq[k] + r->allocated[k];
        if (req <= cap) {
            int64_t m = k == 0 ? 1 : 1000;
            s += (int64_t)((uint64_t)MAX_NODE_SCORE * (uint64_t)(req * m)) / (cap * m);
        }
    }
    if (r->max_pods > 0) w++; /* "pods" in Allocatable: requested pods 0 -> contributes 0 */
    if (w <= 0) return 0;
    return s / w;
}

/* Nominated reservation's score for a feasible pair (NominateReservation nominator.go:348-419 with
 * FilterNominateReservation plugin.go:1195-1212), and the node's order for preferredNode. */
static int64_t rsv_nominate_score(const rsv_ctx* x, int64_t* node_order, int* nom_index) {
    *node_order = 0;
    *nom_index = -1;
    if (!x->v || x->v->count == 0) return 0;
    const kg_rsv_info* infos = x->infos;
    const uint32_t first = x->v->first, count = x->v->count;
    int bi = rsv_most_preferred(infos, first, count, NULL);
    if (bi >= 0) *node_order = infos[first + bi].order;
    const kg_rsv_info* nom = NULL;
    if (count == 1 && x->required) {
        nom = &infos[first];
    } else {
        int ok[64];
        uint32_t nc = 0;
        int last = -1;
        for (uint32_t t = 0; t < count; t++) {
            const kg_rsv_info* r = &infos[first + t];
            ok[t] = 0;
            if (r->allocate_once && r->allocated_pods > 0) continue;
            if (!x->required && !(r->names & x->pnames)) continue;
            uint32_t bn, br;
            if (rsv_fits_one(x, r, &bn, &br) != 0) continue;
            ok[t] = 1;
            nc++;
            last = (int)t;
        }
        if (nc == 1) {
            nom = &infos[first + last];
        } else if (nc > 1) {
            int o = rsv_most_preferred(infos, first, count, ok);
            if (o >= 0) {
                nom = &infos[first + o];
            } else {
                int64_t best = -1;
                for (uint32_t t = 0; t < count; t++) {
                    if (!ok[t]) continue;
                    int64_t sc = rsv_score_reservation(x, &infos[first + t]);
                    if (sc > best) { /* stable sort by score desc: first of the maxima */
                        best = sc;
                        nom = &infos[first + t];
                    }
                }
            }
        }
    }
    if (nom) *nom_index = (int)(nom - &infos[first]);
    return nom ? rsv_score_reservation(x, nom) : 0;
}

/* ---- one pod against every node --------------------------------------------------------------- */

/* (class, node) -> view lookup table, built once per call: vidx[cls * nn + node] = view or -1. */
typedef struct view_index {
    int32_t* v;
    uint32_t nn, ncls;
} view_index;

static void view_index_build(view_index* x, const kgo_ext* e, uint32_t nn) {
    x->v = NULL;
    x->nn = nn;
    x->ncls = 0;
    if (!e || !e->views) return;
    for (uint32_t v = 0; v < e->n_views; v++)
        if (e->views[v].cls + 1 > x->ncls) x->ncls = e->views[v].cls + 1;
    if (!x->ncls) return;
    x->v = (int32_t*)malloc(sizeof(int32_t) * (size_t)x->ncls * (nn ? nn : 1));
    for (size_t t = 0; t < (size_t)x->ncls * nn; t++) x->v[t] = -1;
    for (uint32_t v = 0; v < e->n_views; v++)
        if (e->views[v].node < nn) x->v[(size_t)e->views[v].cls * nn + e->views[v].node] = (int32_t)v;
}

static const kg_rsv_view* find_view(const view_index* x, const kgo_ext* e, int32_t cls, uint32_t i) {
    if (!x || !x->v || cls < 0 || (uint32_t)cls >= x->ncls) return NULL;
    int32_t v = x->v[(size_t)cls * x->nn + i];
    return v < 0 ? NULL : &e->views[v];
}

static int64_t normalize(int64_t s, int64_t max) { return max == 0 ? s : s * MAX_NODE_SCORE / max; }

typedef struct ext_row {
    uint32_t* st;
    int64_t *nrf, *la, *numa, *dev, *rsv, *total, *order;
    int64_t* nom; /* the nominated reservation (index into the views' infos), -1 = none */
    int32_t* zone;
} ext_row;

/* Filter + raw Score of pod j on nodes [lo, hi) (qst: the pod's ElasticQuota PreFilter verdict). */
static void ext_eval_nodes(const kg_config* c, const kg_node_columns* n, uint32_t lo, uint32_t hi, const kg_pod_columns* p,
                           uint32_t j, const kgo_ext* e, const view_index* vx, uint32_t qst, ext_row* o) {
    const int32_t cls = (c->plugins & KG_PLUGIN_RSV) && p->rsv_class ? p->rsv_class[j] : -1;
    const int gpu_pod = (c->plugins & KG_PLUGIN_DEV) && p->dev_count && p->dev_count[j] > 0;
    for (uint32_t i = lo; i < hi; i++) {
        o->nrf[i] = o->la[i] = o->numa[i] = o->dev[i] = o->rsv[i] = o->order[i] = 0;
        o->nom[i] = -1;
        o->zone[i] = -1;
        o->total[i] = -1;
        if (qst) { /* PreFilter rejected the pod: no node is evaluated */
            o->st[i] = qst;
            continue;
        }
        const kg_rsv_view* v = (c->plugins & KG_PLUGIN_RSV) ? find_view(vx, e, cls, i) : NULL;
        kgo_over ov, *ovp = NULL;
        if (v) {
            for (int k = 0; k < KG_RSV_R; k++) ov.req[k] = v->req[k];
            ov.nz_cpu = v->nz_cpu;
            ov.nz_mem = v->nz_mem;
            ov.num_pods = v->num_pods;
            ovp = &ov;
        }
        uint32_t st = 0;
        int64_t s_numa = 0;
        int32_t zone = -1;
        if (c->plugins & KG_PLUGIN_NRF) st |= nrf_filter(c, n, i, ovp, p, j);
        if (c->plugins & KG_PLUGIN_LA) st |= la_filter(c, n, i, p, j);
        /* a GPU pod on a node with a Device object: DeviceShare is a NUMA hint provider there, at the pair's site
         * (its reservation view, if any). On a reservation view the
         * NodeNUMAResource restore (nodenumaresource/reservation.go:188-270) keeps only reservations whose reserve pod
         * holds a NUMA or cpuset allocation; kg_rsv_info describes none, so the plugin runs on the node's zones with
         * the view's NodeInfo. */
        const int gpu_numa = gpu_pod && n->dev_minors && n->dev_minors[i] >= 0;
        numa_gpu_out gx = {e, v, 0, 0};
        uint32_t numa_st = 0;
        if (c->plugins & KG_PLUGIN_NUMA) {
            numa_st = numa_eval(c, n, i, ovp, p, j, &s_numa, &zone, gpu_numa ? &gx : NULL);
            st |= numa_st;
        }
        int64_t dev_raw = 0;
        const int dev_view = gpu_pod && v;
        if (c->plugins & KG_PLUGIN_DEV) {
            if (gx.done) { /* the topology manager stored an affinity: DeviceShare's Filter passes (plugin.go:369-374) */
            } else {
                const uint32_t ds = dev_view ? dev_filter_view(c, n, i, p, j, e, v) : dev_eval(c, n, i, p, j, &dev_raw);
                /* NodeNUMAResource failed with DeviceShare's own reason (its hints or its Allocate): one code */
                st |= (numa_st & KG_ST_DEV_MASK) ? (ds & ~(uint32_t)KG_ST_DEV_MASK) : ds;
            }
        }
        rsv_ctx x;
        if (c->plugins & KG_PLUGIN_RSV) {
            rsv_ctx_init(&x, c, n, i, v, e ? e->infos : NULL, p, j);
            st |= rsv_filter(&x);
        }
        o->st[i] = st;
        o->nrf[i] = (c->plugins & KG_PLUGIN_NRF) ? nrf_score(c, n, i, ovp, p, j) : 0;
        o->la[i] = (c->plugins & KG_PLUGIN_LA) ? la_score(c, n, i, p, j) : 0;
        o->numa[i] = (c->plugins & KG_PLUGIN_NUMA) && !(st & (KG_ST_NUMA_MASK | KG_ST_UNSUPPORTED)) ? s_numa : 0;
        if (st) continue;
        o->zone[i] = zone;
        o->dev[i] = dev_raw;
        int nom = -1;
        if ((c->plugins & KG_PLUGIN_RSV) && v) o->rsv[i] = rsv_nominate_score(&x, &o->order[i], &nom);
        if (nom >= 0) o->nom[i] = (int64_t)v->first + nom;
        if ((c->plugins & KG_PLUGIN_DEV) && (dev_view || gx.done))
            /* DeviceShare Score (scoring.go:45-104): the nominated reservation's table (0 when it reserves no GPU:
             * scoreWithNominatedReservation, reservation.go:492-520), else the view's base table; under the stored
             * NUMA affinity */
            o->dev[i] = gpu_score_site(c, n, i, p, j, e, v, gx.done ? gx.mask : 0u, nom);
    }
}

static void ext_eval_pod(const kg_config* c, const kg_node_columns* n, uint32_t nn, const kg_pod_columns* p,
                         uint32_t j, const kgo_ext* e, const view_index* vx, const kgo_quota_state* q, ext_row* o) {
    ext_eval_nodes(c, n, 0, nn, p, j, e, vx, (c->plugins & KG_PLUGIN_QUOTA) ? quota_gate(q, p, j) : 0, o);
}

/* Worker pool of the parallel config-5 replay: one job per cycle, chunks of nodes taken by an atomic counter (the
 * reference's parallelizer.Until over the nodes, parallelism.go:29-49); the calling thread is worker 0. */
typedef struct ext_par {
    pthread_t* th;
    int n, workers, quit;
    pthread_barrier_t start, done;
    const kg_config* c;
    const kg_node_columns* nodes;
    uint32_t nn, pod, qst;
    const kg_pod_columns* p;
    const kgo_ext* e;
    const view_index* vx;
    ext_row* o;
    int chunk;
    volatile int next;
} ext_par;

static void ext_par_run(ext_par* x) {
    for (;;) {
        const int c0 = __atomic_fetch_add(&x->next, 1, __ATOMIC_RELAXED);
        const uint32_t lo = (uint32_t)c0 * (uint32_t)x->chunk;
        if (lo >= x->nn) break;
        const uint32_t hi = lo + (uint32_t)x->chunk < x->nn ? lo + (uint32_t)x->chunk : x->nn;
        ext_eval_nodes(x->c, x->nodes, lo, hi, x->p, x->pod, x->e, x->vx, x->qst, x->o);
    }
}

static void* ext_par_worker(void* arg) {
    ext_par* x = (ext_par*)arg;
    for (;;) {
        pthread_barrier_wait(&x->start);
        if (x->quit) break;
        ext_par_run(x);
        pthread_barrier_wait(&x->done);
    }
    return NULL;
}

/* PreScore preferredNode (reservation/scoring.go:113-121: smallest non-zero order among the feasible
 * nodes, first in node order) and the NormalizeScore maxima (DefaultNormalizeScore,
 * frameworkext/normalize_score.go:24-52) over this pod's feasible nodes. pref: (order + 2^31) << 32 |
 * global node index, UINT64_MAX = none; the Reservation maximum excludes the preferred node's 1000. */
static void ext_pod_stats(const ext_row* o, uint32_t nn, uint32_t base, int64_t* dev_max, int64_t* rsv_max,
                          uint64_t* pref) {
    *dev_max = 0;
    *rsv_max = 0;
    *pref = UINT64_MAX;
    for (uint32_t i = 0; i < nn; i++) {
        if (o->st[i]) continue;
        if (o->dev[i] > *dev_max) *dev_max = o->dev[i];
        if (o->rsv[i] > *rsv_max) *rsv_max = o->rsv[i];
        if (o->order[i] != 0) {
            uint64_t k = ((uint64_t)(uint32_t)(o->order[i] + 0x80000000ll) << 32) | (uint64_t)(base + i);
            if (k < *pref) *pref = k;
        }
    }
}

/* Score of the preferred node (mostPreferredScore 1000) and the weighted totals after NormalizeScore. */
static void ext_pod_totals(const kg_config* c, ext_row* o, uint32_t nn, uint32_t base, int64_t dev_max, int64_t rsv_max,
                           uint64_t pref) {
    const int has_pref = pref != UINT64_MAX;
    if (has_pref) {
        uint32_t g = (uint32_t)pref;
        if (g >= base && g - base < nn) o->rsv[g - base] = 1000;
        rsv_max = 1000;
    }
    for (uint32_t i = 0; i < nn; i++) {
        if (o->st[i]) continue;
        o->total[i] = c->weight_nrf * o->nrf[i] + c->weight_la * o->la[i] + c->weight_numa * o->numa[i] +
                      c->weight_dev * normalize(o->dev[i], dev_max) + c->weight_rsv * normalize(o->rsv[i], rsv_max);
    }
}

static void ext_pod_finish(const kg_config* c, ext_row* o, uint32_t nn, uint32_t base) {
    int64_t dm, rm;
    uint64_t pf;
    ext_pod_stats(o, nn, base, &dm, &rm, &pf);
    ext_pod_totals(c, o, nn, base, dm, rm, pf);
}

typedef struct ext_buf {
    ext_row r;
    void* mem;
} ext_buf;

static int ext_buf_new(ext_buf* b, uint32_t nn) {
    size_t m = nn ? nn : 1;
    b->mem = calloc(m, 4 + 8 * 8 + 4);
    if (!b->mem) return -1;
    int64_t* q = (int64_t*)b->mem;
    b->r.nrf = q;
    b->r.la = q + m;
    b->r.numa = q + 2 * m;
    b->r.dev = q + 3 * m;
    b->r.rsv = q + 4 * m;
    b->r.total = q + 5 * m;
    b->r.order = q + 6 * m;
    b->r.nom = q + 7 * m;
    b->r.st = (uint32_t*)(q + 8 * m);
    b->r.zone = (int32_t*)(b->r.st + m);
    return 0;
}

int kgo_ext_verify(const kg_config* c, const kg_node_columns* n, uint32_t nn, const kg_pod_columns* p, uint32_t np,
                   const kgo_ext* e, kg_verify_out* out) {
    ext_buf b;
    if (ext_buf_new(&b, nn)) return -1;
    kgo_quota_state* q = (c->plugins & KG_PLUGIN_QUOTA) && e ? quota_state_new(e->quotas, e->n_quotas) : NULL;
    view_index vx;
    view_index_build(&vx, e, nn);
    for (uint32_t j = 0; j < np; j++) {
        ext_eval_pod(c, n, nn, p, j, e, &vx, q, &b.r);
        ext_pod_finish(c, &b.r, nn, 0);
        for (uint32_t i = 0; i < nn; i++) {
            size_t x = (size_t)j * nn + i;
            if (out->status) out->status[x] = b.r.st[i];
            if (out->score_nrf) out->score_nrf[x] = b.r.nrf[i];
            if (out->score_la) out->score_la[x] = b.r.la[i];
            if (out->score_numa) out->score_numa[x] = b.r.numa[i];
            if (out->score_dev) out->score_dev[x] = b.r.dev[i];
            if (out->score_rsv) out->score_rsv[x] = b.r.rsv[i];
            if (out->total) out->total[x] = b.r.total[i];
            if (out->numa_zone) out->numa_zone[x] = (int8_t)b.r.zone[i];
        }
    }
    quota_state_free(q);
    free(vx.v);
    free(b.mem);
    return 0;
}

int kgo_ext_select(const kg_config* c, const kg_node_columns* n, uint32_t nn, uint32_t base, const kg_pod_columns* p,
                   uint32_t np, const kgo_ext* e, uint32_t k, uint64_t* keys) {
    ext_buf b;
    if (ext_buf_new(&b, nn)) return -1;
    kgo_quota_state* q = (c->plugins & KG_PLUGIN_QUOTA) && e ? quota_state_new(e->quotas, e->n_quotas) : NULL;
    view_index vx;
    view_index_build(&vx, e, nn);
    for (uint32_t j = 0; j < np; j++) {
        uint64_t* top = keys + (size_t)j * k;
        memset(top, 0, sizeof(uint64_t) * k);
        ext_eval_pod(c, n, nn, p, j, e, &vx, q, &b.r);
        ext_pod_finish(c, &b.r, nn, base);
        for (uint32_t i = 0; i < nn; i++)
            if (!b.r.st[i]) topk_insert(top, k, make_key(b.r.total[i], base + i));
    }
    free(vx.v);
    quota_state_free(q);
    free(b.mem);
    return 0;
}

/* Node-sharded two-pass selection (kg_shard_select): per-shard NormalizeScore inputs ... */
int kgo_ext_shard_stats(const kg_config* c, const kg_node_columns* n, uint32_t nn, uint32_t base,
                        const kg_pod_columns* p, uint32_t np, const kgo_ext* e, uint32_t* dev_max, uint32_t* rsv_max,
                        uint64_t* pref) {
    ext_buf b;
    if (ext_buf_new(&b, nn)) return -1;
    kgo_quota_state* q = (c->plugins & KG_PLUGIN_QUOTA) && e ? quota_state_new(e->quotas, e->n_quotas) : NULL;
    view_index vx;
    view_index_build(&vx, e, nn);
    for (uint32_t j = 0; j < np; j++) {
        ext_eval_pod(c, n, nn, p, j, e, &vx, q, &b.r);
        int64_t dm, rm;
        ext_pod_stats(&b.r, nn, base, &dm, &rm, &pref[j]);
        dev_max[j] = (uint32_t)dm;
        rsv_max[j] = (uint32_t)rm;
    }
    free(vx.v);
    quota_state_free(q);
    free(b.mem);
    return 0;
}

/* ... and the shard's top-k with the global (all-reduced) inputs. */
int kgo_ext_shard_select(const kg_config* c, const kg_node_columns* n, uint32_t nn, uint32_t base,
                         const kg_pod_columns* p, uint32_t np, const kgo_ext* e, const uint32_t* dev_max,
                         const uint32_t* rsv_max, const uint64_t* pref, uint32_t k, uint64_t* keys) {
    ext_buf b;
    if (ext_buf_new(&b, nn)) return -1;
    kgo_quota_state* q = (c->plugins & KG_PLUGIN_QUOTA) && e ? quota_state_new(e->quotas, e->n_quotas) : NULL;
    view_index vx;
    view_index_build(&vx, e, nn);
    for (uint32_t j = 0; j < np; j++) {
        uint64_t* top = keys + (size_t)j * k;
        memset(top, 0, sizeof(uint64_t) * k);
        ext_eval_pod(c, n, nn, p, j, e, &vx, q, &b.r);
        ext_pod_totals(c, &b.r, nn, base, dev_max[j], rsv_max[j], pref[j]);
        for (uint32_t i = 0; i < nn; i++)
            if (!b.r.st[i]) topk_insert(top, k, make_key(b.r.total[i], base + i));
    }
    free(vx.v);
    quota_state_free(q);
    free(b.mem);
    return 0;
}

/* Sequential scheduling with every Reserve applied before the next pod (DeviceShare minors,
 * ElasticQuota used, NodeInfo / LoadAware / NUMA). Reservation views are not replayed (their restore
 * changes with every placement): returns -1 when KG_PLUGIN_RSV is enabled. out_minors may be NULL. */
/* The reservation NominateReservation picks for pod j on node i (index into e->infos, -1 = none / infeasible pair). */
int64_t kgo_ext_pair_nominated(const kg_config* c, const kg_node_columns* n, uint32_t nn, uint32_t i,
                               const kg_pod_columns* p, uint32_t j, const kgo_ext* e) {
    ext_buf b;
    if (i >= nn || ext_buf_new(&b, nn)) return -1;
    kgo_quota_state* q = (c->plugins & KG_PLUGIN_QUOTA) && e ? quota_state_new(e->quotas, e->n_quotas) : NULL;
    view_index vx;
    view_index_build(&vx, e, nn);
    ext_eval_pod(c, n, nn, p, j, e, &vx, q, &b.r);
    const int64_t r = b.r.st[i] ? -1 : b.r.nom[i];
    free(vx.v);
    quota_state_free(q);
    free(b.mem);
    return r;
}

/* GetNonZeroRequestForResource of a reservation's Allocated for the unmatched correction
 * (updateNodeInfoRequestedForUnmatched, transformer.go:918-935; reservation_info.go:516-529,581-605): the value of a
 * present cpu / memory key, the default of a missing one */
static void rsv_nonzero(const int64_t* a, uint32_t keys, int64_t* nz) {
    nz[0] = (keys & 1u) ? a[0] : 100;
    nz[1] = (keys & 2u) ? a[1] : 200ll * 1024 * 1024;
}

/* Reservation.Reserve of pod j on node i (reservation/plugin.go:1295-1408: assumePod into the nominated reservation,
 * AddAssignedPod: Allocated += Mask(requests, ResourceNames), reservation_info.go:490-500) as the next cycle's
 * restore sees it (transformer.go:740-935). The node's NodeInfo already holds the pod (apply). Every view of the node
 * grows by the pod's requests; with a nominated reservation r the default columns and the views where r is not matched
 * give back its new Allocated share m (r's unmatched correction grows by m, its NonZeroRequested correction changes
 * with its keys), the views where r is matched keep the pod and account m in rAllocated; r's copies take m and the
 * pod. nom: index into infos of r in the pod's view, -1 = none. */
static void rsv_reserve(kgo_state* st, kg_rsv_view* views, uint32_t nv, kg_rsv_info* infos, uint32_t i,
                        const kg_pod_columns* p, uint32_t j, int64_t nom) {
    const int64_t preq[KG_RSV_R] = {p->req_cpu[j], p->req_mem[j], p->req_eph ? p->req_eph[j] : 0,
                                    p->sc_req[0] ? p->sc_req[0][j] : 0, p->sc_req[1] ? p->sc_req[1][j] : 0};
    const int64_t pnz[2] = {p->nz_cpu[j], p->nz_mem[j]};
    int64_t m[KG_RSV_R] = {0, 0, 0, 0, 0}, dnz[2] = {0, 0};
    uint32_t rid = UINT32_MAX, keys1 = 0;
    if (nom >= 0) {
        const kg_rsv_info* r = &infos[nom];
        rid = r->rid;
        for (int k = 0; k < KG_RSV_R; k++) m[k] = ((r->names >> k) & 1u) ? preq[k] : 0;
        const uint32_t f = p->flags[j];
        const uint32_t keys_m = (((f & KG_POD_HAS_CPU) && (r->names & 1u)) ? 1u : 0u) |
                                (((f & KG_POD_HAS_MEM) && (r->names & 2u)) ? 2u : 0u);
        int64_t c0[2] = {0, 0}, c1[2], a1[KG_RSV_R];
        if (r->allocated_pods > 0) rsv_nonzero(r->allocated, r->allocated_keys, c0);
        for (int k = 0; k < KG_RSV_R; k++) a1[k] = r->allocated[k] + m[k];
        keys1 = r->allocated_keys | keys_m;
        rsv_nonzero(a1, keys1, c1);
        dnz[0] = c1[0] - c0[0];
        dnz[1] = c1[1] - c0[1];
        st->col[C_REQ_CPU][i] -= m[0];
        st->col[C_REQ_MEM][i] -= m[1];
        st->col[C_REQ_EPH][i] -= m[2];
        for (int k = 0; k < KG_NSCALAR; k++) st->col[C_SC_REQ + k][i] -= m[3 + k];
        st->col[C_NZ_CPU][i] -= dnz[0];
        st->col[C_NZ_MEM][i] -= dnz[1];
    }
    for (uint32_t x = 0; x < nv; x++) {
        kg_rsv_view* v = &views[x];
        if (v->node != i) continue;
        int matched = 0;
        for (uint32_t t = v->first; t < v->first + v->count && rid != UINT32_MAX; t++) matched |= infos[t].rid == rid;
        for (int k = 0; k < KG_RSV_R; k++) {
            const int64_t d = preq[k] - (matched ? 0 : m[k]);
            v->req[k] += d;
            v->pod_requested[k] += d;
            if (matched) v->r_allocated[k] += m[k];
        }
        v->nz_cpu += pnz[0] - (matched ? 0 : dnz[0]);
        v->nz_mem += pnz[1] - (matched ? 0 : dnz[1]);
        v->num_pods += 1;
        for (uint32_t t = v->first; t < v->first + v->count && matched; t++) {
            kg_rsv_info* r = &infos[t];
            if (r->rid != rid) continue;
            for (int k = 0; k < KG_RSV_R; k++) r->allocated[k] += m[k];
            r->allocated_pods += 1;
            r->allocated_keys = keys1;
        }
    }
}

/* ---- DeviceShare restore of reservations that hold GPUs (deviceshare/reservation.go:139-198,278-380) ----------------
 * A table is [KG_DEV_R][KG_DEV_MINORS] with a minor mask (host restatement: decode.dev_effective / dev_reusable /
 * reservation_restore). The inputs (kg_rsv_gpu, mutable copies): per node its raw used (rid -1), per GPU-holding
 * reservation its allocatable, its pods' allocated, policy and assigned pods. */
#define TX(t, r, m) ((t)[(size_t)(r) * KG_DEV_MINORS + (size_t)(m)])

static uint32_t tab_minors(const int64_t* t) {
    uint32_t m = 0;
    for (int k = 0; k < KG_DEV_MINORS; k++)
        for (int r = 0; r < KG_DEV_R; r++) m |= TX(t, r, k) != 0 ? 1u << k : 0u;
    return m;
}

/* nodeDevice.calcFreeWithPreemptible + filter (device_cache.go:322-410), free = max(0, total - used) */
static void dev_effective_o(const int64_t* tot, const int64_t* used, const int64_t* pre, uint32_t pm, const int64_t* req,
                            uint32_t qm, int64_t* T, int64_t* F) {
    int merged[KG_DEV_MINORS], any = 0;
    int64_t rem[KG_DEV_R * KG_DEV_MINORS];
    for (int m = 0; m < KG_DEV_MINORS; m++) {
        int nz = 0;
        for (int r = 0; r < KG_DEV_R; r++) {
            int64_t u = TX(used, r, m) - TX(pre, r, m);
            u = u < 0 ? 0 : u;
            const int64_t x = TX(tot, r, m) - u;
            TX(rem, r, m) = x < 0 ? 0 : x;
            nz |= TX(rem, r, m) != 0;
        }
        merged[m] = ((pm >> m) & 1u) && nz;
        any |= merged[m];
    }
    for (int m = 0; m < KG_DEV_MINORS; m++)
        for (int r = 0; r < KG_DEV_R; r++) {
            int64_t f = TX(tot, r, m) - TX(used, r, m);
            f = f < 0 ? 0 : f;
            if (any && merged[m]) f = TX(rem, r, m);
            int64_t t = TX(tot, r, m);
            if (req) {
                if ((qm >> m) & 1u) f = f < TX(req, r, m) ? f : TX(req, r, m);
                else f = 0, t = 0;
            }
            TX(T, r, m) = t;
            TX(F, r, m) = f;
        }
}

typedef struct gpu_raw {
    kg_rsv_gpu* g;
    uint32_t n;
} gpu_raw;

static kg_rsv_gpu* raw_entry(gpu_raw* x, uint32_t i, int32_t rid) {
    for (uint32_t k = 0; k < x->n; k++)
        if (x->g[k].node == i && x->g[k].rid == rid) return &x->g[k];
    return NULL;
}

/* allocated masked by the allocatable minors, remained = allocatable - allocated, used part max(allocated, 0) */
static void raw_parts_o(const kg_rsv_gpu* R, int64_t* al, int64_t* rm, int64_t* up, uint32_t* am) {
    *am = tab_minors(&R->a[0][0]);
    for (int r = 0; r < KG_DEV_R; r++)
        for (int m = 0; m < KG_DEV_MINORS; m++) {
            TX(al, r, m) = ((*am >> m) & 1u) ? R->b[r][m] : 0;
            TX(rm, r, m) = R->a[r][m] - TX(al, r, m);
            TX(up, r, m) = TX(al, r, m) > 0 ? TX(al, r, m) : 0;
        }
}

/* RestoreReservation + dev_reusable of node i's views and its record (pods matching nothing) from the raw inputs */
static void gpu_rebuild_o(kgo_state* st, const kgo_ext* e, kg_rsv_dev* devs, gpu_raw* x, uint32_t i) {
    const kg_rsv_gpu* N = raw_entry(x, i, -1);
    if (!N) return;
    const int64_t* tot = &DEVX(st->dev_total, i, 0, 0);
    const int64_t* used = &N->a[0][0];
    const size_t TB = KG_DEV_R * KG_DEV_MINORS;
    int64_t pre[KG_DEV_R * KG_DEV_MINORS], al[KG_DEV_R * KG_DEV_MINORS], rm[KG_DEV_R * KG_DEV_MINORS];
    int64_t up[KG_DEV_R * KG_DEV_MINORS], T[KG_DEV_R * KG_DEV_MINORS];
    uint32_t am, pm = 0;
    memset(pre, 0, sizeof(pre));
    for (uint32_t k = 0; k < x->n; k++) {
        const kg_rsv_gpu* R = &x->g[k];
        if (R->node != i || R->rid < 0 || R->allocated_pods == 0) continue;
        raw_parts_o(R, al, rm, up, &am);
        for (size_t q = 0; q < TB; q++) pre[q] += up[q];
        pm |= tab_minors(up);
    }
    dev_effective_o(tot, used, pre, pm, NULL, 0, T, &DEVX(st->dev_free, i, 0, 0));
    for (uint32_t v = 0; v < e->n_views; v++) {
        const kg_rsv_view* vw = &e->views[v];
        if (vw->node != i || vw->dev_base < 0) continue;
        int64_t uu[KG_DEV_R * KG_DEV_MINORS], ma[KG_DEV_R * KG_DEV_MINORS], mal[KG_DEV_R * KG_DEV_MINORS];
        uint32_t uum = 0, mam = 0, malm = 0;
        memset(uu, 0, sizeof(uu));
        memset(ma, 0, sizeof(ma));
        memset(mal, 0, sizeof(mal));
        for (uint32_t k = 0; k < x->n; k++) {
            const kg_rsv_gpu* R = &x->g[k];
            if (R->node != i || R->rid < 0) continue;
            int matched = 0;
            for (uint32_t t = vw->first; t < vw->first + vw->count; t++)
                matched |= e->infos[t].dev >= 0 && (int32_t)e->infos[t].rid == R->rid;
            raw_parts_o(R, al, rm, up, &am);
            if (matched) {
                for (size_t q = 0; q < TB; q++) ma[q] += al[q], mal[q] += (&R->a[0][0])[q];
                mam |= tab_minors(al);
                malm |= am;
            } else if (R->allocated_pods > 0) {
                for (size_t q = 0; q < TB; q++) uu[q] += up[q];
                uum |= tab_minors(up);
            }
        }
        for (size_t q = 0; q < TB; q++) pre[q] = uu[q] + mal[q];
        kg_rsv_dev* b = &devs[vw->dev_base];
        dev_effective_o(tot, used, pre, uum | malm, NULL, 0, &b->total[0][0], &b->free[0][0]);
        for (uint32_t t = vw->first; t < vw->first + vw->count; t++) {
            const kg_rsv_info* I = &e->infos[t];
            if (I->dev < 0) continue;
            const kg_rsv_gpu* R = raw_entry(x, i, (int32_t)I->rid);
            if (!R) continue;
            raw_parts_o(R, al, rm, up, &am);
            const uint32_t rmask = tab_minors(rm);
            for (size_t q = 0; q < TB; q++) pre[q] = uu[q] + ma[q] + rm[q];
            kg_rsv_dev* d = &devs[I->dev];
            if (R->policy == KG_RSV_RESTRICTED) {
                int64_t req[KG_DEV_R * KG_DEV_MINORS];
                for (int r = 0; r < KG_DEV_R; r++)
                    for (int m = 0; m < KG_DEV_MINORS; m++) TX(req, r, m) = ((rmask >> m) & 1u) ? TX(rm, r, m) : 0;
                dev_effective_o(tot, used, pre, uum | mam | rmask, req, (rmask ? rmask : am) & am, &d->total[0][0],
                                &d->free[0][0]);
            } else {
                dev_effective_o(tot, used, pre, uum | mam | rmask, NULL, 0, &d->total[0][0], &d->free[0][0]);
            }
        }
    }
}

/* DeviceShare's allocate at Reserve (plugin.go:573-637): the nominated reservation's table when it holds GPUs
 * (allocateWithNominated, not required), else or on failure outside (the view's base table, off views the node's) */
static uint32_t dev_choose_site_o(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                                  uint32_t j, const kgo_ext* e, const kg_rsv_view* v, int64_t nom, int32_t zone) {
    gpu_req g;
    gpu_req_of(p, j, &g);
    const int32_t D = n->dev_minors ? n->dev_minors[i] : -1;
    if (g.n == 0 || D <= 0) return 0;
    const uint32_t numa = (zone >= 0 && !zone_fails(zone)) ? numa_code_mask(zone) : 0u;
    uint32_t mask;
    /* the reservation's reserved minors first (tryAllocateFromReusable's preferred set) */
    if (v && nom >= 0 && e->infos[nom].dev >= 0 &&
        !gpu_alloc_tab_numa_pref(c, n, i, p, j, &e->devs[e->infos[nom].dev], numa, e->infos[nom].dev_minors, &mask))
        return mask;
    const uint32_t code = gpu_alloc_tab_numa(c, n, i, p, j, (v && v->dev_base >= 0) ? &e->devs[v->dev_base] : NULL, numa, &mask);
    return code ? 0u : mask;
}

/* A pod's Reserve on a node with GPU-holding reservations: used += its minors' allocation (updateCacheUsed), the
 * reservation it joined (rid) counts the allocation on its own minors (appendAllocatedByHints) and one more pod, then
 * the tables are rebuilt (every pod: the assigned pod count decides which reservations are unmatched with pods) */
static void gpu_apply_o(kgo_state* st, const kgo_ext* e, kg_rsv_dev* devs, gpu_raw* x, uint32_t i, uint32_t mask,
                        const kg_pod_columns* p, uint32_t j, int32_t rid, int64_t sign) {
    kg_rsv_gpu* N = raw_entry(x, i, -1);
    if (!N) return;
    kg_rsv_gpu* R = rid >= 0 ? raw_entry(x, i, rid) : NULL;
    const uint32_t hints = R ? tab_minors(&R->a[0][0]) : 0u;
    int64_t preq[KG_DEV_R];
    uint32_t keys;
    dev_pod_req(p, j, preq, &keys);
    for (int m = 0; m < KG_DEV_MINORS; m++) {
        if (!((mask >> m) & 1u)) continue;
        int64_t a[KG_DEV_R];
        dev_alloc_of(preq, keys, DEVX(st->dev_total, i, KG_DEV_MEM, m), a);
        for (int r = 0; r < KG_DEV_R; r++) {
            /* the Unreserve (sign -1): updateCacheUsed(add=false) subtracts with a non-negative result, and the pod
             * leaves the reservation's AssignedPods (its allocation no longer counts in allocated) */
            const int64_t u = N->a[r][m] + sign * a[r];
            N->a[r][m] = u < 0 ? 0 : u;
            if (R && ((hints >> m) & 1u)) {
                const int64_t b = R->b[r][m] + sign * a[r];
                R->b[r][m] = b < 0 ? 0 : b;
            }
        }
    }
    if (R) R->allocated_pods = sign > 0 ? R->allocated_pods + 1 : (R->allocated_pods > 0 ? R->allocated_pods - 1 : 0);
    gpu_rebuild_o(st, e, devs, x, i);
}

/* Reservations holding GPUs: their DeviceShare restore tables derive from the reserve pods' and assigned pods' GPU
 * allocations, so the replay and the batch cycle follow them only with the raw inputs (kgo_ext.gpu). */
static int rsv_has_gpu_tables(const kgo_ext* e) {
    if (!e) return 0;
    for (uint32_t v = 0; v < e->n_views; v++)
        if (e->views[v].dev_base >= 0) return 1;
    for (uint32_t t = 0; t < e->n_infos; t++)
        if (e->infos[t].dev >= 0) return 1;
    return 0;
}

static int ext_replay_impl(const kg_config* c, kgo_state* st, uint32_t base, const kg_pod_columns* p, uint32_t np,
                           const kgo_ext* e, int32_t* out_node, int64_t* out_total, uint32_t* out_minors,
                           int64_t* quota_used_out, int64_t* quota_np_used_out, uint32_t* out_reason, int workers);

int kgo_ext_replay(const kg_config* c, kgo_state* st, uint32_t base, const kg_pod_columns* p, uint32_t np,
                   const kgo_ext* e, int32_t* out_node, int64_t* out_total, uint32_t* out_minors,
                   int64_t* quota_used_out, int64_t* quota_np_used_out, uint32_t* out_reason) {
    return ext_replay_impl(c, st, base, p, np, e, out_node, out_total, out_minors, quota_used_out, quota_np_used_out,
                           out_reason, 1);
}

/* kgo_ext_replay with each cycle's Filter / Score over the nodes on `workers` threads (the Reserve between cycles
 * stays serial): the CPU baseline of the config-5 replay, same results. */
int kgo_ext_replay_parallel(const kg_config* c, kgo_state* st, uint32_t base, const kg_pod_columns* p, uint32_t np,
                            const kgo_ext* e, int32_t* out_node, int64_t* out_total, uint32_t* out_minors,
                            int64_t* quota_used_out, int64_t* quota_np_used_out, uint32_t* out_reason, int workers) {
    return ext_replay_impl(c, st, base, p, np, e, out_node, out_total, out_minors, quota_used_out, quota_np_used_out,
                           out_reason, workers);
}

static int ext_replay_impl(const kg_config* c, kgo_state* st, uint32_t base, const kg_pod_columns* p, uint32_t np,
                           const kgo_ext* e, int32_t* out_node, int64_t* out_total, uint32_t* out_minors,
                           int64_t* quota_used_out, int64_t* quota_np_used_out, uint32_t* out_reason, int workers) {
    const int rsv = (c->plugins & KG_PLUGIN_RSV) != 0;
    if (rsv && rsv_has_gpu_tables(e) && !e->n_gpu) return -1;
    kg_node_columns v;
    kgo_state_view(st, &v);
    ext_buf b;
    if (ext_buf_new(&b, st->n)) return -1;
    kgo_quota_state* q = (c->plugins & KG_PLUGIN_QUOTA) && e ? quota_state_new(e->quotas, e->n_quotas) : NULL;
    /* mutable copies of the views, their reservations, the GPU restore tables and inputs (the Reserve updates them) */
    kgo_ext e2;
    kg_rsv_view* mv = NULL;
    kg_rsv_info* mi = NULL;
    kg_rsv_dev* md = NULL;
    gpu_raw gx = {NULL, 0};
    view_index vx = {NULL, 0, 0};
    const kgo_ext* ee = e;
    if (rsv && e) {
        e2 = *e;
        mv = (kg_rsv_view*)malloc(sizeof(kg_rsv_view) * (e->n_views ? e->n_views : 1));
        mi = (kg_rsv_info*)malloc(sizeof(kg_rsv_info) * (e->n_infos ? e->n_infos : 1));
        md = (kg_rsv_dev*)malloc(sizeof(kg_rsv_dev) * (e->n_devs ? e->n_devs : 1));
        if (e->n_views) memcpy(mv, e->views, sizeof(kg_rsv_view) * e->n_views);
        if (e->n_infos) memcpy(mi, e->infos, sizeof(kg_rsv_info) * e->n_infos);
        if (e->n_devs) memcpy(md, e->devs, sizeof(kg_rsv_dev) * e->n_devs);
        gx.n = e->n_gpu;
        gx.g = (kg_rsv_gpu*)malloc(sizeof(kg_rsv_gpu) * (e->n_gpu ? e->n_gpu : 1));
        if (e->n_gpu) memcpy(gx.g, e->gpu, sizeof(kg_rsv_gpu) * e->n_gpu);
        e2.views = mv;
        e2.infos = mi;
        e2.devs = md;
        ee = &e2;
        view_index_build(&vx, ee, st->n);
    }
    ext_par par;
    memset(&par, 0, sizeof(par));
    if (workers > 1) {
        par.workers = workers;
        par.n = workers - 1;
        par.th = (pthread_t*)calloc((size_t)par.n, sizeof(pthread_t));
        pthread_barrier_init(&par.start, NULL, (unsigned)workers);
        pthread_barrier_init(&par.done, NULL, (unsigned)workers);
        for (int t = 0; t < par.n; t++) pthread_create(&par.th[t], NULL, ext_par_worker, &par);
    }
    for (uint32_t j = 0; j < np; j++) {
        if (workers > 1) {
            par.c = c;
            par.nodes = &v;
            par.nn = st->n;
            par.pod = j;
            par.qst = (c->plugins & KG_PLUGIN_QUOTA) ? quota_gate(q, p, j) : 0;
            par.p = p;
            par.e = ee;
            par.vx = rsv ? &vx : NULL;
            par.o = &b.r;
            par.chunk = chunk_size((int)st->n, workers);
            par.next = 0;
            pthread_barrier_wait(&par.start);
            ext_par_run(&par);
            pthread_barrier_wait(&par.done);
        } else {
            ext_eval_pod(c, &v, st->n, p, j, ee, rsv ? &vx : NULL, q, &b.r);
        }
        ext_pod_finish(c, &b.r, st->n, base);
        uint64_t best = 0;
        int32_t best_zone = -1;
        uint32_t why = 0;
        for (uint32_t i = 0; i < st->n; i++) {
            why |= b.r.st[i];
            if (b.r.st[i]) continue;
            uint64_t key = make_key(b.r.total[i], base + i);
            if (key > best) {
                best = key;
                best_zone = b.r.zone[i];
            }
        }
        if (out_minors) out_minors[j] = 0;
        if (out_reason) out_reason[j] = why;
        if (!best || zone_fails(best_zone)) { /* no feasible node, or the selected node's Reserve fails */
            if (best && out_reason) out_reason[j] |= zone_fail_bits(best_zone);
            out_node[j] = -1;
            if (out_total) out_total[j] = -1;
            continue;
        }
        uint32_t g = 0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu);
        uint32_t i = g - base;
        const int32_t f = apply(c, st, i, p, j, best_zone, 1, NULL, NULL);
        if (f) { /* the cpuset Reserve fails: the pod stays unscheduled */
            if (out_reason) out_reason[j] |= zone_fail_bits(f);
            out_node[j] = -1;
            if (out_total) out_total[j] = -1;
            continue;
        }
        out_node[j] = (int32_t)g;
        if (out_total) out_total[j] = (int64_t)(best >> 32);
        const int64_t nom = b.r.nom[i];
        const int raw = rsv && mv && raw_entry(&gx, i, -1) != NULL;
        uint32_t mask = 0;
        if ((c->plugins & KG_PLUGIN_DEV) && p->dev_count && p->dev_count[j] > 0 && st->dev_minors &&
            st->dev_minors[i] > 0) {
            const int32_t cls = p->rsv_class ? p->rsv_class[j] : -1;
            const kg_rsv_view* vw = (rsv && mv) ? find_view(&vx, ee, cls, i) : NULL;
            mask = dev_choose_site_o(c, &v, i, p, j, ee, vw, nom, best_zone);
            if (!raw) {
                int64_t preq[KG_DEV_R];
                uint32_t keys;
                dev_pod_req(p, j, preq, &keys);
                dev_apply(st->dev_total, st->dev_free, i, mask, preq, keys, 1);
            }
            if (out_minors) out_minors[j] = mask;
        }
        quota_apply(q, p, j, 1);
        if (rsv && mv) rsv_reserve(st, mv, ee->n_views, mi, i, p, j, nom);
        if (raw) gpu_apply_o(st, ee, md, &gx, i, mask, p, j, nom >= 0 ? (int32_t)mi[nom].rid : -1, 1);
    }
    if (workers > 1) {
        par.quit = 1;
        pthread_barrier_wait(&par.start);
        for (int t = 0; t < par.n; t++) pthread_join(par.th[t], NULL);
        pthread_barrier_destroy(&par.start);
        pthread_barrier_destroy(&par.done);
        free(par.th);
    }
    free(vx.v);
    free(mv);
    free(mi);
    free(md);
    free(gx.g);
    if (q) {
        if (quota_used_out) memcpy(quota_used_out, q->used, (size_t)q->n * KG_QUOTA_R * 8);
        if (quota_np_used_out) memcpy(quota_np_used_out, q->np_used, (size_t)q->n * KG_QUOTA_R * 8);
    }
    quota_state_free(q);
    free(b.mem);
    return 0;
}

/* Inline batch scheduling cycle of a planned job: batch/engine.go:92-294 RunSchedulingCycle with the
 * grouping of ValidateAndGroupByRequest (:348-371) and the cleanup of batch_scheduler.go:146-152.
 * Pods are grouped by plan_node (groups in order of first appearance, each in batch order; the caller
 * orders a node's pods by name). Per pod: PreFilter (ElasticQuota gate on the current used,
 * elasticquota/plugin.go:257-309) and Filter on the planned node (every enabled plugin), then Reserve
 * (NodeInfo / LoadAware / NUMA, DeviceShare minors in scoreDevice order, quota used). The first failure
 * of a group gives its later pods the same status (engine.go:188-192). If any pod failed, every Reserve is
 * undone (CleanupAssumedPods): here by restoring the state copied before the cycle. Codes are the ABI's
 * KG_BATCH_*. Groups run one after another, as lane 0 of k_batch does when ElasticQuota is on; without
 * quota the groups touch disjoint nodes, so their order changes nothing. With reservation views each Reserve also
 * runs Reservation.Reserve on the node's views (rsv_reserve); -1 while a reservation holds GPUs. */
int kgo_batch_schedule(const kg_config* c, kgo_state* st, const kg_pod_columns* p, uint32_t np, const kgo_ext* e,
                       const int32_t* plan_node, uint32_t* out_result, uint32_t* out_status, int32_t* out_zone,
                       uint32_t* out_minors, int64_t* quota_used_out, int64_t* quota_np_used_out) {
    const int rsv = (c->plugins & KG_PLUGIN_RSV) != 0 && e && e->n_views;
    if (rsv && rsv_has_gpu_tables(e) && !e->n_gpu) return -1;
    for (uint32_t j = 0; j < np; j++) {
        out_zone[j] = -1;
        out_minors[j] = 0;
        out_status[j] = 0;
    }
    for (uint32_t j = 0; j < np; j++)
        if (plan_node[j] < 0) { /* batch_scheduler.go:96-101: nothing is assumed */
            for (uint32_t k = 0; k < np; k++) out_result[k] = KG_BATCH_NO_PLAN;
            return 0;
        }
    const int ext = (c->plugins & KG_PLUGIN_EXT) != 0;
    kgo_quota_state* q = (c->plugins & KG_PLUGIN_QUOTA) && e ? quota_state_new(e->quotas, e->n_quotas) : NULL;
    /* the state before the cycle, for the cleanup */
    kg_node_columns v;
    kgo_state_view(st, &v);
    kgo_state* saved = kgo_state_new(&v, st->n);
    ext_buf b;
    if (ext_buf_new(&b, st->n)) return -1;
    /* mutable copies of the views and their reservations (Reservation.Reserve updates them; a cleanup drops them) */
    kgo_ext e2;
    kg_rsv_view* mv = NULL;
    kg_rsv_info* mi = NULL;
    kg_rsv_dev* md = NULL;
    gpu_raw gx = {NULL, 0};
    view_index vx = {NULL, 0, 0};
    const kgo_ext* ee = e;
    if (rsv) {
        e2 = *e;
        mv = (kg_rsv_view*)malloc(sizeof(kg_rsv_view) * e->n_views);
        mi = (kg_rsv_info*)malloc(sizeof(kg_rsv_info) * (e->n_infos ? e->n_infos : 1));
        md = (kg_rsv_dev*)malloc(sizeof(kg_rsv_dev) * (e->n_devs ? e->n_devs : 1));
        memcpy(mv, e->views, sizeof(kg_rsv_view) * e->n_views);
        if (e->n_infos) memcpy(mi, e->infos, sizeof(kg_rsv_info) * e->n_infos);
        if (e->n_devs) memcpy(md, e->devs, sizeof(kg_rsv_dev) * e->n_devs);
        gx.n = e->n_gpu;
        gx.g = (kg_rsv_gpu*)malloc(sizeof(kg_rsv_gpu) * (e->n_gpu ? e->n_gpu : 1));
        if (e->n_gpu) memcpy(gx.g, e->gpu, sizeof(kg_rsv_gpu) * e->n_gpu);
        e2.views = mv;
        e2.infos = mi;
        e2.devs = md;
        ee = &e2;
        view_index_build(&vx, ee, st->n);
    }
    uint8_t* done = (uint8_t*)calloc(np ? np : 1, 1);
    int failed_any = 0;
    for (uint32_t j0 = 0; j0 < np; j0++) {
        if (done[j0]) continue;
        const int32_t node = plan_node[j0];
        uint32_t failed = 0;
        for (uint32_t j = j0; j < np; j++) {
            if (done[j] || plan_node[j] != node) continue;
            done[j] = 1;
            if (failed) {
                out_result[j] = KG_BATCH_SIBLING;
                out_status[j] = failed;
                continue;
            }
            kgo_state_view(st, &v);
            uint32_t s;
            int32_t zone;
            if (ext) {
                ext_eval_pod(c, &v, st->n, p, j, ee, rsv ? &vx : NULL, q, &b.r);
                s = b.r.st[node];
                zone = b.r.zone[node];
            } else {
                kgo_pair o;
                kgo_eval_pair(c, &v, (uint32_t)node, p, j, &o);
                s = o.status;
                zone = o.zone;
            }
            if (!s && zone_fails(zone)) s = zone_fail_bits(zone); /* the Reserve fails (engine.go:275-283) */
            if (s) {
                failed = s;
                failed_any = 1;
                out_result[j] = KG_BATCH_FAILED;
                out_status[j] = s;
                continue;
            }
            const int32_t f = apply(c, st, (uint32_t)node, p, j, zone, 1, NULL, NULL);
            if (f) { /* the cpuset Reserve fails */
                failed = zone_fail_bits(f);
                failed_any = 1;
                out_result[j] = KG_BATCH_FAILED;
                out_status[j] = failed;
                continue;
            }
            const int64_t nom = ext ? b.r.nom[node] : -1;
            const int raw = rsv && raw_entry(&gx, (uint32_t)node, -1) != NULL;
            uint32_t mask = 0;
            if ((c->plugins & KG_PLUGIN_DEV) && p->dev_count && p->dev_count[j] > 0 && st->dev_minors &&
                st->dev_minors[node] > 0) {
                int64_t preq[KG_DEV_R];
                uint32_t keys;
                dev_pod_req(p, j, preq, &keys);
                kg_node_columns nv;
                kgo_state_view(st, &nv);
                const int32_t cls = p->rsv_class ? p->rsv_class[j] : -1;
                const kg_rsv_view* vw = rsv ? find_view(&vx, ee, cls, (uint32_t)node) : NULL;
                mask = dev_choose_site_o(c, &nv, (uint32_t)node, p, j, ee, vw, nom, zone);
                if (!raw) dev_apply(st->dev_total, st->dev_free, (uint32_t)node, mask, preq, keys, 1);
                out_minors[j] = mask;
            }
            quota_apply(q, p, j, 1);
            if (rsv) rsv_reserve(st, mv, ee->n_views, mi, (uint32_t)node, p, j, nom);
            if (raw) gpu_apply_o(st, ee, md, &gx, (uint32_t)node, mask, p, j, nom >= 0 ? (int32_t)mi[nom].rid : -1, 1);
            out_result[j] = KG_BATCH_ASSUMED;
            out_zone[j] = zone;
        }
    }
    if (failed_any) {
        kgo_state_view(saved, &v);
        kgo_state* fresh = kgo_state_new(&v, st->n);
        kgo_state tmp = *st;
        *st = *fresh;
        *fresh = tmp;
        kgo_state_free(fresh);
        for (uint32_t j = 0; j < np; j++)
            if (out_result[j] == KG_BATCH_ASSUMED) out_result[j] = KG_BATCH_ROLLED_BACK;
        if (q) {
            quota_state_free(q);
            q = quota_state_new(e->quotas, e->n_quotas);
        }
    }
    if (q) {
        if (quota_used_out) memcpy(quota_used_out, q->used, (size_t)q->n * KG_QUOTA_R * 8);
        if (quota_np_used_out) memcpy(quota_np_used_out, q->np_used, (size_t)q->n * KG_QUOTA_R * 8);
    }
    quota_state_free(q);
    kgo_state_free(saved);
    free(vx.v);
    free(mv);
    free(mi);
    free(md);
    free(gx.g);
    free(done);
    free(b.mem);
    return 0;
}

/* Reserve of pod j on node i with the plugins kgo_state holds (NodeInfo, LoadAware, NodeNUMAResource incl. cpusets,
 * DeviceShare minors; no quota or reservation state) and the record its Unreserve gives back (kg_reserve_record): 0,
 * or 1 when the NodeNUMAResource Reserve fails (nothing applied; rec->numa_zone holds the failing zone code). */
int kgo_reserve(const kg_config* c, kgo_state* st, uint32_t i, const kg_pod_columns* p, uint32_t j, kg_reserve_record* rec) {
    memset(rec, 0, sizeof(*rec));
    rec->numa_zone = -1;
    rec->rsv_rid = -1;
    kg_node_columns v;
    kgo_state_view(st, &v);
    int32_t zone;
    if (c->plugins & KG_PLUGIN_DEV) { /* DeviceShare joins the NUMA hints: the config-5 evaluation of the pair */
        ext_buf b;
        if (ext_buf_new(&b, st->n)) return -1;
        kg_config c2 = *c;
        c2.plugins &= ~(KG_PLUGIN_QUOTA | KG_PLUGIN_RSV);
        ext_eval_pod(&c2, &v, st->n, p, j, NULL, NULL, NULL, &b.r);
        zone = b.r.st[i] ? -1 : b.r.zone[i];
        free(b.mem);
    } else {
        kgo_pair r;
        kgo_eval_pair(c, &v, i, p, j, &r);
        zone = r.status ? -1 : r.zone;
    }
    rec->numa_zone = zone;
    if (zone_fails(zone)) return 1;
    uint32_t mask = 0;
    if ((c->plugins & KG_PLUGIN_DEV) && p->dev_count && p->dev_count[j] > 0 && st->dev_minors && st->dev_minors[i] > 0)
        mask = dev_choose(c, &v, i, p, j, zone);
    uint64_t cpus[4] = {0, 0, 0, 0};
    int64_t amounts[2 * KG_MAX_ZONES] = {0};
    const int32_t f = apply(c, st, i, p, j, zone, 1, amounts, cpus);
    if (f) {
        rec->numa_zone = f;
        return 1;
    }
    if (mask) {
        int64_t preq[KG_DEV_R];
        uint32_t keys;
        dev_pod_req(p, j, preq, &keys);
        dev_apply(st->dev_total, st->dev_free, i, mask, preq, keys, 1);
    }
    rec->gpu_minors = mask;
    memcpy(rec->zone_amounts, amounts, sizeof(amounts));
    memcpy(rec->cpus, cpus, sizeof(cpus));
    if (cpus[0] | cpus[1] | cpus[2] | cpus[3]) rec->flags |= KG_RECORD_CPUSET;
    return 0;
}

/* Unreserve of a kgo_reserve: NodeInfo / LoadAware (RemovePod, podAssignCache.unAssign), NodeNUMAResource Release of
 * the recorded NUMA amounts and cpuset CPUs (resource_manager.go:478-483, node_allocation.go:164-200), the DeviceShare
 * minors. */
void kgo_unreserve(const kg_config* c, kgo_state* st, uint32_t i, const kg_pod_columns* p, uint32_t j,
                   const kg_reserve_record* rec) {
    int64_t amounts[2 * KG_MAX_ZONES];
    uint64_t cpus[4];
    memcpy(amounts, rec->zone_amounts, sizeof(amounts));
    memcpy(cpus, rec->cpus, sizeof(cpus));
    int any = 0;
    for (int z = 0; z < 2 * KG_MAX_ZONES; z++) any |= amounts[z] != 0;
    const int32_t zone = rec->numa_zone < 0 ? -1 : any ? 0x4F : rec->numa_zone;
    (void)apply(c, st, i, p, j, zone, -1, any ? amounts : NULL, (rec->flags & KG_RECORD_CPUSET) ? cpus : NULL);
    if (rec->gpu_minors && st->dev_total) {
        int64_t preq[KG_DEV_R];
        uint32_t keys;
        dev_pod_req(p, j, preq, &keys);
        dev_apply(st->dev_total, st->dev_free, i, rec->gpu_minors, preq, keys, -1);
    }
}

/* ---- Reserve / Unreserve with every config-5 plugin (a session over one kgo_state) ------------------------------------ */

/* Reservation.Unreserve of pod j on node i (reservation/plugin.go:1409-1460 -> reservationCache.forgetPods ->
 * ReservationInfo.RemoveAssignedPod, frameworkext/reservation_info.go:502-514): the reservation rid the pod joined loses
 * Mask(requests, ResourceNames) from Allocated (quotav1.SubtractWithNonNegativeResult; its keys stay) and one assigned
 * pod. The next cycle's restore (transformer.go:740-935) then sees the node through it: NodeInfo no longer holds the pod
 * (apply has removed it from the state's columns); the reservation's unmatched correction (restoreUnmatchedReservations
 * :891-903: Allocated and its NonZeroRequested while it has assigned pods, nothing after the last) changes from its old
 * to its new value in the record's columns and in the views that do not match it; the views that match it lose the pod
 * and count the new Allocated in rAllocated (:786-790); every view of the node has one pod less. rid -1: the pod joined
 * no reservation (only the pod leaves the views). */
static void rsv_unreserve(kgo_state* st, kg_rsv_view* views, uint32_t nv, kg_rsv_info* infos, uint32_t i,
                          const kg_pod_columns* p, uint32_t j, int32_t rid) {
    const int64_t preq[KG_RSV_R] = {p->req_cpu[j], p->req_mem[j], p->req_eph ? p->req_eph[j] : 0,
                                    p->sc_req[0] ? p->sc_req[0][j] : 0, p->sc_req[1] ? p->sc_req[1][j] : 0};
    const int64_t pnz[2] = {p->nz_cpu[j], p->nz_mem[j]};
    /* the reservation as the node's views hold it (its copies agree) */
    const kg_rsv_info* r = NULL;
    for (uint32_t x = 0; x < nv && rid >= 0 && !r; x++) {
        if (views[x].node != i) continue;
        for (uint32_t t = views[x].first; t < views[x].first + views[x].count; t++)
            if ((int32_t)infos[t].rid == rid) {
                r = &infos[t];
                break;
            }
    }
    int64_t old_a[KG_RSV_R] = {0}, new_a[KG_RSV_R] = {0}, corr0[KG_RSV_R] = {0}, corr1[KG_RSV_R] = {0};
    int64_t nz0[2] = {0, 0}, nz1[2] = {0, 0}, pods1 = 0;
    uint32_t keys = 0;
    if (r) {
        keys = r->allocated_keys;
        const int64_t pods0 = r->allocated_pods;
        pods1 = pods0 > 0 ? pods0 - 1 : 0;
        for (int k = 0; k < KG_RSV_R; k++) {
            const int64_t m = ((r->names >> k) & 1u) ? preq[k] : 0;
            old_a[k] = r->allocated[k];
            new_a[k] = old_a[k] - m < 0 ? 0 : old_a[k] - m;
            corr0[k] = pods0 > 0 ? old_a[k] : 0;
            corr1[k] = pods1 > 0 ? new_a[k] : 0;
        }
        if (pods0 > 0) rsv_nonzero(old_a, keys, nz0);
        if (pods1 > 0) rsv_nonzero(new_a, keys, nz1);
        /* the record (pods matching nothing): the correction is subtracted from NodeInfo's Requested */
        st->col[C_REQ_CPU][i] -= corr1[0] - corr0[0];
        st->col[C_REQ_MEM][i] -= corr1[1] - corr0[1];
        st->col[C_REQ_EPH][i] -= corr1[2] - corr0[2];
        for (int k = 0; k < KG_NSCALAR; k++) st->col[C_SC_REQ + k][i] -= corr1[3 + k] - corr0[3 + k];
        st->col[C_NZ_CPU][i] -= nz1[0] - nz0[0];
        st->col[C_NZ_MEM][i] -= nz1[1] - nz0[1];
    }
    for (uint32_t x = 0; x < nv; x++) {
        kg_rsv_view* v = &views[x];
        if (v->node != i) continue;
        int matched = 0;
        for (uint32_t t = v->first; t < v->first + v->count && r; t++) matched |= (int32_t)infos[t].rid == rid;
        for (int k = 0; k < KG_RSV_R; k++) {
            const int64_t d = -preq[k] - (matched ? 0 : corr1[k] - corr0[k]);
            v->req[k] += d;
            v->pod_requested[k] += d;
            if (matched) v->r_allocated[k] += new_a[k] - old_a[k];
        }
        v->nz_cpu += -pnz[0] - (matched ? 0 : nz1[0] - nz0[0]);
        v->nz_mem += -pnz[1] - (matched ? 0 : nz1[1] - nz0[1]);
        v->num_pods -= 1;
    }
    if (!r) return;
    for (uint32_t x = 0; x < nv; x++) {
        if (views[x].node != i) continue;
        for (uint32_t t = views[x].first; t < views[x].first + views[x].count; t++) {
            kg_rsv_info* c = &infos[t];
            if ((int32_t)c->rid != rid) continue;
            for (int k = 0; k < KG_RSV_R; k++) c->allocated[k] = new_a[k];
            c->allocated_pods = pods1;
        }
    }
}

struct kgo_ext_session {
    kg_config c;
    kgo_state* st; /* borrowed */
    kgo_ext e2;
    kg_rsv_view* mv;
    kg_rsv_info* mi;
    kg_rsv_dev* md;
    gpu_raw gx;
    view_index vx;
    kgo_quota_state* q;
    int rsv;
    ext_buf b;
};

kgo_ext_session* kgo_ext_session_new(const kg_config* c, kgo_state* st, const kgo_ext* e) {
    kgo_ext_session* x = (kgo_ext_session*)calloc(1, sizeof(*x));
    if (!x) return NULL;
    x->c = *c;
    x->st = st;
    x->rsv = (c->plugins & KG_PLUGIN_RSV) && e && e->n_views;
    if (x->rsv && rsv_has_gpu_tables(e) && !e->n_gpu) { /* the GPU restore cannot be followed without its inputs */
        free(x);
        return NULL;
    }
    if (e) x->e2 = *e;
    if (x->rsv) {
        x->mv = (kg_rsv_view*)malloc(sizeof(kg_rsv_view) * e->n_views);
        x->mi = (kg_rsv_info*)malloc(sizeof(kg_rsv_info) * (e->n_infos ? e->n_infos : 1));
        x->md = (kg_rsv_dev*)malloc(sizeof(kg_rsv_dev) * (e->n_devs ? e->n_devs : 1));
        memcpy(x->mv, e->views, sizeof(kg_rsv_view) * e->n_views);
        if (e->n_infos) memcpy(x->mi, e->infos, sizeof(kg_rsv_info) * e->n_infos);
        if (e->n_devs) memcpy(x->md, e->devs, sizeof(kg_rsv_dev) * e->n_devs);
        x->gx.n = e->n_gpu;
        x->gx.g = (kg_rsv_gpu*)malloc(sizeof(kg_rsv_gpu) * (e->n_gpu ? e->n_gpu : 1));
        if (e->n_gpu) memcpy(x->gx.g, e->gpu, sizeof(kg_rsv_gpu) * e->n_gpu);
        x->e2.views = x->mv;
        x->e2.infos = x->mi;
        x->e2.devs = x->md;
        view_index_build(&x->vx, &x->e2, st->n);
    }
    x->q = (c->plugins & KG_PLUGIN_QUOTA) && e ? quota_state_new(e->quotas, e->n_quotas) : NULL;
    if (ext_buf_new(&x->b, st->n)) {
        kgo_ext_session_free(x);
        return NULL;
    }
    return x;
}

void kgo_ext_session_free(kgo_ext_session* x) {
    if (!x) return;
    free(x->mv);
    free(x->mi);
    free(x->md);
    free(x->gx.g);
    free(x->vx.v);
    quota_state_free(x->q);
    free(x->b.mem);
    free(x);
}

/* Reserve of pod j on node i with every enabled plugin, as one scheduling cycle's Reserve runs them on the pair
 * (NodeInfo + LoadAware, NodeNUMAResource incl. cpusets, DeviceShare at the site its Reserve allocates from,
 * ElasticQuota used, Reservation.Reserve into the nominated reservation with the views and the GPU restore following):
 * 0 + the record its Unreserve gives back, or 1 when the NodeNUMAResource Reserve fails (nothing applied). */
int kgo_ext_reserve(kgo_ext_session* x, uint32_t i, const kg_pod_columns* p, uint32_t j, kg_reserve_record* rec) {
    const kg_config* c = &x->c;
    kgo_state* st = x->st;
    memset(rec, 0, sizeof(*rec));
    rec->numa_zone = -1;
    rec->rsv_rid = -1;
    kg_node_columns v;
    kgo_state_view(st, &v);
    const kgo_ext* ee = x->rsv ? &x->e2 : NULL;
    kg_config c2 = *c;
    if (!x->rsv) c2.plugins &= ~KG_PLUGIN_RSV;
    /* the pair's evaluation (the PreFilter's quota gate is not part of it) */
    ext_eval_nodes(&c2, &v, i, i + 1, p, j, ee ? ee : &x->e2, x->rsv ? &x->vx : NULL, 0, &x->b.r);
    const uint32_t s = x->b.r.st[i];
    const int32_t zone = s ? -1 : x->b.r.zone[i];
    const int64_t nom = s ? -1 : x->b.r.nom[i];
    rec->numa_zone = zone;
    if (zone_fails(zone)) return 1;
    const int32_t cls = p->rsv_class ? p->rsv_class[j] : -1;
    const kg_rsv_view* vw = x->rsv ? find_view(&x->vx, &x->e2, cls, i) : NULL;
    uint32_t mask = 0;
    if ((c->plugins & KG_PLUGIN_DEV) && st->dev_minors)
        mask = dev_choose_site_o(c, &v, i, p, j, &x->e2, vw, nom, zone);
    uint64_t cpus[4] = {0, 0, 0, 0};
    int64_t amounts[2 * KG_MAX_ZONES] = {0};
    const int32_t f = apply(c, st, i, p, j, zone, 1, amounts, cpus);
    if (f) {
        rec->numa_zone = f;
        return 1;
    }
    const int raw = x->rsv && raw_entry(&x->gx, i, -1) != NULL;
    if (mask && !raw) {
        int64_t preq[KG_DEV_R];
        uint32_t keys;
        dev_pod_req(p, j, preq, &keys);
        dev_apply(st->dev_total, st->dev_free, i, mask, preq, keys, 1);
    }
    if (x->q) {
        quota_apply(x->q, p, j, 1);
        rec->flags |= KG_RECORD_QUOTA;
    }
    const int32_t rid = nom >= 0 ? (int32_t)x->mi[nom].rid : -1;
    if (x->rsv) rsv_reserve(st, x->mv, x->e2.n_views, x->mi, i, p, j, nom);
    if (raw) gpu_apply_o(st, &x->e2, x->md, &x->gx, i, mask, p, j, rid, 1);
    rec->gpu_minors = mask;
    rec->rsv_rid = x->rsv ? rid : -1;
    memcpy(rec->zone_amounts, amounts, sizeof(amounts));
    memcpy(rec->cpus, cpus, sizeof(cpus));
    if (cpus[0] | cpus[1] | cpus[2] | cpus[3]) rec->flags |= KG_RECORD_CPUSET;
    return 0;
}

/* The pair's Filter status (every enabled plugin but the PreFilter's quota gate) on the session's current state: the
 * Reserve runs only on a node that passed it. */
uint32_t kgo_ext_session_filter(kgo_ext_session* x, uint32_t i, const kg_pod_columns* p, uint32_t j) {
    kg_node_columns v;
    kgo_state_view(x->st, &v);
    kg_config c2 = x->c;
    if (!x->rsv) c2.plugins &= ~KG_PLUGIN_RSV;
    ext_eval_nodes(&c2, &v, i, i + 1, p, j, &x->e2, x->rsv ? &x->vx : NULL, 0, &x->b.r);
    uint32_t s = x->b.r.st[i];
    if (!s && zone_fails(x->b.r.zone[i])) s = zone_fail_bits(x->b.r.zone[i]);
    return s;
}

/* Unreserve of a kgo_ext_reserve: every plugin gives back what the record says it took (load_aware.go:231-233,
 * nodenumaresource/plugin.go:700-720 -> resource_manager.go:478-483 Release, deviceshare Unreserve -> updateCacheUsed,
 * elasticquota/plugin.go:638-652, reservation/plugin.go:1409-1460). -1 (nothing applied) for a record already given
 * back; the record is then marked KG_RECORD_RELEASED. */
int kgo_ext_unreserve(kgo_ext_session* x, uint32_t i, const kg_pod_columns* p, uint32_t j, kg_reserve_record* rec) {
    if (rec->flags & KG_RECORD_RELEASED) return -1;
    const kg_config* c = &x->c;
    kgo_state* st = x->st;
    int64_t amounts[2 * KG_MAX_ZONES];
    uint64_t cpus[4];
    memcpy(amounts, rec->zone_amounts, sizeof(amounts));
    memcpy(cpus, rec->cpus, sizeof(cpus));
    int any = 0;
    for (int z = 0; z < 2 * KG_MAX_ZONES; z++) any |= amounts[z] != 0;
    const int32_t zone = rec->numa_zone < 0 ? -1 : any ? 0x4F : rec->numa_zone;
    (void)apply(c, st, i, p, j, zone, -1, any ? amounts : NULL, (rec->flags & KG_RECORD_CPUSET) ? cpus : NULL);
    if (x->rsv) rsv_unreserve(st, x->mv, x->e2.n_views, x->mi, i, p, j, rec->rsv_rid);
    const int raw = x->rsv && raw_entry(&x->gx, i, -1) != NULL;
    if (raw) {
        gpu_apply_o(st, &x->e2, x->md, &x->gx, i, (p->dev_count && p->dev_count[j] > 0) ? rec->gpu_minors : 0u, p, j,
                    rec->rsv_rid, -1);
    } else if (rec->gpu_minors && st->dev_total) {
        int64_t preq[KG_DEV_R];
        uint32_t keys;
        dev_pod_req(p, j, preq, &keys);
        dev_apply(st->dev_total, st->dev_free, i, rec->gpu_minors, preq, keys, -1);
    }
    if (x->q && (rec->flags & KG_RECORD_QUOTA)) quota_apply(x->q, p, j, -1);
    rec->flags |= KG_RECORD_RELEASED;
    return 0;
}

/* The session's reservation views, infos and GPU restore tables (as uploaded: n_views / n_infos / n_devs entries) and the
 * quota used / non-preemptible used [quota][KG_QUOTA_R]; any pointer may be NULL. */
void kgo_ext_session_read(const kgo_ext_session* x, kg_rsv_view* views, kg_rsv_info* infos, kg_rsv_dev* devs,
                          int64_t* quota_used, int64_t* quota_np_used) {
    if (x->rsv) {
        if (views) memcpy(views, x->mv, sizeof(kg_rsv_view) * x->e2.n_views);
        if (infos && x->e2.n_infos) memcpy(infos, x->mi, sizeof(kg_rsv_info) * x->e2.n_infos);
        if (devs && x->e2.n_devs) memcpy(devs, x->md, sizeof(kg_rsv_dev) * x->e2.n_devs);
    }
    if (x->q) {
        if (quota_used) memcpy(quota_used, x->q->used, (size_t)x->q->n * KG_QUOTA_R * 8);
        if (quota_np_used) memcpy(quota_np_used, x->q->np_used, (size_t)x->q->n * KG_QUOTA_R * 8);
    }
}
