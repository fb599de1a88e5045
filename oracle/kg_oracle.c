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

/* ---------------------------------------------------------------------------------------------- */
/* NodeResourcesFit (upstream v1.35.6)                                              */

static uint32_t nrf_filter(const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j) {
    uint32_t st = 0;
    /* fitsRequest: len(nodeInfo.Pods)+1 > allowedPodNumber */
    if (n->num_pods[i] + 1 > n->alloc_pods[i]) st |= KG_ST_NRF_PODS;
    /* (the all-zero early return yields the same verdict as the guarded checks below) */
    if (p->req_cpu[j] > 0 && p->req_cpu[j] > n->alloc_cpu[i] - n->req_cpu[i]) st |= KG_ST_NRF_CPU;
    if (p->req_mem[j] > 0 && p->req_mem[j] > n->alloc_mem[i] - n->req_mem[i]) st |= KG_ST_NRF_MEM;
    if (p->req_eph[j] > 0 && p->req_eph[j] > n->alloc_eph[i] - n->req_eph[i]) st |= KG_ST_NRF_EPH;
    for (int k = 0; k < KG_NSCALAR; k++) {
        int64_t q = p->sc_req[k][j];
        if (q == 0) continue; /* "Skip in case request quantity is zero" */
        if (q > n->sc_alloc[k][i] - n->sc_req[k][i]) st |= (k == 0 ? KG_ST_NRF_SC0 : KG_ST_NRF_SC1);
    }
    return st;
}

/* resourceAllocationScorer.score + leastResourceScorer with NonZeroRequested for cpu/memory and
 * Requested for scalars; scalars the pod does not request are bypassed (0, 0); resources with
 * allocatable 0 are skipped (mirrors noderesourcefitplus/node_resource_fit_plus_utils.go:114-139). */
static int64_t nrf_score(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                         uint32_t j) {
    int64_t alloc[2 + KG_NSCALAR], req[2 + KG_NSCALAR], w[2 + KG_NSCALAR];
    alloc[0] = n->alloc_cpu[i];
    req[0] = n->nz_cpu[i] + p->nz_cpu[j];
    w[0] = c->nrf_w_cpu;
    alloc[1] = n->alloc_mem[i];
    req[1] = n->nz_mem[i] + p->nz_mem[j];
    w[1] = c->nrf_w_mem;
    for (int k = 0; k < KG_NSCALAR; k++) {
        int64_t q = p->sc_req[k][j];
        if (q == 0) {
            alloc[2 + k] = 0;
            req[2 + k] = 0;
        } else {
            alloc[2 + k] = n->sc_alloc[k][i];
            req[2 + k] = n->sc_req[k][i] + q;
        }
        w[2 + k] = c->nrf_w_sc[k];
    }
    int64_t score = 0, wsum = 0;
    for (int r = 0; r < 2 + KG_NSCALAR; r++) {
        if (w[r] == 0) continue; /* resource not in the scoring strategy */
        if (alloc[r] == 0) continue;
        score += least_requested_score(req[r], alloc[r]) * w[r];
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

/* leastResourceScorer over {cpu, memory} with resources of allocatable 0 dropped
 * (nodenumaresource/scoring.go:222-238, least_allocated.go:30-48). */
static int64_t numa_least_score(int64_t w_cpu, int64_t w_mem, int64_t alloc_cpu, int64_t req_cpu, int64_t alloc_mem,
                                int64_t req_mem) {
    int64_t score = 0, wsum = 0;
    if (alloc_cpu != 0 && w_cpu != 0) {
        score += least_requested_score(req_cpu, alloc_cpu) * w_cpu;
        wsum += w_cpu;
    }
    if (alloc_mem != 0 && w_mem != 0) {
        score += least_requested_score(req_mem, alloc_mem) * w_mem;
        wsum += w_mem;
    }
    if (wsum == 0) return 0;
    return score / wsum;
}

static int64_t sub_nonneg(int64_t a, int64_t b) { return a - b < 0 ? 0 : a - b; }

/* Best single-NUMA-node hint for a non-cpuset pod on a SingleNUMANode node: a zone is usable when
 * tryBestToDistributeEvenly fits the pod's requests into it (resource_manager.go:272-318) and it does
 * not lack any requested resource (generateResourceHints, resource_manager.go:529-626); among usable
 * zones mergeFilteredHints keeps the highest hint score, ties to the lowest zone (policy.go:198-256,
 * bitmask IsNarrowerThan). Returns zone or -1. */
static int32_t numa_best_zone(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                              uint32_t j) {
    uint32_t Z = n->numa_zones[i];
    int has_cpu = (p->flags[j] & KG_POD_HAS_CPU) != 0, has_mem = (p->flags[j] & KG_POD_HAS_MEM) != 0;
    int32_t best = -1;
    int64_t best_score = 0;
    for (uint32_t z = 0; z < Z; z++) {
        int64_t tc = n->zone_cpu[z][i], tm = n->zone_mem[z][i];
        int64_t uc = n->zone_cpu_used[z][i], um = n->zone_mem_used[z][i];
        int64_t ac = sub_nonneg(tc, uc), am = sub_nonneg(tm, um); /* node_allocation.go:240 */
        if (has_cpu && (ac == 0 || p->req_cpu[j] > ac)) continue;
        if (has_mem && (am == 0 || p->req_mem[j] > am)) continue;
        /* hint score: numaScorer over requested = total - available (resource_manager.go:575-579) */
        int64_t rc = sub_nonneg(tc, ac), rm = sub_nonneg(tm, am);
        int64_t s = numa_least_score(c->numa_hint_w_cpu, c->numa_hint_w_mem, tc, rc + p->req_cpu[j], tm,
                                     rm + p->req_mem[j]);
        if (best < 0 || s > best_score) {
            best = (int32_t)z;
            best_score = s;
        }
    }
    return best;
}

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

/* Filter (plugin.go:363-459) + Score (scoring.go:67-151) of one pair. zone_out: -2 = node scored
 * at node level (no NUMA allocation), >=0 zone allocation. */
static uint32_t numa_eval(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p,
                          uint32_t j, int64_t* score_out, int32_t* zone_out) {
    *score_out = 0;
    *zone_out = -1;
    if (p->flags[j] & KG_POD_NUMA_SKIP) return 0; /* PreFilter Skip: no Filter, no Score */
    if (p->flags[j] & KG_POD_CPU_BIND) return KG_ST_UNSUPPORTED;
    int conflict;
    uint32_t policy = numa_merge_policy(n->numa_policy[i], p->numa_policy[j], &conflict);
    if (conflict) return KG_ST_NUMA_CONFLICT;
    if (policy == KG_NUMA_RESTRICTED || policy == KG_NUMA_BEST_EFFORT) return KG_ST_UNSUPPORTED;
    double ratio = n->cpu_amp_ratio[i];
    int64_t pod_cpu = p->req_cpu[j];
    /* filterAmplifiedCPUs: plugin.go:461-498 (requestCPUBind == false) */
    if (pod_cpu != 0 && ratio > 1) {
        int64_t allocated = n->cpuset_alloc_milli[i];
        int64_t requested = n->req_cpu[i];
        if (requested >= allocated && allocated > 0) {
            requested = requested - allocated;
            requested += kgo_amplify(allocated, ratio);
        }
        if (pod_cpu > n->alloc_cpu[i] - requested) return KG_ST_NUMA_AMP_CPU;
    }
    if (policy == KG_NUMA_SINGLE_NODE) {
        /* FilterByNUMANode: topology_hint.go:31-41 -> singleNumaNodePolicy.Merge
         * (frameworkext/topologymanager/policy_single_numa_node.go:69-90) */
        uint32_t Z = n->numa_zones[i];
        if (Z == 0) return KG_ST_NUMA_NO_RES;
        int has_any = (p->flags[j] & (KG_POD_HAS_CPU | KG_POD_HAS_MEM)) != 0;
        int32_t z = -1;
        if (has_any) {
            z = numa_best_zone(c, n, i, p, j);
            if (z < 0) return KG_ST_NUMA_ALIGN;
        }
        /* a best hint equal to the default affinity (all zones) is returned without affinity
         * (policy_single_numa_node.go:79-84): no NUMA allocation, node-level score */
        if (!has_any || Z == 1) {
            *zone_out = -1;
            *score_out = numa_least_score(c->numa_w_cpu, c->numa_w_mem, n->alloc_cpu[i], n->req_cpu[i] + pod_cpu,
                                          n->alloc_mem[i], n->req_mem[i] + p->req_mem[j]);
            return 0;
        }
        /* Score with the zone allocation: calculateAllocatableAndRequested, scoring.go:153-199 */
        *zone_out = z;
        *score_out = numa_least_score(c->numa_w_cpu, c->numa_w_mem, n->zone_cpu[z][i],
                                      n->zone_cpu_used[z][i] + pod_cpu, n->zone_mem[z][i],
                                      n->zone_mem_used[z][i] + p->req_mem[j]);
        return 0;
    }
    /* policy None: scoreWithAmplifiedCPUs, scoring.go:132-151 */
    int64_t req_cpu = n->req_cpu[i];
    if (!(pod_cpu == 0 || ratio <= 1)) {
        int64_t allocated = n->cpuset_alloc_milli[i];
        req_cpu = req_cpu - allocated + kgo_amplify(allocated, ratio);
    }
    *score_out = numa_least_score(c->numa_w_cpu, c->numa_w_mem, n->alloc_cpu[i], req_cpu + pod_cpu, n->alloc_mem[i],
                                  n->req_mem[i] + p->req_mem[j]);
    return 0;
}

/* ---------------------------------------------------------------------------------------------- */

void kgo_eval_pair(const kg_config* c, const kg_node_columns* n, uint32_t i, const kg_pod_columns* p, uint32_t j,
                   kgo_pair* out) {
    uint32_t st = 0;
    int64_t s_numa = 0;
    int32_t zone = -1;
    if (c->plugins & KG_PLUGIN_NRF) st |= nrf_filter(n, i, p, j);
    if (c->plugins & KG_PLUGIN_LA) st |= la_filter(c, n, i, p, j);
    if (c->plugins & KG_PLUGIN_NUMA) st |= numa_eval(c, n, i, p, j, &s_numa, &zone);
    out->status = st;
    /* Score functions are defined for every node (the Go ScorePlugin.Score can be called on any
     * node); the NUMA score exists only where its Filter admitted the pod (it needs the hint). */
    out->s_nrf = (c->plugins & KG_PLUGIN_NRF) ? nrf_score(c, n, i, p, j) : 0;
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
    volatile int next_chunk;
    int chunk, n_items;
    const uint32_t* items; /* phase 1: feasible node list */
} par_job;

typedef struct par_pool {
    pthread_t* th;
    int n;
    pthread_barrier_t start, done;
    par_job* job;
    int quit;
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
                if (jb->c->plugins & KG_PLUGIN_NRF) st |= nrf_filter(jb->n, i, jb->p, jb->pod);
                if (jb->c->plugins & KG_PLUGIN_LA) st |= la_filter(jb->c, jb->n, i, jb->p, jb->pod);
                int64_t s;
                int32_t z;
                if (jb->c->plugins & KG_PLUGIN_NUMA) {
                    st |= numa_eval(jb->c, jb->n, i, jb->p, jb->pod, &s, &z);
                    jb->total[i] = s; /* NUMA score is produced by the same resource-manager walk */
                }
                jb->feasible[i] = st == 0;
            } else {
                uint32_t i = jb->items[x];
                int64_t t = 0;
                const kg_config* c = jb->c;
                if (c->plugins & KG_PLUGIN_NRF) t += c->weight_nrf * nrf_score(c, jb->n, i, jb->p, jb->pod);
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

int kgo_select_parallel(const kg_config* c, const kg_node_columns* n, uint32_t nn, uint32_t base,
                        const kg_pod_columns* p, uint32_t np, int workers, uint64_t* keys) {
    if (workers < 1) workers = 1;
    par_pool pool;
    memset(&pool, 0, sizeof(pool));
    pool.n = workers - 1; /* the calling thread is worker 0 */
    pool.th = (pthread_t*)calloc((size_t)(pool.n > 0 ? pool.n : 1), sizeof(pthread_t));
    uint8_t* feasible = (uint8_t*)malloc(nn);
    int64_t* total = (int64_t*)malloc(sizeof(int64_t) * (nn ? nn : 1));
    uint32_t* items = (uint32_t*)malloc(sizeof(uint32_t) * (nn ? nn : 1));
    if (!pool.th || !feasible || !total || !items) return -1;
    par_job jb;
    memset(&jb, 0, sizeof(jb));
    pool.job = &jb;
    pthread_barrier_init(&pool.start, NULL, (unsigned)workers);
    pthread_barrier_init(&pool.done, NULL, (unsigned)workers);
    for (int t = 0; t < pool.n; t++) pthread_create(&pool.th[t], NULL, par_worker, &pool);
    for (uint32_t j = 0; j < np; j++) {
        /* findNodesThatPassFilters */
        jb.c = c;
        jb.n = n;
        jb.p = p;
        jb.nn = nn;
        jb.pod = j;
        jb.base = base;
        jb.feasible = feasible;
        jb.total = total;
        jb.phase = 0;
        jb.n_items = (int)nn;
        jb.chunk = chunk_size((int)nn, workers);
        jb.next_chunk = 0;
        pthread_barrier_wait(&pool.start);
        par_run(&jb);
        pthread_barrier_wait(&pool.done);
        uint32_t nf = 0;
        for (uint32_t i = 0; i < nn; i++)
            if (feasible[i]) items[nf++] = i;
        uint64_t best = 0;
        if (nf > 1) {
            /* prioritizeNodes */
            jb.phase = 1;
            jb.items = items;
            jb.n_items = (int)nf;
            jb.chunk = chunk_size((int)nf, workers);
            jb.next_chunk = 0;
            pthread_barrier_wait(&pool.start);
            par_run(&jb);
            pthread_barrier_wait(&pool.done);
            /* selectHost (deterministic tie-break) */
            for (uint32_t x = 0; x < nf; x++) {
                uint64_t key = make_key(total[items[x]], base + items[x]);
                if (key > best) best = key;
            }
        } else if (nf == 1) {
            /* exactly one feasible node: chosen without scoring; key still carries its total */
            kgo_pair r;
            kgo_eval_pair(c, n, items[0], p, j, &r);
            best = make_key(r.total, base + items[0]);
        }
        keys[j] = best;
    }
    pool.quit = 1;
    pthread_barrier_wait(&pool.start);
    for (int t = 0; t < pool.n; t++) pthread_join(pool.th[t], NULL);
    pthread_barrier_destroy(&pool.start);
    pthread_barrier_destroy(&pool.done);
    free(pool.th);
    free(feasible);
    free(total);
    free(items);
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
    uint32_t *la_flags, *numa_policy, *numa_zones;
    double* amp;
};

static int64_t* dup64(const int64_t* s, uint32_t n) {
    int64_t* d = (int64_t*)calloc(n ? n : 1, sizeof(int64_t));
    if (s) memcpy(d, s, sizeof(int64_t) * n);
    return d;
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
    if (s->la_flags) memcpy(st->la_flags, s->la_flags, 4 * (size_t)n);
    if (s->numa_policy) memcpy(st->numa_policy, s->numa_policy, 4 * (size_t)n);
    if (s->numa_zones) memcpy(st->numa_zones, s->numa_zones, 4 * (size_t)n);
    if (s->cpu_amp_ratio) memcpy(st->amp, s->cpu_amp_ratio, 8 * (size_t)n);
    return st;
}

void kgo_state_free(kgo_state* st) {
    if (!st) return;
    for (int c = 0; c < C_NCOLS; c++) free(st->col[c]);
    free(st->la_flags);
    free(st->numa_policy);
    free(st->numa_zones);
    free(st->amp);
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
}

static void apply(const kg_config* c, kgo_state* st, uint32_t i, const kg_pod_columns* p, uint32_t j, int32_t zone,
                  int64_t sign) {
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
    /* NodeNUMAResource Reserve -> resourceManager.Update (plugin.go:585-635) */
    if ((c->plugins & KG_PLUGIN_NUMA) && zone >= 0) {
        st->col[C_ZONE_CPU_USED + zone][i] += sign * p->req_cpu[j];
        st->col[C_ZONE_MEM_USED + zone][i] += sign * p->req_mem[j];
    }
}

void kgo_assume(const kg_config* c, kgo_state* st, uint32_t i, const kg_pod_columns* p, uint32_t j) {
    kg_node_columns v;
    kgo_state_view(st, &v);
    kgo_pair r;
    kgo_eval_pair(c, &v, i, p, j, &r);
    int32_t zone = r.status ? -1 : r.zone;
    apply(c, st, i, p, j, zone, 1);
}

void kgo_forget(const kg_config* c, kgo_state* st, uint32_t i, const kg_pod_columns* p, uint32_t j, int32_t zone) {
    apply(c, st, i, p, j, zone, -1);
}

void kgo_replay(const kg_config* c, kgo_state* st, uint32_t base, const kg_pod_columns* p, uint32_t np,
                int32_t* out_node, int64_t* out_total) {
    kg_node_columns v;
    kgo_state_view(st, &v);
    for (uint32_t j = 0; j < np; j++) {
        uint64_t best = 0;
        int32_t best_zone = -1;
        for (uint32_t i = 0; i < st->n; i++) {
            kgo_pair r;
            kgo_eval_pair(c, &v, i, p, j, &r);
            if (r.status) continue;
            uint64_t key = make_key(r.total, base + i);
            if (key > best) {
                best = key;
                best_zone = r.zone;
            }
        }
        if (!best) {
            out_node[j] = -1;
            if (out_total) out_total[j] = -1;
            continue;
        }
        uint32_t g = 0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu);
        out_node[j] = (int32_t)g;
        if (out_total) out_total[j] = (int64_t)(best >> 32);
        apply(c, st, g - base, p, j, best_zone, 1);
    }
}
