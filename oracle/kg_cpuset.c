/* kg_cpuset.c — CPU restatement of koordinator's cpuset accumulator (TEST INFRASTRUCTURE: the parity oracle
 * for the device accumulator in koordinator_amd/csrc/kg_cpuset.h; never part of the product path).
 *
 * Follows pkg/scheduler/plugins/nodenumaresource/cpu_accumulator.go line by line:
 *   takePreferredCPUs :30-86, takeCPUs :88-246, newCPUAccumulator :248-289, take / needs / isSatisfied /
 *   isFailed :291-317, exclusivity :319-331, extractCPU :333-344, sortCores :346-370,
 *   freeCoresInNode :372-463, freeCoresInSocket :465-529, freeCPUsInNode :531-607,
 *   freeCPUsInSocket :609-665, freeCPUs :667-775, getCoreRefCount :777-784, sortCPUsByRefCount :786-797,
 *   spreadCPUs :799-823.
 * Go maps become arrays indexed by the dense ids of kg_cpu_topo; every sort of the reference has a total
 * order (ids break ties) except the two by-length sorts of whole groups in takeCPUs, which run on at most a
 * handful of sockets, where Go's pdqsort is an insertion sort: stable, as here.
 * Pinned by the reference's own KATs (cpu_accumulator_test.go, tests/golden/cpuset_kat.json). */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "kg_oracle.h"

#define MAXC KG_MAX_CPUS

typedef struct {
    const kg_cpu_topo* t;
    int max_ref, excl_policy, strategy, exclusive, needed;
    uint8_t avail[MAXC];          /* allocatableCPUs membership */
    uint8_t ref[MAXC];            /* RefCount of allocatable CPUs (copied only when maxRefCount > 1) */
    uint8_t excl_core[MAXC];      /* exclusiveInCores */
    uint8_t excl_node[MAXC];      /* exclusiveInNUMANodes */
    uint8_t result[MAXC];
} acc_t;

typedef struct {
    int n;
    int c[MAXC];
} list_t;

static int cpc(const kg_cpu_topo* t) { return t->n_cores ? t->n_cpus / t->n_cores : 0; }
static int cpn(const kg_cpu_topo* t) { return t->n_nodes ? t->n_cpus / t->n_nodes : 0; }
static int cps(const kg_cpu_topo* t) { return t->n_sockets ? t->n_cpus / t->n_sockets : 0; }

static int count_avail(const acc_t* a) {
    int n = 0;
    for (int i = 0; i < a->t->n_cpus; i++) n += a->avail[i];
    return n;
}

static void acc_take(acc_t* a, const int* cpus, int n) {
    for (int k = 0; k < n; k++) {
        const int c = cpus[k];
        a->result[c] = 1;
        a->avail[c] = 0;
        if (a->exclusive) {
            if (a->excl_policy == KG_CPU_EXCL_PCPU_LEVEL) a->excl_core[a->t->core[c]] = 1;
            else if (a->excl_policy == KG_CPU_EXCL_NUMA_NODE_LEVEL) a->excl_node[a->t->numa[c]] = 1;
        }
    }
    a->needed -= n;
}

static int needs(const acc_t* a, int n) { return a->needed >= n; }
static int satisfied(const acc_t* a) { return a->needed < 1; }

static int excl_pcpu(const acc_t* a, int c) {
    return a->excl_policy == KG_CPU_EXCL_PCPU_LEVEL && a->excl_core[a->t->core[c]];
}
static int excl_numa(const acc_t* a, int c) {
    return a->excl_policy == KG_CPU_EXCL_NUMA_NODE_LEVEL && a->excl_node[a->t->numa[c]];
}

static int cmp_int(const void* x, const void* y) { return *(const int*)x - *(const int*)y; }

/* getCoreRefCount over the allocatable CPUs (the accumulator passes allocatableCPUs as details) */
static int core_ref(const acc_t* a, int core) {
    int r = 0;
    for (int i = 0; i < a->t->n_cpus; i++)
        if (a->avail[i] && a->t->core[i] == core) r += a->ref[i];
    return r;
}

/* sortCPUsByRefCount: RefCount ascending, then CPU id (insertion sort: tiny lists) */
static void sort_by_ref(const acc_t* a, int* c, int n) {
    for (int i = 1; i < n; i++) {
        int x = c[i], j = i - 1;
        while (j >= 0 && (a->ref[c[j]] > a->ref[x] || (a->ref[c[j]] == a->ref[x] && c[j] > x))) {
            c[j + 1] = c[j];
            j--;
        }
        c[j + 1] = x;
    }
}

/* extractCPU: the first CPU of each core, in list order */
static void extract_cpu(const acc_t* a, list_t* l) {
    uint8_t seen[MAXC] = {0};
    int m = 0;
    for (int k = 0; k < l->n; k++) {
        const int core = a->t->core[l->c[k]];
        if (!seen[core]) {
            seen[core] = 1;
            l->c[m++] = l->c[k];
        }
    }
    l->n = m;
}

/* cores grouped (per CPU membership `in`): cnt[core] CPUs, cpus of core ascending */
typedef struct {
    int cnt[MAXC];
    int cpus[MAXC][8];
} cores_t;

static void group_cores(const acc_t* a, const uint8_t* in, cores_t* g) {
    memset(g->cnt, 0, sizeof(g->cnt));
    for (int i = 0; i < a->t->n_cpus; i++)
        if (in[i]) {
            const int core = a->t->core[i];
            if (g->cnt[core] < 8) g->cpus[core][g->cnt[core]] = i;
            g->cnt[core]++;
        }
}

static const acc_t* g_acc;
static const cores_t* g_cores;
/* sortCores: more CPUs first, then (maxRefCount > 1) smaller core RefCount, then core id */
static int cmp_core(const void* x, const void* y) {
    const int i = *(const int*)x, j = *(const int*)y;
    if (g_cores->cnt[i] != g_cores->cnt[j]) return g_cores->cnt[j] - g_cores->cnt[i];
    if (g_acc->max_ref > 1) {
        const int ri = core_ref(g_acc, i), rj = core_ref(g_acc, j);
        if (ri != rj) return ri - rj;
    }
    return i - j;
}

static int more_free_first(const acc_t* a, int fi, int fj) {
    /* returns <0 when i sorts first: MostAllocated -> fewer free first, else more free first */
    if (a->strategy == KG_NUMA_MOST_ALLOCATED) return fi - fj;
    return fj - fi;
}

/* freeCoresInNode / freeCoresInSocket: per group (NUMA node or socket) the CPUs of its (full) free cores */
static int free_cores(const acc_t* a, int by_node, int filter_full, int filter_excl, list_t* out) {
    const kg_cpu_topo* t = a->t;
    uint8_t in[MAXC] = {0};
    int sock_free[MAXC] = {0};
    for (int i = 0; i < t->n_cpus; i++) {
        if (!a->avail[i]) continue;
        if (by_node && filter_excl && excl_numa(a, i)) continue;
        in[i] = 1;
        sock_free[t->socket[i]]++;
    }
    static _Thread_local cores_t g;
    group_cores(a, in, &g);
    const int ng = by_node ? t->n_nodes : t->n_sockets;
    int* cores_of = (int*)calloc((size_t)ng * MAXC, sizeof(int));
    int* ncores = (int*)calloc((size_t)ng, sizeof(int));
    for (int core = 0; core < t->n_cores; core++) {
        if (!g.cnt[core]) continue;
        if (filter_full && g.cnt[core] != cpc(t)) continue;
        const int c0 = g.cpus[core][0];
        const int grp = by_node ? t->numa[c0] : t->socket[c0];
        cores_of[grp * MAXC + ncores[grp]++] = core;
    }
    int order[MAXC], n = 0;
    for (int grp = 0; grp < ng; grp++) {
        if (!ncores[grp]) continue;
        g_acc = a;
        g_cores = &g;
        qsort(cores_of + grp * MAXC, (size_t)ncores[grp], sizeof(int), cmp_core);
        list_t* l = &out[grp];
        l->n = 0;
        for (int k = 0; k < ncores[grp]; k++) {
            const int core = cores_of[grp * MAXC + k];
            for (int m = 0; m < g.cnt[core]; m++) l->c[l->n++] = g.cpus[core][m];
        }
        order[n++] = grp;
    }
    /* group order: free CPUs of the group (strategy), node groups then their socket's free CPUs, then id */
    for (int x = 1; x < n; x++) {
        int v = order[x], y = x - 1;
        while (y >= 0) {
            const int u = order[y];
            int d = more_free_first(a, out[v].n, out[u].n);
            if (d == 0 && by_node) {
                const int sv = t->socket[out[v].c[0]], su = t->socket[out[u].c[0]];
                d = more_free_first(a, sock_free[sv], sock_free[su]);
            }
            if (d == 0) d = v - u;
            if (d >= 0) break;
            order[y + 1] = order[y];
            y--;
        }
        order[y + 1] = v;
    }
    static _Thread_local list_t tmp[64]; /* per thread: the oracle runs on worker threads */
    for (int k = 0; k < n; k++) tmp[k] = out[order[k]];
    for (int k = 0; k < n; k++) out[k] = tmp[k];
    free(cores_of);
    free(ncores);
    return n;
}

/* freeCPUsInNode (by_node) / freeCPUsInSocket: per group the free CPUs, ascending (RefCount order when
 * maxRefCount > 1), one per core when filtering exclusivity */
static int free_cpus_grouped(const acc_t* a, int by_node, int filter_excl, list_t* out) {
    const kg_cpu_topo* t = a->t;
    const int ng = by_node ? t->n_nodes : t->n_sockets;
    int node_free[MAXC] = {0}, sock_free[MAXC] = {0};
    for (int grp = 0; grp < ng; grp++) out[grp].n = 0;
    for (int i = 0; i < t->n_cpus; i++) {
        if (!a->avail[i]) continue;
        if (filter_excl) {
            if (by_node ? (excl_pcpu(a, i) || excl_numa(a, i)) : excl_pcpu(a, i)) continue;
        }
        const int grp = by_node ? t->numa[i] : t->socket[i];
        out[grp].c[out[grp].n++] = i;
        node_free[t->numa[i]]++;
        sock_free[t->socket[i]]++;
    }
    int order[64], n = 0;
    for (int grp = 0; grp < ng; grp++) {
        if (!out[grp].n) continue;
        qsort(out[grp].c, (size_t)out[grp].n, sizeof(int), cmp_int);
        if (a->max_ref > 1) sort_by_ref(a, out[grp].c, out[grp].n);
        if (filter_excl) extract_cpu(a, &out[grp]);
        order[n++] = grp;
    }
    for (int x = 1; x < n; x++) {
        int v = order[x], y = x - 1;
        while (y >= 0) {
            const int u = order[y];
            int d;
            if (by_node) {
                d = more_free_first(a, node_free[v], node_free[u]);
                if (d == 0) d = more_free_first(a, sock_free[t->socket[out[v].c[0]]], sock_free[t->socket[out[u].c[0]]]);
            } else {
                d = more_free_first(a, out[v].n, out[u].n);  /* after extractCPU */
            }
            if (d == 0) d = v - u;
            if (d >= 0) break;
            order[y + 1] = order[y];
            y--;
        }
        order[y + 1] = v;
    }
    static _Thread_local list_t tmp[64]; /* per thread: the oracle runs on worker threads */
    for (int k = 0; k < n; k++) tmp[k] = out[order[k]];
    for (int k = 0; k < n; k++) out[k] = tmp[k];
    return n;
}

/* freeCPUs: every free CPU, cores ordered by socket colocation with the result, socket / node free CPUs
 * (strategy), fewer free CPUs on the core, socket id, core RefCount (maxRefCount > 1), core id */
static void free_cpus(const acc_t* a, int filter_excl, list_t* out) {
    const kg_cpu_topo* t = a->t;
    uint8_t in[MAXC] = {0};
    int node_free[MAXC] = {0}, sock_free[MAXC] = {0}, colo[MAXC] = {0};
    for (int i = 0; i < t->n_cpus; i++) {
        if (!a->avail[i]) continue;
        if (filter_excl && (excl_pcpu(a, i) || excl_numa(a, i))) continue;
        in[i] = 1;
        node_free[t->numa[i]]++;
        sock_free[t->socket[i]]++;
    }
    for (int i = 0; i < t->n_cpus; i++)
        if (a->result[i]) colo[t->socket[i]]++;
    static _Thread_local cores_t g;
    group_cores(a, in, &g);
    int cores[MAXC], n = 0;
    for (int core = 0; core < t->n_cores; core++)
        if (g.cnt[core]) cores[n++] = core;
    for (int x = 1; x < n; x++) {
        int v = cores[x], y = x - 1;
        while (y >= 0) {
            const int u = cores[y];
            const int sv = t->socket[g.cpus[v][0]], su = t->socket[g.cpus[u][0]];
            const int nv = t->numa[g.cpus[v][0]], nu = t->numa[g.cpus[u][0]];
            int d = colo[su] - colo[sv];
            if (d == 0) d = more_free_first(a, sock_free[sv], sock_free[su]);
            if (d == 0) d = more_free_first(a, node_free[nv], node_free[nu]);
            if (d == 0) d = g.cnt[v] - g.cnt[u];
            if (d == 0) d = sv - su;
            if (d == 0 && a->max_ref > 1) d = core_ref(a, v) - core_ref(a, u);
            if (d == 0) d = v - u;
            if (d >= 0) break;
            cores[y + 1] = cores[y];
            y--;
        }
        cores[y + 1] = v;
    }
    out->n = 0;
    for (int k = 0; k < n; k++) {
        int cp[8], m = g.cnt[cores[k]];
        for (int q = 0; q < m; q++) cp[q] = g.cpus[cores[k]][q];
        qsort(cp, (size_t)m, sizeof(int), cmp_int);
        if (a->max_ref > 1) sort_by_ref(a, cp, m);
        for (int q = 0; q < m; q++) out->c[out->n++] = cp[q];
    }
}

/* spreadCPUs: passes over the list taking the first CPU of each core not yet visited in the pass */
static void spread(const acc_t* a, list_t* l) {
    if (l->n <= cpc(a->t)) return;
    int prep[MAXC], np = l->n;
    memcpy(prep, l->c, sizeof(int) * (size_t)np);
    l->n = 0;
    while (np > 0) {
        uint8_t seen[MAXC] = {0};
        int rest[MAXC], nr = 0;
        for (int k = 0; k < np; k++) {
            const int core = a->t->core[prep[k]];
            if (seen[core]) {
                rest[nr++] = prep[k];
                continue;
            }
            l->c[l->n++] = prep[k];
            seen[core] = 1;
        }
        memcpy(prep, rest, sizeof(int) * (size_t)nr);
        np = nr;
    }
}

static void mask_set(uint64_t* m, int c) { m[c >> 6] |= 1ull << (c & 63); }
static int mask_has(const uint64_t* m, int c) { return (int)((m[c >> 6] >> (c & 63)) & 1ull); }

int kgo_take_cpus(const kg_cpu_topo* t, int max_ref, const uint64_t avail[4], const kg_cpu_alloc* allocated,
                  int needed, int bind_policy, int excl_policy, int strategy, uint64_t out[4]) {
    static _Thread_local acc_t A;
    acc_t* a = &A;
    memset(a, 0, sizeof(*a));
    memset(out, 0, 4 * sizeof(uint64_t));
    a->t = t;
    a->max_ref = max_ref;
    a->excl_policy = excl_policy;
    a->strategy = strategy;
    a->needed = needed;
    a->exclusive = excl_policy == KG_CPU_EXCL_PCPU_LEVEL || excl_policy == KG_CPU_EXCL_NUMA_NODE_LEVEL;
    for (int i = 0; i < t->n_cpus; i++) {
        a->avail[i] = (uint8_t)mask_has(avail, i);
        if (allocated) {
            if (allocated->excl[i] == KG_CPU_EXCL_PCPU_LEVEL) a->excl_core[t->core[i]] = 1;
            else if (allocated->excl[i] == KG_CPU_EXCL_NUMA_NODE_LEVEL) a->excl_node[t->numa[i]] = 1;
            if (max_ref > 1 && a->avail[i]) a->ref[i] = allocated->ref[i];
        }
    }
    static _Thread_local list_t L[64];
    if (satisfied(a)) return 0;
    if (a->needed > count_avail(a)) return -1; /* ErrNotEnoughCPUs */
    const int full = bind_policy == KG_CPU_BIND_FULL_PCPUS;
    int done = 0;
    if (full || cpc(t) == 1) {
        if (a->needed <= cpn(t)) {
            for (int fe = 1; fe >= 0 && !done; fe--) {
                const int n = free_cores(a, 1, 1, fe, L);
                for (int k = 0; k < n; k++)
                    if (L[k].n >= a->needed) {
                        acc_take(a, L[k].c, a->needed);
                        done = 1;
                        break;
                    }
            }
        }
        if (!done && a->needed <= cps(t)) {
            const int n = free_cores(a, 0, 1, 0, L);
            for (int k = 0; k < n; k++)
                if (L[k].n >= a->needed) {
                    acc_take(a, L[k].c, a->needed);
                    done = 1;
                    break;
                }
        }
        if (!done) {
            int n = free_cores(a, 0, 1, 0, L);
            /* stable sort by length, descending */
            for (int x = 1; x < n; x++) {
                list_t v = L[x];
                int y = x - 1;
                while (y >= 0 && L[y].n < v.n) {
                    L[y + 1] = L[y];
                    y--;
                }
                L[y + 1] = v;
            }
            static _Thread_local list_t U[64];
            int nu = 0;
            for (int k = 0; k < n && !done; k++) {
                if (!needs(a, L[k].n)) {
                    U[nu++] = L[k];
                } else {
                    acc_take(a, L[k].c, L[k].n);
                    if (satisfied(a)) done = 1;
                }
            }
            if (!done && needs(a, cpc(t))) {
                for (int x = 1; x < nu; x++) { /* stable, ascending by length */
                    list_t v = U[x];
                    int y = x - 1;
                    while (y >= 0 && U[y].n > v.n) {
                        U[y + 1] = U[y];
                        y--;
                    }
                    U[y + 1] = v;
                }
                const int step = cpc(t);
                for (int k = 0; k < nu && !done; k++) {
                    for (int i = 0; i < U[k].n; i += step) {
                        acc_take(a, U[k].c + i, step);
                        if (satisfied(a)) {
                            done = 1;
                            break;
                        }
                        if (!needs(a, step)) break;
                    }
                }
            }
        }
    }
    if (!done && !full) {
        if (a->needed <= cpn(t)) {
            for (int fe = 1; fe >= 0 && !done; fe--) {
                const int n = free_cpus_grouped(a, 1, fe, L);
                for (int k = 0; k < n; k++)
                    if (L[k].n >= a->needed) {
                        spread(a, &L[k]);
                        acc_take(a, L[k].c, a->needed);
                        done = 1;
                        break;
                    }
            }
        }
        if (!done && a->needed <= cps(t)) {
            for (int fe = 1; fe >= 0 && !done; fe--) {
                const int n = free_cpus_grouped(a, 0, fe, L);
                for (int k = 0; k < n; k++)
                    if (L[k].n >= a->needed) {
                        spread(a, &L[k]);
                        acc_take(a, L[k].c, a->needed);
                        done = 1;
                        break;
                    }
            }
        }
    }
    for (int fe = 1; fe >= 0 && !done; fe--) {
        static _Thread_local list_t F;
        free_cpus(a, fe, &F);
        spread(a, &F);
        for (int k = 0; k < F.n; k++) {
            if (needs(a, 1)) acc_take(a, &F.c[k], 1);
            if (satisfied(a)) {
                done = 1;
                break;
            }
        }
    }
    if (!done) return -2; /* "failed to allocate cpus" */
    for (int i = 0; i < t->n_cpus; i++)
        if (a->result[i]) mask_set(out, i);
    return 0;
}

int kgo_take_preferred_cpus(const kg_cpu_topo* t, int max_ref, const uint64_t avail_in[4], const uint64_t preferred[4],
                            const kg_cpu_alloc* allocated, int needed, int bind_policy, int excl_policy, int strategy,
                            uint64_t out[4]) {
    uint64_t avail[4], pref[4], res[4] = {0, 0, 0, 0};
    int np = 0;
    for (int w = 0; w < 4; w++) {
        avail[w] = avail_in[w];
        pref[w] = avail_in[w] & (preferred ? preferred[w] : 0ull);
        np += __builtin_popcountll(pref[w]);
    }
    memset(out, 0, 4 * sizeof(uint64_t));
    if (np) {
        const int n = needed < np ? needed : np;
        int rc = kgo_take_cpus(t, max_ref, pref, allocated, n, bind_policy, excl_policy, strategy, res);
        if (rc) {
            for (int w = 0; w < 4; w++) out[w] = res[w];
            return rc;
        }
        for (int w = 0; w < 4; w++) {
            needed -= __builtin_popcountll(res[w]);
            avail[w] &= ~pref[w];
        }
    }
    if (needed > 0) {
        uint64_t more[4];
        int rc = kgo_take_cpus(t, max_ref, avail, allocated, needed, bind_policy, excl_policy, strategy, more);
        if (rc) return rc;
        for (int w = 0; w < 4; w++) res[w] |= more[w];
    }
    for (int w = 0; w < 4; w++) out[w] = res[w];
    return 0;
}
