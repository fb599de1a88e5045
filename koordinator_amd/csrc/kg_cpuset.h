// kg_cpuset.h — device cpuset accumulator (NodeNUMAResource cpuset binding for LSE/LSR pods).
//
// The reference picks a pod's CPUs with pkg/scheduler/plugins/nodenumaresource/cpu_accumulator.go
// (takeCPUs :88-246, takePreferredCPUs :30-86): a cascade of candidate groupings — full free cores per
// NUMA node, per socket, socket-sized chunks, spread CPUs per node / socket, and finally every free CPU
// in colocation order — each group sorted by the NUMA allocate strategy with id tie-breaks. Here one
// workgroup (one wave) runs one request; the CPU sets live in LDS, the per-CPU scans are spread over the
// 64 lanes (4 CPUs per lane, ballots build the membership masks and LDS atomics the per-core / per-group
// counts), and the short serial parts — group orderings over at most KG_CPU_GROUPS NUMA nodes or sockets,
// the core orderings and the take itself — run on lane 0 between barriers. Called from Reserve
// (apply_cpuset in kg_kernels.hip) and from the batch entry kg_cpuset_take; the Filter only needs the
// counts maintained in CpuRec (cpu_counts), not a take.
#pragma once
#include <hip/hip_runtime.h>

#include "kg_layout.h"
#include "../../include/koordgpu.h"

namespace kg {

constexpr int CPU_MAX = KG_MAX_CPUS;
constexpr int CPU_GROUPS = 8;      // NUMA nodes / sockets per node on the device path
constexpr int CPU_PER_CORE_MAX = 8;

struct CpuTake {  // one request: the arguments of takeCPUs / takePreferredCPUs
    uint64_t avail[4], preferred[4];
    int32_t needed, max_ref, bind, excl, strategy, has_preferred;
};

// LDS state of one accumulator (per workgroup).
struct CpuAccLds {
    uint8_t avail[CPU_MAX];      // allocatableCPUs
    uint8_t ref[CPU_MAX];        // RefCount (maxRefCount > 1)
    uint8_t excl_core[CPU_MAX];  // exclusiveInCores
    uint8_t excl_node[CPU_MAX];  // exclusiveInNUMANodes
    uint8_t result[CPU_MAX];
    uint8_t in[CPU_MAX];         // scratch membership
    uint8_t cnt[CPU_MAX];        // per core: CPUs in `in`
    uint8_t ccpu[CPU_MAX][CPU_PER_CORE_MAX];  // per core: its CPUs in `in`, ascending
    int16_t corder[CPU_MAX];     // scratch core list
    int16_t lists[CPU_GROUPS][CPU_MAX];
    int16_t nlist[CPU_GROUPS];
    int16_t gorder[CPU_GROUPS];
    int16_t flist[CPU_MAX];      // freeCPUs list
    int16_t tmp[CPU_MAX];
    int32_t gfree_node[CPU_GROUPS], gfree_sock[CPU_GROUPS], colo[CPU_GROUPS];
    int32_t needed, ngroups, nflist;
};

struct CpuAccDev {
    const kg_cpu_topo* t;
    CpuAccLds* s;
    int max_ref, excl_policy, strategy, exclusive;
    __device__ int cpc() const { return t->n_cores ? t->n_cpus / t->n_cores : 0; }
    __device__ int cpn() const { return t->n_nodes ? t->n_cpus / t->n_nodes : 0; }
    __device__ int cps() const { return t->n_sockets ? t->n_cpus / t->n_sockets : 0; }
    __device__ bool excl_pcpu(int c) const { return excl_policy == KG_CPU_EXCL_PCPU_LEVEL && s->excl_core[t->core[c]]; }
    __device__ bool excl_numa(int c) const { return excl_policy == KG_CPU_EXCL_NUMA_NODE_LEVEL && s->excl_node[t->numa[c]]; }
    // <0: i before j (MostAllocated: fewer free first; LeastAllocated: more free first)
    __device__ int free_order(int fi, int fj) const { return strategy == KG_NUMA_MOST_ALLOCATED ? fi - fj : fj - fi; }

    // lane 0 only
    __device__ void take(const int16_t* cpus, int n) {
        for (int k = 0; k < n; k++) {
            const int c = cpus[k];
            s->result[c] = 1;
            s->avail[c] = 0;
            if (exclusive) {
                if (excl_policy == KG_CPU_EXCL_PCPU_LEVEL) s->excl_core[t->core[c]] = 1;
                else if (excl_policy == KG_CPU_EXCL_NUMA_NODE_LEVEL) s->excl_node[t->numa[c]] = 1;
            }
        }
        s->needed -= n;
    }
    __device__ int core_ref(int core) const {
        int r = 0;
        for (int i = 0; i < t->n_cpus; i++)
            if (s->avail[i] && t->core[i] == core) r += s->ref[i];
        return r;
    }
    __device__ void sort_by_ref(int16_t* c, int n) const {
        for (int i = 1; i < n; i++) {
            const int16_t x = c[i];
            int j = i - 1;
            while (j >= 0 && (s->ref[c[j]] > s->ref[x] || (s->ref[c[j]] == s->ref[x] && c[j] > x))) {
                c[j + 1] = c[j];
                j--;
            }
            c[j + 1] = x;
        }
    }

    // ---- wave-parallel: membership `in` and per-core CPU lists (all lanes; barrier inside) ----
    // mode 0: every allocatable CPU; 1: minus NUMA-level exclusive; 2: minus PCPU-level exclusive;
    // 3: minus both
    __device__ void build_in(int mode) {
        const int lane = threadIdx.x;
        for (int c = lane; c < CPU_MAX; c += 64) {
            bool x = c < t->n_cpus && s->avail[c];
            if (x && (mode & 1) && excl_numa(c)) x = false;
            if (x && (mode & 2) && excl_pcpu(c)) x = false;
            s->in[c] = x ? 1 : 0;
            s->cnt[c] = 0;
        }
        __syncthreads();
        if (lane == 0) {  // ascending CPU order within each core
            for (int c = 0; c < t->n_cpus; c++)
                if (s->in[c]) {
                    const int core = t->core[c];
                    if (s->cnt[core] < CPU_PER_CORE_MAX) s->ccpu[core][s->cnt[core]] = (uint8_t)c;
                    s->cnt[core]++;
                }
        }
        __syncthreads();
    }

    // core order inside a group (sortCores): more CPUs, smaller RefCount (maxRefCount > 1), core id
    __device__ bool core_before(int a, int b) const {
        if (s->cnt[a] != s->cnt[b]) return s->cnt[a] > s->cnt[b];
        if (max_ref > 1) {
            const int ra = core_ref(a), rb = core_ref(b);
            if (ra != rb) return ra < rb;
        }
        return a < b;
    }

    // freeCoresInNode (by_node) / freeCoresInSocket; lane 0, after build_in. Fills lists in group order.
    __device__ void free_cores(bool by_node, bool filter_full) {
        const int ng = by_node ? t->n_nodes : t->n_sockets;
        int sock_free[CPU_GROUPS];
        for (int g = 0; g < CPU_GROUPS; g++) sock_free[g] = 0;
        for (int c = 0; c < t->n_cpus; c++)
            if (s->in[c]) sock_free[t->socket[c]]++;
        int16_t glist[CPU_GROUPS];
        int n = 0;
        for (int g = 0; g < ng; g++) {
            int m = 0;
            for (int core = 0; core < t->n_cores; core++) {
                if (!s->cnt[core] || (filter_full && s->cnt[core] != cpc())) continue;
                const int c0 = s->ccpu[core][0];
                if ((by_node ? t->numa[c0] : t->socket[c0]) != g) continue;
                int y = m - 1;  // insertion by core_before
                while (y >= 0 && core_before(core, s->corder[y])) {
                    s->corder[y + 1] = s->corder[y];
                    y--;
                }
                s->corder[y + 1] = (int16_t)core;
                m++;
            }
            if (!m) continue;
            int16_t* l = s->lists[n];
            int k = 0;
            for (int q = 0; q < m; q++) {
                const int core = s->corder[q];
                for (int z = 0; z < s->cnt[core]; z++) l[k++] = s->ccpu[core][z];
            }
            s->nlist[n] = (int16_t)k;
            glist[n] = (int16_t)g;
            n++;
        }
        // group order over the built lists (insertion, by the strategy on free CPUs, node groups then by their
        // socket's free CPUs, then id); lists are permuted through gorder
        for (int x = 0; x < n; x++) s->gorder[x] = (int16_t)x;
        for (int x = 1; x < n; x++) {
            const int v = s->gorder[x];
            int y = x - 1;
            while (y >= 0) {
                const int u = s->gorder[y];
                int d = free_order(s->nlist[v], s->nlist[u]);
                if (d == 0 && by_node) d = free_order(sock_free[t->socket[s->lists[v][0]]], sock_free[t->socket[s->lists[u][0]]]);
                if (d == 0) d = glist[v] - glist[u];
                if (d >= 0) break;
                s->gorder[y + 1] = s->gorder[y];
                y--;
            }
            s->gorder[y + 1] = (int16_t)v;
        }
        s->ngroups = n;
    }

    // freeCPUsInNode (by_node) / freeCPUsInSocket; lane 0, after build_in(by_node ? 3 : 2 or 0)
    __device__ void free_cpus_grouped(bool by_node, bool filter_excl) {
        const int ng = by_node ? t->n_nodes : t->n_sockets;
        int node_free[CPU_GROUPS], sock_free[CPU_GROUPS];
        for (int g = 0; g < CPU_GROUPS; g++) node_free[g] = sock_free[g] = 0;
        int16_t glist[CPU_GROUPS];
        int n = 0;
        for (int c = 0; c < t->n_cpus; c++)
            if (s->in[c]) {
                node_free[t->numa[c]]++;
                sock_free[t->socket[c]]++;
            }
        for (int g = 0; g < ng; g++) {
            int16_t* l = s->lists[n];
            int k = 0;
            for (int c = 0; c < t->n_cpus; c++)
                if (s->in[c] && (by_node ? t->numa[c] : t->socket[c]) == g) l[k++] = (int16_t)c;
            if (!k) continue;
            if (max_ref > 1) sort_by_ref(l, k);
            if (filter_excl) {  // extractCPU: first CPU of each core
                int m = 0;
                for (int q = 0; q < k; q++) {
                    bool seen = false;
                    for (int r = 0; r < m && !seen; r++) seen = t->core[l[r]] == t->core[l[q]];
                    if (!seen) l[m++] = l[q];
                }
                k = m;
            }
            s->nlist[n] = (int16_t)k;
            glist[n] = (int16_t)g;
            n++;
        }
        for (int x = 0; x < n; x++) s->gorder[x] = (int16_t)x;
        for (int x = 1; x < n; x++) {
            const int v = s->gorder[x];
            int y = x - 1;
            while (y >= 0) {
                const int u = s->gorder[y];
                int d;
                if (by_node) {
                    d = free_order(node_free[glist[v]], node_free[glist[u]]);
                    if (d == 0) d = free_order(sock_free[t->socket[s->lists[v][0]]], sock_free[t->socket[s->lists[u][0]]]);
                } else {
                    d = free_order(s->nlist[v], s->nlist[u]);
                }
                if (d == 0) d = glist[v] - glist[u];
                if (d >= 0) break;
                s->gorder[y + 1] = s->gorder[y];
                y--;
            }
            s->gorder[y + 1] = (int16_t)v;
        }
        s->ngroups = n;
    }

    // freeCPUs; lane 0, after build_in(3 or 0)
    __device__ void free_cpus() {
        int node_free[CPU_GROUPS], sock_free[CPU_GROUPS], colo[CPU_GROUPS];
        for (int g = 0; g < CPU_GROUPS; g++) node_free[g] = sock_free[g] = colo[g] = 0;
        for (int c = 0; c < t->n_cpus; c++) {
            if (s->in[c]) {
                node_free[t->numa[c]]++;
                sock_free[t->socket[c]]++;
            }
            if (s->result[c]) colo[t->socket[c]]++;
        }
        int m = 0;
        for (int core = 0; core < t->n_cores; core++) {
            if (!s->cnt[core]) continue;
            const int sv = t->socket[s->ccpu[core][0]], nv = t->numa[s->ccpu[core][0]];
            int y = m - 1;
            while (y >= 0) {
                const int u = s->corder[y];
                const int su = t->socket[s->ccpu[u][0]], nu = t->numa[s->ccpu[u][0]];
                int d = colo[su] - colo[sv];
                if (d == 0) d = free_order(sock_free[sv], sock_free[su]);
                if (d == 0) d = free_order(node_free[nv], node_free[nu]);
                if (d == 0) d = s->cnt[core] - s->cnt[u];
                if (d == 0) d = sv - su;
                if (d == 0 && max_ref > 1) d = core_ref(core) - core_ref(u);
                if (d == 0) d = core - u;
                if (d >= 0) break;
                s->corder[y + 1] = s->corder[y];
                y--;
            }
            s->corder[y + 1] = (int16_t)core;
            m++;
        }
        int k = 0;
        for (int q = 0; q < m; q++) {
            const int core = s->corder[q];
            int16_t cp[CPU_PER_CORE_MAX];
            const int z = s->cnt[core];
            for (int r = 0; r < z; r++) cp[r] = s->ccpu[core][r];
            if (max_ref > 1) sort_by_ref(cp, z);
            for (int r = 0; r < z; r++) s->flist[k++] = cp[r];
        }
        s->nflist = k;
    }

    // spreadCPUs in place (lane 0)
    __device__ void spread(int16_t* l, int n) {
        if (n <= cpc()) return;
        int16_t* out = s->tmp;
        int k = 0;
        uint64_t taken[4] = {0, 0, 0, 0};  // CPUs already emitted
        while (k < n) {
            uint64_t seen[4] = {0, 0, 0, 0};  // cores visited in this pass
            for (int q = 0; q < n; q++) {
                const int c = l[q];
                if ((taken[c >> 6] >> (c & 63)) & 1ull) continue;
                const int core = t->core[c];
                if ((seen[core >> 6] >> (core & 63)) & 1ull) continue;
                seen[core >> 6] |= 1ull << (core & 63);
                taken[c >> 6] |= 1ull << (c & 63);
                out[k++] = (int16_t)c;
            }
        }
        for (int q = 0; q < n; q++) l[q] = out[q];
    }
};

// takeCPUs of one request, the whole wave participating; returns 0 / -1 ErrNotEnoughCPUs / -2 failed.
// avail: allocatable CPUs of this call (the preferred subset in takePreferredCPUs' first round).
__device__ inline int cpuset_take_one(CpuAccDev& a, const uint64_t* avail, const kg_cpu_alloc* al, int needed, int bind) {
    CpuAccLds* s = a.s;
    const kg_cpu_topo* t = a.t;
    const int lane = threadIdx.x;
    for (int c = lane; c < CPU_MAX; c += 64) {
        const bool av = c < t->n_cpus && ((avail[c >> 6] >> (c & 63)) & 1ull);
        s->avail[c] = av ? 1 : 0;
        s->ref[c] = (a.max_ref > 1 && av && al) ? al->ref[c] : 0;
        s->excl_core[c] = 0;
        s->excl_node[c] = 0;
        s->result[c] = 0;
    }
    __syncthreads();
    if (lane == 0) {
        s->needed = needed;
        if (al)
            for (int c = 0; c < t->n_cpus; c++) {
                if (al->excl[c] == KG_CPU_EXCL_PCPU_LEVEL) s->excl_core[t->core[c]] = 1;
                else if (al->excl[c] == KG_CPU_EXCL_NUMA_NODE_LEVEL) s->excl_node[t->numa[c]] = 1;
            }
    }
    __syncthreads();
    int navail = 0;
    for (int c = lane; c < CPU_MAX; c += 64) navail += s->avail[c];
    for (int off = 32; off > 0; off >>= 1) navail += __shfl_xor(navail, off, 64);
    if (needed < 1) return 0;
    if (needed > navail) return -1;
    const bool full = bind == KG_CPU_BIND_FULL_PCPUS;
    bool done = false;  // wave-uniform (read from LDS after each lane-0 step)
    __shared__ int s_done;
    if (lane == 0) s_done = 0;
    __syncthreads();
    auto sync_done = [&]() {
        __syncthreads();
        done = s_done != 0;
    };
    auto try_lists = [&](bool spread_it) {  // lane 0: first group whose list holds the request
        for (int k = 0; k < s->ngroups; k++) {
            int16_t* l = s->lists[s->gorder[k]];
            const int n = s->nlist[s->gorder[k]];
            if (n >= s->needed) {
                if (spread_it) a.spread(l, n);
                a.take(l, s->needed);
                s_done = 1;
                return;
            }
        }
    };
    if (full || a.cpc() == 1) {
        if (s->needed <= a.cpn()) {
            for (int fe = 1; fe >= 0 && !done; fe--) {
                a.build_in(fe ? 1 : 0);
                if (lane == 0) {
                    a.free_cores(true, true);
                    try_lists(false);
                }
                sync_done();
            }
        }
        if (!done && s->needed <= a.cps()) {
            a.build_in(0);
            if (lane == 0) {
                a.free_cores(false, true);
                try_lists(false);
            }
            sync_done();
        }
        if (!done) {
            a.build_in(0);
            if (lane == 0) {
                a.free_cores(false, true);
                // stable by length, descending
                const int n = s->ngroups;
                int16_t* o = s->gorder;
                for (int x = 1; x < n; x++) {
                    const int16_t v = o[x];
                    int y = x - 1;
                    while (y >= 0 && s->nlist[o[y]] < s->nlist[v]) {
                        o[y + 1] = o[y];
                        y--;
                    }
                    o[y + 1] = v;
                }
                int16_t un[CPU_GROUPS];
                int nu = 0;
                for (int k = 0; k < n && !s_done; k++) {
                    const int g = o[k];
                    if (!(s->needed >= s->nlist[g])) {
                        un[nu++] = (int16_t)g;
                    } else {
                        a.take(s->lists[g], s->nlist[g]);
                        if (s->needed < 1) s_done = 1;
                    }
                }
                const int step = a.cpc();
                if (!s_done && s->needed >= step) {
                    for (int x = 1; x < nu; x++) {  // stable by length, ascending
                        const int16_t v = un[x];
                        int y = x - 1;
                        while (y >= 0 && s->nlist[un[y]] > s->nlist[v]) {
                            un[y + 1] = un[y];
                            y--;
                        }
                        un[y + 1] = v;
                    }
                    for (int k = 0; k < nu && !s_done; k++) {
                        const int g = un[k];
                        for (int i = 0; i < s->nlist[g]; i += step) {
                            a.take(s->lists[g] + i, step);
                            if (s->needed < 1) {
                                s_done = 1;
                                break;
                            }
                            if (!(s->needed >= step)) break;
                        }
                    }
                }
            }
            sync_done();
        }
    }
    if (!done && !full) {
        if (s->needed <= a.cpn()) {
            for (int fe = 1; fe >= 0 && !done; fe--) {
                a.build_in(fe ? 3 : 0);
                if (lane == 0) {
                    a.free_cpus_grouped(true, fe != 0);
                    try_lists(true);
                }
                sync_done();
            }
        }
        if (!done && s->needed <= a.cps()) {
            for (int fe = 1; fe >= 0 && !done; fe--) {
                a.build_in(fe ? 2 : 0);
                if (lane == 0) {
                    a.free_cpus_grouped(false, fe != 0);
                    try_lists(true);
                }
                sync_done();
            }
        }
    }
    for (int fe = 1; fe >= 0 && !done; fe--) {
        a.build_in(fe ? 3 : 0);
        if (lane == 0) {
            a.free_cpus();
            a.spread(s->flist, s->nflist);
            for (int k = 0; k < s->nflist; k++) {
                if (s->needed >= 1) a.take(&s->flist[k], 1);
                if (s->needed < 1) {
                    s_done = 1;
                    break;
                }
            }
        }
        sync_done();
    }
    return done ? 0 : -2;
}

// takePreferredCPUs (cpu_accumulator.go:30-86) of one request; out = result mask (all lanes see it).
__device__ inline int cpuset_take(const kg_cpu_topo* t, const kg_cpu_alloc* al, const CpuTake& q, CpuAccLds* s,
                                  uint64_t out[4]) {
    CpuAccDev a;
    a.t = t;
    a.s = s;
    a.max_ref = q.max_ref;
    a.excl_policy = q.excl;
    a.strategy = q.strategy;
    a.exclusive = q.excl == (int)KG_CPU_EXCL_PCPU_LEVEL || q.excl == (int)KG_CPU_EXCL_NUMA_NODE_LEVEL;
    uint64_t avail[4], pref[4], res[4] = {0, 0, 0, 0};
    int np = 0, needed = q.needed;
    for (int w = 0; w < 4; w++) {
        avail[w] = q.avail[w];
        pref[w] = q.has_preferred ? (q.avail[w] & q.preferred[w]) : 0ull;
        np += __popcll(pref[w]);
    }
    auto harvest = [&](uint64_t* m) {
        for (int w = 0; w < 4; w++) {
            uint64_t b = 0;
            for (int k = 0; k < 64; k++)
                if (s->result[w * 64 + k]) b |= 1ull << k;
            m[w] = b;
        }
    };
    if (np) {
        const int n = needed < np ? needed : np;
        const int rc = cpuset_take_one(a, pref, al, n, q.bind);
        uint64_t r1[4];
        harvest(r1);
        __syncthreads();
        if (rc) {
            for (int w = 0; w < 4; w++) out[w] = r1[w];
            return rc;
        }
        for (int w = 0; w < 4; w++) {
            res[w] = r1[w];
            needed -= __popcll(r1[w]);
            avail[w] &= ~pref[w];
        }
    }
    if (needed > 0) {
        const int rc = cpuset_take_one(a, avail, al, needed, q.bind);
        uint64_t r2[4];
        harvest(r2);
        __syncthreads();
        if (rc) {
            for (int w = 0; w < 4; w++) out[w] = 0;
            return rc;
        }
        for (int w = 0; w < 4; w++) res[w] |= r2[w];
    }
    for (int w = 0; w < 4; w++) out[w] = res[w];
    return 0;
}

}  // namespace kg
