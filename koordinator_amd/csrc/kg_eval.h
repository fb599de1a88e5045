// kg_eval.h — per-(pod, node) Filter/Score arithmetic on the device.
//
// One function evaluates every enabled plugin for one pair; the kernels differ only in how they
// map pairs to lanes. The arithmetic restates (with the same integer results):
//   NodeResourcesFit Fits + LeastAllocated   upstream k8s v1.35.6,
//                                            mirror noderesourcefitplus/node_resource_fit_plus_utils.go:47-139
//   LoadAwareScheduling Filter / Score       loadaware/load_aware.go:150-220, 235-292, 316-376
//   NodeNUMAResource Filter / Score          nodenumaresource/plugin.go:363-498, scoring.go:67-151,
//                                            topology_hint.go:31-41, resource_manager.go:272-318,529-626,
//                                            frameworkext/topologymanager/policy.go:198-256
// Divisions: Go's truncating int64 division of non-negative operands is computed as an exactly
// corrected IEEE-double quotient (operands are < 2^46 — the host checks and otherwise selects the
// EXACT=true instantiation that divides in int64). The LoadAware usage-percent filter
// int64(math.Round(float64(e)/float64(t)*100)) <= thr is monotone in e; the host turns it into an
// exact integer cut-off per node, so the kernel compares integers only.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/koordgpu.h"
#include "kg_layout.h"

namespace kg {

// XCD-aware workgroup order of a (pod block x, record chunk y) select grid. Workgroups are dealt round-robin over
// the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch), each with its own L2, so in launch order every XCD's L2
// would pull every record chunk. Renumbering the workgroups dealt to one XCD as a contiguous run of the chunk-major
// order gives each XCD whole chunks (all their pod blocks): a chunk's records come from HBM once. Block order
// changes no result (keys are merged by atomicMax or stored per (chunk, pod)).
struct GridBlock {
    uint32_t x, y;
};
__device__ __forceinline__ GridBlock xcd_block() {
    const uint32_t gx = gridDim.x, total = gx * gridDim.y;
    const uint32_t l = blockIdx.x + blockIdx.y * gx;
    const uint32_t full = total & ~7u;  // the tail of < 8 workgroups keeps its place
    const uint32_t n = l < full ? (l & 7u) * (full >> 3) + (l >> 3) : l;
    return {n % gx, n / gx};
}

struct PodV {
    int64_t req_cpu, req_mem, req_eph, sc0, sc1, nz_cpu, nz_mem, est0, est1;
    uint32_t flags;
};

__device__ __forceinline__ PodV load_pod(const PodsDev& P, uint32_t j) {
    PodV p;
    p.req_cpu = P.req_cpu[j];
    p.req_mem = P.req_mem[j];
    p.req_eph = P.req_eph[j];
    p.sc0 = P.sc_req0[j];
    p.sc1 = P.sc_req1[j];
    p.nz_cpu = P.nz_cpu[j];
    p.nz_mem = P.nz_mem[j];
    p.est0 = P.la_est0[j];
    p.est1 = P.la_est1[j];
    p.flags = P.flags[j];
    return p;
}

__device__ __forceinline__ double as_f64(int64_t bits) { return __longlong_as_double(bits); }

// leastRequestedScore(requested, capacity) = ((capacity - requested) * 100) / capacity,
// 0 when capacity == 0 or requested > capacity.
template <bool EXACT>
__device__ __forceinline__ int64_t least_req(int64_t requested, int64_t capacity, double rcp) {
    const int64_t x = capacity - requested;
    const bool zero = (capacity == 0) | (x < 0);
    if constexpr (EXACT) {
        const int64_t cap = zero ? 1 : capacity;
        return zero ? 0 : ((zero ? 0 : x) * 100) / cap;
    } else {
        const double cap_d = (double)capacity;
        const double t = (double)x * 100.0;  // exact when |x| < 2^46
        double q = floor(t * rcp);
        const double r = fma(-q, cap_d, t);  // exact remainder t - q*cap
        q += (r < 0.0) ? -1.0 : ((r >= cap_d) ? 1.0 : 0.0);
        int64_t s = (int64_t)(int32_t)q;
        // operands outside the exact-double range (|x| or capacity >= 2^46): Go's int64 arithmetic
        // (wrapping multiply, truncating divide) on the rare lanes that need it
        const bool big = ((uint64_t)(x + (1ll << 46)) >= (1ull << 47)) | (capacity >= (1ll << 46));
        if (__builtin_expect(big & !zero, 0)) s = (int64_t)((uint64_t)x * 100ull) / capacity;
        return zero ? 0 : s;
    }
}

// Σ score / Σ weight for small non-negative operands (weights are validated on the host).
__device__ __forceinline__ int64_t wdiv(int64_t sum, int64_t wsum) {
    return wsum == 0 ? 0 : (int64_t)((uint32_t)sum / (uint32_t)(wsum == 0 ? 1 : wsum));
}

template <bool EXACT>
__device__ __forceinline__ int64_t numa_least(int64_t w_cpu, int64_t w_mem, int64_t alloc_cpu, int64_t req_cpu,
                                              double rcp_cpu, int64_t alloc_mem, int64_t req_mem, double rcp_mem) {
    int64_t sum = 0, wsum = 0;
    const bool on_c = (alloc_cpu != 0) & (w_cpu != 0);
    const bool on_m = (alloc_mem != 0) & (w_mem != 0);
    sum += on_c ? least_req<EXACT>(req_cpu, alloc_cpu, rcp_cpu) * w_cpu : 0;
    wsum += on_c ? w_cpu : 0;
    sum += on_m ? least_req<EXACT>(req_mem, alloc_mem, rcp_mem) * w_mem : 0;
    wsum += on_m ? w_mem : 0;
    return wdiv(sum, wsum);
}

// Go's truncating a / c for a score-sized quotient. For 0 <= a < 2^62, 0 < c < 2^62 and a / c < 2^18,
// a * v_rcp_f64(c) is within 2^-22 relative of a / c even at single-precision reciprocal accuracy, so
// it is within 1/16 absolute, its floor is off by at most one and the exact int64 remainder a - q*c
// fixes it; every other operand pair takes the int64 divide.
__device__ __forceinline__ int64_t qdiv(int64_t a, int64_t c) {
    const bool ok = (a >= 0) & (c > 0) & (a < (1ll << 62)) & (c < (1ll << 62));
    const double est = floor((double)a * __builtin_amdgcn_rcp((double)c));
    if (__builtin_expect(!ok || !(est < 262144.0), 0)) return c == 0 ? 0 : a / c;
    int64_t q = (int64_t)(int32_t)est;
    const int64_t r = a - q * c;
    q += (r < 0) ? -1 : ((r >= c) ? 1 : 0);
    return q;
}

__device__ __forceinline__ int64_t most_req(int64_t requested, int64_t capacity) {
    if (capacity == 0) return 0;
    if (requested > capacity) requested = capacity;
    return qdiv(requested * 100, capacity);
}

// LeastAllocated / MostAllocated over {cpu, memory} (nodenumaresource least_allocated.go / most_allocated.go)
template <bool EXACT>
__device__ __forceinline__ int64_t numa_score(bool most, int64_t w_cpu, int64_t w_mem, int64_t alloc_cpu, int64_t req_cpu,
                                              double rcp_cpu, int64_t alloc_mem, int64_t req_mem, double rcp_mem) {
    if (!most) return numa_least<EXACT>(w_cpu, w_mem, alloc_cpu, req_cpu, rcp_cpu, alloc_mem, req_mem, rcp_mem);
    int64_t sum = 0, wsum = 0;
    if (alloc_cpu != 0 && w_cpu != 0) {
        sum += most_req(req_cpu, alloc_cpu) * w_cpu;
        wsum += w_cpu;
    }
    if (alloc_mem != 0 && w_mem != 0) {
        sum += most_req(req_mem, alloc_mem) * w_mem;
        wsum += w_mem;
    }
    return wsum == 0 ? 0 : qdiv(sum, wsum);
}

// ---- NUMA topology manager for non-cpuset pods: hints (resource_manager.go:529-657) and the
//      SingleNUMANode / Restricted / BestEffort merge (frameworkext/topologymanager/policy*.go).
//      Same results as oracle/kg_oracle.c numa_hints / numa_admit, restated for registers: the hint lists
//      are bitmasks over the mask index k (IterateBitMasks order), the per-mask hint scores (0..100) are
//      packed 8 bits each, zone-indexed values are read through select chains. No private arrays, so no
//      scratch memory on the integer path.

// NUMA masks of IterateBitMasks (pkg/util/bitmask/bitmask.go:206-221) for Z = 1..4 zones, 4 bits per mask index
constexpr uint64_t NUMA_MASK_NIB[4] = {0x1ull, 0x321ull, 0x7653421ull, 0xfedb7ca69538421ull};

__device__ __forceinline__ uint64_t numa_mask_nib(uint32_t Z) {
    return Z <= 1 ? NUMA_MASK_NIB[0] : Z == 2 ? NUMA_MASK_NIB[1] : Z == 3 ? NUMA_MASK_NIB[2] : NUMA_MASK_NIB[3];
}

struct NumaZ {
    uint32_t Z, status;
    int64_t tot[2][MAX_ZONES], used[2][MAX_ZONES], avail[2][MAX_ZONES];
};

__device__ __forceinline__ void numa_load(const ZoneRec* __restrict__ zr, uint32_t Z, NumaZ& x) {
    x.Z = Z;
    x.status = zr->status;
    for (uint32_t z = 0; z < (uint32_t)MAX_ZONES; z++) {
        const bool on = z < Z;
        x.tot[0][z] = on ? zr->cpu[z] : 0;
        x.tot[1][z] = on ? zr->mem[z] : 0;
        x.used[0][z] = on ? zone_cpu_alloc(*zr, z) : 0;
        x.used[1][z] = on ? zr->mem_used[z] : 0;
        for (int r = 0; r < 2; r++) x.avail[r][z] = x.tot[r][z] - x.used[r][z] < 0 ? 0 : x.tot[r][z] - x.used[r][z];
    }
}

__device__ __forceinline__ int64_t sel4(const int64_t (&a)[MAX_ZONES], uint32_t i) {
    return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}

// Go's truncating q / d for the split divisor d in 1..4 (constant divisions, no int64 divide loop)
__device__ __forceinline__ int64_t div_small(int64_t q, uint32_t d) {
    return d == 1 ? q : d == 2 ? q / 2 : d == 3 ? q / 3 : q / 4;
}

// tryBestToDistributeEvenly of one resource over the zones of `mask` (resource_manager.go:264-318): the
// zone order comes from sort.Slice whose less(i, j) reads the availability by the positions i, j rather
// than by the zone ids being sorted (insertion sort for n <= 12, so the swaps depend only on the
// availability of zones 0..n-1); each zone in turn takes min(available, remaining / zones left).
// Returns whether the whole request was placed; AL: the per-zone amounts into al (added).
// bm (cpu of a cpuset-binding pod, splitQuantity :320-334): 1 = whole CPUs of quantity.Value() (rounded up), 2 = whole
// cores of cpc CPUs (required FullPCPUs); 0 = the quantity itself (milli-cpu / bytes).
template <bool AL>
__device__ __forceinline__ bool numa_split_r(const NumaZ& x, uint32_t mask, const int64_t (&av)[MAX_ZONES], int64_t req,
                                             int64_t (&al)[MAX_ZONES], int bm = 0, int64_t cpc = 1) {
    uint32_t s = 0, n = 0;  // the mask's zones, ascending, 4 bits per position
#pragma unroll
    for (uint32_t z = 0; z < (uint32_t)MAX_ZONES; z++) {
        const bool in = z < x.Z && ((mask >> z) & 1u);
        s |= in ? z << (4 * n) : 0u;
        n += in ? 1u : 0u;
    }
#pragma unroll
    for (uint32_t a = 1; a < (uint32_t)MAX_ZONES; a++) {
        bool go = a < n;
#pragma unroll
        for (uint32_t b = a; b > 0; b--) {
            go = go && av[b] < av[b - 1];
            if (go) {  // swap positions b and b - 1
                const uint32_t hi = (s >> (4 * b)) & 15u, lo = (s >> (4 * (b - 1))) & 15u;
                s = (s & ~(0xFFu << (4 * (b - 1)))) | (hi << (4 * (b - 1))) | (lo << (4 * b));
            }
        }
    }
    int64_t q = req;
#pragma unroll
    for (uint32_t t = 0; t < (uint32_t)MAX_ZONES; t++) {
        if (t >= n) break;
        int64_t split = div_small(q, n - t);
        if (bm) {
            const int64_t v = (q + 999) / 1000;
            split = bm == 2 ? div_small(v / cpc, n - t) * cpc * 1000 : div_small(v, n - t) * 1000;
        }
        const uint32_t zone = (s >> (4 * t)) & 15u;
        const int64_t a0 = sel4(av, zone);
        const int64_t got = a0 > split ? split : a0;
        if constexpr (AL) {
#pragma unroll
            for (uint32_t zz = 0; zz < (uint32_t)MAX_ZONES; zz++) al[zz] += (zz == zone) ? got : 0;
        }
        q -= got;
    }
    return q == 0;
}

__device__ __forceinline__ int popc(uint32_t x) { return __popc(x); }

// leastRequestedScore with an exact truncating quotient (qdiv), the integer path's arithmetic
__device__ __forceinline__ int64_t least_req_q(int64_t requested, int64_t capacity) {
    const int64_t x = capacity - requested;
    if (capacity == 0 || x < 0) return 0;
    return qdiv(x * 100, capacity);
}

// NUMA LeastAllocated / MostAllocated over {cpu, memory} with exact integer quotients
__device__ __forceinline__ int64_t numa_score_q(bool most, int64_t w_cpu, int64_t w_mem, int64_t alloc_cpu, int64_t req_cpu,
                                                int64_t alloc_mem, int64_t req_mem) {
    int64_t sum = 0, wsum = 0;
    if (alloc_cpu != 0 && w_cpu != 0) {
        sum += (most ? most_req(req_cpu, alloc_cpu) : least_req_q(req_cpu, alloc_cpu)) * w_cpu;
        wsum += w_cpu;
    }
    if (alloc_mem != 0 && w_mem != 0) {
        sum += (most ? most_req(req_mem, alloc_mem) : least_req_q(req_mem, alloc_mem)) * w_mem;
        wsum += w_mem;
    }
    if (wsum == 0) return 0;
    return most ? qdiv(sum, wsum) : wdiv(sum, wsum);
}

// A cpuset-binding pod under a NUMA policy (oracle numa_bind, resource_manager.go:168-194,320-334,357-463): the CPU
// side of every allocation under a hint. cnt: the available CPUs per NUMA node after the required policy's filter
// (ZoneRec.cz_*).
struct NumaBind {
    bool required, full;
    int64_t cpc, needed;
    int64_t cnt[MAX_ZONES];
};

__device__ __forceinline__ NumaBind numa_bind_of(const ZoneRec* __restrict__ zr, bool required, uint32_t bind, int64_t pod_cpu) {
    NumaBind b;
    b.required = required;
    b.full = bind == KG_CPU_BIND_FULL_PCPUS;
    b.cpc = (zr->cpu_meta >> CPU_META_CPC_SHIFT) & 15u;
    b.needed = pod_cpu / 1000;
#pragma unroll
    for (int z = 0; z < MAX_ZONES; z++)
        b.cnt[z] = !required ? zr->cz_free[z] : b.full ? zr->cz_full[z] : zr->cz_cores[z];
    return b;
}

__device__ __forceinline__ int numa_bind_mode(const NumaBind* b) { return !b ? 0 : (b->required && b->full) ? 2 : 1; }

// trimNUMANodeResources (:168-194): a required policy's available cpu per NUMA node at most its filtered CPUs
__device__ __forceinline__ void numa_bind_trim(NumaZ& x, const NumaBind& b) {
    if (!b.required) return;
#pragma unroll
    for (int z = 0; z < MAX_ZONES; z++) x.avail[0][z] = min(x.avail[0][z], b.cnt[z] * 1000);
}

// allocateCPUSet over the allocated NUMA nodes (:391-429): min(available CPUs there, allocated cpu / 1000) per node,
// numCPUsNeeded together, whole cores each under a required FullPCPUs policy. 0, KG_ST_NUMA_CPUS or KG_ST_NUMA_CPU_BIND.
__device__ __forceinline__ uint32_t numa_bind_check(const NumaBind& b, const int64_t (&al0)[MAX_ZONES],
                                                    const int64_t (&al1)[MAX_ZONES], uint32_t Z) {
    int64_t sum = 0;
    bool partial = false;
#pragma unroll
    for (uint32_t z = 0; z < (uint32_t)MAX_ZONES; z++) {
        if (z >= Z || (al0[z] == 0 && al1[z] == 0)) continue;
        const int64_t k = min(b.cnt[z], al0[z] / 1000);
        sum += k;
        partial = partial || (b.required && b.full && b.cpc != 0 && k % b.cpc != 0);
    }
    if (sum != b.needed) return KG_ST_NUMA_CPUS;
    return partial ? (uint32_t)KG_ST_NUMA_CPU_BIND : 0u;
}

// requestCPUBind + getCPUBindPolicy (util.go:101-138) of a pair whose numa_eval checks passed: the pod's NumaBind
// and whether its CPUs fit the whole node (node_take); false when the pod binds no CPUs there
__device__ __forceinline__ bool numa_bind_pair(const ZoneRec* __restrict__ zr, const PodV& p, NumaBind& b, bool& node_take) {
    const uint32_t node_bind = (zr->cpu_meta >> CPU_META_BIND_SHIFT) & 3u;
    const bool cpu_bind = (p.flags & KG_POD_CPU_BIND) || (p.req_cpu != 0 && node_bind != KG_NODE_CPU_BIND_NONE);
    if (!cpu_bind || zr->cpu_topo < 0) return false;
    const uint32_t cpu_pol = (p.flags >> KG_POD_CPU_POLICY_SHIFT) & 3u;
    uint32_t required = (p.flags & KG_POD_CPU_REQUIRED) ? cpu_pol : KG_CPU_BIND_NONE;
    if (node_bind == KG_NODE_CPU_BIND_FULL_PCPUS_ONLY) required = KG_CPU_BIND_FULL_PCPUS;
    else if (node_bind == KG_NODE_CPU_BIND_SPREAD_BY_PCPUS) required = KG_CPU_BIND_SPREAD_BY_PCPUS;
    const int64_t have = required == KG_CPU_BIND_FULL_PCPUS    ? zr->cpu_free_full
                         : required == KG_CPU_BIND_SPREAD_BY_PCPUS ? zr->cpu_free_cores
                                                                   : zr->cpu_free;
    node_take = p.req_cpu / 1000 <= have;
    b = numa_bind_of(zr, required != KG_CPU_BIND_NONE, required != KG_CPU_BIND_NONE ? required : cpu_pol, p.req_cpu);
    return true;
}

struct NumaHint {
    uint32_t mask;  // 0 = nil affinity
    bool pref, unsat;
    int64_t score;
};

__device__ __forceinline__ bool numa_excl_ok(uint32_t mask, uint32_t status) {
    if (popc(mask) > 1) {
        for (uint32_t z = 0; z < (uint32_t)MAX_ZONES; z++)
            if (((mask >> z) & 1u) && ((status >> (2 * z)) & 3u) == 1u) return false;
        return true;
    }
    const uint32_t z = (uint32_t)(__ffs(mask) - 1);
    return ((status >> (2 * z)) & 3u) != 2u;
}

// mergePermutation + the bestHint update of mergeFilteredHints (policy.go:98-137,198-260) for a
// permutation of np = 0..3 hints (a, b, c3)
__device__ __forceinline__ void numa_merge_perm(uint32_t all, bool excl, uint32_t status, int np, const NumaHint& a,
                                                const NumaHint& b, NumaHint& best, const NumaHint& c3 = NumaHint{0u, true, false, 0}) {
    uint32_t merged = all, first = 0;
    bool pref = true, unsat = false;
    int naff = 0, maxc = 0;
#pragma unroll
    for (int t = 0; t < 3; t++) {
        if (t >= np) break;
        const NumaHint& v = t == 0 ? a : t == 1 ? b : c3;
        if (v.mask) {
            if (naff == 0) first = v.mask;
            else if (v.mask != first) pref = false;
            naff++;
            merged &= v.mask;
            maxc = max(maxc, popc(v.mask));
        }
        pref = pref && v.pref;
        unsat = unsat || v.unsat;
    }
    const bool satisfied = (naff == 0 || maxc == popc(merged)) && !unsat;
    if (popc(merged) == 0) return;
    if (excl && !numa_excl_ok(merged, status)) pref = false;
    int64_t score = 0;
    if (np >= 1 && a.mask && a.mask == merged) score += a.score;
    if (np >= 2 && b.mask && b.mask == merged) score += b.score;
    if (np >= 3 && c3.mask && c3.mask == merged) score += c3.score;
    const NumaHint m{merged, pref, !satisfied, score};
    if (m.pref && !best.pref) {
        best = m;
        return;
    }
    if (!m.pref && best.pref) return;
    const int cm = popc(m.mask), cb = popc(best.mask);
    const bool narrower = cm == cb ? m.mask < best.mask : cm < cb;
    if (!narrower) {
        if (cm == cb && m.score > best.score) best = m;
        return;
    }
    best = m;
}

constexpr uint32_t NUMA_NIL_K = 15u;  // hint-list bit of the unsatisfied nil hint (filterProvidersHints)

// DeviceShare's "gpu" hint list for the merge (deviceshare/topology_hint.go:159-280): entry t has the NUMA mask
// nibble t of `masks`, Preferred bit t of `pref`, Score 500 when bit t of `s500`; `set` holds the entries
// (after filterSingleNumaHints), NUMA_NIL_K = the provider's "no preference" hint (nil affinity, Preferred).
struct GpuHints {
    uint64_t masks;
    uint32_t set, pref, s500;
};

__device__ __forceinline__ NumaHint gpu_hint_at(const GpuHints& g, uint32_t t) {
    if (t == NUMA_NIL_K) return NumaHint{0u, true, false, 0};
    return NumaHint{(uint32_t)(g.masks >> (4 * t)) & 15u, ((g.pref >> t) & 1u) != 0, false,
                    ((g.s500 >> t) & 1u) ? 500 : 0};
}

__device__ __forceinline__ NumaHint numa_hint_at(uint64_t nib, uint32_t k, uint32_t pref_bits, uint64_t sc_lo, uint64_t sc_hi) {
    if (k == NUMA_NIL_K) return NumaHint{0u, false, true, 0};
    const uint32_t m = (uint32_t)(nib >> (4 * k)) & 15u;
    const uint64_t sc = k < 8 ? (sc_lo >> (8 * k)) : (sc_hi >> (8 * (k - 8)));
    return NumaHint{m, ((pref_bits >> k) & 1u) != 0, false, (int64_t)(sc & 0xFFu)};
}

// Policy merge: 0 = admitted with affinity `mask` (0 = none), else a KG_ST_NUMA_* reason. GPU: a third hint list,
// DeviceShare's (gh, provider order: NodeNUMAResource's cpu, memory, then DeviceShare's gpu).
// bind (nullable): a cpuset-binding pod (x already trimmed); score_cpu: the cpu request the hint scores count (amplified
// for a cpuset-binding pod, getResourceOptions plugin.go:774-778)
template <bool EXACT, bool GPU = false>
__device__ __forceinline__ uint32_t numa_admit(const KCfg& c, const NumaZ& x, const int64_t* req, const bool* has,
                                              uint32_t policy, bool excl, uint32_t& mask_out,
                                              const GpuHints* gh = nullptr, const NumaBind* bind = nullptr,
                                              int64_t score_cpu = -1) {
    if (score_cpu < 0) score_cpu = req[0];
    const uint32_t Z = x.Z;
    const uint64_t nib = numa_mask_nib(Z);
    const uint32_t nm = (1u << Z) - 1u;
    uint32_t lack0 = 0, lack1 = 0;
#pragma unroll
    for (uint32_t z = 0; z < (uint32_t)MAX_ZONES; z++) {
        if (z >= Z) break;
        lack0 |= x.avail[0][z] == 0 ? 1u << z : 0u;
        lack1 |= x.avail[1][z] == 0 ? 1u << z : 0u;
    }
    uint32_t okm0 = 0, okm1 = 0;
    int min0 = (int)Z, min1 = (int)Z;
    uint64_t sc_lo = 0, sc_hi = 0;  // hint score of mask k (0..100), 8 bits each
    const bool most_hint = (c.most & MOST_NUMA_HINT) != 0;
    int64_t dummy[MAX_ZONES] = {0, 0, 0, 0};
    for (uint32_t k = 0; k < nm; k++) {
        const uint32_t m = (uint32_t)(nib >> (4 * k)) & 15u;
        int64_t T0 = 0, T1 = 0, A0 = 0, A1 = 0;
#pragma unroll
        for (uint32_t z = 0; z < (uint32_t)MAX_ZONES; z++) {
            const bool in = (m >> z) & 1u;
            T0 += in ? x.tot[0][z] : 0;
            T1 += in ? x.tot[1][z] : 0;
            A0 += in ? x.avail[0][z] : 0;
            A1 += in ? x.avail[1][z] : 0;
        }
        // numaScorer over requested = SubtractWithNonNegativeResult(total, available) + the pod's request
        const int64_t sc = numa_score_q(most_hint, c.numa_hint_w_cpu, c.numa_hint_w_mem, T0,
                                        (T0 - A0 < 0 ? 0 : T0 - A0) + score_cpu, T1, (T1 - A1 < 0 ? 0 : T1 - A1) + req[1]);
        if (k < 8) sc_lo |= (uint64_t)(sc & 0xFF) << (8 * k);
        else sc_hi |= (uint64_t)(sc & 0xFF) << (8 * (k - 8));
        // tryAllocateFromNode under the mask: every requested resource must be placed
        bool ok = true;
        if (bind) {  // the whole allocation with the CPUs (tryAllocateFromNode)
            int64_t al0[MAX_ZONES] = {0, 0, 0, 0}, al1[MAX_ZONES] = {0, 0, 0, 0};
            if (has[0]) ok = numa_split_r<true>(x, m, x.avail[0], req[0], al0, numa_bind_mode(bind), bind->cpc);
            if (ok && has[1]) ok = numa_split_r<true>(x, m, x.avail[1], req[1], al1);
            ok = ok && numa_bind_check(*bind, al0, al1, Z) == 0u;
        } else {
            if (has[0]) ok = numa_split_r<false>(x, m, x.avail[0], req[0], dummy);
            if (ok && has[1]) ok = numa_split_r<false>(x, m, x.avail[1], req[1], dummy);
        }
        if (!ok) continue;
        const int pc = popc(m);
        if (has[0] && !(m & lack0)) {
            okm0 |= 1u << k;
            min0 = min(min0, pc);
        }
        if (has[1] && !(m & lack1)) {
            okm1 |= 1u << k;
            min1 = min(min1, pc);
        }
    }
    mask_out = 0;
    const bool nil0 = has[0] && okm0 == 0, nil1 = has[1] && okm1 == 0;
    if ((nil0 || nil1) && policy != KG_NUMA_BEST_EFFORT) return KG_ST_NUMA_UNSATISFIED;
    // Preferred: the narrowest size, or every hint under Restricted
    uint32_t pref0 = 0, pref1 = 0;
    for (uint32_t k = 0; k < nm; k++) {
        const int pc = popc((uint32_t)(nib >> (4 * k)) & 15u);
        const bool r = policy == KG_NUMA_RESTRICTED;
        pref0 |= (pc == min0 || r) ? 1u << k : 0u;
        pref1 |= (pc == min1 || r) ? 1u << k : 0u;
    }
    uint32_t L0 = okm0, L1 = okm1;
    if (policy == KG_NUMA_SINGLE_NODE) {  // filterSingleNumaHints: preferred single-zone hints (the first Z masks)
        const uint32_t single = (1u << Z) - 1u;
        L0 &= pref0 & single;
        L1 &= pref1 & single;
    }
    if (nil0) L0 = 1u << NUMA_NIL_K;
    if (nil1) L1 = 1u << NUMA_NIL_K;
    const uint32_t all = (1u << Z) - 1u;
    NumaHint best{all, false, false, 0};
    const NumaHint none{0u, false, false, 0};
    const int nl = (has[0] ? 1 : 0) + (has[1] ? 1 : 0);
    if constexpr (GPU) {
        // iterateAllProviderTopologyHints over [cpu,] [memory,] gpu (policy.go:262-299)
        uint32_t G = gh->set;
        if (policy == KG_NUMA_SINGLE_NODE) {  // filterSingleNumaHints on the gpu list
            uint32_t keep = 0;
            for (uint32_t l = G; l; l &= l - 1u) {
                const uint32_t t = (uint32_t)(__ffs(l) - 1);
                const NumaHint h = gpu_hint_at(*gh, t);
                keep |= (h.pref && (h.mask == 0u || popc(h.mask) == 1)) ? 1u << t : 0u;
            }
            G = keep;
        }
        const uint32_t S0 = has[0] ? L0 : L1, P0 = has[0] ? pref0 : pref1;  // the first NUMA list present
        if (nl == 0) {
            for (uint32_t lc = G; lc; lc &= lc - 1u)
                numa_merge_perm(all, excl, x.status, 1, gpu_hint_at(*gh, (uint32_t)(__ffs(lc) - 1)), none, best);
        } else if (nl == 1) {
            for (uint32_t la = S0; la; la &= la - 1u) {
                const NumaHint ha = numa_hint_at(nib, (uint32_t)(__ffs(la) - 1), P0, sc_lo, sc_hi);
                for (uint32_t lc = G; lc; lc &= lc - 1u)
                    numa_merge_perm(all, excl, x.status, 2, ha, gpu_hint_at(*gh, (uint32_t)(__ffs(lc) - 1)), best);
            }
        } else {
            for (uint32_t la = L0; la; la &= la - 1u) {
                const NumaHint ha = numa_hint_at(nib, (uint32_t)(__ffs(la) - 1), pref0, sc_lo, sc_hi);
                for (uint32_t lb = L1; lb; lb &= lb - 1u) {
                    const NumaHint hb = numa_hint_at(nib, (uint32_t)(__ffs(lb) - 1), pref1, sc_lo, sc_hi);
                    for (uint32_t lc = G; lc; lc &= lc - 1u)
                        numa_merge_perm(all, excl, x.status, 3, ha, hb, best, gpu_hint_at(*gh, (uint32_t)(__ffs(lc) - 1)));
                }
            }
        }
    } else if (nl == 0) {
        numa_merge_perm(all, excl, x.status, 0, none, none, best);
    } else if (nl == 2 && policy != KG_NUMA_BEST_EFFORT) {
        // mergeFilteredHints over (cpu, memory) without a nil hint (nil lists fail above): a merged hint is preferred
        // only when both lists' masks are equal and preferred (and the exclusive check passes); once one exists no
        // non-preferred hint replaces it, and without one the policy fails (KG_ST_NUMA_ALIGN) whatever the mask. The
        // preferred candidates come out of the nested loops in ascending k (la = lb = k): visit only those.
        for (uint32_t l = L0 & L1 & pref0 & pref1; l; l &= l - 1u) {
            const NumaHint h = numa_hint_at(nib, (uint32_t)(__ffs(l) - 1), pref0, sc_lo, sc_hi);
            numa_merge_perm(all, excl, x.status, 2, h, h, best);
        }
    } else if (nl == 1) {
        const uint32_t L = has[0] ? L0 : L1, P = has[0] ? pref0 : pref1;
        for (uint32_t l = L; l; l &= l - 1u) {
            const NumaHint h = numa_hint_at(nib, (uint32_t)(__ffs(l) - 1), P, sc_lo, sc_hi);
            numa_merge_perm(all, excl, x.status, 1, h, none, best);
        }
    } else {
        for (uint32_t la = L0; la; la &= la - 1u) {
            const NumaHint ha = numa_hint_at(nib, (uint32_t)(__ffs(la) - 1), pref0, sc_lo, sc_hi);
            for (uint32_t lb = L1; lb; lb &= lb - 1u) {
                const NumaHint hb = numa_hint_at(nib, (uint32_t)(__ffs(lb) - 1), pref1, sc_lo, sc_hi);
                numa_merge_perm(all, excl, x.status, 2, ha, hb, best);
            }
        }
    }
    if (policy == KG_NUMA_BEST_EFFORT) {
        mask_out = best.unsat ? all : best.mask;
        return 0;
    }
    if (!best.pref) return KG_ST_NUMA_ALIGN;
    mask_out = (policy == KG_NUMA_SINGLE_NODE && best.mask == all) ? 0u : best.mask;
    return 0;
}

__device__ __forceinline__ int32_t numa_code(uint32_t mask) {
    if (!mask) return -1;
    return popc(mask) == 1 ? (int32_t)(__ffs(mask) - 1) : (int32_t)(0x40u | mask);
}

// tryBestToDistributeEvenly of the pod's cpu / memory over `mask`: the allocation and a failure bit per
// resource (bit 0 cpu, bit 1 memory: "Insufficient NUMA <resource>", resource_manager.go:300-309)
__device__ __forceinline__ uint32_t numa_split(const NumaZ& x, uint32_t mask, const int64_t* req, const bool* has,
                                               int64_t (&al)[2][MAX_ZONES], const NumaBind* bind = nullptr) {
    uint32_t fail = 0;
#pragma unroll
    for (int r = 0; r < 2; r++) {
#pragma unroll
        for (int z = 0; z < MAX_ZONES; z++) al[r][z] = 0;
        const int bm = r == 0 ? numa_bind_mode(bind) : 0;
        if (has[r] && !numa_split_r<true>(x, mask, x.avail[r], req[r], al[r], bm, bind ? bind->cpc : 1)) fail |= 1u << r;
    }
    return fail;
}

// The topology manager for one (pod, node) pair: hints, policy merge, the allocation's zone code and
// the NUMA score (score_node when no allocation is made). Returns 0 or KG_ST_* bits.
// bind (nullable): a cpuset-binding pod (its CPUs in every allocation, score_cpu its amplified cpu, bind_cpu the node's
// cpuset CPUs amplified: the Score's requested cpu, scoring.go:190-197); node_take: without an affinity its CPUs come
// from the whole node (allocateCPUSet without NUMA nodes) and fit there.
__device__ __forceinline__ uint32_t numa_topology(const KCfg* cp, const ZoneRec* zr, uint32_t Z, int64_t req_cpu,
                                               int64_t req_mem, uint32_t pflags, uint32_t pol, bool excl,
                                               int64_t score_node, int32_t* zone_out, int64_t* score_out,
                                               const NumaBind* bind = nullptr, int64_t score_cpu = -1,
                                               int64_t bind_cpu = 0, bool node_take = true) {
    const KCfg& c = *cp;
    NumaZ x;
    numa_load(zr, Z, x);
    if (bind) numa_bind_trim(x, *bind);
    const int64_t req[2] = {req_cpu, req_mem};
    const bool has[2] = {(pflags & KG_POD_HAS_CPU) != 0, (pflags & KG_POD_HAS_MEM) != 0};
    uint32_t mask = 0;
    const uint32_t st = numa_admit<true>(c, x, req, has, pol, excl, mask, nullptr, bind, score_cpu);
    if (st) return st;
    int64_t al[2][MAX_ZONES];
    // allocateResources under the best hint: a preferred best hint is one of the lists' feasible masks (not reached)
    if (mask && numa_split(x, mask, req, has, al, bind)) return KG_ST_UNSUPPORTED;
    if (mask && bind && numa_bind_check(*bind, al[0], al[1], Z)) return KG_ST_UNSUPPORTED;
    if (!mask && bind && !node_take) return KG_ST_NUMA_CPUS;
    *zone_out = numa_code(mask);
    // no NUMANodeResources (no affinity, or no cpu / memory request): node allocatable / requested (scoring.go:168-189)
    if (pol == KG_NUMA_BEST_EFFORT || !mask || !(req_cpu | req_mem)) {
        *score_out = score_node;
        return 0;
    }
    int64_t T[2] = {0, 0}, U[2] = {0, 0};
#pragma unroll
    for (uint32_t z = 0; z < (uint32_t)MAX_ZONES; z++) {
        if (z >= Z || (al[0][z] == 0 && al[1][z] == 0)) continue;
        for (int r = 0; r < 2; r++) {
            T[r] += x.tot[r][z];
            U[r] += x.used[r][z];
        }
    }
    *score_out = numa_score_q((c.most & MOST_NUMA) != 0, c.numa_w_cpu, c.numa_w_mem, T[0],
                              (bind ? bind_cpu : U[0]) + (score_cpu < 0 ? req_cpu : score_cpu), T[1], U[1] + req_mem);
    return 0;
}

// Node quantities a Reservation restore changes for pods of one owner class (kg_rsv_view): the
// NodeResourcesFit and NodeNUMAResource terms read these instead of the record's int section.
struct Over {
    int64_t req[5];  // cpu, memory, ephemeral-storage, scalar0, scalar1
    int64_t nz_cpu, nz_mem, num_pods;
};

// record slot s, or its restored value when a view applies
template <bool OV>
__device__ __forceinline__ int64_t nv(const int64_t* __restrict__ n, const Over* ov, int s) {
    if constexpr (OV) {
        switch (s) {
            case N_REQ_CPU: return ov->req[0];
            case N_REQ_MEM: return ov->req[1];
            case N_REQ_EPH: return ov->req[2];
            case N_SC_REQ0: return ov->req[3];
            case N_SC_REQ1: return ov->req[4];
            case N_NZ_CPU: return ov->nz_cpu;
            case N_NZ_MEM: return ov->nz_mem;
            case N_NUM_PODS: return ov->num_pods;
            default: return n[s];
        }
    } else {
        return n[s];
    }
}

struct PairOut {
    uint32_t status;
    int64_t s_nrf, s_la, s_numa;
    int32_t zone;
};

// NodeNUMAResource Filter + Score for a SingleNUMANode / None node. TOPO = false drops the general
// topology manager (numa_topology) from the instantiation: the host picks it only when no node is
// Restricted / BestEffort and no pod carries a NUMA policy, and only for select-mode kernels, where a
// SingleNUMANode pair without a fitting zone just needs some failure bit (the reason is unused).
// SCORE = false: the filter outcome only (status bits; scores and zone choice by score not computed),
// for the config-5 statistics pass.
// The Reserve of a BestEffort node (plugin.go:612-623): FilterByNUMANode under BestEffort (the merge always
// admits) and the allocation of its best hint; the zone code of the allocation, or ZONE_RESERVE_FAIL | bits
// when the topology hints fail ("node(s) Insufficient NUMA Node resources", no zones) or the allocation does
// ("Insufficient NUMA <resource>", resource_manager.go:300-309).
// A cpuset-binding pod (bind): its CPUs join every allocation; allocateCPUSet failing fails the Reserve (ZONE_CPUSET_FAIL).
__device__ __forceinline__ int32_t numa_reserve_best_effort(const KCfg& c, const ZoneRec* zr, uint32_t Z, const PodV& p,
                                                            bool excl, const NumaBind* bind = nullptr,
                                                            int64_t score_cpu = -1, bool node_take = true) {
    if (Z == 0) return ZONE_RESERVE_FAIL | (int32_t)(KG_ST_NUMA_INSUF_NODE >> 12);
    NumaZ x;
    numa_load(zr, Z, x);
    if (bind) numa_bind_trim(x, *bind);
    const int64_t req[2] = {p.req_cpu, p.req_mem};
    const bool has[2] = {(p.flags & KG_POD_HAS_CPU) != 0, (p.flags & KG_POD_HAS_MEM) != 0};
    uint32_t mask = 0;
    numa_admit<true>(c, x, req, has, KG_NUMA_BEST_EFFORT, excl, mask, nullptr, bind, score_cpu);
    int64_t al[2][MAX_ZONES];
    const uint32_t fail = mask ? numa_split(x, mask, req, has, al, bind) : 0u;
    if (fail) return ZONE_RESERVE_FAIL | (int32_t)fail;
    if (bind && (mask ? numa_bind_check(*bind, al[0], al[1], Z) != 0u : !node_take)) return ZONE_CPUSET_FAIL;
    return numa_code(mask);
}

// ZONE = false (select kernels): the pair's Reserve zone is not needed, so a BestEffort node skips its
// topology manager entirely (the Filter / Score do not depend on it).
template <bool EXACT, bool OV = false, bool TOPO = true, bool SCORE = true, bool ZONE = true>
__device__ __forceinline__ void numa_eval(const KCfg& c, const int64_t* __restrict__ n, const ZoneRec* __restrict__ zr,
                                          const PodV& p, uint32_t flags, PairOut& o, const Over* ov = nullptr) {
    if (p.flags & KG_POD_NUMA_SKIP) return;
    const uint32_t node_pol = (flags >> F_NUMA_POLICY_SHIFT) & 15u;
    const uint32_t pod_pol = (p.flags >> 16) & 15u;
    if (node_pol != KG_NUMA_NONE && pod_pol != KG_NUMA_NONE && pod_pol != node_pol) {
        o.status |= KG_ST_NUMA_CONFLICT;
        return;
    }
    const uint32_t pol = pod_pol != KG_NUMA_NONE ? pod_pol : node_pol;
    const bool amp = (flags & F_AMP) != 0;
    const int64_t pod_cpu = p.req_cpu;
    // requestCPUBind (util.go:121-138): the pod's own cpuset request, or a node CPU bind policy and a cpu request
    const uint32_t node_bind = (zr->cpu_meta >> CPU_META_BIND_SHIFT) & 3u;
    bool cpu_bind = (p.flags & KG_POD_CPU_BIND) != 0;
    if (!cpu_bind && pod_cpu != 0 && node_bind != KG_NODE_CPU_BIND_NONE) {
        if (pod_cpu % 1000 != 0) {  // ErrInvalidRequestedCPUs
            o.status |= KG_ST_NUMA_CPU_BIND;
            return;
        }
        cpu_bind = true;
    }
    // filterAmplifiedCPUs (plugin.go:461-498): a cpuset-binding pod's request is amplified too
    if (pod_cpu != 0 && amp) {
        int64_t requested = nv<OV>(n, ov, N_REQ_CPU);
        const int64_t cs = n[N_CPUSET];
        if (requested >= cs && cs > 0) requested = requested - cs + n[N_AMP_CPUSET];
        const int64_t need = cpu_bind ? (int64_t)ceil(__dmul_rn((double)pod_cpu, zr->amp_ratio)) : pod_cpu;
        if (need > n[N_ALLOC_CPU] - requested) {
            o.status |= KG_ST_NUMA_AMP_CPU;
            return;
        }
    }
    NumaBind bind;
    const NumaBind* bp = nullptr;
    bool node_take = true;
    if (cpu_bind) {  // plugin.go:396-440
        if (zr->cpu_topo < 0) {
            o.status |= KG_ST_NUMA_CPU_TOPO;
            return;
        }
        const uint32_t cpu_pol = (p.flags >> KG_POD_CPU_POLICY_SHIFT) & 3u;
        const bool pod_required = (p.flags & KG_POD_CPU_REQUIRED) != 0;
        uint32_t required = pod_required ? cpu_pol : KG_CPU_BIND_NONE;
        if (node_bind == KG_NODE_CPU_BIND_FULL_PCPUS_ONLY) required = KG_CPU_BIND_FULL_PCPUS;
        else if (node_bind == KG_NODE_CPU_BIND_SPREAD_BY_PCPUS) required = KG_CPU_BIND_SPREAD_BY_PCPUS;
        const int64_t needed = pod_cpu / 1000;
        const int64_t cpc = (zr->cpu_meta >> CPU_META_CPC_SHIFT) & 15u;
        if ((pod_required && cpu_pol != required) || (required == KG_CPU_BIND_FULL_PCPUS && (cpc == 0 || needed % cpc != 0))) {
            o.status |= KG_ST_NUMA_CPU_BIND;  // ErrCPUBindPolicyConflict / ErrSMTAlignmentError
            return;
        }
        if (flags & F_RSV_NUMA) {  // below: the restore of NUMA / cpuset-holding reservations (rsv_numa_unsupported)
            o.status |= KG_ST_UNSUPPORTED;
            return;
        }
        // allocateCPUSet over the whole node: the required policy's CPUs (filterCPUsByRequiredCPUBindPolicy) or the
        // available ones must cover the pod; takeCPUs then always succeeds on them and satisfies the policy
        const int64_t have = required == KG_CPU_BIND_FULL_PCPUS    ? zr->cpu_free_full
                             : required == KG_CPU_BIND_SPREAD_BY_PCPUS ? zr->cpu_free_cores
                                                                       : zr->cpu_free;
        node_take = needed <= have;
        if (pol != KG_NUMA_NONE) {  // the CPUs join every allocation the topology manager tries
            bind = numa_bind_of(zr, required != KG_CPU_BIND_NONE, required != KG_CPU_BIND_NONE ? required : cpu_pol, pod_cpu);
            bp = &bind;
        } else if (required != KG_CPU_BIND_NONE) {
            if (!node_take) {  // tryAllocateFromNode in Filter
                o.status |= KG_ST_NUMA_CPUS;
                return;
            }
        } else if (!node_take) {
            // no Filter check: the Reserve fails (ErrNotEnoughCPUs)
            if constexpr (ZONE) o.zone = ZONE_CPUSET_FAIL;
        }
    }
    // reservations on the node hold NUMA / cpuset allocations: RestoreReservation (nodenumaresource/reservation.go
    // :188-262) gives them back to the pod (matched) or returns the owners' double-counted usage (unmatched) on every
    // path that reads them from here on (hints, tryAllocateFromReusable / FromNode, the Reserve); the device does not
    // follow it (kg_node_columns.rsv_numa)
    if ((flags & F_RSV_NUMA) && pol != KG_NUMA_NONE) {
        o.status |= KG_ST_UNSUPPORTED;
        return;
    }
    // a cpuset-binding pod under a NUMA policy: its cpu request amplified where the options' requests count (hint and
    // node scores, getResourceOptions plugin.go:774-778), the node's cpuset CPUs amplified as the Score's requested
    // cpu (calculateAllocatableAndRequested, scoring.go:190-197)
    const int64_t score_cpu = (bp && amp) ? (int64_t)ceil(__dmul_rn((double)pod_cpu, zr->amp_ratio)) : pod_cpu;
    const int64_t bind_cpu = amp ? n[N_AMP_CPUSET] : n[N_CPUSET];
    const double rcp_cpu = as_f64(n[N_RCP_CPU]), rcp_mem = as_f64(n[N_RCP_MEM]);
    const bool most = (c.most & MOST_NUMA) != 0;
    // pods with their own NUMA policy default to the Required exclusive policy (plugin.go:449-454)
    const bool excl = pod_pol != KG_NUMA_NONE;
    if (pol == KG_NUMA_BEST_EFFORT) {
        // no FilterByNUMANode under BestEffort (plugin.go:446-455); Score without an allocation: node
        // allocatable / requested as they are (scoring.go:184-189; a cpuset-binding pod's CPUs from the whole node,
        // score 0 when they do not fit); the Reserve's zone from the topology manager
        if constexpr (SCORE) {
            if (bp)
                o.s_numa = node_take ? numa_score<EXACT>(most, c.numa_w_cpu, c.numa_w_mem, n[N_ALLOC_CPU], bind_cpu + score_cpu,
                                                         rcp_cpu, n[N_ALLOC_MEM], nv<OV>(n, ov, N_REQ_MEM) + p.req_mem, rcp_mem)
                                     : 0;
            else
                o.s_numa = numa_score<EXACT>(most, c.numa_w_cpu, c.numa_w_mem, n[N_ALLOC_CPU], nv<OV>(n, ov, N_REQ_CPU) + pod_cpu,
                                             rcp_cpu, n[N_ALLOC_MEM], nv<OV>(n, ov, N_REQ_MEM) + p.req_mem, rcp_mem);
        }
        if constexpr (ZONE && TOPO)
            o.zone = numa_reserve_best_effort(c, zr, (flags >> F_NUMA_ZONES_SHIFT) & 15u, p, excl, bp, score_cpu, node_take);
        return;
    }
    if (pol == KG_NUMA_RESTRICTED || (pol == KG_NUMA_SINGLE_NODE && (excl || bp))) {
        if constexpr (!TOPO) {
            o.status |= KG_ST_UNSUPPORTED;  // unreachable under the host's TOPO selection
            return;
        }
        const uint32_t Z = (flags >> F_NUMA_ZONES_SHIFT) & 15u;
        if (Z == 0) {
            o.status |= KG_ST_NUMA_NO_RES;
            return;
        }
        const int64_t score_node = numa_score<EXACT>(most, c.numa_w_cpu, c.numa_w_mem, n[N_ALLOC_CPU],
                                                     (bp ? bind_cpu : nv<OV>(n, ov, N_REQ_CPU)) + score_cpu, rcp_cpu,
                                                     n[N_ALLOC_MEM], nv<OV>(n, ov, N_REQ_MEM) + p.req_mem, rcp_mem);
        int32_t zone = -1;
        int64_t s = 0;
        const uint32_t st = numa_topology(&c, zr, Z, p.req_cpu, p.req_mem, p.flags, pol, excl, score_node, &zone, &s, bp,
                                          score_cpu, bind_cpu, node_take);
        if (st) {
            o.status |= st;
            return;
        }
        o.zone = zone;
        o.s_numa = s;
        return;
    }
    if (pol == KG_NUMA_SINGLE_NODE) {
        const uint32_t Z = (flags >> F_NUMA_ZONES_SHIFT) & 15u;
        if (Z == 0) {
            o.status |= KG_ST_NUMA_NO_RES;
            return;
        }
        const bool has_cpu = (p.flags & KG_POD_HAS_CPU) != 0, has_mem = (p.flags & KG_POD_HAS_MEM) != 0;
        int32_t best = -1;
        if (has_cpu || has_mem) {
            int64_t best_score = 0;
            for (uint32_t z = 0; z < Z; z++) {
                const int64_t tc = zr->cpu[z], tm = zr->mem[z];
                const int64_t uc = zone_cpu_alloc(*zr, z), um = zr->mem_used[z];
                const int64_t ac = tc - uc < 0 ? 0 : tc - uc;
                const int64_t am = tm - um < 0 ? 0 : tm - um;
                const bool ok = (!has_cpu || (ac != 0 && p.req_cpu <= ac)) && (!has_mem || (am != 0 && p.req_mem <= am));
                const int64_t rc = tc - ac < 0 ? 0 : tc - ac;
                const int64_t rm = tm - am < 0 ? 0 : tm - am;
                int64_t s = 0;
                if constexpr (SCORE)
                    s = numa_score<EXACT>((c.most & MOST_NUMA_HINT) != 0, c.numa_hint_w_cpu, c.numa_hint_w_mem, tc,
                                          rc + p.req_cpu, zr->rcp_cpu[z], tm, rm + p.req_mem, zr->rcp_mem[z]);
                const bool take = ok && (best < 0 || s > best_score);
                best = take ? (int32_t)z : best;
                best_score = take ? s : best_score;
            }
            if (best < 0) {
                // no single zone fits: the reason is ErrUnsatisfiedNUMAResource when some requested
                // resource has no hint at all, else the alignment failure (general merge decides)
                if constexpr (!TOPO) {
                    o.status |= KG_ST_NUMA_ALIGN;
                    return;
                }
                int32_t zone = -1;
                int64_t s = 0;
                o.status |= numa_topology(&c, zr, Z, p.req_cpu, p.req_mem, p.flags, KG_NUMA_SINGLE_NODE, false, 0, &zone, &s);
                return;
            }
        }
        if constexpr (!SCORE) return;
        if (best < 0 || Z == 1) {  // best hint == default affinity: no NUMA allocation
            o.zone = -1;
            o.s_numa = numa_score<EXACT>(most, c.numa_w_cpu, c.numa_w_mem, n[N_ALLOC_CPU], nv<OV>(n, ov, N_REQ_CPU) + pod_cpu,
                                         rcp_cpu, n[N_ALLOC_MEM], nv<OV>(n, ov, N_REQ_MEM) + p.req_mem, rcp_mem);
            return;
        }
        o.zone = best;
        o.s_numa = numa_score<EXACT>(most, c.numa_w_cpu, c.numa_w_mem, zr->cpu[best], zone_cpu_alloc(*zr, best) + pod_cpu,
                                     zr->rcp_cpu[best], zr->mem[best], zr->mem_used[best] + p.req_mem,
                                     zr->rcp_mem[best]);
        return;
    }
    // policy None: scoreWithAmplifiedCPUs; a cpuset-binding pod's own request is amplified (getResourceOptions,
    // plugin.go:772-778)
    if constexpr (!SCORE) return;
    int64_t req_cpu = nv<OV>(n, ov, N_REQ_CPU);
    if (pod_cpu != 0 && amp) req_cpu = req_cpu - n[N_CPUSET] + n[N_AMP_CPUSET];
    const int64_t own_cpu = (cpu_bind && amp) ? (int64_t)ceil(__dmul_rn((double)pod_cpu, zr->amp_ratio)) : pod_cpu;
    o.s_numa = numa_score<EXACT>(most, c.numa_w_cpu, c.numa_w_mem, n[N_ALLOC_CPU], req_cpu + own_cpu, rcp_cpu,
                                 n[N_ALLOC_MEM], nv<OV>(n, ov, N_REQ_MEM) + p.req_mem, rcp_mem);
}

template <bool EXACT, bool OV = false, bool TOPO = true, bool SCORE = true, bool ZONE = true>
__device__ __forceinline__ PairOut eval_pair(const KCfg& c, const int64_t* __restrict__ n,
                                             const ZoneRec* __restrict__ zr, const PodV& p, const Over* ov = nullptr) {
    PairOut o;
    o.status = 0;
    o.s_nrf = o.s_la = o.s_numa = 0;
    o.zone = -1;
    const uint32_t flags = (uint32_t)n[N_FLAGS];

    if (c.plugins & KG_PLUGIN_NRF) {
        // Fits
        uint32_t st = 0;
        st |= (nv<OV>(n, ov, N_NUM_PODS) + 1 > n[N_ALLOC_PODS]) ? KG_ST_NRF_PODS : 0u;
        st |= (p.req_cpu > 0 && p.req_cpu > n[N_ALLOC_CPU] - nv<OV>(n, ov, N_REQ_CPU)) ? KG_ST_NRF_CPU : 0u;
        st |= (p.req_mem > 0 && p.req_mem > n[N_ALLOC_MEM] - nv<OV>(n, ov, N_REQ_MEM)) ? KG_ST_NRF_MEM : 0u;
        st |= (p.req_eph > 0 && p.req_eph > n[N_ALLOC_EPH] - nv<OV>(n, ov, N_REQ_EPH)) ? KG_ST_NRF_EPH : 0u;
        st |= (p.sc0 != 0 && !(c.nrf_ign & 1u) && p.sc0 > n[N_SC_ALLOC0] - nv<OV>(n, ov, N_SC_REQ0)) ? KG_ST_NRF_SC0 : 0u;
        st |= (p.sc1 != 0 && !(c.nrf_ign & 2u) && p.sc1 > n[N_SC_ALLOC1] - nv<OV>(n, ov, N_SC_REQ1)) ? KG_ST_NRF_SC1 : 0u;
        o.status |= st;
        if constexpr (SCORE) {
        // LeastAllocated (or, per resource, MostAllocated) over {cpu, memory, scalar0, scalar1}
        int64_t sum = 0, wsum = 0;
        auto term = [&](int r, int64_t req, int64_t cap, double rcp) -> int64_t {
            return ((c.nrf_most >> r) & 1u) ? most_req(req, cap) : least_req<EXACT>(req, cap, rcp);
        };
        {
            const int64_t cap = n[N_ALLOC_CPU], w = c.nrf_w[0];
            const bool on = (w != 0) & (cap != 0);
            sum += on ? term(0, nv<OV>(n, ov, N_NZ_CPU) + p.nz_cpu, cap, as_f64(n[N_RCP_CPU])) * w : 0;
            wsum += on ? w : 0;
        }
        {
            const int64_t cap = n[N_ALLOC_MEM], w = c.nrf_w[1];
            const bool on = (w != 0) & (cap != 0);
            sum += on ? term(1, nv<OV>(n, ov, N_NZ_MEM) + p.nz_mem, cap, as_f64(n[N_RCP_MEM])) * w : 0;
            wsum += on ? w : 0;
        }
        {
            const int64_t cap = n[N_SC_ALLOC0], w = c.nrf_w[2];
            const bool on = (w != 0) & (cap != 0) & (p.sc0 != 0);
            sum += on ? term(2, nv<OV>(n, ov, N_SC_REQ0) + p.sc0, cap, as_f64(n[N_RCP_SC0])) * w : 0;
            wsum += on ? w : 0;
        }
        {
            const int64_t cap = n[N_SC_ALLOC1], w = c.nrf_w[3];
            const bool on = (w != 0) & (cap != 0) & (p.sc1 != 0);
            sum += on ? term(3, nv<OV>(n, ov, N_SC_REQ1) + p.sc1, cap, as_f64(n[N_RCP_SC1])) * w : 0;
            wsum += on ? w : 0;
        }
        o.s_nrf = wdiv(sum, wsum);
        }
    }

    if (c.plugins & KG_PLUGIN_LA) {
        // Filter
        if (!(p.flags & KG_POD_DAEMONSET)) {
            const bool prod = (flags & F_LA_PROD_THR) && (p.flags & KG_POD_PROD);
            const uint32_t mode = (flags >> (prod ? F_LA_FMODE_PROD_SHIFT : F_LA_FMODE_NP_SHIFT)) & 3u;
            if (mode == FMODE_FAIL_EXPIRED) {
                o.status |= KG_ST_LA_EXPIRED;
            } else if (mode == FMODE_CHECK) {
                const int64_t e0 = (prod ? n[N_LA_FBASE_PROD0] : n[N_LA_FBASE_NP0]) + p.est0;
                const int64_t e1 = (prod ? n[N_LA_FBASE_PROD1] : n[N_LA_FBASE_NP1]) + p.est1;
                const int64_t c0 = prod ? n[N_LA_FCUT_PROD0] : n[N_LA_FCUT_NP0];
                const int64_t c1 = prod ? n[N_LA_FCUT_PROD1] : n[N_LA_FCUT_NP1];
                const uint32_t agg = (!prod && (flags & F_LA_NP_AGG)) ? KG_ST_LA_AGG : 0u;
                o.status |= (e0 > c0) ? (KG_ST_LA_CPU | agg) : ((e1 > c1) ? (KG_ST_LA_MEM | agg) : 0u);
            }
        }
        // Score
        if (SCORE && c.la_score_enabled && !(flags & F_LA_SCORE_ZERO)) {
            const bool prod = c.la_score_prod && (p.flags & KG_POD_PROD);
            const int64_t u0 = (prod ? n[N_LA_SBASE_PROD0] : n[N_LA_SBASE_NP0]) + p.est0;
            const int64_t u1 = (prod ? n[N_LA_SBASE_PROD1] : n[N_LA_SBASE_NP1]) + p.est1;
            const int64_t s0 = least_req<EXACT>(u0, n[N_LA_ALLOC0], as_f64(n[N_RCP_LA0]));
            const int64_t s1 = least_req<EXACT>(u1, n[N_LA_ALLOC1], as_f64(n[N_RCP_LA1]));
            int64_t dom = c.la_dom_w != 0 ? 100 : 0;
            dom = dom > s0 ? s0 : dom;
            dom = dom > s1 ? s1 : dom;
            const int64_t sum = s0 * c.la_w[0] + s1 * c.la_w[1] + dom * c.la_dom_w;
            o.s_la = c.la_wsum <= 0 ? 0 : wdiv(sum, c.la_wsum);
        }
    }

    if (c.plugins & KG_PLUGIN_NUMA) numa_eval<EXACT, OV, TOPO, SCORE, ZONE>(c, n, zr, p, flags, o, ov);
    if (o.status & (KG_ST_NUMA_MASK | KG_ST_UNSUPPORTED)) o.s_numa = 0;
    if (o.status) o.zone = -1;
    return o;
}

__device__ __forceinline__ int64_t pair_total(const KCfg& c, const PairOut& o) {
    return c.w_nrf * o.s_nrf + c.w_la * o.s_la + c.w_numa * o.s_numa;
}

__device__ __forceinline__ uint64_t pair_key(const KCfg& c, const PairOut& o, uint32_t gidx) {
    const uint64_t key = ((uint64_t)pair_total(c, o) << 32) | (uint64_t)(0xFFFFFFFFu - gidx);
    return o.status ? 0ull : key;
}

// Reserve of a multi-zone NUMA allocation: the split recomputed on the zone state the pair was
// evaluated on. Out of line, so that its private arrays stay out of the callers' frames.
// split_out (nullable): the per-zone amounts taken, cpu [0, MAX_ZONES) then memory (the allocation the
// Unreserve releases, resource_manager.go:478-483).
__device__ __forceinline__ void numa_reserve_split(ZoneRec* zr, uint32_t Z, int64_t req_cpu, int64_t req_mem, uint32_t pflags,
                                                uint32_t mask, int64_t* split_out = nullptr) {
    NumaZ x;
    numa_load(zr, Z, x);
    const int64_t req[2] = {req_cpu, req_mem};
    const bool has[2] = {(pflags & KG_POD_HAS_CPU) != 0, (pflags & KG_POD_HAS_MEM) != 0};
    int64_t al[2][MAX_ZONES];
    if (!numa_split(x, mask, req, has, al))
        for (int z = 0; z < MAX_ZONES; z++) {
            zr->cpu_used[z] += al[0][z];
            zr->mem_used[z] += al[1][z];
            zr->status |= (al[0][z] | al[1][z]) ? 1u << (ZONE_RECORD_SHIFT + z) : 0u;
            if (split_out) {
                split_out[z] = al[0][z];
                split_out[MAX_ZONES + z] = al[1][z];
            }
        }
}

// A cpuset-binding pod under a NUMA policy on a node with a CPU topology: its Reserve's NUMA split (with the CPUs,
// numa_split under NumaBind) is recorded by the cpuset Reserve kernel before the take changes the counts
// (k_cpuset_reserve), not by apply_assume.
__device__ __forceinline__ bool cpuset_numa_reserve(const KCfg& c, const int64_t* __restrict__ n, const ZoneRec* zr,
                                                    const PodV& p) {
    if (!(c.plugins & KG_PLUGIN_NUMA) || zr->cpu_topo < 0 || (p.flags & KG_POD_NUMA_SKIP)) return false;
    const uint32_t node_bind = (zr->cpu_meta >> CPU_META_BIND_SHIFT) & 3u;
    if (!((p.flags & KG_POD_CPU_BIND) || (node_bind != KG_NODE_CPU_BIND_NONE && p.req_cpu != 0))) return false;
    const uint32_t node_pol = ((uint32_t)n[N_FLAGS] >> F_NUMA_POLICY_SHIFT) & 15u, pod_pol = (p.flags >> 16) & 15u;
    return (pod_pol != KG_NUMA_NONE ? pod_pol : node_pol) != KG_NUMA_NONE;
}

// Reserve (sign = +1) / Unreserve (sign = -1) of pod p on node record n (a16).
// split (nullable): a multi-zone allocation's per-zone amounts, written by the Reserve and taken back by the
// Unreserve (cpu [0, MAX_ZONES) then memory).
__device__ __forceinline__ void apply_assume(const KCfg& c, int64_t* n, ZoneRec* zr, const PodV& p, int32_t zone,
                                             int64_t sign, int64_t* split = nullptr) {
    n[N_REQ_CPU] += sign * p.req_cpu;
    n[N_REQ_MEM] += sign * p.req_mem;
    n[N_REQ_EPH] += sign * p.req_eph;
    n[N_SC_REQ0] += sign * p.sc0;
    n[N_SC_REQ1] += sign * p.sc1;
    n[N_NZ_CPU] += sign * p.nz_cpu;
    n[N_NZ_MEM] += sign * p.nz_mem;
    n[N_NUM_PODS] += sign;
    const uint32_t flags = (uint32_t)n[N_FLAGS];
    if ((c.plugins & KG_PLUGIN_LA) && (flags & F_LA_HAS_METRIC)) {
        const int64_t d0 = sign * (p.est0 > 0 ? p.est0 : 0), d1 = sign * (p.est1 > 0 ? p.est1 : 0);
        n[N_LA_FBASE_NP0] += d0;
        n[N_LA_FBASE_NP1] += d1;
        n[N_LA_SBASE_NP0] += d0;
        n[N_LA_SBASE_NP1] += d1;
        if (p.flags & KG_POD_PROD) {
            n[N_LA_FBASE_PROD0] += d0;
            n[N_LA_FBASE_PROD1] += d1;
            n[N_LA_SBASE_PROD0] += d0;
            n[N_LA_SBASE_PROD1] += d1;
        }
    }
    if (sign > 0 && zone >= 0 && cpuset_numa_reserve(c, n, zr, p)) {
        // the zone split is in place already (k_cpuset_reserve)
    } else if ((c.plugins & KG_PLUGIN_NUMA) && zone >= 0 && zone < MAX_ZONES) {
        zr->cpu_used[zone] += sign * p.req_cpu;
        zr->mem_used[zone] += sign * p.req_mem;
        if (sign > 0 && (p.req_cpu | p.req_mem)) zr->status |= 1u << (ZONE_RECORD_SHIFT + zone);
        if (split && sign > 0) {
            split[zone] = p.req_cpu;
            split[MAX_ZONES + zone] = p.req_mem;
        }
    } else if ((c.plugins & KG_PLUGIN_NUMA) && zone >= 0x40 && sign > 0) {
        numa_reserve_split(zr, (flags >> F_NUMA_ZONES_SHIFT) & 15u, p.req_cpu, p.req_mem, p.flags, (uint32_t)zone & 0xFu,
                           split);
    } else if ((c.plugins & KG_PLUGIN_NUMA) && zone >= 0x40 && zone < 0x80 && split) {
        for (int z = 0; z < MAX_ZONES; z++) {
            zr->cpu_used[z] += sign * split[z];
            zr->mem_used[z] += sign * split[MAX_ZONES + z];
        }
    }
    derive_node(*reinterpret_cast<NodeRec*>(n), *zr);
}

// ------------------------------------------------------------------------------------------------
// Fast path of the select kernel. Node values come from the record's fast block (wave-uniform, in
// SGPRs); pod values are scaled by 100 once per lane. Every quotient is exact by construction, so
// results equal eval_pair's bit for bit; nodes or pods outside the fast domain (F_BIG, host pod
// check) take eval_pair instead.
//
// leastRequestedScore(requested, capacity) = (capacity - requested) * 100 / capacity (0 if the
// request exceeds capacity or capacity is 0): with F = capacity - node requested (0 <= F <= capacity
// < 2^44, node-side, x100) and r the pod request (x100), t = F100 - r100 is exact and
//   y = RN(t * rcp_up),  rcp_up = 1/capacity rounded toward +inf,
// satisfies floor(t/c) <= y < floor(t/c) + 1 for t >= 0: y >= t/c because rcp_up >= 1/c and rounding
// is monotone; y - t/c <= (t/c) 2^-52 + ulp(y)/2 <= 100 * 2^-52 + 2^-46 < 1/c <= distance from t/c
// to the next integer. A saturating float->uint convert truncates y and maps t < 0 to 0. Capacity 0
// has rcp_up = 0, so y = 0.
//
// Weighted mean Σ s_i w_i / Σ w_i (s_i <= 100, host-checked w_i <= 4096, Σ w_i <= 16384): with
// doubled weights, trunc((2 Σ s_i w_i + 1) * (0.5 / Σ w_i)) in float32: the exact value sits at least
// 0.5/Σw (>= 3.05e-5) away from any integer and the float error is <= 101 * 1.5 * 2^-23 (1.8e-5).

struct PodF {
    double cpu, mem, eph, sc0, sc1, nzc, nzm, e0, e1;  // x100
    double la_sprod;   // 1.0 when the LoadAware score uses the prod profile (la_score_prod && prod pod)
    double has_cpu;    // 1.0 when the cpu request is non-zero (amplified-cpu score)
    uint32_t sc0_on, sc1_on;  // 1 when the scalar request is non-zero (LeastAllocated counts it)
    uint32_t flags;
};

__device__ __forceinline__ PodF to_podf(const PodV& p, const KCfg& c) {
    PodF q;
    q.la_sprod = (c.la_score_prod && (p.flags & KG_POD_PROD)) ? 1.0 : 0.0;
    q.has_cpu = p.req_cpu != 0 ? 1.0 : 0.0;
    q.sc0_on = p.sc0 != 0 ? 1u : 0u;
    q.sc1_on = p.sc1 != 0 ? 1u : 0u;
    q.cpu = x100(p.req_cpu);
    q.mem = x100(p.req_mem);
    q.eph = x100(p.req_eph);
    q.sc0 = x100(p.sc0);
    q.sc1 = x100(p.sc1);
    q.nzc = x100(p.nz_cpu);
    q.nzm = x100(p.nz_mem);
    q.e0 = x100(p.est0);
    q.e1 = x100(p.est1);
    q.flags = p.flags;
    return q;
}

// saturating float64 -> uint32 (v_cvt_u32_f64 clamps negatives to 0)
__device__ __forceinline__ uint32_t cvt_sat_u32(double y) {
    uint32_t r;
    asm("v_cvt_u32_f64 %0, %1" : "=v"(r) : "v"(y));
    return r;
}

__device__ __forceinline__ uint32_t lr100(double f100, double r100, double rcp_up) {
    return cvt_sat_u32((f100 - r100) * rcp_up);
}

// trunc(sum2 * hw) for sum2 = 2 Σ s_i w_i + 1, hw = 0.5 / Σ w_i
__device__ __forceinline__ uint32_t wq(uint32_t sum2, float hw) { return (uint32_t)((float)sum2 * hw); }

__device__ __forceinline__ uint32_t mad24(uint32_t a, uint32_t b, uint32_t c) { return __umul24(a, b) + c; }

__device__ __forceinline__ uint32_t lo32(uint64_t pack) { return (uint32_t)pack; }

__device__ __forceinline__ uint32_t hi32(uint64_t pack) { return (uint32_t)(pack >> 32); }

__device__ __forceinline__ float f32hi(uint64_t pack) { return __uint_as_float((uint32_t)(pack >> 32)); }

__device__ __forceinline__ float f32lo(uint64_t pack) { return __uint_as_float((uint32_t)pack); }

// Copy a wave-uniform kernel argument into a VGPR: keeps the select loop's SGPRs for the node
// record (the compiler would otherwise pin the configuration in SGPRs and spill the record).
__device__ __forceinline__ int32_t in_vgpr(int32_t x) {
    int32_t y;
    asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "s"(x));
    return y;
}

__device__ __forceinline__ KCfg cfg_in_vgprs(const KCfg& c) {
    KCfg v = c;
    v.w_nrf = in_vgpr(c.w_nrf);
    v.w_la = in_vgpr(c.la_score_enabled ? c.w_la : 0);
    v.w_numa = in_vgpr(c.w_numa);
    v.la_w[0] = in_vgpr(2 * c.la_w[0]);  // doubled for wq
    v.la_w[1] = in_vgpr(2 * c.la_w[1]);
    v.la_dom_w = in_vgpr(2 * c.la_dom_w);
    v.la_hw = __int_as_float(in_vgpr(__float_as_int(c.la_hw)));
    return v;
}

// Selection key of one (pod, node) pair on the fast path. `r` is the node's fast block (by value:
// wide scalar loads, one wait); plugin arithmetic is branch-free except for the SingleNUMANode
// zone walk. `c` comes from cfg_in_vgprs (LoadAware weights doubled).
// PM: enabled plugins (KG_PLUGIN_* mask); CLS: node storage class (node_class), both compile-time.
// Wave kinds of the fast select (a wave whose 64 pods all share one of these shapes runs a loop
// specialised for it; the host groups a batch's pods by kind, kg_pods_upload):
//   FK_PROD  - prod pods (KG_POD_PROD) requesting cpu or memory, no DaemonSet, no scalar (batch) requests,
//              NodeNUMAResource not skipped, no cpuset binding: the LoadAware prod profile, no scalar Fits /
//              LeastAllocated terms, no node-level NUMA score on multi-zone SingleNUMANode nodes;
//   FK_BATCH - non-prod pods with both scalar requests and no cpu / memory request (koord-batch pods),
//              no DaemonSet, no HAS_CPU / HAS_MEM, not skipped, no cpuset binding: the non-prod profile, both scalar terms,
//              the cpu / memory Fits reduce to the node's "Too many pods" bit, no NUMA zone walk.
// Every kind computes exactly what the general loop (FK_ANY) computes for those pods.
enum : int { FK_ANY = 0, FK_PROD = 1, FK_BATCH = 2 };

__device__ __forceinline__ bool fast_kind_match(int kind, const PodV& p) {
    const uint32_t f = p.flags;
    if (kind == FK_PROD)
        return (f & (KG_POD_PROD | KG_POD_DAEMONSET | KG_POD_NUMA_SKIP | KG_POD_CPU_BIND)) == KG_POD_PROD &&
               (f & (KG_POD_HAS_CPU | KG_POD_HAS_MEM)) != 0 && p.sc0 == 0 && p.sc1 == 0;
    return (f & (KG_POD_PROD | KG_POD_DAEMONSET | KG_POD_NUMA_SKIP | KG_POD_CPU_BIND | KG_POD_HAS_CPU | KG_POD_HAS_MEM)) == 0 &&
           p.req_cpu == 0 && p.req_mem == 0 && p.sc0 != 0 && p.sc1 != 0;
}

// fast_eval: the weighted total in `total`, feasibility as the return value (select loops fold it into
// their top-key update); eval_fast_key: the selection key, 0 when infeasible.
// GZ (CLS 1, a GPU pod): DeviceShare's hints join the zone walk (gz = gpu_zone_sum's word of the record and the pod's
// GPU request class): a zone needs its preferred single-zone GPU hint (unless the provider has no preference) and the
// merged hint's score is the sum over the providers' lists, (cpu, memory listed) x the zone's hint score + 500 when
// DeviceShare's hint scores 500 (policy.go mergePermutation); a failing provider fails the pair. Needs a cpu or memory
// request (with neither, the merge runs on DeviceShare's list alone: general path).
template <uint32_t PM, int CLS, int KIND = FK_ANY, bool GZ = false>
__device__ __forceinline__ bool fast_eval(const KCfg& c, const FastRec& r, const ZoneRec* __restrict__ zr, const PodF& p,
                                          uint32_t& total_out, int32_t* zone_out = nullptr, uint64_t gz = 0) {
    constexpr bool KP = KIND == FK_PROD, KB = KIND == FK_BATCH;
    const uint32_t f = (uint32_t)r.flags;
    bool ok = true;
    uint32_t total = 0;

    if constexpr ((PM & KG_PLUGIN_NRF) != 0) {
        // Fits: request r fails iff r > 0 and r > alloc - requested, i.e. 100 r > 100 max(0, headroom)
        // ("Too many pods" is folded into fit_cpu by derive_node: -1.0, the only negative fit value)
        bool fit_fail = p.eph > r.fit_eph;
        if constexpr (KB) fit_fail = fit_fail | ((f & F_PODS_FULL) != 0);  // 0 > fit_cpu: only the folded bit
        else fit_fail = fit_fail | (p.cpu > r.fit_cpu) | (p.mem > r.fit_mem);
        if constexpr (!KP) fit_fail = fit_fail | (p.sc0 > r.fit_sc0) | (p.sc1 > r.fit_sc1);
        ok = ok & !fit_fail;
        // LeastAllocated (NonZeroRequested for cpu / memory, Requested for scalars the pod requests)
        const uint32_t w0 = lo32(r.w_nrf01), w1 = hi32(r.w_nrf01);
        uint32_t sum2 = mad24(lr100(r.lr_nz_cpu, p.nzc, r.rcp_cpu), w0, 1u);
        sum2 = mad24(lr100(r.lr_nz_mem, p.nzm, r.rcp_mem), w1, sum2);
        // h = 1 / max(Σ 2w, 2) (Σ 2w = 0 -> sum2 = 1 and trunc(1 * 0.5) = 0): set by the host for the two
        // kinds (correctly rounded), else rcp + one Newton step (<= 1 ulp)
        float h;
        if constexpr (KP) {
            h = f32hi(r.w_aux);
        } else {
            const uint32_t w23 = lo32(r.w_nrf23), w2s = w23 & 0xFFFFu, w3s = w23 >> 16;
            const uint32_t w2 = KB ? w2s : (p.sc0_on ? w2s : 0u), w3 = KB ? w3s : (p.sc1_on ? w3s : 0u);
            sum2 = mad24(lr100(r.lr_sc0, p.sc0, r.rcp_sc0), w2, sum2);
            sum2 = mad24(lr100(r.lr_sc1, p.sc1, r.rcp_sc1), w3, sum2);
            if constexpr (KB) {
                h = f32hi(r.w_nrf23);
            } else {
                const float wsum = (float)max(w0 + w1 + w2 + w3, 2u);
                h = __builtin_amdgcn_rcpf(wsum);
                h = fmaf(h, fmaf(-wsum, h, 1.0f), h);
            }
        }
        total = mad24(c.w_nrf, wq(sum2, h), total);
    }

    if constexpr ((PM & KG_PLUGIN_LA) != 0) {
        // Filter: usage cut-offs of the pod's profile (100 * (cut - base) vs 100 * estimate); the
        // node's filter modes and profile choice are folded into the heads by derive_node
        bool la_fail;
        if constexpr (KP) {
            la_fail = (p.e0 > r.la_head_prod0) | (p.e1 > r.la_head_prod1);
        } else if constexpr (KB) {
            la_fail = (p.e0 > r.la_head_np0) | (p.e1 > r.la_head_np1);
        } else {
            const bool pod_prod = (p.flags & KG_POD_PROD) != 0;
            const bool over_np = (p.e0 > r.la_head_np0) | (p.e1 > r.la_head_np1);
            const bool over_pr = (p.e0 > r.la_head_prod0) | (p.e1 > r.la_head_prod1);
            la_fail = ((p.flags & KG_POD_DAEMONSET) == 0) & (pod_prod ? over_pr : over_np);
        }
        ok = ok & !la_fail;
        // Score: least-used over the estimated usage; profile select as an exact fma:
        // (free_np - e) + delta * {0, 1}. Nodes whose score is 0 carry rcp_la = 0.
        uint32_t s0, s1;
        if constexpr (KB) {  // non-prod pods: la_sprod = 0
            s0 = cvt_sat_u32((r.la_sfree_np0 - p.e0) * r.rcp_la0);
            s1 = cvt_sat_u32((r.la_sfree_np1 - p.e1) * r.rcp_la1);
        } else {
            s0 = cvt_sat_u32(fma(r.la_sdelta0, p.la_sprod, r.la_sfree_np0 - p.e0) * r.rcp_la0);
            s1 = cvt_sat_u32(fma(r.la_sdelta1, p.la_sprod, r.la_sfree_np1 - p.e1) * r.rcp_la1);
        }
        const uint32_t dom = min(min(s0, s1), 100u);
        uint32_t sum2 = mad24(s0, (uint32_t)c.la_w[0], 1u);
        sum2 = mad24(s1, (uint32_t)c.la_w[1], sum2);
        sum2 = mad24(dom, (uint32_t)c.la_dom_w, sum2);
        total = mad24(c.w_la, wq(sum2, c.la_hw), total);  // c.w_la is 0 when the score is disabled
    }

    if constexpr ((PM & KG_PLUGIN_NUMA) != 0) {
        const bool skip = (KP || KB) ? false : (p.flags & KG_POD_NUMA_SKIP) != 0;
        // filterAmplifiedCPUs (amp_fit is 2^62 without amplification, -1 on Restricted / BestEffort
        // nodes, which are F_BIG and leave the fast path; FK_BATCH pods request no cpu)
        const bool nok0 = KB ? true : ((p.flags & KG_POD_CPU_BIND) == 0) & !(p.cpu > r.amp_fit);
        uint32_t s_numa;
        bool nok = nok0;
        if constexpr (CLS == 1) {  // SingleNUMANode nodes (their own storage class): zone walk
            const uint32_t Z = (f >> F_NUMA_ZONES_SHIFT) & 15u;
            const bool has_cpu = KB ? false : (p.flags & KG_POD_HAS_CPU) != 0;
            const bool has_mem = KB ? false : (p.flags & KG_POD_HAS_MEM) != 0;
            const bool has_any = KP ? true : has_cpu | has_mem;
            int32_t best = -1;
            uint32_t best_score = 0;
            // with DeviceShare's hints (not "no preference") a zone is chosen even without a cpu / memory request
            const bool gsel = GZ && !KB && (gz & 2ull) == 0;
            if constexpr (!KB) {
                uint32_t best_hint = 0;
                uint32_t gmask = 0xFu, g500 = 0u, mult = 1u;
                if constexpr (GZ) {
                    const bool nopref = (gz & 2ull) != 0;
                    gmask = nopref ? 0xFu : (uint32_t)(gz >> 4) & 15u;
                    g500 = nopref ? 0u : (uint32_t)(gz >> 8) & 15u;
                    mult = (has_cpu ? 1u : 0u) + (has_mem ? 1u : 0u);
                }
#pragma unroll 1
                for (uint32_t z = 0; z < Z; z++) {
                    const ZoneFast q = zr->zf[z];
                    bool elig = (!has_cpu | (p.cpu <= q.avail_cpu)) & (!has_mem | (p.mem <= q.avail_mem));
                    const uint32_t hc = lr100(q.hint_cpu, p.cpu, q.rcp_cpu), hm = lr100(q.hint_mem, p.mem, q.rcp_mem);
                    const uint32_t fc = lr100(q.free_cpu, p.cpu, q.rcp_cpu), fm = lr100(q.free_mem, p.mem, q.rcp_mem);
                    uint32_t hint = wq(mad24(hm, hi32(q.w_hint), mad24(hc, lo32(q.w_hint), 1u)), f32lo(q.hpack));
                    if constexpr (GZ) {
                        elig = elig & (((gmask >> z) & 1u) != 0);
                        hint = mult * hint + (((g500 >> z) & 1u) ? 500u : 0u);
                    }
                    const uint32_t fin = wq(mad24(fm, hi32(q.w_score), mad24(fc, lo32(q.w_score), 1u)), f32hi(q.hpack));
                    const bool take = elig & ((best < 0) | (hint > best_hint));
                    best = take ? (int32_t)z : best;
                    best_hint = take ? hint : best_hint;
                    best_score = take ? fin : best_score;
                }
            }
            const bool need = has_any | gsel;
            nok = nok & (Z != 0) & !(need & (best < 0));
            if constexpr (GZ) nok = nok & ((gz & 1ull) == 0);
            // a best hint equal to the default affinity (no request on NUMA resources, or one zone)
            // carries no affinity: node-level score without amplification
            uint32_t node_level = 0;
            if (!KP || Z == 1) {  // FK_PROD: a wave-uniform branch on the record's zone count
                const uint32_t sc = lr100(r.numa_free_cpu, p.cpu, r.rcp_cpu), sm = lr100(r.numa_free_mem, p.mem, r.rcp_mem);
                node_level = wq(mad24(sm, hi32(r.w_numa), mad24(sc, lo32(r.w_numa), 1u)), f32lo(r.w_aux));
            }
            // (a zone chosen by DeviceShare's hints alone allocates no cpu / memory: no NUMANodeResources, node-level
            // score, calculateAllocatableAndRequested scoring.go:168-189)
            s_numa = (!has_any || Z == 1) ? node_level : best_score;
            if (zone_out) *zone_out = (skip || !need || Z == 1) ? -1 : best;  // the Reserve's zone (eval_pair o.zone)
        } else {
            // amplified requested for pods with a cpu request: (free - r) + delta * {0, 1}
            const uint32_t sc = KB ? cvt_sat_u32(r.numa_free_cpu * r.rcp_cpu)
                                   : cvt_sat_u32(fma(r.amp_delta, p.has_cpu, r.numa_free_cpu - p.cpu) * r.rcp_cpu);
            const uint32_t sm = lr100(r.numa_free_mem, p.mem, r.rcp_mem);
            s_numa = wq(mad24(sm, hi32(r.w_numa), mad24(sc, lo32(r.w_numa), 1u)), f32lo(r.w_aux));
        }
        ok = ok & (skip | nok);
        total = mad24(c.w_numa, skip ? 0u : s_numa, total);
    }
    total_out = total;
    return ok;
}

template <uint32_t PM, int CLS, bool GZ = false>
__device__ __forceinline__ uint64_t eval_fast_key(const KCfg& c, const FastRec& r, const ZoneRec* __restrict__ zr,
                                                  const PodF& p, uint32_t gidx, int32_t* zone_out = nullptr, uint64_t gz = 0) {
    uint32_t total;
    const bool ok = fast_eval<PM, CLS, FK_ANY, GZ>(c, r, zr, p, total, zone_out, gz);
    const uint64_t key = ((uint64_t)total << 32) | (uint64_t)(0xFFFFFFFFu - gidx);
    return ok ? key : 0ull;
}

}  // namespace kg
