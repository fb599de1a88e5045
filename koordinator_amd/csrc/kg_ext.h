// kg_ext.h — device arithmetic of the config-5 plugins (integer path, one (pod, node) pair per lane):
//   DeviceShare  Filter / Score / Reserve   deviceshare/plugin.go:345-421,507-569, scoring.go:45-112,197-281,
//                                           device_allocator.go:98-141,331-437, devicehandler_gpu.go:53-135
//   Reservation  Filter / nominate / Score  reservation/plugin.go:319-527,858-1057,1195-1212,
//                                           nominator.go:348-419, scoring.go:113-121,180-314
//   ElasticQuota PreFilter / Reserve        elasticquota/plugin.go:257-309,622-636,
//                                           core/group_quota_manager.go:765-805,1008-1046
// The CPU restatement these must equal bit for bit is oracle/kg_oracle.c (ext section).
#pragma once
#include "kg_eval.h"

namespace kg {

struct PodX {
    int64_t dreq[DEV_R];  // per-instance GPU request (keys in dkeys)
    uint32_t dcount, dkeys;
    int32_t quota;
    uint32_t qkeys;
    int32_t cls;
    uint32_t dflags;  // KG_GPU_POD_*
    uint32_t dtmpl;   // candidate template counts per node key (KG_GPU_POD_TEMPLATE)
    int64_t dbw;      // ring bus bandwidth request (KG_GPU_POD_RING_BW)
};

__device__ __forceinline__ PodX load_podx(const PodsDev& P, uint32_t j) {
    PodX x;
    x.dcount = P.dev_count ? P.dev_count[j] : 0u;
    x.dkeys = P.dev_keys ? P.dev_keys[j] : 0u;
    x.dflags = (P.dev_flags && x.dcount) ? P.dev_flags[j] : 0u;
    x.dbw = (P.dev_bw && (x.dflags & KG_GPU_POD_RING_BW)) ? P.dev_bw[j] : 0;
    x.dtmpl = (P.dev_tmpl && (x.dflags & KG_GPU_POD_TEMPLATE)) ? P.dev_tmpl[j] : 0u;
    for (int r = 0; r < DEV_R; r++) x.dreq[r] = (P.dev_req && ((x.dkeys >> r) & 1u)) ? P.dev_req[(size_t)j * DEV_R + r] : 0;
    x.quota = P.quota ? P.quota[j] : -1;
    x.qkeys = P.quota_keys ? P.quota_keys[j] : 0u;
    x.cls = P.rsv_class ? P.rsv_class[j] : -1;
    return x;
}

// ---- DeviceShare ------------------------------------------------------------------------------------

__device__ __forceinline__ int64_t least_score_i64(int64_t requested, int64_t capacity) {
    if (capacity == 0 || requested > capacity) return 0;
    return qdiv((capacity - requested) * 100, capacity);
}

// leastResourceScorer / mostResourceScorer (deviceshare/scoring.go:263-323) over {gpu-core,
// gpu-memory-ratio, gpu-memory}: zero totals skipped, requested = total >= free ? total - free +
// request : total (scoreNode / scoreDevice).
__device__ __forceinline__ int64_t dev_least(const KCfg& c, const int64_t* total, const int64_t* fr, const int64_t* preq) {
    int64_t score = 0, wsum = 0;
#pragma unroll
    for (int r = 0; r < DEV_R; r++) {
        const int64_t w = c.dev_w[r];
        if (w == 0 || total[r] == 0) continue;
        const int64_t req = total[r] >= fr[r] ? total[r] - fr[r] + preq[r] : total[r];
        score += ((c.most & MOST_DEV) ? most_req(req, total[r]) : least_score_i64(req, total[r])) * w;
        wsum += w;
    }
    return wsum == 0 ? 0 : qdiv(score, wsum);
}

__device__ __forceinline__ bool dev_minor_fits(const int64_t* fr, const PodX& x) {
    if (fr[0] == 0 && fr[1] == 0 && fr[2] == 0) return false;  // unhealthy / exhausted minor
    bool ok = true;
#pragma unroll
    for (int r = 0; r < DEV_R; r++) ok &= !(((x.dkeys >> r) & 1u) && x.dreq[r] > fr[r]);
    return ok;
}

// ---- GPU allocator (GPUAllocator.Allocate, deviceshare/allocator_gpu.go:72-133) ------------------------
// Order of the reference: a partition table (allocateByPartition :177-237), then the topology tree
// (allocateByDeviceTopology :312-451), then defaultAllocateDevices (device_allocator.go:355-437), behind
// allocateByTemplate (:135-159) for a pod that enforces a shared-resource template (gpu_template).

struct GpuAlloc {
    uint32_t code;  // KG_DEV_CODE_* (0 = allocated)
    uint32_t mask;  // minors taken (when asked for)
};

// Minor sets of one table as the allocator's AllocateContext sees them (bit m = minor m < D):
//   used  deviceUsedMinorsHash = hashDevices(getRealUsed(...)) (:59-70,83-86): minors with something used
//         (free != total) in the table, plus `outside`: minors used on the node that the table leaves out
//         (a reservation restore's filtered nodeDevice);
//   total hashDevices(removeZeroDevice(deviceTotal)) (:87,112-120,200);
//   sat   DeviceLevelContext.satisfied (:404-414): LessThanOrEqual(requestsPerGPU, free) and in total.
//   fit   defaultAllocateDevices' per-minor test (dev_minor_fits): free not all zero and covering the request.
struct GpuMinors {
    uint32_t used, total, sat, fit;
};

// allowed: the minors a NUMA affinity keeps (nodeDevice.filter, device_cache.go:367-415): the others leave the
// total, the satisfied and the fitting sets, and count as used outside the table (getRealUsed).
__device__ __forceinline__ GpuMinors gpu_minors(const DevRec* __restrict__ d, int32_t D, const PodX& x, uint32_t outside,
                                                uint32_t allowed = ~0u) {
    GpuMinors g{outside, 0u, 0u, 0u};
    for (int32_t m = 0; m < D; m++) {
        bool any_t = false, diff = false, le = true, any_f = false;
#pragma unroll
        for (int r = 0; r < DEV_R; r++) {
            const int64_t t = d->total[r][m], f = d->free_[r][m];
            any_t |= t != 0;
            any_f |= f != 0;
            diff |= f != t;
            le &= !(((x.dkeys >> r) & 1u) && x.dreq[r] > f);
        }
        g.used |= diff ? 1u << m : 0u;
        g.total |= any_t ? 1u << m : 0u;
        g.sat |= (any_t && le) ? 1u << m : 0u;
        g.fit |= (any_f && le) ? 1u << m : 0u;
    }
    g.used = (g.used & allowed) | outside;
    g.total &= allowed;
    g.sat &= allowed;
    g.fit &= allowed;
    return g;
}

// Σ AllocationScore of the partitions of the lowest-score group of (table tbl, n2 GPUs) that do not overlap
// `allocated` (selectPartitionByBinPack's inner loop, allocator_gpu.go:275-284), tabulated by the runtime at
// upload for every allocated mask: binpack[((tbl - 1) * 3 + k) * 256 + allocated], k = 0, 1, 2 for 8, 4, 2 GPUs.
__device__ __forceinline__ int64_t free_partitions(const ExtDev& e, uint32_t tbl, uint32_t k, uint32_t allocated) {
    return e.binpack[((tbl - 1u) * 3u + k) * 256u + (allocated & 0xFFu)];
}

__device__ __forceinline__ bool partition_ok(const kg_gpu_partition& q, const GpuMinors& g, const PodX& x) {
    if ((uint32_t)q.minors & g.used) return false;
    if ((g.total & (uint32_t)q.minors) != (uint32_t)q.minors) return false;
    if (x.dflags & KG_GPU_POD_RING_BW) return q.ring_bw >= 0 && x.dbw <= q.ring_bw;
    return true;
}

// allocateByPartition for a non-shared request on partition table `tbl` (1-based; 0 = none).
// (An earlier form with the bin-pack weights in a local array indexed by the loop counter returned a wrong
// partition on gfx950 at -O1 and -O3 while the same source was right on the host and right with a printf in
// the loop: tools/dbg_part.hip keeps it as a reproducer; this form is checked by tests/test_gpu_alloc_kat.py.)
__device__ __forceinline__ GpuAlloc gpu_partition(const ExtDev& e, uint32_t tbl, const PodX& x, const GpuMinors& g,
                                                  bool want_mask = true) {
    if (tbl == 0u || !e.parts) return {KG_DEV_CODE_NO_PARTITION, 0u};
    const uint32_t N = x.dcount;
    if (N > 8u) return {KG_DEV_CODE_PART_COUNT, 0u};
    const uint32_t rng = e.part_rng[(tbl - 1u) * 9u + N];
    const uint32_t b = rng & 0xFFFFu, en = rng >> 16;
    if (b >= en) return {KG_DEV_CODE_PART_COUNT, 0u};
    const bool restricted = (x.dflags & KG_GPU_POD_RESTRICTED) != 0;
    // the feasible partitions all come from one AllocationScore group: the first that has any (only the
    // first group under the Restricted policy)
    uint32_t gb = b, ge = b, nfeas = 0;
    while (gb < en) {
        const int32_t sg = e.parts[gb].alloc_score;
        ge = gb;
        while (ge < en && e.parts[ge].alloc_score == sg) {
            nfeas += partition_ok(e.parts[ge], g, x) ? 1u : 0u;
            ge++;
        }
        if (nfeas > 0u || restricted) break;
        gb = ge;
    }
    if (nfeas == 0u) return {KG_DEV_CODE_PARTITIONED, 0u};
    if (!want_mask) return {0u, 0u};  // the Filter: which partition the bin-pack picks does not matter
    // selectPartitionByBinPack (:261-296): the first of the highest bin-pack scores (sort.Slice of <= 12
    // elements is an insertion sort, stable); scoreOfNumOfGPUs 8: 10000, 4: 100, 2: 1
    uint32_t best_mask = 0u;
    int64_t best = -1;
    for (uint32_t t = gb; t < ge; t++) {
        const kg_gpu_partition q = e.parts[t];
        if (!partition_ok(q, g, x)) continue;
        if (nfeas == 1u) return {0u, (uint32_t)q.minors};
        const uint32_t allocated = g.used | (uint32_t)q.minors;
        int64_t score = 0;
        if (N <= 8u) score += 10000 * free_partitions(e, tbl, 0u, allocated);
        if (N <= 4u) score += 100 * free_partitions(e, tbl, 1u, allocated);
        if (N <= 2u) score += free_partitions(e, tbl, 2u, allocated);
        if (score > best) {
            best = score;
            best_mask = q.minors;
        }
    }
    return {0u, best_mask};
}

struct ScopeRes {
    uint32_t mask;
    int32_t depth, cne;
    int64_t score;
};

// allocateFromScope's take at one scope (:393-449): the first numberOfGPUs satisfied minors in minor
// order, or for a shared GPU the satisfied minor of the highest scoreDevice (first on ties). The shared
// score is scoreDevice(requestsPerGPU, free, total) with total and free swapped as the call site passes them
// (:412): dev_least over (free, total).
__device__ __forceinline__ ScopeRes scope_take(const KCfg& c, const DevRec* __restrict__ d, const PodX& x, uint32_t mask,
                                               const GpuMinors& g, bool shared, int32_t depth, int32_t cne) {
    ScopeRes r{0u, depth, cne, -1};
    uint32_t cand = mask & g.sat;
    if (!shared) {
        uint32_t got = 0, pick = 0;
        while (cand && got < x.dcount) {
            const uint32_t m = __builtin_ctz(cand);
            cand &= cand - 1u;
            pick |= 1u << m;
            got++;
        }
        if (got == x.dcount) r.mask = pick;
        return r;
    }
    int32_t bm = -1;
    while (cand) {
        const uint32_t m = __builtin_ctz(cand);
        cand &= cand - 1u;
        int64_t t[DEV_R], f[DEV_R];
#pragma unroll
        for (int k = 0; k < DEV_R; k++) {
            t[k] = d->total[k][m];
            f[k] = d->free_[k][m];
        }
        const int64_t sc = dev_least(c, f, t, x.dreq);
        if (sc > r.score || bm < 0) {
            if (sc > r.score) r.score = sc;
            bm = (int32_t)m;
        }
    }
    if (bm >= 0) r.mask = 1u << bm;
    return r;
}

// bestAllocateResult update over the child scopes in order (:372-387)
__device__ __forceinline__ void scope_merge(ScopeRes& best, const ScopeRes& r, bool shared) {
    if (!r.mask) return;
    if (!best.mask) {
        best = r;
        return;
    }
    if (best.depth < r.depth || (best.depth == r.depth && best.cne < r.cne)) best = r;
    if (shared && best.depth == r.depth && best.cne == r.cne && best.score < r.score) best = r;
}

// The node's GPU tree from dev_topo: per NUMA rank and per PCIe rank the minor mask, 8 bits per rank (ranks and
// minors < 8), and per PCIe rank its NUMA rank (3 bits each). Packed in registers: indexed local arrays would live in
// scratch memory.
struct GpuTree {
    uint64_t numa, pcie;
    uint32_t pcie_numa;
};

__device__ __forceinline__ GpuTree gpu_tree(int32_t D, uint64_t topo) {
    GpuTree t{0ull, 0ull, 0u};
    for (int32_t m = 0; m < D; m++) {
        const uint32_t b = (uint32_t)(topo >> (8 * m)) & 0xFFu;
        if (b == KG_GPU_NO_SCOPE) continue;
        const uint32_t q = (b >> 4) & 7u, r = b & 7u;
        t.numa |= (uint64_t)(1u << m) << (8u * q);
        t.pcie |= (uint64_t)(1u << m) << (8u * r);
        t.pcie_numa = (t.pcie_numa & ~(7u << (3u * r))) | (q << (3u * r));
    }
    return t;
}
__device__ __forceinline__ uint32_t tree_numa(const GpuTree& t, uint32_t q) { return (uint32_t)(t.numa >> (8u * q)) & 0xFFu; }
__device__ __forceinline__ uint32_t tree_pcie(const GpuTree& t, uint32_t r) { return (uint32_t)(t.pcie >> (8u * r)) & 0xFFu; }
__device__ __forceinline__ uint32_t tree_pcie_numa(const GpuTree& t, uint32_t r) { return (t.pcie_numa >> (3u * r)) & 7u; }

// allocateFromScope over the node -> NUMA node -> PCIe tree of dev_topo (GetGPUTopologyScope,
// allocator_gpu_helper.go:201-262: NUMA scopes in NUMA id order, PCIe scopes in PCIe id order). `level`:
// DeviceTopologyScopeLevel of the required scope (0 = none). Depth: node 1, NUMA 2, PCIe 3.
__device__ __forceinline__ uint32_t gpu_scope(const KCfg& c, const DevRec* __restrict__ d, int32_t D, uint64_t topo,
                                              const PodX& x, const GpuMinors& g, int32_t level, bool shared) {
    const uint32_t N = x.dcount;
    const uint32_t root = D >= 32 ? ~0u : (1u << D) - 1u;
    if ((uint32_t)__popc(root) < N) return 0u;
    // scope minor sets from the per-minor ranks (dense: NUMA ranks 0..nq-1, PCIe ranks 0..np-1, both <= D)
    const GpuTree tr = gpu_tree(D, topo);
    const int32_t cne1 = (root & g.used) ? 1 : 0;
    ScopeRes best{0u, 0, 0, -1};
    for (uint32_t q = 0; q < (uint32_t)DEV_MINORS; q++) {  // NUMA scopes in rank order
        const uint32_t qm = tree_numa(tr, q);
        if (!qm) break;
        if ((uint32_t)__popc(qm) < N) continue;
        const int32_t cne2 = cne1 + ((qm & g.used) ? 1 : 0);
        ScopeRes bq{0u, 0, 0, -1};
        if (level <= 3) {  // a PCIe scope has no children; below the required level it yields nothing
            for (uint32_t r = 0; r < (uint32_t)DEV_MINORS; r++) {  // PCIe scopes of this NUMA node in rank order
                const uint32_t rm = tree_pcie(tr, r);
                if (!rm) break;
                if (tree_pcie_numa(tr, r) != q || (uint32_t)__popc(rm) < N) continue;
                scope_merge(bq, scope_take(c, d, x, rm, g, shared, 3, cne2 + ((rm & g.used) ? 1 : 0)), shared);
            }
        }
        if (!bq.mask && level <= 2) bq = scope_take(c, d, x, qm, g, shared, 2, cne2);
        scope_merge(best, bq, shared);
    }
    if (best.mask) return best.mask;
    if (level > 1) return 0u;
    return scope_take(c, d, x, root, g, shared, 1, cne1).mask;
}

// gpu_scope's outcome without the choice (the Filter): a take at a scope succeeds iff the scope holds N satisfied
// minors, and a scope's minors include its children's, so the tree allocates iff some scope the required level
// admits (PCIe: level <= 3, NUMA: <= 2, the node: <= 1) has N satisfied minors.
__device__ __forceinline__ bool gpu_scope_fits(int32_t D, uint64_t topo, uint32_t N, const GpuMinors& g, int32_t level) {
    const uint32_t root = D >= 32 ? ~0u : (1u << D) - 1u;
    if ((uint32_t)__popc(root) < N) return false;
    if (level <= 1) return (uint32_t)__popc(root & g.sat) >= N;
    const GpuTree tr = gpu_tree(D, topo);
    for (uint32_t q = 0; q < (uint32_t)DEV_MINORS; q++) {
        const uint32_t qm = tree_numa(tr, q);
        if (!qm) break;
        if ((uint32_t)__popc(qm) < N) continue;
        if (level <= 3)
            for (uint32_t r = 0; r < (uint32_t)DEV_MINORS; r++) {
                const uint32_t rm = tree_pcie(tr, r);
                if (!rm) break;
                if (tree_pcie_numa(tr, r) == q && (uint32_t)__popc(rm) >= N && (uint32_t)__popc(rm & g.sat) >= N) return true;
            }
        if (level <= 2 && (uint32_t)__popc(qm & g.sat) >= N) return true;
    }
    return false;
}

// defaultAllocateDevices (device_allocator.go:355-437): minors by (preferred first, scoreDevice desc, minor asc;
// sortDeviceResourcesByMinor, device_resources.go:187-209), the first numberOfGPUs whose free resources are not all
// zero and cover the request. pref: the preferred minors (a reservation's reserved ones when the pod allocates from it,
// deviceshare/reservation.go:308). want_mask = false: only whether enough minors fit (the Filter; the order cannot
// change that).
__device__ __forceinline__ GpuAlloc dev_default(const KCfg& c, const DevRec* __restrict__ d, int32_t D, const PodX& x,
                                                bool want_mask, uint32_t allowed = ~0u, uint32_t pref = 0u) {
    uint32_t fit = 0;
    for (int32_t m = 0; m < D; m++) {
        const int64_t fr[DEV_R] = {d->free_[0][m], d->free_[1][m], d->free_[2][m]};
        fit += (((allowed >> m) & 1u) && dev_minor_fits(fr, x)) ? 1u : 0u;
    }
    if (fit < x.dcount) return {KG_DEV_CODE_INSUFFICIENT, 0u};
    if (!want_mask) return {0u, 0u};
    // the minors in (score desc, minor asc) order (the reference's stable sort) by repeated selection of the best
    // remaining one; the loops over DEV_MINORS unroll, so sc[] and the fitting set stay in registers
    int64_t sc[DEV_MINORS];
    uint32_t fits = 0;
#pragma unroll
    for (int m = 0; m < DEV_MINORS; m++) {
        sc[m] = 0;
        if (m >= D) continue;
        int64_t t[DEV_R], f[DEV_R];
#pragma unroll
        for (int r = 0; r < DEV_R; r++) {
            t[r] = d->total[r][m];
            f[r] = d->free_[r][m];
        }
        sc[m] = dev_least(c, t, f, x.dreq);
        fits |= (((allowed >> m) & 1u) && dev_minor_fits(f, x)) ? 1u << m : 0u;
    }
    uint32_t left = D >= 32 ? ~0u : (1u << D) - 1u, mask = 0, got = 0;
    while (left && got < x.dcount) {
        int32_t bm = -1;
        int64_t bs = 0;
#pragma unroll
        for (int m = 0; m < DEV_MINORS; m++) {
            const bool pm = (pref >> m) & 1u, pb = bm >= 0 && ((pref >> bm) & 1u);
            const bool take = ((left >> m) & 1u) && (bm < 0 || (pm && !pb) || (pm == pb && sc[m] > bs));
            bs = take ? sc[m] : bs;
            bm = take ? m : bm;
        }
        left &= ~(1u << bm);
        if ((fits >> bm) & 1u) {
            mask |= 1u << bm;
            got++;
        }
    }
    return {0u, mask};
}

// allocateByTemplate (allocator_gpu.go:135-159): how many of the pod's candidate templates carry the node's
// vendor-model key. 0 fails the allocation (KG_DEV_CODE_NO_TEMPLATE), 1 goes straight to generalAllocate (the
// partition stage is skipped; the template name only annotates the allocation), more fall through. Pods that
// enforce no template: 2.
__device__ __forceinline__ uint32_t gpu_template(const PodX& x, uint32_t part) {
    if (!(x.dflags & KG_GPU_POD_TEMPLATE)) return 2u;
    const uint32_t key = (part >> KG_GPU_TMPL_SHIFT) & 15u;
    return key == KG_GPU_TMPL_NONE ? 0u : (x.dtmpl >> (2 * key)) & 3u;
}

// GPUAllocator.Allocate's outcome (the Filter: no minors chosen) from the table's minor sets.
__device__ __forceinline__ uint32_t gpu_allocate_code(const ExtDev& e, int32_t D, uint64_t topo, uint32_t part,
                                                      const PodX& x, const GpuMinors& g) {
    // (g.fit already holds only the allowed minors)
    const uint32_t tm = gpu_template(x, part);
    if (tm == 0u) return KG_DEV_CODE_NO_TEMPLATE;
    const bool shared = (x.dflags & KG_GPU_POD_SHARED) != 0;
    const uint32_t sfield = (x.dflags >> KG_GPU_POD_SCOPE_SHIFT) & 7u;
    const bool required = sfield != 0u;
    const int32_t level = sfield > 4u ? 0 : (int32_t)sfield;
    const uint32_t tbl = part & 0xFFu;
    const bool honor = (x.dflags & KG_GPU_POD_HONOR) || (part & KG_GPU_HONOR);
    if (!shared && tm != 1u && (tbl != 0u || honor)) {
        const uint32_t code = gpu_partition(e, tbl, x, g, false).code;
        if (code == 0u || honor) return code;
    }
    if (part & KG_GPU_TREE) {
        if (!(shared && x.dcount > 1u))
            return gpu_scope_fits(D, topo, x.dcount, g, level) ? 0u
                                                                : (required ? KG_DEV_CODE_TOPO_SCOPED : KG_DEV_CODE_GPU_DEVICES);
        if (required) return KG_DEV_CODE_MULTI_SHARED;
    } else if (required) {
        return KG_DEV_CODE_NO_TREE;
    }
    return (uint32_t)__popc(g.fit) >= x.dcount ? 0u : KG_DEV_CODE_INSUFFICIENT;
}

// GPUAllocator.Allocate for a pod with a GPU request on a node with D > 0 minors. topo / part: the node's
// ZoneRec.dev_topo / dev_part; outside: minors used on the node outside the table (0 for the node's own).
__device__ __forceinline__ GpuAlloc gpu_allocate(const KCfg& c, const ExtDev& e, const DevRec* __restrict__ d, int32_t D,
                                                 uint64_t topo, uint32_t part, const PodX& x, uint32_t outside,
                                                 bool want_mask, uint32_t allowed = ~0u, uint32_t pref = 0u) {
    if (!want_mask) return {gpu_allocate_code(e, D, topo, part, x, gpu_minors(d, D, x, outside, allowed)), 0u};
    const uint32_t tm = gpu_template(x, part);
    if (tm == 0u) return {KG_DEV_CODE_NO_TEMPLATE, 0u};
    const bool shared = (x.dflags & KG_GPU_POD_SHARED) != 0;
    const uint32_t sfield = (x.dflags >> KG_GPU_POD_SCOPE_SHIFT) & 7u;
    const bool required = sfield != 0u;
    const int32_t level = sfield > 4u ? 0 : (int32_t)sfield;  // 5: a scope name without a level
    const bool tree = (part & KG_GPU_TREE) != 0;
    const uint32_t tbl = part & 0xFFu;
    // partitions apply to whole GPUs; a node without table or a non-honored miss falls through
    if (!shared && tm != 1u && (tbl != 0u || (x.dflags & KG_GPU_POD_HONOR) || (part & KG_GPU_HONOR))) {
        const GpuMinors g = gpu_minors(d, D, x, outside, allowed);
        const GpuAlloc pa = gpu_partition(e, tbl, x, g);
        if (pa.code == 0u) return pa;
        if ((x.dflags & KG_GPU_POD_HONOR) || (part & KG_GPU_HONOR)) return pa;
    }
    if (tree) {
        if (!(shared && x.dcount > 1u)) {
            const GpuMinors g = gpu_minors(d, D, x, outside, allowed);
            const uint32_t mask = gpu_scope(c, d, D, topo, x, g, level, shared);
            if (mask) return {0u, mask};
            return {required ? KG_DEV_CODE_TOPO_SCOPED : KG_DEV_CODE_GPU_DEVICES, 0u};
        }
        if (required) return {KG_DEV_CODE_MULTI_SHARED, 0u};
    } else if (required) {
        return {KG_DEV_CODE_NO_TREE, 0u};
    }
    return dev_default(c, d, D, x, want_mask, allowed, pref);
}

__device__ __forceinline__ uint32_t dev_code_status(uint32_t code) { return code ? KG_ST_DEV_MAKE(code) : 0u; }

// ---- DeviceShare under a NUMA affinity (deviceshare/topology_hint.go:40-290, device_allocator.go:143-176) ---------

// the minors filterNodeDevice keeps under NUMA affinity `numa` (bit per zone): a Topology whose NodeID is -1 or in
// the affinity (device_allocator.go:155-159)
__device__ __forceinline__ uint32_t gpu_numa_allowed(uint32_t dev_numa, int32_t D, uint32_t numa) {
    uint32_t a = 0;
    for (int32_t m = 0; m < D && m < DEV_MINORS; m++) {
        const uint32_t q = (dev_numa >> (4 * m)) & 15u;
        a |= (q == KG_GPU_NUMA_ANY || (q < (uint32_t)MAX_ZONES && ((numa >> q) & 1u))) ? 1u << m : 0u;
    }
    return a;
}

// The allocator on one table under NUMA affinity `numa` (0 = nil): the node's own devices (tab == nullptr, unfiltered
// when numa is 0) or a reservation restore table (kg_rsv_dev, already a filtered nodeDevice). The filtered nodeDevice
// keeps the table's minors the affinity allows (gpu_minors' `allowed`); getRealUsed (allocator_gpu.go:59-70) counts
// the node's used minors it leaves out (`outside`). When no free is left the filter drops the GPU type, which every
// allocator stage then fails on alike.
__device__ __forceinline__ GpuAlloc gpu_alloc_tab_numa(const KCfg& c, const ExtDev& e, const DevRec* __restrict__ d,
                                                       const DevRec* __restrict__ tab, int32_t D,
                                                       const ZoneRec* __restrict__ zr, const PodX& x, uint32_t numa,
                                                       bool want_mask, uint32_t pref = 0u) {
    if (D == 0) return {KG_DEV_CODE_NO_DEVICE, 0u};  // Prepare (devicehandler_gpu.go:41-44)
    uint32_t in = ~0u, outside = 0u;  // the node's own devices without an affinity: no filter
    if (tab || numa) {
        const uint32_t allowed = numa ? gpu_numa_allowed(zr->dev_numa, D, numa) : (D >= 32 ? ~0u : (1u << D) - 1u);
        uint32_t in_tab = tab ? 0u : ~0u, node_used = 0;
        for (int32_t m = 0; m < D && m < DEV_MINORS; m++) {
            bool it = false, nu = false;
#pragma unroll
            for (int r = 0; r < DEV_R; r++) {
                if (tab) it |= tab->total[r][m] != 0;
                nu |= d->free_[r][m] != d->total[r][m];
            }
            in_tab |= it ? 1u << m : 0u;
            node_used |= nu ? 1u << m : 0u;
        }
        in = allowed & in_tab;
        outside = node_used & ~in;
    }
    return gpu_allocate(c, e, tab ? tab : d, D, zr->dev_topo, zr->dev_part, x, outside, want_mask, in, pref);
}

__device__ __forceinline__ GpuAlloc gpu_alloc_numa(const KCfg& c, const ExtDev& e, const DevRec* __restrict__ d,
                                                   int32_t D, const ZoneRec* __restrict__ zr, const PodX& x, uint32_t numa,
                                                   bool want_mask) {
    return gpu_alloc_tab_numa(c, e, d, nullptr, D, zr, x, numa, want_mask);
}

// AutopilotAllocator.score (device_allocator.go:486-508) on a table under NUMA affinity `numa`: scoreNode over the
// filtered devices' sums; 0 when the filter drops the GPU type (no free left in the table; the node's unfiltered
// devices without an affinity skip that check). tab == nullptr: the node's devices.
__device__ __forceinline__ int64_t dev_score_tab_numa(const KCfg& c, const DevRec* __restrict__ d,
                                                      const DevRec* __restrict__ tab, int32_t D, uint32_t dev_numa,
                                                      const PodX& x, uint32_t numa) {
    const DevRec* t = tab ? tab : d;
    const int32_t Dt = tab ? DEV_MINORS : D;
    const uint32_t allowed = numa ? gpu_numa_allowed(dev_numa, D, numa) : ~0u;
    int64_t T[DEV_R] = {0, 0, 0}, F[DEV_R] = {0, 0, 0};
    bool any = false;
    for (int32_t m = 0; m < Dt; m++) {
        const bool in = ((allowed >> m) & 1u) != 0;
#pragma unroll
        for (int r = 0; r < DEV_R; r++) {
            T[r] += in ? t->total[r][m] : 0;
            F[r] += in ? t->free_[r][m] : 0;
            any |= t->free_[r][m] != 0;
        }
    }
    return ((tab || numa) && !any) ? 0 : dev_least(c, T, F, x.dreq);
}

// Filter (GPUAllocator.Allocate succeeds) + node Score before NormalizeScore.
__device__ __forceinline__ uint32_t dev_eval(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                             const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d,
                                             const PodX& x, int64_t& raw, uint32_t outside = 0u) {
    raw = 0;
    if (x.dcount == 0) return 0;  // PreFilter Skip
    const int32_t D = (int32_t)n[N_DEV_MINORS];
    if (D < 0) return 0;  // no Device object
    if (D == 0) return KG_ST_DEV_NO_DEVICE;
    const GpuAlloc a = gpu_allocate(c, e, d, D, zr->dev_topo, zr->dev_part, x, outside, false);
    if (a.code) return dev_code_status(a.code);
    int64_t T[DEV_R] = {0, 0, 0}, F[DEV_R] = {0, 0, 0};
    for (int32_t m = 0; m < D; m++) {
#pragma unroll
        for (int r = 0; r < DEV_R; r++) {
            T[r] += d->total[r][m];
            F[r] += d->free_[r][m];
        }
    }
    raw = dev_least(c, T, F, x.dreq);
    return 0;
}

// DeviceShare Filter + node Score from the record's DevSum for a pod of GPU request class cls (same
// results as dev_eval; a pod outside the batch's classes runs the allocator).
__device__ __forceinline__ uint32_t dev_eval_sum(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                                 const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d,
                                                 const DevSum* __restrict__ ds, const PodX& x, uint32_t cls, int64_t& raw) {
    raw = 0;
    if (x.dcount == 0) return 0;
    const int32_t D = (int32_t)n[N_DEV_MINORS];
    if (D < 0) return 0;
    if (D == 0) return KG_ST_DEV_NO_DEVICE;
    if (cls >= (uint32_t)DEV_CLASSES) return dev_eval(c, e, n, zr, d, x, raw);
    const uint32_t code = ds->code[cls];
    if (code) return dev_code_status(code);
    raw = ds->score[cls];  // k_dev_sum: dev_sum_score of the class
    return 0;
}

// dev_eval_sum for a pod that has a class (the fast-base kernels run only when every GPU pod of the batch has one):
// the tabulated allocator outcome and Score, no allocator code in the kernel.
__device__ __forceinline__ uint32_t dev_eval_cls(const int64_t* __restrict__ n, const DevSum* __restrict__ ds,
                                                 const PodX& x, uint32_t cls, int64_t& raw) {
    raw = 0;
    if (x.dcount == 0) return 0;
    const int32_t D = (int32_t)n[N_DEV_MINORS];
    if (D < 0) return 0;
    if (D == 0) return KG_ST_DEV_NO_DEVICE;
    const uint32_t code = ds->code[cls];
    if (code) return dev_code_status(code);
    raw = ds->score[cls];
    return 0;
}

// The node Score of one GPU instance of a class from the record's minor sums (dev_eval's arithmetic).
__device__ __forceinline__ int64_t dev_sum_score(const KCfg& c, const DevSum* __restrict__ ds, const PodX& x) {
    int64_t raw = 0;
    if (c.most & MOST_DEV) {
        return dev_least(c, ds->T, ds->F, x.dreq);
    }
    int64_t score = 0, wsum = 0;
#pragma unroll
    for (int r = 0; r < DEV_R; r++) {
        const int64_t w = c.dev_w[r], T = ds->T[r], F = ds->F[r];
        if (w == 0 || T == 0) continue;
        const int64_t req = T >= F ? T - F + x.dreq[r] : T;
        score += least_req<false>(req, T, ds->rcp[r]) * w;
        wsum += w;
    }
    raw = wdiv(score, wsum);
    return raw;
}

// DeviceShare Score on a restore table (AutopilotAllocator.score, device_allocator.go:486-508): a table
// whose free is zero everywhere leaves the GPU type out (nodeDevice.filter skips it): score 0.
__device__ __forceinline__ int64_t dev_score(const KCfg& c, const DevRec* __restrict__ d, const PodX& x) {
    int64_t T[DEV_R] = {0, 0, 0}, F[DEV_R] = {0, 0, 0};
    bool any = false;
    for (int m = 0; m < DEV_MINORS; m++) {
#pragma unroll
        for (int r = 0; r < DEV_R; r++) {
            T[r] += d->total[r][m];
            F[r] += d->free_[r][m];
            any |= d->free_[r][m] != 0;
        }
    }
    return any ? dev_least(c, T, F, x.dreq) : 0;
}

// Reserve: the minors GPUAllocator.Allocate takes on the node (0 when it fails), inside the NUMA affinity the
// topology manager stored for the pair (DeviceShare Reserve, plugin.go:585-600): the pair's zone code.
__device__ __forceinline__ uint32_t dev_choose(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                               const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d,
                                               const PodX& x, int32_t zone) {
    const int32_t D = (int32_t)n[N_DEV_MINORS];
    if (x.dcount == 0 || D <= 0) return 0;
    const GpuAlloc a = gpu_alloc_numa(c, e, d, D, zr, x, zone_affinity(zone), true);
    return a.code ? 0u : a.mask;
}

// fillGPUTotalMem: gpu-memory from the ratio, or the ratio from gpu-memory in float64 like Go.
__device__ __forceinline__ void dev_alloc_of(const PodX& x, int64_t total_mem, int64_t* a) {
    a[0] = ((x.dkeys >> 0) & 1u) ? x.dreq[0] : 0;
    const bool hr = ((x.dkeys >> 1) & 1u) != 0, hm = ((x.dkeys >> 2) & 1u) != 0;
    if (hr && hm) {
        a[1] = x.dreq[1];
        a[2] = x.dreq[2];
    } else if (hm) {
        a[2] = x.dreq[2];
        const double q = __ddiv_rn((double)x.dreq[2], (double)total_mem);
        a[1] = (int64_t)__dmul_rn(q, 100.0);
    } else {
        const int64_t ratio = hr ? x.dreq[1] : 0;
        a[1] = ratio;
        a[2] = ratio * total_mem / 100;
    }
}

__device__ __forceinline__ void dev_apply(DevRec* __restrict__ d, uint32_t mask, const PodX& x, int64_t sign) {
    for (int m = 0; m < DEV_MINORS; m++) {
        if (!((mask >> m) & 1u)) continue;
        int64_t a[DEV_R];
        dev_alloc_of(x, d->total[2][m], a);
#pragma unroll
        for (int r = 0; r < DEV_R; r++) d->free_[r][m] -= sign * a[r];
    }
}

// ---- ElasticQuota -----------------------------------------------------------------------------------

__device__ __forceinline__ void quota_req(const PodV& p, const PodX& x, int64_t* q) {
    const int64_t v[QUOTA_R] = {p.req_cpu, p.req_mem, p.sc0, p.sc1};
#pragma unroll
    for (int r = 0; r < QUOTA_R; r++) q[r] = ((x.qkeys >> r) & 1u) ? v[r] : 0;
}

// quotav1.LessThanOrEqual(a, b) over the keys of b that a has
__device__ __forceinline__ bool quota_le(const int64_t* a, uint32_t ak, const int64_t* b, uint32_t bk) {
    bool ok = true;
#pragma unroll
    for (int r = 0; r < QUOTA_R; r++) ok &= !((((ak & bk) >> r) & 1u) && a[r] > b[r]);
    return ok;
}

// PreFilter of the pod's quota given that quota's current state
__device__ __forceinline__ uint32_t quota_gate(const QuotaLim& L, const QuotaState& S, const PodV& p, const PodX& x) {
    int64_t q[QUOTA_R], a[QUOTA_R];
    quota_req(p, x, q);
#pragma unroll
    for (int r = 0; r < QUOTA_R; r++) a[r] = q[r] + S.used[r];
    if (!quota_le(a, x.qkeys | S.used_keys, L.limit, L.limit_keys)) return KG_ST_QUOTA;
    if (p.flags & KG_POD_NON_PREEMPTIBLE) {
#pragma unroll
        for (int r = 0; r < QUOTA_R; r++) a[r] = q[r] + S.np_used[r];
        if (!quota_le(a, x.qkeys | S.np_keys, L.min, L.min_keys)) return KG_ST_QUOTA;
    }
    return 0;
}

__device__ __forceinline__ void quota_add(QuotaState& S, const PodV& p, const PodX& x, int64_t sign) {
    int64_t q[QUOTA_R];
    quota_req(p, x, q);
    const bool np = (p.flags & KG_POD_NON_PREEMPTIBLE) != 0;
#pragma unroll
    for (int r = 0; r < QUOTA_R; r++) {
        if (!((x.qkeys >> r) & 1u)) continue;
        const int64_t u = S.used[r] + sign * q[r];
        S.used[r] = u < 0 ? 0 : u;
        if (np) {
            const int64_t v = S.np_used[r] + sign * q[r];
            S.np_used[r] = v < 0 ? 0 : v;
        }
    }
    S.used_keys |= x.qkeys;
    if (np) S.np_keys |= x.qkeys;
}

// ---- Reservation ------------------------------------------------------------------------------------

__device__ __forceinline__ const RsvView* find_view(const ExtDev& e, int32_t cls, uint32_t rec,
                                                   const int64_t* __restrict__ n) {
    // one dependent load instead of a binary search over the class's views
    const uint64_t mask = (uint64_t)n[N_RSV_CLASSES];
    if (!((mask >> cls) & 1ull)) return nullptr;
    return &e.views[e.vmap[e.vfirst[rec] + (uint32_t)__popcll(mask & ((1ull << cls) - 1ull))]];
}

struct RsvPod {
    int64_t preq[RSV_R];
    uint32_t names;
    bool required;
};

__device__ __forceinline__ RsvPod rsv_pod(const PodV& p) {
    RsvPod r;
    r.preq[0] = p.req_cpu;
    r.preq[1] = p.req_mem;
    r.preq[2] = p.req_eph;
    r.preq[3] = p.sc0;
    r.preq[4] = p.sc1;
    r.names = ((p.flags & KG_POD_HAS_CPU) ? 1u : 0u) | ((p.flags & KG_POD_HAS_MEM) ? 2u : 0u) |
              (p.req_eph != 0 ? 4u : 0u) | (p.sc0 != 0 ? 8u : 0u) | (p.sc1 != 0 ? 16u : 0u);
    r.required = (p.flags & KG_POD_RSV_REQUIRED) != 0;
    return r;
}

// fitsNode: bitmask of insufficient resources (bit 5 = pods); rem == nullptr -> zero remained
__device__ __forceinline__ uint32_t rsv_fits_node(const RsvPod& q, const int64_t* __restrict__ n, const RsvView& v,
                                                  const int64_t* rem, uint32_t ign) {
    uint32_t bad = 0;
    if (v.num_pods - (int64_t)v.count + 1 > n[N_ALLOC_PODS]) bad |= 1u << 5;
    if (q.preq[0] == 0 && q.preq[1] == 0 && q.preq[2] == 0 && !(q.names & 0x18u)) return bad;
    const int64_t alloc[RSV_R] = {n[N_ALLOC_CPU], n[N_ALLOC_MEM], n[N_ALLOC_EPH], n[N_SC_ALLOC0], n[N_SC_ALLOC1]};
#pragma unroll
    for (int k = 0; k < RSV_R; k++) {
        if (k >= 3 && !((q.names >> k) & 1u)) continue;
        if (k >= 3 && ((ign >> (k - 3)) & 1u)) continue;  // isResourceIgnored (reservation/plugin.go:951-953)
        const int64_t rk = rem ? rem[k] : 0;
        if (q.preq[k] > alloc[k] - (v.pod_requested[k] - rk - v.r_allocated[k])) bad |= 1u << k;
    }
    return bad;
}

__device__ __forceinline__ uint32_t rsv_fits_reservation(const RsvPod& q, const RsvInfo& r, uint32_t ign) {
    uint32_t bad = 0;
    if (r.max_pods >= 0 && r.allocated_pods + 1 > r.max_pods) bad |= 1u << 5;
#pragma unroll
    for (int k = 0; k < RSV_R; k++) {
        if (!((r.names >> k) & 1u)) continue;
        if (k >= 3 && ((ign >> (k - 3)) & 1u)) continue;
        if (!((q.names >> k) & 1u) || q.preq[k] == 0) continue;
        const int64_t used = r.allocated[k] < 0 ? 0 : r.allocated[k];
        const int64_t cap = r.allocatable[k] - r.reserved[k];
        if (q.preq[k] <= cap - used) continue;
        bad |= 1u << k;
    }
    return bad;
}

// fitsNodeAndReservation: true when the pod fits node + reservation r
__device__ __forceinline__ bool rsv_fits_one(const RsvPod& q, const int64_t* __restrict__ n, const RsvView& v,
                                             const RsvInfo& r, uint32_t& bn, uint32_t& br, uint32_t ign) {
    int64_t rem[RSV_R];
#pragma unroll
    for (int k = 0; k < RSV_R; k++) {
        const int64_t x = r.allocatable[k] - r.allocated[k] - r.reserved[k];
        rem[k] = x < 0 ? 0 : x;
    }
    bn = rsv_fits_node(q, n, v, rem, ign);
    br = 0;
    if (r.policy == KG_RSV_RESTRICTED) {
        br = rsv_fits_reservation(q, r, ign);
        return bn == 0 && br == 0;
    }
    return bn == 0;
}

__device__ __forceinline__ uint32_t rsv_filter(const RsvPod& q, const int64_t* __restrict__ n, const RsvView* v,
                                               const RsvInfo* __restrict__ infos, uint32_t ign) {
    if (!v) return q.required ? KG_ST_RSV_AFFINITY : 0u;
    uint32_t any_node = 0, any_resv = 0;
    for (uint32_t t = 0; t < v->count; t++) {
        const RsvInfo& r = infos[v->first + t];
        if (!q.required && !(r.names & q.names)) continue;
        uint32_t bn, br;
        if (rsv_fits_one(q, n, *v, r, bn, br, ign)) return 0;
        any_node |= bn;
        any_resv |= br;
    }
    if (q.required)
        return ((any_resv != 0 || any_node == 0) ? KG_ST_RSV_RESERVATION : 0u) | (any_node ? KG_ST_RSV_NODE : 0u);
    if (any_node) return KG_ST_RSV_NODE;
    return rsv_fits_node(q, n, *v, nullptr, ign) ? KG_ST_RSV_NODE : 0u;
}

__device__ __forceinline__ int64_t rsv_score_reservation(const RsvPod& q, const RsvInfo& r) {
    int64_t w = 0, s = 0;
#pragma unroll
    for (int k = 0; k < RSV_R; k++) {
        const int64_t cap = r.allocatable[k];
        if (cap == 0) continue;
        w++;
        const int64_t req = q.preq[k] + r.allocated[k];
        if (req <= cap) {
            const int64_t m = k == 0 ? 1 : 1000;
            s += (int64_t)(100ull * (uint64_t)(req * m)) / (cap * m);
        }
    }
    if (r.max_pods > 0) w++;
    return w <= 0 ? 0 : qdiv(s, w);
}

// nominated reservation's ScoreReservation and the node's most-preferred order (0 = none)
__device__ __forceinline__ int64_t rsv_nominate_score(const RsvPod& q, const int64_t* __restrict__ n, const RsvView& v,
                                                      const RsvInfo* __restrict__ infos, int64_t& node_order,
                                                      uint32_t ign, int& nom_out) {
    node_order = 0;
    nom_out = -1;
    int64_t sel = INT64_MAX;
    for (uint32_t t = 0; t < v.count; t++) {
        const int64_t o = infos[v.first + t].order;
        if (o != 0 && sel > o) {
            sel = o;
            node_order = o;
        }
    }
    if (v.count == 0) return 0;
    int nom = -1;
    if (v.count == 1 && q.required) {
        nom = 0;
    } else {
        uint32_t okm = 0, nc = 0;
        int last = -1;
        for (uint32_t t = 0; t < v.count; t++) {
            const RsvInfo& r = infos[v.first + t];
            if (r.allocate_once && r.allocated_pods > 0) continue;
            if (!q.required && !(r.names & q.names)) continue;
            uint32_t bn, br;
            if (!rsv_fits_one(q, n, v, r, bn, br, ign)) continue;
            okm |= 1u << t;
            nc++;
            last = (int)t;
        }
        if (nc == 1) {
            nom = last;
        } else if (nc > 1) {
            int64_t so = INT64_MAX;
            for (uint32_t t = 0; t < v.count; t++) {
                if (!((okm >> t) & 1u)) continue;
                const int64_t o = infos[v.first + t].order;
                if (o != 0 && so > o) {
                    so = o;
                    nom = (int)t;
                }
            }
            if (nom < 0) {
                int64_t best = -1;
                for (uint32_t t = 0; t < v.count; t++) {
                    if (!((okm >> t) & 1u)) continue;
                    const int64_t sc = rsv_score_reservation(q, infos[v.first + t]);
                    if (sc > best) {
                        best = sc;
                        nom = (int)t;
                    }
                }
            }
        }
    }
    nom_out = nom;
    return nom >= 0 ? rsv_score_reservation(q, infos[v.first + nom]) : 0;
}

// DeviceShare Filter of a GPU pod on a node where its class has a restore view (plugin.go:397-419):
// tryAllocateFromReusable over the matched reservations that reserve GPUs, in view order (reservation.go
// :344-410); if none fits, a pod with a reservation affinity fails there, any other pod allocates outside
// the reservations (the view's base table).
// Minors used on the node (free != total) that a restore table leaves out (total 0): getRealUsed's first
// term (allocator_gpu.go:59-70), the node's own used minors outside the filtered nodeDevice.
__device__ __forceinline__ uint32_t dev_outside_used(const DevRec* __restrict__ node, const DevRec* __restrict__ tab,
                                                     int32_t D) {
    uint32_t o = 0;
    for (int32_t m = 0; m < D; m++) {
        bool used = false, in_tab = false;
#pragma unroll
        for (int r = 0; r < DEV_R; r++) {
            used |= node->free_[r][m] != node->total[r][m];
            in_tab |= tab->total[r][m] != 0;
        }
        o |= (used && !in_tab) ? 1u << m : 0u;
    }
    return o;
}

// dcls < DEV_CLASSES with e.rcode: the restore tables' allocator outcomes come from k_rdev_codes, and the node's own
// table (a view without a base table) from the batch's DevSum.
__device__ __forceinline__ uint32_t dev_filter_view(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                                    const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d,
                                                    const RsvView& v, const PodX& x, bool required, uint32_t rec,
                                                    uint32_t dcls = (uint32_t)DEV_CLASSES) {
    const int32_t D = (int32_t)n[N_DEV_MINORS];
    if (D < 0) return 0;  // no Device object
    if (D == 0) return KG_ST_DEV_NO_DEVICE;
    const bool tab_codes = e.rcode && dcls < (uint32_t)DEV_CLASSES;
    bool any = false;
    for (uint32_t t = 0; t < v.count; t++) {
        const int32_t di = e.infos[v.first + t].dev;
        if (di < 0) continue;
        any = true;
        int64_t raw;
        if (tab_codes) {
            if (e.rcode[(size_t)di * DEV_CLASSES + dcls] == 0) return 0;
            continue;
        }
        const DevRec* tab = e.rdev + di;
        if (dev_eval(c, e, n, zr, tab, x, raw, dev_outside_used(d, tab, D)) == 0) return 0;
    }
    if (any && required) return KG_ST_DEV_RSV;
    int64_t raw;
    if (tab_codes) {
        if (v.dev_base >= 0) return dev_code_status(e.rcode[(size_t)v.dev_base * DEV_CLASSES + dcls]);
        if (e.dsum) return dev_code_status(e.dsum[rec].code[dcls]);
    }
    const DevRec* tab = v.dev_base >= 0 ? e.rdev + v.dev_base : d;
    return dev_eval(c, e, n, zr, tab, x, raw, tab == d ? 0u : dev_outside_used(d, tab, D));
}

// DeviceShare's allocation for a pair under NUMA affinity `numa`: off views the node's devices; on a view
// tryAllocateFromReusable over the matched reservations reserving GPUs in view order (deviceshare/reservation.go
// :344-410), then, unless the pod requires a reservation ("Reservation(s) Insufficient gpu devices"), the allocation
// outside them (the view's base table). Returns 0 (minors in `minors`) or the status bits.
__device__ __forceinline__ uint32_t gpu_alloc_site(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                                   const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d,
                                                   const RsvView* v, const PodX& x, bool required, uint32_t numa,
                                                   bool want_mask, uint32_t& minors) {
    const int32_t D = (int32_t)n[N_DEV_MINORS];
    minors = 0;
    if (v && D == 0) return KG_ST_DEV_NO_DEVICE;
    // the candidate tables in order: the view's reservations reserving GPUs, then the base (t == count); off views
    // only the node's own devices
    const uint32_t count = v ? v->count : 0u;
    bool any = false;
    for (uint32_t t = 0; t <= count; t++) {
        const DevRec* tab = nullptr;
        if (t < count) {
            const int32_t di = e.infos[v->first + t].dev;
            if (di < 0) continue;
            any = true;
            tab = e.rdev + di;
        } else {
            if (any && required) return KG_ST_DEV_RSV;
            if (v && v->dev_base >= 0) tab = e.rdev + v->dev_base;
        }
        const GpuAlloc a = gpu_alloc_tab_numa(c, e, d, tab, D, zr, x, numa, want_mask);
        if (!a.code || t == count) {
            minors = a.mask;
            return dev_code_status(a.code);
        }
    }
    return 0;  // not reached
}

// DeviceShare's Score of a feasible pair (scoring.go:45-104): on a view the nominated reservation's table (0 when it
// reserves no GPU, scoreWithNominatedReservation) or the base table, off views the node's devices; under NUMA
// affinity `numa` (0 = nil).
__device__ __forceinline__ int64_t gpu_score_site(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                                  const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d,
                                                  const RsvView* v, const PodX& x, uint32_t numa, int nom) {
    const int32_t D = (int32_t)n[N_DEV_MINORS];
    const DevRec* tab = nullptr;
    if (v) {
        if (nom >= 0) {
            const int32_t di = e.infos[v->first + (uint32_t)nom].dev;
            if (di < 0) return 0;
            tab = e.rdev + di;
        } else if (v->dev_base >= 0) {
            tab = e.rdev + v->dev_base;
        }
    }
    return dev_score_tab_numa(c, d, tab, D, zr->dev_numa, x, numa);
}

__device__ __forceinline__ uint32_t gpu_numa_count(uint32_t dev_numa, int32_t D, uint32_t m) {
    uint32_t cnt = 0;
    for (int32_t mi = 0; mi < D && mi < DEV_MINORS; mi++) {
        const uint32_t q = (dev_numa >> (4 * mi)) & 15u;
        cnt += (q < (uint32_t)MAX_ZONES && ((m >> q) & 1u)) ? 1u : 0u;
    }
    return cnt;
}

// DeviceShare's NUMA hints (generateTopologyHints, topology_hint.go:159-280): per mask over the GPUs' NUMA node ids
// (IterateBitMasks order) the GPUs inside must number the request and DeviceShare's allocation at the pair's site must
// succeed under the mask; Preferred = narrowest feasible width, Score 500 when the allocation equals the full mask's.
// Returns 0 with the list in h, or the status bits of the provider's failure: the full mask's status, which stands
// even when narrower masks fit (:191-196,271-279); the full mask is the last one iterated, so it is evaluated first.
__device__ __forceinline__ uint32_t gpu_numa_hints(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                                   const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d,
                                                   const RsvView* v, const PodX& x, bool required, GpuHints& h) {
    const int32_t D = (int32_t)n[N_DEV_MINORS];
    h.masks = 0;
    h.set = h.pref = h.s500 = 0;
    uint32_t ids = 0;
    for (int32_t m = 0; m < D && m < DEV_MINORS; m++) {
        const uint32_t q = (zr->dev_numa >> (4 * m)) & 15u;
        ids |= q < (uint32_t)MAX_ZONES ? 1u << q : 0u;
    }
    if (!ids) {  // no GPU with a NUMA node: the provider has no preference
        h.set = 1u << NUMA_NIL_K;
        return 0;
    }
    const uint32_t gn = (uint32_t)popc(ids);
    const uint64_t nib = numa_mask_nib(gn);
    const uint32_t nm = (1u << gn) - 1u;
    int minsize = (int)gn;
    uint32_t full_alloc = 0, alloc_of[15];
    uint32_t ok = 0;  // bit k: mask k feasible
    // masks in the order nm-1 (the full mask), 0, 1, ..., nm-2: the full mask's allocation is the Score-500
    // reference and its failure the provider's status
    for (uint32_t step = 0; step < nm; step++) {
        const uint32_t k = step == 0 ? nm - 1u : step - 1u;
        const uint32_t km = (uint32_t)(nib >> (4 * k)) & 15u;
        uint32_t m = 0, rest = ids;  // index bit b -> the b-th smallest NUMA id
        for (uint32_t b = 0; b < gn; b++) {
            const uint32_t id = (uint32_t)(__ffs(rest) - 1);
            rest &= rest - 1u;
            m |= ((km >> b) & 1u) ? 1u << id : 0u;
        }
        uint32_t st = gpu_numa_count(zr->dev_numa, D, m) < x.dcount ? (uint32_t)KG_ST_DEV_MAKE(KG_DEV_CODE_NUMA_SCOPED) : 0u;
        uint32_t alloc = 0;
        if (!st) st = gpu_alloc_site(c, e, n, zr, d, v, x, required, m, true, alloc);
        if (step == 0) {
            if (st) return st;
            full_alloc = alloc;
        }
        if (st) continue;
        ok |= 1u << k;
        alloc_of[k] = alloc;
        minsize = min(minsize, popc(m));
        h.masks |= (uint64_t)m << (4 * k);
    }
    // the list in IterateBitMasks order: entry k = mask k (kept only if feasible)
    for (uint32_t k = 0; k < nm; k++) {
        if (!((ok >> k) & 1u)) continue;
        h.set |= 1u << k;
        h.pref |= popc((uint32_t)(h.masks >> (4 * k)) & 15u) == minsize ? 1u << k : 0u;
        h.s500 |= alloc_of[k] == full_alloc ? 1u << k : 0u;
    }
    return 0;
}

// ---- DeviceShare in the NUMA topology manager ------------------------------------------------------------
// A GPU pod on a node (off reservation views) whose merged NUMA policy is not None: NodeNUMAResource's topology
// manager gathers DeviceShare's hints too (manager.go:65-154, topology_hint.go:40-290) and calls its Allocate
// under the best hint; the stored affinity then replaces DeviceShare's own Filter (plugin.go:369-374) and
// restricts its Score and Reserve. `b` is eval_pair's result: when NodeNUMAResource's Filter got as far as the
// topology manager, its NUMA part is recomputed here. BestEffort: Filter and Score as they are, the Reserve's
// zone with both providers (ZONE_GPU_FAIL | code when DeviceShare fails there).
template <bool EXACT, bool SCORE>
__device__ __forceinline__ void numa_gpu_eval(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                              const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d, const RsvView* v,
                                              const PodV& p, const PodX& x, PairOut& b, bool& dev_done, uint32_t& dev_mask) {
    if (p.flags & KG_POD_NUMA_SKIP) return;
    const uint32_t flags = (uint32_t)n[N_FLAGS];
    const uint32_t node_pol = (flags >> F_NUMA_POLICY_SHIFT) & 15u, pod_pol = (p.flags >> 16) & 15u;
    const uint32_t pol = pod_pol != KG_NUMA_NONE ? pod_pol : node_pol;
    if (pol == KG_NUMA_NONE) return;
    // the Filter stopped before the topology manager (policy conflict, amplified cpu, cpuset checks, the cpuset
    // path under a NUMA policy): eval_pair's status stands
    if (b.status & (KG_ST_NUMA_CONFLICT | KG_ST_NUMA_AMP_CPU | KG_ST_NUMA_CPU_BIND | KG_ST_NUMA_CPU_TOPO | KG_ST_NUMA_CPUS |
                    KG_ST_UNSUPPORTED))
        return;
    const uint32_t Z = (flags >> F_NUMA_ZONES_SHIFT) & 15u;
    const bool be = pol == KG_NUMA_BEST_EFFORT;  // admits at Reserve only: Filter / Score as eval_pair has them
    if (!be) {
        b.status &= ~(uint32_t)(KG_ST_NUMA_NO_RES | KG_ST_NUMA_ALIGN | KG_ST_NUMA_UNSATISFIED);
        b.zone = -1;
        b.s_numa = 0;
    }
    if (Z == 0) {  // FilterByNUMANode: "node(s) missing NUMA resources" (BestEffort: b.zone's Reserve failure)
        if (!be) b.status |= KG_ST_NUMA_NO_RES;
        return;
    }
    const bool excl = pod_pol != KG_NUMA_NONE;
    const bool required = (p.flags & KG_POD_RSV_REQUIRED) != 0;
    const int64_t req[2] = {p.req_cpu, p.req_mem};
    const bool has[2] = {(p.flags & KG_POD_HAS_CPU) != 0, (p.flags & KG_POD_HAS_MEM) != 0};
    GpuHints gh;
    const uint32_t fst = gpu_numa_hints(c, e, n, zr, d, v, x, required, gh);
    if (fst) {  // the provider's status (accumulateProvidersHints): the Filter fails / the Reserve fails
        if (be) b.zone = zone_gpu_fail(fst);
        else b.status |= fst;
        return;
    }
    NumaZ xz;
    numa_load(zr, Z, xz);
    // a cpuset-binding pod: its CPUs join every allocation (numa_eval's bind block)
    NumaBind bind;
    bool node_take = true;
    const NumaBind* bp = numa_bind_pair(zr, p, bind, node_take) ? &bind : nullptr;
    const bool amp = (flags & F_AMP) != 0;
    const int64_t score_cpu = (bp && amp) ? (int64_t)ceil(__dmul_rn((double)p.req_cpu, zr->amp_ratio)) : p.req_cpu;
    if (bp) numa_bind_trim(xz, bind);
    uint32_t mask = 0;
    const uint32_t st = numa_admit<true, true>(c, xz, req, has, pol, excl, mask, &gh, bp, score_cpu);
    if (st) {  // not under BestEffort (its merge always admits)
        b.status |= st;
        return;
    }
    int64_t al[2][MAX_ZONES];
    const uint32_t fail = mask ? numa_split(xz, mask, req, has, al, bp) : 0u;
    if (fail) {  // BestEffort: the Reserve's NUMA allocation fails; else not reached (a preferred hint places)
        if (be) b.zone = ZONE_RESERVE_FAIL | (int32_t)fail;
        else b.status |= KG_ST_UNSUPPORTED;
        return;
    }
    if (bp) {  // allocateCPUSet over the allocated NUMA nodes, or the whole node without an affinity
        const bool cfail = mask ? numa_bind_check(bind, al[0], al[1], Z) != 0u : !node_take;
        if (cfail) {
            if (be) b.zone = ZONE_CPUSET_FAIL;
            else b.status |= mask ? (uint32_t)KG_ST_UNSUPPORTED : (uint32_t)KG_ST_NUMA_CPUS;
            return;
        }
    }
    // allocateResources: DeviceShare's Allocate at the pair's site under the best hint
    uint32_t minors;
    const uint32_t ast = gpu_alloc_site(c, e, n, zr, d, v, x, required, mask, false, minors);
    if (be) {
        b.zone = ast ? zone_gpu_fail(ast) : numa_code(mask);
        return;
    }
    if (ast) {
        b.status |= ast;
        return;
    }
    dev_done = true;
    dev_mask = mask;
    b.zone = numa_code(mask);
    if constexpr (!SCORE) return;
    const bool most = (c.most & MOST_NUMA) != 0;
    // a cpuset-binding pod's requested cpu: the node's cpuset CPUs (amplified), its own request amplified
    const int64_t bind_cpu = amp ? n[N_AMP_CPUSET] : n[N_CPUSET];
    if (!mask || !(p.req_cpu | p.req_mem)) {  // no NUMANodeResources: node allocatable / requested (the view's NodeInfo on a view)
        const int64_t rc = bp ? bind_cpu : v ? v->req[0] : n[N_REQ_CPU], rm = v ? v->req[1] : n[N_REQ_MEM];
        b.s_numa = numa_score<EXACT>(most, c.numa_w_cpu, c.numa_w_mem, n[N_ALLOC_CPU], rc + score_cpu,
                                     as_f64(n[N_RCP_CPU]), n[N_ALLOC_MEM], rm + p.req_mem, as_f64(n[N_RCP_MEM]));
        return;
    }
    int64_t T[2] = {0, 0}, U[2] = {0, 0};
#pragma unroll
    for (uint32_t z = 0; z < (uint32_t)MAX_ZONES; z++) {
        if (z >= Z || (al[0][z] == 0 && al[1][z] == 0)) continue;
        for (int r = 0; r < 2; r++) {
            T[r] += xz.tot[r][z];
            U[r] += xz.used[r][z];
        }
    }
    b.s_numa = numa_score_q(most, c.numa_w_cpu, c.numa_w_mem, T[0], (bp ? bind_cpu : U[0]) + score_cpu, T[1],
                            U[1] + p.req_mem);
}

// ---- SingleNUMANode records on the fast-base path (storage class 1) --------------------------------------
// What DeviceShare brings to the topology manager of a fast pod (no pod NUMA policy, no cpuset) on a SingleNUMANode
// record off reservation views depends on the record and the pod's GPU request class only; k_gpu_zone_sum packs it
// per (record, class) so the fast-base kernels merge it into the class-1 zone walk (fast_eval<.., GZ>):
//   GZ_FAIL    the provider fails (its status stands: the pair is infeasible);
//   GZ_NOPREF  no GPU with a NUMA node: its single hint is the preferred nil affinity;
//   GZ_NODEV   no Device object: DeviceShare is no provider (its Filter / Score as without NUMA);
//   bits 4-7   the zones z whose hint {z} is in the list and preferred (what filterSingleNumaHints keeps);
//   bits 8-11  the zones whose hint {z} scores 500;
//   bits 12-15 the zones z under whose affinity {z} the allocation succeeds (allocateResources);
//   bits 16+8z DeviceShare's Score under the affinity {z} (0..100).
constexpr uint64_t GZ_FAIL = 1, GZ_NOPREF = 2, GZ_NODEV = 4;

__device__ __forceinline__ uint64_t gpu_zone_sum(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                                 const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d, const PodX& x) {
    const int32_t D = (int32_t)n[N_DEV_MINORS];
    if (D < 0) return GZ_NOPREF | GZ_NODEV;
    GpuHints gh;
    if (gpu_numa_hints(c, e, n, zr, d, nullptr, x, false, gh)) return GZ_FAIL;
    uint64_t w = 0;
    if (gh.set == (1u << NUMA_NIL_K)) {
        w |= GZ_NOPREF;
    } else {
        for (uint32_t l = gh.set; l; l &= l - 1u) {
            const uint32_t t = (uint32_t)(__ffs(l) - 1);
            const uint32_t m = (uint32_t)(gh.masks >> (4 * t)) & 15u;
            if (popc(m) != 1) continue;
            const uint32_t z = (uint32_t)(__ffs(m) - 1);
            w |= ((gh.pref >> t) & 1u) ? (uint64_t)1 << (4 + z) : 0ull;
            w |= ((gh.s500 >> t) & 1u) ? (uint64_t)1 << (8 + z) : 0ull;
        }
    }
    const uint32_t Z = ((uint32_t)n[N_FLAGS] >> F_NUMA_ZONES_SHIFT) & 15u;
    for (uint32_t z = 0; z < Z && z < (uint32_t)MAX_ZONES; z++) {
        uint32_t minors;
        if (gpu_alloc_site(c, e, n, zr, d, nullptr, x, false, 1u << z, false, minors)) continue;
        w |= (uint64_t)1 << (12 + z);
        w |= (uint64_t)((uint32_t)dev_score_tab_numa(c, d, nullptr, D, zr->dev_numa, x, 1u << z) & 0xFFu) << (16 + 8 * z);
    }
    return w;
}

// ---- one pair with every plugin ---------------------------------------------------------------------

struct PairX {
    uint32_t status;
    int32_t zone;
    int64_t s_nrf, s_la, s_numa, s_dev, s_rsv, order;
    int32_t nom;  // the nominated reservation (index into e.infos), -1 = none
};

// SCORE = false (statistics pass): status, raw DeviceShare score and the nominated reservation only;
// the NodeResourcesFit / LoadAware / NodeNUMAResource scores stay 0.
// dcls: the pod's GPU request class; with the batch's DevSum table (e.dsum) the DeviceShare Filter / Score of a
// pair off a reservation view read the record's tabulated allocator outcome instead of running the allocator.
template <bool EXACT, bool TOPO = true, bool SCORE = true>
__device__ __forceinline__ PairX eval_pair_ext(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                               const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d,
                                               uint32_t rec, const PodV& p, const PodX& x, uint32_t qst,
                                               uint32_t dcls = (uint32_t)DEV_CLASSES) {
    PairX o;
    o.status = 0;
    o.zone = -1;
    o.nom = -1;
    o.s_nrf = o.s_la = o.s_numa = o.s_dev = o.s_rsv = o.order = 0;
    if (qst) {  // ElasticQuota PreFilter rejected the pod: no node is evaluated
        o.status = qst;
        return o;
    }
    const RsvView* v = nullptr;
    if ((c.plugins & KG_PLUGIN_RSV) && x.cls >= 0 && x.cls < RSV_MAX_CLASSES &&
        (((uint64_t)n[N_RSV_CLASSES] >> x.cls) & 1ull))
        v = find_view(e, x.cls, rec, n);
    PairOut b;
    if (v) {
        Over ov;
#pragma unroll
        for (int k = 0; k < RSV_R; k++) ov.req[k] = v->req[k];
        ov.nz_cpu = v->nz_cpu;
        ov.nz_mem = v->nz_mem;
        ov.num_pods = v->num_pods;
        // NodeNUMAResource's restore keeps only reservations holding a NUMA / cpuset allocation
        // (nodenumaresource/reservation.go:188-270); kg_rsv_info describes none, so the plugin runs on the node's
        // zones with the view's NodeInfo
        b = eval_pair<EXACT, true, TOPO, SCORE>(c, n, zr, p, &ov);
    } else {
        b = eval_pair<EXACT, false, TOPO, SCORE>(c, n, zr, p);
    }
    // a GPU pod on a node with a Device object: DeviceShare is a NUMA hint provider there, at the pair's site
    // (its reservation view, if any)
    bool dev_done = false;
    uint32_t dev_mask = 0;
    if ((c.plugins & KG_PLUGIN_NUMA) && (c.plugins & KG_PLUGIN_DEV) && x.dcount > 0 && n[N_DEV_MINORS] >= 0)
        numa_gpu_eval<EXACT, SCORE>(c, e, n, zr, d, v, p, x, b, dev_done, dev_mask);
    uint32_t st = b.status;
    int64_t dev_raw = 0;
    const bool dev_view = (c.plugins & KG_PLUGIN_DEV) && v && x.dcount > 0;
    if (c.plugins & KG_PLUGIN_DEV) {
        if (dev_done) {  // the topology manager stored an affinity: DeviceShare's Filter passes
        } else {
            uint32_t ds;
            if (dev_view)
                ds = dev_filter_view(c, e, n, zr, d, *v, x, (p.flags & KG_POD_RSV_REQUIRED) != 0, rec, dcls);
            else if (e.dsum && dcls < (uint32_t)DEV_CLASSES)
                ds = dev_eval_sum(c, e, n, zr, d, e.dsum + rec, x, dcls, dev_raw);
            else
                ds = dev_eval(c, e, n, zr, d, x, dev_raw);
            // NodeNUMAResource already failed with a DeviceShare reason: one reason code
            st |= (b.status & KG_ST_DEV_MASK) ? (ds & ~(uint32_t)KG_ST_DEV_MASK) : ds;
        }
    }
    RsvPod q;
    if (c.plugins & KG_PLUGIN_RSV) {
        q = rsv_pod(p);
        st |= rsv_filter(q, n, v, e.infos, c.rsv_ign);
    }
    o.status = st;
    o.s_nrf = b.s_nrf;
    o.s_la = b.s_la;
    o.s_numa = (st & (KG_ST_NUMA_MASK | KG_ST_UNSUPPORTED)) ? 0 : b.s_numa;
    if (st) return o;
    o.zone = b.zone;
    o.s_dev = dev_raw;
    int nom = -1;
    if (v) o.s_rsv = rsv_nominate_score(q, n, *v, e.infos, o.order, c.rsv_ign, nom);
    if (v && nom >= 0) o.nom = (int32_t)(v->first + (uint32_t)nom);
    if (dev_view || dev_done)
        // Score (scoring.go:45-104): with a nominated reservation, its table, or 0 when it reserves no GPU
        // (scoreWithNominatedReservation, reservation.go:492-520); without one, the view's base table; off views
        // the node's devices; under the stored NUMA affinity
        o.s_dev = gpu_score_site(c, e, n, zr, d, v, x, dev_done ? dev_mask : 0u, nom);
    return o;
}

// ---- Reservation.Reserve (reservation/plugin.go:1295-1408) -------------------------------------------------------
// The pod (already in the node's NodeInfo: apply_assume) joins its nominated reservation (index nom into e.infos, -1 =
// none): AddAssignedPod adds m = Mask(requests, ResourceNames) to the reservation's Allocated
// (reservation_info.go:490-500), and the next cycle's restore (transformer.go:740-935) sees it: the record (the view
// of pods matching nothing) and the views where the reservation is not matched give back m (its unmatched correction
// grows) and the change of its NonZeroRequested correction (present keys count their value, a missing key the
// 100m / 200Mi default); the views where it is matched keep the pod and count m in rAllocated; every view of the node
// counts one more pod. Oracle: kg_oracle.c rsv_reserve. Called by one lane; the node's views are its own.
__device__ __forceinline__ void rsv_nonzero_dev(const int64_t* a, uint32_t keys, int64_t& c0, int64_t& c1) {
    c0 = (keys & 1u) ? a[0] : 100;
    c1 = (keys & 2u) ? a[1] : 200ll * 1024 * 1024;
}

__device__ __forceinline__ void rsv_reserve_dev(const ExtDev& e, int64_t* n, ZoneRec* zr, uint32_t rec, const PodV& p,
                                                int32_t nom) {
    const int64_t preq[RSV_R] = {p.req_cpu, p.req_mem, p.req_eph, p.sc0, p.sc1};
    int64_t m[RSV_R] = {0, 0, 0, 0, 0};
    int64_t d0 = 0, d1 = 0;
    uint32_t rid = 0xFFFFFFFFu, keys1 = 0;
    RsvInfo* infos = const_cast<RsvInfo*>(e.infos);
    RsvView* views = const_cast<RsvView*>(e.views);
    if (nom >= 0) {
        const RsvInfo& r = infos[nom];
        rid = r.rid;
#pragma unroll
        for (int k = 0; k < RSV_R; k++) m[k] = ((r.names >> k) & 1u) ? preq[k] : 0;
        const uint32_t keys_m = (((p.flags & KG_POD_HAS_CPU) && (r.names & 1u)) ? 1u : 0u) |
                                (((p.flags & KG_POD_HAS_MEM) && (r.names & 2u)) ? 2u : 0u);
        int64_t a1[RSV_R], c00 = 0, c01 = 0, c10, c11;
        if (r.allocated_pods > 0) rsv_nonzero_dev(r.allocated, r.allocated_keys, c00, c01);
#pragma unroll
        for (int k = 0; k < RSV_R; k++) a1[k] = r.allocated[k] + m[k];
        keys1 = r.allocated_keys | keys_m;
        rsv_nonzero_dev(a1, keys1, c10, c11);
        d0 = c10 - c00;
        d1 = c11 - c01;
        n[N_REQ_CPU] -= m[0];
        n[N_REQ_MEM] -= m[1];
        n[N_REQ_EPH] -= m[2];
        n[N_SC_REQ0] -= m[3];
        n[N_SC_REQ1] -= m[4];
        n[N_NZ_CPU] -= d0;
        n[N_NZ_MEM] -= d1;
        derive_node(*reinterpret_cast<NodeRec*>(n), *zr);
    }
    const uint64_t mask = (uint64_t)n[N_RSV_CLASSES];
    for (uint64_t l = mask; l; l &= l - 1ull) {
        const int32_t cls = (int32_t)(__ffsll((unsigned long long)l) - 1);
        const RsvView* cv = find_view(e, cls, rec, n);
        if (!cv) continue;
        RsvView& v = views[cv - e.views];
        bool matched = false;
        for (uint32_t t = v.first; t < v.first + v.count && rid != 0xFFFFFFFFu; t++) matched = matched || infos[t].rid == rid;
#pragma unroll
        for (int k = 0; k < RSV_R; k++) {
            const int64_t d = preq[k] - (matched ? 0 : m[k]);
            v.req[k] += d;
            v.pod_requested[k] += d;
            if (matched) v.r_allocated[k] += m[k];
        }
        v.nz_cpu += p.nz_cpu - (matched ? 0 : d0);
        v.nz_mem += p.nz_mem - (matched ? 0 : d1);
        v.num_pods += 1;
        if (!matched) continue;
        for (uint32_t t = v.first; t < v.first + v.count; t++) {
            RsvInfo& r = infos[t];
            if (r.rid != rid) continue;
#pragma unroll
            for (int k = 0; k < RSV_R; k++) r.allocated[k] += m[k];
            r.allocated_pods += 1;
            r.allocated_keys = keys1;
        }
    }
}

// ---- Reservation.Unreserve (reservation/plugin.go:1409-1460) ------------------------------------------------------
// The pod leaves the reservation it joined (forgetPods -> RemoveAssignedPod, reservation_info.go:502-514: Allocated -=
// Mask(requests, ResourceNames) with a non-negative result, one assigned pod less; keys stay) and the node's views as
// the next restore (transformer.go:740-935) builds them: the unmatched correction of the reservation is its Allocated
// while it has pods and nothing after the last one (restoreUnmatchedReservations :891-903), so the record and the views
// that do not match it change by the pod and the change of that correction; the views that match it lose the pod and
// count the new Allocated in rAllocated; every view counts one pod less. rid: the reservation's kg_rsv_info.rid (found
// among the node's views; none: the pod joined no reservation). The NodeInfo part is apply_assume(-1)'s. One lane.
__device__ __forceinline__ void rsv_unreserve_dev(const ExtDev& e, int64_t* n, ZoneRec* zr, uint32_t rec, const PodV& p,
                                                  int32_t rid_in) {
    const int64_t preq[RSV_R] = {p.req_cpu, p.req_mem, p.req_eph, p.sc0, p.sc1};
    RsvInfo* infos = const_cast<RsvInfo*>(e.infos);
    RsvView* views = const_cast<RsvView*>(e.views);
    const uint64_t cmask = (uint64_t)n[N_RSV_CLASSES];
    const uint32_t rid = rid_in < 0 ? 0xFFFFFFFFu : (uint32_t)rid_in;
    // the reservation as the node's views hold it (every copy agrees)
    const RsvInfo* r = nullptr;
    for (uint64_t l = cmask; l && rid != 0xFFFFFFFFu && !r; l &= l - 1ull) {
        const RsvView* cv = find_view(e, (int32_t)(__ffsll((unsigned long long)l) - 1), rec, n);
        if (!cv) continue;
        for (uint32_t t = cv->first; t < cv->first + cv->count; t++)
            if (infos[t].rid == rid) {
                r = &infos[t];
                break;
            }
    }
    int64_t a1[RSV_R] = {0, 0, 0, 0, 0}, dc[RSV_R] = {0, 0, 0, 0, 0}, dra[RSV_R] = {0, 0, 0, 0, 0};
    int64_t dn0 = 0, dn1 = 0, p1 = 0;
    if (r) {
        const int64_t p0 = r->allocated_pods;
        p1 = p0 > 0 ? p0 - 1 : 0;
        int64_t n00 = 0, n01 = 0, n10 = 0, n11 = 0;
#pragma unroll
        for (int k = 0; k < RSV_R; k++) {
            const int64_t m = ((r->names >> k) & 1u) ? preq[k] : 0;
            a1[k] = r->allocated[k] - m < 0 ? 0 : r->allocated[k] - m;
            dc[k] = (p1 > 0 ? a1[k] : 0) - (p0 > 0 ? r->allocated[k] : 0);
            dra[k] = a1[k] - r->allocated[k];
        }
        if (p0 > 0) rsv_nonzero_dev(r->allocated, r->allocated_keys, n00, n01);
        if (p1 > 0) rsv_nonzero_dev(a1, r->allocated_keys, n10, n11);
        dn0 = n10 - n00;
        dn1 = n11 - n01;
        n[N_REQ_CPU] -= dc[0];
        n[N_REQ_MEM] -= dc[1];
        n[N_REQ_EPH] -= dc[2];
        n[N_SC_REQ0] -= dc[3];
        n[N_SC_REQ1] -= dc[4];
        n[N_NZ_CPU] -= dn0;
        n[N_NZ_MEM] -= dn1;
        derive_node(*reinterpret_cast<NodeRec*>(n), *zr);
    }
    for (uint64_t l = cmask; l; l &= l - 1ull) {
        const RsvView* cv = find_view(e, (int32_t)(__ffsll((unsigned long long)l) - 1), rec, n);
        if (!cv) continue;
        RsvView& v = views[cv - e.views];
        bool matched = false;
        for (uint32_t t = v.first; t < v.first + v.count && r; t++) matched = matched || infos[t].rid == rid;
#pragma unroll
        for (int k = 0; k < RSV_R; k++) {
            const int64_t d = -preq[k] - (matched ? 0 : dc[k]);
            v.req[k] += d;
            v.pod_requested[k] += d;
            if (matched) v.r_allocated[k] += dra[k];
        }
        v.nz_cpu += -p.nz_cpu - (matched ? 0 : dn0);
        v.nz_mem += -p.nz_mem - (matched ? 0 : dn1);
        v.num_pods -= 1;
    }
    if (!r) return;
    // every copy of the reservation (after the views: r points into infos)
    for (uint64_t l = cmask; l; l &= l - 1ull) {
        const RsvView* cv = find_view(e, (int32_t)(__ffsll((unsigned long long)l) - 1), rec, n);
        if (!cv) continue;
        for (uint32_t t = cv->first; t < cv->first + cv->count; t++) {
            RsvInfo& x = infos[t];
            if (x.rid != rid || x.allocated_pods != p1 + 1) continue;
#pragma unroll
            for (int k = 0; k < RSV_R; k++) x.allocated[k] = a1[k];
            x.allocated_pods = p1;
        }
    }
}

// ---- DeviceShare restore of reservations that hold GPUs (deviceshare/reservation.go:139-198,278-380) ---------------
// A device table is [DEV_R][DEV_MINORS] with a minor mask (a deviceResources map holds a minor or not); host restatement:
// decode.dev_effective / dev_reusable / reservation_restore.

__device__ __forceinline__ uint32_t dtab_mask(const int64_t (&t)[DEV_R][DEV_MINORS]) {
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < DEV_MINORS; k++) m |= (t[0][k] != 0 || t[1][k] != 0 || t[2][k] != 0) ? 1u << k : 0u;
    return m;
}

// nodeDevice.calcFreeWithPreemptible + filter (device_cache.go:322-410): a minor holding preemptible resources frees
// them from its used (never below zero); if any such minor then has something left, those minors take that remainder
// and the others keep their free; allocating from a reservation's required resources (req != nullptr) keeps only the
// required minors, each capped by them. Minors outside have total and free 0. free = max(0, total - used).
__device__ inline void dev_effective(const DevRec& node, const int64_t (&used)[DEV_R][DEV_MINORS],
                                     const int64_t (&pre)[DEV_R][DEV_MINORS], uint32_t pre_mask,
                                     const int64_t (*req)[DEV_MINORS], uint32_t req_mask, DevRec& out) {
    bool merged[DEV_MINORS];
    int64_t rem[DEV_R][DEV_MINORS];
    bool any = false;
    for (int m = 0; m < DEV_MINORS; m++) {
        bool nz = false;
        for (int r = 0; r < DEV_R; r++) {
            const int64_t u = max(used[r][m] - pre[r][m], (int64_t)0);
            rem[r][m] = max(node.total[r][m] - u, (int64_t)0);
            nz |= rem[r][m] != 0;
        }
        merged[m] = ((pre_mask >> m) & 1u) && nz;
        any |= merged[m];
    }
    for (int m = 0; m < DEV_MINORS; m++)
        for (int r = 0; r < DEV_R; r++) {
            int64_t f = max(node.total[r][m] - used[r][m], (int64_t)0);
            if (any && merged[m]) f = rem[r][m];
            int64_t t = node.total[r][m];
            if (req) {
                if ((req_mask >> m) & 1u) f = min(f, req[r][m]);
                else f = 0, t = 0;
            }
            out.total[r][m] = t;
            out.free_[r][m] = f;
        }
}

__device__ __forceinline__ const GpuRawRsv* raw_rsv(const ExtDev& e, const GpuRawNode& N, uint32_t rid) {
    for (uint32_t r = N.first; r < N.first + N.count; r++)
        if (e.grsv[r].rid == rid) return &e.grsv[r];
    return nullptr;
}

// the parts of one reservation (dev_reservation_parts): allocatable (alloc, its mask), allocated masked by it, remained =
// alloc - allocated (negative kept) and the used part max(allocated, 0)
__device__ __forceinline__ void raw_parts(const GpuRawRsv& R, int64_t (&al)[DEV_R][DEV_MINORS], int64_t (&rm)[DEV_R][DEV_MINORS],
                                          int64_t (&up)[DEV_R][DEV_MINORS], uint32_t& amask) {
    amask = dtab_mask(R.alloc);
    for (int r = 0; r < DEV_R; r++)
        for (int m = 0; m < DEV_MINORS; m++) {
            al[r][m] = ((amask >> m) & 1u) ? R.allocated[r][m] : 0;
            rm[r][m] = R.alloc[r][m] - al[r][m];
            up[r][m] = max(al[r][m], (int64_t)0);
        }
}

// RestoreReservation + dev_reusable of every view of record `rec` and the record's own free (pods matching nothing see
// every GPU reservation with assigned pods as unmatched), from the raw inputs: rewrites d->free_ and the views' base and
// reservation tables (e.rdev). One lane.
__device__ inline void gpu_restore_rebuild(const ExtDev& e, const int64_t* __restrict__ n, uint32_t rec, DevRec* d) {
    const GpuRawNode& N = e.gnodes[e.graw[rec]];
    DevRec* rdev = const_cast<DevRec*>(e.rdev);
    int64_t pre[DEV_R][DEV_MINORS], al[DEV_R][DEV_MINORS], rm[DEV_R][DEV_MINORS], up[DEV_R][DEV_MINORS];
    uint32_t am = 0;
    {  // the record
        uint32_t pm = 0;
        for (int r = 0; r < DEV_R; r++)
            for (int m = 0; m < DEV_MINORS; m++) pre[r][m] = 0;
        for (uint32_t x = N.first; x < N.first + N.count; x++) {
            if (e.grsv[x].pods <= 0) continue;
            raw_parts(e.grsv[x], al, rm, up, am);
            for (int r = 0; r < DEV_R; r++)
                for (int m = 0; m < DEV_MINORS; m++) pre[r][m] += up[r][m];
            pm |= dtab_mask(up);
        }
        DevRec out;
        dev_effective(*d, N.used, pre, pm, nullptr, 0u, out);
        for (int r = 0; r < DEV_R; r++)
            for (int m = 0; m < DEV_MINORS; m++) d->free_[r][m] = out.free_[r][m];
    }
    const uint64_t cmask = (uint64_t)n[N_RSV_CLASSES];
    for (uint64_t l = cmask; l; l &= l - 1ull) {
        const RsvView* v = find_view(e, (int32_t)(__ffsll((unsigned long long)l) - 1), rec, n);
        if (!v || v->dev_base < 0) continue;
        // matched GPU reservations of the view (by rid), the others with pods are unmatched
        int64_t uu[DEV_R][DEV_MINORS], ma[DEV_R][DEV_MINORS], mal[DEV_R][DEV_MINORS];
        uint32_t uum = 0, mam = 0, malm = 0;
        for (int r = 0; r < DEV_R; r++)
            for (int m = 0; m < DEV_MINORS; m++) uu[r][m] = ma[r][m] = mal[r][m] = 0;
        for (uint32_t x = N.first; x < N.first + N.count; x++) {
            const GpuRawRsv& R = e.grsv[x];
            bool matched = false;
            for (uint32_t t = v->first; t < v->first + v->count; t++) matched = matched || (e.infos[t].dev >= 0 && e.infos[t].rid == R.rid);
            raw_parts(R, al, rm, up, am);
            if (matched) {
                for (int r = 0; r < DEV_R; r++)
                    for (int m = 0; m < DEV_MINORS; m++) ma[r][m] += al[r][m], mal[r][m] += R.alloc[r][m];
                mam |= dtab_mask(al);
                malm |= am;
            } else if (R.pods > 0) {
                for (int r = 0; r < DEV_R; r++)
                    for (int m = 0; m < DEV_MINORS; m++) uu[r][m] += up[r][m];
                uum |= dtab_mask(up);
            }
        }
        // outside the reservations (plugin.go:417-419): unmatched used + matched allocatable
        for (int r = 0; r < DEV_R; r++)
            for (int m = 0; m < DEV_MINORS; m++) pre[r][m] = uu[r][m] + mal[r][m];
        dev_effective(*d, N.used, pre, uum | malm, nullptr, 0u, rdev[v->dev_base]);
        // each matched reservation (tryAllocateFromReusable :344-410): unmatched used + matched allocated + its remained;
        // the Restricted policy only its minors, capped by calcRequiredDeviceResources (:436-455)
        for (uint32_t t = v->first; t < v->first + v->count; t++) {
            const RsvInfo& I = e.infos[t];
            if (I.dev < 0) continue;
            const GpuRawRsv* R = raw_rsv(e, N, I.rid);
            if (!R) continue;
            raw_parts(*R, al, rm, up, am);
            const uint32_t rmask = dtab_mask(rm);
            for (int r = 0; r < DEV_R; r++)
                for (int m = 0; m < DEV_MINORS; m++) pre[r][m] = uu[r][m] + ma[r][m] + rm[r][m];
            const uint32_t pm = uum | mam | rmask;
            if (R->policy == KG_RSV_RESTRICTED) {
                int64_t req[DEV_R][DEV_MINORS];
                for (int r = 0; r < DEV_R; r++)
                    for (int m = 0; m < DEV_MINORS; m++) req[r][m] = ((rmask >> m) & 1u) ? rm[r][m] : 0;
                const uint32_t qm = (rmask ? rmask : am) & am;
                dev_effective(*d, N.used, pre, pm, req, qm, rdev[I.dev]);
            } else {
                dev_effective(*d, N.used, pre, pm, nullptr, 0u, rdev[I.dev]);
            }
        }
    }
}

// the pod's reservation view on record rec (nullptr: none)
__device__ __forceinline__ const RsvView* pod_view(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                                   uint32_t rec, const PodX& x) {
    if (!(c.plugins & KG_PLUGIN_RSV) || !e.views || x.cls < 0 || x.cls >= RSV_MAX_CLASSES ||
        !(((uint64_t)n[N_RSV_CLASSES] >> x.cls) & 1ull))
        return nullptr;
    return find_view(e, x.cls, rec, n);
}

// DeviceShare's allocate at Reserve (plugin.go:573-637): from the nominated reservation's table when it holds GPUs
// (allocateWithNominated -> tryAllocateFromReusable, not required), else or on its failure outside the reservations
// (the view's base table; off views the node's devices), under the pair's NUMA affinity. The minors taken (0 = none).
__device__ __forceinline__ uint32_t dev_choose_site(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n,
                                                    const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d,
                                                    const RsvView* v, int32_t nom, const PodX& x, int32_t zone) {
    const int32_t D = (int32_t)n[N_DEV_MINORS];
    if (x.dcount == 0 || D <= 0) return 0;
    const uint32_t numa = zone_affinity(zone);
    if (v && nom >= 0 && e.infos[nom].dev >= 0) {
        // the reservation's reserved minors first (tryAllocateFromReusable's preferred set)
        const GpuAlloc a = gpu_alloc_tab_numa(c, e, d, e.rdev + e.infos[nom].dev, D, zr, x, numa, true, e.infos[nom].dev_pref);
        if (!a.code) return a.mask;
    }
    const DevRec* tab = (v && v->dev_base >= 0) ? e.rdev + v->dev_base : nullptr;
    const GpuAlloc a = gpu_alloc_tab_numa(c, e, d, tab, D, zr, x, numa, true);
    return a.code ? 0u : a.mask;
}

// A GPU pod's Reserve (sign 1) / Unreserve (-1) of `mask` on a record with GPU-holding reservations: the node's used
// (updateCacheUsed), the reservation the pod joins / leaves (rid, -1 = none: its assigned pods' allocations on its own
// minors, appendAllocatedByHints, and its pod count), then the restore tables. Instead of dev_apply. One lane.
__device__ inline void gpu_restore_apply(const ExtDev& e, const int64_t* __restrict__ n, uint32_t rec, DevRec* d,
                                         uint32_t mask, const PodX& x, int32_t rid, int64_t sign) {
    GpuRawNode& N = e.gnodes[e.graw[rec]];
    GpuRawRsv* R = rid >= 0 ? const_cast<GpuRawRsv*>(raw_rsv(e, N, (uint32_t)rid)) : nullptr;
    const uint32_t hints = R ? dtab_mask(R->alloc) : 0u;
    for (int m = 0; m < DEV_MINORS; m++) {
        if (!((mask >> m) & 1u)) continue;
        int64_t a[DEV_R];
        dev_alloc_of(x, d->total[2][m], a);
        for (int r = 0; r < DEV_R; r++) {
            N.used[r][m] = sign > 0 ? N.used[r][m] + a[r] : max(N.used[r][m] - a[r], (int64_t)0);
            if (R && ((hints >> m) & 1u))
                R->allocated[r][m] = sign > 0 ? R->allocated[r][m] + a[r] : max(R->allocated[r][m] - a[r], (int64_t)0);
        }
    }
    if (R) R->pods = max(R->pods + sign, (int64_t)0);
    gpu_restore_rebuild(e, n, rec, d);
}

// DeviceShare + Reservation Reserve bookkeeping of a placed pod with the minors `mask` it took (mask from
// dev_choose_site) and its nominated reservation nom (index into e.infos, -1 = none): on a record with GPU-holding
// reservations the raw inputs and restore tables (gpu_restore_apply, every pod: the reservation's assigned pods count
// too), else the node's minors. sign -1: the Unreserve (rid of the reservation left). One lane.
__device__ __forceinline__ void dev_reserve_apply(const KCfg& c, const ExtDev& e, const int64_t* __restrict__ n, uint32_t rec,
                                                  DevRec* d, uint32_t mask, const PodX& x, int32_t rid, int64_t sign) {
    if (!(c.plugins & KG_PLUGIN_DEV) || !d) return;
    if (e.graw && e.graw[rec] >= 0) {
        gpu_restore_apply(e, n, rec, d, x.dcount > 0 ? mask : 0u, x, rid, sign);
        return;
    }
    if (x.dcount > 0) dev_apply(d, mask, x, sign);
}

// per-pod NormalizeScore inputs: max DeviceShare raw score, max nominated Reservation score, and the
// preferred node key ((order + 2^31) << 32 | snapshot index, minimum; ~0 = none)
constexpr uint64_t PREF_NONE = ~0ull;

__device__ __forceinline__ uint64_t pref_key(int64_t order, uint32_t gidx) {
    return ((uint64_t)(uint32_t)(order + 0x80000000ll) << 32) | gidx;
}

__device__ __forceinline__ int64_t norm100(int64_t s, int64_t mx) { return mx == 0 ? s : qdiv(s * 100, mx); }

// A general pair's selection inputs as the statistics pass stores them (ExtDev::xpairs): infeasible, infeasible with
// KG_ST_UNSUPPORTED, "evaluate again" (a value outside the packing), or bit 63 | base total << 24 | raw DeviceShare score
// << 12 | nominated-reservation score (the weighted NodeResourcesFit / LoadAware / NodeNUMAResource part is below 2^31:
// weights <= 2^20, scores <= 100).
constexpr uint64_t XPAIR_INFEASIBLE = 0, XPAIR_LIVE = 1, XPAIR_UNSUP = 2;

__device__ __forceinline__ uint64_t xpair_pack(const KCfg& c, const PairX& r) {
    if (r.status) return (r.status & KG_ST_UNSUPPORTED) ? XPAIR_UNSUP : XPAIR_INFEASIBLE;
    const int64_t base = (int64_t)c.w_nrf * r.s_nrf + (int64_t)c.w_la * r.s_la + (int64_t)c.w_numa * r.s_numa;
    if (base < 0 || base >= (1ll << 31) || r.s_dev < 0 || r.s_dev > 4095 || r.s_rsv < 0 || r.s_rsv > 4095) return XPAIR_LIVE;
    return (1ull << 63) | ((uint64_t)base << 24) | ((uint64_t)r.s_dev << 12) | (uint64_t)r.s_rsv;
}

__device__ __forceinline__ int64_t total_ext(const KCfg& c, const PairX& o, uint32_t gidx, uint32_t dev_max,
                                             uint32_t rsv_max, uint64_t pref) {
    const bool has_pref = pref != PREF_NONE;
    const int64_t rsv = (has_pref && (uint32_t)pref == gidx) ? 1000 : o.s_rsv;
    const int64_t rmax = has_pref ? 1000 : (int64_t)rsv_max;
    return (int64_t)c.w_nrf * o.s_nrf + (int64_t)c.w_la * o.s_la + (int64_t)c.w_numa * o.s_numa +
           (int64_t)c.w_dev * norm100(o.s_dev, dev_max) + (int64_t)c.w_rsv * norm100(rsv, rmax);
}

// total_ext of a packed pair (xpair_pack, bit 63 set)
__device__ __forceinline__ int64_t total_xpair(const KCfg& c, uint64_t x, uint32_t gidx, uint32_t dev_max, uint32_t rsv_max,
                                               uint64_t pref) {
    const bool has_pref = pref != PREF_NONE;
    const int64_t s_rsv = (int64_t)(x & 0xFFFull), s_dev = (int64_t)((x >> 12) & 0xFFFull);
    const int64_t rsv = (has_pref && (uint32_t)pref == gidx) ? 1000 : s_rsv;
    const int64_t rmax = has_pref ? 1000 : (int64_t)rsv_max;
    return (int64_t)((x >> 24) & 0x7FFFFFFFull) + (int64_t)c.w_dev * norm100(s_dev, dev_max) +
           (int64_t)c.w_rsv * norm100(rsv, rmax);
}

}  // namespace kg
