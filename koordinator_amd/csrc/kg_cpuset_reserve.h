// kg_cpuset_reserve.h — NodeNUMAResource Reserve / Unreserve of a cpuset-binding pod on the device (one workgroup of
// one wave): resourceManager.Allocate + Update (nodenumaresource/plugin.go:585-635, resource_manager.go:197-262,
// 357-463, node_allocation.go:111-143) and Release (plugin.go:700-720, resource_manager.go:478-483,
// node_allocation.go:164-200). Used by k_cpuset_reserve (kg_assume*, the replays) and by the cooperative batch cycle.
#pragma once
#include "kg_cpuset.h"
#include "kg_eval.h"

namespace kg {

// LDS of one cpuset Reserve: the node's CPU topology, the accumulator, the node's allocation and the broadcast words.
struct CpusetLds {
    kg_cpu_topo st;
    CpuAccLds acc;
    kg_cpu_alloc sa;
    uint64_t avail[4];
    int32_t zone;
};

// getCPUBindPolicy (util.go:101-138): the pod binds CPUs on this record (its own policy, or the node's policy with a
// cpu request) and the record has a CPU topology.
__device__ __forceinline__ bool cpuset_bound_dev(const ZoneRec& z, uint32_t pf, int64_t req_cpu) {
    if (z.cpu_topo < 0 || (pf & KG_POD_NUMA_SKIP)) return false;
    const uint32_t node_bind = (z.cpu_meta >> CPU_META_BIND_SHIFT) & 3u;
    return (pf & KG_POD_CPU_BIND) || (node_bind != KG_NODE_CPU_BIND_NONE && req_cpu != 0);
}

// NUMANodeSharedStatus counts after a cpuset allocation (sign +1) or its release (-1) over the NUMA nodes `used` (bit per
// node): the pod's uid joins / leaves singleNUMANode of its one node, or sharedNode of each of several
// (node_allocation.go:111-143,164-200); the 2-bit statuses follow (NUMANodeSharedStatus :60-68).
__device__ __forceinline__ void cpuset_zone_count(ZoneRec& z, uint32_t used, int sign) {
    const bool multi = (used & (used - 1)) != 0;
    for (uint32_t q = 0; q < (uint32_t)MAX_ZONES; q++) {
        if (!((used >> q) & 1u)) continue;
        uint8_t& c = multi ? z.cz_shared[q] : z.cz_single[q];
        const int v = (int)c + sign;  // saturating at 0 and 255, as the host's zone_pods and the oracle count
        c = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
    z.status = zone_status_of_counts(z);
}

// The cpuset Reserve of pod `pod` on record `rec` under the pair's zone code `zone` (not a failing one); every lane of
// the workgroup calls it with the same arguments. Under a NUMA affinity allocateCPUSet takes per allocated NUMA node
// (resource_manager.go:391-429) and the NUMA split with the CPUs is recorded here, before the take changes the counts
// it trims with (apply_assume leaves it, cpuset_numa_reserve). Runs before the Reserve of the NodeInfo columns
// (apply_assume, which re-derives the record). 0: the CPUs entered the node's allocation (RefCount++, the pod's
// exclusive policy; taken[0, 4), if given, receives them and taken[4, 12) the NUMA split under an affinity), 1: Allocate
// fails (ErrNotEnoughCPUs), nothing applied.
__device__ inline int cpuset_reserve_wave(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones,
                                          kg_cpu_alloc* __restrict__ allocs, const kg_cpu_topo* __restrict__ topos,
                                          const PodsDev& pods, uint32_t pod, uint32_t rec, int32_t zone, CpusetLds& L,
                                          uint64_t* __restrict__ taken) {
    kg_cpu_topo& st = L.st;
    kg_cpu_alloc& sa = L.sa;
    const uint32_t pf = pods.flags[pod];
    const int64_t req_cpu = pods.req_cpu[pod];
    ZoneRec& z = zones[rec];
    int64_t* n = nodes[rec].v;
    const uint32_t node_bind = (z.cpu_meta >> CPU_META_BIND_SHIFT) & 3u;
    const uint32_t node_pol = ((uint32_t)n[N_FLAGS] >> F_NUMA_POLICY_SHIFT) & 15u, pod_pol = (pf >> 16) & 15u;
    const bool numa_pol = (pod_pol != KG_NUMA_NONE ? pod_pol : node_pol) != KG_NUMA_NONE;
    const uint32_t mask = numa_pol ? zone_affinity(zone) : 0u;  // the NUMA affinity of the Reserve (0: the whole node)
    const uint32_t* src = reinterpret_cast<const uint32_t*>(topos + z.cpu_topo);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&st);
    for (uint32_t k = threadIdx.x; k < sizeof(kg_cpu_topo) / 4; k += 64) dst[k] = src[k];
    const uint32_t* as = reinterpret_cast<const uint32_t*>(allocs + rec);
    uint32_t* ad = reinterpret_cast<uint32_t*>(&sa);
    for (uint32_t k = threadIdx.x; k < sizeof(kg_cpu_alloc) / 4; k += 64) ad[k] = as[k];
    __syncthreads();
    // getCPUBindPolicy (util.go:101-119): the pod's required policy, else the node's, else the preferred one
    const bool pod_req = (pf & KG_POD_CPU_REQUIRED) != 0;
    uint32_t bind = (pf >> KG_POD_CPU_POLICY_SHIFT) & 3u;
    bool required = pod_req;
    if (!pod_req && node_bind == KG_NODE_CPU_BIND_SPREAD_BY_PCPUS) bind = KG_CPU_BIND_SPREAD_BY_PCPUS, required = true;
    if (!pod_req && node_bind == KG_NODE_CPU_BIND_FULL_PCPUS_ONLY) bind = KG_CPU_BIND_FULL_PCPUS, required = true;
    const int max_ref = (int)(z.cpu_meta & 0xFFu);
    CpuTake q;
    for (int w = 0; w < 4; w++) q.avail[w] = q.preferred[w] = 0;
    // getAvailableCPUs, then filterCPUsByRequiredCPUBindPolicy for a required policy (lane 0)
    if (threadIdx.x == 0) {
        const int cpc = st.n_cores ? st.n_cpus / st.n_cores : 1;
        for (int c = 0; c < st.n_cpus; c++) {
            if (sa.ref[c] >= max_ref) continue;
            bool keep = true;
            if (required) {
                int cnt = 0, first = -1;
                for (int d = 0; d < st.n_cpus; d++)
                    if (st.core[d] == st.core[c] && sa.ref[d] < max_ref) {
                        cnt++;
                        if (first < 0) first = d;
                    }
                keep = bind == KG_CPU_BIND_FULL_PCPUS ? cnt == cpc : first == c;
            }
            if (keep) q.avail[c >> 6] |= 1ull << (c & 63);
        }
        for (int w = 0; w < 4; w++) L.avail[w] = q.avail[w];
    }
    __syncthreads();
    for (int w = 0; w < 4; w++) q.avail[w] = L.avail[w];
    q.needed = (int32_t)(req_cpu / 1000);
    q.max_ref = max_ref;
    q.bind = (int32_t)bind;
    q.excl = (int32_t)((pf >> KG_POD_CPU_EXCL_SHIFT) & 3u);
    q.strategy = (int32_t)((z.cpu_meta >> CPU_META_STRATEGY_SHIFT) & 1u);
    q.has_preferred = 0;
    uint64_t res[4] = {0, 0, 0, 0};
    int code = 0;
    int64_t al[2][MAX_ZONES];
    if (!mask) {
        code = cpuset_take(&st, &sa, q, &L.acc, res);
    } else {
        // the NUMA split with the CPUs (trimmed to the policy's CPUs, whole CPUs / cores per node) on the pre-take state,
        // then one take per allocated NUMA node of min(its CPUs, allocated cpu / 1000)
        const uint32_t Z = ((uint32_t)n[N_FLAGS] >> F_NUMA_ZONES_SHIFT) & 15u;
        NumaZ x;
        numa_load(&z, Z, x);
        const NumaBind nb = numa_bind_of(&z, required, bind, req_cpu);
        numa_bind_trim(x, nb);
        const PodV pv = load_pod(pods, pod);
        const int64_t req[2] = {pv.req_cpu, pv.req_mem};
        const bool has[2] = {(pf & KG_POD_HAS_CPU) != 0, (pf & KG_POD_HAS_MEM) != 0};
        code = (numa_split(x, mask, req, has, al, &nb) || numa_bind_check(nb, al[0], al[1], Z)) ? 1 : 0;
        for (uint32_t zq = 0; zq < (uint32_t)MAX_ZONES && code == 0; zq++) {
            if (zq >= Z || (al[0][zq] == 0 && al[1][zq] == 0)) continue;
            const int64_t k = min(nb.cnt[zq], al[0][zq] / 1000);
            if (k == 0) continue;
            CpuTake qz = q;
            for (int w = 0; w < 4; w++) qz.avail[w] = 0;
            for (int c = 0; c < st.n_cpus; c++)
                if (st.numa[c] == zq && ((q.avail[c >> 6] >> (c & 63)) & 1ull)) qz.avail[c >> 6] |= 1ull << (c & 63);
            qz.needed = (int32_t)k;
            uint64_t rz[4];
            code = cpuset_take(&st, &sa, qz, &L.acc, rz);
            __syncthreads();
            for (int w = 0; w < 4; w++) res[w] |= rz[w];
        }
    }
    __syncthreads();
    if (code != 0 || threadIdx.x != 0) return code;
    if (mask) {  // resourceManager.Update: the NUMA split enters the zones, each gets its allocation record
        for (int zq = 0; zq < MAX_ZONES; zq++) {
            z.cpu_used[zq] += al[0][zq];
            z.mem_used[zq] += al[1][zq];
            z.status |= (al[0][zq] | al[1][zq]) ? 1u << (ZONE_RECORD_SHIFT + zq) : 0u;
        }
    }
    kg_cpu_alloc& A = allocs[rec];
    uint32_t used = 0;  // NUMA nodes of the CPUs taken (addPodAllocation's usedNUMA)
    for (int c = 0; c < st.n_cpus; c++)
        if ((res[c >> 6] >> (c & 63)) & 1ull) {
            A.ref[c] = (uint8_t)(A.ref[c] + 1);
            A.excl[c] = (uint8_t)q.excl;
            used |= 1u << st.numa[c];
        }
    cpuset_zone_count(z, used, 1);
    cpu_counts(st, &A, max_ref, z);
    n[N_CPUSET] = 1000 * (int64_t)z.cpu_allocated;
    n[N_AMP_CPUSET] = z.amp_ratio > 1.0 ? (int64_t)ceil(__dmul_rn((double)n[N_CPUSET], z.amp_ratio)) : n[N_CPUSET];
    if (taken) {  // the record of the Reserve: the CPUs, then (under an affinity) the NUMA split it recorded
        for (int w = 0; w < 4; w++) taken[w] = res[w];
        for (int zq = 0; zq < MAX_ZONES && mask; zq++) {
            taken[4 + zq] = (uint64_t)al[0][zq];
            taken[4 + MAX_ZONES + zq] = (uint64_t)al[1][zq];
        }
    }
    return 0;
}

// NodeAllocation.release of a cpuset pod's CPUs (node_allocation.go:164-200; one lane): RefCount-- per CPU (a CPU at 0
// leaves allocatedCPUs with its exclusive policy), the pod leaves the NUMA nodes' single / shared sets, the Filter
// counts and cpuset_alloc_milli follow. The NUMA split is given back by the caller (apply_assume with the amounts).
__device__ inline void cpuset_release_lane(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones,
                                           kg_cpu_alloc* __restrict__ allocs, const kg_cpu_topo* __restrict__ topos,
                                           uint32_t rec, const uint64_t* cpus) {
    ZoneRec& z = zones[rec];
    if (z.cpu_topo < 0) return;
    const kg_cpu_topo& t = topos[z.cpu_topo];
    kg_cpu_alloc& A = allocs[rec];
    uint32_t used = 0;
    for (int c = 0; c < t.n_cpus; c++) {
        if (!((cpus[c >> 6] >> (c & 63)) & 1ull) || A.ref[c] == 0) continue;  // allocatedCPUs[cpuID] missing: skipped
        A.ref[c] = (uint8_t)(A.ref[c] - 1);
        if (A.ref[c] == 0) A.excl[c] = 0;
        used |= 1u << t.numa[c];
    }
    cpuset_zone_count(z, used, -1);
    cpu_counts(t, &A, (int)(z.cpu_meta & 0xFFu), z);
    int64_t* n = nodes[rec].v;
    n[N_CPUSET] = 1000 * (int64_t)z.cpu_allocated;
    n[N_AMP_CPUSET] = z.amp_ratio > 1.0 ? (int64_t)ceil(__dmul_rn((double)n[N_CPUSET], z.amp_ratio)) : n[N_CPUSET];
}

}  // namespace kg
