// kg_cpuset.hip — batch entry of the device cpuset accumulator (kg_cpuset_take): one workgroup (one wave)
// per request, the CPU topology staged in LDS, the accumulator state in LDS (kg_cpuset.h).
#include <hip/hip_runtime.h>

#include "kg_cpuset.h"
#include "kg_eval.h"
#include "kg_kernels.h"

namespace kg {

__global__ __launch_bounds__(64) void k_cpuset_take(const kg_cpu_topo* __restrict__ topos,
                                                    const kg_cpu_alloc* __restrict__ allocs,
                                                    const kg_cpuset_request* __restrict__ reqs, uint32_t n,
                                                    uint64_t* __restrict__ out, int32_t* __restrict__ rc) {
    __shared__ kg_cpu_topo st;
    __shared__ CpuAccLds acc;
    __shared__ kg_cpu_alloc sa;
    const uint32_t r = blockIdx.x;
    if (r >= n) return;  // uniform per workgroup
    const kg_cpuset_request& q = reqs[r];
    const uint32_t* src = reinterpret_cast<const uint32_t*>(topos + q.topo);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&st);
    for (uint32_t k = threadIdx.x; k < sizeof(kg_cpu_topo) / 4; k += 64) dst[k] = src[k];
    const bool has_alloc = allocs && q.alloc >= 0;
    if (has_alloc) {
        const uint32_t* as = reinterpret_cast<const uint32_t*>(allocs + q.alloc);
        uint32_t* ad = reinterpret_cast<uint32_t*>(&sa);
        for (uint32_t k = threadIdx.x; k < sizeof(kg_cpu_alloc) / 4; k += 64) ad[k] = as[k];
    }
    __syncthreads();
    CpuTake t;
    for (int w = 0; w < 4; w++) {
        t.avail[w] = q.avail[w];
        t.preferred[w] = q.preferred[w];
    }
    t.needed = q.needed;
    t.max_ref = q.max_ref;
    t.bind = q.bind;
    t.excl = q.excl;
    t.strategy = q.strategy;
    t.has_preferred = q.has_preferred;
    uint64_t res[4];
    const int code = cpuset_take(&st, has_alloc ? &sa : nullptr, t, &acc, res);
    if (threadIdx.x == 0) {
        for (int w = 0; w < 4; w++) out[(size_t)r * 4 + w] = res[w];
        rc[r] = code;
    }
}

hipError_t launch_cpuset_take(const kg_cpu_topo* topos, const kg_cpu_alloc* allocs, const kg_cpuset_request* reqs,
                              uint32_t n, uint64_t* out, int32_t* rc, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_cpuset_take<<<n, 64, 0, s>>>(topos, allocs, reqs, n, out, rc);
    return hipGetLastError();
}

}  // namespace kg

namespace kg {

// NodeNUMAResource Reserve of a cpuset-binding pod (plugin.go:585-635 -> resourceManager.Allocate/Update): the
// accumulator's CPUs enter the node's allocation (RefCount++, the pod's exclusive policy, node_allocation.go:111-130),
// the Filter counts and cpuset_alloc_milli follow. Under a NUMA affinity (the pair's zone code: in replay the previous
// step's, else evaluated here) allocateCPUSet takes per allocated NUMA node (resource_manager.go:391-429) and the
// NUMA split with the CPUs is recorded here, before the take changes the counts it trims with (apply_assume leaves it,
// cpuset_numa_reserve). Runs before the Reserve of the NodeInfo columns (apply_assume, which re-derives the record).
// The pod and record come from (pod, rec), or in replay from the previous step's winner.
__global__ __launch_bounds__(64) void k_cpuset_reserve(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones,
                                                       kg_cpu_alloc* __restrict__ allocs,
                                                       const kg_cpu_topo* __restrict__ topos, PodsDev pods, KCfg cfg,
                                                       uint32_t pod, uint32_t rec, const uint64_t* __restrict__ winners,
                                                       const uint32_t* __restrict__ step_base, uint32_t step_off,
                                                       const uint32_t* __restrict__ pos, uint32_t index_base,
                                                       uint32_t n_pods, int8_t* __restrict__ zsel,
                                                       int32_t* __restrict__ fail_out) {
    __shared__ kg_cpu_topo st;
    __shared__ CpuAccLds acc;
    __shared__ kg_cpu_alloc sa;
    if (!(cfg.plugins & KG_PLUGIN_NUMA)) return;
    if (winners) {  // replay: Reserve of pod step-1 on its winner
        const uint32_t step = *step_base + step_off;
        if (step == 0 || step > n_pods) return;  // the graph runs whole blocks of steps past the batch
        const uint64_t prev = __hip_atomic_load(&winners[step - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == 0ull) return;
        pod = step - 1;
        rec = pos[(0xFFFFFFFFu - (uint32_t)(prev & 0xFFFFFFFFull)) - index_base];
    }
    const uint32_t pf = pods.flags[pod];
    const int64_t req_cpu = pods.req_cpu[pod];
    ZoneRec& z = zones[rec];
    int64_t* n = nodes[rec].v;
    if (z.cpu_topo < 0 || (pf & KG_POD_NUMA_SKIP)) return;
    const uint32_t node_bind = (z.cpu_meta >> CPU_META_BIND_SHIFT) & 3u;
    if (!((pf & KG_POD_CPU_BIND) || (node_bind != KG_NODE_CPU_BIND_NONE && req_cpu != 0))) return;
    const uint32_t node_pol = ((uint32_t)n[N_FLAGS] >> F_NUMA_POLICY_SHIFT) & 15u, pod_pol = (pf >> 16) & 15u;
    const bool numa_pol = (pod_pol != KG_NUMA_NONE ? pod_pol : node_pol) != KG_NUMA_NONE;
    uint32_t mask = 0;  // the NUMA affinity of the Reserve (0: the whole node)
    // the pair's zone code on the pre-Reserve state: in replay the select step's; else the one k_ext_assume's evaluation
    // pass preset, or evaluated here. Outside replay it is handed on to the kernel that applies the pod (ZONE_PRESET).
    __shared__ int32_t s_zone;
    if (threadIdx.x == 0) {
        const int32_t w = (!winners && fail_out) ? *fail_out : 0;
        s_zone = winners ? (numa_pol ? (int32_t)zsel[rec] : -1)
               : zone_is_preset(w) ? zone_of_preset(w) : eval_pair<false>(cfg, n, &z, load_pod(pods, pod)).zone;
    }
    __syncthreads();
    const int32_t zone = s_zone;
    if (zone_reserve_fails(zone)) {  // the Reserve fails on the pair's zone code (reported by the Reserve kernel)
        if (!winners && fail_out && threadIdx.x == 0) *fail_out = zone_preset(zone);
        return;
    }
    if (numa_pol) mask = zone_affinity(zone);
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
    }
    __shared__ uint64_t s_avail[4];
    if (threadIdx.x == 0)
        for (int w = 0; w < 4; w++) s_avail[w] = q.avail[w];
    __syncthreads();
    for (int w = 0; w < 4; w++) q.avail[w] = s_avail[w];
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
        code = cpuset_take(&st, &sa, q, &acc, res);
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
            code = cpuset_take(&st, &sa, qz, &acc, rz);
            __syncthreads();
            for (int w = 0; w < 4; w++) res[w] |= rz[w];
        }
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    if (code != 0) {  // Allocate fails (ErrNotEnoughCPUs): the Reserve fails, nothing of the pod is applied
        if (winners) zsel[rec] = (int8_t)ZONE_CPUSET_FAIL;  // read by the replay step that applies the pod
        else if (fail_out) *fail_out = zone_preset(ZONE_CPUSET_FAIL);  // read by k_assume / k_ext_assume
        return;
    }
    if (!winners && fail_out) *fail_out = zone_preset(zone);
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
    z.status = cpuset_zone_status(z.status, used);
    cpu_counts(st, &A, max_ref, z);
    n[N_CPUSET] = 1000 * (int64_t)z.cpu_allocated;
    n[N_AMP_CPUSET] = z.amp_ratio > 1.0 ? (int64_t)ceil(__dmul_rn((double)n[N_CPUSET], z.amp_ratio)) : n[N_CPUSET];
}

hipError_t launch_cpuset_reserve(NodeRec* nodes, ZoneRec* zones, kg_cpu_alloc* allocs, const kg_cpu_topo* topos,
                                 const PodsDev& pods, const KCfg& cfg, uint32_t pod, uint32_t rec, const uint64_t* winners,
                                 const uint32_t* step_base, uint32_t step_off, const uint32_t* pos, uint32_t index_base,
                                 uint32_t n_pods, int8_t* zsel, int32_t* fail_out, hipStream_t s) {
    k_cpuset_reserve<<<1, 64, 0, s>>>(nodes, zones, allocs, topos, pods, cfg, pod, rec, winners, step_base, step_off, pos,
                                      index_base, n_pods, zsel, fail_out);
    return hipGetLastError();
}

}  // namespace kg
