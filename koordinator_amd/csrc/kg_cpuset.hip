// kg_cpuset.hip — batch entry of the device cpuset accumulator (kg_cpuset_take): one workgroup (one wave)
// per request, the CPU topology staged in LDS, the accumulator state in LDS (kg_cpuset.h).
#include <hip/hip_runtime.h>

#include "kg_cpuset_reserve.h"
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

// NodeNUMAResource Reserve of a cpuset-binding pod (cpuset_reserve_wave, kg_cpuset_reserve.h) as a launch of its own: the
// pod and record come from (pod, rec), or in replay from the previous step's winner. The pair's zone code on the
// pre-Reserve state: in replay the select step's (zsel); else the one k_ext_assume's evaluation pass preset, or
// evaluated here. Outside replay it is handed on to the kernel that applies the pod (ZONE_PRESET), and taken_out (if
// given) receives the CPUs taken, which the pod's Unreserve gives back (kg_unreserve).
__global__ __launch_bounds__(64) void k_cpuset_reserve(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones,
                                                       kg_cpu_alloc* __restrict__ allocs,
                                                       const kg_cpu_topo* __restrict__ topos, PodsDev pods, KCfg cfg,
                                                       uint32_t pod, uint32_t rec, const uint64_t* __restrict__ winners,
                                                       const uint32_t* __restrict__ step_base, uint32_t step_off,
                                                       const uint32_t* __restrict__ pos, uint32_t index_base,
                                                       uint32_t n_pods, int8_t* __restrict__ zsel, uint32_t zsel_stride,
                                                       int32_t* __restrict__ fail_out, uint64_t* __restrict__ taken_out) {
    __shared__ CpusetLds L;
    if (!(cfg.plugins & KG_PLUGIN_NUMA)) return;
    if (winners) {  // replay: Reserve of pod step-1 on its winner
        const uint32_t step = *step_base + step_off;
        if (step == 0 || step > n_pods) return;  // the graph runs whole blocks of steps past the batch
        const uint64_t prev = __hip_atomic_load(&winners[step - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == 0ull) return;
        pod = step - 1;
        rec = pos[(0xFFFFFFFFu - (uint32_t)(prev & 0xFFFFFFFFull)) - index_base];
        // the zone codes of step-1's pairs: one buffer (k_replay), or the step-parity half of a double buffer
        // (k_ext_replay: zsel_stride = the record count)
        zsel += (size_t)((step - 1) & 1u) * zsel_stride;
    }
    const uint32_t pf = pods.flags[pod];
    const int64_t req_cpu = pods.req_cpu[pod];
    ZoneRec& z = zones[rec];
    int64_t* n = nodes[rec].v;
    if (!cpuset_bound_dev(z, pf, req_cpu)) return;
    const uint32_t node_pol = ((uint32_t)n[N_FLAGS] >> F_NUMA_POLICY_SHIFT) & 15u, pod_pol = (pf >> 16) & 15u;
    const bool numa_pol = (pod_pol != KG_NUMA_NONE ? pod_pol : node_pol) != KG_NUMA_NONE;
    if (threadIdx.x == 0) {
        const int32_t w = (!winners && fail_out) ? *fail_out : 0;
        L.zone = winners ? (numa_pol ? (int32_t)zsel[rec] : -1)
               : zone_is_preset(w) ? zone_of_preset(w) : eval_pair<false>(cfg, n, &z, load_pod(pods, pod)).zone;
    }
    __syncthreads();
    const int32_t zone = L.zone;
    if (zone_reserve_fails(zone)) {  // the Reserve fails on the pair's zone code (reported by the Reserve kernel)
        if (!winners && fail_out && threadIdx.x == 0) *fail_out = zone_preset(zone);
        return;
    }
    const int code = cpuset_reserve_wave(nodes, zones, allocs, topos, pods, pod, rec, zone, L, taken_out);
    if (threadIdx.x != 0) return;
    if (code != 0) {  // Allocate fails (ErrNotEnoughCPUs): the Reserve fails, nothing of the pod is applied
        if (winners) zsel[rec] = (int8_t)ZONE_CPUSET_FAIL;  // read by the replay step that applies the pod
        else if (fail_out) *fail_out = zone_preset(ZONE_CPUSET_FAIL);  // read by k_assume / k_ext_assume
        return;
    }
    if (!winners && fail_out) *fail_out = zone_preset(zone);
}

hipError_t launch_cpuset_reserve(NodeRec* nodes, ZoneRec* zones, kg_cpu_alloc* allocs, const kg_cpu_topo* topos,
                                 const PodsDev& pods, const KCfg& cfg, uint32_t pod, uint32_t rec, const uint64_t* winners,
                                 const uint32_t* step_base, uint32_t step_off, const uint32_t* pos, uint32_t index_base,
                                 uint32_t n_pods, int8_t* zsel, int32_t* fail_out, hipStream_t s, uint32_t zsel_stride,
                                 uint64_t* taken_out) {
    k_cpuset_reserve<<<1, 64, 0, s>>>(nodes, zones, allocs, topos, pods, cfg, pod, rec, winners, step_base, step_off, pos,
                                      index_base, n_pods, zsel, zsel_stride, fail_out, taken_out);
    return hipGetLastError();
}

}  // namespace kg
