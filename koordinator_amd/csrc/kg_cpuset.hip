// kg_cpuset.hip — batch entry of the device cpuset accumulator (kg_cpuset_take): one workgroup (one wave)
// per request, the CPU topology staged in LDS, the accumulator state in LDS (kg_cpuset.h).
#include <hip/hip_runtime.h>

#include "kg_cpuset.h"
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
